# bench.py N>1 value-leg watchdog: a 3 s limit must end the run with rank 0's
# error line and status 2; then the normal two-rank rehearsal must pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/vwd
rm -rf $O && mkdir -p $O
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --steps 3 --warmup 1 --rsb-bytes 268435456 --value-timeout 3 > $O/wd.json 2> $O/wd.err
echo "watchdog run rc=$?"
cat $O/wd.json
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 \
    --steps 3 --warmup 1 --rsb-bytes 268435456 > $O/n2.json 2> $O/n2.err
rc=$?
echo "normal run rc=$rc"
tail -c 400 $O/n2.json
exit $rc
