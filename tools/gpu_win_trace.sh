# Four-rank rehearsal with the exchange trace on: which pull windows verify.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/win_trace
rm -rf $O && mkdir -p $O
MPIX_COLL_TRACE=1 MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 \
    --steps 3 --warmup 1 --rsb-bytes 536870912 > $O/n4.json 2> $O/n4.err
rc=$?
grep -E "pull window|shared-window|alloc_shared" $O/n4.err > $O/win_lines.txt || true
grep -c "" $O/n4.err
head -60 $O/win_lines.txt
exit $rc
