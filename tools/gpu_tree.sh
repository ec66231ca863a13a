set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tree
rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --durations=5 --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_coll_c.py tests/test_coll_multiproc.py tests/test_coll_fuzz.py \
    -k "tree or pull or device_local or staged or copy_multi or allreduce" > $O/t.log 2>&1 &&
tail -3 $O/t.log &&
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --steps 3 --warmup 1 --rsb-bytes 268435456 > $O/n2.json 2> $O/n2.err
rc=$?
tail -4 $O/t.log
tail -c 1200 $O/n2.json
exit $rc
