# Round-2 check: the new GPU tests first (multi-process schedules, boundary),
# then the whole GPU suite, the default bench line and a 2-rank same-device
# rehearsal of the N>1 flow (gloo transport through pinned staging).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2a
rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_boundary_gpu.py tests/test_coll_multiproc.py tests/test_ipc_gpu.py > $O/new_tests.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && \
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --steps 3 --warmup 1 --rsb-bytes 268435456 > $O/bench_n2_rehearsal.json 2> $O/bench_n2.err
rc=$?
echo rc=$rc
tail -3 $O/new_tests.log; tail -3 $O/pytest_gpu.log
cat $O/bench_n1.json $O/bench_n2_rehearsal.json
exit $rc
