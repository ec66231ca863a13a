# Session 3 re-entry check on a fresh box: GPU tests, smoke, headline bench,
# and the N>1 watchdog rehearsal (2 ranks on device 0, gloo, rank 1 stalls).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/s3_pytest_gpu.log 2>&1 && \
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/s3_smoke.log 2>&1 && \
timeout -k 10 300 python3 bench.py > $O/s3_bench.json 2> $O/s3_bench.err && \
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo MPIX_BENCH_STALL_RANK=1 timeout -k 10 240 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --steps 5 --warmup 2 --rsb-bytes 268435456 --extras-timeout 30 > $O/s3_watchdog.json 2> $O/s3_watchdog.err
echo rc=$?
tail -n 2 $O/s3_pytest_gpu.log
cat $O/s3_smoke.log $O/s3_bench.json $O/s3_watchdog.json
