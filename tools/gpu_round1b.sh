# Host-path latency (pageable bounce), misaligned at 256 MiB / 1 GiB, the
# host-buffer parity tests, and the N=2 flow rehearsal (gloo, one device).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider \
    -k "pageable or host or staged" > $O/r1b_pytest.log 2>&1 && \
timeout -k 10 300 python3 tools/perf_latency.py > $O/r1b_latency.json 2> $O/r1b_latency.err && \
timeout -k 10 300 python3 tools/perf_types.py > $O/r1b_perf_types.json 2> $O/r1b_perf_types.err && \
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 240 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --steps 5 --warmup 2 --rsb-bytes 1073741824 > $O/r1b_rehearse.json 2> $O/r1b_rehearse.err
echo rc=$?
tail -2 $O/r1b_pytest.log
cat $O/r1b_latency.json
cat $O/r1b_rehearse.json
