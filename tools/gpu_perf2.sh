set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python3 tools/perf_types.py > $O/r1_perf_types.json 2> $O/r1_perf_types.err && \
timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 20 > $O/r1_bench2.json 2> $O/r1_bench2.err && \
MPIX_REDOP_SYNC=block timeout -k 10 200 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extras > $O/r1_bench_block.json 2>> $O/r1_bench2.err
echo rc=$?
cat $O/r1_bench2.json
cat $O/r1_bench_block.json
