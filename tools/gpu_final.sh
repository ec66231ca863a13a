# Round-end evidence refresh: GPU tests, rocprofv3 kernel-trace stats of the
# bench command, separate FETCH_SIZE / WRITE_SIZE PMC passes, the full bench
# (with cpu_baseline) and the per-type sweep.  Outputs under gpurun_out/r1f_*.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -m pytest tests -q -m gpu -p no:cacheprovider > $O/r1f_pytest_gpu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/r1f_kt -o kt --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/r1f_prof_bench.json 2> $O/r1f_prof_bench.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/r1f_fetch -o fetch --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > /dev/null 2> $O/r1f_pmc.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/r1f_write -o write --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > /dev/null 2>> $O/r1f_pmc.err && \
timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 20 --sweep > $O/r1f_bench.json 2> $O/r1f_bench.err && \
timeout -k 10 300 python3 tools/perf_types.py > $O/r1f_perf_types.json 2> $O/r1f_perf_types.err
echo rc=$?
tail -2 $O/r1f_pytest_gpu.log
cat $O/r1f_bench.json
