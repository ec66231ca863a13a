# GPU box: kernel sweep, rocprofv3 kernel-trace stats and PMC traffic passes,
# full GPU test suite.  Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I mpich_amd/csrc -I include \
    tools/tune_sum.hip -o /tmp/tune_sum && \
timeout -k 10 240 /tmp/tune_sum $((1<<28)) 3 10 > $O/r1_tune.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/prof_kt -o kt --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/r1_prof_bench.json 2> $O/r1_prof_bench.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/prof_fetch -o fetch --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $O/r1_pmc_fetch.json 2> $O/r1_pmc_fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/prof_write -o write --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $O/r1_pmc_write.json 2> $O/r1_pmc_write.err && \
timeout -k 10 900 python3 -m pytest tests -q -m gpu -p no:cacheprovider > $O/r1_pytest_gpu.log 2>&1
rc=$?
echo "rc=$rc"
tail -3 $O/r1_pytest_gpu.log
tail -12 $O/r1_tune.txt
find $O/prof_kt $O/prof_fetch $O/prof_write -name "*.csv" | head -20
