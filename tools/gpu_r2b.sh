# Round-2 check b: whole GPU suite + default bench line (+ rocprofv3 kernel
# stats of the bench command for profiles/).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2b
rm -rf $O && mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/kt -o kt --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/prof_bench.json 2> $O/prof_bench.err
rc=$?
echo rc=$rc
tail -2 $O/pytest_gpu.log
cat $O/bench_n1.json $O/prof_bench.json
exit $rc
