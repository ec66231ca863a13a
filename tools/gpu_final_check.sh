# Round-end rehearsal of what the driver runs: GPU suite, smoke(), default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?
tail -n 2 gpurun_out/gpu_tests.log
tail -n 1 gpurun_out/smoke.log
cat gpurun_out/bench_default.json
exit $rc
