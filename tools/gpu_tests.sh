# GPU test suite only (one process, per-test thread timeout); log under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
    -p no:cacheprovider ${MPIX_TEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -n 30 gpurun_out/gpu_tests.log
exit $rc
