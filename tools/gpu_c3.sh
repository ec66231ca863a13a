# BASELINE config 3 at its size: the 170-case parity sweep at 256 MiB per
# operand (after a 4 MiB shake-out of the device-side generators), then the
# per-(op, type) kernel table at 1 GiB per operand (past the 256 MB MALL).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c3
rm -rf $O && mkdir -p $O
MPIX_C3_BYTES=4194304 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_c3_full.py > $O/c3_4MiB.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest -x -v --durations=10 --timeout 120 --timeout-method thread \
    -m gpu tests/test_c3_full.py > $O/c3_256MiB.log 2>&1 && \
PERF_BYTES=1073741824 timeout -k 10 300 python3 tools/perf_types.py > $O/perf_types_1GiB.json 2> $O/perf.err
rc=$?
echo rc=$rc
tail -3 $O/c3_4MiB.log; tail -15 $O/c3_256MiB.log
exit $rc
