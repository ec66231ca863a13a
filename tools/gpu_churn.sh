set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/churn
rm -rf $O && mkdir -p $O
MPIX_COLL_TRACE=1 timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py -k "churn" > $O/trace.log 2>&1 &&
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py tests/test_coll_c.py tests/test_coll_fuzz.py -k "pull or staged or churn or device" > $O/t.log 2>&1
rc=$?
grep -v "^\[mpix_coll" $O/trace.log | tail -3
grep "pull window" $O/trace.log | head -8
tail -3 $O/t.log
exit $rc
