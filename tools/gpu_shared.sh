set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/shared
rm -rf $O && mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py tests/test_coll_c.py -k "shared or pull or churn or fault or verification or staged" > $O/t.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/t.log | tail -12
tail -2 $O/t.log
exit $rc
