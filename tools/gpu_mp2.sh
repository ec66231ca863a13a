set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/mp2
rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py tests/test_coll_c.py > $O/t.log 2>&1
rc=$?
tail -3 $O/t.log
exit $rc
