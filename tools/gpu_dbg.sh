set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/dbg
rm -rf $O && mkdir -p $O
MPIX_COLL_TRACE=1 timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu \
    "tests/test_coll_multiproc.py::test_staged_rsb_matches_oracle[3]" > $O/t.log 2>&1
echo rc=$?
grep -v "^\[mpix_coll" $O/t.log | tail -5
