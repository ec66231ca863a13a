set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/mp
rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --durations=5 --timeout 400 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py > $O/mp.log 2>&1
rc=$?
tail -15 $O/mp.log
exit $rc
