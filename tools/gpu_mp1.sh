set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/mp1
rm -rf $O && mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py tests/test_ipc_gpu.py > $O/mp.log 2>&1
rc=$?
grep -E "AssertionError|bad of|assert" $O/mp.log | head
exit $rc
