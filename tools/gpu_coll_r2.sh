# Collective GPU tests after the window/stream changes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/coll_r2b
rm -rf $O && mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py tests/test_ipc_gpu.py > $O/t.log 2>&1
rc=$?
tail -15 $O/t.log
exit $rc
