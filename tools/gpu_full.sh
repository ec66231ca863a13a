# The driver's round-end GPU tier, rehearsed: the whole -m gpu suite in one
# process, then smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/full
rm -rf $O && mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?
tail -4 $O/pytest_gpu.log
cat $O/smoke.log | tail -2
exit $rc
