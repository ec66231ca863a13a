set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tree
rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --durations=5 --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_coll_c.py tests/test_coll_multiproc.py \
    -k "tree or recursive_halving_pull or device_local or staged" > $O/t.log 2>&1
rc=$?
tail -8 $O/t.log
exit $rc
