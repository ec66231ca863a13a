set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -m pytest tests -q -x -m gpu -p no:cacheprovider > $O/r1_pytest_gpu6.log 2>&1
echo rc=$?
tail -3 $O/r1_pytest_gpu6.log
