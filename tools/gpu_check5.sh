set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python3 -m pytest tests/test_ipc_gpu.py -q -x -m gpu -p no:cacheprovider > $O/r1_ipc.log 2>&1
echo rc=$?
tail -30 $O/r1_ipc.log
