# Random parity sweep at 256 MiB per operand (170 (op, type) cases).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MPIX_PARITY_BYTES=268435456 timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_parity.py -q -m gpu -x \
    -k test_random_parity --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/sweep256.log 2>&1
rc=$?
tail -n 3 gpurun_out/sweep256.log
exit $rc
