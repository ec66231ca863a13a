# A/B of the synchronous call's completion word at the headline size: the
# stream write (hipStreamWriteValue32, default MPIX_REDOP_SYNC=flag) against a
# one-lane signal kernel (MPIX_REDOP_SYNC=kernel), alternating processes; then
# the GPU parity/boundary suites under the kernel mode.  The kernel mode was
# removed after this A/B (no gain, profiles/r02_sync_kernel_ab.json); rerunning
# this script needs it back in redop_capi.cpp.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/synck
rm -rf $O && mkdir -p $O
for r in 1 2 3; do
    for m in flag kernel; do
        MPIX_REDOP_SYNC=$m timeout -k 10 120 python3 bench.py --steps 100 --warmup 5 \
            --no-cpu-baseline --no-extras > $O/bench_${m}_$r.json 2> $O/bench_${m}_$r.err || exit 1
    done
done
MPIX_REDOP_SYNC=kernel timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_boundary_gpu.py \
    > $O/tests_kernel_mode.log 2>&1
rc=$?
echo rc=$rc
tail -2 $O/tests_kernel_mode.log
exit $rc
