# Completion-wait variants of the synchronous call (tools/sync_probe.hip),
# then the collective GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -w -I mpich_amd/csrc -I include tools/sync_probe.hip -o /tmp/sync_probe && \
timeout -k 10 120 /tmp/sync_probe 2000 60 > gpurun_out/sync_probe.txt 2>&1 && \
timeout -k 10 400 python3 -u -m pytest tests/test_coll_c.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/s3j.log 2>&1
rc=$?
cat gpurun_out/sync_probe.txt
tail -n 3 gpurun_out/s3j.log
exit $rc
