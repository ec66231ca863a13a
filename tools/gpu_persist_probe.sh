# Resident-worker latency probe (tools/persist_probe.hip).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 -w tools/persist_probe.hip -o /tmp/persist_probe && \
timeout -k 10 40 /tmp/persist_probe 1000 > gpurun_out/persist_probe.txt 2>&1
rc=$?
cat gpurun_out/persist_probe.txt
exit $rc
