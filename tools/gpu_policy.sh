# Cache-policy / pipelining sweep of the fp32 SUM packet kernel (tools/tune_policy.hip)
# at 1 GiB and 256 MiB, plus the RCCL two-ranks-on-one-GPU probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -w -I mpich_amd/csrc -I include tools/tune_policy.hip -o /tmp/tune_policy && \
hipcc -O2 -w tools/rccl_probe.cpp -o /tmp/rccl_probe -lrccl && \
timeout -k 10 240 /tmp/tune_policy 268435456 4 10 > $O/r1h_tune_policy_1g.txt 2>&1 && \
timeout -k 10 120 /tmp/tune_policy 67108864 4 20 > $O/r1h_tune_policy_256m.txt 2>&1
rc=$?
echo tune rc=$rc
cat $O/r1h_tune_policy_1g.txt | head -30
head -24 $O/r1h_tune_policy_256m.txt
[ $rc -eq 0 ] && (NCCL_DEBUG=WARN timeout -k 10 60 /tmp/rccl_probe > $O/r1h_rccl_probe.txt 2>&1; echo probe rc=$?; tail -20 $O/r1h_rccl_probe.txt)
exit $rc
