# Kernel experiments: XCD-aware block remap for the contiguous combine, and
# vector-target variants (two pairs per lane, NT source, block size).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -w -I mpich_amd/csrc -I include tools/tune_sum.hip -o /tmp/tune_sum && \
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -w -I mpich_amd/csrc -I include tools/tune_vector.hip -o /tmp/tune_vector && \
timeout -k 10 300 /tmp/tune_sum 268435456 6 10 xcd > $O/r1_tune_xcd.txt 2>&1 && \
timeout -k 10 300 /tmp/tune_vector > $O/r1_tune_vector2.txt 2>&1
echo rc=$?
cat $O/r1_tune_xcd.txt | head -12
cat $O/r1_tune_vector2.txt
