# LDS-DMA variants of the fp32 SUM packet kernel (tools/tune_lds.hip) at 1 GiB and 256 MiB.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -w -I mpich_amd/csrc -I include tools/tune_lds.hip -o /tmp/tune_lds && \
timeout -k 10 240 /tmp/tune_lds 268435456 4 10 > $O/s3_tune_lds_1g.txt 2>&1 && \
timeout -k 10 120 /tmp/tune_lds 67108864 4 20 > $O/s3_tune_lds_256m.txt 2>&1
rc=$?
cat $O/s3_tune_lds_1g.txt
head -12 $O/s3_tune_lds_256m.txt
exit $rc
