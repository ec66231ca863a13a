set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I mpich_amd/csrc -I include \
    tools/tune_vector.hip -o /tmp/tune_vector && \
timeout -k 10 120 /tmp/tune_vector > $O/r1_tune_vector.txt 2>&1 && \
timeout -k 10 300 python3 tools/perf_latency.py > $O/r1_latency.json 2> $O/r1_latency.err && \
MPIX_REDOP_STAGE_CHUNK=16777216 timeout -k 10 300 python3 tools/perf_latency.py > $O/r1_latency_c16.json 2>> $O/r1_latency.err && \
MPIX_REDOP_STAGE_CHUNK=268435456 timeout -k 10 300 python3 tools/perf_latency.py > $O/r1_latency_c256.json 2>> $O/r1_latency.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -T -d $O/prof_vec -o vec --output-format csv -- /tmp/tune_vector > /dev/null 2> $O/r1_prof_vec.err
echo rc=$?
cat $O/r1_tune_vector.txt
