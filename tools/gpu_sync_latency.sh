# Synchronous-call latency, kernel-stored vs stream-written completion word
# (tools/sync_latency.cpp), then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
g++ -O2 -w -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/sync_latency.cpp \
    -Lmpich_amd -lmpix_redop -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/mpich_amd \
    -Wl,-rpath,/opt/rocm/lib -o /tmp/sync_latency && \
nproc > gpurun_out/sync_latency.txt && \
MPIX_REDOP_SYNC=stream timeout -k 10 120 /tmp/sync_latency >> gpurun_out/sync_latency.txt 2>&1 && \
MPIX_REDOP_SYNC=flag timeout -k 10 120 /tmp/sync_latency >> gpurun_out/sync_latency.txt 2>&1 && \
MPIX_REDOP_SYNC=stream timeout -k 10 120 /tmp/sync_latency >> gpurun_out/sync_latency.txt 2>&1 && \
MPIX_REDOP_SYNC=flag timeout -k 10 120 /tmp/sync_latency >> gpurun_out/sync_latency.txt 2>&1 && \
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
cat gpurun_out/sync_latency.txt
tail -n 5 gpurun_out/gpu_tests.log
exit $rc
