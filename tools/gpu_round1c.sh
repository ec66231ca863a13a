# Self-signalling small-call kernel: full GPU suite, latency with it on and
# off, and the pageable bounce threshold (64 KiB default vs 1 MiB).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -m pytest tests -q -m gpu -p no:cacheprovider -x > $O/r1c_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/perf_latency.py > $O/r1c_latency.json 2> $O/r1c_latency.err && \
MPIX_REDOP_SMALL_BYTES=0 PERF_COUNTS=1,16,256,4096 timeout -k 10 120 python3 tools/perf_latency.py > $O/r1c_latency_nosmall.json 2>> $O/r1c_latency.err && \
MPIX_REDOP_BOUNCE_BYTES=1048576 PERF_COUNTS=16384,65536,262144 timeout -k 10 120 python3 tools/perf_latency.py > $O/r1c_latency_bounce1m.json 2>> $O/r1c_latency.err && \
g++ -O2 -w -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/lat_probe.cpp \
    -Lmpich_amd -lmpix_redop -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/mpich_amd \
    -Wl,-rpath,/opt/rocm/lib -o /tmp/lat_probe && \
timeout -k 10 120 /tmp/lat_probe > $O/r1c_lat_probe.txt 2>&1
echo rc=$?
tail -3 $O/r1c_pytest_gpu.log
cat $O/r1c_latency.json; echo; cat $O/r1c_latency_nosmall.json; echo; cat $O/r1c_latency_bounce1m.json
