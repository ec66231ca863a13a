set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
g++ -O2 -std=c++17 -w -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/lat_probe.cpp \
    -Lmpich_amd -lmpix_redop -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/mpich_amd \
    -Wl,-rpath,/opt/rocm/lib -o /tmp/lat_probe && \
timeout -k 10 120 /tmp/lat_probe > $O/r1_lat_probe.txt 2>&1 && \
timeout -k 10 900 python3 -m pytest tests -q -x -m gpu -p no:cacheprovider > $O/r1_pytest_gpu2.log 2>&1 && \
timeout -k 10 300 python3 tools/perf_latency.py > $O/r1_latency_zc.json 2> $O/r1_latency.err && \
timeout -k 10 300 python3 tools/perf_types.py > $O/r1_perf_types2.json 2> $O/r1_perf_types.err
echo rc=$?
tail -2 $O/r1_pytest_gpu2.log
cat $O/r1_lat_probe.txt
