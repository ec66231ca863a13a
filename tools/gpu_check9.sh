set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -m pytest tests -q -x -m gpu -p no:cacheprovider > $O/r1_pytest_gpu9.log 2>&1 && \
g++ -O2 -std=c++17 -w -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/lat_probe.cpp \
    -Lmpich_amd -lmpix_redop -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/mpich_amd \
    -Wl,-rpath,/opt/rocm/lib -o /tmp/lat_probe && \
timeout -k 10 120 /tmp/lat_probe > $O/r1_lat_probe2.txt 2>&1 && \
MPIX_REDOP_SYNC=flag timeout -k 10 120 /tmp/lat_probe > $O/r1_lat_probe_flag.txt 2>&1 && \
MPIX_REDOP_SYNC=flag timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "random_parity and FLOAT or concurrent or host_buffers or op_table" -p no:cacheprovider > $O/r1_pytest_flag.log 2>&1 && \
timeout -k 10 300 python3 tools/perf_types.py > $O/r1_perf_types3.json 2> $O/r1_perf_types3.err
echo rc=$?
tail -2 $O/r1_pytest_gpu9.log
cat $O/r1_lat_probe2.txt
grep Reduce_local $O/r1_lat_probe_flag.txt
tail -1 $O/r1_pytest_flag.log
python3 -c "import json;d=json.load(open('$O/r1_perf_types3.json'));print(d['misaligned'], d['vector'])"
