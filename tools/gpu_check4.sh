set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -T -d $O/prof_vfetch -o vf --output-format csv -- python3 tools/run_vector.py > /dev/null 2> $O/r1_vf.err && \
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -T -d $O/prof_vwrite -o vw --output-format csv -- python3 tools/run_vector.py > /dev/null 2> $O/r1_vw.err && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -d $O/prof_vkt -o vkt --output-format csv -- python3 tools/run_vector.py > /dev/null 2> $O/r1_vkt.err && \
MPIX_PARITY_BYTES=268435456 timeout -k 10 1000 python3 -m pytest tests/test_gpu_parity.py -q -x -m gpu -k test_random_parity -p no:cacheprovider > $O/r1_parity_256MiB.log 2>&1
echo rc=$?
tail -3 $O/r1_parity_256MiB.log
