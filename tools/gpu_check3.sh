set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I mpich_amd/csrc -I include \
    tools/tune_sum.hip -o /tmp/tune_sum && \
timeout -k 10 900 python3 -m pytest tests -q -x -m gpu -p no:cacheprovider > $O/r1_pytest_gpu3.log 2>&1 && \
timeout -k 10 240 /tmp/tune_sum $((1<<28)) 8 20 focus > $O/r1_tune_focus.txt 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 20 > $O/r1_bench3.json 2> $O/r1_bench3.err
echo rc=$?
tail -2 $O/r1_pytest_gpu3.log
grep -v "^#" $O/r1_tune_focus.txt | tail -15
cat $O/r1_bench3.json
