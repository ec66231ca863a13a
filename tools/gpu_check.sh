set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocminfo | grep -m3 -E "Marketing|gfx"; nproc; lscpu | grep "Model name") > gpurun_out/r1_env.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/r1_pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/r1_pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 8 --sweep > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err
echo "bench rc=$?"
tail -3 gpurun_out/r1_pytest_gpu.log
cat gpurun_out/r1_bench.json
