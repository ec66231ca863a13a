set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -m pytest tests -q -x -m gpu -p no:cacheprovider > $O/r1_pytest_gpu7.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --sweep > $O/r1_bench_sweep2.json 2> $O/r1_bench_sweep2.err
echo rc=$?
tail -3 $O/r1_pytest_gpu7.log
python3 -c "import json;d=json.load(open('$O/r1_bench_sweep2.json'));print(json.dumps(d['sweep']))"
