# Grouped-load k_contig: parity, the default bench, per-(op, type) at 1 GiB.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/grp
rm -rf $O && mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_c3_full.py tests/test_fuzz.py > $O/t.log 2>&1 &&
tail -2 $O/t.log &&
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err &&
PERF_BYTES=1073741824 timeout -k 10 300 python3 tools/perf_types.py > $O/perf_types_1GiB.json 2> $O/perf.err
rc=$?
tail -c 700 $O/bench.json | head -c 400; echo
python3 -c "import json; d=json.load(open('$O/perf_types_1GiB.json')); r=sorted(x['GBs'] for x in d['per_type']); print('per-type min/median/max', r[0], r[len(r)//2], r[-1])" || true
exit $rc
