# Full GPU suite, then the per-type / vector / multi perf table (config 3 + 5).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 tools/perf_types.py > $O/perf_types.json 2> $O/perf_types.err
rc=$?
tail -n 2 $O/gpu_tests.log
python3 -c "import json; d=json.load(open('$O/perf_types.json')); print(d['vector']); print(min(r['GBs'] for r in d['per_type']), max(r['GBs'] for r in d['per_type']))" || true
exit $rc
