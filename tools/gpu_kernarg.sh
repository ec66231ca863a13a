# HIP runtime kernarg settings vs launch issue cost and the library's small-call
# figures: tools/kernarg_probe.hip and tools/latency_small.py per setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/kernarg2
rm -rf $O && mkdir -p $O
run() {
  env "$@" timeout -k 10 60 tools/bin/kernarg_probe >> $O/probe.jsonl &&
  env "$@" timeout -k 10 120 python3 tools/latency_small.py >> $O/lat.jsonl 2>> $O/lat.err
}
run X=1 && run HIP_FORCE_DEV_KERNARG=0 && run DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 && \
run ROC_USE_FGS_KERNARG=1 && run DEBUG_HIP_KERNARG_COPY_OPT=0 && run X=2
rc=$?
cat $O/probe.jsonl
python3 - <<PY
import json
for l in open('$O/lat.jsonl'):
    d = json.loads(l)
    print(d['env'], [s['median_us'] for s in d['sync']], [(c['chunk_bytes'] >> 10, c['us_per_call']) for c in d['chunked']])
PY
exit $rc
