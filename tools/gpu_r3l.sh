# Round 3: wave form with the result returned through HBM + copy engine (split)
# vs the kernel writing the page-locked buffer; pageable/host GPU tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3l
rm -rf $O && mkdir -p $O
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
    local rc=$?
    echo "$name rc=$rc" | tee -a $O/steps.txt
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
step tests 300 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "pageable or host"
step split 600 env PAGEABLE_CONFIGS=8:64:0:none:1:wave,8:128:0:none:1:wave,8:32:0:none:1:wave python3 tools/pageable_probe.py sweep $O/r03_pageable_split.jsonl
step nosplit 400 env MPIX_REDOP_PAGEABLE_SPLIT=0 PAGEABLE_CONFIGS=8:64:0:none:1:wave python3 tools/pageable_probe.py sweep $O/r03_pageable_nosplit.jsonl
cat $O/steps.txt
tail -n 2 $O/tests.out
cat $O/r03_pageable_split.jsonl $O/r03_pageable_nosplit.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print(d.get('bytes'), d.get('mode'), d.get('W'), d.get('chunk_MiB'), d.get('ms'), d.get('best_ms'), d.get('pinned_call_ms'), d.get('vs_pinned'), d.get('frac_of_pcie'), d.get('checked'), d.get('error','')[:300])
"
