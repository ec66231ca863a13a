# Round 3: the default (wave) pageable path by operand size vs the pinned call
# and the staging path; the GPU suite's host-operand tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3g
rm -rf $O && mkdir -p $O
step() {    # name timeout cmd...: stop the script on a fault / abort / time limit
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
    local rc=$?
    echo "$name rc=$rc" | tee -a $O/steps.txt
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
step tests 300 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "pageable or host"
for B in 67108864 268435456 1073741824; do
  step size_$B 600 env PAGEABLE_BYTES=$B PAGEABLE_CONFIGS=8:64:0:none:1:wave,0:64:0:none:1:wave python3 tools/pageable_probe.py sweep $O/r03_pageable_size_$B.jsonl
done
cat $O/steps.txt
tail -n 2 $O/tests.out
cat $O/r03_pageable_size_*.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print(d.get('bytes'), d.get('mode'), d.get('W'), d.get('chunk_MiB'), d.get('ms'), d.get('pinned_call_ms'), d.get('vs_pinned'), d.get('frac_of_pcie'), d.get('checked'), d.get('error','')[:200])
"
