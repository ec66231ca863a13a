# Round 3: the wave form of the pageable path (all workers on one chunk, one
# kernel per chunk, three buffers in rotation) vs the per-worker form.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3f
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
step pageable 900 env PAGEABLE_CONFIGS=8:16:1:none:1:worker,8:32:1:none:1:wave,8:64:1:none:1:wave,12:64:1:none:1:wave,8:128:1:none:1:wave,12:128:1:none:1:wave,8:64:1:none:0:wave python3 tools/pageable_probe.py sweep $O/r03_pageable_wave_ramp.jsonl
cat $O/steps.txt
tail -n 2 $O/tests.out
python3 -c "
import json
for l in open('$O/r03_pageable_wave_ramp.jsonl'):
    d=json.loads(l)
    print(d.get('mode'), d.get('W'), d.get('chunk_MiB'), d.get('aff'), d.get('ms'), d.get('best_ms'), d.get('frac_of_pcie'), d.get('checked'), d.get('error','')[:300])
"
