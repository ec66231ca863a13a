# Round 3, fourth GPU session: the pageable workers with non-temporal copies
# into the pinned buffers (vs memcpy), traced per chunk; the pageable GPU tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3d
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
step pageable 900 env PAGEABLE_CONFIGS=8:16:1:none:0,8:16:1:none:1,8:16:0:none:1,4:16:1:none:1,8:32:1:none:1,12:16:1:none:1,8:16:1:gpu:1,6:16:1:none:1 python3 tools/pageable_probe.py sweep $O/r03_pageable_nt.jsonl
cat $O/steps.txt
tail -n 2 $O/tests.out
python3 -c "
import json
for l in open('$O/r03_pageable_nt.jsonl'):
    d=json.loads(l); t=d.get('trace_last_call') or {}
    print(d.get('W'), d.get('chunk_MiB'), d.get('db'), d.get('aff'), d.get('nt'), d.get('ms'), d.get('best_ms'), d.get('frac_of_pcie'), '|', t.get('span_ms'), t.get('copy_in_ms_sum'), t.get('wait_ms_sum'), t.get('copy_out_ms_sum'), t.get('worker_busy_frac'))
"
