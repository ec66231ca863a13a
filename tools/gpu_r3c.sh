# Round 3, third GPU session: config-3 A/B with fp32 SUM timed beside every
# row, and the pageable workers traced per chunk (where the time goes).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c
rm -rf $O && mkdir -p $O
step() {    # name timeout cmd...: stop the script on a fault / abort / time limit
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
    local rc=$?
    echo "$name rc=$rc" | tee -a $O/steps.txt
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
step ab_new1 300 python3 tools/ab_types.py mpich_amd/libmpix_redop.so r03c
step ab_old1 300 python3 tools/ab_types.py tools/bin/r02k/libmpix_redop.so r02
step ab_new2 300 python3 tools/ab_types.py mpich_amd/libmpix_redop.so r03c
step ab_old2 300 python3 tools/ab_types.py tools/bin/r02k/libmpix_redop.so r02
step pageable 900 env PAGEABLE_CONFIGS=8:16:0:none,1:16:1:none,2:16:1:none,4:16:1:none,4:64:1:none,8:32:1:none,8:16:1:none,6:32:0:none python3 tools/pageable_probe.py sweep $O/r03_pageable_trace.jsonl
cat $O/steps.txt
python3 -c "
import json
for f in ('ab_new1','ab_old1','ab_new2','ab_old2'):
    try:
        d=json.loads(open('$O/%s.out'%f).read().strip().splitlines()[-1]); print(f, d['fp32_sum_ms'], d['min_vs_fp32_sum'], d['within_2pct'], d['rows'], [(r['type'],r['op'],r['vs_fp32_sum']) for r in d['slowest'][:6]])
    except Exception as e: print(f, e)
"
cat $O/pageable.out
