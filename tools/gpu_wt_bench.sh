# The default bench's value leg (50 synchronous 1 GiB fp32 SUM calls, kernel
# timed with HIP events) under alternating write-through settings, one process
# each.  A setting is TAIL:EVERY (MPIX_REDOP_WT_TAIL, MPIX_REDOP_WT_EVERY).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wtb
rm -rf $O && mkdir -p $O
i=0
for WT in ${WT_LIST:-0:0 0:4 0:0 0:4}; do
    i=$((i+1))
    MPIX_REDOP_WT_TAIL=${WT%%:*} MPIX_REDOP_WT_EVERY=${WT##*:} timeout -k 10 300 python3 bench.py \
        --no-cpu-baseline --no-extras > $O/b_${WT}_$i.json 2> $O/b_${WT}_$i.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/b_${WT}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']
print('WT=$WT', 'value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_ms', r['kernel_ms_avg'], 'frac', r['frac'], 'triad', r.get('triad_measured_GBs'), 'of_triad', r.get('frac_of_triad'))"
done
