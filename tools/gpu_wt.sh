# A/B of MPIX_REDOP_WT_TAIL (the last N blocks of the contiguous kernel store
# write-through, leaving less dirty in the XCD L2s for the end-of-kernel
# write-back): the synchronous 1 GiB call split on the GPU clock
# (tools/sync_gap.py under rocprofv3 --kernel-trace), settings alternating in
# separate processes.  Writes gpurun_out/wt/<setting>_<i>.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wt
rm -rf $O && mkdir -p $O
i=0
# a setting is TAIL or TAIL:EVERY (MPIX_REDOP_WT_TAIL, MPIX_REDOP_WT_EVERY)
for WT in ${WT_LIST:-0 2048 0 2048 8192 0 8192}; do
    i=$((i+1))
    D=$O/tr_${WT}_$i
    TAIL=${WT%%:*}; EVERY=0
    case $WT in *:*) EVERY=${WT##*:};; esac
    MPIX_REDOP_WT_TAIL=$TAIL MPIX_REDOP_WT_EVERY=$EVERY timeout -k 10 200 rocprofv3 --kernel-trace -d $D -o tr --output-format csv -- \
        python3 tools/sync_gap.py run $O/host_${WT}_$i.json 40 > $O/run_${WT}_$i.out 2>&1 || exit $?
    python3 tools/sync_gap.py report $O/host_${WT}_$i.json "$(find $D -name '*kernel_trace.csv' | head -n 1)" \
        $O/${WT}_$i.json > /dev/null || exit $?
    python3 -c "
import json; d=json.load(open('$O/${WT}_$i.json')); m=d['median_us']
print('WT=$WT', 'kernel', m['kernel'], 'end_to_signal', m.get('end_to_signal'), 'signal', m.get('signal'), 'to_next', m.get('signal_to_next_kernel'), 'host_call', m['host_call'], 'overhead', d['overhead_us'])"
    rm -rf $D
done
