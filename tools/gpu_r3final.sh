# Round 3 evidence on the final tree: the GPU suite + smoke (the driver's
# tier), the rocprofv3 / PMC evidence pass with the default bench, and the
# pageable path by size on the shipped defaults.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh > gpurun_out/full_summary.txt 2>&1
rc=$?
echo "full rc=$rc"; cat gpurun_out/full_summary.txt
if [ $rc -ge 124 ]; then exit $rc; fi
R=r03 bash tools/gpu_evidence.sh > gpurun_out/evidence_summary.txt 2>&1
rc=$?
echo "evidence rc=$rc"; tail -c 1500 gpurun_out/evidence_summary.txt
if [ $rc -ge 124 ]; then exit $rc; fi
O=gpurun_out/r3final
rm -rf $O && mkdir -p $O
for B in 134217728 1073741824; do
  timeout -k 10 400 env PAGEABLE_BYTES=$B PAGEABLE_CONFIGS=8:64:0:none:1:wave,8:128:0:none:1:wave,0:64:0:none:1:wave,8:16:0:none:1:worker python3 tools/pageable_probe.py sweep $O/r03_pageable_size_$B.jsonl > $O/size_$B.out 2> $O/size_$B.err
  rc=$?; echo "size $B rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
cat $O/r03_pageable_size_*.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print(d.get('bytes'), d.get('mode'), d.get('W'), d.get('chunk_MiB'), d.get('ms'), d.get('pinned_call_ms'), d.get('vs_pinned'), d.get('frac_of_pcie'), d.get('checked'), d.get('error','')[:200])
"
