# Memory-side counters of the contiguous kernel with the store policy off
# (mask 0) and on (0x88): DRAM credit stalls and queue levels of the L2 -> EA
# requests, then request counts and L2 hits, one rocprofv3 --pmc pass per
# counter group (<= 4 TCC counters a pass).  Summarised by the python at the end.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wtpmc
rm -rf $O && mkdir -p $O
for M in 0 0x88; do
    i=0
    for G in "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum" \
             "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" \
             "GRBM_GUI_ACTIVE TCC_EA0_WRREQ_64B_sum"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $G -d $O/m${M}_g$i -o p --output-format csv -- \
            python3 tools/wt_pmc.py $M > $O/m${M}_g$i.out 2>&1 || { echo "pass $M $i failed"; tail -5 $O/m${M}_g$i.out; exit 1; }
    done
done
python3 - <<'PY'
import csv, glob, json, collections
res = {}
for path in sorted(glob.glob('gpurun_out/wtpmc/m*_g*/**/*counter_collection.csv', recursive=True)):
    key = path.split('/')[2].split('_')[0]
    rows = [r for r in csv.DictReader(open(path)) if 'k_contig' in r.get('Kernel_Name', '')]
    per = collections.defaultdict(list)
    for r in rows:
        per[r['Counter_Name']].append(float(r['Counter_Value']))
    for c, v in per.items():
        # one value per kernel dispatch (dimension-summed): median over dispatches
        v.sort()
        res.setdefault(key, {})[c] = v[len(v) // 2]
json.dump(res, open('gpurun_out/wtpmc/summary.json', 'w'), indent=1)
print(json.dumps(res))
PY
