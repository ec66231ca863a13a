# Round 3: where the zero-copy per-call ramp sits -- kernel trace of pinned
# 16 MiB / 64 MiB chunked calls (kernel durations vs gaps between kernels)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3k
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 tools/pinned_chunk_probe.py $O/chunks.json > $O/probe.out 2> $O/probe.err
echo rc=$?
python3 - <<'PY'
import csv, glob, json, statistics
f = glob.glob('gpurun_out/r3k/kt/**/*kernel_trace.csv', recursive=True)[0]
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], int(r['Grid_Size_X'])) for r in csv.DictReader(open(f)))
ks = [e for e in ev if 'k_contig' in e[2]]
by = {}
for i, e in enumerate(ks):
    by.setdefault(e[3], []).append(e)
out = {}
for g, lst in sorted(by.items()):
    d = [(e[1] - e[0]) / 1e3 for e in lst]
    gaps = [(lst[i + 1][0] - lst[i][1]) / 1e3 for i in range(len(lst) - 1)]
    out[g] = dict(n=len(lst), dur_us_median=round(statistics.median(d), 1), gap_us_median=round(statistics.median(gaps), 1) if gaps else None)
print(json.dumps(out))
json.dump(out, open('gpurun_out/r3k/r03_zero_copy_trace.json', 'w'), indent=1)
PY
cat $O/probe.out
