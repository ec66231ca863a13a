# Config 2 with the final kernel: bench.py --sweep (16 MiB-1 GiB sizes, chunked
# async, HIP-graph replay) and rocprofv3 kernel stats of the same command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sweep_r2
rm -rf $O && mkdir -p $O
timeout -k 10 400 python3 bench.py --sweep --no-cpu-baseline > $O/sweep.json 2> $O/sweep.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/kt -o kt --output-format csv -- \
    python3 bench.py --sweep --no-cpu-baseline --no-extras --steps 20 > $O/prof_sweep.json 2> $O/prof_sweep.err
rc=$?
find $O/kt -name '*kernel_stats.csv' -exec cp {} $O/r02_rocprof_sweep_kernel_stats.csv \;
head -5 $O/r02_rocprof_sweep_kernel_stats.csv | cut -c1-300
python3 -c "
import json
d=json.loads(open('$O/sweep.json').read().strip().splitlines()[-1])
print(d['roofline']['frac'], d['sweep'])
"
exit $rc
