# Evidence pass for the headline kernel: rocprofv3 kernel-trace stats of the
# bench command, separate FETCH_SIZE / WRITE_SIZE PMC passes (summarised by
# tools/pmc_summary.py into the file bench.py quotes as roofline.traffic),
# then the default bench reading that summary.  R names the round's files.
# usage (on the GPU box): R=r03 bash tools/gpu_evidence.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${R:-r03}
O=gpurun_out/ev_$R
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/kt -o kt --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/prof_bench.json 2> $O/prof_bench.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/fetch -o fetch --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > /dev/null 2> $O/pmc_fetch.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/write -o write --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > /dev/null 2> $O/pmc_write.err && \
python3 tools/pmc_summary.py --kt "$(find $O/kt -name '*kernel_stats.csv' | head -n 1)" \
    --fetch "$(find $O/fetch -name '*counter_collection.csv' | head -n 1)" \
    --write "$(find $O/write -name '*counter_collection.csv' | head -n 1)" \
    --out $O/${R}_pmc_summary.json --stats-copy $O/${R}_rocprof_kernel_stats.csv \
    --trace "$(find $O/kt -name '*kernel_trace.csv' | head -n 1)" \
    --traced-line $O/prof_bench.json > /dev/null && \
timeout -k 10 500 python3 bench.py --pmc $O/${R}_pmc_summary.json > $O/bench.json 2> $O/bench.err
rc=$?
echo rc=$rc
cat $O/${R}_pmc_summary.json
head -c 1500 $O/bench.json
exit $rc
