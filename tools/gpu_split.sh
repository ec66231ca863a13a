# Per-process kernel split: 10 fresh processes, each timing
# the shipped combine, the STREAM triad and a one-slab placement; then the
# gfx950 counter list and two PMC passes over more probe processes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/split
rm -rf $O && mkdir -p $O
for i in 0 1 2 3 4 5 6 7 8 9; do
    timeout -k 10 90 python3 tools/split_probe.py seq$i >> $O/probe.jsonl 2>> $O/probe.err || exit $?
done
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for i in 0 1 2; do
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT \
        -d $O/pmc_a$i -o a --output-format csv -- python3 tools/split_probe.py pmc_a$i \
        >> $O/probe_pmc.jsonl 2>> $O/pmc.err || exit $?
    timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum \
        -d $O/pmc_b$i -o b --output-format csv -- python3 tools/split_probe.py pmc_b$i \
        >> $O/probe_pmc.jsonl 2>> $O/pmc.err || exit $?
done
cat $O/probe.jsonl $O/probe_pmc.jsonl
