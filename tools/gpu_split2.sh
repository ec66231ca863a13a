# Placement study for the per-process split: operand
# offsets inside one allocation vs separate allocations, for the combine and
# the triad; then DRAM-side stall counters of one-slab vs separate placement.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/split2
rm -rf $O && mkdir -p $O
for i in 0 1 2; do
    timeout -k 10 120 python3 tools/split_probe.py offsets$i >> $O/offsets.jsonl 2>> $O/probe.err || exit $?
done
for i in 0 1; do
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum \
        -d $O/pmc_c$i -o c --output-format csv -- python3 tools/split_probe.py pmc_c$i \
        >> $O/probe_pmc.jsonl 2>> $O/pmc.err || exit $?
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_BUBBLE_sum \
        -d $O/pmc_d$i -o d --output-format csv -- python3 tools/split_probe.py pmc_d$i \
        >> $O/probe_pmc.jsonl 2>> $O/pmc.err || exit $?
done
cat $O/offsets.jsonl $O/probe_pmc.jsonl
