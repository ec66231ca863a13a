# Round 3: zero-copy rate by page-locked memory kind (coherent / non-coherent / write-combined)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3j
rm -rf $O && mkdir -p $O
timeout -k 10 500 python3 tools/hostmem_kind_probe.py $O/r03_hostmem_kinds.json > $O/probe.out 2> $O/probe.err
echo rc=$?
cat $O/probe.out | head -8; tail -3 $O/probe.err
