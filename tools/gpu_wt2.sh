# Store-policy evidence: patterns by XCD mask / block period across operand
# placements (tools/wt_probe.py), then every config-3 row with the policy off
# and on (tools/wt_types.py).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wtp
mkdir -p $O
timeout -k 10 400 python3 tools/wt_probe.py $O/wt_probe_xcd.json > $O/out2.txt 2> $O/err2.txt || { tail -5 $O/err2.txt; exit 1; }
cat $O/out2.txt
for P in ${TYPES_POLICIES:-0x88,0,0}; do
    timeout -k 10 600 python3 tools/wt_types.py $O/wt_types_$P.json $P > $O/types_$P.txt 2> $O/types_$P.err || { tail -5 $O/types_$P.err; exit 1; }
    cat $O/types_$P.txt
done
