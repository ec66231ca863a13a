# Round 3: zero-copy rate on hipHostMalloc (4 KiB) vs THP-backed registered host memory
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3h
rm -rf $O && mkdir -p $O
timeout -k 10 300 python3 tools/thp_pinned_probe.py $O/r03_thp_pinned.json > $O/probe.out 2> $O/probe.err
echo rc=$?
cat $O/probe.out; tail -5 $O/probe.err; cat /sys/kernel/mm/transparent_hugepage/enabled
