# Round 3: the pageable workers' GPU side -- pinned operands in 16 MiB chunks
# from T threads vs one call, and where the buffers' pages sit.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3e
rm -rf $O && mkdir -p $O
timeout -k 10 300 env CHUNK_MIB=4,16,64,256 CHUNK_T=1,4 python3 tools/pinned_chunk_probe.py $O/r03_pinned_chunks.json > $O/probe.out 2> $O/probe.err
echo rc=$?
cat $O/probe.out; tail -3 $O/probe.err
