# Round 3: zero-copy (pinned operand) calls with a capped, grid-stride grid
# (MPIX_REDOP_MAXGRID) -- do reads and writes overlap better in small kernels?
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3i
rm -rf $O && mkdir -p $O
for G in 0 256 512 1024 2048; do
  timeout -k 10 200 env MPIX_REDOP_MAXGRID=$G CHUNK_MIB=16,64 CHUNK_T=1 python3 tools/pinned_chunk_probe.py $O/grid_$G.json > $O/grid_$G.out 2> $O/grid_$G.err
  rc=$?; echo "grid $G rc=$rc $(cat $O/grid_$G.out)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
