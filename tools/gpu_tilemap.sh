# Block -> tile mapping vs operand placement (tools/tile_map_probe.hip), three processes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tilemap
rm -rf $O && mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 tools/bin/tile_map_probe >> $O/tile_map.jsonl 2> $O/err$i.txt || exit $?
done
cat $O/tile_map.jsonl
