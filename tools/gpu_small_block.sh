# Block sizes 64 / 128 vs the shipped 256 (tools/small_block_probe.hip), two processes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/smallblk
rm -rf $O && mkdir -p $O
for i in 1 2; do timeout -k 10 120 tools/bin/small_block_probe >> $O/small_block.jsonl || exit $?; done
cat $O/small_block.jsonl
