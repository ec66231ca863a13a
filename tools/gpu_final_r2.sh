# Final-tree checks (round 2, last session): tile-map probe (one process), the
# N>1 bench flow rehearsed with four ranks on the one GPU (gloo control plane,
# staged transport; RCCL at N>1 needs one GPU per rank).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final_r2
rm -rf $O && mkdir -p $O
timeout -k 10 120 tools/bin/tile_map_probe > $O/tile_map.json 2> $O/tile_map.err &&
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 \
    --steps 3 --warmup 1 --rsb-bytes 536870912 > $O/n4.json 2> $O/n4.err
rc=$?
cat $O/tile_map.json
tail -c 600 $O/n4.json
exit $rc
