# Rehearse the N>1 bench flow on a 1-GPU box: 2 ranks share device 0, gloo
# control plane (RCCL-transport figures error out by design; replicas, IPC
# pull and the JSON line are exercised).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 240 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --steps 5 --warmup 2 --rsb-bytes 1073741824 > $O/r1_rehearse.json 2> $O/r1_rehearse.err
echo rc=$?
cat $O/r1_rehearse.json
tail -5 $O/r1_rehearse.err
