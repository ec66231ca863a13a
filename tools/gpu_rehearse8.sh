# Eight-rank rehearsal of the N>1 bench flow on the one GPU (gloo control plane,
# staged transport): multipath at P = 8, pulls with 8 windows exported one at a time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/n8
rm -rf $O && mkdir -p $O
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 700 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 \
    --steps 3 --warmup 1 --count 67108864 --rsb-bytes 268435456 > $O/n8.json 2> $O/n8.err
rc=$?
echo rc=$rc
python3 -c "
import json
d=json.loads(open('$O/n8.json').read().strip().splitlines()[-1])
print('value', d.get('value'), 'error', d.get('error'), 'parity', d.get('parity'))
print({k: (v.get('ms'), v.get('bit_identical_to')) for k, v in d.get('reduce_scatter_block_other', {}).items() if isinstance(v, dict)})
print({k: v for k, v in d.get('allreduce', {}).items()})
" || tail -20 $O/n8.err
exit $rc
