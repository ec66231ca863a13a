# Collective GPU tests after the window/stream changes, then the four-rank rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/coll_r2
rm -rf $O && mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py tests/test_ipc_gpu.py tests/test_coll_c.py tests/test_coll_fuzz.py tests/test_support.py > $O/t.log 2>&1 &&
tail -2 $O/t.log &&
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 \
    --steps 3 --warmup 1 --rsb-bytes 536870912 > $O/n4.json 2> $O/n4.err
rc=$?
tail -3 $O/t.log
python3 -c "
import json
d=json.loads(open('$O/n4.json').read().strip().splitlines()[-1])
print({k: v['ms'] for k, v in d['reduce_scatter_block_other'].items()})
print({k: v for k, v in d['allreduce'].items() if isinstance(v, dict)})
" || true
exit $rc
