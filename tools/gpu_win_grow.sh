# Pull-window growth with the shipped one-at-a-time exports: multi-process GPU
# tests of the pulls, 12 probe rounds (tools/win_grow_probe.py), then the
# four-rank rehearsal of the N>1 bench flow.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wg4
rm -rf $O && mkdir -p $O/serial
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_coll_multiproc.py tests/test_ipc_gpu.py > $O/t.log 2>&1 &&
tail -2 $O/t.log &&
timeout -k 10 300 python3 -u tools/win_grow_probe.py --ranks 4 --rounds 12 --mib 512 --out $O/serial > $O/serial.jsonl 2> $O/serial.err &&
MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 \
    --steps 3 --warmup 1 --rsb-bytes 536870912 > $O/n4.json 2> $O/n4.err
rc=$?
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/serial.jsonl') if l.startswith('{')]
print('serial', [r['failed_attempts'] for r in rows], 'bad rounds', sum(1 for r in rows if r['bad']))
"
tail -c 700 $O/n4.json
exit $rc
