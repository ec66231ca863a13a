# Rehearsal of the N>1 bench flow on the one-GPU box (every rank on device 0,
# gloo control plane, staged transport -- RCCL refuses two ranks on one GPU):
# the line must show `schedule_ran` for every leg.  Run twice: as is, and with
# MPIX_COLL_WINDOW_FAULT=1 (rank 1 publishes a window its memory does not
# hold), where every pull leg must be reported as "fell back to ..." and not
# timed under the pull's name.
# usage (on the GPU box): P=4 bash tools/gpu_rehearse.sh
# (RSB=<bytes per rank> STEPS=<k> MODES="normal" for the full-size form: round 5
# ran P=8 RSB=4294967296 STEPS=2 MODES=normal, the driver's N = 8 shape;
# LAUNCH=torchrun starts the ranks with python -m torch.distributed.run, the
# driver's launcher, instead of bench.py's own)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${P:-4}
RSB=${RSB:-268435456}
STEPS=${STEPS:-3}
MODES=${MODES:-normal fault}
O=gpurun_out/rehearse
rm -rf $O && mkdir -p $O
summ() {
python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('value', d.get('value'), 'schedule_ran', d.get('schedule_ran'), 'error', d.get('error'))
for sec in ('reduce_scatter_block_other', 'allreduce'):
    for k, v in d.get(sec, {}).items():
        if isinstance(v, dict):
            print(' ', sec, k, 'ran:', v.get('schedule_ran'), 'ms:', v.get('ms'), 'error:', v.get('error'))
" $1
}
for mode in $MODES; do
    if [ $mode = fault ]; then export MPIX_COLL_WINDOW_FAULT=1; fi
    # bench.py starts the P ranks itself, or (LAUNCH=torchrun) torch.distributed.run does
    L="python3"
    if [ "${LAUNCH:-self}" = torchrun ]; then
        L="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 --master-port 29517"
    fi
    MPIX_BENCH_SAME_DEVICE=1 MPIX_BENCH_BACKEND=gloo timeout -k 10 ${LIMIT:-500} $L bench.py --gpus $P \
        --steps $STEPS --warmup 1 --ab-reps 1 --count 67108864 --rsb-bytes $RSB $BENCH_ARGS \
        > $O/n${P}_$mode.json 2> $O/n${P}_$mode.err
    rc=$?
    echo "$mode rc=$rc"
    summ $O/n${P}_$mode.json || tail -20 $O/n${P}_$mode.err
    if [ $rc -ne 0 ]; then exit $rc; fi
done
