# the synchronous entry's own store-policy mask (round 6
# default 0x22) against the stream-ordered default 0x88 for it, alternating
# processes, the default bench line (--no-extras: the headline loop, its
# kernel timing); then the store-policy GPU tests.  Outputs in
# gpurun_out/syncab/.  usage (gpurun): N=3 bash tools/gpu_sync_mask_ab.sh
# (MASKS="0x22 0x88 0x2a ..." sweeps other masks for the synchronous entry;
# "default" = the library's own; TESTS=0 skips the tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/syncab
mkdir -p $O
for i in $(seq 1 ${N:-3}); do
    for m in ${MASKS:-default 0x88}; do
        if [ $m = default ]; then unset MPIX_REDOP_WT_XCD_SYNC; else export MPIX_REDOP_WT_XCD_SYNC=$m; fi
        echo "run $i sync mask $m ($(date +%T))"
        timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --steps 100 \
            > $O/bench_${m}_$i.json 2> $O/bench_${m}_$i.err || exit 1
    done
done
unset MPIX_REDOP_WT_XCD_SYNC
[ "${TESTS:-1}" = 0 ] || timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_store_policy.py > $O/pytest_store_policy.log 2>&1 || exit 1
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/syncab/bench_*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['frac'],
          r['back_to_back']['kernel_ms_avg'], d['config'].get('store_policy_xcd_mask'))
PY
