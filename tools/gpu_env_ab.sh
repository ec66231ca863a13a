# A/B of two environment settings of the shipped library (e.g. launch
# geometry knobs), alternating processes: config-3 rows (tools/ab_types.py),
# the multi-input / tree folds (tools/multi_probe.py) and the default bench
# line.  Outputs in gpurun_out/envab/.
# usage (gpurun): A="MPIX_REDOP_BLOCK=256" B="MPIX_REDOP_BLOCK=64" bash tools/gpu_env_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/envab
mkdir -p $O
for i in 1 2; do
    for v in A B; do
        eval "settings=\$$v"
        echo "run $i $v: $settings ($(date +%T))"
        env $settings timeout -k 10 300 python3 tools/ab_types.py mpich_amd/libmpix_redop.so $v \
            >> $O/types.jsonl 2>> $O/types.err || exit 1
        env $settings timeout -k 10 120 python3 tools/multi_probe.py --ks 1,3,7,15 --tree-ks 2,4,8,16 \
            > $O/multi_${v}_$i.json 2>> $O/multi.err || exit 1
        env $settings timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_${v}_$i.json \
            2> $O/bench_${v}_$i.err || exit 1
    done
done
