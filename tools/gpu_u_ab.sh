# A/B of the contiguous kernel's packets per lane (MPIX_REDOP_UNROLL) through
# the library: the shipped build against one built with another unroll,
#   make -C mpich_amd/csrc BUILD=build_alt OUT=../libmpix_redop_alt.so \
#        EXTRA_FLAGS=-DMPIX_REDOP_UNROLL=4 ../libmpix_redop_alt.so
# (round 5 ran it with the shipped U = 4 against an alternative U = 1, which
# then became the default: profiles/r05_unroll_ab.json).  Alternating
# processes: tools/contig_u_probe.hip, config-3 rows (tools/ab_types.py) and the
# default bench line (the box's copy of libmpix_redop.so swapped per run).
# Outputs in gpurun_out/uab/.   usage (gpurun): bash tools/gpu_u_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/uab
mkdir -p $O
cp mpich_amd/libmpix_redop.so $O/../shipped.so.keep
timeout -k 10 100 tools/bin/contig_u_probe 1024 > $O/contig_u.json || exit 1
for i in 1 2; do
    for v in shipped alt; do
        lib=mpich_amd/libmpix_redop_alt.so; [ $v = shipped ] && lib=$O/../shipped.so.keep
        echo "types $v run $i ($(date +%T))"
        timeout -k 10 300 python3 tools/ab_types.py $lib $v >> $O/types.jsonl 2>> $O/types.err || exit 1
    done
done
for i in 1 2; do
    for v in shipped alt; do
        lib=mpich_amd/libmpix_redop_alt.so; [ $v = shipped ] && lib=$O/../shipped.so.keep
        cp $lib mpich_amd/libmpix_redop.so
        echo "bench $v run $i ($(date +%T))"
        timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    done
done
cp $O/../shipped.so.keep mpich_amd/libmpix_redop.so
rm -f $O/../shipped.so.keep
