# Round 3, second GPU session: the whole -m gpu suite on the new kernels
# (tile loads before combines, deferred Annex G fixup, packed fp16 complex
# product, SWAR 1-byte logicals) and the double-buffered pageable workers;
# then the config-3 A/B again, the C3 parity sweep at 256 MiB, and the
# pageable sweep.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b
rm -rf $O && mkdir -p $O
step() {    # name timeout cmd...: stop the script on a fault / abort / time limit
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
    local rc=$?
    echo "$name rc=$rc" | tee -a $O/steps.txt
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
step suite 900 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider
step c3 300 env MPIX_PARITY_BYTES=268435456 python3 -u -m pytest tests/test_c3_full.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
step ab_new1 200 python3 tools/ab_types.py mpich_amd/libmpix_redop.so r03b
step ab_old1 200 python3 tools/ab_types.py tools/bin/r02k/libmpix_redop.so r02
step ab_new2 200 python3 tools/ab_types.py mpich_amd/libmpix_redop.so r03b
step ab_old2 200 python3 tools/ab_types.py tools/bin/r02k/libmpix_redop.so r02
step pageable 900 python3 tools/pageable_probe.py sweep $O/r03_pageable_sweep.jsonl
cat $O/steps.txt
tail -n 3 $O/suite.out
tail -n 2 $O/c3.out
python3 -c "
import json
for f in ('ab_new1','ab_old1','ab_new2','ab_old2'):
    try:
        d=json.loads(open('$O/%s.out'%f).read().strip().splitlines()[-1]); print(f, d['fp32_sum_ms'], d['min_vs_fp32_sum'], d['within_2pct'], d['rows'], [(r['type'],r['op'],r['vs_fp32_sum']) for r in d['slowest'][:6]])
    except Exception as e: print(f, e)
"
cat $O/pageable.out
