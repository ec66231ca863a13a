# Round 3, first GPU session: the new tests (peer access, schedule state,
# P=2 in-place, knob independence, window/node fault reporting), the config-3
# A/B (round-2 kernels vs sched_barrier + deferred Annex G fixup), NaN payload
# record, the synchronous-call gap under a kernel trace, the default bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3a
rm -rf $O && mkdir -p $O
step() {    # name timeout cmd...: stop the script on a fault / abort / time limit
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
    local rc=$?
    echo "$name rc=$rc" | tee -a $O/steps.txt
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
(cat /sys/fs/cgroup/cpu.max; nproc; lscpu | head -30; numactl -H 2>/dev/null | head -20;
 python3 -c "import torch; p=torch.cuda.get_device_properties(0); print(p.pci_bus_id, p.pci_device_id, p.pci_domain_id)";
 for d in /sys/bus/pci/devices/*; do if [ -f $d/class ] && grep -q 0x038 $d/class 2>/dev/null; then echo $d $(cat $d/numa_node) $(cat $d/local_cpulist 2>/dev/null); fi; done) > $O/env.txt 2>&1
step tests 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_peer_gpu.py tests/test_coll_multiproc.py::test_staged_pull_window_verification_failure \
    tests/test_coll_c.py -k "peer or nan or window_verification or in_place_overlap or ignore_support or state_on_device or distinct_devices or same_device"
step ab_new1 200 python3 tools/ab_types.py mpich_amd/libmpix_redop.so r03
step ab_old1 200 python3 tools/ab_types.py tools/bin/r02k/libmpix_redop.so r02
step ab_new2 200 python3 tools/ab_types.py mpich_amd/libmpix_redop.so r03
step ab_old2 200 python3 tools/ab_types.py tools/bin/r02k/libmpix_redop.so r02
step nan 200 python3 tools/nan_payload_probe.py $O/r03_nan_payloads.json
step syncgap 200 rocprofv3 --kernel-trace -d $O/sg -o sg --output-format csv -- python3 tools/sync_gap.py run $O/sync_host.json 40
python3 tools/sync_gap.py report $O/sync_host.json "$(find $O/sg -name '*kernel_trace.csv' | head -n 1)" $O/r03_sync_gap.json > $O/sync_report.out 2>&1
step bench 500 python3 bench.py
cat $O/steps.txt
tail -n 3 $O/tests.out
python3 -c "
import json
for f in ('ab_new1','ab_old1','ab_new2','ab_old2'):
    try:
        d=json.loads(open('$O/%s.out'%f).read().strip().splitlines()[-1]); print(f, d['fp32_sum_ms'], d['min_vs_fp32_sum'], d['within_2pct'], d['rows'], [(r['type'],r['op'],r['vs_fp32_sum']) for r in d['slowest'][:5]])
    except Exception as e: print(f, e)
"
cat $O/sync_report.out
head -c 600 $O/bench.out
