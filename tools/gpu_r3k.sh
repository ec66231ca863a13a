# Session 2 of round 3: the restored tree re-verified (GPU suite + smoke +
# default bench), then the AQL direct-dispatch probe (tools/aql_probe.hip).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3k
bash tools/gpu_full.sh
rc=$?; echo "full rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py > gpurun_out/r3k/bench.json 2> gpurun_out/r3k/bench.err
rc=$?; echo "bench rc=$rc"; head -c 2500 gpurun_out/r3k/bench.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 90 tools/bin/aql_probe 50 > gpurun_out/r3k/aql_probe.json 2> gpurun_out/r3k/aql_probe.err
rc=$?; echo "aql rc=$rc"; cat gpurun_out/r3k/aql_probe.err | tail -5; cat gpurun_out/r3k/aql_probe.json
exit $rc
