# GPU command file: run the named steps in order on the GPU box, each under its
# own time limit, stopping at the first that fails.  Outputs under
# gpurun_out/steps/ (copied into profiles/ by hand when kept).
# usage (gpurun): bash tools/gpu_steps.sh <step> [<step> ...]
#   tests=<pytest -k expr>  the -m gpu tests matching the expression
#   gputests                the whole -m gpu suite (the driver's tier)
#   smoke                   __graft_entry__.smoke()
#   rehearse                bench.py --gpus 4 on the one GPU (gloo, shared device)
#   swing                   tools/pageable_swing.py, default and GPU-node worker affinity
#   floor                   tools/call_floor.py
#   policy                  tools/policy_concurrent.py
#   pgrid                   tools/pinned_grid.py: zero-copy calls against the grid cap
#   pmcmulti                FETCH/WRITE passes over tools/multi_probe.py (multi-input and tree)
#   bench                   the default bench.py line
#   pmcwide                 tools/pmc_wide.py: FETCH/WRITE passes over the 32-byte-unit kernels
#   evidence                tools/gpu_evidence.sh (R=r04): rocprofv3 stats + PMC passes + bench
#   pmctree                 FETCH/WRITE passes over the tree folds k = 8, 16 (default form)
# (round 5's treeab / treeab2 / treeab3 steps A/B-ed two library knobs since removed;
#  their results are profiles/r05_tree_knob_ab.json, the step text in git history)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/steps
mkdir -p $O
run() {     # run <name> <seconds> <command...>: stdout to $O/<name>.out, stderr to .err
    local name=$1 secs=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
    local rc=$?
    echo "== $name rc=$rc"
    tail -3 $O/$name.out
    if [ $rc -ne 0 ]; then tail -20 $O/$name.err; fi
    return $rc
}
for step in "$@"; do
    case $step in
        tests=*) run tests 600 python3 -u -m pytest tests -x -q -m gpu -k "${step#tests=}" \
                     --timeout 200 --timeout-method thread -p no:cacheprovider || exit $? ;;
        gputests) run gputests 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 \
                     --timeout-method thread -p no:cacheprovider || exit $? ;;
        smoke) run smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
        rehearse) run rehearse 1100 env P=4 bash tools/gpu_rehearse.sh || exit $? ;;
        swing) run swing_default 300 python3 tools/pageable_swing.py --label default || exit $?
               run swing_gpuaff 300 env MPIX_REDOP_PAGEABLE_AFFINITY=gpu python3 \
                   tools/pageable_swing.py --label gpu_affinity || exit $? ;;
        swingchunk) run swing_c16 300 python3 tools/pageable_swing.py --label chunk16 --chunk 16 \
                        --sizes 32,48,64,128 || exit $?
                    run swing_c8 300 python3 tools/pageable_swing.py --label chunk8 --chunk 8 \
                        --sizes 16,24,32,64 || exit $? ;;
        floor) run floor 200 python3 tools/call_floor.py || exit $? ;;
        policy) run policy 300 python3 tools/policy_concurrent.py || exit $? ;;
        pgrid) run pgrid 300 python3 tools/pinned_grid.py || exit $? ;;
        pmcmulti) run pmcmulti_fetch 180 rocprofv3 --pmc FETCH_SIZE -T -d $O/pm_fetch -o f \
                      --output-format csv -- python3 tools/multi_probe.py || exit $?
                  run pmcmulti_write 180 rocprofv3 --pmc WRITE_SIZE -T -d $O/pm_write -o w \
                      --output-format csv -- python3 tools/multi_probe.py || exit $?
                  run pmcmulti_sum 60 python3 tools/pmc_multi.py \
                      "$(find $O/pm_fetch -name '*counter_collection.csv' | head -n 1)" \
                      "$(find $O/pm_write -name '*counter_collection.csv' | head -n 1)" \
                      $O/r04_pmc_multi.json || exit $? ;;
        bench) run bench 600 python3 bench.py || exit $? ;;
        pmctree) run pmctree_fetch 180 rocprofv3 --pmc FETCH_SIZE -T -d $O/pt_fetch -o f \
                     --output-format csv -- python3 tools/multi_probe.py --ks 7 --tree-ks 8,16 || exit $?
                 run pmctree_write 180 rocprofv3 --pmc WRITE_SIZE -T -d $O/pt_write -o w \
                     --output-format csv -- python3 tools/multi_probe.py --ks 7 --tree-ks 8,16 || exit $?
                 run pmctree_sum 60 python3 tools/pmc_multi.py \
                     "$(find $O/pt_fetch -name '*counter_collection.csv' | head -n 1)" \
                     "$(find $O/pt_write -name '*counter_collection.csv' | head -n 1)" \
                     $O/r05_pmc_tree8.json --ks 7 --tree-ks 8,16 || exit $? ;;
        pmcwide) run pmcwide_run 120 python3 tools/pmc_wide.py || exit $?
                 run pmcwide_fetch 120 rocprofv3 --pmc FETCH_SIZE -T -d $O/pw_fetch -o f \
                     --output-format csv -- python3 tools/pmc_wide.py || exit $?
                 run pmcwide_write 120 rocprofv3 --pmc WRITE_SIZE -T -d $O/pw_write -o w \
                     --output-format csv -- python3 tools/pmc_wide.py || exit $?
                 tail -n 1 $O/pmcwide_run.out > $O/pmcwide_run.json
                 run pmcwide_sum 60 python3 tools/pmc_wide.py --summarise \
                     "$(find $O/pw_fetch -name '*counter_collection.csv' | head -n 1)" \
                     "$(find $O/pw_write -name '*counter_collection.csv' | head -n 1)" \
                     $O/r04_pmc_wide.json $O/pmcwide_run.json || exit $? ;;
        evidence) run evidence 1100 env R=${R:-r04} bash tools/gpu_evidence.sh || exit $? ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
