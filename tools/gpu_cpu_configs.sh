# CPU baselines for BASELINE configs 2-5 on the GPU box's host cores (no GPU work).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python3 tools/cpu_configs.py > gpurun_out/s3_cpu_configs.json 2> gpurun_out/s3_cpu_configs.err
rc=$?
tail -n 3 gpurun_out/s3_cpu_configs.err
exit $rc
