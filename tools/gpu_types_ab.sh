# A/B of config-3 rows: the shipped library against mpich_amd/libmpix_redop_alt.so (a copy of
# the previous build), after the parity tests that cover the change.  usage (gpurun): bash tools/gpu_types_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh "tests=random_parity or c3 or golden_on_gpu or batch or fuzz" || exit 1
O=gpurun_out/${OUT:-uab2}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 tools/ab_types.py mpich_amd/libmpix_redop.so ${LA:-shipped} >> $O/types.jsonl || exit 1
  timeout -k 10 300 python3 tools/ab_types.py mpich_amd/libmpix_redop_alt.so ${LB:-alt} >> $O/types.jsonl || exit 1
done
