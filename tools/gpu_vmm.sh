# hipIpc vs VMM/POSIX-fd sharing between 4 processes on the one GPU (tools/vmm_ipc_probe.cpp).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/vmm
rm -rf $O && mkdir -p $O
timeout -k 10 120 tools/bin/vmm_ipc_probe 4 8 512 keep > $O/keep.jsonl 2> $O/keep.err &&
timeout -k 10 120 tools/bin/vmm_ipc_probe 4 8 512 free > $O/free.jsonl 2> $O/free.err &&
timeout -k 10 120 tools/bin/vmm_ipc_probe 8 6 256 keep > $O/keep8.jsonl 2> $O/keep8.err
rc=$?
cat $O/*.jsonl; tail -3 $O/*.err
exit $rc
