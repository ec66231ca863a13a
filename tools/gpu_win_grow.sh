# Pull-window growth probe (tools/win_grow_probe.py): 4 ranks on the one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wg2
rm -rf $O && mkdir -p $O/base
timeout -k 10 300 python3 -u tools/win_grow_probe.py --ranks 4 --rounds 8 --mib 512 --out $O/base > $O/base.jsonl 2> $O/base.err
rc=$?
grep -h -A4 "reads" $O/base/r*_rank*.txt | head -40
exit $rc
