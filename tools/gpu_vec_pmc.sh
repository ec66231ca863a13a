# config-5 variants: timing again + FETCH_SIZE / WRITE_SIZE per kernel (separate passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/vecpmc
rm -rf $O && mkdir -p $O
timeout -k 10 120 ./tools/bin/tune_vector2 > $O/timing.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- ./tools/bin/tune_vector2 > /dev/null 2> $O/pmc.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- ./tools/bin/tune_vector2 > /dev/null 2>> $O/pmc.err
rc=$?
cat $O/timing.txt
exit $rc
