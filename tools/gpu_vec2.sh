set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/vec2
rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "vector or iov or Vector" \
    tests/test_gpu_parity.py tests/test_iovec.py tests/test_fuzz.py > $O/t.log 2>&1 && \
timeout -k 10 120 ./tools/bin/tune_vector2 > $O/timing.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- ./tools/bin/tune_vector2 > /dev/null 2> $O/pmc.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- ./tools/bin/tune_vector2 > /dev/null 2>> $O/pmc.err
rc=$?
tail -2 $O/t.log; cat $O/timing.txt
exit $rc
