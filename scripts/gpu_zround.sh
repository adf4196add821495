# zstd round evidence (config 5): GPU zstd tests, bench, rocprofv3 kernel
# trace + PMC passes of the same bench command.  Each GPU step has its own
# time limit and the steps are chained with &&.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zround
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log &&
timeout -k 10 600 python bench.py --codec zstd > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --codec zstd --profile --steps 5 --warmup 1 > $O/trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python bench.py --codec zstd --profile --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python bench.py --codec zstd --profile --steps 2 --warmup 1 > $O/pmc_write.log 2>&1
rc=$?
find $O -name "*.csv" | head -20
exit $rc
