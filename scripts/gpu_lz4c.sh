# GPU LZ4 compression: bench line, kernel trace, HBM
# traffic passes (FETCH_SIZE / WRITE_SIZE separately) and SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lz4c
mkdir -p $O
timeout -k 10 300 python bench.py --codec lz4c --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --codec lz4c --profile --steps 5 --warmup 1 > $O/trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python bench.py --codec lz4c --profile --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python bench.py --codec lz4c --profile --steps 2 --warmup 1 > $O/pmc_write.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/sq -- python bench.py --codec lz4c --profile --steps 2 --warmup 1 > $O/sq.log 2>&1
rc=$?
cat $O/bench.json
find $O -name "*kernel_stats.csv" | head -1 | xargs cat
exit $rc
