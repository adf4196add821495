# round 5 evidence: default bench line (config 2, with its CPU baseline,
# end-to-end and latency), rocprofv3 kernel trace of the same command, PMC
# passes (FETCH_SIZE, WRITE_SIZE, the L2 EA request counters in three passes,
# two SQ passes); the same for config 5 (zstd); config-3 sweep lines and the
# 1 MiB trace; single-frame latency traces (LZ4, zstd).  Each GPU step has its
# own time limit; steps chained with &&.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/round5
Z=gpurun_out/zround5
S=gpurun_out/sweep5
mkdir -p $O $Z $S
E1="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
E2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
E3="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum"
pmc() {   # $1 dir, $2 counters, rest: the bench arguments
  local d=$1 c=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -- python bench.py --profile --steps 2 --warmup 1 "$@" > $d.log 2>&1
}
part1() {
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --profile --steps 5 --warmup 1 > $O/trace.log 2>&1 &&
pmc $O/pmc_fetch FETCH_SIZE && pmc $O/pmc_write WRITE_SIZE &&
pmc $O/ea_p1 "$E1" && pmc $O/ea_p2 "$E2" && pmc $O/ea_p3 "$E3" &&
pmc $O/p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" &&
pmc $O/p2 "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES" &&
python3 scripts/pmc_summary.py $O > $O/sq_summary.txt 2>&1 &&
echo "config 2 profiles done"
rc=$?
[ "$1" = "c2" ] && exit $rc
[ $rc -eq 0 ] || exit $rc
}
part2() {
timeout -k 10 600 python bench.py --codec zstd > $Z/bench.json 2> $Z/bench.err && cat $Z/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $Z/trace -- python bench.py --codec zstd --profile --steps 5 --warmup 1 > $Z/trace.log 2>&1 &&
pmc $Z/pmc_fetch FETCH_SIZE --codec zstd && pmc $Z/pmc_write WRITE_SIZE --codec zstd &&
pmc $Z/ea_p1 "$E1" --codec zstd && pmc $Z/ea_p2 "$E2" --codec zstd && pmc $Z/ea_p3 "$E3" --codec zstd &&
echo "config 5 profiles done" &&
timeout -k 10 400 python bench.py --frame 4096 --steps 5 --warmup 2 --no-e2e > $S/f4096.json 2> $S/f4096.err && cat $S/f4096.json &&
timeout -k 10 400 python bench.py --frame 1048576 --steps 5 --warmup 2 --no-e2e > $S/f1048576.json 2> $S/f1048576.err && cat $S/f1048576.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $S/trace1m -- python bench.py --frame 1048576 --profile --steps 5 --warmup 1 > $S/trace1m.log 2>&1 &&
bash scripts/gpu_latency_probe.sh round5/lat_lz4 lz4 300 > /dev/null && grep reads: $O/lat_lz4/probe.log &&
bash scripts/gpu_latency_probe.sh round5/lat_zstd zstd 300 > /dev/null && grep reads: $O/lat_zstd/probe.log
}
# $1: c2 (config 2 part), rest (config 5, sweeps, latency), or both (default)
case "${1:-both}" in
  c2) part1 c2 ;;
  rest) part2 ;;
  *) part1 && part2 ;;
esac
