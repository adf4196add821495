# One entry point for every GPU step (replaces round 1-5's ~80 one-off
# gpu_*.sh wrappers).  Each step has its own time limit; chain steps with &&
# in the gpurun command so the first failure ends the call:
#
#   bash scripts/gpu.sh suite                      GPU test suite, one process (as the driver runs it)
#   bash scripts/gpu.sh smoke                      __graft_entry__.smoke()
#   bash scripts/gpu.sh bench TAG [bench args]     bench.py line -> gpurun_out/TAG/bench.json
#   bash scripts/gpu.sh trace TAG [bench args]     rocprofv3 kernel trace + stats of bench.py --profile
#   bash scripts/gpu.sh pmc TAG NAME "COUNTERS" [args]
#                                                  one rocprofv3 --pmc pass of bench.py --profile -> gpurun_out/TAG/NAME
#   bash scripts/gpu.sh evidence TAG [args]        bench + trace + FETCH/WRITE + EA passes + SQ passes
#   bash scripts/gpu.sh kbab TAG VARIANTS [PMC_VARIANTS] [COUNTERS]
#                                                  tuning-build A/B (scripts/gpu_kbab.sh)
#   bash scripts/gpu.sh latency TAG lz4|zstd [N] [FRAME]
#                                                  single-frame latency probe under a kernel trace
#                                                  (scripts/latency_probe.py; FRAME bytes, default 64 KiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
step=$1; shift
case "$step" in
suite)
  mkdir -p gpurun_out/suite
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/suite/suite.log 2>&1 || { tail -40 gpurun_out/suite/suite.log; exit 1; }
  tail -2 gpurun_out/suite/suite.log ;;
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 ;;
bench)
  tag=$1; shift; mkdir -p gpurun_out/$tag
  timeout -k 10 600 python bench.py "$@" > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err \
      || { tail -20 gpurun_out/$tag/bench.err; exit 1; }
  cat gpurun_out/$tag/bench.json ;;
trace)
  tag=$1; shift; mkdir -p gpurun_out/$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/trace \
      -- python bench.py --profile --steps 5 --warmup 1 "$@" > gpurun_out/$tag/trace.log 2>&1 \
      || { tail -20 gpurun_out/$tag/trace.log; exit 1; }
  python3 scripts/kernel_stats.py gpurun_out/$tag/trace > gpurun_out/$tag/kernel_medians.csv 2>&1; head -12 gpurun_out/$tag/kernel_medians.csv ;;
pmc)
  tag=$1; name=$2; c=$3; shift 3; mkdir -p gpurun_out/$tag
  d=gpurun_out/$tag/$name
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -- python bench.py --profile --steps 2 --warmup 1 "$@" \
      > $d.log 2>&1 || { tail -5 $d.log; exit 1; } ;;
evidence)
  tag=$1; shift
  E1="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  E2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
  E3="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum"
  S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
  S2="SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES"
  bash scripts/gpu.sh bench $tag "$@" && bash scripts/gpu.sh trace $tag "$@" &&
  bash scripts/gpu.sh pmc $tag pmc_fetch FETCH_SIZE "$@" && bash scripts/gpu.sh pmc $tag pmc_write WRITE_SIZE "$@" &&
  bash scripts/gpu.sh pmc $tag ea_p1 "$E1" "$@" && bash scripts/gpu.sh pmc $tag ea_p2 "$E2" "$@" &&
  bash scripts/gpu.sh pmc $tag ea_p3 "$E3" "$@" &&
  bash scripts/gpu.sh pmc $tag p1 "$S1" "$@" && bash scripts/gpu.sh pmc $tag p2 "$S2" "$@" &&
  python3 scripts/pmc_summary.py gpurun_out/$tag > gpurun_out/$tag/sq_summary.txt 2>&1 &&
  echo "evidence $tag done" ;;
kbab)
  tag=$1; shift; bash scripts/gpu_kbab.sh $tag "$@" ;;
latency)
  tag=$1; codec=$2; n=${3:-300}; fr=${4:-65536}; mkdir -p gpurun_out/$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/lat_${codec}_$fr \
      -- python scripts/latency_probe.py $n $codec $fr > gpurun_out/$tag/lat_${codec}_$fr.log 2>&1 \
      || { tail -20 gpurun_out/$tag/lat_${codec}_$fr.log; exit 1; }
  grep -E "reads:" gpurun_out/$tag/lat_${codec}_$fr.log
  python3 scripts/kernel_stats.py gpurun_out/$tag/lat_${codec}_$fr --skip 20 | cut -d, -f1,2,4,7 | head -12 ;;
*)
  echo "unknown step $step"; exit 2 ;;
esac
