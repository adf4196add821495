# round 4 baseline diagnostics at config 2: SQ instruction counters of the
# LZ4 kernels (two PMC passes of <= 8 SQ counters each), then the tuning
# build's interleaved variants: production, parse-only per route, execute
# only, execute section timers (0x110), lean sub-step counters (0x204).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04diag
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -- python bench.py --profile --steps 2 --warmup 1 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES --output-format csv -d $O/p2 -- python bench.py --profile --steps 2 --warmup 1 > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
python3 scripts/pmc_summary.py $O > $O/summary.txt 2>&1
timeout -k 10 400 python scripts/kbench.py --variants 0,12,13,14,20,272,516 --rounds 3 > $O/kb.log 2>&1 || { tail -30 $O/kb.log; exit 1; }
cat $O/summary.txt $O/kb.log
