# LZ4 kernels' SQ counters (config 2) (two passes of <= 8 SQ counters), pipeline off
# (one chunk, one stream) so each kernel runs alone
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lpmc
mkdir -p $O

timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -- python bench.py --profile --steps 2 --warmup 1 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM --output-format csv -d $O/p2 -- python bench.py --profile --steps 2 --warmup 1 > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
python3 scripts/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
