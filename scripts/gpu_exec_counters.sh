# execute-kernel instruction counters per wave for kbench variants (tuning
# build): one PMC pass of SQ counters + one of VMEM / LDS-wait counters.
# $1: output dir, $2: kbench variants (run once each, in order).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-xcnt}
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/p1 -- python scripts/kbench.py --variants "$2" --rounds 1 --reps 1 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES --output-format csv -d $O/p2 -- python scripts/kbench.py --variants "$2" --rounds 1 --reps 1 > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
python3 scripts/exec_counters.py $O
