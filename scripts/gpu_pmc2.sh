# PMC passes (one rocprofv3 run each, no tracing) over kbench variants; the
# counter sets are in $SETS separated by '|'.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_OUT:-pmc2}
mkdir -p $OUT
V=${VARIANTS:-0}
K=${PMC_CMD:-"python scripts/kbench.py --size 1073741824 --variants $V --rounds 1 --reps 1"}
SETS=${SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY|SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum|FETCH_SIZE"}
IFS='|' read -ra ARR <<< "$SETS"
i=0
for set in "${ARR[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -- $K > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $OUT | tee $OUT/summary.txt
