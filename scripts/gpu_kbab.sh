# Execute / decode A/B on the tuning build: kbench of $2 (interleaved rounds),
# then one rocprofv3 --pmc pass per variant in $3 with counters $4 (default:
# VALU / SALU / LDS instructions, waves, wave cycles, LDS waits), summarized
# per kernel by scripts/pmc_variants.py.  $1: output directory under gpurun_out.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-kbab}
mkdir -p $O
C=${4:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"}
timeout -k 10 400 python scripts/kbench.py --variants "$2" --rounds ${ROUNDS:-5} $KBARGS > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
cat $O/kbench.log
for v in $(echo "$3" | tr ',' ' '); do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$v -- python scripts/kbench.py --variants 10,$v --rounds 1 --reps 1 $KBARGS > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
done
[ -z "$3" ] || python3 scripts/pmc_variants.py $O
