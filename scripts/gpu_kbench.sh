set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python scripts/kbench.py --variants ${VARIANTS:-0,1,2,3,4,5,6} --rounds 3 --reps 2 ${KARGS} 2>&1 | tee gpurun_out/kbench.log
