# quick iteration: GPU parity tests + kernel variant sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/kbench.py --variants ${VARIANTS:-0,1,2,3,4,5,6,7,8,9} --rounds 3 --reps 2 ${KARGS} 2>&1 | tee gpurun_out/kbench.log
