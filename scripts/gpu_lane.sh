set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kbench.py --variants 50,30 --rounds 2 --reps 2 > gpurun_out/kbench.log 2>&1; rc=$?; cat gpurun_out/kbench.log; [ $rc -eq 0 ] || exit $rc
ZSEEK_HIP_KERNEL=lane timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; exit $rc
