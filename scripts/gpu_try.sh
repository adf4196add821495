set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "exec4" > gpurun_out/pt_scan.log 2>&1; rc=$?; tail -3 gpurun_out/pt_scan.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --size 4294967296 --variants 61,68,66 --rounds 3 > gpurun_out/kb39.log 2>&1; rc=$?; grep -v "^$" gpurun_out/kb39.log | tail -12; exit $rc
