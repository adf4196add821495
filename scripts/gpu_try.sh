set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "scan or exec3" > gpurun_out/pt_scan.log 2>&1; rc=$?; tail -15 gpurun_out/pt_scan.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --size 4294967296 --variants 50,37,39,60 --rounds 3 > gpurun_out/kb39.log 2>&1; rc=$?; tail -9 gpurun_out/kb39.log; exit $rc
