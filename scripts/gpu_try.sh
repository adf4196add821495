set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_zstd.py -x -q -m gpu > gpurun_out/pt_zstd.log 2>&1; rc=$?; tail -30 gpurun_out/pt_zstd.log; exit $rc
