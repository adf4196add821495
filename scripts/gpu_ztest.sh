set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pyz.log 2>&1; rc=$?; tail -15 gpurun_out/pyz.log; exit $rc
