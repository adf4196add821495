# zstd one-frame route: zstd GPU tests, then the cycle counters (tuning build)
# and the production latency probe with a kernel trace.  $1 output dir
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-zone}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_zstd.py > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
bash scripts/gpu_zstd_timers.sh ${1:-zone}/timers 0 && bash scripts/gpu_latency_probe.sh ${1:-zone}/lat zstd 300 > /dev/null && grep reads: $O/lat/probe.log && python3 scripts/trace_request.py $O/lat/trace 300 14
