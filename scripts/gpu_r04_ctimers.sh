# round 4: the one-frame parse's phase cycles (tuning build, ZSEEK_CHUNK_TIMERS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_CHUNK_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 > gpurun_out/ctimers.log 2>&1 || { tail -5 gpurun_out/ctimers.log; exit 1; }
grep "chunk one-route" gpurun_out/ctimers.log | tail -2
grep "p50" gpurun_out/ctimers.log | tail -1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ct_suite.log 2>&1 || { tail -30 gpurun_out/ct_suite.log; exit 1; }
tail -1 gpurun_out/ct_suite.log
timeout -k 10 300 python scripts/latency_probe.py 300 2>&1 | grep p50
