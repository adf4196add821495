# round 4: the one-frame execute's phase cycles (tuning build,
# ZSEEK_FRAME_TIMERS) under 300 single-frame 4 KiB reads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_FRAME_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 > gpurun_out/ftimers.log 2>&1 || { tail -5 gpurun_out/ftimers.log; exit 1; }
grep -E "p50|frame execute" gpurun_out/ftimers.log | tail -3
