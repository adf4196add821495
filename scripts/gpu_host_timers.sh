# the reader's host steps per batch (tuning build, ZSEEK_HOST_TIMERS) over the
# single-frame latency probe: $1 output dir, $2 codec (lz4 | zstd)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-htimers}
mkdir -p $O
ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_HOST_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 600 ${2:-lz4} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
tail -2 $O/probe.log
