# one-frame zstd sequence kernel cycle counters (tuning build): $1 output dir
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ztimers}
mkdir -p $O
ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_SEQ_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 zstd > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
tail -4 $O/probe.log
