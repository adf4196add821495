# one-frame zstd kernel cycle counters (tuning build), per sequence-chain
# variant (ZSEEK_ZSEQ_ONE): $1 output dir, $2 variants (default "0 1")
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ztimers}
mkdir -p $O
for v in ${2:-0 1}; do
  ZSEEK_ZSEQ_ONE=$v ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_SEQ_TIMERS=1 ZSEEK_ZFRAME_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 zstd > $O/probe_v$v.log 2>&1 || { tail -20 $O/probe_v$v.log; exit 1; }
  echo "variant $v"; tail -3 $O/probe_v$v.log
done
