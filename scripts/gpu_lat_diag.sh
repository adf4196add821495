# single-frame latency diagnostics (tuning build): the reader's host steps per
# batch (ZSEEK_HOST_TIMERS) for LZ4 and zstd, and the LZ4 one-frame parse's
# phase cycles (ZSEEK_CHUNK_TIMERS).  $1 output dir
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-latdiag}
mkdir -p $O
T=$PWD/libzseek_amd/lib/libzseek_tune.so
ZSEEK_AMD_LIB=$T ZSEEK_HOST_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 600 lz4 > $O/ht_lz4.log 2>&1 &&
tail -2 $O/ht_lz4.log &&
ZSEEK_AMD_LIB=$T ZSEEK_HOST_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 600 zstd > $O/ht_zstd.log 2>&1 &&
tail -2 $O/ht_zstd.log &&
ZSEEK_AMD_LIB=$T ZSEEK_CHUNK_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 lz4 > $O/ct_lz4.log 2>&1 &&
grep "chunk one-route" $O/ct_lz4.log | tail -1 && tail -1 $O/ct_lz4.log
