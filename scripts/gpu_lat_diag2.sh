# single-frame latency: host steps per batch (tuning build, warm-up left out)
# for LZ4 and zstd, then a kernel + memory-copy trace of the LZ4 probe.
# $1 output dir
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
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -- python scripts/latency_probe.py 300 lz4 > $O/probe.log 2>&1 &&
grep reads: $O/probe.log
