# single-frame read latency (scripts/latency_probe.py) with a kernel trace:
# $1 output dir, $2 codec (lz4 | zstd), $3 requests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-latprobe}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python scripts/latency_probe.py ${3:-300} ${2:-zstd} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -E "reads:" $O/probe.log
python3 scripts/kernel_stats.py $O/trace --skip 20 | cut -d, -f1,2,4,7 | head -20
