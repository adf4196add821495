# zstd final line: the config-5 bench (with its latency lines) and the
# single-frame latency trace.  Output under gpurun_out/zround5f
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
Z=gpurun_out/zround5f
mkdir -p $Z
timeout -k 10 600 python bench.py --codec zstd > $Z/bench.json 2> $Z/bench.err && cut -c1-300 $Z/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $Z/trace -- python bench.py --codec zstd --profile --steps 5 --warmup 1 > $Z/trace.log 2>&1 &&
bash scripts/gpu_latency_probe.sh zround5f/lat_zstd zstd 300 > /dev/null && grep reads: $Z/lat_zstd/probe.log
