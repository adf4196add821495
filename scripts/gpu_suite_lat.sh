# the whole GPU suite (one process), then the zstd and LZ4 single-frame
# latency probes with kernel traces.  $1 output dir
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-suitelat}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
bash scripts/gpu_latency_probe.sh ${1:-suitelat}/lat_zstd zstd 300 > /dev/null && grep reads: $O/lat_zstd/probe.log &&
bash scripts/gpu_latency_probe.sh ${1:-suitelat}/lat_lz4 lz4 300 > /dev/null && grep reads: $O/lat_lz4/probe.log
