set -o pipefail
# zstd kernel times vs batch size (1 / 2 / 4 GiB): latency- or throughput-bound?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/zscale
export TMPDIR=/tmp
for sz in 1073741824 2147483648 4294967296; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/zscale/p$sz -o run -- python3 bench.py --codec zstd --profile --steps 2 --warmup 1 --size $sz > gpurun_out/zscale/p$sz.log 2>&1 || exit 1
done
