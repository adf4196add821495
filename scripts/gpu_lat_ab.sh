# single-frame latency A/B (no profiler): the probe for LZ4 and zstd with the
# small upload / download kernels, then with DMA copies (ZSEEK_HOST_DMA=1).
# $1 output dir
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-latab}
mkdir -p $O
for c in lz4 zstd; do
  timeout -k 10 300 python scripts/latency_probe.py 600 $c > $O/k_$c.log 2>&1 && echo "kernels: $(tail -1 $O/k_$c.log)" &&
  ZSEEK_HOST_DMA=1 timeout -k 10 300 python scripts/latency_probe.py 600 $c > $O/d_$c.log 2>&1 && echo "dma:     $(tail -1 $O/d_$c.log)" || exit 1
done
