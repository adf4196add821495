# LZ4 single-frame latency with / without the zero-copy small batch, and the
# LZ4 GPU tests: $1 output dir
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-lz4zc}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_checksum.py > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for zc in 1 0 1 0; do
  ZSEEK_ZEROCOPY=$zc timeout -k 10 300 python scripts/latency_probe.py 600 lz4 > $O/probe_$zc.log 2>&1 || { tail -20 $O/probe_$zc.log; exit 1; }
  echo "zerocopy $zc: $(tail -1 $O/probe_$zc.log)"
done
