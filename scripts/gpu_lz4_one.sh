# LZ4 one-frame route: the GPU suite, the parse's phase cycles (tuning
# build, ZSEEK_CHUNK_TIMERS) and the latency probe.  $1 output dir
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-lz4one}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_CHUNK_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 lz4 > $O/ct.log 2>&1 &&
grep "chunk one-route" $O/ct.log | tail -1 &&
timeout -k 10 300 python scripts/latency_probe.py 600 lz4 > $O/lat.log 2>&1 && tail -1 $O/lat.log
