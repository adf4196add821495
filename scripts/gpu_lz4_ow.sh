# LZ4 one-frame parse over 4 or 8 waves (ZSEEK_ONE_WAVES): the GPU suite at
# the default, then per wave count and lead-in the parse's phase cycles
# (tuning build) and the latency probe.  $1 output dir, then "WAVES:LEAD" pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-lz4ow}
shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for pr in "$@"; do
  w=${pr%:*}; ld=${pr#*:}
  ZSEEK_ONE_WAVES=$w ZSEEK_ONE_LEAD=$ld ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_CHUNK_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 lz4 > $O/ct_${w}_$ld.log 2>&1 || { tail -20 $O/ct_${w}_$ld.log; exit 1; }
  echo "waves $w lead $ld: $(grep 'chunk one-route' $O/ct_${w}_$ld.log | tail -1)"
  ZSEEK_ONE_WAVES=$w ZSEEK_ONE_LEAD=$ld timeout -k 10 300 python scripts/latency_probe.py 600 lz4 > $O/lat_${w}_$ld.log 2>&1 || { tail -20 $O/lat_${w}_$ld.log; exit 1; }
  echo "   $(tail -1 $O/lat_${w}_$ld.log)"
done
