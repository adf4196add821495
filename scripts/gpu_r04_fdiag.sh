# round 4: one-frame execute phase cycles with parts switched off (tuning
# build, ZSEEK_FRAME_DIAG: 1 no literal copies, 2 no literal marks (only with 4: the matches would wait forever), 4 no
# matches; outputs not checked)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fdiag
mkdir -p $O
for dg in 0 1 4 5 6; do
ZSEEK_FRAME_DIAG=$dg ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_FRAME_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 200 > $O/d$dg.log 2>&1 || { tail -5 $O/d$dg.log; exit 1; }
echo "diag $dg: $(grep -E 'frame execute' $O/d$dg.log | tail -1)"
done
