# round 4: production execute (3,584-byte stage) against the 4,096 stage on a
# fresh tuning build; the GPU suite and the churn probe with streams / events
# destroyed by default (ZSEEK_HIP_POOL unset).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04combo3
mkdir -p $O
timeout -k 10 300 python scripts/kbench.py --variants 0,321 --rounds 5 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep -v amdgpu.ids $O/kb.log | grep "median\|MISMATCH\|bit-exact"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 400 python -u scripts/hang_probe.py both 250 > $O/probe.log 2>&1
rc=$?
tail -3 $O/probe.log
echo "probe rc=$rc"
exit 0
