# round 4: execute variants (interleaved), the GPU suite, then the round-3
# heap-corruption probe with streams / events destroyed again
# (ZSEEK_HIP_DESTROY=1) now that the reference lives in its own link namespace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04combo
mkdir -p $O
timeout -k 10 300 python scripts/kbench.py --variants 12,20,321,784,0 --rounds 5 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep -v amdgpu.ids $O/kb.log | grep "median\|MISMATCH\|bit-exact"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
ZSEEK_HIP_DESTROY=1 timeout -k 10 400 python -u scripts/hang_probe.py both 250 > $O/probe_destroy.log 2>&1
rc=$?
tail -3 $O/probe_destroy.log
echo "probe rc=$rc"
exit 0
