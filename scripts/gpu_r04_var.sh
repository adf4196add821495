# round 4: execute tuning variants against the production execute (kbench
# variant 20 = execute alone over variant 12's items): 0x320 deal descriptor
# reads together, 0x340 readiness by broadcast, 0x360 both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04var
mkdir -p $O
timeout -k 10 300 python scripts/kbench.py --variants 12,640,704 --rounds 5 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep -v amdgpu.ids $O/kb.log | grep "median\|MISMATCH\|bit-exact"
