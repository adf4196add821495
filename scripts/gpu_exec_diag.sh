# execute-kernel section diagnostics at config 2 (tuning build, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/xdiag
mkdir -p $O
timeout -k 10 500 python scripts/kbench.py --variants 0,10,20,272,257,260,264,290,258 --rounds 3 > $O/kb.log 2>&1 || { tail -30 $O/kb.log; exit 1; }
cat $O/kb.log
