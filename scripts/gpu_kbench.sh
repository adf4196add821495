# kbench A/B (tuning build, interleaved rounds).  $1: output dir, $2: variants,
# $3: extra kbench args.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-kbench}
mkdir -p $O
timeout -k 10 400 python scripts/kbench.py --variants "$2" --rounds 5 $3 > $O/kbench.log 2>&1
rc=$?
cat $O/kbench.log | tail -20
exit $rc
