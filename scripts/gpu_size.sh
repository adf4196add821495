set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sz in 268435456 1073741824 4294967296; do
  timeout -k 10 300 python scripts/kbench.py --size $sz --variants 1,3 --rounds 3 --reps 3 2>&1 | grep -E "median|MISMATCH|Error" | sed "s/^/size=$sz /" || exit 1
done
