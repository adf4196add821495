set -o pipefail
# lean parse: per-lane LDS stride A/B (ZSEEK_LEAN_STRIDE = 560 default / 564 / 568)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in 1 2; do
  for st in 560 564 568; do
    echo "== stride $st"
    ZSEEK_LEAN_STRIDE=$st timeout -k 10 200 python scripts/kbench.py --variants 99 --rounds 3 --reps 2 2>&1 | grep -E "variant|input" || exit 1
  done
done
