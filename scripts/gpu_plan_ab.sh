# A/B: plan by offsets (default) vs plan by scan (ZSEEK_PLAN_SCAN=1), same box, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/planab
mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python bench.py --profile --steps 10 --warmup 3 > $O/direct$i.json 2>/dev/null && cat $O/direct$i.json | python -c "import json,sys; d=json.load(sys.stdin); print('direct', d['ms_per_step'], d['roofline']['stages'])" &&
ZSEEK_PLAN_SCAN=1 timeout -k 10 300 python bench.py --profile --steps 10 --warmup 3 > $O/scan$i.json 2>/dev/null && cat $O/scan$i.json | python -c "import json,sys; d=json.load(sys.stdin); print('scan', d['ms_per_step'], d['roofline']['stages'])" || exit 1
done
