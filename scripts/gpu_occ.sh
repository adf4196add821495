# Occupancy probe of the execute (tuning build): kbench of the execute alone
# at 7 (production) and 6..2 waves per SIMD (LDS padding), then the L2's EA
# read requests of each in its own rocprofv3 pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/occ
mkdir -p $O
timeout -k 10 400 python scripts/kbench.py --variants 10,20,0x606,0x605,0x604,0x603,0x602 --rounds 5 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
cat $O/kbench.log
for v in 20 0x605 0x604 0x603 0x602; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum --output-format csv -d $O/ea_$v -- python scripts/kbench.py --variants 10,$v --rounds 1 --reps 1 > $O/ea_$v.log 2>&1 || { tail -5 $O/ea_$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/occ/ea_*")):
    if d.endswith(".log"): continue
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "seq_exec_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(d, {k: [round(x * (128 if "128B" in k else 64 if "64B" in k else 1) / 1e9, 3) if "B_" in k else x for x in v] for k, v in agg.items()})
PY
