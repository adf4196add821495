"""Per-wave instruction counters of every seq_exec dispatch in a
`scripts/gpu.sh pmc` run (passes p1, p2 lined up by dispatch order).
Optional second argument: the kernel-name fragment to select (default
seq_exec); a third, "mean": one line, the mean over the selected dispatches."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
pick = sys.argv[2] if len(sys.argv) > 2 else "seq_exec"
mean = len(sys.argv) > 3 and sys.argv[3] == "mean"
per = {}
for pas in ("p1", "p2"):
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(root, pas, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if pick not in r["Kernel_Name"]:
                continue
            k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            rows[k][r["Counter_Name"]] += float(r["Counter_Value"])
    per[pas] = [rows[k] | {"_name": k[1]} for k in sorted(rows)]
if mean:
    tot = collections.defaultdict(float)
    for i, c in enumerate(per["p1"]):
        c2 = per["p2"][i] if i < len(per["p2"]) else {}
        for k, v in list(c.items()) + list(c2.items()):
            if not k.startswith("_"):
                tot[k] += v
    w = tot.pop("SQ_WAVES", 1.0)
    print(f"{pick}: {len(per['p1'])} dispatches, {w:.0f} waves; per wave: " + " ".join(
        f"{k.replace('SQ_', '')} {v / w:.0f}" for k, v in sorted(tot.items())))
    sys.exit(0)
for i, c in enumerate(per["p1"]):
    c2 = per["p2"][i] if i < len(per["p2"]) else {}
    w = c["SQ_WAVES"]
    name = c["_name"].split("seq_exec_kernel<")[-1].split(">")[0]
    vals = {k: v / w for k, v in list(c.items()) + list(c2.items()) if not k.startswith("_") and k != "SQ_WAVES"}
    print(f"seq_exec_kernel<{name}> waves {w:.0f}: " + " ".join(
        f"{k.replace('SQ_', '')} {v:.0f}" for k, v in sorted(vals.items())))
