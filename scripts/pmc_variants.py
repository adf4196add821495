"""Per-kernel PMC summary of gpu_kbab.sh's passes: for every pmc_<variant>
directory, the counters of each kernel (the last dispatch of that kernel in the
pass) and per-wave figures."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
    if d.endswith(".log"):
        continue
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        last = collections.OrderedDict()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-60:]
            last.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        for k, c in last.items():
            if "zsk" not in k:
                continue
            w = c.get("SQ_WAVES", 0) or 1
            per = "  ".join(f"{n.replace('SQ_', '')} {v / w:.0f}" for n, v in sorted(c.items()) if n != "SQ_WAVES")
            extra = ""
            if "SQ_WAIT_INST_LDS" in c and "SQ_WAVE_CYCLES" in c:
                extra = f"  waitLDS/cyc {c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.3f}"
            print(f"{os.path.basename(d)} {k}: waves {w:.0f}  per wave: {per}{extra}")
