"""Copy a `scripts/gpu.sh evidence TAG --codec lz4c` run into profiles/ (tracked) and derive
profiles/pmc_traffic_lz4c.json for bench.py --codec lz4c's roofline.traffic.

  python scripts/lz4c_profiles.py r03 [gpurun_out/lz4c]

Memory-side bytes per launch = FETCH_SIZE + WRITE_SIZE of lz4_compress_kernel
(KiB, separate --pmc passes, median over dispatches).  FETCH_SIZE is not
doubled: the compressor's reads are narrow random loads (table entries,
candidate words), not the wide streaming reads the MI355X_MICROARCH.md HBM
correction is calibrated for; Infinity-Cache hits are included (same guide).
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

tag = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/lz4c"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")
KERNEL = "lz4_compress_kernel"


def median_counter(d, ctr):
    vals = []
    files = glob.glob(os.path.join(src, d, "**", "*counter_collection.csv"), recursive=True)
    for f in [max(files, key=os.path.getmtime)] if files else []:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == ctr and KERNEL in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    return statistics.median(vals) if vals else None


stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
if stats:   # the newest run (gpurun_out/ accumulates earlier calls' files)
    shutil.copy(max(stats, key=os.path.getmtime), os.path.join(prof, f"{tag}_lz4c_kernel_stats.csv"))
bench = json.load(open(os.path.join(src, "bench.json")))
json.dump(bench, open(os.path.join(prof, f"{tag}_lz4c_bench.json"), "w"), indent=1)
fetch, write = median_counter("pmc_fetch", "FETCH_SIZE"), median_counter("pmc_write", "WRITE_SIZE")
alg = bench["roofline"]["algorithmic_bytes_per_launch"]
rec = {"kernel": KERNEL, "workload": bench["config"]["workload"],
       "fetch_kib": fetch, "write_kib": write,
       "hbm_bytes_per_launch": int((fetch + write) * 1024) if fetch and write else None,
       "algorithmic_bytes_per_launch": alg,
       "ratio": round((fetch + write) * 1024 / alg, 2) if fetch and write else None,
       "note": "memory-side bytes (L2 misses, Infinity-Cache hits included), FETCH_SIZE not doubled: "
               "narrow random loads, outside the guide's calibrated wide-stream case"}
json.dump(rec, open(os.path.join(prof, "pmc_traffic_lz4c.json"), "w"), indent=1)
print(json.dumps(rec))
