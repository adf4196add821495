"""Copy a gpu_round.sh run's rocprofv3 summaries into profiles/ (tracked)
and derive profiles/pmc_traffic.json for bench.py's roofline.traffic.

  python scripts/round_profiles.py r01 [gpurun_out/round]

HBM bytes per launch of the decode kernel = 2 x FETCH_SIZE (gfx950 reports
half the bytes of a wide streaming read, MI355X_MICROARCH.md HBM section) +
WRITE_SIZE, both in KiB from separate --pmc passes, median over dispatches.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

tag = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/round"
dst = "profiles"
os.makedirs(dst, exist_ok=True)


def one(pattern):
    f = glob.glob(os.path.join(src, pattern))
    if not f:
        raise SystemExit(f"missing {pattern} under {src}")
    return f[0]


bench = json.load(open(os.path.join(src, "bench.json")))
KERNEL = bench["roofline"]["kernel"]   # the dominant kernel bench.py reports


def is_decode(name):
    return KERNEL in name


stats = one("trace/*/*_kernel_stats.csv")
shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
kern = None
for row in csv.DictReader(open(stats)):
    if is_decode(row["Name"]):
        kern = (row["Name"], float(row["AverageNs"]), int(row["Calls"]))
        break
counters = {}
for name in ("fetch", "write"):
    f = one(f"pmc_{name}/*/*_counter_collection.csv")
    shutil.copy(f, os.path.join(dst, f"{tag}_pmc_{name}.csv"))
    for row in csv.DictReader(open(f)):
        if is_decode(row["Kernel_Name"]):
            counters.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
fetch = statistics.median(counters["FETCH_SIZE"]) * 1024
write = statistics.median(counters["WRITE_SIZE"]) * 1024
alg = bench["roofline"]["algorithmic_bytes_per_launch"]
out = {
    "round": tag,
    "kernel": kern[0],
    "avg_kernel_ns_rocprof": kern[1],
    "calls": kern[2],
    "bench_avg_kernel_ms": bench["roofline"]["avg_kernel_ms"],
    "fetch_size_bytes_raw": fetch,
    "fetch_bytes_corrected_x2": 2 * fetch,
    "write_size_bytes": write,
    "hbm_bytes_per_launch": 2 * fetch + write,
    "algorithmic_bytes_per_launch": alg,
    "traffic_over_algorithmic": (2 * fetch + write) / alg,
}
json.dump(out, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))
print(json.dumps(out, indent=1))
