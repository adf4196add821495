"""Copy a gpu_round.sh run's rocprofv3 summaries into profiles/ (tracked)
and derive profiles/pmc_traffic.json for bench.py's roofline.traffic.

  python scripts/round_profiles.py r01 [gpurun_out/round]
  python scripts/round_profiles.py r01_zstd gpurun_out/zround   (config 5)

HBM bytes per decode launch = sum over its kernels of 2 x FETCH_SIZE (gfx950
reports half the bytes of a wide streaming read, MI355X_MICROARCH.md HBM
section) + WRITE_SIZE, both in KiB from separate --pmc passes, median over
dispatches per kernel.
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
    """the newest match (gpurun_out/ accumulates earlier calls' files)"""
    f = glob.glob(os.path.join(src, pattern))
    if not f:
        raise SystemExit(f"missing {pattern} under {src}")
    return max(f, key=os.path.getmtime)


bench = json.load(open(os.path.join(src, "bench.json")))
KERNEL = bench["roofline"]["kernel"]   # the dominant kernel bench.py reports
# kernels of one decode launch (zsk_lz4_decode_frames): the two-phase decoder
# runs plan + parse + execute + the (normally empty) hand-off pass
LAUNCH = ("lz4_plan_direct_kernel", "lz4_block_plan_kernel", "lz4_lean_kernel", "lz4_chunk_kernel",
          "lz4_scan_kernel",
          "seq_exec_kernel", "lz4_wave_kernel",
          "lz4_lane_kernel", "lz4_parse_kernel", "lz4_exec_kernel")
ZSTD = "zstd" in bench["metric"]
if ZSTD:   # zsk_zstd_decode_frames: plan + scan + frame + literal + sequence + execute + check
    LAUNCH = ("zstd_plan_kernel", "zstd_scan_kernel", "zstd_bounds_kernel", "zstd_frame_kernel", "zstd_huf_kernel",
              "zstd_seq_kernel", "zstd_lit_fix_kernel", "seq_exec_kernel", "zstd_check_kernel")
OUT = "pmc_traffic_zstd.json" if ZSTD else "pmc_traffic.json"


def part(name):
    for k in LAUNCH:
        if k in name:
            return k
    return None


# dispatches per decode launch: the plan kernel runs once per launch (the
# zstd decode dispatches its frame / Huffman / sequence / execute / check
# kernels once per chunk)
PLAN = "zstd_plan_kernel" if ZSTD else "lz4_plan_direct_kernel"
stats = one("trace/*/*_kernel_stats.csv")
shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
kern = {}
for row in csv.DictReader(open(stats)):
    k = part(row["Name"])
    if k:
        nm = row["Name"].replace("(anonymous namespace)::", "").split("(")[0]
        kern[k] = {"name": nm, "avg_ns": float(row["AverageNs"]),
                   "calls": int(row["Calls"])}
plan_calls = kern.get(PLAN, {}).get("calls", 1)
for k, v in kern.items():
    v["per_launch"] = round(v["calls"] / plan_calls, 3)
counters = {}
for name in ("fetch", "write"):
    f = one(f"pmc_{name}/*/*_counter_collection.csv")
    shutil.copy(f, os.path.join(dst, f"{tag}_pmc_{name}.csv"))
    for row in csv.DictReader(open(f)):
        k = part(row["Kernel_Name"])
        if k:
            counters.setdefault((k, row["Counter_Name"]), []).append(float(row["Counter_Value"]))
per = {}
# per launch: the median dispatch x dispatches per launch (in the PMC pass)
plan_n = {c: len(v) for (k, c), v in counters.items() if k == PLAN}
for (k, c), v in counters.items():
    per.setdefault(k, {})[c] = statistics.median(v) * 1024 * len(v) / max(plan_n.get(c, len(v)), 1)
fetch = sum(d.get("FETCH_SIZE", 0.0) for d in per.values())
write = sum(d.get("WRITE_SIZE", 0.0) for d in per.values())
alg = bench["roofline"]["algorithmic_bytes_per_launch"]
out = {
    "round": tag,
    "kernel": KERNEL,
    "workload": bench["config"]["workload"],
    "launch_kernels": {k: {**kern.get(k, {}), "fetch_bytes_raw": per.get(k, {}).get("FETCH_SIZE"),
                           "write_bytes": per.get(k, {}).get("WRITE_SIZE")} for k in sorted(set(kern) | set(per))},
    "launch_avg_ns_rocprof": sum(v["avg_ns"] * v["per_launch"] for v in kern.values()),
    "bench_avg_launch_ms": bench["roofline"]["avg_launch_ms"],
    "fetch_size_bytes_raw": fetch,
    "fetch_bytes_corrected_x2": 2 * fetch,
    "write_size_bytes": write,
    "hbm_bytes_per_launch": 2 * fetch + write,
    "algorithmic_bytes_per_launch": alg,
    "traffic_over_algorithmic": (2 * fetch + write) / alg,
}
json.dump(out, open(os.path.join(dst, OUT), "w"), indent=1)
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))
print(json.dumps(out, indent=1))
