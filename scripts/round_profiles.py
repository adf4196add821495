"""Copy a `scripts/gpu.sh evidence` run's rocprofv3 summaries into profiles/ (tracked)
and derive profiles/pmc_traffic.json for bench.py's roofline.traffic.

  python scripts/round_profiles.py r01 [gpurun_out/round]
  python scripts/round_profiles.py r01_zstd gpurun_out/zround   (config 5)

HBM bytes per decode launch = sum over its kernels of 2 x FETCH_SIZE (gfx950
reports half the bytes of a wide streaming read, MI355X_MICROARCH.md HBM
section) + WRITE_SIZE, both in KiB from separate --pmc passes, median over
dispatches per kernel.  Round 5: when the run also holds the L2's memory-side
request counters (passes ea_p1..3: TCC_EA0_RDREQ_{32B,64B,128B},
TCC_EA0_WRREQ{,_64B}; `scripts/gpu.sh evidence`), `hbm_bytes_per_launch` is their
exact byte count instead (reads = 32 n32 + 64 n64 + 128 n128, writes = 64 n64
+ 32 (n - n64)); the FETCH-based figure stays beside it.  The calibration
(profiles/r05_fetch_calib.json: frames whose execute reads are known) found
the EA read bytes equal to 2 x FETCH_SIZE (the guide's correction holds) and
1.18x / 1.36x the known reads (whole 32 / 64-byte requests under unaligned
16-byte pieces): memory-side bytes, not algorithmic ones.
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
FRAME = bench["config"].get("frame_bytes", 65536)
# config 3's frame-size sweep lines get files of their own (bench.py looks
# for the one recorded on its workload)
OUT = "pmc_traffic_zstd.json" if ZSTD else "pmc_traffic.json" if FRAME == 65536 else f"pmc_traffic_f{FRAME}.json"


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
# EA request bytes (exact), per launch: per kernel the median dispatch x
# dispatches per launch, as above
ea = {}
if glob.glob(os.path.join(src, "ea_p1", "**", "*_counter_collection.csv"), recursive=True):
    cnt = {}
    for i in (1, 2, 3):
        # (the newest pass only: gpurun_out/ keeps earlier calls' files too)
        for f in [one(f"ea_p{i}/*/*_counter_collection.csv")]:
            shutil.copy(f, os.path.join(dst, f"{tag}_ea_p{i}.csv"))
            for row in csv.DictReader(open(f)):
                k = part(row["Kernel_Name"])
                if k:
                    key = (k, row["Counter_Name"], int(row["Dispatch_Id"]))
                    cnt[key] = cnt.get(key, 0.0) + float(row["Counter_Value"])
    byk = {}
    for (k, c, d), v in cnt.items():
        byk.setdefault(k, {}).setdefault(c, []).append(v)
    plan_d = len(byk.get(PLAN, {}).get("TCC_EA0_RDREQ_32B_sum", [])) or 1
    for k, c in byk.items():
        m = {n: statistics.median(v) * len(v) / plan_d for n, v in c.items()}
        rd = 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + \
            128 * m.get("TCC_EA0_RDREQ_128B_sum", 0)
        wq, w64 = m.get("TCC_EA0_WRREQ_sum", 0), m.get("TCC_EA0_WRREQ_64B_sum", 0)
        ea[k] = {"read_bytes": rd, "write_bytes": 64 * w64 + 32 * (wq - w64)}
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
    "fetch_based_bytes_per_launch": 2 * fetch + write,
    "algorithmic_bytes_per_launch": alg,
}
if ea:
    out["ea_kernels"] = ea
    out["ea_read_bytes"] = sum(v["read_bytes"] for v in ea.values())
    out["ea_write_bytes"] = sum(v["write_bytes"] for v in ea.values())
    out["hbm_bytes_per_launch"] = out["ea_read_bytes"] + out["ea_write_bytes"]
    out["traffic_source"] = "TCC_EA0 request bytes (exact)"
else:
    out["hbm_bytes_per_launch"] = 2 * fetch + write
    out["traffic_source"] = "2 x FETCH_SIZE + WRITE_SIZE"
out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / alg
json.dump(out, open(os.path.join(dst, OUT), "w"), indent=1)
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))
print(json.dumps(out, indent=1))
