"""Summarise rocprofv3 --pmc CSVs: per kernel dispatch, counter totals and
per-wave / derived figures."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in glob.glob(os.path.join(root, "p*", "*", "*_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        if "lz4" not in name and "seq_" not in name and "zstd" not in name:
            continue
        # dispatches of one kernel in the same position across passes line up
        key = (name, os.path.basename(os.path.dirname(os.path.dirname(f))), row["Dispatch_Id"])
        agg[key][row["Counter_Name"]] += float(row["Counter_Value"])
        names[key] = row.get("LDS_Block_Size"), row.get("VGPR_Count"), row.get("SGPR_Count")
by_kernel = collections.defaultdict(dict)
for (name, pas, disp), c in agg.items():
    short = name.split("lz4_frames_kernel")[-1][:60]
    for k, v in c.items():
        by_kernel[short].setdefault(k, []).append(v)
for k, c in by_kernel.items():
    print("kernel", k)
    m = {n: sorted(v)[len(v) // 2] for n, v in c.items()}
    for n in sorted(m):
        print(f"  {n:24s} {m[n]:.4g}")
    w = m.get("SQ_WAVES")
    if w:
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                  "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in m:
                print(f"  per-wave {n:20s} {m[n] / w:.4g}")
    if "FETCH_SIZE" in m:
        print(f"  FETCH_SIZE x2 (gfx950 correction) = {2 * m['FETCH_SIZE'] * 1024 / 1e9:.3f} GB")
    if "WRITE_SIZE" in m:
        print(f"  WRITE_SIZE = {m['WRITE_SIZE'] * 1024 / 1e9:.3f} GB")
