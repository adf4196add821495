"""Memory-side bytes per kernel dispatch from `scripts/gpu.sh pmc` passes: reads
= 32 n32 + 64 n64 + 128 n128 (TCC_EA0_RDREQ_{32B,64B,128B}), the share of
read requests destined for DRAM (TCC_EA0_RDREQ_DRAM / TCC_EA0_RDREQ; the rest
served by the Infinity Cache / other dies), writes = 64 n64 + 32 (n - n64)
(TCC_EA0_WRREQ, _64B).  Median over a kernel's dispatches, per workload."""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
for wl in ("calib", "c2"):
    per = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> values
    for i in (1, 2, 3):
        rows = collections.defaultdict(float)
        names = {}
        for f in glob.glob(os.path.join(root, f"{wl}_p{i}", "**", "*_counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = (int(r["Dispatch_Id"]), r["Counter_Name"])
                rows[k] += float(r["Counter_Value"])
                names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        for (d, c), v in rows.items():
            n = names[d]
            if "zsk::" not in n:
                continue
            short = n.split("(anonymous namespace)::")[-1].split("(")[0][:48]
            per[(short, d if wl == "calib" else 0)][c].append(v)
    print(f"== {wl}")
    for (k, d), c in sorted(per.items(), key=lambda x: (x[0][1], x[0][0])):
        m = {n: statistics.median(v) for n, v in c.items()}
        rd = 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + \
            128 * m.get("TCC_EA0_RDREQ_128B_sum", 0)
        rq = m.get("TCC_EA0_RDREQ_sum", 0)
        dram = m.get("TCC_EA0_RDREQ_DRAM_sum", 0) / rq if rq else 0
        wq, w64 = m.get("TCC_EA0_WRREQ_sum", 0), m.get("TCC_EA0_WRREQ_64B_sum", 0)
        wr = 64 * w64 + 32 * (wq - w64)
        wdram = m.get("TCC_EA0_WRREQ_DRAM_sum", 0) / wq if wq else 0
        if rd + wr < 1e6:
            continue
        print(f"{k:48s} {'#' + str(d) if d else ''} read {rd / 1e9:7.3f} GB (DRAM share {dram:.2f})  "
              f"write {wr / 1e9:7.3f} GB (DRAM share {wdram:.2f})")
