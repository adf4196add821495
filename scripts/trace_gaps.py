"""Median host gap per request in a latency-probe kernel trace: from each
download kernel's end to the next upload kernel's start, and the median
duration of each kernel.  usage: trace_gaps.py <rocprofv3 output dir>..."""
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*_kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    gaps, dur = [], {}
    for a, b in zip(rows, rows[1:]):
        if "d2h_small" in a["Kernel_Name"] and "h2d_small" in b["Kernel_Name"]:
            gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(d, f"host gap p50 {statistics.median(gaps):.1f} us over {len(gaps)}",
          " ".join(f"{k} {statistics.median(v):.1f}" for k, v in dur.items() if len(v) > 50))
