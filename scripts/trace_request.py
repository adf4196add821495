"""Kernel timeline of a few consecutive dispatches from a rocprofv3
--kernel-trace run (e.g. `scripts/gpu.sh latency`'s): start offset and duration
(us) of each, to see a request's launch gaps.  Args: trace dir, first row
(default 400), rows (default 16)."""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
a = int(sys.argv[2]) if len(sys.argv) > 2 else 400
n = int(sys.argv[3]) if len(sys.argv) > 3 else 16
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a: a + n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(anonymous namespace)::")[-1].split("(")[0]
    print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f}  {name[:60]}")
