"""Timeline of one decode launch from a rocprofv3 kernel trace: each kernel's
[start, end) relative to the launch's first kernel, and the time no kernel
runs (gaps).  A launch starts at a zstd_plan_kernel (zstd) or at the first
kernel after a gap > 200 us.  Usage: trace_timeline.py TRACE.csv [launch#]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
want = int(sys.argv[2]) if len(sys.argv) > 2 else -2
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"])
             for r in rows), key=lambda k: k[0])
launches, cur = [], []
for k in ks:
    if cur and ("zstd_plan_kernel" in k[2] or k[0] - max(c[1] for c in cur) > 200_000):
        launches.append(cur)
        cur = []
    cur.append(k)
if cur:
    launches.append(cur)
L = launches[want]
t0 = L[0][0]
end = max(k[1] for k in L)
print(f"{len(launches)} launches; launch {want}: {(end - t0) / 1e6:.3f} ms, {len(L)} kernels")
for s, e, n, q in L:
    m = re.search(r"(zstd_\w+|seq_exec_kernel|lz4_\w+|frame_\w+|__amd_\w+)", n)
    short = (m.group(1) if m else n)[:34]
    print(f"  q{q:>3} {short:34s} {(s - t0) / 1e3:9.1f} -> {(e - t0) / 1e3:9.1f} us  ({(e - s) / 1e3:8.1f})")
ivs = sorted((s, e) for s, e, _, _ in L)
busy, cs, ce = 0, ivs[0][0], ivs[0][1]
for s, e in ivs[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"busy {busy / 1e6:.3f} ms of {(end - t0) / 1e6:.3f} (idle {(end - t0 - busy) / 1e3:.1f} us)")
