"""Per-kernel statistics from a rocprofv3 kernel trace (`*_kernel_trace.csv`,
`--kernel-trace --output-format csv`) that do not average warm-up launches
into the figure:

    Name, Calls, AverageNs (all launches, rocprof's own figure),
    MedianNs, SteadyCalls, SteadyAverageNs

SteadyAverageNs / SteadyMedianNs drop each kernel's first `--skip` launches
(default 1: the bench's first step, which sizes scratch and pages in code
objects).  SteadyMedianPerLaunchNs sums the `--per-launch` dispatches one
decode launch makes of a kernel (zstd: one per chunk) and takes the median
over launches: the figure to compare with bench.py's per-stage HIP-event
medians (`stages[*].median_ms`).

    python scripts/kernel_stats.py gpurun_out/round/trace [--skip 1] > profiles/r04_kernel_stats.csv
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--skip", type=int, default=1, help="launches dropped as warm-up")
    ap.add_argument("--per-launch", type=int, default=1,
                    help="dispatches of a kernel per decode launch (zstd: its chunk count)")
    a = ap.parse_args()
    files = [a.path] if a.path.endswith(".csv") else \
        glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {a.path}")
    durs = defaultdict(list)   # name -> durations in dispatch order
    for f in files:
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "AverageNs", "MedianNs", "SteadyCalls", "SteadyAverageNs", "SteadyMedianNs",
                "PerLaunch", "SteadyMedianPerLaunchNs"])
    for name, d in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        k = a.per_launch if len(d) % a.per_launch == 0 else 1
        steady = d[a.skip * k:] if len(d) > a.skip * k else d
        # a decode launch that runs this kernel k times (zstd: once per chunk)
        # -> the sum of its k dispatches, median over launches
        groups = [sum(steady[i: i + k]) for i in range(0, len(steady) - k + 1, k)]
        w.writerow([name, len(d), round(sum(d) / len(d), 1), round(statistics.median(d), 1),
                    len(steady), round(sum(steady) / len(steady), 1), round(statistics.median(steady), 1),
                    k, round(statistics.median(groups), 1) if groups else ""])


if __name__ == "__main__":
    main()
