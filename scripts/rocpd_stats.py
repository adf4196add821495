"""Kernel statistics CSV from a rocprofv3 SQLite result (`run_results.db`,
the default output format when `--output-format csv` is not given):
Name, Calls, TotalDurationNs, AverageNs, Percentage — the columns of
rocprofv3's own `kernel_stats.csv`.

    python scripts/rocpd_stats.py gpurun_out/zstd/prof > profiles/x_kernel_stats.csv
"""
from __future__ import annotations

import csv
import glob
import os
import sqlite3
import sys


def main(path: str) -> None:
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    if not dbs:
        raise SystemExit(f"no .db under {path}")
    db = max(dbs, key=os.path.getmtime)
    con = sqlite3.connect(db)
    rows = con.execute(
        "select name, count(*), sum(end - start) from kernels group by name order by 3 desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, calls, dur in rows:
        w.writerow([name, calls, dur, round(dur / calls, 1), round(100.0 * dur / total, 4)])


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
