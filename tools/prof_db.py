#!/usr/bin/env python3
"""Per-kernel summary (calls, total / average ms) of a rocprofv3 run_results.db (rocpd sqlite,
the default output of rocprofv3 --kernel-trace on ROCm 7.2), optionally as CSV.
    python3 tools/prof_db.py gpurun_out/<dir>/run_results.db [--csv out.csv] [--top N]"""
import argparse
import csv
import sqlite3
import sys


def summary(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                     f"from kernels group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(r[0], r[1], r[2], r[3], 100.0 * r[2] / tot, r[4], r[5]) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = summary(a.db)
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            w.writerows(rows)
    for r in rows[: a.top]:
        nm = r[0] if len(r[0]) < 60 else r[0][:57] + "..."
        sys.stdout.write(f"{nm:60s} {r[1]:6d} {r[2] / 1e6:10.3f} ms {r[3] / 1e3:10.1f} us {r[4]:5.1f}%\n")


if __name__ == "__main__":
    main()
