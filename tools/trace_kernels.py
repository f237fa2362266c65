#!/usr/bin/env python3
"""Kernel timeline from a rocprofv3 run_results.db: every dispatch of the kernels whose names
contain one of the given substrings, with queue-relative start / end (ms) and duration.
    python3 tools/trace_kernels.py DB k_entropy_seq k_spec_plan ..."""
import sqlite3
import sys


def main():
    db, keys = sys.argv[1], sys.argv[2:]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    qcol = next((q for q in ("queue_id", "stream_id", "queue") if q in cols), None)
    rows = c.execute(f"select {name}, start, end{', ' + qcol if qcol else ''} from kernels order by start").fetchall()
    t0 = rows[0][1] if rows else 0
    for r in rows:
        if not keys or any(k in r[0] for k in keys):
            q = r[3] if qcol else ""
            print(f"{(r[1] - t0) / 1e6:10.3f} {(r[2] - t0) / 1e6:10.3f} {(r[2] - r[1]) / 1e6:9.3f} q{q} {r[0].split('(')[0][:50]}")


if __name__ == "__main__":
    main()
