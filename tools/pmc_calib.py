#!/usr/bin/env python3
"""Calibrate FETCH_SIZE / WRITE_SIZE against known byte counts (GPU box; measurement tooling).

    python3 tools/pmc_calib.py run [--out profiles/r02_pmc_calibration.json]

Runs tools/pmc_calib (calib_read16 / calib_read4 / calib_write16: exactly 1 GiB each per launch,
from a buffer 4x the Infinity Cache) under two separate rocprofv3 --pmc passes (FETCH_SIZE, then
WRITE_SIZE; never combined with tracing domains) and reports, per kernel, counter bytes / bytes
moved. tools/pmc_traffic.py divides raw FETCH_SIZE by the read16 ratio instead of assuming the
guide's x2."""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BYTES = 1 << 30


def _per_kernel(d, counter):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            k = row["Kernel_Name"].split("(")[0]
            key = (f, row.get("Dispatch_Id"))
            per.setdefault(k, {}).setdefault(key, 0.0)
            per[k][key] += float(row["Counter_Value"])
    return {k: sorted(v.values()) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run"])
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_pmc_calibration.json"))
    a = ap.parse_args()
    exe = os.path.join(ROOT, "tools", "pmc_calib")
    out = os.path.join(ROOT, "gpurun_out", "pmc_calib")
    res = {"bytes_per_launch": BYTES, "buffer": "1 GiB (4x the 256 MiB Infinity Cache)", "kernels": {}}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out, ctr.lower())
        cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", d,
               "-o", "run", "--", exe]
        print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, cwd="/tmp")
        for k, vals in _per_kernel(d, ctr).items():
            kib = sum(vals) / len(vals)
            res["kernels"].setdefault(k, {})[ctr.lower() + "_kib_per_launch"] = round(kib, 1)
            res["kernels"][k][ctr.lower() + "_ratio"] = round(kib * 1024.0 / BYTES, 4)
    r16 = res["kernels"].get("calib_read16", {}).get("fetch_size_ratio")
    res["fetch_correction_read16"] = round(1.0 / r16, 4) if r16 else None
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
