#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from two rocprofv3 PMC passes (GPU box).

    python3 tools/pmc_traffic.py run  [--workload c3] [--kernel k_gw_lane] [--out profiles/traffic.json]
    python3 tools/pmc_traffic.py parse FETCH_DIR WRITE_DIR [...]

`run` profiles `bench.py --steps 1 --warmup 0 --no-cpu --no-pcie` twice, once with --pmc FETCH_SIZE and once
with --pmc WRITE_SIZE (the two cannot share a pass on gfx950; counters are collected in runs of their
own, never together with tracing domains), then parses both. Per MI355X_MICROARCH.md (HBM section):
FETCH_SIZE counts wide (16 B/lane) streaming reads at exactly half their bytes on gfx950, so it is
doubled; WRITE_SIZE is taken as is. Both are reported in KiB by rocprofv3 and converted to bytes.
The result (bytes per launch, averaged over the kernel's dispatches) is what bench.py reports as
roofline.traffic when the workload and kernel match.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _values(d, counter, kernel):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                continue
            key = (f, row.get("Dispatch_Id"))
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    if not per:
        raise SystemExit(f"{counter}: no dispatches of {kernel} in {d}")
    return list(per.values())


def parse(fetch_dir, write_dir, kernel, workload, images):
    fv = _values(fetch_dir, "FETCH_SIZE", kernel)
    wv = _values(write_dir, "WRITE_SIZE", kernel)
    f_kib = sum(fv) / len(fv)
    w_kib = sum(wv) / len(wv)
    corr, src = fetch_correction()
    fetch_b = corr * f_kib * 1024.0  # gfx950: FETCH_SIZE = half the bytes of 16 B/lane reads
    write_b = w_kib * 1024.0
    n_images = images or {"c3": 512, "c2": 1024}.get(workload)
    return {"workload": workload, "kernel": kernel, "images_per_bench_step": n_images,
            "images_per_launch": n_images // len(fv) if n_images else None,
            "launches": len(fv), "fetch_size_kib_raw": round(f_kib, 1), "write_size_kib_raw": round(w_kib, 1),
            "fetch_bytes": round(fetch_b), "write_bytes": round(write_b),
            "bytes_per_launch": round(fetch_b + write_b),
            "fetch_correction": corr, "fetch_correction_source": src,
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; FETCH_SIZE x the "
                      "correction measured by tools/pmc_calib.py (1 GiB of 16 B/lane reads); KiB -> bytes"}


def fetch_correction():
    """FETCH_SIZE -> bytes factor for 16 B/lane streaming reads, as measured in this repo by
    tools/pmc_calib.py (profiles/r02_pmc_calibration.json); the guide's x2 if absent."""
    p = os.path.join(ROOT, "profiles", "r02_pmc_calibration.json")
    try:
        c = json.load(open(p))["fetch_correction_read16"]
        if c:
            return float(c), os.path.relpath(p, ROOT)
    except (OSError, KeyError, ValueError):
        pass
    return 2.0, "MI355X_MICROARCH.md HBM section (not yet calibrated here)"


def run(args):
    os.environ.setdefault("TMPDIR", "/tmp")
    out = os.path.join(ROOT, "gpurun_out", "pmc")
    bench = ["python3", os.path.join(ROOT, "bench.py"), "--workload", args.workload, "--steps", "1",
             "--warmup", "0", "--no-cpu", "--no-pcie"]
    if args.images:
        bench += ["--images", str(args.images)]
    dirs = []
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out, ctr.lower())
        cmd = ["timeout", "-k", "10", "600", "rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", d,
               "-o", "run", "--"] + bench
        print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, cwd="/tmp")
        dirs.append(d)
    res = parse(dirs[0], dirs[1], args.kernel, args.workload, args.images or None)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps(res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "parse"])
    ap.add_argument("dirs", nargs="*")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--images", type=int, default=0)
    ap.add_argument("--kernel", default="k_gw_lane")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "traffic.json"))
    args = ap.parse_args()
    if args.mode == "run":
        run(args)
    else:
        print(json.dumps(parse(args.dirs[0], args.dirs[1], args.kernel, args.workload, args.images or None)))


if __name__ == "__main__":
    sys.exit(main())
