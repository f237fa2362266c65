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
    # launches with (almost) no work -- a second entropy round with nothing deferred -- are not
    # launches of the kernel's work: averaging them in would halve the per-launch bytes
    top = max(per.values())
    return [v for v in per.values() if v >= 0.01 * top]


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


def _per_kernel(d, counter):
    """{kernel short name: summed counter value (KiB) over all its dispatches} in one PMC pass."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    agg, disp = {}, {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("icx::", "").strip()
            agg[k] = agg.get(k, 0.0) + float(row["Counter_Value"])
            disp.setdefault(k, set()).add((f, row.get("Dispatch_Id")))
    return agg, {k: len(v) for k, v in disp.items()}


# launched by bench.py after the timed steps (the final records gather), not by the decode
NOT_IN_STEP = {"k_records"}


def pipeline(fetch_dir, write_dir, workload, images, w, h, comp_bytes_per_image, out=None):
    """Whole-pipeline HBM traffic of one bench step: FETCH_SIZE (x the calibrated correction) +
    WRITE_SIZE summed over every kernel the step launches, per image, beside the algorithmic bytes
    per image (compressed + W*H*3). moved_over_alg is the number that bounds the
    pipeline's roofline fraction: a pipeline that moves X times its algorithmic bytes cannot exceed
    (achievable HBM / peak) / X of peak in algorithmic terms."""
    fk, fd = _per_kernel(fetch_dir, "FETCH_SIZE")
    wk, wd = _per_kernel(write_dir, "WRITE_SIZE")
    corr, src = fetch_correction()
    ks = sorted(set(fk) | set(wk), key=lambda k: -(corr * fk.get(k, 0) + wk.get(k, 0)))
    per = {}
    tot_f = tot_w = 0.0
    for k in ks:
        if k in NOT_IN_STEP:
            continue
        f = corr * fk.get(k, 0.0) * 1024.0 / images
        wb = wk.get(k, 0.0) * 1024.0 / images
        tot_f += f
        tot_w += wb
        if f + wb < 1e3:  # bookkeeping launches (bytes per image below 1 KB)
            continue
        per[k] = {"fetch_MB_per_image": round(f / 1e6, 3), "write_MB_per_image": round(wb / 1e6, 3),
                  "dispatches": max(fd.get(k, 0), wd.get(k, 0))}
    alg = comp_bytes_per_image + w * h * 3.0
    res = {"workload": workload, "images": images, "width": w, "height": h,
           "alg_MB_per_image": round(alg / 1e6, 3), "compressed_MB_per_image": round(comp_bytes_per_image / 1e6, 3),
           "moved_MB_per_image": round((tot_f + tot_w) / 1e6, 3),
           "fetch_MB_per_image": round(tot_f / 1e6, 3), "write_MB_per_image": round(tot_w / 1e6, 3),
           "moved_over_alg": round((tot_f + tot_w) / alg, 3), "kernels": per,
           "fetch_correction": corr, "fetch_correction_source": src,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of the same bench step; "
                     "every kernel's dispatches summed; FETCH_SIZE x the calibrated correction (16 B and 4 B "
                     "lane reads both read 0.5 on gfx950, profiles/r02_pmc_calibration.json); KiB -> bytes"}
    if out:
        os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
        json.dump(res, open(out, "w"), indent=1)
    return res


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
    if args.pipeline_out:
        n = args.images or {"c3": 512, "c2": 1024}.get(args.workload)
        w, h = {"c2": (1024, 1024)}.get(args.workload, (4096, 4096))
        comp = _comp_bytes_per_image(args.workload, n)
        print(json.dumps(pipeline(dirs[0], dirs[1], args.workload, n, w, h, comp, args.pipeline_out)))


def _comp_bytes_per_image(workload, n):
    """Mean compressed bytes per image of the bench's batch (the pool cycled to n images)."""
    sys.path.insert(0, ROOT)
    import bench
    wl = bench.WORKLOADS[workload]
    seeds = [1234 + i for i in range(min(64, n))]
    pool = bench.make_pool(seeds, wl["w"], wl["h"], wl["sampling"], wl["quality"], procs=16,
                           restart=wl.get("restart", 0))
    return sum(len(pool[i % len(pool)]) for i in range(n)) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "parse", "pipeline"])
    ap.add_argument("dirs", nargs="*")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--images", type=int, default=0)
    ap.add_argument("--kernel", default="k_gw_lane")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--pipeline-out", default="", help="also write the whole-pipeline per-kernel traffic here")
    args = ap.parse_args()
    if args.mode == "run":
        run(args)
    elif args.mode == "pipeline":  # re-parse two PMC dirs of a run into the whole-pipeline table
        w, h = {"c2": (1024, 1024)}.get(args.workload, (4096, 4096))
        comp = _comp_bytes_per_image(args.workload, args.images)
        print(json.dumps(pipeline(args.dirs[0], args.dirs[1], args.workload, args.images, w, h, comp,
                                  args.pipeline_out or None)))
    else:
        print(json.dumps(parse(args.dirs[0], args.dirs[1], args.kernel, args.workload, args.images or None)))


if __name__ == "__main__":
    sys.exit(main())
