#!/usr/bin/env python3
"""Per-kernel SQ counter summary from rocprofv3 --pmc CSV directories (GPU box output).
usage: tools/sq_summary.py DIR [DIR ...]"""
import collections
import csv
import glob
import sys


def load(dirs):
    agg = collections.defaultdict(float)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("icx::", "")
                agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
    return agg


def main():
    agg = load(sys.argv[1:])
    kernels = sorted({k for k, _ in agg}, key=lambda k: -agg.get((k, "SQ_WAVE_CYCLES"), 0))
    g = lambda k, c: agg.get((k, c), 0.0)
    print(f"{'kernel':18s} {'waves':>7s} {'act%':>5s} {'wait%':>5s} {'issue%':>6s} | per wave: {'VALU':>7s} {'SALU':>7s} {'LDS':>6s} | active VALU/LDS/SCA/VMEM % of cycles")
    for k in kernels:
        wc = g(k, "SQ_WAVE_CYCLES")
        if wc <= 0:
            continue
        w = max(1.0, g(k, "SQ_WAVES"))
        print(f"{k:18s} {w:7.0f} {100*g(k,'SQ_ACTIVE_INST_ANY')/wc:5.1f} {100*g(k,'SQ_WAIT_ANY')/wc:5.1f} "
              f"{100*g(k,'SQ_WAIT_INST_ANY')/wc:6.1f} | {g(k,'SQ_INSTS_VALU')/w:15.0f} {g(k,'SQ_INSTS_SALU')/w:7.0f} "
              f"{g(k,'SQ_INSTS_LDS')/w:6.0f} | {100*g(k,'SQ_ACTIVE_INST_VALU')/wc:4.1f} {100*g(k,'SQ_ACTIVE_INST_LDS')/wc:4.1f} "
              f"{100*g(k,'SQ_ACTIVE_INST_SCA')/wc:4.1f} {100*g(k,'SQ_ACTIVE_INST_VMEM')/wc:4.1f}")
    dump_all(agg, kernels)


def dump_all(agg, kernels):
    """Every counter collected, per kernel (raw sums; GRBM_* are chip-wide ticks summed over XCDs)."""
    names = sorted({c for _, c in agg})
    print()
    for k in kernels[:12]:
        vals = ", ".join(f"{c}={agg[(k, c)]:.4g}" for c in names if (k, c) in agg)
        print(f"{k}: {vals}")


if __name__ == "__main__":
    main()
