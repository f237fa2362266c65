#!/usr/bin/env python3
"""Summary of the VALU issue-rate calibration (tools/probe/valu_issue, tools/probe/sel_issue):
SIMD cycles per vector instruction by instruction mix and waves per SIMD (from the probes' own
clocks: the slowest wave's s_memtime cycles / (waves x instructions per wave)), and what the SQ
counters read for the same kernels (one rocprofv3 --pmc pass over valu_issue).
    python3 tools/valu_calib.py VALU_JSONL SEL_JSONL PMC_DIR > profiles/r06_valu_issue_calibration.json"""
import collections
import csv
import glob
import json
import sys

MIX = {0: "add", 1: "bfe", 2: "shl64", 3: "cnd", 4: "gw", 5: "dep", 6: "gwlds"}


def table(path, key):
    rows = [json.loads(l) for l in open(path) if l.startswith("{")]
    out = collections.OrderedDict()
    for r in rows:
        out.setdefault(r[key], {})[r["waves_per_simd"]] = {
            "simd_cyc_per_inst": round(r["simd_cyc_per_valu"], 3), "clock_ghz": round(r["clock_ghz"], 3)}
    return out


def pmc(d):
    agg = collections.OrderedDict()
    meta = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            agg.setdefault(k, collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
            meta[k] = (r["Kernel_Name"], int(r["Grid_Size"]))
    out = []
    for k, c in agg.items():
        name, grid = meta[k]
        if c.get("SQ_INSTS_VALU", 0) < 1e7:  # the 16-iteration warm-up launches
            continue
        mix = MIX.get(int(name.split("<")[1].split(">")[0]), name) if "<" in name else name
        w = grid // 256 // 256
        simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024  # GRBM is summed over the 8 XCDs
        out.append({
            "mix": mix, "waves_per_simd": w,
            "valu_per_simd_cycle_from_grbm": round(c["SQ_INSTS_VALU"] / simd_cycles, 3),
            "active_inst_valu_over_insts_valu": round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"], 3),
            "valu2_quadcycles_over_insts_valu": round(c["SQ_ACTIVE_INST_VALU2"] / c["SQ_INSTS_VALU"], 3),
            "design_r05_valu_busy_x4": round(c["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles, 3),
        })
    return out


def main():
    vj, sj, pd = sys.argv[1:4]
    res = {
        "what": "SIMD cycles per wave64 vector instruction on gfx950 (MI355X), by mix and waves per SIMD",
        "probes": ["tools/probe/valu_issue.hip", "tools/probe/sel_issue.hip"],
        "valu_issue": table(vj, "mix"),
        "sel_issue": table(sj, "case"),
        "pmc_valu_issue": pmc(pd),
    }
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
