#!/usr/bin/env python3
"""Timing aid (GPU box): icx_exr_decode of synthetic half RGBA EXRs per compression, host in ->
host out, and the per-kernel split from rocprofv3 when run under it."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import imagecodecs_amd as icx  # noqa: E402
from tools import exrwrite as W  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    y, x = np.mgrid[0:n, 0:n].astype(np.float32)
    rng = np.random.default_rng(1)
    chans = [(c, (np.sin(x * (0.01 + 0.003 * k)) * np.cos(y * 0.013) * 50 + rng.normal(0, 0.05, (n, n))).astype(np.float16))
             for k, c in enumerate("RGBA")]
    ctx = icx.Context(0)
    for comp, name in ((W.NONE, "none"), (W.ZIPS, "zips"), (W.ZIP, "zip")):  # (RLE: the writer is pure Python)
        data = W.write_exr(chans, compression=comp)
        ctx.exr_decode(data)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            code, w, h, img = ctx.exr_decode(data)
        dt = (time.perf_counter() - t0) / reps
        print(f"{name:5s} {n}x{n} {len(data) / 1e6:7.2f} MB  {dt * 1e3:8.2f} ms  {n * n / dt / 1e6:8.1f} MP/s  code {code}", flush=True)


if __name__ == "__main__":
    main()
