#!/usr/bin/env python3
"""Benchmark: batched JPEG decode on MI355X (BASELINE.json metric: megapixels/s JPEG decode of
synthetic RGB batches at 1/2/4/8 GPUs, plus % of HBM roofline).

A "step" = one call of the device-resident batch decode (icx_jpeg_batch_decode) over this
rank's shard of images, compressed input already resident in HBM, RGB output written to HBM.
Workloads:
  c3   (default) per GPU: 512 synthetic 4096x4096 baseline JPEGs, 4:2:0, q90 -- config C3's
       per-GPU shard (C3 = 4096 images on 8 GPUs). Weak scaling: every rank decodes its own
       512 images; the only collective is the final gather of per-image statuses (RCCL).
  c2   per GPU: 1024 synthetic 1024x1024 4:2:0 q90 JPEGs (config C2).
Images come from a pool of --pool distinct synthetic images (tools/synth.c, seeded per rank)
cycled to fill the batch.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N>1 under torch.distributed.run
(one rank per GPU; RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the env). Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import json
from multiprocessing.pool import ThreadPool
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

# stage (icx_batch_stage_times) -> the kernel it times
STAGE_KERNEL = {"write": "k_gw_lane", "idct": "k_idct420s (4:2:0 chroma planes; plane mode 5)",
                "convert": "k_fused420s (4:2:0 luma IDCT + conversion)+k_convert_stream+k_convert_edge",
                "unstuff": "k_ustf_count+k_ustf_scan+k_ustf_write",
                "entropy": "k_gw_check+k_gw_count+k_gw_repair+k_gw_scan+k_gw_map",
                "parse": "k_parse", "upsample": "k_upsample"}
GW_MIN_PIXELS = 2048 * 2048  # icx_internal.h kGwMinPixels: larger workspaces take the guess-write path
DRI_GW_MIN = 4096  # icx_internal.h kDriGwMin: restart intervals from this many bytes take guess-write lanes


def coef_cell_bytes():
    """Bytes one coefficient block occupies in the pool (icx_internal.h: 64 int16 cells)."""
    return 128


def pipeline_traffic(workload, n, alg_bytes):
    """Whole-step HBM traffic from the committed PMC profile (tools/pmc_traffic.py pipeline: every
    kernel's FETCH_SIZE x correction + WRITE_SIZE, per image), scaled to this run's n images, and
    its ratio to the step's algorithmic bytes. Empty when no profile of this workload exists."""
    p = os.path.join(ROOT, "profiles", "pipeline_traffic.json")
    if not os.path.exists(p):
        return {}
    tj = json.load(open(p))
    if tj.get("workload") != workload:
        return {}
    moved = tj["moved_MB_per_image"] * 1e6 * n
    return {"pipeline_traffic": round(moved), "moved_over_alg": round(moved / alg_bytes, 3),
            "pipeline_traffic_source": "profiles/pipeline_traffic.json (" + tj.get("source", "PMC run") + ")"}


def stage_kernels(w, h, restart=0, interval_bytes=0):
    """STAGE_KERNEL for a batch of w x h images: the three-pass entropy path's kernels where the
    library takes it (ICX_GW=0, or a workspace for images of at most GW_MIN_PIXELS); with restart
    markers the write stage is the restart-interval lanes (icx_spec.hip: one lane per interval),
    unless the guess-write path cuts the intervals into lanes (k_spec_plan: intervals averaging
    DRI_GW_MIN compressed bytes or more; ICX_DRI_GW=0 never, 1 from 512)."""
    env = os.environ.get("ICX_GW")
    gw = env != "0" if env is not None else w * h > GW_MIN_PIXELS
    k = dict(STAGE_KERNEL)
    if not gw:
        k.update(write="k_spec_write", entropy="k_spec_guess+k_spec_count+k_spec_scan")
    if restart:
        denv = os.environ.get("ICX_DRI_GW")
        dmin = (512 if denv != "0" else None) if denv is not None else DRI_GW_MIN
        if gw and dmin is not None and interval_bytes >= dmin:
            k.update(write="k_gw_lane (interval-aligned lanes)+k_spec_write<256> (fallbacks)")
        else:
            k.update(write="k_spec_write<256> (restart-interval lanes)")
    return k

WORKLOADS = {
    "c3": dict(n=512, w=4096, h=4096, sampling="420", quality=90,
               desc="C3 per-GPU shard: 512 x 4096x4096 4:2:0 q90 baseline JPEG (C3 = 4096 images / 8 GPUs)"),
    "c2": dict(n=1024, w=1024, h=1024, sampling="420", quality=90,
               desc="C2: 1024 x 1024x1024 4:2:0 q90 baseline JPEG"),
    "c2048": dict(n=256, w=2048, h=2048, sampling="420", quality=90,
                  desc="256 x 2048x2048 4:2:0 q90 baseline JPEG (between C2 and C3: entropy path crossover)"),
    "c3dri": dict(n=512, w=4096, h=4096, sampling="420", quality=90, restart=256,
                  desc="C3 shard with restart markers every MCU row (DRI 256): camera-style streams"),
    "c4": dict(n=64, w=4096, h=4096, sampling="420", quality=90,
               desc="C4 encode: 64 x 4096x4096 RGB -> baseline JPEG 4:2:0 q90 per GPU (encode extension)"),
    "c5": dict(n=8, w=8192, h=8192,
               desc="C5 PNG encode: 8 x 8192x8192 RGBA (alpha = horizontal gradient, lodepng keeps RGBA) per GPU"),
    "hdr": dict(n=32, w=4096, h=4096, mode=0,
                desc="HDR read: 32 x 4096x4096 Radiance RGBE, new-style RLE scanlines -> 4 floats/px (readHdr)"),
    "hdrflat": dict(n=32, w=4096, h=4096, mode=1,
                    desc="HDR read: 32 x 4096x4096 Radiance RGBE, flat pixel data -> 4 floats/px (readHdr)"),
    "exr": dict(n=32, w=2048, h=2048,
                desc="EXR read: 32 x 2048x2048 half RGBA, ZIP scanline chunks -> 4 floats/px (readExr -> tinyexr)"),
}

# encode stage (icx_encoder_stage_times) -> kernels it times
ENC_STAGE_KERNEL = {"encode": "k_enc_run", "stuff": "k_stuff_count_b+scan+k_stuff_write_b"}


def _gen(args):
    seed, w, h, sampling, quality, restart = args
    from tools import synthpy
    return synthpy.synth_jpeg(seed, w, h, sampling, quality, restart)


def make_pool(seeds, w, h, sampling, quality, procs, restart=0):
    # threads, not processes: the generator is a ctypes call into C (the GIL is released), and
    # forked workers do not mix with profilers that preload into the process
    jobs = [(s, w, h, sampling, quality, restart) for s in seeds]
    if procs <= 1 or len(jobs) == 1:
        return [_gen(j) for j in jobs]
    with ThreadPool(procs) as p:
        return p.map(_gen, jobs)


def _oracle_decode(data):
    from oracle import pyoracle
    t = time.perf_counter()
    code, w, h, n, pix = pyoracle.decode(data)
    return time.perf_counter() - t, code, hashlib.sha256(pix).hexdigest(), w * h


def host_cores(value_1core, unit):
    """The box's core counts beside the measured share. A one-GPU box runs its jobs on a 16-CPU
    share of a shared host (the pool's rule: size worker pools to it), so the all-core figure is
    stated as the one-core rate times the host's cores (decodes are independent, one image per
    core; memory bandwidth is not the limit at ~30 MP/s per core), never measured by loading the
    whole machine."""
    total = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = total
    return {"host_cores_total": total, "host_cores_usable": usable,
            "value_all_cores_est": round(value_1core * total, 1),
            "all_cores_note": f"one-core rate x {total} host cores ({unit}); linear estimate, not measured: the "
                              f"GPU box's jobs are limited to a 16-CPU share of the host"}


def cpu_baseline(pool, target_s, cores):
    """Time the oracle (bit-exact CPU restatement of NanoJPEG; the reference is not on the GPU
    box) on a bounded sample of the same pool: one image per worker thread on `cores` cores, then
    one core alone. The restatement's speed relative to the reference NanoJPEG build is measured
    in the container (tools/cpu_calibrate.py -> profiles/cpu_calibration.json) and reported."""
    probe_t, _, _, px = _oracle_decode(pool[0])
    per_core = max(1, int(target_s / max(probe_t, 1e-3)))
    sample = [pool[i % len(pool)] for i in range(per_core * cores)]
    t0 = time.perf_counter()
    if cores > 1:  # one oracle decode per thread; ctypes releases the GIL for the C decode
        with ThreadPool(cores) as p:
            res = p.map(_oracle_decode, sample)
    else:
        res = [_oracle_decode(s) for s in sample]
    wall = time.perf_counter() - t0
    mpx = sum(r[3] for r in res) / 1e6
    hashes = {}
    for s, r in zip(sample, res):
        hashes[hashlib.sha256(s).hexdigest()] = r[2]
    # one core: a third of the budget, whole images in sequence
    n1 = max(1, int(target_s / 3 / max(probe_t, 1e-3)))
    t1 = time.perf_counter()
    res1 = [_oracle_decode(pool[i % len(pool)]) for i in range(n1)]
    wall1 = time.perf_counter() - t1
    out = {"value": round(mpx / wall, 2), "unit": "megapixels/s", "cores": cores, "kind": "port",
           "sample": f"{len(sample)} images of the same pool ({len(sample) // cores} per core), oracle/ "
                     f"NanoJPEG restatement, {wall:.1f} s wall",
           "value_1core": round(sum(r[3] for r in res1) / 1e6 / wall1, 2),
           "sample_1core": f"{n1} images on one core, {wall1:.1f} s"}
    out.update(host_cores(out["value_1core"], "megapixels/s"))
    cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if os.path.exists(cal):
        c = json.load(open(cal))
        out["port_over_reference"] = c.get("ratio_4096")
        out["calibration"] = "profiles/cpu_calibration.json (restatement vs oracle/_ref NanoJPEG, same images, container)"
    return out, hashes


def _oracle_encode(args):
    from oracle import pyoracle
    px, w, h, q, sub = args
    t = time.perf_counter()
    jpg = pyoracle.jpeg_encode(q, sub, w, h, 3, px)
    return time.perf_counter() - t, hashlib.sha256(jpg).hexdigest(), w * h


def cpu_baseline_encode(images, w, h, q, sub, target_s, cores):
    """Time the oracle encoder (or_jpeg_encode, the C4 definition) on a bounded sample."""
    probe_t = _oracle_encode((images[0], w, h, q, sub))[0]
    per_core = max(1, int(target_s / max(probe_t, 1e-3)))
    sample = [(images[i % len(images)], w, h, q, sub) for i in range(per_core * cores)]
    t0 = time.perf_counter()
    with ThreadPool(max(1, cores)) as p:
        res = p.map(_oracle_encode, sample)
    wall = time.perf_counter() - t0
    hashes = {i % len(images): r[1] for i, r in enumerate(res)}
    return {"value": round(sum(r[2] for r in res) / 1e6 / wall, 2), "unit": "megapixels/s", "cores": cores,
            "kind": "port", "sample": f"{len(sample)} encodes of the same images ({per_core} per core), "
                                      f"oracle/ or_jpeg_encode, {wall:.1f} s wall"}, hashes


def main_encode(args, wl, world, rank, local):
    """C4: device-resident encode of a per-rank batch of RGB images (one icx_jpeg_encode_device_batch
    call per step, inputs resident in HBM, files written to HBM)."""
    from imagecodecs_amd import shard
    from tools import synthpy
    n = args.images or wl["n"]
    W, H, Q, SUB = wl["w"], wl["h"], wl["quality"], int(wl["sampling"])
    first, _ = shard.shard_range(n * world, world, rank)
    npool = min(args.pool, n)
    with ThreadPool(min(16, npool)) as p:
        images = p.map(lambda i: synthpy.rgb(1234 + first + i, W, H, 3).tobytes(), range(npool))
    cpu, cpu_hashes = None, {}
    if rank == 0 and not args.no_cpu:
        cpu, cpu_hashes = cpu_baseline_encode(images[:4], W, H, Q, SUB, args.cpu_seconds, args.cpu_cores)

    import torch
    import imagecodecs_amd as icx
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    d_src = torch.empty((npool, H * W * 3), dtype=torch.uint8, device=dev)
    for i, im in enumerate(images):
        d_src[i].copy_(torch.frombuffer(bytearray(im), dtype=torch.uint8))
    cap = W * H * 3 + (1 << 16)
    d_out = torch.empty((n, cap), dtype=torch.uint8, device=dev)
    sizes = np.zeros(n, np.int64)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    ctx = icx.Context(local)
    enc = icx.Encoder(ctx)
    stream = torch.cuda.current_stream(dev)

    srcs = [d_src[i % npool].data_ptr() for i in range(n)]

    def step():  # one batch call: one fused encode launch + the stuffing pair, one host wait
        st, sz = enc.encode_device_batch(Q, SUB, W, H, 3, srcs, d_out.data_ptr(), cap, stream.cuda_stream)
        sizes[:] = sz
        if (st != icx.OK).any():
            d_st.copy_(torch.from_numpy(st.astype(np.int32)))
        return d_st

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    enc.stage_times()  # reset the accumulators
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    last = d_st
    for _ in range(args.steps):
        last = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    stages = {k: v / args.steps for k, v in enc.stage_times().items()}  # ms per step
    if world > 1:  # the final gather of every rank's statuses, after the timed steps
        last = shard.gather_results(last, dist)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    ok_all = bool((last.cpu().numpy() == 0).all())
    checked = mismatches = 0
    for i, hx in cpu_hashes.items():
        if i < n:
            got = hashlib.sha256(d_out[i, : sizes[i]].cpu().numpy().tobytes()).hexdigest()
            checked += 1
            mismatches += got != hx
    comp = float(sizes.sum())
    alg_bytes = n * W * H * 3.0 + comp  # read RGB + write the files
    ms_step = elapsed / args.steps * 1e3
    value = world * n * W * H / 1e6 / (elapsed / args.steps)
    dom = max((k for k in stages if stages[k] > 0), key=lambda k: stages[k], default=None)
    roof = None
    if dom:
        # per-launch algorithmic bytes of the dominant kernel: one k_enc_run launch per step
        # encodes every image of the batch, reading its RGB pixels (3 B/px) and writing its
        # entropy-coded stream (the words the stuffing pass reads); the stuffing pass reads that
        # stream and writes the stuffed file
        per_img = {"encode": W * H * 3 + comp / n, "stuff": 2 * comp / n}.get(dom, W * H * 3)
        avg = stages[dom]
        achieved = n * per_img / (avg * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": ENC_STAGE_KERNEL.get(dom, dom), "launches_per_step": 1,
                "alg_bytes_per_launch": round(n * per_img), "avg_launch_ms": round(avg, 4),
                "stage_ms": {k: round(v, 3) for k, v in stages.items()},
                "pipeline_frac": round(alg_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
    out = {
        "metric": "megapixels/s JPEG encode, 4096x4096 RGB", "value": round(value, 2), "unit": "megapixels/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (tools/synth.c RGB, seeded)",
        "config": {"workload": wl["desc"], "images_per_gpu": n, "pool": npool, "width": W, "height": H,
                   "quality": Q, "subsampling": SUB, "bytes_per_pixel_compressed": round(comp / (n * W * H), 4),
                   "parallelism": f"dp{world} (images sharded; one RCCL all-gather of statuses after the timed steps)"},
        "roofline": roof, "cpu_baseline": cpu,
        "parity": {"all_status_ok": ok_all, "images_checked_vs_oracle": checked, "mismatches": mismatches},
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


PNG_STAGE_KERNEL = {"stats": "k_png_stats", "filter": "k_png_filter", "lz77": "k_png_lz77",
                    "huff": "k_png_huff+k_png_segbits+hipcub scan+k_png_adler", "emit": "k_png_emit",
                    "crc": "k_png_crc_seg+k_png_crc_combine"}


def _oracle_png(args):
    from oracle import pyoracle
    px, w, h = args
    t = time.perf_counter()
    png = pyoracle.png_encode_zlib(px, w, h, 4, 6)
    return time.perf_counter() - t, len(png), w * h


def main_png(args, wl, world, rank, local):
    """C5: device-resident PNG encode (png_encoder::saveToFile) of a per-rank batch of RGBA images,
    one icx_png_encode_device_batch call per step (--png-single: one icx_png_encode_device call per
    image), pixels resident in HBM, files written to HBM."""
    import zlib
    from imagecodecs_amd import shard
    from tests import pngutil
    n = args.images or wl["n"]
    W, H = wl["w"], wl["h"]
    first, _ = shard.shard_range(n * world, world, rank)
    npool = min(args.pool, n, 2)
    images = [pngutil.synth_rgba(1234 + first + i, W, H).tobytes() for i in range(npool)]
    cpu = None
    if rank == 0 and not args.no_cpu:
        # bounded sample: one whole image per worker, concurrently (ctypes drops the GIL)
        cores = args.cpu_cores
        sample = [(images[i % npool], W, H) for i in range(cores)]
        t0 = time.perf_counter()
        with ThreadPool(cores) as p:
            res = p.map(_oracle_png, sample)
        wall = time.perf_counter() - t0
        cpu = {"value": round(sum(r[2] for r in res) / 1e6 / wall, 2), "unit": "megapixels/s", "cores": cores,
               "kind": "port", "sample": f"{len(sample)} encodes of the same images (1 per core), oracle/ restated "
                                         f"lodepng colour choice + MINSUM filters, deflate by system zlib level 6 "
                                         f"(stand-in for lodepng's deflate), {wall:.1f} s wall"}

    import torch
    import imagecodecs_amd as icx
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    d_src = torch.empty((npool, H * W * 4), dtype=torch.uint8, device=dev)
    for i, im in enumerate(images):
        d_src[i].copy_(torch.frombuffer(bytearray(im), dtype=torch.uint8))
    cap = W * H * 4 + W * H // 16 + (1 << 20)
    d_out = torch.empty((n, cap), dtype=torch.uint8, device=dev)
    sizes = np.zeros(n, np.int64)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    ctx = icx.Context(local)
    enc = icx.PngEncoder(ctx)
    stream = torch.cuda.current_stream(dev)

    srcs = [d_src[i % npool].data_ptr() for i in range(n)]

    def step():
        if args.png_single:  # one icx_png_encode_device call per image (round 2's loop)
            for i in range(n):
                rc, sizes[i] = enc.encode_device(W, H, 4, srcs[i], d_out[i].data_ptr(), cap, stream.cuda_stream)
                if rc != icx.OK:
                    d_st[i] = rc
        else:  # icx_png_encode_device_batch: ICX_PNG_INFLIGHT (default 8) images in flight
            st, sz = enc.encode_device_batch(W, H, 4, srcs, d_out.data_ptr(), cap, stream.cuda_stream)
            sizes[:] = sz
            if (st != icx.OK).any():
                d_st.copy_(torch.from_numpy(st.astype(np.int32)))
        return d_st

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    enc.stage_times()  # reset the accumulators
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    last = d_st
    for _ in range(args.steps):
        last = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    stages = {k: v / args.steps for k, v in enc.stage_times().items()}  # ms per step
    if world > 1:  # the final gather of every rank's statuses, after the timed steps
        last = shard.gather_results(last, dist)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ok_all = bool((last.cpu().numpy() == 0).all())
    checked = mismatches = 0
    if rank == 0 and not args.no_cpu:
        # parity of the measured output: IHDR/colour type as lodepng chooses, and the IDAT inflates
        # to exactly the oracle's filtered stream (lodepng's filter bytes)
        from oracle import pyoracle
        for i in range(npool):
            info = pngutil.info(d_out[i, : sizes[i]].cpu().numpy().tobytes())
            mode = pyoracle.png_choose(images[i], W, H, 4)
            want = pyoracle.png_filtered(images[i], W, H, 4, mode)
            checked += 1
            mismatches += (info["colortype"] != mode.colortype or info["bitdepth"] != mode.bitdepth or
                           zlib.decompress(info["idat"]) != want)
    out_b = float(sizes.sum())
    N = H * (1 + W * 4)  # filtered stream bytes per image (RGBA kept)
    alg_bytes = n * W * H * 4.0 + out_b  # read RGBA + write the files
    ms_step = elapsed / args.steps * 1e3
    value = world * n * W * H / 1e6 / (elapsed / args.steps)
    dom = max((k for k in stages if stages[k] > 0), key=lambda k: stages[k], default=None)
    roof = None
    if dom:
        # per-launch algorithmic bytes of the dominant stage (one launch per image): stats reads the
        # pixels; filter reads the pixels and writes the filtered stream; lz77 reads the filtered
        # stream; emit and crc touch the output file
        per_img = {"stats": W * H * 4.0, "filter": W * H * 4.0 + N, "lz77": float(N), "huff": 0.0,
                   "emit": out_b / n, "crc": out_b / n}.get(dom, alg_bytes / n)
        avg = stages[dom] / n
        achieved = per_img / (avg * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": PNG_STAGE_KERNEL.get(dom, dom), "launches_per_step": n,
                "alg_bytes_per_launch": round(per_img), "avg_launch_ms": round(avg, 4),
                "stage_ms": {k: round(v, 3) for k, v in stages.items()},
                "stage_ms_note": ("per-image HIP events summed over the images; with the batch entry several "
                                  "images run at once on their own streams, so the sums overlap and exceed the "
                                  "wall time, and avg_launch_ms (hence achieved) understates the kernel's rate")
                                 if not args.png_single else "per-image HIP events summed over the images",
                "pipeline_frac": round(alg_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
    out = {
        "metric": "megapixels/s PNG encode, 8192x8192 RGBA", "value": round(value, 2), "unit": "megapixels/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (tools/synth.c RGB + alpha gradient, seeded)",
        "config": {"workload": wl["desc"], "images_per_gpu": n, "pool": npool, "width": W, "height": H,
                   "png_bytes_per_pixel": round(out_b / (n * W * H), 4),
                   "parallelism": f"dp{world} (images sharded; one RCCL all-gather of statuses after the timed steps)"},
        "roofline": roof, "cpu_baseline": cpu,
        "parity": {"all_status_ok": ok_all, "images_checked_vs_oracle": checked, "mismatches": mismatches},
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


HDR_STAGE_KERNEL = {"parse": "k_hdr_parse", "locate": "k_hdr_scan+k_hdr_flatcheck+k_hdr_link+k_hdr_walk",
                    "unpack": "k_hdr_unpack", "convert": "k_hdr_convert+k_hdr_finish"}


def _oracle_hdr(data):
    from oracle import pyoracle
    t = time.perf_counter()
    code, w, h, rows, arr = pyoracle.hdr_decode(data)
    return time.perf_counter() - t, code, hashlib.sha256(arr.tobytes()).hexdigest(), w * h


def main_hdr(args, wl, world, rank, local):
    """Radiance .hdr read: one icx_hdr_batch_decode of the rank's images
    per step, files resident in HBM, floats written to HBM."""
    from imagecodecs_amd import shard
    from tools import synthpy
    n = args.images or wl["n"]
    W, H = wl["w"], wl["h"]
    first, _ = shard.shard_range(n * world, world, rank)
    npool = min(args.pool, n, 4)
    with ThreadPool(npool) as p:
        files = p.map(lambda i: synthpy.hdr(synthpy.rgbe(1234 + first + i, W, H), wl["mode"]), range(npool))
    cpu, cpu_hashes = None, {}
    if rank == 0 and not args.no_cpu:
        probe_t = _oracle_hdr(files[0])[0]
        cores = args.cpu_cores
        per_core = max(1, int(args.cpu_seconds / max(probe_t, 1e-3)))
        sample = [files[i % npool] for i in range(per_core * cores)]
        t0 = time.perf_counter()
        with ThreadPool(cores) as p:
            res = p.map(_oracle_hdr, sample)
        wall = time.perf_counter() - t0
        cpu = {"value": round(sum(r[3] for r in res) / 1e6 / wall, 2), "unit": "megapixels/s", "cores": cores,
               "kind": "port", "sample": f"{len(sample)} decodes of the same files ({per_core} per core), oracle/ "
                                         f"readHdr restatement, {wall:.1f} s wall"}
        cpu_hashes = {i % npool: r[2] for i, r in enumerate(res)}

    import torch
    import imagecodecs_amd as icx
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    fl = [files[i % npool] for i in range(n)]
    sizes = np.array([len(f) for f in fl], np.int64)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum((sizes[:-1] + 15) // 16 * 16)
    blob = np.zeros(int(offs[-1] + sizes[-1]), np.uint8)
    for i, f in enumerate(fl):
        blob[offs[i]: offs[i] + sizes[i]] = np.frombuffer(f, np.uint8)
    d_data = torch.from_numpy(blob).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_sz = torch.from_numpy(sizes).to(dev)
    stride = W * H * 4
    d_out = torch.empty(n * stride, dtype=torch.float32, device=dev)
    d_st = torch.empty(n, dtype=torch.int32, device=dev)
    d_dims = torch.empty((n, 3), dtype=torch.int32, device=dev)
    ctx = icx.Context(local)
    batch = icx.HdrBatch(ctx, n, W, H)
    stream = torch.cuda.current_stream(dev)
    stage_acc = {}

    def step():
        batch.decode_device(n, d_data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), d_out.data_ptr(), stride,
                            d_st.data_ptr(), d_dims.data_ptr(), stream.cuda_stream)
        return d_st

    for _ in range(args.warmup):
        step()
    if args.graph:  # one step captured (the library launches without host waits under capture), then replays
        if M != 1:
            raise SystemExit("--graph takes one batch (no --inflight)")
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            batch.decode_device(n, d_data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), d_out[0].data_ptr(), stride,
                                d_st[0].data_ptr(), d_dims[0].data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)

        def step():
            graph.replay()
            return 0
        for _ in range(max(1, args.warmup)):
            step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for k, v in batch.stage_times().items():  # synchronises on the step's stage events
            stage_acc[k] = stage_acc.get(k, 0.0) + v
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    last = shard.gather_results(d_st, dist) if world > 1 else d_st
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    stages = {k: v / args.steps for k, v in stage_acc.items()}
    ok_all = bool((last.cpu().numpy() == 0).all())
    checked = mismatches = 0
    for i, hx in cpu_hashes.items():
        got = hashlib.sha256(d_out[i * stride: (i + 1) * stride].cpu().numpy().tobytes()).hexdigest()
        checked += 1
        mismatches += got != hx
    ms_step = elapsed / args.steps * 1e3
    value = world * n * W * H / 1e6 / (elapsed / args.steps)
    file_b = float(sizes.sum())
    alg_bytes = file_b + n * W * H * 16.0  # read the files, write 4 floats per pixel
    dom = max((k for k in stages if stages[k] > 0), key=lambda k: stages[k], default=None)
    roof = None
    if dom:
        # per-launch algorithmic bytes of the dominant stage over the whole batch (one launch per
        # step): convert reads RGBE (planes or file) 4 B/px and writes 16 B/px; locate and unpack
        # read the pixel data once (unpack also writes the 4 B/px RGBE planes)
        per = {"convert": n * W * H * 20.0, "unpack": file_b + n * W * H * 4.0, "locate": file_b,
               "parse": 0.0}.get(dom, alg_bytes)
        achieved = per / (stages[dom] * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "kernel": HDR_STAGE_KERNEL.get(dom, dom),
                "launches_per_step": 1, "alg_bytes_per_launch": round(per), "avg_launch_ms": round(stages[dom], 4),
                "stage_ms": {k: round(v, 3) for k, v in stages.items()},
                "pipeline_frac": round(alg_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
    out = {
        "metric": "megapixels/s Radiance HDR read, 4096x4096 RGBE -> float", "value": round(value, 2),
        "unit": "megapixels/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8->f32", "data": "synthetic (tools/synth.c synth_rgbe + hdr_encode, seeded)",
        "config": {"workload": wl["desc"], "images_per_gpu": n, "pool": npool, "width": W, "height": H,
                   "file_bytes_per_pixel": round(file_b / (n * W * H), 4),
                   "parallelism": f"dp{world} (images sharded; one RCCL all-gather of statuses after the timed steps)"},
        "roofline": roof, "cpu_baseline": cpu,
        "parity": {"all_status_ok": ok_all, "images_checked_vs_oracle": checked, "mismatches": mismatches},
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def _exr_image(seed, w, h):
    """Synthetic half RGBA EXR (ZIP): smooth waves plus noise, as tools/exr_time.py."""
    from tools import exrwrite as EW
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    rng = np.random.default_rng(seed)
    chans = [(c, (np.sin(x * (0.01 + 0.003 * k)) * np.cos(y * (0.013 + 0.001 * (seed % 5))) * 50 +
                  rng.normal(0, 0.05, (h, w))).astype(np.float16)) for k, c in enumerate("RGBA")]
    return EW.write_exr(chans, compression=EW.ZIP)


def _oracle_exr(data):
    from oracle import exr_oracle
    t0 = time.perf_counter()
    code, w, h, arr = exr_oracle.decode(data)
    return time.perf_counter() - t0, code, hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest(), w * h


def main_exr(args, wl, world, rank, local):
    """OpenEXR read (the row beside readHdr, tinyexr LoadEXRFromMemory): the files resident in HBM,
    one icx_exr_decode_device_batch per step over the rank's files (headers and offset tables
    planned on the host from their copies; every file's chunks inflated and un-predicted by one
    launch, then converted per file on the GPU; floats written to HBM; the call synchronises)."""
    from imagecodecs_amd import shard
    n = args.images or wl["n"]
    W, H = wl["w"], wl["h"]
    first, _ = shard.shard_range(n * world, world, rank)
    npool = min(args.pool, n, 4)
    with ThreadPool(npool) as p:
        files = p.map(lambda i: _exr_image(1234 + first + i, W, H), range(npool))
    cpu, cpu_hashes = None, {}
    if rank == 0 and not args.no_cpu:
        probe_t = _oracle_exr(files[0])[0]
        cores = args.cpu_cores
        per_core = max(1, int(args.cpu_seconds / max(probe_t, 1e-3)))
        per_core = max(1, min(per_core, 24))
        sample = [files[i % npool] for i in range(per_core * cores)]
        import multiprocessing as mp
        t0 = time.perf_counter()
        with mp.get_context("fork").Pool(cores) as p:  # (before any GPU use: fork is safe)
            res = p.map(_oracle_exr, sample)
        wall = time.perf_counter() - t0
        cpu = {"value": round(sum(r[3] for r in res) / 1e6 / wall, 2), "unit": "megapixels/s", "cores": cores,
               "kind": "port", "sample": f"{len(sample)} reads of the same files ({per_core} per core, {cores} processes), "
                                         f"oracle/ tinyexr restatement (numpy + zlib), {wall:.1f} s wall"}
        cpu_hashes = {i % npool: r[2] for i, r in enumerate(res)}

    import ctypes as C
    import torch
    import imagecodecs_amd as icx
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    fl = [files[i % npool] for i in range(n)]
    sizes = np.array([len(f) for f in fl], np.int64)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum((sizes[:-1] + 16 + 255) // 256 * 256)  # each file + 16 zero bytes, 256-aligned
    blob = np.zeros(int(offs[-1] + sizes[-1] + 16), np.uint8)
    for i, f in enumerate(fl):
        blob[offs[i]: offs[i] + sizes[i]] = np.frombuffer(f, np.uint8)
    d_data = torch.from_numpy(blob).to(dev)
    per_img = W * H * 4
    d_out = torch.empty(n * per_img, dtype=torch.float32, device=dev)
    ctx = icx.Context(local)
    L = icx.lib()
    hbuf = [C.create_string_buffer(f, len(f)) for f in files]  # host copies the plans read
    base_in, base_out = d_data.data_ptr(), d_out.data_ptr()
    hp = (C.c_void_p * n)(*[C.cast(hbuf[i % npool], C.c_void_p) for i in range(n)])
    dp = (C.c_void_p * n)(*[base_in + int(offs[i]) for i in range(n)])
    szp = (C.c_size_t * n)(*[int(x) for x in sizes])
    op = (C.c_void_p * n)(*[base_out + 4 * i * per_img for i in range(n)])
    ofp = (C.c_size_t * n)(*([per_img] * n))
    codes, ws_, hs_ = np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int32)

    def step():  # one icx_exr_decode_device_batch over the rank's files
        rc = L.icx_exr_decode_device_batch(ctx._p, n, hp, dp, szp, op, ofp, codes.ctypes.data, ws_.ctypes.data,
                                           hs_.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"icx_exr_decode_device_batch: {rc}")

    for _ in range(args.warmup):
        step()
    if args.graph:  # one step captured (the library launches without host waits under capture), then replays
        if M != 1:
            raise SystemExit("--graph takes one batch (no --inflight)")
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            batch.decode_device(n, d_data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), d_out[0].data_ptr(), stride,
                                d_st[0].data_ptr(), d_dims[0].data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)

        def step():
            graph.replay()
            return 0
        for _ in range(max(1, args.warmup)):
            step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ok_all = bool((codes == 0).all())
    if world > 1:
        st = torch.from_numpy(codes.copy()).to(dev)
        ok_all = bool((shard.gather_results(st, dist).cpu().numpy() == 0).all())
    checked = mismatches = 0
    for i, hx in cpu_hashes.items():
        got = hashlib.sha256(d_out[i * per_img: (i + 1) * per_img].cpu().numpy().tobytes()).hexdigest()
        checked += 1
        mismatches += got != hx
    ms_step = elapsed / args.steps * 1e3
    value = world * n * W * H / 1e6 / (elapsed / args.steps)
    file_b = float(sizes.sum())
    alg_bytes = file_b + n * W * H * 16.0  # read the files, write 4 floats per pixel
    achieved = alg_bytes / (ms_step * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
            "kernel": "whole batch read (host plans, k_exr_unpack over all chunks, k_exr_convert per file)",
            "launches_per_step": 1, "alg_bytes_per_launch": round(alg_bytes), "avg_launch_ms": round(ms_step, 4),
            "pipeline_frac": round(achieved / HBM_PEAK_GBS, 5)}
    out = {
        "metric": "megapixels/s OpenEXR read, 2048x2048 half RGBA ZIP -> float", "value": round(value, 2),
        "unit": "megapixels/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f16->f32", "data": "synthetic (waves + noise, tools/exrwrite.py ZIP, seeded)",
        "config": {"workload": wl["desc"], "images_per_gpu": n, "pool": npool, "width": W, "height": H,
                   "file_bytes_per_pixel": round(file_b / (n * W * H), 4),
                   "parallelism": f"dp{world} (images sharded; one RCCL all-gather of statuses after the timed steps)"},
        "roofline": roof, "cpu_baseline": cpu,
        "parity": {"all_status_ok": ok_all, "images_checked_vs_oracle": checked, "mismatches": mismatches},
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--images", type=int, default=0, help="override images per GPU")
    ap.add_argument("--pool", type=int, default=64, help="distinct images per rank (SURVEY §8(d): 64)")
    ap.add_argument("--group", type=int, default=0, help="images per workspace group (0=auto)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (rank 0)")
    ap.add_argument("--cpu-cores", type=int, default=min(16, os.cpu_count() or 1),
                    help="CPU-baseline workers (default: the 16-core share of a GPU box)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive sub-batch (decode workloads)")
    ap.add_argument("--png-single", action="store_true", help="C5: one encode call per image (no batch entry)")
    ap.add_argument("--graph", action="store_true",
                    help="decode workloads: capture one step (the whole batch call) in a HIP graph and replay it "
                         "(every entropy round and every layout's back half are enqueued: no host waits)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="decode workloads: steps in flight (0 = the workload's default); step k runs on batch "
                         "k %% M with its own stream and output buffers, so one step's back half overlaps the "
                         "next step's front half")
    args = ap.parse_args()

    # --gpus N: one rank per GPU. Without a launcher (WORLD_SIZE unset) the bench starts
    # torch.distributed.run itself -- as a child, before anything touches the GPU -- and exits
    # with its status; a launcher whose world size differs from --gpus is an error, never a
    # silent single-rank run.
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        import socket
        import subprocess
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
        sys.exit(subprocess.run(cmd).returncode)
    if env_world is not None and int(env_world) != args.gpus and "--gpus" in " ".join(sys.argv):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        sys.exit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    wl = dict(WORKLOADS[args.workload])
    if args.workload == "c4":
        return main_encode(args, wl, world, rank, local)
    if args.workload == "c5":
        return main_png(args, wl, world, rank, local)
    if args.workload.startswith("hdr"):
        return main_hdr(args, wl, world, rank, local)
    if args.workload == "exr":
        return main_exr(args, wl, world, rank, local)
    n = args.images or wl["n"]
    W, H = wl["w"], wl["h"]

    # this rank's shard of the job's image range (weak scaling: n images per GPU); its inputs are
    # generated first (CPU only, before any GPU init so fork() is safe)
    from imagecodecs_amd import shard
    first, last = shard.shard_range(n * world, world, rank)
    seeds = [1234 + first + i for i in range(min(args.pool, n))]
    t = time.perf_counter()
    pool = make_pool(seeds, W, H, wl["sampling"], wl["quality"], procs=min(16, len(seeds)),
                     restart=wl.get("restart", 0))
    gen_s = time.perf_counter() - t
    cpu = None
    cpu_hashes = {}
    if rank == 0 and not args.no_cpu:
        cpu, cpu_hashes = cpu_baseline(pool, args.cpu_seconds, args.cpu_cores)

    import torch
    import imagecodecs_amd as icx

    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    jpegs = [pool[i % len(pool)] for i in range(n)]
    sizes = np.array([len(j) for j in jpegs], np.int64)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum((sizes[:-1] + 15) // 16 * 16)
    blob = np.zeros(int(offs[-1] + sizes[-1]), np.uint8)
    for i, j in enumerate(jpegs):
        blob[offs[i]: offs[i] + sizes[i]] = np.frombuffer(j, np.uint8)
    d_data = torch.from_numpy(blob).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_sz = torch.from_numpy(sizes).to(dev)
    stride = W * H * 3
    # Steps in flight (--inflight M): M batches (each its own workspace groups, pipelines and
    # streams), M output sets, step k on set k % M. A batch call returns once its groups are
    # planned and enqueued, so step k + 1's front half (parse, unstuff, entropy) runs while step k's
    # back half (IDCT, convert) still does: a data loader decoding batch after batch. Every step
    # still decodes all n images into its own buffers; the timed region ends when every stream is
    # done. The batches share the HBM budget: the auto group size takes 80% of free HBM for one
    # batch, so a workload whose workspaces are large gives M > 1 an explicit group per batch
    # (--group, or the workload's inflight_group).
    M = max(1, args.inflight or wl.get("inflight", 1))
    d_out = [torch.empty(n * stride, dtype=torch.uint8, device=dev) for _ in range(M)]
    d_st = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(M)]
    d_dims = [torch.empty((n, 3), dtype=torch.int32, device=dev) for _ in range(M)]

    ctx = icx.Context(local)
    group = args.group or (wl.get("inflight_group", 0) if M > 1 else 0)
    batches = [icx.Batch(ctx, n, W, H, group) for _ in range(M)]
    batch = batches[0]
    stream = torch.cuda.current_stream(dev)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(M - 1)]
    seq = [0]

    def step():  # no collective inside the timed loop: the records gather after it is the only one
        k = seq[0] % M
        seq[0] += 1
        batches[k].decode_device(n, d_data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), d_out[k].data_ptr(), stride,
                                 d_st[k].data_ptr(), d_dims[k].data_ptr(), streams[k].cuda_stream)
        return k

    for _ in range(args.warmup):
        step()
    if args.graph:  # one step captured (the library launches without host waits under capture), then replays
        if M != 1:
            raise SystemExit("--graph takes one batch (no --inflight)")
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            batch.decode_device(n, d_data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), d_out[0].data_ptr(), stride,
                                d_st[0].data_ptr(), d_dims[0].data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)

        def step():
            graph.replay()
            return 0
        for _ in range(max(1, args.warmup)):
            step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    stages = batch.stage_times()  # HIP events on this stream, last step
    paths = batch.path_stats()
    # (outputs of the last step on set 0: every set decodes the same images)
    d_out, d_st, d_dims, last = d_out[0], d_st[0], d_dims[0], d_st[0]

    # Final gather: every rank's per-image records {status, w, h, ncomp,
    # checksum64}, computed on its device (icx_jpeg_records) from the last step's outputs,
    # gathered over RCCL with padding to the largest shard. Outside the timed region.
    d_rec = torch.empty(n * 24, dtype=torch.uint8, device=dev)
    icx.records_device(ctx, n, d_out.data_ptr(), stride, d_st.data_ptr(), d_dims.data_ptr(), W, H, d_rec.data_ptr(),
                       stream.cuda_stream)
    r32 = d_rec.view(torch.int32).reshape(n, 6).to(torch.int64)
    rec = torch.cat([r32[:, :4], ((r32[:, 5] << 32) | (r32[:, 4] & 0xFFFFFFFF))[:, None]], dim=1)
    allrec, counts = shard.gather_records(rec, dist) if world > 1 else (rec, [n])
    allrec = allrec.cpu().numpy()
    # the pool is cycled: every repeat of an image must carry the same checksum (per rank)
    consistent = True
    o = 0
    for r, c in enumerate(counts):
        cs = allrec[o: o + c, 4]
        p = min(args.pool, c)
        consistent &= bool(all((cs[k::p] == cs[k]).all() for k in range(p)))
        o += c
    records = {"gathered": int(allrec.shape[0]), "per_rank": counts, "status_ok": bool((allrec[:, 0] == 0).all()),
               "repeats_consistent": consistent}

    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    # correctness of the measured run: every image of the job OK (the gathered records carry every
    # rank's statuses); this rank's pool images bit-exact vs the oracle
    ok_all = bool((last.cpu().numpy() == 0).all()) and records["status_ok"]
    checked = 0
    mismatches = 0
    if rank == 0 and cpu_hashes:
        for i in range(min(len(pool), n)):
            key = hashlib.sha256(pool[i]).hexdigest()
            if key in cpu_hashes:
                img = d_out[i * stride: i * stride + W * H * 3].cpu().numpy()
                got = hashlib.sha256(img.tobytes()).hexdigest()
                checked += 1
                mismatches += got != cpu_hashes[key]
                # and the gathered record's checksum is that of the oracle-identical pixels
                mismatches += int(int(allrec[i:i + 1, 4].view(np.uint64)[0]) != shard.checksum64(img))

    # PCIe-inclusive rate (rank 0, reported beside `value`, never as it): a bounded sub-batch goes
    # host (pinned) -> HBM, is decoded, and its RGB comes back to pinned host memory, serially
    pcie = None
    if rank == 0 and not args.no_pcie:
        m = min(n, 64)
        nb_in = int(offs[m - 1] + sizes[m - 1])
        h_in = torch.from_numpy(blob[:nb_in]).pin_memory()
        h_out = torch.empty(m * stride, dtype=torch.uint8).pin_memory()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        d_data[:nb_in].copy_(h_in, non_blocking=True)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        batch.decode_device(m, d_data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), d_out.data_ptr(), stride,
                            d_st.data_ptr(), d_dims.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        h_out.copy_(d_out[: m * stride], non_blocking=True)
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        pcie = {"value": round(m * W * H / 1e6 / (t3 - t0), 2), "unit": "megapixels/s", "images": m,
                "h2d_ms": round((t1 - t0) * 1e3, 3), "decode_ms": round((t2 - t1) * 1e3, 3),
                "d2h_ms": round((t3 - t2) * 1e3, 3),
                "note": "serial H2D (pinned) -> decode -> D2H (pinned) of a sub-batch; not overlapped"}
        del h_in, h_out

    comp_bytes = float(sizes.sum())
    alg_bytes = comp_bytes + n * W * H * 3.0  # compressed + W*H*3 per image
    mpx = n * W * H / 1e6
    ms_step = elapsed / args.steps * 1e3
    value = world * mpx / (elapsed / args.steps)
    # dominant kernel: the stage with the largest event-timed share (stages are summed over the
    # workspace groups of one step; each single-kernel stage launches once per group)
    dom = max((k for k in stages if stages[k] > 0), key=lambda k: stages[k], default=None)
    roof = None
    if dom:
        launches = batch.groups_per_call(n)
        achieved = alg_bytes / (stages[dom] * 1e-3) / 1e9  # = per-launch alg bytes / avg launch time
        traffic = None
        tpath = os.path.join(ROOT, "profiles", "traffic.json")
        rst = wl.get("restart", 0)
        ibytes = 0
        if rst:  # average compressed bytes per restart interval (interval_bytes: the scan's share)
            mcus = -(-W // 16) * -(-H // 16) if wl["sampling"] == "420" else -(-W // 8) * -(-H // 8)
            ibytes = sum(len(p) for p in pool) / len(pool) / -(-mcus // rst)
        kname = stage_kernels(W, H, rst, ibytes).get(dom, dom)
        if os.path.exists(tpath):
            tj = json.load(open(tpath))
            # PMC runs may group images differently (the profiler holds HBM, so fewer images fit a
            # group): the per-image traffic is scaled to this run's images per launch
            if tj.get("workload") == args.workload and tj.get("kernel") == kname and tj.get("images_per_launch"):
                traffic = round(tj["bytes_per_launch"] / tj["images_per_launch"] * (-(-n // launches)))
        # the dominant kernel's own necessary bytes (what `traffic` is to be read against): the
        # entropy decode reads the unstuffed stream (<= the compressed bytes) and writes the
        # coefficient blocks (128 B each); the other stages' kernels move their own planes
        blocks = n * sum((-(-W // 8)) * (-(-H // 8)) // d for d in (1, 4, 4))  # 4:2:0: Y + two quarter planes
        own = {"write": comp_bytes + blocks * coef_cell_bytes(), "unstuff": 2 * comp_bytes}.get(dom)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "kernel": kname, "launches_per_step": launches,
                "alg_bytes_per_launch": round(alg_bytes / launches),
                "kernel_own_bytes_per_launch": round(own / launches) if own else None,
                "avg_launch_ms": round(stages[dom] / launches, 3),
                "stage_ms": {k: round(v, 3) for k, v in stages.items()},
                "pipeline_frac": round(alg_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
        if kname == "k_gw_lane":
            roof["kernel_note"] = ("the write stage's events bracket both k_gw_lane instances on the stream: "
                                   "<512,false> and the CHK instance <512,true> (128 workgroups; streams ending in "
                                   "a syntax error); their rocprofv3 averages add up to avg_launch_ms")
        roof.update(pipeline_traffic(args.workload, n, alg_bytes))
    out = {
        "metric": f"megapixels/s JPEG decode, {W}x{H} RGB batch",
        "value": round(value, 2), "unit": "megapixels/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (tools/synth.c, seeded)",
        "config": {"workload": wl["desc"], "images_per_gpu": n, "pool": len(pool), "width": W, "height": H,
                   "bytes_per_pixel_compressed": round(comp_bytes / (n * W * H), 4),
                   "parallelism": f"dp{world} (images sharded; one RCCL all-gather of per-image records after the "
                                          f"timed steps)"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "parity": {"all_status_ok": ok_all, "images_checked_vs_oracle": checked, "mismatches": mismatches},
        "entropy_paths": paths,
        "inflight": {"steps_in_flight": M, "group": group or "auto", "groups_per_call": batch.groups_per_call(n)},
        "hip_graph": bool(args.graph),
        "records": records,
        "pcie_inclusive": pcie,
        "gen_seconds": round(gen_s, 1),
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
