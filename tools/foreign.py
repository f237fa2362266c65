"""Foreign-encoder JPEG inputs for parity tests (test tooling, not product, not oracle).

tools/synth.c writes Annex K Huffman tables and IJG-scaled Annex K quant tables only. Real files
come from other encoders: libjpeg-turbo with optimised (per-image) Huffman tables, its own quant
scaling, restart markers, or RGB colour space. PIL (libjpeg-turbo 3.x in this image) writes those
here; the expected pixels never come from PIL (its decoder is not NanoJPEG)
but from the reference decoder compiled in place (oracle/_ref), recorded by
tools/make_foreign_goldens.py.

Large inputs are regenerated on the fly (a committed 4096^2 JPEG would be megabytes): `photo()`
is a deterministic numpy image with the bit-density contrasts of a photograph (flat regions next
to hard edges and fine texture), and `pil_jpeg()` encodes it; the manifest pins the JPEG bytes by
sha256, so a different PIL build fails the test instead of silently testing other bytes.
"""
from __future__ import annotations

import io

import numpy as np

from tools import synthpy as S


def photo(seed: int, w: int, h: int) -> np.ndarray:
    """(h, w, 3) uint8: the smooth-plus-noise synth image with a flat band (very few bits per
    block), a high-noise band (many), hard-edged rectangles and discs, and thin stripes."""
    rng = np.random.default_rng(seed)
    img = S.rgb(seed, w, h, 3).astype(np.int32)
    yy, xx = np.mgrid[0:h, 0:w]
    # flat "sky": the top fifth, a slow gradient with no noise
    sky = h // 5
    grad = (np.linspace(180, 120, max(sky, 1))[:, None] * np.ones((1, w))).astype(np.int32)
    img[:sky, :, 0] = grad[:sky]
    img[:sky, :, 1] = grad[:sky] + 20
    img[:sky, :, 2] = 235
    # high-noise band: heavy uniform noise
    b0, b1 = (3 * h) // 5, (3 * h) // 5 + max(1, h // 10)
    img[b0:b1] = rng.integers(0, 256, (b1 - b0, w, 3))
    # hard-edged flat shapes
    for _ in range(24):
        x0, y0 = int(rng.integers(0, w)), int(rng.integers(sky, h))
        rw, rh = int(rng.integers(w // 64 + 1, w // 6 + 2)), int(rng.integers(h // 64 + 1, h // 6 + 2))
        col = rng.integers(0, 256, 3)
        if rng.random() < 0.5:
            img[y0:y0 + rh, x0:x0 + rw] = col
        else:
            r = max(rw, rh) // 2
            m = (xx - x0) ** 2 + (yy - y0) ** 2 < r * r
            img[m] = col
    # thin stripes (text-like high frequencies) in the lower right quarter
    m = (xx > w // 2) & (yy > (3 * h) // 4) & (((xx // 2) + (yy // 3)) % 3 == 0)
    img[m] = 20
    return np.clip(img, 0, 255).astype(np.uint8)


def pil_jpeg(px: np.ndarray, **kw) -> bytes:
    """PIL/libjpeg-turbo baseline (or progressive) JPEG of an RGB (h, w, 3) or gray (h, w) array."""
    from PIL import Image
    im = Image.fromarray(px, "L" if px.ndim == 2 else "RGB")
    b = io.BytesIO()
    im.save(b, "JPEG", **kw)
    return b.getvalue()


# Regenerated large cases: name -> (generator args, PIL save args). The manifest
# (tests/golden/foreign_large.json) holds each one's JPEG sha256 and NanoJPEG pixel sha256.
LARGE = {
    "photo4096_q90_420_opt": ((7001, 4096, 4096), {"quality": 90, "subsampling": 2, "optimize": True}),
    "photo2048_q95_444_opt": ((7002, 2048, 2048), {"quality": 95, "subsampling": 0, "optimize": True}),
    "photo2048_q75_422_opt_rst": ((7003, 2048, 1536), {"quality": 75, "subsampling": 1, "optimize": True,
                                                       "restart_marker_rows": 1}),
    "photo1999_q100_420_opt": ((7004, 1999, 1001), {"quality": 100, "subsampling": 2, "optimize": True}),
    "photo1024_q50_420_std": ((7005, 1024, 1024), {"quality": 50, "subsampling": 2}),
    "photo4096_q100_444_opt": ((7006, 4096, 2048), {"quality": 100, "subsampling": 0, "optimize": True}),
}


def large(name: str) -> bytes:
    args, kw = LARGE[name]
    return pil_jpeg(photo(*args), **kw)
