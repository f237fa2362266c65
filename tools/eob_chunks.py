"""How many 16-byte zig-zag chunks of a coefficient block lie at or before its last nonzero
coefficient, on the bench's C3 images (tools/synthpy.rgb, 4:2:0, q90): what EOB-truncated block
stores could save. The blocks are recomputed here from the pixels with the IJG q90 tables and an
orthonormal float DCT (the encoder's quantised values up to rounding), on a 1024^2 crop.

    python tools/eob_chunks.py [seed] [size]
"""
import json
import sys

import numpy as np
from scipy.fft import dctn

from tools import synthpy

_LQ = [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
       14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
       49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99]
_CQ = [17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99,
       47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32
_ZZ = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
       21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60,
       61, 54, 47, 55, 62, 63]


def _q(tab, quality=90):
    s = 200 - 2 * quality
    return np.clip((np.array(tab) * s + 50) // 100, 1, 255).reshape(8, 8)


def chunks(plane, q):
    """Per block: chunks 1..8 up to the last nonzero zig-zag coefficient (1 for a DC-only block)."""
    h, w = plane.shape
    b = plane.reshape(h // 8, 8, w // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 8, 8)
    c = np.round(dctn(b, axes=(1, 2), norm="ortho") / q).reshape(-1, 64)[:, _ZZ]
    nz = c != 0
    last = np.where(nz.any(1), 63 - np.argmax(nz[:, ::-1], 1), 0)
    return last // 8 + 1


def main(seed=1234, size=1024):
    px = synthpy.rgb(seed, size, size, 3).astype(np.float64)
    r, g, b = px[..., 0], px[..., 1], px[..., 2]
    y = 0.299 * r + 0.587 * g + 0.114 * b - 128
    cb = (-0.168736 * r - 0.331264 * g + 0.5 * b).reshape(size // 2, 2, size // 2, 2).mean((1, 3))
    cr = (0.5 * r - 0.418688 * g - 0.081312 * b).reshape(size // 2, 2, size // 2, 2).mean((1, 3))
    ly, lc = chunks(y, _q(_LQ)), np.concatenate([chunks(cb, _q(_CQ)), chunks(cr, _q(_CQ))])
    every = np.concatenate([ly, lc])
    out = {
        "images": f"synthpy.rgb({seed}, {size}, {size}), 4:2:0 q90 (the C3 generator)",
        "mean_chunks_of_8": {"luma": round(float(ly.mean()), 3), "chroma": round(float(lc.mean()), 3),
                             "all": round(float(every.mean()), 3)},
        "histogram_all": [round(float(x), 4) for x in np.bincount(every, minlength=9)[1:] / len(every)],
        "coefficient_bytes_saved": round(1 - float(every.mean()) / 8, 3),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
