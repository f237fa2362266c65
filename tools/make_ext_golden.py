"""Regression pins for the C4 encode extension (oracle/tje_oracle.c or_jpeg_encode).

The extension has no upstream counterpart (tiny_jpeg stops at quality 3, 4:4:4), so its bytes
are defined by the oracle restatement; this manifest freezes them so a change to the oracle
or the GPU encoder shows up as a diff. Inputs are tools/synth.c images (seeded).
Run: python tools/make_ext_golden.py  -> tests/golden/ext_manifest.json
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as O  # noqa: E402
from tools import synthpy as S  # noqa: E402

CASES = [  # (seed, w, h, comps, quality, subsampling)
    (1, 1, 1, 3, 90, 420), (2, 7, 5, 3, 50, 420), (3, 17, 33, 4, 90, 420), (4, 64, 48, 3, 100, 444),
    (5, 33, 17, 3, 1, 444), (6, 130, 97, 3, 10, 420), (7, 256, 256, 3, 75, 420), (8, 31, 64, 4, 95, 444),
]


def main():
    out = {}
    for seed, w, h, c, q, sub in CASES:
        px = S.rgb(seed, w, h, c).tobytes()
        jpg = O.jpeg_encode(q, sub, w, h, c, px)
        out[f"{seed}:{w}x{h}x{c}:q{q}:{sub}"] = {
            "seed": seed, "w": w, "h": h, "comps": c, "quality": q, "subsampling": sub,
            "len": len(jpg), "sha256": hashlib.sha256(jpg).hexdigest()}
    path = os.path.join(ROOT, "tests", "golden", "ext_manifest.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(path, len(out))


if __name__ == "__main__":
    main()
