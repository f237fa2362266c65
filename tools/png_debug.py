"""Locate where a GPU-encoded PNG's IDAT stops inflating to the oracle's filtered stream
(debug aid for the segment-parallel deflate; prints the first mismatching stream offset)."""
import os, sys, zlib
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np
import imagecodecs_amd as icx
import pngutil as P
from oracle import pyoracle as O

w = h = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ctx = icx.Context()
px = P.synth_rgba(8192, w, h)
png = ctx.png_encode(w, h, 4, px.tobytes())
I = P.info(png)
m = O.png_choose(px.tobytes(), w, h, 4)
ref = O.png_filtered(px.tobytes(), w, h, 4, m)
d = zlib.decompressobj(-15)
try:
    out = d.decompress(I["idat"][2:-4])
    err = None
except zlib.error as e:
    out, err = b"", str(e)
tail = d.unused_data
print("N", len(ref), "inflated", len(out), "err", err, "unused", len(tail), "eof", d.eof)
a = np.frombuffer(ref, np.uint8); b = np.frombuffer(out, np.uint8)
n = min(len(a), len(b))
bad = np.nonzero(a[:n] != b[:n])[0]
print("mismatches", len(bad), "first", bad[:10].tolist(), "seg", (bad[:10] // 4096).tolist(), "off", (bad[:10] % 4096).tolist())
adl = zlib.adler32(out) ; print("adler ours", hex(adl), "trailer", I["idat"][-4:].hex(), "ref", hex(zlib.adler32(ref)))
