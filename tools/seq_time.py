"""Sequential-fallback cost on the GPU: one image per size that only k_entropy_seq takes (Y 4x4
sampling: 18 blocks per MCU), decode time against a clean 4:2:0 image of the same size, plus
bit-exactness against the oracle. Usage: python3 tools/seq_time.py [sizes...]"""
import hashlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import imagecodecs_amd as icx
from oracle import pyoracle as O
from tools import synthpy as S

ctx = icx.Context(0)
for n in [int(a) for a in sys.argv[1:]] or [512, 1024, 2048]:
    for samp in ("y44", "420"):
        data = S.synth_jpeg(77, n, n, samp, 90)
        b = icx.Batch(ctx, 1, n, n)
        b.decode_host([data])
        t0 = time.perf_counter()
        code, w, h, c, pix = b.decode_host([data])[0]
        dt = time.perf_counter() - t0
        st = b.path_stats()
        ok = pix.tobytes() == O.decode(data)[4]
        print(f"{samp} {n}x{n}: {dt*1e3:9.2f} ms  {n*n/dt/1e6:8.2f} MP/s  {len(data)/dt/1e6:7.2f} MB/s of scan  bit-exact {ok}  {st}", flush=True)
        b.close()
