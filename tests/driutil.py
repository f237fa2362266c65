"""Restart-interval (DRI) stream helpers for the tests: marker offsets, corrupt variants, and the
crafted stream whose interval ends at a stuffed FF D0+(j&7)."""
from tools import synthpy as S


def scan_start(data):
    sos = data.index(b"\xff\xda")
    return sos + 2 + ((data[sos + 2] << 8) | data[sos + 3])


def rst_markers(data):
    """File offsets of the restart markers in the scan (stream order)."""
    s = scan_start(data)
    return [k for k in range(s, len(data) - 1) if data[k] == 0xFF and 0xD0 <= data[k + 1] <= 0xD7]


def dri_corruptions(data, rng, n):
    """Corrupt variants of a DRI stream around its restart markers (what damaged camera files
    hold): renumbered, shifted, missing, duplicated or swapped markers, flipped data bytes,
    truncation."""
    d0 = bytes(data)
    mk = rst_markers(d0)
    s = scan_start(d0)
    out = []
    for t in range(n):
        k = mk[int(rng.integers(0, len(mk)))]
        kind = t % 8
        if kind == 0:  # wrong number
            v = bytearray(d0)
            v[k + 1] = 0xD0 + ((v[k + 1] - 0xD0 + 1 + int(rng.integers(0, 7))) & 7)
        elif kind == 1:  # a byte inserted before the marker
            v = d0[:k] + bytes([int(rng.integers(0, 255))]) + d0[k:]
        elif kind == 2:  # a byte lost before the marker
            v = d0[:k - 1] + d0[k:]
        elif kind == 3:  # marker missing
            v = d0[:k] + d0[k + 2:]
        elif kind == 4:  # marker doubled
            v = d0[:k] + d0[k:k + 2] + d0[k:]
        elif kind == 5:  # two markers swapped
            v = bytearray(d0)
            j = mk.index(k)
            if j + 1 < len(mk):
                k2 = mk[j + 1]
                v[k + 1], v[k2 + 1] = v[k2 + 1], v[k + 1]
        elif kind == 6:  # data bytes flipped
            v = bytearray(d0)
            for _ in range(1 + t % 3):
                v[int(rng.integers(s, len(v) - 2))] ^= int(rng.integers(1, 256))
        else:  # truncated (with and without EOI)
            cut = int(rng.integers(s + 1, len(d0) - 2))
            v = d0[:cut] + (b"\xff\xd9" if t % 2 else b"")
        out.append(bytes(v))
    return out


def elsewhere_case(seed=8300, w=512, h=512):
    """A DRI stream in which interval j's data is followed, after cutting out marker j and the
    start of interval j+1, by stuffed data FF 00 D0+(j&7): NanoJPEG reads that as marker j and
    goes on from there, where no lane starts (dri_end_kind: elsewhere)."""
    data = S.synth_jpeg(seed, w, h, "420", 95, 1)
    mk = rst_markers(data)
    for j in range(len(mk) - 1):
        k, k2 = mk[j], mk[j + 1]
        want = 0xD0 + (j & 7)
        q = data.find(bytes([0xFF, 0x00, want]), k + 2, k2)
        if q > 0:
            return data[:k] + data[q:], j
    raise AssertionError("no stuffed FF 00 Dn in the stream")
