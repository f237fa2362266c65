"""Radiance .hdr oracle (oracle/hdr_oracle.c): Image::readHdr (codecs.cpp:706-777) restated.

codecs.cpp does not compile here (MSVC-only constructs, absent codec libraries), so the
restatement is pinned by (1) the reference's own fixture data/test.hdr (tests/golden/test.hdr, a
flat RGBE file written by GEGL), whose floats must equal an independent numpy statement of
workOnRGBE/convertComponent (codecs.cpp:617-628, 610-615), and (2) round trips of seeded
synthetic files in all three pixel-data layouts decrunchHDR/oldDecrunchHDR accept
(codecs.cpp:630-703). Beyond that, the outcome codes for malformed files are this build's reading
of the reference's undefined behaviour (DESIGN.md "HDR").
"""
import hashlib
import os

import numpy as np
import pytest

import hdrutil as H
from oracle import pyoracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _test_hdr():
    return open(os.path.join(GOLDEN, "test.hdr"), "rb").read()


def test_oracle_hdr_reference_fixture():
    data = _test_hdr()
    code, w, h, rows, arr = O.hdr_decode(data)
    assert (code, w, h, rows) == (O.HDR_OK, 499, 289, 289)
    ds = data.index(b"-Y 289 +X 499\n") + len(b"-Y 289 +X 499\n")
    assert len(data) - ds == 499 * 289 * 4  # flat RGBE, as GEGL writes it
    rgbe = np.frombuffer(data[ds:], np.uint8).reshape(289, 499, 4)
    exp = H.expected_floats(rgbe)
    np.testing.assert_array_equal(arr.view(np.uint32), exp.view(np.uint32))
    # convertComponent as the reference writes it: (v / 256.0f) * (float)pow(2, E - 128)
    v = rgbe[..., :3].astype(np.float32) / np.float32(256.0)
    d = np.power(2.0, rgbe[..., 3:4].astype(np.float64) - 128).astype(np.float32)
    np.testing.assert_array_equal(arr[..., :3].view(np.uint32), (v * d).view(np.uint32))


@pytest.mark.parametrize("case", H.valid_cases(), ids=lambda c: c[0])
def test_oracle_hdr_round_trip(case):
    name, data, px = case
    code, w, h, rows, arr = O.hdr_decode(data)
    assert (code, w, h, rows) == (O.HDR_OK, px.shape[1], px.shape[0], px.shape[0])
    np.testing.assert_array_equal(arr.view(np.uint32), H.expected_floats(px).view(np.uint32))


EXPECTED_CODES = {
    "empty": O.HDR_NOT_RADIANCE, "not_radiance": O.HDR_NOT_RADIANCE, "short_magic": O.HDR_NOT_RADIANCE,
    "no_blank_line": O.HDR_BAD_HEADER, "no_reso_newline": O.HDR_BAD_HEADER, "reso_x_first": O.HDR_BAD_HEADER,
    "reso_only_y": O.HDR_BAD_HEADER, "reso_zero": O.HDR_BAD_HEADER, "reso_negative": O.HDR_BAD_HEADER,
    "reso_huge": O.HDR_BAD_HEADER, "reso_spaces": O.HDR_OK, "header_only": O.HDR_TRUNCATED,
    "rle_run_overflow": O.HDR_MALFORMED, "rle_literal_overflow": O.HDR_MALFORMED,
    "old_run_first_px": O.HDR_MALFORMED, "old_run_zero_first_px": O.HDR_OK, "old_rshift_24_zero": O.HDR_OK,
    "old_rshift_32": O.HDR_MALFORMED, "old_run_past_end": O.HDR_MALFORMED, "rle_width_mismatch": O.HDR_OK,
    "narrow_2_2": O.HDR_OK, "rle_trailing": O.HDR_OK, "flat_trailing": O.HDR_OK,
    "trunc_flat_minus1": O.HDR_TRUNCATED, "trunc_rle_minus1": O.HDR_TRUNCATED,
    "trunc_in_row_header": O.HDR_TRUNCATED,
}


def test_oracle_hdr_edge_codes():
    seen = set()
    for name, data in H.edge_cases():
        code, w, h, rows, arr = O.hdr_decode(data)
        if name in EXPECTED_CODES:
            assert code == EXPECTED_CODES[name], name
            seen.add(name)
        if name.startswith("trunc_"):
            assert code == O.HDR_TRUNCATED and rows < h, name
        if code in (O.HDR_OK, O.HDR_TRUNCATED, O.HDR_MALFORMED):
            assert arr is not None and arr.shape == (h, w, 4)
            assert not arr[rows:].any(), name  # rows the reference leaves uninitialised are zero
    assert seen == set(EXPECTED_CODES)


def test_oracle_hdr_truncated_rows_are_prefix():
    """A truncated file decodes to a prefix of the full file's rows."""
    px = np.ascontiguousarray(H.S.rgbe(9, 40, 6))
    full = H.expected_floats(px)
    for name, data in H.edge_cases():
        if name.startswith("trunc_") and name != "trunc_in_row_header":
            code, w, h, rows, arr = O.hdr_decode(data)
            np.testing.assert_array_equal(arr[:rows], full[:rows])


def test_oracle_hdr_manifest():
    """The reference fixture's decoded floats, frozen (tests/golden/hdr_manifest.json)."""
    import json
    man = json.load(open(os.path.join(GOLDEN, "hdr_manifest.json")))
    code, w, h, rows, arr = O.hdr_decode(_test_hdr())
    assert hashlib.sha256(arr.tobytes()).hexdigest() == man["test.hdr"]["float_sha256"]
    assert hashlib.sha256(_test_hdr()).hexdigest() == man["test.hdr"]["file_sha256"]
