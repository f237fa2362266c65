"""CPU-side checks of the C ABI: libicx.so builds, loads, exports every symbol include/icx.h
declares, and its host-only logic (the NanoJPEG header walk behind icx_jpeg_probe) agrees with
the oracle. No compute call is made here -- those need a GPU (tests/test_gpu_*.py)."""
import json
import os
import re
import subprocess

import pytest

from conftest import GOLDEN, ROOT
import imagecodecs_amd as icx

HEADER = os.path.join(ROOT, "include", "icx.h")
MANIFEST = json.load(open(os.path.join(GOLDEN, "decode_manifest.json")))


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(icx_[a-z0-9_]+)\s*\(", src))
    return sorted(names - {"icx_write_func"})


def test_library_builds_and_loads():
    if not os.path.exists(icx.LIB_PATH):
        icx.build()
    L = icx.lib()
    assert L.icx_version().decode().startswith("icx ")


def test_exports_every_declared_symbol():
    icx.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", icx.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (icx_\w+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    assert len(declared()) >= 20


def test_python_binding_covers_header():
    assert set(declared()) <= set(icx._SIGS)


def test_library_is_gfx950_code_object():
    blob = open(icx.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # embedded HIP fat-binary target id


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_probe_header_walk_matches_reference(name):
    """icx_jpeg_probe runs the same __host__ __device__ parser k_parse runs on the GPU."""
    exp = MANIFEST[name]
    data = open(os.path.join(GOLDEN, name), "rb").read()
    code, w, h, n = icx.probe(data)
    if code != icx.OK:
        assert code == exp["code"], (code, exp)
    else:  # header OK: the final verdict belongs to the entropy decode
        assert exp["code"] in (icx.OK, icx.SYNTAX_ERROR)
        if exp["code"] == icx.OK:
            assert (w, h, n) == (exp["w"], exp["h"], exp["ncomp"])


def test_no_cpu_fallback_without_gpu():
    """The product fails loudly instead of decoding on the CPU when no GPU is visible."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(icx.ICXError):
        icx.Context(0)
