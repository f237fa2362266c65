"""ASan + UBSan over the CPU code the parity claims rest on: the
oracle restatements (oracle/*.c) and the parallel entropy decoder's lane code run by the
emulator (icx_spec_core.h through tests/emu/spec_emu.cpp), built by tests/san/Makefile and run
over every committed JPEG / HDR fixture. A sanitizer report aborts the driver (non-zero exit)."""
import glob
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

SAN = os.path.join(ROOT, "tests", "san")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", SAN], check=True)
    return SAN


def _files(with_hdr):
    fs = sorted(glob.glob(os.path.join(GOLDEN, "**", "*.jpg"), recursive=True))
    if with_hdr:
        fs.append(os.path.join(GOLDEN, "test.hdr"))
    return fs


def _run(exe, files):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, *files], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, \
        r.stderr[-3000:]
    assert f"sanitized {len(files)} files" in r.stdout


def test_oracle_under_asan_ubsan(built):
    _run(os.path.join(built, "oracle_san"), _files(True))


def test_lane_emulator_under_asan_ubsan(built):
    _run(os.path.join(built, "emu_san"), _files(False))
