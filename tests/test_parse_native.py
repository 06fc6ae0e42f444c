"""The device feature-string parsers (csrc/kernels/parse.h) compiled for the host and fuzzed
against strtod/strtoll: whatever the gfx950 ingest kernels accept must equal the host parser."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_device_parsers_fuzz_against_strtod(tmp_path):
    exe = tmp_path / "parse_fuzz"
    subprocess.check_call(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", "parse_fuzz.cpp"), "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
