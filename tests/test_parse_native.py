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


def test_host_parse_features_fast_path_matches_python_float():
    """hm_parse_features' exact decimal fast path (<= 15 significant digits, one IEEE division)
    and its strtod fallback give float32(float(text)) for every value string, in parallel."""
    import numpy as np

    from hivemall_amd.utils.features import FeatureEncoder

    rng = np.random.default_rng(5)
    vals = []
    for _ in range(200_000):
        k = rng.integers(0, 6)
        if k == 0:
            vals.append(str(rng.integers(-10**6, 10**6)))
        elif k == 1:
            vals.append(f"{rng.standard_normal() * 10.0 ** rng.integers(-6, 7):.{rng.integers(0, 12)}f}")
        elif k == 2:
            vals.append(repr(float(rng.standard_normal())))          # 17 digits -> strtod
        elif k == 3:
            vals.append(f"{rng.random():.3e}")                        # exponent -> strtod
        elif k == 4:
            vals.append("-0" if rng.random() < 0.5 else "+1.5")
        else:
            vals.append("0." + "".join(map(str, rng.integers(0, 10, rng.integers(1, 16)))))
    rows = [[f"{i % 97 + 1}:{v}" for i, v in enumerate(vals[j:j + 40])] for j in range(0, len(vals), 40)]
    csr = FeatureEncoder("int").encode(rows)
    want = np.array([np.float32(float(v)) for v in vals], dtype=np.float32)
    got = np.asarray(csr.val, dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
