"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the native CPU engines
(SURVEY.md §5.2).  GPU ASan / XNACK runs are not available on the MI355X pool, so the
sanitizers cover the host code: every C++ engine (hashing, feature parsing, linear, FM, FFM,
MF/BPR, trees) is rebuilt with -fsanitize=address,undefined (``_build.build_host_sanitized``)
and the CPU test files that drive those engines are re-run against it in a subprocess with the
ASan runtime preloaded.  Any heap/stack overflow, use-after-free or UB aborts the subprocess.
"""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
ENGINE_TESTS = ["test_ffm.py", "test_fm.py", "test_linear.py", "test_mf.py", "test_trees.py",
                "test_xgboost.py", "test_functions.py", "test_topic_recommend.py"]


def _runtime(name):
    cxx = shutil.which("g++") or shutil.which("gcc")
    if not cxx:
        return None
    p = subprocess.run([cxx, f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if p and os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.timeout(1200)
def test_host_engines_clean_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not available")
    sys.path.insert(0, str(ROOT))
    from hivemall_amd import _build

    lib = _build.build_host_sanitized()
    env = dict(os.environ)
    env.update(LD_PRELOAD=f"{asan}:{ubsan}", HM_HOST_LIB=str(lib), HM_NO_AUTOBUILD="1",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider"]
    cmd += [str(ROOT / "tests" / t) for t in ENGINE_TESTS]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1100)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
