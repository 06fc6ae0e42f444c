"""In-tree build of the native libraries.

Two shared objects are produced under ``hivemall_amd/_lib``:

* ``libhm_hip.so``  — every ``csrc/kernels/*.hip`` compiled by ``hipcc --offload-arch=gfx950``
  (CDNA4 only; no other targets, no CUDA).  C ABI, launched from Python through ctypes on
  the current torch HIP stream.
* ``libhm_host.so`` — ``csrc/host/*.cpp`` (the CPU data plane + CPU learner engine),
  compiled with g++ -O3 -fopenmp.  Loadable everywhere, needs no GPU.

The build is incremental (per-object mtime check against sources + headers) and runs the
per-file compiles in parallel.  ``python -m hivemall_amd._build`` builds everything.
"""
from __future__ import annotations

import concurrent.futures as _cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "_lib"
OBJDIR = ROOT / "build" / "obj"

HIP_ARCH = os.environ.get("HM_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", shutil.which("g++") or "c++")

HIP_FLAGS = [
    f"--offload-arch={HIP_ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
    "-munsafe-fp-atomics", "-Wno-unused-result",
]
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-fopenmp", "-march=x86-64-v2", "-Wall",
              "-Wno-unused-function"]

HIP_LIB = Path(os.environ["HM_HIP_LIB"]) if os.environ.get("HM_HIP_LIB") else LIBDIR / "libhm_hip.so"
HOST_LIB = Path(os.environ["HM_HOST_LIB"]) if os.environ.get("HM_HOST_LIB") else LIBDIR / "libhm_host.so"
# host library built with AddressSanitizer + UBSan (sanitizer runs on host code only; the GPU
# pool has no GPU ASan / XNACK): build_host_sanitized(), used by tests/test_sanitizers.py
ASAN_HOST_LIB = ROOT / "build" / "asan" / "libhm_host_asan.so"
SAN_FLAGS = ["-O1", "-g", "-std=c++17", "-fPIC", "-fopenmp", "-fno-omit-frame-pointer",
             "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-Wall",
             "-Wno-unused-function"]


def _headers(d: Path):
    return [p for p in d.glob("*.h")] + [p for p in d.glob("*.hpp")]


def _newest(paths):
    return max((p.stat().st_mtime for p in paths), default=0.0)


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    return target.stat().st_mtime < _newest(deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), file=sys.stderr)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def source_hash(srcs, hdrs, flags) -> str:
    """sha256 over the sources and headers a library is built from (path relative to csrc,
    contents) and the compile flags: the library's provenance."""
    h = hashlib.sha256()
    for f in sorted(set(srcs) | set(hdrs)):
        h.update(str(Path(f).relative_to(CSRC)).encode())
        h.update(b"\0")
        h.update(Path(f).read_bytes())
        h.update(b"\0")
    h.update(" ".join(map(str, flags)).encode())
    return h.hexdigest()[:32]


def _deps(srcs):
    hdrs = _headers(CSRC / "kernels")  # shared rule headers are used by host code too
    for s in srcs:
        hdrs.extend(_headers(s.parent))
    return sorted(set(hdrs))


def lib_hash_file(lib: Path) -> Path:
    return lib.with_name(lib.name + ".srchash")


def expected_hash(kind: str) -> str:
    """Source hash the in-tree ``kind`` ("hip" / "host") library must carry."""
    if kind == "hip":
        srcs = sorted((CSRC / "kernels").glob("*.hip"))
        return source_hash(srcs, _deps(srcs), HIP_FLAGS)
    srcs = sorted((CSRC / "host").glob("*.cpp"))
    return source_hash(srcs, _deps(srcs), HOST_FLAGS)


def _build_lib(srcs, compiler, flags, lib: Path, link_flags, verbose, jobs, objdir: Path = OBJDIR):
    objdir.mkdir(parents=True, exist_ok=True)
    lib.parent.mkdir(parents=True, exist_ok=True)
    hdrs = _deps(srcs)
    want = source_hash(srcs, hdrs, flags)
    hf = lib_hash_file(lib)
    if lib.exists() and hf.exists() and hf.read_text().strip() == want:
        # the library was built from exactly these sources and flags (content hash, embedded in
        # the library as hm_build_id() and checked at load by _native): nothing to do, whether
        # or not the object files are around (a GPU box gets the tree without build/, and
        # recompiling the kernels there cost the first launch ~12 s: BENCH_r03.json)
        return lib
    objs = []
    todo = []
    # the provenance object: hm_build_id() returns the source hash of this build
    gen = objdir / f"build_id_{lib.stem}{srcs[0].suffix if srcs else '.cpp'}"
    gen_txt = ('extern "C" __attribute__((visibility("default"))) const char* hm_build_id() '
               f'{{ return "{want}"; }}\n')
    if not gen.exists() or gen.read_text() != gen_txt:
        gen.write_text(gen_txt)
    go = gen.with_suffix(gen.suffix + ".o")
    objs.append(go)
    if _stale(go, [gen]):
        todo.append((gen, go))
    for s in srcs:
        o = objdir / (s.parent.name + "_" + s.name + ".o")
        objs.append(o)
        if _stale(o, [s] + hdrs):
            todo.append((s, o))
    if todo:
        with _cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_run, [compiler, *flags, "-c", s, "-o", o], verbose) for s, o in todo]
            for f in futs:
                f.result()
    if todo or _stale(lib, objs) or not hf.exists() or hf.read_text().strip() != want:
        tmp = lib.with_suffix(".so.tmp")
        _run([compiler, "-shared", "-o", tmp, *objs, *link_flags], verbose)
        os.replace(tmp, lib)
        hf.write_text(want + "\n")
    return lib


def build_host(verbose: bool = False, jobs: int = 8) -> Path:
    srcs = sorted((CSRC / "host").glob("*.cpp"))
    return _build_lib(srcs, CXX, HOST_FLAGS, HOST_LIB, ["-fopenmp"], verbose, jobs)


def build_host_sanitized(verbose: bool = False, jobs: int = 8) -> Path:
    """CPU library with ASan + UBSan (load it with libasan preloaded: tests/test_sanitizers.py)."""
    srcs = sorted((CSRC / "host").glob("*.cpp"))
    return _build_lib(srcs, CXX, SAN_FLAGS, ASAN_HOST_LIB, ["-fopenmp", "-fsanitize=address,undefined"],
                      verbose, jobs, objdir=ROOT / "build" / "asan" / "obj")


def build_hip(verbose: bool = False, jobs: int = 8) -> Path:
    srcs = sorted((CSRC / "kernels").glob("*.hip"))
    return _build_lib(srcs, HIPCC, HIP_FLAGS, HIP_LIB, [f"--offload-arch={HIP_ARCH}"], verbose, jobs)


def build_all(verbose: bool = False, jobs: int | None = None) -> None:
    jobs = jobs or min(8, os.cpu_count() or 4)
    build_host(verbose, jobs)
    build_hip(verbose, jobs)


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv)
    print("built:", HOST_LIB, HIP_LIB)
