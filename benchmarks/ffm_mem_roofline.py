"""Roofline of the FFM slot traffic on MI355X (benchmarks/probes/ffm_mem_probe.hip): the same
262,144 Criteo-shaped rows and 2^20 x 39 packed bf16 V|G table as bench.py, access pattern only.

    python benchmarks/ffm_mem_roofline.py build   # CPU side: hipcc -> benchmarks/probes/libffm_mem_probe.so
    python benchmarks/ffm_mem_roofline.py         # GPU box: rows/s per mode and grid
"""
import ctypes as C
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "probes", "ffm_mem_probe.hip")
LIB = os.path.join(HERE, "probes", "libffm_mem_probe.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-shared", SRC, "-o", LIB])
    print("built", LIB)


def run():
    import torch

    sys.path.insert(0, os.path.dirname(HERE))
    from hivemall_amd.io.synthetic import criteo_like

    lib = C.CDLL(LIB)
    lib.hm_probe_ffm_mem.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                     C.c_int, C.c_int, C.c_void_p]
    dev = torch.device("cuda")
    B, F, NF = 262144, 39, 1 << 20
    idx, _ = criteo_like(B * 8, 20, seed=1000, device=dev)
    VG = torch.zeros(NF * 896 // 2, dtype=torch.bfloat16, device=dev)   # large enough for every mode
    out = torch.zeros(B * 8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    modes = [int(m) for m in os.environ.get("MODES", "0,1,3,4,5,6,7").split(",")]
    if 7 in modes:
        from hivemall_amd.io.synthetic import criteo_ffm

        lib.hm_probe_ffm_mem_fv.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_int, C.c_void_p]
        fidx, ffld, fval, _ = criteo_ffm(B * 8, 20, seed=1000, device=dev)
    for mode in modes:
        for blocks in (4096, 8192):
            def launch(k):
                s = (k % 8) * B
                if mode == 7:
                    rc = lib.hm_probe_ffm_mem_fv(fidx[s:s + B].data_ptr(), ffld[s:s + B].data_ptr(),
                                                 fval[s:s + B].data_ptr(), B, F, VG.data_ptr(), out.data_ptr(),
                                                 blocks, st)
                else:
                    rc = lib.hm_probe_ffm_mem(idx[s:s + B].data_ptr(), B, F, F, VG.data_ptr(),
                                              out.data_ptr(), mode, blocks, st)
                assert rc == 0
            for k in range(3):
                launch(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 20
            for k in range(n):
                launch(k)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            print(json.dumps({"mode": mode, "blocks": blocks, "ms": round(dt * 1e3, 3),
                              "rows_per_s": round(B / dt / 1e6, 1),
                              "requested_TBps": round(B * 1482 * 16 * (1 if mode == 0 else 2) / dt / 1e12, 2)
                              if mode < 5 else round(B * 39 * (512 if mode == 6 else 896) * 2 / dt / 1e12, 2)}),
                  flush=True)


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else run()
