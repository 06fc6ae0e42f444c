"""Run benchmarks/probes/lds_dma12_probe.hip: prints where 12-B LDS-DMA lanes land."""
import ctypes as C
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC, LIB = os.path.join(HERE, "probes", "lds_dma12_probe.hip"), os.path.join(HERE, "probes", "liblds_dma12_probe.so")

if sys.argv[1:] == ["build"]:
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", SRC, "-o", LIB])
    sys.exit(0)
import torch  # noqa: E402
lib = C.CDLL(LIB)
lib.hm_probe_lds_dma12.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
src = torch.arange(1024, dtype=torch.int32, device="cuda")          # dword k holds k
out = torch.zeros(512, dtype=torch.int32, device="cuda")
assert lib.hm_probe_lds_dma12(src.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
o = out.cpu().tolist()
fmt = lambda v: "----" if v == -559038737 else str(v)
print("dwordx3 from src+12l, LDS dwords 0..63:", [fmt(v) for v in o[:64]])
print("dwordx3 LDS dwords 192..255:", [fmt(v) for v in o[192:256]])
ok12 = all(o[3 * l + k] == 3 * l + k for l in range(64) for k in range(3))
print("dwordx3 packed at 12 B per lane:", ok12)
print("dwordx4 from src+12l (4-B aligned), LDS dwords 0..31:", [fmt(v) for v in o[256:288]])
ok16 = all(o[256 + 4 * l + k] == 3 * l + k for l in range(64) for k in range(4))
print("dwordx4 unaligned source at 16 B per lane correct:", ok16)
