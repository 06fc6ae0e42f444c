"""Run the device decimal parser on a list of strings and compare with the host (strtod)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "probes", "libparse_probe.so")

if __name__ == "__main__" and "--build" in sys.argv:
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=fast", "-shared",
                           "-fPIC", os.path.join(HERE, "probes", "parse_probe.hip"), "-o", SO])
    sys.exit(0)

strs = ["1", "0.5", "2.5e+1", "1E3", "3.0e-2", "1e-2", "12345.678", ".5", "-7", "1e5", "2e1", "1.5e0"]
b = [s.encode() for s in strs]
off = np.zeros(len(b) + 1, np.int64)
off[1:] = np.cumsum([len(x) for x in b])
buf = torch.tensor(list(b"".join(b)), dtype=torch.uint8, device="cuda")
offt = torch.from_numpy(off).cuda()
val = torch.zeros(len(b), device="cuda")
ok = torch.zeros(len(b), dtype=torch.int32, device="cuda")
lib = ctypes.CDLL(SO)
rc = lib.parse_probe(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(offt.data_ptr()), len(b),
                     ctypes.c_void_p(val.data_ptr()), ctypes.c_void_p(ok.data_ptr()))
for s, o, v in zip(strs, ok.tolist(), val.tolist()):
    print(f"{s:>12} ok={o} dev={v!r} host={np.float32(float(s))!r}")
print("rc", rc)
