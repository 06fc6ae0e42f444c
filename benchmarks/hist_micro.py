"""Histogram kernel in isolation (csrc/kernels/trees.hip hm_hist_build) on HIGGS-sized rows:
11 M x 28 features, 256 bins, at the root (one segment, every row) and at a depth-7 level (128
segments over a random half of the rows), for NS = 2 / 3 statistics and 16- / 32-feature
groups.  HM_HIST_PACK=1 selects the 64-bit packed LDS accumulation (read once per process).

    python benchmarks/hist_micro.py [n_rows]
"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from hivemall_amd import _native
    from hivemall_amd.models import trees  # noqa: F401  (registers hm_hist_build)

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 11_000_000
    d, B, dpad = 28, 256, 32
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    bins = torch.randint(0, B, (n, dpad), dtype=torch.uint8, device=dev, generator=g)
    p = _native.ptr
    lib = _native.hip()
    st = _native.stream_of(dev)
    out = []
    for level in ("root", "depth7"):
        if level == "root":
            rows = torch.arange(n, dtype=torch.int32, device=dev)
            seg = torch.tensor([0, n], dtype=torch.int64, device=dev)
        else:
            m = n // 2
            rows = torch.randperm(n, device=dev, generator=g)[:m].sort().values.to(torch.int32)
            cuts = torch.linspace(0, m, 129, device=dev).to(torch.int64)
            seg = cuts
            # rows of one node are spread over the table: shuffle the node assignment
            rows = rows[torch.randperm(m, device=dev, generator=g)].contiguous()
        n_seg = seg.numel() - 1
        for NS in (2, 3):
            stats = torch.randn((n, NS), device=dev, generator=g)
            stats[:, -1] = 1.0
            smax = stats.abs().amax(0).contiguous()
            for FG in (16, 32):
                if FG * B * NS * 4 > 160 * 1024 or (FG == 16 and 16 * B * NS * 4 > 64 * 1024):
                    continue
                nblk = 256
                hist = torch.zeros((n_seg, d, B, NS), device=dev)
                args = (p(bins), d, dpad, B, p(rows), p(seg), n_seg, p(stats), p(smax), NS, FG, p(hist), nblk, st)
                _native.check(lib.hm_hist_build(*args), "hm_hist_build")
                torch.cuda.synchronize()
                # exactness against a float64 reference of one feature
                f = 5
                r = rows.long()
                k = torch.searchsorted(seg[1:], torch.arange(rows.numel(), device=dev), right=True)
                ref = torch.zeros((n_seg, B, NS), dtype=torch.float64, device=dev)
                ref.index_put_((k, bins[r, f].long()), stats[r].double(), accumulate=True)
                err = (hist[:, f].double() - ref).abs().max().item() / max(1e-30, ref.abs().max().item())
                reps = 10
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    hist.zero_()
                    _native.check(lib.hm_hist_build(*args), "hm_hist_build")
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                m_rows = rows.numel()
                res = {"level": level, "rows": m_rows, "segments": n_seg, "NS": NS, "FG": FG,
                       "pack": os.environ.get("HM_HIST_PACK", "0"), "us": round(ms * 1e3, 1),
                       "g_rows_per_s": round(m_rows / ms / 1e6, 2),
                       "lds_atomics_per_s_T": round(m_rows * d * NS / ms / 1e9, 2),
                       "rel_err_f5": float(f"{err:.2e}")}
                print(json.dumps(res), flush=True)
                out.append(res)


if __name__ == "__main__":
    main()
