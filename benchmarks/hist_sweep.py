"""Histogram kernel grid sweep (csrc/kernels/trees.hip hm_hist_build): HIGGS-shaped root level
(11M rows, one segment) and a deep level (256 segments) per blocks-per-group setting.

    python benchmarks/hist_sweep.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd import _native  # noqa: E402
import hivemall_amd.models.trees  # noqa: E402,F401  (registers the signatures)


def run(n=11_000_000, d=28, NS=3, B=256):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    dpad = (d + 15) // 16 * 16
    bins = torch.randint(0, B, (n, dpad), generator=g, device=dev, dtype=torch.uint8)
    stats = torch.randn(n, NS, generator=g, device=dev)
    smax = stats.abs().amax(0).contiguous()
    rows_all = torch.arange(n, dtype=torch.int32, device=dev)
    cases = {"root": (rows_all, torch.tensor([0, n], device=dev), 1)}
    S = 256
    node = torch.randint(0, S, (n // 2,), generator=g, device=dev)
    order = torch.argsort(node)
    rows = torch.randperm(n, generator=g, device=dev)[: n // 2][order].to(torch.int32).contiguous()
    seg = torch.zeros(S + 1, dtype=torch.int64, device=dev)
    seg[1:] = torch.cumsum(torch.bincount(node, minlength=S), 0)
    cases["deep256"] = (rows, seg, S)
    p = _native.ptr
    for name, (r, sg, ns) in cases.items():
        for FG in (16, 8):
            for nblk in (128, 256, 512, 768, 1024, 2048, 4096):
                out = torch.zeros(ns, d, B, NS, device=dev)
                args = (p(bins), d, dpad, B, p(r), p(sg), ns, p(stats), p(smax), NS, FG, p(out), nblk,
                        _native.stream_of(dev))
                for _ in range(2):
                    _native.check(_native.hip().hm_hist_build(*args), "hist")
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    _native.hip().hm_hist_build(*args)
                b.record()
                b.synchronize()
                ms = a.elapsed_time(b) / 10
                rows_n = int(sg[-1] - sg[0])
                print(json.dumps({"case": name, "FG": FG, "nblk": nblk, "ms": round(ms, 4),
                                  "Grow_feat_per_s": round(rows_n * d / ms / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    run()
