"""Top-k recommendation for every user (MovieLens-20M shape) — fused MFMA kernel vs
GEMM + torch.topk.

    python benchmarks/mips_bench.py [--users 138493] [--items 27278] [--dim 64] [--k 10]

Prints one JSON line per variant: ms per full sweep, effective TFLOP/s of the score GEMM,
and agreement of the fused result with the unfused one (fraction of identical top-k sets).
Synthetic random-init factors (bf16 operands, fp32 accumulation in both variants)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hivemall_amd.ops.topk_mips import mips_topk  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        out = fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=138493)
    ap.add_argument("--items", type=int, default=27278)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=32768, help="user rows per GEMM+topk chunk")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    U = (torch.randn(a.users, a.dim, device=dev, generator=g) * 0.3).bfloat16()
    V = (torch.randn(a.items, a.dim, device=dev, generator=g) * 0.3).bfloat16()
    bias = torch.randn(a.items, device=dev, generator=g) * 0.05
    flop = 2.0 * a.users * a.items * a.dim

    ms, (fi, fs) = timed(lambda: mips_topk(U, V, a.k, item_bias=bias), a.reps)
    print(json.dumps({"variant": "fused_mfma_topk", "ms": round(ms, 3), "tflops": round(flop / ms / 1e9, 1),
                      "users": a.users, "items": a.items, "dim": a.dim, "k": a.k}), flush=True)

    def unfused():
        outs_i, outs_s = [], []
        for r0 in range(0, a.users, a.chunk):
            S = (U[r0:r0 + a.chunk] @ V.T).float() + bias[None, :]
            t = torch.topk(S, a.k, dim=1)
            outs_i.append(t.indices)
            outs_s.append(t.values)
        return torch.cat(outs_i), torch.cat(outs_s)

    ms2, (ui, us) = timed(unfused, a.reps)
    same = (torch.sort(fi, 1).values == torch.sort(ui, 1).values).all(1).float().mean().item()
    err = (fs - us).abs().max().item()
    print(json.dumps({"variant": "gemm_bf16+torch.topk", "ms": round(ms2, 3), "tflops": round(flop / ms2 / 1e9, 1),
                      "speedup_fused": round(ms2 / ms, 2), "same_topk_set_frac": round(same, 4),
                      "max_score_diff": err}), flush=True)


if __name__ == "__main__":
    main()
