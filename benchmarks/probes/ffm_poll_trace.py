"""Per-row loss traces at grid 1 on bf16 state: the polled pipelined FFM kernel (variant 5) vs
the round-1 packed kernel (variant 1, no lookahead: the sequential order) — the first row where
they differ, on Criteo-like rows (shared features) and on rows with disjoint features.
    python benchmarks/probes/ffm_poll_trace.py
"""
import torch

from hivemall_amd.io.synthetic import criteo_like
from hivemall_amd.ops import ffm as ffm_op
from hivemall_amd.ops.ffm import FFMHyper, ffm_step, new_state_tables


def trace(variant, idx, y, nf, use_linear):
    ffm_op._VARIANT = variant
    B, F = idx.shape
    g = torch.Generator().manual_seed(0)
    V, G = new_state_tables(nf, F, 4, torch.bfloat16, "cuda", packed=True)
    V.copy_((torch.rand(nf, F, 4, generator=g) * 0.5).to(torch.bfloat16))
    st = dict(V=V, G=G, w=torch.zeros(nf, device="cuda"), wz=torch.zeros(nf, device="cuda"),
              wn=torch.zeros(nf, device="cuda"), bias=torch.zeros(4, device="cuda"))
    h = FFMHyper(use_linear=use_linear, use_bias=False)
    loss = torch.empty(B, device="cuda")
    ffm_step(st, idx, None, None, y, h, loss=loss, grid=1)
    torch.cuda.synchronize()
    return loss.cpu(), st["V"].float().cpu()


def main():
    for name, (idx, y) in {"criteo_like": criteo_like(4096, hash_bits=12, seed=5),
                           "disjoint": (torch.arange(4096 * 39, dtype=torch.int32).reshape(4096, 39),
                                        torch.where(torch.rand(4096) < 0.3, 1.0, -1.0))}.items():
        nf = int(idx.max()) + 1
        for lin in (False, True):
            a, Va = trace(5, idx.cuda(), y.cuda(), nf, lin)
            b, Vb = trace(1, idx.cuda(), y.cuda(), nf, lin)
            d = (a - b).abs()
            bad = torch.nonzero(d > 1e-6).flatten()
            first = int(bad[0]) if bad.numel() else -1
            print(f"{name} linear={lin}: rows differing {bad.numel()}/{len(a)}, first {first}, "
                  f"max|dloss| {d.max().item():.3g}, max|dV| {(Va - Vb).abs().max().item():.3g}", flush=True)
            if first >= 0:
                r = first
                print("   loss poll  ", a[max(0, r - 2): r + 3].tolist(), "\n   loss packed", b[max(0, r - 2): r + 3].tolist())
                prev = idx[r - 1].tolist() if r else []
                print("   shared features with the previous row:", len(set(prev) & set(idx[r].tolist())),
                      "with row-2:", len(set(idx[r - 2].tolist()) & set(idx[r].tolist())) if r > 1 else None)


if __name__ == "__main__":
    main()
