"""Fused top-k maximum inner product search (``csrc/kernels/topk_mips.hip``).

``mips_topk(Q, I, k)`` returns, for every query row, the ``k`` items with the largest
``<Q[q], I[n]> + item_bias[n]`` (+ ``row_bias[q]`` on the returned scores), best first,
optionally excluding a per-query sorted item list (already-seen items, Hivemall's
``populate_not_in``) and/or the query's own index (item-item kNN).

On ``cuda`` tensors this is one gfx950 kernel: bf16 MFMA score tiles filtered against a
running per-row top-k in LDS — the M x N score matrix never reaches HBM.  CPU tensors use a
blocked fp32 ``matmul`` + ``topk`` with the same contract (and tie order: higher score first,
then lower item index).

This is the fused form of the reference's recommendation query
``each_top_k(k, user, mf_predict(...) / bprmf_predict(...), item)`` over the user x item
join (core/src/main/java/hivemall/tools/EachTopKUDTF.java, mf/MFPredictionUDF.java,
mf/BPRMFPredictionUDF.java; SURVEY.md §2.3.5 kernel K8) and of cosine-similarity kNN
(knn/similarity/CosineSimilarityUDF.java).
"""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native

_P = C.c_void_p
_native.register_hip("hm_mips_topk", [C.c_int] * 7 + [_P] * 7 + [_P])

KMAX = 64
_KD = (32, 64, 128, 256)


def _pad_bf16(x: torch.Tensor, kd: int) -> torch.Tensor:
    out = torch.zeros(x.shape[0], kd, dtype=torch.bfloat16, device=x.device)
    out[:, : x.shape[1]] = x.to(torch.bfloat16)
    return out.contiguous()


def exclusion_csr(rows, items, n_rows: int, device=None):
    """(query row, item) pairs -> (ptr int64 [n_rows+1], items sorted per row int32)."""
    r = torch.as_tensor(rows, device=device).long()
    i = torch.as_tensor(items, device=device).long()
    key = torch.unique(r * (1 << 32) + i)
    rr = key >> 32
    ii = (key & 0xFFFFFFFF).to(torch.int32)
    ptr = torch.zeros(n_rows + 1, dtype=torch.int64, device=r.device)
    ptr[1:] = torch.cumsum(torch.bincount(rr, minlength=n_rows), 0)
    return ptr.contiguous(), ii.contiguous()


def _splits_for(M: int, N: int, sms: int) -> int:
    blocks = (M + 63) // 64
    s = 1
    # at least ~4 blocks per CU, each split still sweeping >= 8 tiles of 64 items
    while blocks * s < 4 * sms and N // (64 * s * 2) >= 8:
        s *= 2
    return s


def _merge(idx: torch.Tensor, sc: torch.Tensor, k: int):
    """[S, M, k] partial results -> [M, k] (score desc, index asc)."""
    S, M, _ = idx.shape
    idx = idx.permute(1, 0, 2).reshape(M, S * k)
    sc = sc.permute(1, 0, 2).reshape(M, S * k)
    # lexicographic (score desc, idx asc): sort by idx first, then stable sort by score
    big = torch.where(idx < 0, torch.full_like(idx, 2**31 - 1), idx)
    o = torch.argsort(big, dim=1, stable=True)
    idx, sc = idx.gather(1, o), sc.gather(1, o)
    o = torch.argsort(sc, dim=1, descending=True, stable=True)[:, :k]
    return idx.gather(1, o), sc.gather(1, o)


def mips_topk(Q: torch.Tensor, I: torch.Tensor, k: int, item_bias: torch.Tensor | None = None,
              row_bias: torch.Tensor | None = None, exclude: tuple | None = None,
              exclude_self_offset: int | None = None, splits: int | None = None):
    """Top-``k`` items per query row; returns (indices int64 [M,k], scores fp32 [M,k]).
    Missing entries (fewer than k admissible items) are index -1 / score -inf.

    exclude: (ptr int64 [M+1], items int32 sorted per row) from ``exclusion_csr``.
    exclude_self_offset: drop item ``q + offset`` for query ``q`` (0 for Q is I)."""
    M, d = Q.shape
    N, d2 = I.shape
    if d != d2:
        raise ValueError(f"mips_topk: dimension mismatch {d} vs {d2}")
    if not 0 < k <= KMAX:
        raise ValueError(f"mips_topk: k must be in 1..{KMAX}")
    if Q.is_cuda:
        return _mips_gpu(Q, I, k, item_bias, row_bias, exclude, exclude_self_offset, splits)
    return _mips_cpu(Q, I, k, item_bias, row_bias, exclude, exclude_self_offset)


def _mips_gpu(Q, I, k, item_bias, row_bias, exclude, self_off, splits):
    dev = Q.device
    M, d = Q.shape
    N = I.shape[0]
    kd = next((x for x in _KD if x >= d), None)
    if kd is None:
        raise ValueError(f"mips_topk: dimension {d} > {_KD[-1]}")
    Qb, Ib = _pad_bf16(Q, kd), _pad_bf16(I.to(dev), kd)
    bias = item_bias.to(device=dev, dtype=torch.float32).contiguous() if item_bias is not None else None
    if splits is None:
        splits = _splits_for(M, N, torch.cuda.get_device_properties(dev).multi_processor_count)
    ex_ptr = ex_idx = None
    if exclude is not None:
        ex_ptr, ex_idx = (t.to(dev).contiguous() for t in exclude)
        if ex_ptr.dtype != torch.int64 or ex_idx.dtype != torch.int32 or ex_ptr.numel() != M + 1:
            raise ValueError("mips_topk: exclude must be (int64 ptr [M+1], int32 items)")
    oi = torch.empty(splits, M, k, dtype=torch.int32, device=dev)
    os_ = torch.empty(splits, M, k, dtype=torch.float32, device=dev)
    p = _native.ptr
    rc = _native.hip().hm_mips_topk(M, N, kd, k, splits, int(self_off is not None), int(self_off or 0),
                                    p(Qb), p(Ib), p(bias), p(ex_ptr), p(ex_idx), p(oi), p(os_),
                                    _native.stream_of(dev))
    _native.check(rc, "hm_mips_topk")
    if splits > 1:
        idx, sc = _merge(oi, os_, k)
    else:
        idx, sc = oi[0], os_[0]
    idx = idx.long()
    if row_bias is not None:
        sc = torch.where(idx >= 0, sc + row_bias.to(dev, torch.float32)[:, None], sc)
    return idx, sc


def _mips_cpu(Q, I, k, item_bias, row_bias, exclude, self_off, block: int = 4096):
    M = Q.shape[0]
    N = I.shape[0]
    Qf, If = Q.float(), I.float()
    out_i = torch.full((M, k), -1, dtype=torch.int64)
    out_s = torch.full((M, k), -float("inf"))
    for r0 in range(0, M, block):
        r1 = min(M, r0 + block)
        S = Qf[r0:r1] @ If.T
        if item_bias is not None:
            S += item_bias.float()[None, :]
        if self_off is not None:
            cols = torch.arange(r0, r1) + self_off
            ok = (cols >= 0) & (cols < N)
            S[torch.nonzero(ok).flatten(), cols[ok]] = -float("inf")
        if exclude is not None:
            ptr, ex = exclude
            ptr = ptr.cpu()
            lo, hi = int(ptr[r0]), int(ptr[r1])
            rows = torch.repeat_interleave(torch.arange(r1 - r0), (ptr[r0 + 1: r1 + 1] - ptr[r0:r1]))
            S[rows, ex.cpu()[lo:hi].long()] = -float("inf")
        # (score desc, index asc): topk over a stably index-ordered matrix
        kk = min(k, N)
        o = torch.argsort(S, dim=1, descending=True, stable=True)[:, :kk]
        sc = S.gather(1, o)
        o = torch.where(torch.isinf(sc) & (sc < 0), torch.full_like(o, -1), o)
        out_i[r0:r1, :kk] = o
        out_s[r0:r1, :kk] = sc
    if row_bias is not None:
        out_s = torch.where(out_i >= 0, out_s + row_bias.float()[:, None], out_s)
    return out_i, out_s
