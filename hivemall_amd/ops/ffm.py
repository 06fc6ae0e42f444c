"""FFM train/predict op: gfx950 kernel on ``cuda`` tensors, C++ engine on CPU tensors.

Kernel: ``csrc/kernels/ffm.hip`` (hm_ffm_step).  CPU twin: ``csrc/host/ffm_cpu.cpp``.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native


@dataclass
class FFMHyper:
    eta0: float = 0.2
    eps: float = 1.0
    lambda_v: float = 1e-4
    alpha: float = 0.2
    beta: float = 1.0
    lambda1: float = 1e-3
    lambda2: float = 1e-4
    min_target: float = -3.4e38
    max_target: float = 3.4e38
    classification: bool = True
    use_linear: bool = True
    use_bias: bool = True
    norm: bool = True
    # re-read the own slot right before its update (short Hogwild read-modify-write window).
    # None = by layout: packed -> False (the gathered V/G stay in registers; measured +20 %
    # rows/s at the same held-out logloss, profiles/ffm_layout_ab_r1.log), split -> True.
    reload: bool | None = None
    seed: int = 31        # stochastic-rounding stream (bf16 state)

    def hp(self) -> np.ndarray:
        return np.array([self.eta0, self.eps, self.lambda_v, self.alpha, self.beta, self.lambda1,
                         self.lambda2, self.min_target, self.max_target], dtype=np.float32)


_CALLS = 0  # per-launch counter mixed into the stochastic-rounding seed
# kernel variant (A/B only; csrc/kernels/ffm.hip hm_ffm_step): 0 = auto (per-slot G: the
# sg12 / sg32 LDS-DMA pipelines; per-element G, K <= 4 packed: bf16 ffm_pipe_kernel, fp32
# ffm_lean_kernel), 1 = the generic ffm_row_kernel, 2 = ffm_lean_kernel for bf16,
# 3 = ffm_pipe_kernel for fp32
_VARIANT = int(os.environ.get("HM_FFM_VARIANT", "0"))


def is_packed(V: torch.Tensor, G: torch.Tensor) -> bool:
    """True when V and G are the two halves of one [NF, FS, 2, Kp] table, FS >= NFLD (the packed
    slot layout of csrc/kernels/ffm.hip: one 16-B access moves a slot's V and G)."""
    if V.dim() != 3 or G.shape != V.shape or G.dtype != V.dtype or G.device != V.device:
        return False
    _, NFLD, Kp = V.shape
    fs = V.stride(0) // (2 * Kp)
    st = (fs * 2 * Kp, 2 * Kp, 1)
    return (fs >= NFLD and V.stride() == st and G.stride() == st
            and G.data_ptr() == V.data_ptr() + Kp * V.element_size())


def field_stride(V: torch.Tensor) -> int:
    """Slots between consecutive features of the V table (NFLD, or the padded FS)."""
    return V.stride(0) // V.stride(1) if V.dim() == 3 and V.stride(1) > 0 else V.shape[1]


def padded_fields(num_fields: int, kp: int, dtype) -> int:
    """Field count of a packed table padded so every feature block is whole 128-B lines (39
    fields of 16-B bf16 slots -> 40 = 640 B = 5 lines).  Measured on MI355X with the bench's
    access pattern (benchmarks/ffm_mem_roofline.py, profiles/ffm_roofline_r2.log): gather +
    write-back of the row's slots 127M rows/s unaligned -> 141M aligned -> 146M aligned with the
    whole block written (diagonal + pad slots)."""
    slot_b = 2 * kp * torch.empty(0, dtype=dtype).element_size()
    per_line = max(1, 128 // slot_b) if 128 % slot_b == 0 else 1
    return (num_fields + per_line - 1) // per_line * per_line


def slot_block_layout(num_fields: int, kp: int, dtype) -> tuple[int, int, int]:
    """Per-slot-G block layout of one feature (GPU): ``[V: FS x Kp (dtype) | G: FS x fp32]``
    padded to whole 128-B lines.  Returns (FS, block bytes, G byte offset); FS is the field
    count padded so the V region is whole lines (fp32 k=4: 40 slots = 640 B, G 160 B, block
    896 B = 7 lines; bf16: 320 B + 160 B -> 512 B = 4 lines)."""
    es = torch.empty(0, dtype=dtype).element_size()
    vsb = kp * es
    per_line = max(1, 128 // vsb) if 128 % vsb == 0 else 1
    fs = (num_fields + per_line - 1) // per_line * per_line
    goff = fs * vsb
    bs = (goff + fs * 4 + 127) // 128 * 128
    return fs, bs, goff


def slot12_layout(num_fields: int) -> tuple[int, int]:
    """12-B slot layout of bf16 V with per-slot G (GPU, k <= 4): per feature FS slots
    {V bf16 x 4 | G fp32} then a zero tail, the block padded to whole 128-B lines (39 fields:
    40 x 12 = 480 B + 32 -> 512 B = 4 lines).  Returns (FS, block bytes)."""
    fs = (num_fields + 3) // 4 * 4            # FS * 12 is a multiple of 16: the tail is 16-B chunks
    return fs, (fs * 12 + 127) // 128 * 128


def lin_record_views(V: torch.Tensor, G: torch.Tensor) -> tuple | None:
    """(w, wz, wn) as views of the 16-B chunk after each feature's slots in the GPU per-slot block
    layouts (fp32 V: after the G region, byte 800 of 896 for 39 fields; bf16 12-B slots: byte 480
    of 512), or None when V / G are not such a layout.  The kernels then read and write a feature's
    {w, z, n} as one 16-B record in a line the row already touches (csrc/kernels/ffm.hip
    FFMParams.lpack)."""
    if not V.is_cuda or G.dim() != 2 or V.dim() != 3:
        return None
    NF, nfld, kp = V.shape
    es = V.element_size()
    bs = V.stride(0) * es
    d = G.data_ptr() - V.data_ptr()
    if V.dtype == torch.bfloat16 and d == 8:                 # 12-B slots {V bf16 x 4 | G}
        fs, bs12 = slot12_layout(nfld)
        off, ok = fs * 12, bs12 == bs
    elif V.dtype == torch.float32 and d > 0:
        fs, bs32, goff = slot_block_layout(nfld, kp, V.dtype)
        off, ok = goff + fs * 4, bs32 == bs and goff == d
    else:
        return None
    if not ok or off + 16 > bs or off % 16 or bs % 16:
        return None
    raw = torch.empty(0, dtype=torch.uint8, device=V.device).set_(
        V.untyped_storage(), V.storage_offset() * es, (NF, bs), (bs, 1))
    rec = raw[:, off:off + 16].view(torch.float32)          # [NF, 4]: w, z, n, pad
    return rec[:, 0], rec[:, 1], rec[:, 2]


def _lin_addressing(state: dict) -> tuple[int, int]:
    """(lstride, lpack) of the state's linear tables for hm_ffm_step."""
    w, wz, wn = state["w"], state["wz"], state["wn"]
    ls = w.stride(0) if w.dim() == 1 else 1
    pack = int(w.is_cuda and ls > 1 and wz.stride(0) == ls and wn.stride(0) == ls
               and wz.data_ptr() == w.data_ptr() + 4 and wn.data_ptr() == w.data_ptr() + 8
               and w.data_ptr() % 16 == 0 and ls % 4 == 0
               and os.environ.get("HM_FFM_LPACK", "1") != "0")   # 0: 4-B accesses (A/B only)
    if not pack:
        assert ls == 1 or w.is_cuda, "CPU FFM state: contiguous linear tables"
    return ls, pack


def linear_mix_tensors(state: dict) -> list:
    """The FTRL linear state as the replica mixer should see it: with the 16-B records of
    :func:`lin_record_views` one [NF, 4] row view {w, z, n, pad} (a uniform row view, so the fused
    mix kernels of parallel/mix.py take it in one pass; the pad stays 0 on every rank), otherwise
    the three arrays [wz, wn, w]."""
    w = state["w"]
    ls, pack = _lin_addressing(state)
    if pack:
        return [torch.as_strided(w, (w.shape[0], 4), (ls, 1))]
    return [state["wz"], state["wn"], w]


def new_state_tables(num_features: int, num_fields: int, kp: int, dtype, device,
                     packed: bool, slot_g: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """Zeroed (V, G).

    ``slot_g`` (one AdaGrad accumulator per (feature, field) slot, G is [NF, NFLD] fp32):
    ``packed`` -> views of one byte table whose feature blocks hold V then G
    (:func:`slot_block_layout`); else a contiguous V [NF, NFLD, Kp] and G [NF, NFLD].
    Per-element G (G shaped like V): views of one packed [NF, FS, 2, Kp] table (FS =
    line-padded field count), or two split tables."""
    if slot_g:
        if packed and dtype == torch.bfloat16 and kp == 4:
            # 12-B slots {V bf16 x 4 | G fp32} in 512-B blocks (ffm_pipe_sg12_kernel)
            fs, bs = slot12_layout(num_fields)
            buf = torch.zeros((num_features, bs), dtype=torch.uint8, device=device)
            sl = buf[:, :fs * 12]
            V = sl.view(torch.bfloat16).view(num_features, fs, 6)[:, :num_fields, :4]
            G = sl.view(torch.float32).view(num_features, fs, 3)[:, :num_fields, 2]
            return V, G
        if packed:
            fs, bs, goff = slot_block_layout(num_fields, kp, dtype)
            es = torch.empty(0, dtype=dtype).element_size()
            buf = torch.zeros((num_features, bs), dtype=torch.uint8, device=device)
            V = buf[:, :goff].view(dtype).view(num_features, fs, kp)[:, :num_fields]
            G = buf[:, goff:goff + fs * 4].view(torch.float32)[:, :num_fields]
            assert V.stride(0) * es == bs and G.stride(0) * 4 == bs
            return V, G
        return (torch.zeros((num_features, num_fields, kp), dtype=dtype, device=device),
                torch.zeros((num_features, num_fields), dtype=torch.float32, device=device))
    if packed:
        fs = padded_fields(num_fields, kp, dtype)
        VG = torch.zeros((num_features, fs, 2, kp), dtype=dtype, device=device)
        return VG[:, :num_fields, 0, :], VG[:, :num_fields, 1, :]
    shape = (num_features, num_fields, kp)
    return (torch.zeros(shape, dtype=dtype, device=device),
            torch.zeros(shape, dtype=dtype, device=device))


_DEFER: dict = {}   # (device, stream) -> int32 [1 + B] deferral buffer of multi-hot rows (csrc hm_ffm_step)
# Global-bias FTRL state sharded over this many 128-B lines during a training launch (csrc/kernels/
# ffm.hip FFMParams.bias_sh): one same-address pair of atomics per row held -w0 runs at 5.5 M
# rows/s (profiles/r5/ffm_w0_rate.jsonl).  HM_FFM_BIAS_SHARDS=0: the single address (A/B only).
BIAS_SHARDS = int(os.environ.get("HM_FFM_BIAS_SHARDS", "64"))
# rows between a block's re-reads of the shards: 16 -> 32 in round 5 (fp32 -w0 77.1 -> 80.2 M
# rows/s, held-out gap vs sequential +1.9e-3 / +2.0e-3 / +1.8e-3 at 16 / 32 / 64, i.e. noise;
# profiles/r5/ffm_w0_every_quality.jsonl, ffm_w0_every_rate_*.jsonl)
BIAS_EVERY = int(os.environ.get("HM_FFM_BIAS_EVERY", "32"))
_BIAS_SH: dict = {}


def _launch_key(device: torch.device):
    """Scratch buffers (_DEFER, _BIAS_SH) are per (device, stream): two learners training on one
    device from different streams must not share a deferral counter or bias shards (launches on
    ONE stream are ordered, so they may)."""
    return (device, _native.stream_of(device))


def _bias_shards(device: torch.device) -> torch.Tensor:
    key = _launch_key(device)
    sh = _BIAS_SH.get(key)
    if sh is None or sh.shape[0] != BIAS_SHARDS:
        sh = torch.zeros((BIAS_SHARDS, 32), dtype=torch.float32, device=device)
        _BIAS_SH[key] = sh
    return sh
# HM_FFM_DEFER=0 (A/B only): no multi-hot detection in the pipelined kernels (a row with a
# repeated field or feature is then updated slot by slot: racing stores of one address)
_DEFER_ON = os.environ.get("HM_FFM_DEFER", "1") != "0"
# HM_FFM_LIN_DEFER=0 (A/B only): the fp32 kernel's W_LIN wave waits for the next row's linear-state
# DMA at phase A with the slot DMAs, instead of at its first use in the forward pass
_LIN_DEFER = int(os.environ.get("HM_FFM_LIN_DEFER", "1") != "0")
# Linear FTRL steps of the pipelined fp32 kernel without lost updates (HM_FFM_LIN_ATOMIC):
#   4 (default): the top HM_FFM_LIN_HOT features (by frequency in the learner's first batch) keep
#     (z, n) in a dense side table during a launch; each block sums its rows' steps of them in LDS
#     and adds the sums by float atomics when it ends; the other features keep plain record stores
#     (csrc/kernels/ffm.hip ffm_hacc_kernel).
#   1: every row's (z, n) steps by float atomics on the records (A/B: 8.7 M rows/s — the atomics
#     drop the hot features' block lines from L2)
#   0: plain record stores (a concurrent row's step to the same feature is lost)
# The host model benchmarks/ffm_hogwild_sim.py puts ~80 % of the same-stream gap on lost linear
# steps (docs/perf_notes.md, round 6).
_LIN_ATOMIC = int(os.environ.get("HM_FFM_LIN_ATOMIC", "4"))
_LIN_HOT_N = min(int(os.environ.get("HM_FFM_LIN_HOT", "2048")), 2048)   # <= HD_SIZE of the kernel
_LIN_HOT: dict = {}   # (device, w.data_ptr(), NF, H) -> (hidx int32 [NF], hot_id int32 [H], hacc f32 [H, 32], [launches])
_LIN_HOT_KEEP = 8     # states whose tables are kept (4 MB index each at 2^20 features); an evicted
                      # state rebuilds its table from its next batch (its records hold the folded
                      # state after every launch, so nothing is lost)


_LIN_HOT_REFRESH = int(os.environ.get("HM_FFM_LIN_HOT_REFRESH", "256"))   # launches between rebuilds


def _lin_hot_tables(state: dict, idx: torch.Tensor, nhot: int):
    """lin_atomic 4: the hot-feature side tables of this state: the nhot most frequent features of
    its first batch, rebuilt from the current batch every _LIN_HOT_REFRESH launches (a stream whose
    hot features drift; between launches every record holds its folded state, so a rebuild loses
    nothing, and the bincount costs ~2 ms per rebuild)."""
    w = state["w"]
    nf = w.shape[0]
    key = (w.device, w.data_ptr(), nf, nhot)
    t = _LIN_HOT.get(key)
    if t is not None:
        t[3][0] += 1
        if _LIN_HOT_REFRESH > 0 and t[3][0] % _LIN_HOT_REFRESH == 0:
            del _LIN_HOT[key]
            t = None
    if t is None:
        cnt = torch.bincount(idx.reshape(-1).long().clamp(0, nf - 1), minlength=nf)
        top = torch.argsort(cnt, descending=True)[:nhot]
        top = top[cnt[top] > 0].to(torch.int32)
        hidx = torch.full((nf,), -1, dtype=torch.int32, device=w.device)
        hidx[top.long()] = torch.arange(top.numel(), dtype=torch.int32, device=w.device)
        hacc = torch.zeros(max(1, top.numel()), 32, dtype=torch.float32, device=w.device)  # HACC_STRIDE
        while len(_LIN_HOT) >= _LIN_HOT_KEEP:        # the oldest states' tables go first
            _LIN_HOT.pop(next(iter(_LIN_HOT)))
        t = _LIN_HOT[key] = (hidx, top, hacc, [0])
    return t[:3]


def _defer_buffer(device: torch.device, B: int) -> torch.Tensor:
    key = _launch_key(device)
    buf = _DEFER.get(key)
    if buf is None or buf.numel() < 1 + B:
        buf = torch.empty(1 + max(B, 1 << 16), dtype=torch.int32, device=device)
        _DEFER[key] = buf
    return buf


def _has_multihot(idx: torch.Tensor, fld: torch.Tensor | None) -> bool:
    """Any row with a repeated feature or a repeated field (padding / invalid ids excluded)."""
    if idx.numel() == 0 or idx.shape[1] < 2:
        return False
    big = torch.iinfo(torch.int32).max
    pos = torch.arange(idx.shape[1], device=idx.device, dtype=torch.int32)

    def rep(t: torch.Tensor, valid: torch.Tensor) -> bool:
        # invalid entries get distinct sentinels, so they never compare equal
        u = torch.where(valid, t, big - pos.unsqueeze(0))
        s = u.sort(dim=1).values
        return bool((s[:, 1:] == s[:, :-1]).any().item())

    valid = idx >= 0
    if rep(idx, valid):
        return True
    return fld is not None and rep(fld, valid & (fld >= 0))


def ffm_step(state: dict, idx: torch.Tensor, fld: torch.Tensor | None, val: torch.Tensor | None,
             y: torch.Tensor | None, hyper: FFMHyper, train: bool = True,
             pred: torch.Tensor | None = None, loss: torch.Tensor | None = None,
             grid: int = 0, variant: int | None = None, hot: torch.Tensor | None = None,
             lin_mode: int | None = None) -> None:
    """One fused pass over a padded-ELL batch.  ``lin_mode``: the linear steps' form
    (HM_FFM_LIN_ATOMIC values; None = the module default, the side table).

    state: dict with V, G ([NF, NFLD, Kp] f32 or bf16; either two contiguous tables or the two
    halves of one packed [NF, NFLD, 2, Kp] table, see :func:`is_packed`), w, wz, wn ([NF] f32),
    bias ([4] f32).
    idx/fld int32 [B, F]; val f32 [B, F]; y f32 [B] in {-1,+1} (classification) or real.
    """
    V = state["V"]
    B, F = idx.shape
    NF, NFLD, Kp = V.shape
    assert idx.dtype == torch.int32 and idx.is_contiguous()
    for t in (fld, val, y, pred, loss):
        if t is not None:
            assert t.device == V.device and t.is_contiguous(), "tensor device/layout mismatch"
    if fld is not None:
        assert fld.dtype == torch.int32 and fld.shape == idx.shape
    if val is not None:
        assert val.dtype == torch.float32 and val.shape == idx.shape
    if y is not None:
        assert y.shape[0] == B
    if pred is not None:
        assert pred.shape[0] >= B
    if loss is not None:
        assert loss.shape[0] >= B
    if V.is_cuda and train and int(grid) == 1 and variant is None and _VARIANT == 0 and _has_multihot(idx, fld):
        # one block is documented as the sequential learner: a multi-hot row would be deferred by
        # the pipelined kernels until after the batch's other rows, so the whole launch
        # goes to the generic kernel, which trains every row in order with grouped updates
        variant = 1
    G = state["G"]
    bf16 = V.dtype == torch.bfloat16
    slot_g = G.dim() == 2
    gstride = 0
    block = (0, 0)
    if slot_g:
        # one fp32 AdaGrad accumulator per (feature, field) slot: G [NF, NFLD]
        assert G.dtype == torch.float32 and G.shape == V.shape[:2] and G.stride(1) in (1, 3), \
            "per-slot G: fp32 [num_features, num_fields], field stride 1 (or 3: 12-B bf16 slots)"
        assert V.stride(2) == 1 and (V.stride(1) == Kp or (G.stride(1) == 3 and V.stride(1) == 6)), \
            "V: [NF, FS, Kp] slots (or the V part of 12-B {V | G} slots)"
        packed = False
        gstride = G.stride(0)
        # block layout (slot_block_layout): G right after the V region of each feature block
        es = V.element_size()
        d = G.data_ptr() - V.data_ptr()
        bs = V.stride(0) * es
        if G.stride(1) == 3:
            fs, bs12 = slot12_layout(NFLD)
            assert V.is_cuda and bf16 and d == 8 and G.stride(0) * 4 == bs12, "12-B slot layout"
            block = (fs, (bs12 - fs * 12) // 16)
        elif V.is_cuda and G.stride(1) == 1 and 0 < d < bs and d % (Kp * es) == 0 and G.stride(0) * 4 == bs:
            vpad = d // (Kp * es)
            tail = bs - d - vpad * 4
            if tail >= 0 and tail % 16 == 0:
                block = (vpad, tail // 16)
    else:
        assert G.dtype == V.dtype, "V and G must share the storage dtype"
        packed = is_packed(V, G)
        if not packed:
            assert V.is_contiguous() and G.is_contiguous(), \
                "FFM state: two contiguous V/G tables or the halves of one packed table"
    assert not bf16 or V.is_cuda, "bf16 FFM state is a device-only layout"
    global _CALLS
    _CALLS += 1
    ip = np.array([B, F, NF, NFLD, Kp, int(hyper.classification), int(train), int(hyper.use_linear),
                   int(hyper.use_bias), int(hyper.norm), int(grid),
                   int((not packed) if hyper.reload is None else hyper.reload), int(bf16),
                   (hyper.seed * 1000003 + _CALLS) & 0x7FFFFFFF, int(packed),
                   _VARIANT if variant is None else int(variant),
                   field_stride(V), int(slot_g), gstride, block[0], block[1],
                   G.stride(1) if slot_g else 0, _LIN_DEFER, BIAS_EVERY] + list(_lin_addressing(state))
                  + [_LIN_ATOMIC, 0],
                  dtype=np.int32)
    hp = hyper.hp()
    p = _native.ptr
    args = (ip.ctypes.data, hp.ctypes.data, p(idx), p(fld), p(val), p(y), p(V), p(G),
            p(state["w"]), p(state["wz"]), p(state["wn"]), p(state["bias"]), p(pred), p(loss))
    if V.is_cuda:
        if hot is not None:
            assert hot.dtype == torch.uint8 and hot.numel() >= NF and hot.device == V.device
        # multi-hot rows (a repeated field or feature) are deferred by the pipelined kernels to
        # the grouped-update kernel through this buffer (same stream, no host sync)
        bsh = _bias_shards(V.device) if (train and hyper.use_bias and BIAS_SHARDS > 0) else None
        if bsh is not None:
            # shard 0 <- the bias FTRL state (z0, n0), the other shards 0; the pipelined kernels add
            # each row's step to shard (block % S), the generic kernel (deferred rows) to bias itself
            b = state["bias"]
            zn0 = b[1:3].clone()
            bsh.zero_()
            bsh[0, :2] = zn0
        lin_mode, hidx, hot_id, hacc = _LIN_ATOMIC if lin_mode is None else int(lin_mode), None, None, None
        if lin_mode == 4:
            if train and hyper.use_linear and _lin_addressing(state)[1]:
                # the bf16 kernel's LDS holds the sums of 1,024 hot features (HD12_SIZE)
                hidx, hot_id, hacc = _lin_hot_tables(state, idx, 1024 if bf16 else _LIN_HOT_N)
            if hot_id is None or hot_id.numel() == 0:
                lin_mode, hidx, hot_id, hacc = 0, None, None, None
        ip[26], ip[27] = lin_mode, hot_id.numel() if hot_id is not None else 0
        aux = (ctypes.c_void_p * 7)(p(hot), p(_defer_buffer(V.device, B)) if (train and _DEFER_ON) else None,
                                    p(bsh), bsh.shape[0] if bsh is not None else 0,
                                    p(hidx), p(hot_id), p(hacc))
        rc = _native.hip().hm_ffm_step(*args, ctypes.addressof(aux), _native.stream_of(V.device))
        _native.check(rc, "hm_ffm_step")
        if bsh is not None:
            # (z0, n0) = the shard sums plus whatever the generic kernel added to bias directly
            b[1:3] = bsh[:, :2].sum(0) + (b[1:3] - zn0)
        if train and hyper.use_bias:
            # w0 = f(z0, n0): the kernel accumulates z0/n0 atomically and its cached bias[0] is
            # whichever block wrote last; refresh it (FTRL weight with l1 = l2 = 0)
            b = state["bias"]
            b[0] = -b[1] / ((hyper.beta + b[2].sqrt()) / hyper.alpha)
    else:
        rc = _native.host().hm_ffm_step_cpu(*args)
        if rc != 0:
            raise RuntimeError(f"hm_ffm_step_cpu failed: {rc}")
