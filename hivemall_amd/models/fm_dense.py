"""Mini-batch FM engine for low-dimensional dense inputs (``train_fm -engine minibatch``).

Why: the per-row Hogwild kernel (``csrc/kernels/fm.hip``) runs one row per wave with thousands
of rows in flight.  On sparse, high-cardinality rows (Criteo) concurrent rows rarely share a
feature; on dense rows (HIGGS: the same 28 features in every row) every row in flight
read-modify-writes the same 28 x (1 + k) parameters and the model diverges (measured:
held-out logloss 1e13 at 257 M rows/s, while the sequential engine reaches 0.540-0.549;
``benchmarks/probes/fm_dense_probe.py``, ``profiles/fm_dense_r2/``).

MI355X design: the rows are densified once into an HBM-resident fp32 matrix X [n, d]; a step of
B rows computes
    XV = X V,  p = w0 + X w + 0.5 sum_f ((XV)^2 - X^2 V^2)_f,  g = dloss/dp,
    dV = X^T (g * XV) - V * (X^2)^T g,  dw = X^T g,  dw0 = sum g
and an AdaGrad update of the mean gradient (L2 terms lambda0 / lambda_w / lambda).  On the GPU
(d <= 64, padded k <= 32) a step is two launches of ``csrc/kernels/fm_dense.hip``: a gradient
kernel whose two GEMM-shaped products (X V and (g X)^T [XV | 1]) run on f32 MFMA
(v_mfma_f32_16x16x4_f32: exact f32) with the partial gradient held in accumulator registers over
the workgroup's row tiles, then a parameter-parallel AdaGrad kernel; elsewhere it is the
same math as torch ops (the GEMM formulation — on the GPU hipBLASLt's MFMA kernels — measured
9-56 M rows/s, launch- and skinny-GEMM-bound).  A whole epoch (up to 256 steps per graph) is
captured once as HIP graphs and replayed, so the host issues one launch per 256 steps.
Semantics: mini-batch AdaGrad, not Hivemall's per-row SGD (documented in docs/compat.md); the
learning rate is ``-eta0``.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native

GRAPH_STEPS = 256
_P = _native.c_p
_native.register_hip("hm_fmd_step", [_P] * 13)     # ..., loss_sum, stream
_native.register_hip("hm_fmd_max_blocks", [], restype=__import__("ctypes").c_int64)


class DenseMinibatchFM:
    def __init__(self, dims: int, k: int, V0: torch.Tensor, device, batch: int, lr: float,
                 lambda0: float, lambda_w: float, lambda_v: float, classification: bool,
                 min_target: float, max_target: float, eps: float = 1e-8, variant: int = 0,
                 blocks: int = 0):
        dev = torch.device(device)
        self.dims, self.k, self.B, self.dev = int(dims), int(k), int(batch), dev
        self.KP = int(V0.shape[1])             # padded factors (columns >= k stay zero)
        self.V = torch.zeros(dims, self.KP, dtype=torch.float32, device=dev)
        self.V[:, :k] = V0[:, :k].to(dev, torch.float32)
        self.w = torch.zeros(dims, dtype=torch.float32, device=dev)
        self.w0 = torch.zeros(1, dtype=torch.float32, device=dev)
        self.GV = torch.zeros_like(self.V)
        self.Gw = torch.zeros_like(self.w)
        self.Gw0 = torch.zeros_like(self.w0)
        self.lr, self.eps = float(lr), float(eps)
        self.l0, self.lw, self.lv = float(lambda0), float(lambda_w), float(lambda_v)
        self.cls = bool(classification)
        self.lo, self.hi = float(min_target), float(max_target)
        self.loss_sum = torch.zeros(1, dtype=torch.float64, device=dev)
        self._graphs: list | None = None
        self._key = None
        self.kernel = dev.type == "cuda" and self.dims <= 64 and self.KP <= 32
        if self.kernel:
            self._hp = np.array([self.lr, self.eps, self.l0, self.lw, self.lv, self.lo, self.hi], dtype=np.float32)
            # variant 0: the f32-MFMA gradient kernel, 1: the VALU kernel; blocks: workgroups per
            # step (0 = the kernel's default); partial rows for up to hm_fmd_max_blocks() workgroups
            self.variant, self.blocks = int(variant), int(blocks)
            nblk = min(max(128, int(_native.hip().hm_fmd_max_blocks())), (self.B + 63) // 64)
            self._partial = torch.empty(nblk * (self.dims * self.KP + self.dims + 2),
                                        dtype=torch.float32, device=dev)
            self._ips: dict = {}

    # ------------------------------------------------------------------ math
    def _pred(self, x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        XV = x @ self.V
        x2 = x * x
        p = self.w0 + x @ self.w + 0.5 * (XV.square().sum(1) - x2 @ self.V.square().sum(1))
        return p, XV, x2

    def step(self, x: torch.Tensor, y: torch.Tensor) -> None:
        """One AdaGrad step on the mean gradient of rows x [b, d] with targets y [b]."""
        b = x.shape[0]
        if self.kernel and b <= self.B:
            ip = self._ips.get(b)
            if ip is None:      # kept alive: a captured graph bakes the pointer values in
                ip = self._ips[b] = np.array([b, self.dims, self.KP, self.k, int(self.cls), self.variant,
                                              self.blocks], dtype=np.int64)
            p = _native.ptr
            rc = _native.hip().hm_fmd_step(ip.ctypes.data, self._hp.ctypes.data, p(x), p(y), p(self.V), p(self.w),
                                           p(self.w0), p(self.GV), p(self.Gw), p(self.Gw0), p(self._partial),
                                           p(self.loss_sum), _native.stream_of(self.dev))
            _native.check(rc, "hm_fmd_step")
            return
        p, XV, x2 = self._pred(x)
        if self.cls:
            # y in {-1, +1}: loss = log(1 + exp(-y p)), dloss/dp = -y sigmoid(-y p)
            z = -y * p
            g = -y * torch.sigmoid(z)
            self.loss_sum += torch.nn.functional.softplus(z).sum().double()
        else:
            pc = p.clamp(self.lo, self.hi)
            g = pc - y
            self.loss_sum += (0.5 * g.square()).sum().double()
        g = g / b
        dV = x.t() @ (g[:, None] * XV) - self.V * (x2.t() @ g)[:, None] + self.lv * self.V
        dw = x.t() @ g + self.lw * self.w
        dw0 = g.sum().reshape(1) + self.l0 * self.w0
        for P, G, D in ((self.V, self.GV, dV), (self.w, self.Gw, dw), (self.w0, self.Gw0, dw0)):
            G.addcmul_(D, D)
            P.addcdiv_(D, G.sqrt().add_(self.eps), value=-self.lr)

    # ------------------------------------------------------------------ epochs
    def _capture(self, X: torch.Tensor, y: torch.Tensor) -> list:
        n = X.shape[0]
        nb = n // self.B
        graphs = []
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        # warm the kernels (and the allocator) outside the capture on throwaway copies
        saved = [t.clone() for t in (self.V, self.w, self.w0, self.GV, self.Gw, self.Gw0, self.loss_sum)]
        with torch.cuda.stream(s):
            self.step(X[: self.B], y[: self.B])
        torch.cuda.current_stream(self.dev).wait_stream(s)
        for t, v in zip((self.V, self.w, self.w0, self.GV, self.Gw, self.Gw0, self.loss_sum), saved):
            t.copy_(v)
        for c0 in range(0, nb, GRAPH_STEPS):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for b in range(c0, min(nb, c0 + GRAPH_STEPS)):
                    self.step(X[b * self.B:(b + 1) * self.B], y[b * self.B:(b + 1) * self.B])
            graphs.append(g)
        return graphs

    def epoch(self, X: torch.Tensor, y: torch.Tensor) -> float:
        """One pass over X [n, d] fp32 / y [n] in order; returns the summed loss."""
        n = X.shape[0]
        nb = n // self.B
        self.loss_sum.zero_()
        if self.dev.type == "cuda" and nb > 0:
            key = (X.data_ptr(), y.data_ptr(), n, self.B)
            if self._graphs is None or self._key != key:
                self._graphs, self._key = self._capture(X, y), key
            for g in self._graphs:
                g.replay()
        else:
            for b in range(nb):
                self.step(X[b * self.B:(b + 1) * self.B], y[b * self.B:(b + 1) * self.B])
        if n > nb * self.B:                       # the tail rows: one smaller eager step
            self.step(X[nb * self.B:], y[nb * self.B:])
        return float(self.loss_sum.item())

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        with torch.no_grad():
            return self._pred(X)[0]


def densify(indptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor | None, dims: int,
            device) -> torch.Tensor:
    """CSR rows -> dense fp32 [n, dims] on ``device`` (duplicate indices add up)."""
    dev = torch.device(device)
    n = indptr.numel() - 1
    ip = indptr.to(dev)
    counts = ip[1:] - ip[:-1]
    rows = torch.repeat_interleave(torch.arange(n, device=dev), counts)
    cols = idx.to(dev).long()
    v = val.to(dev, torch.float32) if val is not None else torch.ones(cols.numel(), device=dev)
    ok = (cols >= 0) & (cols < dims)
    X = torch.zeros(n * dims, dtype=torch.float32, device=dev)
    X.index_add_(0, rows[ok] * dims + cols[ok], v[ok])
    return X.view(n, dims)
