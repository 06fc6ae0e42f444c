"""Model mixing over RCCL — the MixServer / ``GROUP BY feature avg(weight)`` replacement.

Upstream (reference hivemall/mix/**, mixserv/**):
* one-shot averaging: every mapper trains an independent model, the query then does
  ``avg(weight) GROUP BY feature`` (or ``argmin_kld(weight, covar)`` for CW/AROW/SCW);
* iterative mixing: learners push (w, covar) to a MixServer that replies with the mixed
  value (``PartialAverage`` / ``PartialArgminKLD``).

MI355X-native: every rank holds the whole (hashed, dense) model in HBM, so mixing is a
collective on dense tensors:
* AVERAGE    = all_reduce(SUM) / world
* ARGMIN_KLD = all_reduce over the interleaved pair [w/σ, 1/σ] -> w = Σ(w/σ)/Σ(1/σ),
               σ = 1/Σ(1/σ)
Bucketing: small tensors are coalesced into one flat buffer; big ones are reduced in
place in ``bucket_mb`` chunks, all issued asynchronously so RCCL keeps several rings'
worth of work in flight over the 7 xGMI links.  Chunks default to 64 MB (a single ring
step then moves 8 MB per link; big enough to be bandwidth-bound, small enough for ≥7
chunks on any model over 448 MB).  Optimizer state stays local by default (upstream only
mixes weights/covariance).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .dist import DistContext, context


class ModelMixer:
    def __init__(self, ctx: DistContext | None = None, bucket_mb: float = 64.0,
                 small_bytes: int = 4 << 20, wire_dtype: torch.dtype | None = None):
        self.ctx = ctx or context()
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.small_bytes = small_bytes
        self.wire_dtype = wire_dtype
        self.bytes_reduced = 0
        self.calls = 0

    @property
    def world(self) -> int:
        return self.ctx.world_size

    def _active(self) -> bool:
        return self.ctx.is_dist and self.world > 1

    def all_reduce_sum(self, tensors: list[torch.Tensor]) -> None:
        """In-place SUM all-reduce of a list of tensors (bucketed, async; non-contiguous views
        are reduced through a contiguous copy)."""
        if not self._active():
            return
        small = [t for t in tensors if t.numel() * t.element_size() <= self.small_bytes]
        big = [t for t in tensors if t.numel() * t.element_size() > self.small_bytes]
        works = []
        flat = None
        if small:
            flat = torch.cat([t.reshape(-1).to(torch.float32) for t in small])
            works.append(dist.all_reduce(flat, async_op=True))
        staged = []   # strided views (e.g. the V half of the packed FFM table) go via a copy
        for t in big:
            buf = t if t.is_contiguous() else t.contiguous()
            if buf is not t:
                staged.append((t, buf))
            v = buf.view(-1)
            step = max(1, self.bucket_bytes // buf.element_size())
            for s in range(0, v.numel(), step):
                works.append(dist.all_reduce(v[s:s + step], async_op=True))
        for w in works:
            w.wait()
        for t, buf in staged:
            t.copy_(buf)
        if flat is not None:
            off = 0
            for t in small:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t).to(t.dtype))
                off += n
        self.calls += 1
        self.bytes_reduced += sum(t.numel() * t.element_size() for t in tensors)

    def average(self, tensors: list[torch.Tensor]) -> None:
        if not self._active():
            return
        self.all_reduce_sum(tensors)
        inv = 1.0 / self.world
        for t in tensors:
            t.mul_(inv)

    def argmin_kld(self, w: torch.Tensor, covar: torch.Tensor, eps: float = 1e-12) -> None:
        """Mix (w, covar) in place with the argmin-KLD rule (PartialArgminKLD)."""
        if not self._active():
            return
        inv = 1.0 / covar.clamp_min(eps)
        num = w * inv
        self.all_reduce_sum([num, inv])
        w.copy_(num / inv)
        covar.copy_(1.0 / inv)

    def broadcast(self, tensors: list[torch.Tensor], src: int = 0) -> None:
        if not self._active():
            return
        works = [dist.broadcast(t, src, async_op=True) for t in tensors]
        for w in works:
            w.wait()

    def all_gather_cat(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenation (dim 0, rank order) of an equally-shaped tensor from every rank."""
        if not self._active():
            return t
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t.contiguous())
        return torch.cat(out, 0)

    def all_reduce_scalar(self, x: float, op: str = "sum") -> float:
        if not self._active():
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.ctx.device)
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                               "min": dist.ReduceOp.MIN}[op])
        return float(t.item())


class OverlappedMixer:
    """Stale-by-one model averaging whose all-reduce runs behind the training kernels.

    ``start(tensors)`` snapshots the replicas (one device copy on the compute stream) and
    launches the bucketed all-reduce of the snapshot asynchronously (RCCL's own stream);
    training continues.  ``finish()`` (at the next mix point) waits for the collective on the
    device — not on the host — and merges it without discarding the local progress made in the
    meantime:

        x  <-  x + (mean_r(snapshot_r) - snapshot_local)

    i.e. every rank moves by the consensus correction of the snapshot.  This is the
    asynchronous MixServer semantics (replies arrive while the learner keeps training) on
    xGMI, and it hides the collective completely when one mix interval of compute takes longer
    than the all-reduce.  Buffers are allocated once (2x the mixed bytes).
    """

    def __init__(self, mixer: ModelMixer):
        self.m = mixer
        self.snap: list[torch.Tensor] | None = None
        self.buf: list[torch.Tensor] | None = None
        self.works: list = []
        self.targets: list[torch.Tensor] = []

    def pending(self) -> bool:
        return bool(self.works)

    def start(self, tensors: list[torch.Tensor]) -> None:
        if not self.m._active():
            return
        if self.works:
            self.finish()
        if self.snap is None:
            # bf16 replicas are reduced in fp32: an 8-way sum rounded to 8 mantissa bits would
            # inject noise into every mix (the wire cost is hidden behind compute anyway).  The
            # snapshot keeps the replica's own dtype (an exact copy), which halves its bytes.
            wide = lambda t: torch.empty(t.shape, dtype=torch.float32 if t.dtype in (
                torch.bfloat16, torch.float16) else t.dtype, device=t.device)
            self.snap = [torch.empty(t.shape, dtype=t.dtype, device=t.device) for t in tensors]
            self.buf = [wide(t) for t in tensors]
        self.targets = tensors
        for s, b, t in zip(self.snap, self.buf, tensors):
            s.copy_(t)          # one strided read of the replica (e.g. the V half of packed VG)
            b.copy_(s)
        self.works = []
        for b in self.buf:
            v = b.view(-1)
            step = max(1, self.m.bucket_bytes // b.element_size())
            for s0 in range(0, v.numel(), step):
                self.works.append(dist.all_reduce(v[s0:s0 + step], async_op=True))
        self.m.calls += 1
        self.m.bytes_reduced += sum(t.numel() * t.element_size() for t in tensors)

    def finish(self) -> None:
        if not self.works:
            return
        for w in self.works:
            w.wait()
        self.works = []
        inv = 1.0 / self.m.world
        for t, s, b in zip(self.targets, self.snap, self.buf):
            # x <- x + (mean - snapshot): in place, fp32 math, one rounding to t's dtype
            b.mul_(inv).sub_(s)
            t.add_(b)


class SparseDeltaMixer:
    """Touched-row model averaging: all-gather of (row index, Δrow) instead of a dense
    all-reduce (SURVEY.md §5.8 "sparse alternative"; upstream's MixClient likewise only pushes
    the features a learner updated, reference hivemall/mix/client/MixClient.java).

    Every rank keeps ``base`` = the last mixed model.  Rows that a rank did not touch since then
    equal ``base`` on that rank, so the replica mean is exactly

        mean_r(x_r) = base + Σ_r Δ_r / world,   Δ_r = x_r - base  (non-zero on touched rows only)

    ``mix(tensors)`` finds the touched rows of dim 0 (any element changed), all-gathers their
    counts, then the padded (index, Δ) payloads, scatter-adds them into ``base`` (index_add_,
    fp32) and copies the result back — bit-for-bit the dense average up to summation order.
    Wire bytes per rank are ``world · touched · (row_bytes + 8)`` against ``≈2 · rows ·
    row_bytes`` for a ring all-reduce, so when the touched fraction exceeds ``dense_fraction``
    (default ``1 / world``) the step falls back to the dense bucketed all-reduce of
    :class:`ModelMixer` — decided collectively (max over ranks) so every rank takes the same
    path.  Costs one fp32 copy of the mixed tensors for ``base``.
    """

    def __init__(self, mixer: ModelMixer, dense_fraction: float | None = None):
        self.m = mixer
        self.dense_fraction = dense_fraction
        self.base: list[torch.Tensor] | None = None
        self.sparse_rows = 0
        self.dense_mixes = 0

    def _touched(self, t: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
        d = t.to(torch.float32) != b
        if d.dim() == 0:
            return d.reshape(1).nonzero().view(-1)
        if d.dim() > 1:
            d = d.reshape(d.shape[0], -1).any(1)
        return d.nonzero().view(-1)

    def mix(self, tensors: list[torch.Tensor]) -> None:
        if not self.m._active():
            return
        if self.base is None:
            # first call: the replicas may differ everywhere (independent init) -> dense
            self.m.average(tensors)
            self.base = [t.detach().to(torch.float32).clone() for t in tensors]
            self.dense_mixes += 1
            return
        world = self.m.world
        frac = self.dense_fraction if self.dense_fraction is not None else 1.0 / world
        idx = [self._touched(t, b) for t, b in zip(tensors, self.base)]
        dev = tensors[0].device
        counts = torch.tensor([i.numel() for i in idx], dtype=torch.int64, device=dev)
        gathered = [torch.empty_like(counts) for _ in range(world)]
        dist.all_gather(gathered, counts)
        allc = torch.stack(gathered).cpu()                  # [world, n_tensors]
        maxc = allc.max(0).values.tolist()
        for k, (t, b, ix) in enumerate(zip(tensors, self.base, idx)):
            if t.dim() == 0:
                self.m.average([t])
                b.copy_(t)
                continue
            rows = t.shape[0]
            if maxc[k] == 0:
                t.copy_(b)
                continue
            if maxc[k] > frac * rows:
                self.m.average([t])
                b.copy_(t)
                self.dense_mixes += 1
                continue
            n = maxc[k]
            tail = tuple(t.shape[1:])
            pad_i = torch.full((n,), -1, dtype=torch.int64, device=dev)
            pad_i[:ix.numel()] = ix
            delta = torch.zeros((n,) + tail, dtype=torch.float32, device=dev)
            delta[:ix.numel()] = t[ix].to(torch.float32) - b[ix]
            all_i = [torch.empty_like(pad_i) for _ in range(world)]
            all_d = [torch.empty_like(delta) for _ in range(world)]
            w1 = dist.all_gather(all_i, pad_i, async_op=True)
            w2 = dist.all_gather(all_d, delta, async_op=True)
            w1.wait()
            w2.wait()
            gi = torch.cat(all_i)
            gd = torch.cat(all_d)
            keep = gi >= 0
            b.index_add_(0, gi[keep], gd[keep], alpha=1.0 / world)
            t.copy_(b)
            self.sparse_rows += int(allc[:, k].sum())
            self.m.bytes_reduced += n * world * (delta[0].numel() * 4 + 8)
        self.m.calls += 1
