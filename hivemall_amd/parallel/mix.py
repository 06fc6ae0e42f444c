"""Model mixing over RCCL — the MixServer / ``GROUP BY feature avg(weight)`` replacement.

Upstream (reference hivemall/mix/**, mixserv/**):
* one-shot averaging: every mapper trains an independent model, the query then does
  ``avg(weight) GROUP BY feature`` (or ``argmin_kld(weight, covar)`` for CW/AROW/SCW);
* iterative mixing: learners push (w, covar) to a MixServer that replies with the mixed
  value (``PartialAverage`` / ``PartialArgminKLD``).

MI355X-native: every rank holds the whole (hashed, dense) model in HBM, so mixing is a
collective on dense tensors.

AVERAGE (:meth:`ModelMixer.average`) is a *shard mean*, not a ring all-reduce:

    all_to_all(flat)  ->  fp32 sum of the world's copies of my 1/world shard, one rounding
                      ->  all_gather(shard means)

* the wire carries the replica's storage dtype (bf16 state: half the bytes of an fp32 wire),
  yet the sum is formed in fp32 (``csrc/kernels/mix.hip``) — a bf16 ring all-reduce would
  round the partial sum at every hop;
* wire bytes per rank are 2(N-1)/N of the payload, the same as a ring all-reduce;
* the all-to-all sends to all N-1 peers at once: on a fully connected xGMI node that is all 7
  point-to-point links of a GPU busy together, where one ring uses two of them;
* every rank computes its shard's mean once and gathers the others, so all replicas are
  bit-identical after a mix (the order of the fp32 sum is fixed: rank 0..N-1).

Tensors are grouped by dtype into one flat, world-padded wire buffer per group (allocated once
per tensor list), so a model of five tensors costs two collectives per dtype, never a small
all-reduce per tensor.  Strided views (the V half of the packed FFM V|G table) are packed by one
strided copy.  What travels is the caller's choice: the learners mix the weights and keep the
AdaGrad accumulators local, as upstream; FFM also mixes the FTRL (z, n) of its linear term,
because its weight w is a function of (z, n) recomputed at every update (a mixed w alone would be
overwritten by the next local update).

ARGMIN_KLD = SUM all-reduce over [w/σ, 1/σ] -> w = Σ(w/σ)/Σ(1/σ), σ = 1/Σ(1/σ) (fp32).
SUM (:meth:`ModelMixer.all_reduce_sum`, histograms / counters) widens bf16/fp16 to fp32.
"""
from __future__ import annotations

import time
import weakref

import torch
import torch.distributed as dist

from .. import _native
from .dist import DistContext, context

_native.register_hip("hm_mix_shard_mean", [_native.c_p, _native.c_int, _native.c_i64,
                                           _native.c_int, _native.c_p, _native.c_p])
_native.register_hip("hm_mix_pack3", [_native.c_p, _native.c_p, _native.c_i64, _native.c_int, _native.c_int,
                                      _native.c_i64, _native.c_i64, _native.c_int, _native.c_p])
_native.register_hip("hm_mix_merge3", [_native.c_p, _native.c_p, _native.c_p, _native.c_p, _native.c_i64,
                                       _native.c_int, _native.c_int, _native.c_i64, _native.c_i64, _native.c_int,
                                       _native.c_p])
_native.register_hip("hm_mix_unpack3", [_native.c_p, _native.c_p, _native.c_i64, _native.c_int, _native.c_int,
                                        _native.c_i64, _native.c_i64, _native.c_int, _native.c_p])
_native.register_hip("hm_mix_merge", [_native.c_p, _native.c_p, _native.c_p, _native.c_i64,
                                      _native.c_int, _native.c_i64, _native.c_int, _native.c_p])
_native.register_hip("hm_mix_delta3", [_native.c_p, _native.c_p, _native.c_p, _native.c_p, _native.c_i64,
                                       _native.c_int, _native.c_int, _native.c_i64, _native.c_i64, _native.c_int,
                                       _native.c_int, _native.c_int, _native.c_p])

# fused delta passes (csrc/kernels/mix.hip hm_mix_delta3); 0 = the torch formulation (A/B, tests)
_FUSED_DELTA = True

_LOWP = (torch.bfloat16, torch.float16)


def _dtype_code(dt: torch.dtype) -> int | None:
    return {torch.float32: 0, torch.bfloat16: 1}.get(dt)


def _row_view(t: torch.Tensor):
    """(rows, inner, row_stride) when ``t`` is rows of ``inner`` contiguous elements at a uniform
    stride (contiguous tensors and the packed V half), else None."""
    if t.is_contiguous():
        return (t.numel() // 4, 4, 4) if t.numel() % 4 == 0 else None
    if t.dim() < 2 or t.stride(-1) != 1:
        return None
    for i in range(t.dim() - 2):
        if t.stride(i) != t.shape[i + 1] * t.stride(i + 1):
            return None
    rows = t.numel() // t.shape[-1]
    inner, rs = t.shape[-1], t.stride(-2)
    if inner % 4 or rs % 4:
        return None
    return rows, inner, rs


def _view3(t: torch.Tensor):
    """(n0, d1, inner, s0, s1) when ``t`` is an [n0][d1][inner] view with strides (s0, s1, 1)
    and inner % 4 == 0 (contiguous tensors, row views, and the V part of the per-slot FFM
    feature blocks), else None."""
    if t.is_contiguous():
        return (t.numel() // 4, 1, 4, 4, 4) if t.numel() % 4 == 0 else None
    if t.stride(-1) != 1 or t.shape[-1] % 4:
        return None
    if t.dim() == 2:
        return (t.shape[0], 1, t.shape[1], t.stride(0), t.shape[1])
    if t.dim() == 3:
        return (t.shape[0], t.shape[1], t.shape[2], t.stride(0), t.stride(1))
    return None


def _shard_mean(recv: torch.Tensor, world: int, shard: int, dtype: torch.dtype, out: torch.Tensor) -> None:
    """out <- fp32 sum over ranks 0..world-1 of recv[r] / world, one rounding (recv [world, shard])."""
    code = _dtype_code(dtype)
    if recv.is_cuda and code is not None and shard % 4 == 0:
        rc = _native.hip().hm_mix_shard_mean(recv.data_ptr(), world, shard, code, out.data_ptr(),
                                             _native.stream_of(recv.device))
        _native.check(rc, "hm_mix_shard_mean")
    else:
        s = recv.view(world, shard).sum(0, dtype=torch.float32)
        out.copy_(s.mul_(1.0 / world))


class _FlatGroup:
    """Same-dtype tensors packed into one flat wire buffer, padded to a multiple of 4*world."""

    def __init__(self, tensors: list[torch.Tensor], world: int, wire: torch.dtype | None = None):
        # weak references: a cached plan must not keep a discarded model alive in HBM
        self._refs = [weakref.ref(t) for t in tensors]
        self.world = world
        self.shapes = [tuple(t.shape) for t in tensors]
        self.busy = False            # an OverlappedMixer collective is in flight on the buffers
        self.prepacked = False       # send already holds the current snapshot (fused merge)
        self.base: torch.Tensor | None = None   # fp32 consensus of the last mix (delta modes)
        self.dtype = wire if wire is not None else tensors[0].dtype     # the wire's dtype
        dev = tensors[0].device
        self.offs = []
        off = 0
        for t in tensors:
            self.offs.append(off)
            off += (t.numel() + 3) // 4 * 4          # 16-B / 8-B aligned segments
        q = 4 * world
        self.n = (off + q - 1) // q * q
        self.shard = self.n // world
        self.send = torch.zeros(self.n, dtype=self.dtype, device=dev)   # = the snapshot
        self.recv = torch.empty(self.n, dtype=self.dtype, device=dev)
        self.mean = torch.empty(self.shard, dtype=self.dtype, device=dev)
        self.out = torch.empty(self.n, dtype=self.dtype, device=dev)
        self.nbytes = self.n * self.send.element_size()
        self.buf_bytes = 3 * self.nbytes + self.mean.numel() * self.mean.element_size()

    @property
    def tensors(self) -> list[torch.Tensor]:
        ts = [r() for r in self._refs]
        if any(t is None for t in ts):
            raise RuntimeError("mix plan: a mixed tensor was freed while its plan was in use")
        return ts

    def matches(self, tensors: list[torch.Tensor]) -> bool:
        return all(r() is t for r, t in zip(self._refs, tensors))

    def seg(self, buf: torch.Tensor, k: int) -> torch.Tensor:
        n = 1
        for d in self.shapes[k]:
            n *= d
        return buf[self.offs[k]:self.offs[k] + n].view(self.shapes[k])

    def pack(self) -> None:
        if self.prepacked:           # the previous merge already wrote this snapshot
            self.prepacked = False
            return
        code = _dtype_code(self.dtype)
        for k, t in enumerate(self.tensors):
            d = self.seg(self.send, k)
            v3 = _view3(t) if t.is_cuda and code is not None else None
            if v3 is not None:
                rc = _native.hip().hm_mix_pack3(t.data_ptr(), d.data_ptr(), *v3, code,
                                                _native.stream_of(t.device))
                _native.check(rc, "hm_mix_pack3")
            else:
                d.copy_(t)

    def unpack(self) -> None:
        """x <- out for every tensor (fused view kernel where the view allows, bit-exact)."""
        ts = self.tensors
        self.merge_rows([(k, 0, self.rows_of(k, t)[0]) for k, t in enumerate(ts) if t.numel()], delta=False)

    def _delta3(self, k: int, t: torch.Tensor, mode: int) -> bool:
        """One fused delta pass over tensor k (hm_mix_delta3); False when it does not apply."""
        xc, wc = _dtype_code(t.dtype), _dtype_code(self.dtype)
        v3 = _view3(t) if (_FUSED_DELTA and t.is_cuda and xc is not None and wc is not None) else None
        if v3 is None:
            return False
        b = self.seg(self.base, k)
        wire = self.seg(self.send if mode == 2 else self.out, k)
        sent = self.seg(self.send, k) if mode == 4 else None
        rc = _native.hip().hm_mix_delta3(t.data_ptr(), b.data_ptr(), wire.data_ptr(),
                                         sent.data_ptr() if sent is not None else None, *v3, mode, xc, wc,
                                         _native.stream_of(t.device))
        _native.check(rc, "hm_mix_delta3")
        return True

    # ---- row ranges (the bucketed pipeline of ModelMixer.average / average_delta) ----
    def rows_of(self, k: int, t: torch.Tensor) -> tuple[int, int]:
        """(rows, elements per row) of tensor k: the n0 rows of its _view3 (one feature's slots of
        the FFM V view, one 4-element quad of a contiguous tensor), else one row."""
        v3 = _view3(t)
        n = t.numel()
        if v3 is not None and n:
            return v3[0], v3[1] * v3[2]
        return 1, n

    def sub(self, t: torch.Tensor, ra: int, rb: int, rl: int) -> torch.Tensor:
        """Rows [ra, rb) of tensor t (rl elements per row) as a view of t."""
        if rb - ra == t.numel() // max(1, rl) and ra == 0:
            return t
        if t.is_contiguous():
            return t.view(-1)[ra * rl:rb * rl]
        return t[ra:rb]

    def flat(self, buf: torch.Tensor, k: int, ra: int, rb: int, rl: int) -> torch.Tensor:
        return buf[self.offs[k] + ra * rl:self.offs[k] + rb * rl]

    def buckets(self, elems: int) -> list[tuple[int, int, list, list]]:
        """Contiguous buckets of the flat wire buffer, each a multiple of 4 * world elements and
        about ``elems`` long: (lo, hi, pack_rows, merge_rows), the row ranges per tensor as
        (k, ra, rb).  A bucket packs every row that has an element in [lo, hi) (a row straddling
        two buckets is packed by both: the pack is idempotent while x and base are unchanged) and
        merges the rows whose LAST element is in [lo, hi) — every element of those is in this or
        an earlier bucket, so its mean has arrived; each row is merged exactly once."""
        q = 4 * self.world
        step = max(q, (int(elems) // q) * q)
        ts = self.tensors
        spans = []
        for k, t in enumerate(ts):
            nr, rl = self.rows_of(k, t)
            spans.append((k, self.offs[k], nr, rl))
        out = []
        for lo in range(0, self.n, step):
            hi = min(self.n, lo + step)
            pk, mg = [], []
            for k, off, nr, rl in spans:
                if rl == 0 or nr == 0:
                    continue
                a, b = off, off + nr * rl                    # tensor k's flat range
                if b <= lo or a >= hi:
                    continue
                ra = max(0, (lo - a) // rl)
                rb = min(nr, -(-(hi - a) // rl))
                pk.append((k, ra, rb))
                # rows whose last element a + (r + 1) rl - 1 lies in [lo, hi)
                ma = max(0, -((a - lo - 1) // rl) - 1)      # ceil((lo - a + 1) / rl) - 1
                mb = min(nr, (hi - a) // rl)
                if mb > ma:
                    mg.append((k, ma, mb))
            out.append((lo, hi, pk, mg))
        return out

    def pack_rows(self, rows, delta: bool) -> None:
        """pack (delta: send <- x - base; else send <- x) over the given row ranges."""
        code = _dtype_code(self.dtype)
        ts = self.tensors
        for k, ra, rb in rows:
            t = ts[k]
            nr, rl = self.rows_of(k, t)
            x = self.sub(t, ra, rb, rl)
            d = self.flat(self.send, k, ra, rb, rl)
            if delta:
                if self._delta3_rows(k, t, 2, ra, rb, rl):
                    continue
                d.copy_(x.reshape(-1).to(torch.float32) - self.flat(self.base, k, ra, rb, rl))
                continue
            v3 = _view3(x) if x.is_cuda and code is not None else None
            if v3 is not None:
                rc = _native.hip().hm_mix_pack3(x.data_ptr(), d.data_ptr(), *v3, code,
                                                _native.stream_of(x.device))
                _native.check(rc, "hm_mix_pack3")
            else:
                d.copy_(x.reshape(-1))

    def merge_rows(self, rows, delta: bool) -> None:
        """delta: base <- base + m, x <- base; else x <- out; over the given row ranges."""
        ts = self.tensors
        for k, ra, rb in rows:
            t = ts[k]
            nr, rl = self.rows_of(k, t)
            x = self.sub(t, ra, rb, rl)
            m = self.flat(self.out, k, ra, rb, rl)
            if delta:
                if self._delta3_rows(k, t, 3, ra, rb, rl):
                    continue
                b = self.flat(self.base, k, ra, rb, rl)
                b.add_(m.to(torch.float32))
                x.copy_(b.view(x.shape))
            else:
                code = _dtype_code(self.dtype)
                v3 = _view3(x) if x.is_cuda and code is not None and x.dtype == self.dtype else None
                if v3 is not None:
                    rc = _native.hip().hm_mix_unpack3(x.data_ptr(), m.data_ptr(), *v3, code,
                                                      _native.stream_of(x.device))
                    _native.check(rc, "hm_mix_unpack3")
                else:
                    x.copy_(m.view(x.shape))

    def _delta3_rows(self, k: int, t: torch.Tensor, mode: int, ra: int, rb: int, rl: int) -> bool:
        xc, wc = _dtype_code(t.dtype), _dtype_code(self.dtype)
        v3 = _view3(t) if (_FUSED_DELTA and t.is_cuda and xc is not None and wc is not None) else None
        if v3 is None:
            return False
        n0, d1, inner, s0, s1 = v3
        es = t.element_size()
        b = self.flat(self.base, k, ra, rb, rl)
        wire = self.flat(self.send if mode == 2 else self.out, k, ra, rb, rl)
        rc = _native.hip().hm_mix_delta3(t.data_ptr() + ra * s0 * es, b.data_ptr(), wire.data_ptr(), None,
                                         rb - ra, d1, inner, s0, s1, mode, xc, wc,
                                         _native.stream_of(t.device))
        _native.check(rc, "hm_mix_delta3")
        return True

    def pack_delta(self) -> None:
        """send <- x - base (the local progress since the last consensus), in the wire dtype."""
        for k, t in enumerate(self.tensors):
            if self._delta3(k, t, 2):
                continue
            d = self.seg(self.send, k)
            d.copy_(t.to(torch.float32) - self.seg(self.base, k))

    def merge_delta(self) -> None:
        """Delta merge: ``out`` holds the consensus step m (per element), so
        base <- base + m (rounded to the storage dtype, identically on every rank) and x keeps
        its progress since the snapshot: x <- x + m - delta_local."""
        for k, t in enumerate(self.tensors):
            if self._delta3(k, t, 4):
                continue
            m = self.seg(self.out, k).to(torch.float32)
            b = self.seg(self.base, k)
            b.add_(m)
            if t.dtype != torch.float32:
                b.copy_(b.to(t.dtype))               # exactly representable: untouched x == base
            t.copy_(t.to(torch.float32) + (m - self.seg(self.send, k).to(torch.float32)))

    def merge_delta_sync(self) -> None:
        """Synchronous delta merge (:meth:`ModelMixer.average_delta`): base <- base + m and
        x <- base."""
        for k, t in enumerate(self.tensors):
            if self._delta3(k, t, 3):
                continue
            b = self.seg(self.base, k)
            b.add_(self.seg(self.out, k).to(torch.float32))
            t.copy_(b)

    def shard_mean(self, world: int, changers: bool = False) -> None:
        """mean = fp32 sum over ranks of recv[r] / world, rounded once to the wire dtype.
        ``changers``: divide by the number of ranks whose value is non-zero instead (the mean of
        the deltas of the ranks that updated the element; 0 where none did)."""
        code = _dtype_code(self.dtype)
        if changers:
            r = self.recv.view(world, self.shard).to(torch.float32)
            cnt = (r != 0).sum(0).clamp_min_(1).to(torch.float32)
            self.mean.copy_(r.sum(0) / cnt)
            return
        if self.recv.is_cuda and code is not None:
            rc = _native.hip().hm_mix_shard_mean(self.recv.data_ptr(), world, self.shard, code,
                                                 self.mean.data_ptr(),
                                                 _native.stream_of(self.recv.device))
            _native.check(rc, "hm_mix_shard_mean")
        else:
            s = self.recv.view(world, self.shard).sum(0, dtype=torch.float32)
            self.mean.copy_(s.mul_(1.0 / world))

    def merge(self, repack: bool = False) -> None:
        """t <- t + (mean - snapshot), fp32 math, one rounding (overlapped mixing).
        ``repack``: also write the merged t into the snapshot buffer, in the same pass — the
        next mix's pack (its ``pack()`` is then skipped)."""
        code = _dtype_code(self.dtype)
        fused = repack and all(t.is_cuda and code is not None and _view3(t) is not None
                               for t in self.tensors)
        for k, t in enumerate(self.tensors):
            m, s = self.seg(self.out, k), self.seg(self.send, k)
            v3 = _view3(t) if t.is_cuda and code is not None else None
            if v3 is not None:
                rc = _native.hip().hm_mix_merge3(t.data_ptr(), m.data_ptr(), s.data_ptr(),
                                                 s.data_ptr() if fused else None, *v3, code,
                                                 _native.stream_of(t.device))
                _native.check(rc, "hm_mix_merge3")
                continue
            rv = _row_view(t) if t.is_cuda else None
            if rv is not None and code is not None and t.data_ptr() % 16 == 0:
                rows, inner, rs = rv
                rc = _native.hip().hm_mix_merge(t.data_ptr(), m.data_ptr(), s.data_ptr(), rows,
                                                inner, rs, code, _native.stream_of(t.device))
                _native.check(rc, "hm_mix_merge")
            else:
                t.copy_(t.to(torch.float32) + (m.to(torch.float32) - s.to(torch.float32)))
        self.prepacked = fused


class ModelMixer:
    # cached shard-mean plans: at most this many, holding at most this many buffer bytes
    MAX_PLANS = 4
    MAX_PLAN_BYTES = 16 << 30

    def __init__(self, ctx: DistContext | None = None, bucket_mb: float = 64.0,
                 small_bytes: int = 4 << 20, wire_dtype: torch.dtype | None = None,
                 min_world: int = 2):
        self.ctx = ctx or context()
        # min_world = 1: run the collectives even in a one-rank process group (the RCCL smoke
        # test drives the real all_to_all / all_gather / all_reduce calls on one GPU)
        self.min_world = int(min_world)
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.small_bytes = small_bytes
        self.wire_dtype = wire_dtype
        self.bytes_reduced = 0       # payload bytes mixed (sum over calls)
        self.wire_bytes = 0          # bytes this rank sent over the fabric (sum over calls)
        self.calls = 0
        self._plans: dict = {}

    @property
    def world(self) -> int:
        return self.ctx.world_size

    def _active(self) -> bool:
        if self.world > 1:
            return self.ctx.is_dist
        return self.min_world <= 1 and dist.is_available() and dist.is_initialized()

    # ---------------------------------------------------------------- shard-mean plan
    def plan(self, tensors: list[torch.Tensor]) -> list[_FlatGroup]:
        """Flat wire groups for this exact tensor list (cached by identity and shape).

        The cache holds at most ``MAX_PLANS`` plans and ``MAX_PLAN_BYTES`` of wire buffers (3x
        the mixed bytes each); the oldest idle plan is evicted first, and a plan whose
        overlapped collective is still in flight is never evicted.  Plans refer to the model
        tensors weakly: a freed model's plan is dropped, never matched by a new model that
        happens to reuse its addresses."""
        key = tuple((t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype) for t in tensors)
        p = self._plans.get(key)
        if p is not None and not all(g.matches([t for t in tensors if t.dtype == g.dtype])
                                     for g in p):
            del self._plans[key]
            p = None
        if p is None:
            by_dt: dict = {}
            for t in tensors:
                by_dt.setdefault(t.dtype, []).append(t)
            p = [_FlatGroup(ts, self.world) for ts in by_dt.values()]
            self._plans[key] = p
            self._evict(keep=key)
        return p

    def _plan_bytes(self) -> int:
        return sum(g.buf_bytes for p in self._plans.values() for g in p)

    def _evict(self, keep) -> None:
        for k in list(self._plans):
            if len(self._plans) <= self.MAX_PLANS and self._plan_bytes() <= self.MAX_PLAN_BYTES:
                break
            if k != keep and not any(g.busy for g in self._plans[k]):
                del self._plans[k]

    def release(self) -> None:
        """Drop every idle cached plan (frees its wire buffers)."""
        for k in list(self._plans):
            if not any(g.busy for g in self._plans[k]):
                del self._plans[k]

    def _count(self, groups: list[_FlatGroup], tensors) -> None:
        self.calls += 1
        self.bytes_reduced += sum(t.numel() * t.element_size() for t in tensors)
        self.wire_bytes += sum(2 * (self.world - 1) * g.nbytes // self.world for g in groups)

    def _a2a(self, g: _FlatGroup, async_op: bool = False):
        return dist.all_to_all_single(g.recv, g.send, async_op=async_op)

    def _gather(self, g: _FlatGroup, async_op: bool = False):
        return dist.all_gather_into_tensor(g.out, g.mean, async_op=async_op)

    # wire bytes per bucket of the pipelined shard mean (SURVEY.md:739-742: 32-128 MB buckets; on
    # one card, where the collectives are device copies, 64 MB cost 1.81 vs 1.68 ms monolithic per
    # fp32 delta mix and 32 MB 2.08: per-bucket launches, profiles/r6/mix_pipe_probe.jsonl);
    # 0 = one monolithic collective pair per dtype group (A/B, tests)
    PIPE_BUCKET_MB = 64.0

    def _pipelined(self, g: _FlatGroup, delta: bool) -> None:
        """Bucketed, software-pipelined shard mean of one flat group: bucket b+1's pack (compute
        stream) and its all-to-all (the RCCL stream) are issued before bucket b's shard mean and
        all-gather, and bucket b-1's merge runs while bucket b's gather is in flight, so at most
        one bucket's device work is exposed next to the wire.  Every element's mean is the same
        fp32 sum over ranks 0..N-1 as in the monolithic path, rounded once: bit-identical."""
        elems = int(self.PIPE_BUCKET_MB * (1 << 20)) // g.send.element_size()
        bks = g.buckets(elems) if elems > 0 else []
        if len(bks) <= 1:
            (g.pack_delta if delta else g.pack)()
            self._a2a(g)
            g.shard_mean(self.world)
            self._gather(g)
            (g.merge_delta_sync if delta else g.unpack)()
            return
        W = self.world
        views = []
        for lo, hi, pk, mg in bks:
            sh = (hi - lo) // W
            views.append((g.send[lo:hi], g.recv[lo:hi], g.out[lo:hi], sh))
        # two bucket-sized shard-mean buffers, alternating: bucket b + 2's mean overwrites bucket
        # b's only after bucket b's gather was waited on (the wait orders the compute stream after it)
        mbuf = getattr(g, "mbuf", None)
        if mbuf is None or mbuf[0].numel() < views[0][3]:
            mbuf = g.mbuf = [torch.empty(views[0][3], dtype=g.dtype, device=g.send.device) for _ in range(2)]
        a2a, gat = [None] * len(bks), [None] * len(bks)

        def start(b):
            g.pack_rows(bks[b][2], delta)
            a2a[b] = dist.all_to_all_single(views[b][1], views[b][0], async_op=True)

        start(0)
        for b in range(len(bks)):
            if b + 1 < len(bks):
                start(b + 1)
            a2a[b].wait()
            _, r, o, sh = views[b]
            mb = mbuf[b & 1][:sh]
            _shard_mean(r, W, sh, g.dtype, mb)
            gat[b] = dist.all_gather_into_tensor(o, mb, async_op=True)
            if b >= 1:
                gat[b - 1].wait()
                g.merge_rows(bks[b - 1][3], delta)
        gat[-1].wait()
        g.merge_rows(bks[-1][3], delta)

    def average(self, tensors: list[torch.Tensor]) -> None:
        """In-place replica mean (shard-mean collective, see the module docstring), bucketed and
        pipelined (:meth:`_pipelined`)."""
        if not self._active():
            return
        groups = self.plan(tensors)
        for g in groups:
            if g.prepacked:          # an overlapped mix left a snapshot: repack from x
                g.prepacked = False
            self._pipelined(g, delta=False)
        self._count(groups, tensors)

    # ---------------------------------------------------------------- mean of deltas, bf16 wire
    def average_delta(self, tensors: list[torch.Tensor], wire: torch.dtype = torch.bfloat16) -> None:
        """In-place replica mean with half the wire bytes for fp32 replicas: every rank keeps the
        fp32 consensus ``base`` of the last mix and sends ``x - base`` (the progress since then)
        in ``wire`` (bf16); the shard mean of the deltas is summed in fp32 (csrc/kernels/mix.hip)
        and gathered in ``wire``; every rank then sets ``x = base = base + mean_delta`` — the same
        fp32 value everywhere.  Only the step since the last mix is rounded (a relative 2^-9 of
        the step, not of the weight).  The first call (no consensus yet) is a full-precision
        :meth:`average`, which also seeds ``base``."""
        if not self._active():
            return
        key = ("delta", wire) + tuple((t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype) for t in tensors)
        p = self._plans.get(key)
        g = p[0] if p is not None else None
        if g is not None and not g.matches(tensors):
            del self._plans[key]
            g = None
        if g is None:
            self.average(tensors)
            g = _FlatGroup(tensors, self.world, wire=wire)
            g.base = torch.empty(g.n, dtype=torch.float32, device=tensors[0].device)
            g.buf_bytes += g.n * 4
            for k, t in enumerate(g.tensors):
                g.seg(g.base, k).copy_(t)
            self._plans[key] = [g]
            self._evict(keep=key)
            return
        # per bucket: send <- x - base; all-to-all; fp32 shard mean; all-gather; base <- base +
        # mean delta, x <- base (fused passes per tensor row range, pipelined over the buckets)
        self._pipelined(g, delta=True)
        self.calls += 1
        self.bytes_reduced += sum(t.numel() * t.element_size() for t in tensors)
        self.wire_bytes += 2 * (self.world - 1) * g.nbytes // self.world

    # ---------------------------------------------------------------- collective timing
    def time_collectives(self, on: bool = True) -> None:
        """Start (or stop) timing the sum all-reduces: events on the caller's stream bracket each
        call, from its first enqueue to the point the stream may use the result, so the total is
        the time the computation waits on the fabric (no host sync per call)."""
        self._timings = [] if on else None

    def collective_ms(self) -> float:
        """Milliseconds the timed sum all-reduces held the computation (time_collectives)."""
        total = 0.0
        for a, b in getattr(self, "_timings", None) or []:
            if isinstance(a, float):
                total += (b - a) * 1e3
            else:
                b.synchronize()
                total += a.elapsed_time(b)
        return total

    def _time_start(self, t: torch.Tensor):
        if getattr(self, "_timings", None) is None:
            return None
        if t.is_cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        import time
        return time.perf_counter()

    def _time_end(self, start) -> None:
        if start is None:
            return
        if isinstance(start, float):
            import time
            self._timings.append((start, time.perf_counter()))
        else:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._timings.append((start, e))

    # ---------------------------------------------------------------- sum all-reduce
    def all_reduce_sum(self, tensors: list[torch.Tensor]) -> None:
        """In-place SUM all-reduce of a list of tensors (bucketed, async).  bf16/fp16 tensors are
        summed in fp32 (an N-way sum rounded at every ring hop would lose their low bits)."""
        if not self._active():
            return
        ev = self._time_start(tensors[0])
        small = [t for t in tensors if t.numel() * t.element_size() <= self.small_bytes]
        big = [t for t in tensors if t.numel() * t.element_size() > self.small_bytes]
        works = []
        flat = None
        if small:
            flat = torch.cat([t.reshape(-1).to(torch.float32) for t in small])
            works.append(dist.all_reduce(flat, async_op=True))
        staged = []   # strided views and low-precision tensors go via an fp32/contiguous copy
        for t in big:
            buf = t
            if t.dtype in _LOWP:
                buf = t.to(torch.float32)
            elif not t.is_contiguous():
                buf = t.contiguous()
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
        self._time_end(ev)
        self.calls += 1
        nb = sum(t.numel() * t.element_size() for t in tensors)
        self.bytes_reduced += nb
        self.wire_bytes += 2 * (self.world - 1) * nb // self.world

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

    # ---------------------------------------------------------------- measurement
    def probe(self, tensors: list[torch.Tensor], reps: int = 3, fn=None) -> dict:
        """Time ``reps`` synchronous mixes of ``tensors`` by ``fn`` (default :meth:`average`;
        device events on the GPU, after a barrier); returns ms per mix, wire bytes per rank and
        bus GB/s (nccl-tests convention: 2(N-1)/N * payload / time).  The tensors are left mixed."""
        if not self._active() or reps <= 0:
            return {}
        fn = fn or self.average
        fn(tensors)                                # warm the communicators / buffers
        w1 = self.wire_bytes                       # (average_delta: the first call seeds it)
        fn(tensors)
        wire = self.wire_bytes - w1                # bytes one rank sends per mix
        if self.world > 1:
            payload = wire * self.world // (2 * (self.world - 1))
        else:                                      # one rank sends nothing: the mixed bytes
            payload = sum(t.numel() * (2 if fn == self.average_delta else t.element_size()) for t in tensors)
        self.ctx.barrier()
        cuda = tensors[0].is_cuda
        if cuda:
            torch.cuda.synchronize(tensors[0].device)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn(tensors)
        if cuda:
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / reps
        else:
            ms = 1000.0 * (time.perf_counter() - t0) / reps
        ms = self.all_reduce_scalar(ms, "max")
        return {"mix_ms": round(ms, 4), "mix_payload_bytes": int(payload),
                "mix_wire_bytes_per_rank": int(wire),
                "mix_bus_gbps": round(wire / (ms * 1e-3) / 1e9, 2) if ms > 0 else None,
                "mix_algo": "all_to_all + fp32 shard mean + all_gather" +
                            (" (bf16 deltas, fp32 consensus)" if fn == self.average_delta else "")}


class OverlappedMixer:
    """Stale-by-one model averaging whose collectives run behind the training kernels.

    ``start(tensors)`` snapshots the replicas into the flat wire buffers (one strided copy on the
    compute stream) and launches the shard-mean collective (all-to-all -> fp32 shard mean ->
    all-gather) on a side stream; training continues.  ``finish()`` (at the next mix point)
    makes the compute stream wait for the all-gather — on the device, not the host — and merges
    without discarding the local progress made in the meantime:

        x  <-  x + (mean_r(snapshot_r) - snapshot_local)

    i.e. every rank moves by the consensus correction of the snapshot.  This is the
    asynchronous MixServer semantics (replies arrive while the learner keeps training) on
    xGMI, and it hides the collective completely when one mix interval of compute takes longer
    than the collective.  The wire carries the storage dtype (bf16 V: half the bytes) and the
    sum is still exact fp32 (the shard mean).  Buffers: 3x the mixed bytes, allocated once.
    """

    def __init__(self, mixer: ModelMixer, mode: str = "mean", power: float = 1.0):
        if mode not in ("mean", "sum", "touched"):
            raise ValueError("OverlappedMixer mode: mean | sum | touched")
        self.m = mixer
        self.mode = mode
        self.power = power           # sum mode: consensus step = mean_r(delta_r) * world**power
        self.groups: list[_FlatGroup] | None = None
        self.works: list = []
        self.side = None
        self._sum_now = False        # the in-flight mix is a delta-sum one

    def pending(self) -> bool:
        return bool(self.works)

    def start(self, tensors: list[torch.Tensor]) -> None:
        if not self.m._active():
            return
        groups = self.m.plan(tensors)
        if self.works:
            # mean mode, same tensors: the merge also writes the next snapshot (one pass less)
            self.finish(repack=self.mode == "mean" and groups is self.groups)
        self.groups = groups
        # delta-sum mode needs a consensus to measure deltas from: the first mix is a mean
        self._sum_now = self.mode != "mean" and all(g.base is not None for g in self.groups)
        for g in self.groups:
            if self._sum_now:
                g.pack_delta()                       # this rank's progress since the consensus
            else:
                g.pack()                             # the snapshot (exact copy of the replica)
            g.busy = True
        world = self.m.world
        if tensors[0].is_cuda:
            if self.side is None:
                self.side = torch.cuda.Stream(device=tensors[0].device)
            self.side.wait_stream(torch.cuda.current_stream(tensors[0].device))
            with torch.cuda.stream(self.side):
                for g in self.groups:
                    self.m._a2a(g, async_op=True).wait()    # side stream waits, host does not
                    self._reduce(g, world)
                    self.works.append(self.m._gather(g, async_op=True))
        else:
            # gloo: the shard mean needs the all-to-all's data on the host, so the first half
            # runs synchronously; the all-gather stays in flight behind the caller's compute
            for g in self.groups:
                self.m._a2a(g)
                self._reduce(g, world)
                self.works.append(self.m._gather(g, async_op=True))
        self.m._count(self.groups, tensors)

    def _reduce(self, g: _FlatGroup, world: int) -> None:
        if not self._sum_now:
            g.shard_mean(world)
        elif self.mode == "touched":
            g.shard_mean(world, changers=True)
        else:
            g.shard_mean(world)
            g.mean.mul_(float(world) ** self.power)

    def finish(self, repack: bool = False) -> None:
        if not self.works:
            return
        for w in self.works:
            w.wait()
        self.works = []
        for g in self.groups:
            if self._sum_now:
                g.merge_delta()
            else:
                g.merge(repack)
                if self.mode != "mean":              # the first consensus: deltas start here
                    g.base = g.out.to(torch.float32, copy=True)
            g.busy = False


class SparseDeltaMixer:
    """Touched-row model averaging: all-gather of (row index, Δrow) instead of a dense
    all-reduce (SURVEY.md §5.8 "sparse alternative"; upstream's MixClient likewise only pushes
    the features a learner updated, reference hivemall/mix/client/MixClient.java).

    Every rank keeps ``base`` = the last mixed model (as stored: a bf16 replica's base is the
    bf16 value widened, so untouched rows compare equal).  Rows that a rank did not touch since
    then equal ``base`` on that rank, so the replica mean is exactly

        mean_r(x_r) = base + Σ_r Δ_r / world,   Δ_r = x_r - base  (non-zero on touched rows only)

    ``mix(tensors)`` finds the touched rows of dim 0 (any element changed), all-gathers their
    counts, then the padded (index, Δ) payloads, scatter-adds them into ``base`` (index_add_,
    fp32) and copies the result back — bit-for-bit the dense average up to summation order.
    Wire bytes per rank are ``world · touched · (row_bytes + 8)`` against ``≈2 · rows ·
    row_bytes`` for a ring all-reduce, so when the touched fraction exceeds ``dense_fraction``
    (default ``1 / world``) the step falls back to the dense shard mean of
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
                b.copy_(t.to(torch.float32))
                continue
            rows = t.shape[0]
            if maxc[k] == 0:
                t.copy_(b)
                continue
            if maxc[k] > frac * rows:
                self.m.average([t])
                b.copy_(t.to(torch.float32))
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
            if t.dtype != torch.float32:
                # the replica now holds base rounded to its dtype: keep base equal to what is
                # stored, or every mixed row would look touched at the next mix
                b.copy_(t.to(torch.float32))
            self.sparse_rows += int(allc[:, k].sum())
            self.m.bytes_reduced += n * world * (delta[0].numel() * 4 + 8)
            self.m.wire_bytes += n * (world - 1) * (delta[0].numel() * 4 + 8)
        self.m.calls += 1
