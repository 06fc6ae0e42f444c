"""Device-side ingest: Arrow ``list<string>`` feature columns -> device batches.

SURVEY.md §2.5 K1 / §3.2 (string -> hash -> CSR on the device) and §1 N1 (pinned host -> HBM
staging).  An Arrow list<string> column already holds exactly what the parse kernels need —
one UTF-8 byte buffer, int offsets per string, int offsets per row — so a batch is uploaded as
those three buffers (no per-string Python work) and parsed by ``csrc/kernels/ingest.hip``
where the model lives:

* rows are processed in chunks; each chunk's buffers are copied into one of two pinned staging
  slots and sent H2D on a copy stream, while the parse kernel of the previous chunk runs on the
  compute stream (double buffering: the copy of chunk k+1 overlaps the parse of chunk k);
* a chunk the device cannot parse exactly (malformed strings, values outside the exact decimal
  fast path) is re-parsed by the host parser, which also raises its usual error;
* Python lists of strings are first converted by ``pyarrow.array`` (C++), never joined in
  Python.

``IngestStats`` reports bytes, chunks, host/device seconds; ``HM_INGEST_HOST=1`` forces the host
parser (A/B).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import _native

_native.register_hip("hm_ffm_parse", [_native.c_p, _native.c_p, _native.c_p, _native.c_i64, _native.c_int,
                                      _native.c_i32, _native.c_i32, _native.c_int, _native.c_u32,
                                      _native.c_p, _native.c_p, _native.c_p, _native.c_p, _native.c_p])
_native.register_hip("hm_feat_parse", [_native.c_p, _native.c_p, _native.c_i64, _native.c_int, _native.c_i32,
                                       _native.c_u32, _native.c_p, _native.c_p, _native.c_p, _native.c_p])
_native.register_hip("hm_feat_parse32", [_native.c_p, _native.c_p, _native.c_i64, _native.c_int, _native.c_i32,
                                         _native.c_u32, _native.c_p, _native.c_p, _native.c_p, _native.c_p])

NO_ERR = (1 << 64) - 1
DEFAULT_SEED = 0x9747b28c


@dataclass
class IngestStats:
    rows: int = 0
    strings: int = 0
    bytes: int = 0
    chunks: int = 0
    host_fallback_chunks: int = 0
    refused: list = field(default_factory=list)   # first string the device refused, per chunk
    host_s: float = 0.0          # arrow conversion + staging copies on the host
    wall_s: float = 0.0          # whole ingest (host + H2D + parse), synchronised
    events: list = field(default_factory=list)

    def as_dict(self) -> dict:
        return {k: (round(v, 4) if isinstance(v, float) else v) for k, v in self.__dict__.items()
                if k not in ("events", "refused")}


LAST_STATS = IngestStats()


def is_arrow_like(x) -> bool:
    try:
        import pyarrow as pa
    except ImportError:  # pragma: no cover
        return False
    if isinstance(x, (pa.Array, pa.ChunkedArray)):
        return True
    import pandas as pd

    return isinstance(x, pd.Series) and isinstance(x.dtype, pd.ArrowDtype)


def to_arrow_lists(x):
    """Arrow list<string> array (one chunk) from an Arrow array, an Arrow-backed pandas Series
    or Python lists of strings (converted in C++ by pyarrow)."""
    import pyarrow as pa
    import pandas as pd

    if isinstance(x, pd.Series):
        x = pa.array(x) if not isinstance(x.dtype, pd.ArrowDtype) else x.array._pa_array
    if isinstance(x, pa.ChunkedArray):
        x = x.combine_chunks() if x.num_chunks != 1 else x.chunk(0)
    if not isinstance(x, pa.Array):
        x = pa.array([[] if r is None else [str(v) for v in r] for r in x], type=pa.list_(pa.string())) \
            if not _all_str_lists(x) else pa.array(x, type=pa.list_(pa.string()))
    if not (pa.types.is_list(x.type) or pa.types.is_large_list(x.type)):
        raise TypeError(f"expected a list<string> column, got {x.type}")
    vt = x.type.value_type
    if not (pa.types.is_string(vt) or pa.types.is_large_string(vt)):
        x = x.cast(pa.list_(pa.string()))
    return x


def _all_str_lists(rows) -> bool:
    for r in rows[:64] if hasattr(rows, "__getitem__") else []:
        if r is not None and any(not isinstance(v, str) for v in r):
            return False
    return True


def arrow_buffers(arr, wide: bool = True):
    """(data uint8 ndarray, string offsets [n+1], row offsets int64 [B+1]) of a list<string>
    array, rebased to start at 0 (slices honoured, zero-copy views where possible).  The string
    offsets are int64, or (``wide=False``) the column's own int32 offsets when it has them —
    a zero-copy view unless they need rebasing."""
    import pyarrow as pa

    lo = np.array(arr.offsets, dtype=np.int64)
    vals = arr.values.slice(int(lo[0]), int(lo[-1] - lo[0]))
    if lo[0]:
        lo -= lo[0]
    bufs = vals.buffers()
    odt = np.int64 if pa.types.is_large_string(vals.type) else np.int32
    if bufs[1] is None:
        so = np.zeros(1, np.int64)
    else:
        so = np.frombuffer(bufs[1], dtype=odt)[vals.offset:vals.offset + len(vals) + 1]
        if wide or odt == np.int64:
            so = so.astype(np.int64)
    buf = bufs[2]
    data = np.frombuffer(buf, dtype=np.uint8) if buf is not None else np.zeros(0, np.uint8)
    data = data[int(so[0]):int(so[-1])] if len(so) else data[:0]
    if len(so) and so[0]:
        so = so - so[0]
    return data, so, lo


_POOL = None


def _parallel_copy(jobs, piece: int = 16 << 20) -> None:
    """dst[:] = src for every (dst, src) byte-array pair, split into ``piece``-byte copies run by
    a small thread pool (numpy releases the GIL in the copy): the pinned staging of a chunk is
    a few hundred MB of memcpy, which one core does at ~10 GB/s."""
    global _POOL
    tasks = [(d[o:o + piece], s[o:o + piece]) for d, s in jobs for o in range(0, s.size, piece)]
    if len(tasks) <= 1:
        for d, s in tasks:
            np.copyto(d, s)
        return
    if _POOL is None:
        import concurrent.futures as cf

        _POOL = cf.ThreadPoolExecutor(max_workers=max(1, min(8, (os.cpu_count() or 2) // 2)))
    list(_POOL.map(lambda ds: np.copyto(ds[0], ds[1]), tasks))


class _Stager:
    """Two pinned host slots + a copy stream: stage(k) copies chunk k's buffers into slot k % 2
    and enqueues its H2D on the copy stream; the compute stream waits on that copy's event."""

    def __init__(self, device, cap_bytes: int):
        self.dev = device
        self.slots = [torch.empty(cap_bytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self.dbuf = [torch.empty(cap_bytes, dtype=torch.uint8, device=device) for _ in range(2)]
        self.done = [None, None]      # event: the slot's H2D finished (slot reusable)
        self.used = [None, None]      # event: the compute stream finished with the device buffer
        self.copy = torch.cuda.Stream(device=device)

    def stage(self, k: int, parts: list[np.ndarray]) -> list[torch.Tensor]:
        s = k % 2
        if self.done[s] is not None:
            self.done[s].synchronize()            # the pinned slot's previous copy has left
        if self.used[s] is not None:
            self.copy.wait_event(self.used[s])    # ... and its device buffer is no longer read
        host, dev = self.slots[s], self.dbuf[s]
        views, off = [], 0
        hn = host.numpy()
        jobs = []
        for a in parts:
            b = a.view(np.uint8).reshape(-1)
            jobs.append((hn[off:off + b.size], b))
            views.append((off, b.size, a.dtype, a.shape))
            off = (off + b.size + 15) // 16 * 16
        _parallel_copy(jobs)
        with torch.cuda.stream(self.copy):
            dev[:off].copy_(host[:off], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy)
        self.done[s] = ev
        torch.cuda.current_stream(self.dev).wait_event(ev)
        tdt = {np.dtype(np.uint8): torch.uint8, np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32}
        return [dev[o:o + n].view(tdt[np.dtype(dt)]).view(*shape) if n else
                torch.zeros(shape, dtype=tdt[np.dtype(dt)], device=self.dev) for o, n, dt, shape in views]

    def release(self, k: int) -> None:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        self.used[k % 2] = ev


def _chunks(lo: np.ndarray, so: np.ndarray, chunk_rows: int):
    B = len(lo) - 1
    chunks = [(r0, min(B, r0 + chunk_rows)) for r0 in range(0, B, chunk_rows)]
    cap = 0
    for r0, r1 in chunks:
        s0, s1 = int(lo[r0]), int(lo[r1])
        cap = max(cap, int(so[s1] - so[s0]) + 8 * (s1 - s0 + 1) + 8 * (r1 - r0 + 1) + 64)
    return chunks, cap


def _ingest(arr, chunk_rows: int, dev, launch, host_chunk, narrow: bool = False) -> IngestStats:
    """Stage every row chunk's (bytes, string offsets, row offsets) through the double-buffered
    pinned slots, ``launch(k, r0, r1, s0, d_data, d_so, d_lo, err_k)`` its parse kernel, then
    re-run the chunks the device refused through ``host_chunk(r0, r1)`` (one sync).
    ``narrow``: ``launch`` takes int32 string offsets, so an Arrow string column's own offsets
    travel as they are (half the offset bytes, no widening pass)."""
    st = IngestStats()
    t0 = time.perf_counter()
    data, so, lo = arrow_buffers(arr, wide=not narrow)
    B = len(lo) - 1
    st.rows, st.strings, st.bytes = B, len(so) - 1, int(data.size)
    chunks, cap = _chunks(lo, so, chunk_rows)
    force_host = os.environ.get("HM_INGEST_HOST", "0") == "1" or dev.type != "cuda"
    host_s = time.perf_counter() - t0
    if force_host:
        for r0, r1 in chunks:
            host_chunk(r0, r1)
            st.host_fallback_chunks += 1
    elif chunks:
        err = torch.full((len(chunks),), -1, dtype=torch.int64, device=dev)
        stager = _Stager(dev, cap)
        for k, (r0, r1) in enumerate(chunks):
            s0, s1 = int(lo[r0]), int(lo[r1])
            th = time.perf_counter()
            b0 = int(so[s0])
            sok = so[s0:s1 + 1] if b0 == 0 else so[s0:s1 + 1] - so.dtype.type(b0)
            d_data, d_so, d_lo = stager.stage(k, [data[b0:int(so[s1])], sok,
                                                  lo[r0:r1 + 1] if s0 == 0 else lo[r0:r1 + 1] - s0])
            host_s += time.perf_counter() - th
            launch(k, r0, r1, s0, d_data, d_so, d_lo, err[k:k + 1])
            stager.release(k)
            st.chunks += 1
        ev = err.tolist()                                        # the one sync of the ingest
        for k, e in enumerate(ev):
            if e == -1:
                continue
            si = int(lo[chunks[k][0]]) + (e if e >= 0 else e + (1 << 64))
            if len(st.refused) < 8 and 0 <= si < len(so) - 1:
                st.refused.append(bytes(data[int(so[si]):int(so[si + 1])]).decode("utf-8", "replace"))
            host_chunk(*chunks[k])
            st.host_fallback_chunks += 1
        torch.cuda.synchronize(dev)
    st.host_s = host_s
    st.wall_s = time.perf_counter() - t0
    global LAST_STATS
    LAST_STATS = st
    return st


def ffm_ell_device(features, num_features: int, num_fields: int, hash_ints: bool, width: int | None = None,
                   device="cuda", chunk_rows: int = 1 << 20, seed: int = DEFAULT_SEED):
    """Parse FFM rows ("field:index[:value]") into device ELL tensors (idx, fld, val) [B, F]
    (padding: idx -1, fld 0, val 0 — the layout ``csr_to_ffm_batch`` builds on the host)."""
    dev = torch.device(device)
    arr = to_arrow_lists(features)
    lo = np.asarray(arr.offsets, dtype=np.int64)
    B = len(lo) - 1
    F = max(1, int(width if width is not None else (np.diff(lo).max() if B else 1)))
    idx = torch.empty((B, F), dtype=torch.int32, device=dev)
    fld = torch.empty((B, F), dtype=torch.int32, device=dev)
    val = torch.empty((B, F), dtype=torch.float32, device=dev)

    def launch(k, r0, r1, s0, d_data, d_so, d_lo, e):
        rc = _native.hip().hm_ffm_parse(d_data.data_ptr(), d_so.data_ptr(), d_lo.data_ptr(), r1 - r0, F,
                                        int(num_features), int(num_fields), int(bool(hash_ints)), seed,
                                        fld[r0:r1].data_ptr(), idx[r0:r1].data_ptr(), val[r0:r1].data_ptr(),
                                        e.data_ptr(), _native.stream_of(dev))
        _native.check(rc, "hm_ffm_parse")

    def host_chunk(r0, r1):
        from ..utils.features import parse_ffm_rows

        csr = parse_ffm_rows(arr.slice(r0, r1 - r0).to_pylist(), num_features, num_fields,
                             hash_ints=hash_ints, seed=seed)
        i, v, f = csr.to_ell(F)
        for dst, src, dt in ((idx, i, np.int32), (fld, f, np.int32), (val, v, np.float32)):
            dst[r0:r1].copy_(torch.from_numpy(np.ascontiguousarray(src, dtype=dt)))

    st = _ingest(arr, chunk_rows, dev, launch, host_chunk)
    return idx, fld, val, st


def csr_device(features, mode: str, num_features: int = 0, device="cuda", chunk_rows: int = 1 << 20,
               seed: int = DEFAULT_SEED):
    """Parse ``name[:value]`` rows into device CSR (indptr int64 [B+1], idx int64 [nnz], val f32
    [nnz]).  mode "hash": idx = mhash(name, num_features) (1-based, FeatureEncoder("hash"));
    mode "int": integer names (FeatureEncoder("int"))."""
    from ..utils.features import FeatureEncoder

    m = {"int": 0, "hash": 2}[mode]
    dev = torch.device(device)
    arr = to_arrow_lists(features)
    lo = np.asarray(arr.offsets, dtype=np.int64)
    lo = lo - lo[0]
    nnz = int(lo[-1])
    idx = torch.empty(nnz, dtype=torch.int64, device=dev)
    val = torch.empty(nnz, dtype=torch.float32, device=dev)

    def launch(k, r0, r1, s0, d_data, d_so, d_lo, e):
        n = int(lo[r1] - lo[r0])
        fn = _native.hip().hm_feat_parse32 if d_so.dtype == torch.int32 else _native.hip().hm_feat_parse
        rc = fn(d_data.data_ptr(), d_so.data_ptr(), n, m, int(num_features), seed,
                idx[s0:].data_ptr(), val[s0:].data_ptr(), e.data_ptr(), _native.stream_of(dev))
        _native.check(rc, "hm_feat_parse")

    def host_chunk(r0, r1):
        enc = FeatureEncoder(mode, num_features=num_features or (1 << 24), seed=seed)
        csr = enc.encode(arr.slice(r0, r1 - r0).to_pylist())
        s0, s1 = int(lo[r0]), int(lo[r1])
        idx[s0:s1].copy_(torch.from_numpy(csr.idx.astype(np.int64)))
        val[s0:s1].copy_(torch.from_numpy(csr.val.astype(np.float32)))

    st = _ingest(arr, chunk_rows, dev, launch, host_chunk, narrow=True)
    return torch.from_numpy(lo).to(dev), idx, val, st


@dataclass
class DeviceFeatures:
    """A feature column that already lives on the device as CSR — what the SQL planner hands a
    learner for ``train_*(add_bias(feature_hashing(features)), ...)`` on a GPU session
    (sql/device_ftvec.py) instead of a column of hashed strings the learner would parse again.

    ``indptr`` int64 [B+1], ``idx`` int64 [nnz] (integer feature ids, as the learners' "int"
    encoder reads ``"id:value"`` strings), ``val`` f32 [nnz]."""
    indptr: torch.Tensor
    idx: torch.Tensor
    val: torch.Tensor
    stats: IngestStats | None = None

    def __len__(self) -> int:
        return self.indptr.numel() - 1

    def take_rows(self, rank: int, world: int) -> "DeviceFeatures":
        """Rows rank, rank + world, ... (a data-parallel rank's share), still on the device."""
        B = len(self)
        rows = torch.arange(rank, B, world, device=self.indptr.device)
        cnt = self.indptr[rows + 1] - self.indptr[rows]
        ip = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=self.indptr.device)
        ip[1:] = torch.cumsum(cnt, 0)
        pos = torch.repeat_interleave(self.indptr[rows], cnt) + \
            (torch.arange(int(ip[-1]), device=ip.device) - torch.repeat_interleave(ip[:-1], cnt))
        return DeviceFeatures(ip, self.idx[pos], self.val[pos])


def hashed_csr_device(features, num_features: int, bias: bool, device="cuda",
                      chunk_rows: int = 1 << 20, seed: int = DEFAULT_SEED) -> DeviceFeatures:
    """``[add_bias(]feature_hashing(features, '-num_features N')[)]`` evaluated on the device:
    the raw ``name[:value]`` strings go up as Arrow buffers, ``hm_feat_parse`` (mode 2) turns
    each into (mhash(name, N), value) — what ``feature_hashing`` writes as ``"h:value"`` and the
    learner's int encoder reads back — and the bias ``0:1.0`` is appended to every row on the
    device.  A chunk the device refuses (two-colon names, inexact decimals) goes through the host
    ``feature_hashing`` + int parse, so the result equals the string path bit for bit."""
    dev = torch.device(device)
    arr = to_arrow_lists(features)
    lo = np.asarray(arr.offsets, dtype=np.int64)
    lo = lo - lo[0]
    B, nnz = len(lo) - 1, int(lo[-1])
    idx = torch.empty(nnz, dtype=torch.int64, device=dev)
    val = torch.empty(nnz, dtype=torch.float32, device=dev)

    def launch(k, r0, r1, s0, d_data, d_so, d_lo, e):
        n = int(lo[r1] - lo[r0])
        fn = _native.hip().hm_feat_parse32 if d_so.dtype == torch.int32 else _native.hip().hm_feat_parse
        rc = fn(d_data.data_ptr(), d_so.data_ptr(), n, 2, int(num_features), seed,
                idx[s0:].data_ptr(), val[s0:].data_ptr(), e.data_ptr(), _native.stream_of(dev))
        _native.check(rc, "hm_feat_parse")

    def host_chunk(r0, r1):
        from ..ftvec.functions import feature_hashing
        from ..utils.features import FeatureEncoder

        rows = arr.slice(r0, r1 - r0).to_pylist()
        hashed = [feature_hashing(r, f"-num_features {int(num_features)}") if r is not None else [] for r in rows]
        csr = FeatureEncoder("int").encode(hashed)
        s0, s1 = int(lo[r0]), int(lo[r1])
        idx[s0:s1].copy_(torch.from_numpy(csr.idx.astype(np.int64)))
        val[s0:s1].copy_(torch.from_numpy(csr.val.astype(np.float32)))

    st = _ingest(arr, chunk_rows, dev, launch, host_chunk, narrow=True)
    ip = torch.from_numpy(lo).to(dev)
    if bias:
        # row r's entries shift by r; its bias lands in the new last slot of the row
        cnt = ip[1:] - ip[:-1]
        nip = ip + torch.arange(B + 1, dtype=torch.int64, device=dev)
        pos = torch.arange(nnz, dtype=torch.int64, device=dev) + \
            torch.repeat_interleave(torch.arange(B, dtype=torch.int64, device=dev), cnt, output_size=nnz)
        bidx = torch.zeros(nnz + B, dtype=torch.int64, device=dev)
        bval = torch.ones(nnz + B, dtype=torch.float32, device=dev)
        bidx[pos] = idx
        bval[pos] = val
        ip, idx, val = nip, bidx, bval
    return DeviceFeatures(ip, idx, val, st)
