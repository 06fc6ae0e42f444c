"""Row-sharded model tables across ranks (SURVEY.md §2.4 "Sharded parameter server": upstream's
MixRequestRouter hashes a feature to a MixServer shard; here a row lives in the HBM of one rank).

A ``ShardedTable`` of ``n_rows x dim`` keeps global row ``r`` on rank ``r % world`` (local row
``r // world``), so each GPU holds 1/world of a table that may not fit one GPU.  A training step
is *pull -> compute -> push*:

* ``pull(ids)``   — the rows a batch touches (unique ids) are routed to their owners with one
  ``all_to_all_single`` of ids and one of rows back (RCCL over xGMI; gloo on CPU);
* the learner runs its normal kernel on the compact gathered table (ids remapped to 0..U-1);
* ``push_add(ids, delta)`` — the changes (new - pulled) travel back to the owners, which add
  them: concurrent pushes of one row from several ranks all land (Hogwild across ranks with
  no lost update, like the MixServer summing its clients' deltas).

Every rank must call ``pull`` / ``push_add`` the same number of times (collectives);
``steps_agreed`` helps loops with rank-dependent batch counts.  ``full()`` all-gathers the
table (model-table export).  World size 1 degenerates to plain indexing.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class ShardedTable:
    def __init__(self, n_rows: int, dim: int, ctx=None, dtype=torch.float32, device=None,
                 init=None):
        """``init(global_ids) -> [len(ids), dim]`` fills this rank's rows (default zeros)."""
        self.ctx = ctx
        self.world = ctx.world_size if (ctx is not None and ctx.is_dist) else 1
        self.rank = ctx.rank if self.world > 1 else 0
        self.n_rows, self.dim = int(n_rows), int(dim)
        self.device = torch.device(device) if device is not None else (
            ctx.device if ctx is not None else torch.device("cpu"))
        n_local = (self.n_rows - self.rank + self.world - 1) // self.world if self.n_rows > self.rank else 0
        gid = self.local_ids(n_local)
        if init is None:
            self.local = torch.zeros((n_local, self.dim), dtype=dtype, device=self.device)
        else:
            self.local = init(gid).to(self.device, dtype).reshape(n_local, self.dim).contiguous()

    # ------------------------------------------------------------------ layout
    def local_ids(self, n_local: int | None = None) -> torch.Tensor:
        n_local = self.local.shape[0] if n_local is None else n_local
        return torch.arange(n_local, dtype=torch.int64, device=self.device) * self.world + self.rank

    def owner(self, ids: torch.Tensor) -> torch.Tensor:
        return ids % self.world

    # ------------------------------------------------------------------ routing
    def _route(self, ids: torch.Tensor):
        """Sort ids by owner; exchange counts; returns (order, send_ids, send_counts,
        recv_ids, recv_counts)."""
        own = self.owner(ids)
        order = torch.argsort(own, stable=True)
        send_ids = ids[order].contiguous()
        send_counts = torch.bincount(own, minlength=self.world).to(torch.int64)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts)
        sc, rc = send_counts.tolist(), recv_counts.tolist()
        recv_ids = torch.empty(sum(rc), dtype=ids.dtype, device=ids.device)
        dist.all_to_all_single(recv_ids, send_ids, rc, sc)
        return order, sc, recv_ids, rc

    def pull(self, ids: torch.Tensor) -> torch.Tensor:
        """Rows of the global ``ids`` ([m] int64, typically unique) as an [m, dim] tensor."""
        ids = ids.to(self.device, torch.int64).contiguous()
        if self.world == 1:
            return self.local[ids]
        order, sc, recv_ids, rc = self._route(ids)
        rows = self.local[recv_ids // self.world].contiguous()
        back = torch.empty((ids.numel(), self.dim), dtype=self.local.dtype, device=self.device)
        dist.all_to_all_single(back, rows, sc, rc)
        out = torch.empty_like(back)
        out[order] = back
        return out

    def push_add(self, ids: torch.Tensor, delta: torch.Tensor) -> None:
        """local[ids] += delta on the owners (duplicates and concurrent ranks all add)."""
        ids = ids.to(self.device, torch.int64).contiguous()
        delta = delta.to(self.device, self.local.dtype).reshape(-1, self.dim)
        if self.world == 1:
            self.local.index_add_(0, ids, delta)
            return
        order, sc, recv_ids, rc = self._route(ids)
        d_sorted = delta[order].contiguous()
        recv = torch.empty((sum(rc), self.dim), dtype=self.local.dtype, device=self.device)
        dist.all_to_all_single(recv, d_sorted, rc, sc)
        self.local.index_add_(0, recv_ids // self.world, recv)

    def full(self) -> torch.Tensor:
        """The whole table on every rank (all-gather of the shards)."""
        if self.world == 1:
            return self.local.clone()
        n_max = (self.n_rows + self.world - 1) // self.world
        pad = torch.zeros((n_max, self.dim), dtype=self.local.dtype, device=self.device)
        pad[: self.local.shape[0]] = self.local
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(parts, pad)
        out = torch.empty((self.n_rows, self.dim), dtype=self.local.dtype, device=self.device)
        for r, p in enumerate(parts):
            n_r = (self.n_rows - r + self.world - 1) // self.world if self.n_rows > r else 0
            out[r::self.world] = p[:n_r]
        return out

    def steps_agreed(self, n_local_steps: int) -> int:
        """The largest step count of any rank (ranks with fewer steps pull/push empty batches)."""
        if self.world == 1:
            return int(n_local_steps)
        t = torch.tensor([int(n_local_steps)], dtype=torch.int64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    @property
    def local_bytes(self) -> int:
        return self.local.numel() * self.local.element_size()
