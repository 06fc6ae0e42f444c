"""Device-side cost of the overlapped shard-mean mix next to the FFM kernel, on ONE MI355X.

bench.py's N-rank schedule mixes [V, wz, wn, w, bias] every ``--mix-every`` steps through
``OverlappedMixer``: pack (compute stream) -> all_to_all -> ``hm_mix_shard_mean`` -> all_gather
(side stream) -> ``hm_mix_merge`` (compute stream, at the next mix point).  Without peers the
two collectives are stood in for by device copies of the same sizes (recv <- send; out <- the
gathered shards), so this measures every byte the GPU itself moves for a mix at world
``--world`` and how much of it the FFM kernel hides; the xGMI transfer time is the fabric's
and is not included.

    python benchmarks/mix_overlap_probe.py [--world 8] [--steps 40] [--mix-every 10]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402
from hivemall_amd.parallel.mix import _FlatGroup  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--mix-every", type=int, default=10)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--state", default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, F, NF = a.batch, 39, 1 << 20
    nres = 8
    idx, y = criteo_like(B * nres, 20, seed=1000, device=dev)
    tr = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 20" +
                    (" -bf16_state" if a.state == "bf16" else ""), device=dev)
    tr.init_state(NF, F)
    st, hyper = tr.state, tr.hyper
    tensors = [st["V"], st["wz"], st["wn"], st["w"], st["bias"]]
    by_dt = {}
    for t in tensors:
        by_dt.setdefault(t.dtype, []).append(t)
    groups = [_FlatGroup(ts, a.world) for ts in by_dt.values()]
    side = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    pending = []

    def mix_start():
        for g in groups:
            g.pack()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for g in groups:
                g.recv.copy_(g.send)                     # stands in for the all_to_all
                g.shard_mean(a.world)
                g.out.view(a.world, g.shard).copy_(g.mean.expand(a.world, g.shard))   # all_gather
        pending.append(True)

    def mix_finish(repack=False):
        if pending:
            cur.wait_stream(side)
            for g in groups:
                g.merge(repack)
            pending.clear()

    def step(i, mix):
        s = (i % nres) * B
        ffm_step(st, idx[s:s + B], None, None, y[s:s + B], hyper, train=True)
        if mix and (i + 1) % a.mix_every == 0:
            mix_finish(repack=True)     # OverlappedMixer.start: merge fused with the next pack
            mix_start()

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for i in range(8):                                   # warm-up (code objects, plans)
        step(i, True)
    mix_finish()
    n_mix = a.steps // a.mix_every
    res = {"world": a.world, "state": a.state, "steps": a.steps, "mix_every": a.mix_every,
           "mixed_bytes": int(sum(t.numel() * t.element_size() for t in tensors)),
           "wire_buffer_bytes": int(sum(g.buf_bytes for g in groups))}
    reps = {"alone": [], "with_mix": [], "mix_only": []}
    for _ in range(3):
        reps["alone"].append(timed(lambda: [step(i, False) for i in range(a.steps)]))

        def with_mix():
            for i in range(a.steps):
                step(i, True)
            mix_finish()
        reps["with_mix"].append(timed(with_mix))

        def mix_only():
            for _ in range(n_mix):
                mix_start()
                mix_finish()
        reps["mix_only"].append(timed(mix_only))
    t_alone, t_mix, t_only = (min(v) for v in reps.values())
    res.update({"ms_per_step_alone": round(1e3 * t_alone / a.steps, 4),
                "ms_per_step_with_mix": round(1e3 * t_mix / a.steps, 4),
                "ms_per_mix_device_alone": round(1e3 * t_only / max(1, n_mix), 3),
                "ms_per_mix_exposed": round(1e3 * (t_mix - t_alone) / max(1, n_mix), 3),
                "rows_per_s_alone": round(B * a.steps / t_alone),
                "rows_per_s_with_mix": round(B * a.steps / t_mix)})
    res["hidden_frac"] = round(1 - max(0.0, t_mix - t_alone) / max(1e-9, t_only), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
