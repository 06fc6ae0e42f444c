"""Early-training gap of the FFM kernel by launch grid: held-out logloss after N rows of the bench
stream (criteo_ffm, seed 1000, fp32, no ramp) vs the sequential engine on the same rows, per
kernel variant and grid (0 = the kernel's default).

The round-5 attribution runs of this probe (profiles/r5/ffm_xcd_probe.jsonl, ffm_sc1_probe.jsonl,
ffm_uncached_xcd8.jsonl, ffm_reload_wt_probe.jsonl, ffm_inflight_probe.jsonl) also swept
experiment switches (table memory type, one-XCD placement, SC1 / write-through / acquire
variants, rows in flight per CU) that were removed after the measurement: they ran at commit
7cffa38 plus the variants described in docs/perf_notes.md.

    [PROBE_VARIANTS=0,6] python benchmarks/ffm_xcd_probe.py [n_rows] [grids...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

B, BITS, F = 262144, 20, 39
OPTS = f"-classification -factors 4 -feature_hashing {BITS} -num_fields {F} -seed 31 -batch_size {B}"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    grids = [int(g) for g in sys.argv[2:]] or [8, 64, 0]
    idx, fld, val, y = criteo_ffm(n, BITS, seed=1000)
    eidx, efld, evl, ey, _ = criteo_ffm(B, BITS, seed=999_999, return_logit=True)
    yy = (ey > 0).float()

    def heldout(tr, dev):
        pred = torch.empty(B, device=dev)
        ffm_step(tr.state, eidx.to(dev), efld.to(dev), evl.to(dev), None, tr.hyper, train=False, pred=pred)
        return torch.nn.functional.binary_cross_entropy_with_logits(pred.cpu(), yy).item()

    t0 = time.time()
    seq = FFMTrainer(OPTS, device="cpu")
    seq.init_state(1 << BITS, F)
    for s in range(0, n, B):
        ffm_step(seq.state, idx[s:s + B], fld[s:s + B], val[s:s + B], y[s:s + B], seq.hyper)
    ll_seq = heldout(seq, "cpu")
    print(json.dumps({"rows": n, "seq": round(ll_seq, 5), "cpu_s": round(time.time() - t0, 1)}), flush=True)
    dev = torch.device("cuda")
    gi, gf, gv, gy = (t.to(dev) for t in (idx, fld, val, y))
    variants = [int(v) for v in os.environ.get("PROBE_VARIANTS", "0").split(",")]
    for var, G in [(v, G) for v in variants for G in grids]:
        tr = FFMTrainer(OPTS, device=dev)
        tr.init_state(1 << BITS, F)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for s in range(0, n, B):
            ffm_step(tr.state, gi[s:s + B], gf[s:s + B], gv[s:s + B], gy[s:s + B], tr.hyper, variant=var, grid=G)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        ll = heldout(tr, dev)
        print(json.dumps({"variant": var, "blocks": G or "default", "gpu": round(ll, 5),
                          "gap": round(ll - ll_seq, 5), "rows_per_s": round(n / dt)}), flush=True)


if __name__ == "__main__":
    main()
