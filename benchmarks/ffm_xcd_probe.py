"""Is the FFM kernel's same-stream gap an XCD-coherence effect?  MI355X has 8 XCDs, each with its
own L2; plain loads of a line another XCD keeps updating can hit this XCD's stale copy.  Same
rows in flight, different XCD spread: G blocks dealt round-robin over the 8 XCDs, against the
same G blocks all on XCD 0 (HM_FFM_XCD_ONLY=1: a grid of 8G where only blocks b % 8 == 0 work).
Held-out logloss after N rows of the bench stream (criteo_ffm, seed 1000, fp32, no ramp) vs the
sequential engine on the same rows.

    python benchmarks/ffm_xcd_probe.py [n_rows] [grids...]
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
    mems = os.environ.get("PROBE_MEM", "default").split(",")
    for mem, G, one_xcd in [(m, G, x) for m in mems for G in grids for x in ((0, 1) if G else (0,))]:
            os.environ["HM_FFM_MEM"] = mem
            os.environ["HM_FFM_XCD_ONLY"] = str(one_xcd)
            tr = FFMTrainer(OPTS, device=dev)
            tr.init_state(1 << BITS, F)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for s in range(0, n, B):
                ffm_step(tr.state, gi[s:s + B], gf[s:s + B], gv[s:s + B], gy[s:s + B], tr.hyper, variant=0,
                         grid=(8 * G if one_xcd else G))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            ll = heldout(tr, dev)
            print(json.dumps({"mem": mem, "blocks_working": G or "default", "one_xcd": bool(one_xcd), "gpu": round(ll, 5),
                              "gap": round(ll - ll_seq, 5), "rows_per_s": round(n / dt)}), flush=True)
    os.environ["HM_FFM_XCD_ONLY"] = "0"


if __name__ == "__main__":
    main()
