"""train_fm (bf16 V, config-2 engine) held-out logloss vs Hivemall's 8-mapper average on the
3 x 2^20-row stream of tests/test_fm.py::test_fm_gpu_logloss_parity_past_2p20_rows, by kernel grid
(Hogwild rows in flight = 4 x grid) and repetition: the spread of the Hogwild gap.

    python benchmarks/fm_grid_parity_probe.py [grids...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.fm import FMTrainer  # noqa: E402
from tests.test_fm import _rows, mapper_average_fm  # noqa: E402


def main():
    grids = [int(g) for g in sys.argv[1:]] or [64, 128, 256]
    extra = os.environ.get("PROBE_OPTS", "")          # e.g. "-fp32" (with HM_FM_VARIANT=2)
    reps = int(os.environ.get("PROBE_REPS", "3"))
    n = 3 << 20
    idx, y = criteo_like(n, 20, seed=5)
    eidx, ey = criteo_like(100000, 20, seed=77)
    yy = (ey > 0).float()
    opts = "-c -factors 8 -num_features 1048576 -eta0 0.01 -sigma 0.01"
    gopts = opts + " " + extra
    ll = lambda t, dev: torch.nn.functional.binary_cross_entropy_with_logits(  # noqa: E731
        t.predict_raw(rows=_rows(eidx).to(dev)).cpu(), yy).item()
    m8 = ll(mapper_average_fm(opts, idx, y, 8, 1 << 20), "cpu")
    print(json.dumps({"mappers8": round(m8, 5)}), flush=True)
    rows = _rows(idx, y).to("cuda")
    # PROBE_VARIANTS="0,2,3": kernel variants (HM_FM_VARIANT) interleaved in one process
    variants = os.environ.get("PROBE_VARIANTS", os.environ.get("HM_FM_VARIANT", "0")).split(",")
    # PROBE_HOT="0.01,0": the hot-feature write-through threshold (ops/fm.py HOT_FRAC; 0 = off)
    import hivemall_amd.ops.fm as fm_ops
    hots = [float(h) for h in os.environ.get("PROBE_HOT", str(fm_ops.HOT_FRAC)).split(",")]
    # PROBE_HOT_EVERY="1,8,32": write-through on one hot update in N (ops/fm.py HOT_EVERY)
    evs = [int(e) for e in os.environ.get("PROBE_HOT_EVERY", str(fm_ops.HOT_EVERY)).split(",")]
    # PROBE_XCDS="8,1,2": the waves on that many XCDs (ops/fm.py XCDS)
    xcds = [int(x) for x in os.environ.get("PROBE_XCDS", "8").split(",")]
    for rep in range(reps):
        for g in grids:
            for var, hot, ev, xc in [(v, h, e, x) for v in variants for h in hots for e in evs for x in xcds]:
                fm_ops.HOT_FRAC = hot
                fm_ops.HOT_EVERY = ev
                fm_ops.XCDS = xc
                os.environ["HM_FM_VARIANT"] = var
                torch.cuda.synchronize()
                t = time.perf_counter()
                m = FMTrainer(gopts + f" -grid {g}", device="cuda").fit(rows=rows)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                os.environ["HM_FM_VARIANT"] = "0"
                v = ll(m, "cuda")
                print(json.dumps({"opts": extra, "variant": var, "hot_frac": hot, "hot_every": ev, "xcds": xc, "grid": g, "rep": rep, "gpu": round(v, 5),
                                  "delta_vs_mappers8": round(v - m8, 5), "rows_per_s": round(n / dt)}), flush=True)


if __name__ == "__main__":
    main()
