"""Where does train_fm's Hogwild gap live?  fp32 V, grid 256, 3 x 2^20 criteo_like rows (the
stream of tests/test_fm.py::test_fm_gpu_logloss_parity_past_2p20_rows): the updates of the top-H
features by frequency added by float atomics (kernel variant 3), every other feature stored;
H = all is variant 2.  Held-out logloss vs Hivemall's 8-mapper average on the same rows.

    python benchmarks/fm_hot_probe.py [H ...]

Kernel variants 2 / 3 (fm_pipe_kernel with `atomicAdd` of the w and V steps for every / flagged
features, flags set by an `hm_fm_set_hot` entry point) were experiment code, removed after this
measurement (profiles/r5/fm_hot_probe.jsonl, fm_atomic_probe.jsonl; docs/perf_notes.md).  The probe
needs them restored to run.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd import _native  # noqa: E402
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.fm import FMTrainer  # noqa: E402
from tests.test_fm import _rows, mapper_average_fm  # noqa: E402


def main():
    hs = [int(h) for h in sys.argv[1:]] or [0, 32, 512, 8192, 65536]
    n = 3 << 20
    idx, y = criteo_like(n, 20, seed=5)
    eidx, ey = criteo_like(100000, 20, seed=77)
    yy = (ey > 0).float()
    opts = "-c -factors 8 -num_features 1048576 -eta0 0.01 -sigma 0.01 -fp32"
    ll = lambda t, dev: torch.nn.functional.binary_cross_entropy_with_logits(  # noqa: E731
        t.predict_raw(rows=_rows(eidx).to(dev)).cpu(), yy).item()
    m8 = ll(mapper_average_fm(opts.replace(" -fp32", ""), idx, y, 8, 1 << 20), "cpu")
    print(json.dumps({"mappers8": round(m8, 5)}), flush=True)
    cnt = torch.bincount(idx.flatten().long(), minlength=1 << 20)
    order = torch.argsort(cnt, descending=True)
    tot = float(cnt.sum())
    rows = _rows(idx, y).to("cuda")
    hot = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    _native.hip().hm_fm_set_hot(_native.ptr(hot))
    for H in hs:
        hot.zero_()
        if H > 0:
            hot[order[:H].cuda()] = 1
        os.environ["HM_FM_VARIANT"] = "3" if H > 0 else "0"
        torch.cuda.synchronize()
        t = time.perf_counter()
        m = FMTrainer(opts, device="cuda").fit(rows=rows)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        v = ll(m, "cuda")
        print(json.dumps({"hot": H, "position_share": round(float(cnt[order[:H]].sum()) / tot, 3) if H else 0.0,
                          "gpu": round(v, 5), "delta_vs_mappers8": round(v - m8, 5), "fit_rows_per_s": round(n / dt)}),
              flush=True)
    os.environ["HM_FM_VARIANT"] = "0"
    _native.hip().hm_fm_set_hot(None)


if __name__ == "__main__":
    main()
