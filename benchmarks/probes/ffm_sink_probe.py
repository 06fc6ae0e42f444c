"""Pipelined FFM kernel variants at fixed grids: polled DMA targets with the next row's slot DMA
issued early (C, HM_FFM_VARIANT 5) or late (after this row's stores, 4) vs vmcnt(0) waits (the
default, 0) and the round-1 packed kernel (1, no lookahead).
Held-out logloss of bf16-state training on one stream, to separate a semantic difference
(visible at grid 1, where the only concurrency is the kernel's own one-row lookahead) from
Hogwild staleness (full grid).
    python benchmarks/probes/ffm_sink_probe.py
"""
import json

import torch

from hivemall_amd.io.synthetic import criteo_like
from hivemall_amd.models.ffm import FFMBatch, FFMTrainer
from hivemall_amd.ops import ffm as ffm_op


def run(variant, grid, n, bits, opts=""):
    ffm_op._VARIANT = variant
    idx, y = criteo_like(n, hash_bits=bits, seed=5)
    eidx, ey = criteo_like(100000, hash_bits=bits, seed=99)
    t = FFMTrainer(f"-classification -factors 4 -num_fields 39 -feature_hashing {bits} -seed 1 -bf16_state {opts}",
                   device="cuda")
    t.grid = grid
    t.fit(batch=FFMBatch(idx, None, None, y).to("cuda"))
    ffm_op._VARIANT = 0
    p = t.predict_raw(batch=FFMBatch(eidx, None, None, None).to("cuda")).cpu()
    return torch.nn.functional.binary_cross_entropy_with_logits(p, (ey > 0).float()).item()


def main():
    for grid, n, bits, opts in ((1, 30000, 16, ""), (1, 30000, 16, "-disable_wi"),
                                (0, 1000000, 20, ""), (0, 1000000, 20, "-disable_wi")):
        r = {v: round(run(v, grid, n, bits, opts), 6) for v in (5, 0, 4, 1)}
        print(json.dumps({"grid": grid, "rows": n, "bits": bits, "opts": opts,
                          "logloss_poll_early_dma": r[5], "logloss_vmcnt": r[0], "logloss_poll_late_dma": r[4], "logloss_round1_packed": r[1]}),
              flush=True)


if __name__ == "__main__":
    main()
