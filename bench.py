#!/usr/bin/env python
"""Headline benchmark: train_ffm rows/sec on Criteo-shaped sparse data (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W

N>1 without a launcher: the parent process starts ``torch.distributed.run`` with N ranks on
127.0.0.1 itself (before it touches the GPU) and exits with the launcher's code; under a
launcher (``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N``) every
rank checks WORLD_SIZE == N and that the process group really holds N ranks, else exits 2.

One process per GPU.  Each rank holds a full FFM model replica in HBM
(2^20 hashed features x 39 fields x k=4, fp32 V + AdaGrad G + FTRL state, ~1.3 GB) and
trains on its own shard of synthetic Criteo-shaped rows (weak scaling: per-GPU batch is
fixed).  A step = one fused ``hm_ffm_step`` launch over ``--batch`` rows per GPU; every
``--mix-every`` steps the replicas are averaged with a bucketed RCCL all-reduce over xGMI
(the MixServer replacement) — that mixing cost is inside the timed region.

Timing: W untimed warmup steps, then barrier + synchronize, K timed steps, synchronize +
barrier; the max over ranks is reported.  After timing, rank 0 evaluates logloss of the
mixed model on held-out rows and the planted model's logloss (the Bayes floor).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_METRIC = "rows/sec (node) FFM on Criteo-shaped sparse at 1/2/4/8 MI355X; logloss parity"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=262144, help="rows per GPU per step")
    ap.add_argument("--hash-bits", type=int, default=20)
    ap.add_argument("--factors", type=int, default=4)
    ap.add_argument("--mix-every", type=int, default=10)
    ap.add_argument("--mix-overlap", type=int, default=1,
                    help="1: stale-by-one mixing overlapped with compute (async MixServer semantics)")
    ap.add_argument("--resident-batches", type=int, default=8)
    ap.add_argument("--eval-rows", type=int, default=262144)
    ap.add_argument("--grid", type=int, default=0, help="kernel grid override (0 = auto)")
    ap.add_argument("--state", choices=("bf16", "fp32"), default="bf16",
                    help="V / AdaGrad state storage (bf16 = stochastic-rounded, fp32 accumulate)")
    ap.add_argument("--layout", choices=("packed", "split"), default="packed",
                    help="V/G state layout: packed V|G slots (one 16-B access per slot) or split tables")
    ap.add_argument("--reload", type=int, default=-1,
                    help="1: re-read the own slot right before its update (short Hogwild window); "
                         "0: keep the gathered slot in registers; -1: by layout (packed -> 0)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--gen-device", choices=("auto", "cpu"), default="auto",
                    help="where the synthetic rows are drawn (cpu = the exact stream of "
                         "benchmarks/ffm_parity_bench_scale.py, copied to the GPU before timing)")
    ap.add_argument("--mix-probe", type=int, default=3,
                    help="synchronous mixes timed after the run (ms, wire bytes, bus GB/s)")
    return ap.parse_args(argv)


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(args, argv) -> int | None:
    """--gpus N > 1 outside a launcher: run N ranks under torch.distributed.run as a CHILD
    process (this process never initialises the GPU, so nothing is exec'd over a HIP context)
    and return its exit code.  None when this process is itself a rank."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)]
    cmd += list(sys.argv[1:] if argv is None else argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def check_world(args, ctx) -> None:
    """Every rank: the job must really be N ranks (driver contract: value = whole-job rate)."""
    import torch.distributed as dist

    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    pg_world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
    bad = []
    if env_world != args.gpus:
        bad.append(f"WORLD_SIZE={env_world}")
    if pg_world != args.gpus or ctx.world_size != args.gpus:
        bad.append(f"process group world={pg_world}")
    if ctx.device.type == "cuda" and torch.cuda.device_count() < args.gpus:
        bad.append(f"only {torch.cuda.device_count()} visible GPUs")
    if bad:
        print(f"[bench] --gpus {args.gpus} but " + ", ".join(bad), file=sys.stderr, flush=True)
        sys.exit(2)


def main(argv=None):
    args = parse_args(argv)
    rc = self_launch(args, argv)
    if rc is not None:
        sys.exit(rc)
    from hivemall_amd.parallel.dist import init_distributed
    from hivemall_amd.parallel.mix import ModelMixer, OverlappedMixer
    from hivemall_amd.models.ffm import FFMTrainer
    from hivemall_amd.ops.ffm import ffm_step
    from hivemall_amd.io.synthetic import criteo_like

    ctx = init_distributed(device=args.device)
    dev = ctx.device
    world, rank = ctx.world_size, ctx.rank
    check_world(args, ctx)
    F = 39
    NF = 1 << args.hash_bits
    B = args.batch
    nres = max(1, args.resident_batches)

    # per-rank shard of synthetic Criteo-shaped rows, resident in HBM
    gdev = torch.device("cpu") if args.gen_device == "cpu" else dev
    idx, y = criteo_like(B * nres, args.hash_bits, seed=1000 + rank, device=gdev)
    idx, y = idx.to(dev), y.to(dev)
    opts = (f"-classification -factors {args.factors} -feature_hashing {args.hash_bits} "
            f"-num_fields {F} -seed 31 -batch_size {B}" +
            (" -bf16_state" if args.state == "bf16" and dev.type == "cuda" else "") +
            (" -split_state" if args.layout == "split" else ""))
    tr = FFMTrainer(opts, device=dev)
    tr.init_state(NF, F)
    st, hyper = tr.state, tr.hyper
    hyper.reload = None if args.reload < 0 else bool(args.reload)
    mixer = ModelMixer(ctx)
    mix_tensors = [st["V"], st["wz"], st["wn"], st["w"], st["bias"]]
    grid = args.grid

    overlap = OverlappedMixer(mixer) if args.mix_overlap else None

    def step(i):
        s = (i % nres) * B
        ffm_step(st, idx[s:s + B], None, None, y[s:s + B], hyper, train=True, grid=grid)
        if world > 1 and (i + 1) % args.mix_every == 0:
            if overlap is not None:
                overlap.start(mix_tensors)   # finishes the previous mix, launches this one
            else:
                mixer.average(mix_tensors)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for i in range(args.warmup):
        step(i)
    sync()
    ctx.barrier()
    sync()
    calls0 = mixer.calls
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
    if overlap is not None:
        overlap.finish()   # the last in-flight mix is applied inside the timed region
    sync()
    ctx.barrier()
    t1 = time.perf_counter()
    mixes_timed = mixer.calls - calls0
    elapsed = t1 - t0
    elapsed = mixer.all_reduce_scalar(elapsed, "max")
    ms_per_step = 1000.0 * elapsed / max(1, args.steps)
    rows_total = float(B) * world * args.steps
    rows_per_s = rows_total / elapsed
    if os.environ.get("HM_TRACE"):
        # host + device timeline of a few extra steps (outside the timed region)
        from hivemall_amd.prof import host_trace

        with host_trace(os.environ["HM_TRACE"], name="bench_ffm", rank=ctx.rank):
            for i in range(3):
                step(args.warmup + args.steps + i)
            if overlap is not None:
                overlap.finish()
            sync()

    # ---- mix cost on its own (synchronous, outside the timed region); leaves the model mixed ----
    probe = mixer.probe(mix_tensors, args.mix_probe) if world > 1 else {}
    # ---- quality: final mix, then held-out logloss vs the planted-model floor ----
    if world > 1:
        mixer.average(mix_tensors)
    ll = floor = None
    if rank == 0:
        eidx, ey, elogit = criteo_like(args.eval_rows, args.hash_bits, seed=999_999, device=gdev,
                                       return_logit=True)
        eidx, ey, elogit = eidx.to(dev), ey.to(dev), elogit.to(dev)
        pred = torch.empty(args.eval_rows, dtype=torch.float32, device=dev)
        for s in range(0, args.eval_rows, B):
            e = min(args.eval_rows, s + B)
            ffm_step(st, eidx[s:e], None, None, None, hyper, train=False, pred=pred[s:e])
        yy = (ey > 0).float()
        ll = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
        floor = torch.nn.functional.binary_cross_entropy_with_logits(elogit, yy).item()
    if rank == 0:
        out = {
            "metric": BASELINE_METRIC,
            "value": round(rows_per_s, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if (args.state == "bf16" and dev.type == "cuda") else "fp32",
            "data": "synthetic (Criteo-shaped: 39 fields, Kaggle-DAC cardinalities, power-law "
                    "values, planted FM logit), random-init weights",
            "config": {
                "model": f"train_ffm (k={args.factors}, 2^{args.hash_bits} hashed features, "
                         f"{F} fields, AdaGrad V + FTRL w, instance L2 norm)",
                "global_batch": B * world,
                "seq_len": F,
                "nnz_per_row": F,
                "parallelism": f"dp{world}",
                "mix_every": args.mix_every,
                "state_layout": args.layout if dev.type == "cuda" else "split",
                "reload": (args.layout == "split") if args.reload < 0 else bool(args.reload),
                "mixed_bytes_per_mix": int(sum(t.numel() * t.element_size() for t in mix_tensors)),
                "mixes_in_timed_region": mixes_timed,
                "mix_overlapped": bool(overlap is not None),
            },
            "rccl_world": world if ctx.backend == "nccl" else None,
            "dist_backend": ctx.backend,
            "world": world,
            **probe,
            "logloss_heldout": round(ll, 5) if ll is not None else None,
            "logloss_planted_floor": round(floor, 5) if floor is not None else None,
            "rows_trained_per_rank": B * (args.steps + args.warmup),
        }
        print(json.dumps(out), flush=True)
    from hivemall_amd.parallel.dist import shutdown
    shutdown()


if __name__ == "__main__":
    main()
