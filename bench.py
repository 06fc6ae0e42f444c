#!/usr/bin/env python
"""Headline benchmark: train_ffm rows/sec on Criteo-shaped sparse data (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W

N>1 without a launcher: the parent process starts ``torch.distributed.run`` with N ranks on
127.0.0.1 itself (before it touches the GPU) and exits with the launcher's code; under a
launcher (``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N``) every
rank checks WORLD_SIZE == N and that the process group really holds N ranks, else exits 2.

One process per GPU.  Each rank holds a full FFM model replica in HBM (2^20 hashed features x
39 fields x k=4, one AdaGrad accumulator per (feature, field) slot as Hivemall's AdaGradEntry,
in line-padded feature blocks [V | G]: fp32 V + fp32 G by default = Hivemall's precision, 0.9 GB;
``--state bf16`` = bf16 V (stochastic rounding, fp32 math) in 12-B {V | G} slots, 0.5 GB; FTRL
w/z/n of the linear term fp32; ``--adagrad element`` = one accumulator per V element, stored like
V) and trains on its own shard of synthetic Criteo-for-FFM rows (``--data criteo_ffm``: explicit
field ids and values, log-scaled counts on the 13 integer fields; weak scaling: per-GPU batch
is fixed).  A step = one fused ``hm_ffm_step``
launch over ``--batch`` rows per GPU; every ``--mix-every`` steps the replicas are averaged
with the shard-mean collective of ``parallel/mix.py`` (all-to-all -> fp32 mean of each rank's
1/N shard -> all-gather, over RCCL/xGMI: the MixServer replacement), synchronously by default
(``--mix-overlap 1``: stale-by-one, overlapped); that mixing cost is inside the timed region.
At N > 1 every replica steps with eta0 and alpha times N^p (``--dp-lr-power``, default
``models.ffm.DP_LR_POWER``): the averaged replicas then track one learner over all N shards
(docs/compat.md, benchmarks/dp_sim.py).

Timing: W untimed warmup steps, then barrier + synchronize, K timed steps, synchronize +
barrier; the max over ranks is reported.  With fp32 state the first warmup step runs the
learner's early-training ramp (``--ramp-rows``, the atomic-update kernel that ``train_ffm`` uses
for its first 2^18 rows, docs/compat.md); the timed steps always run the default kernel.  After timing, rank 0 evaluates logloss of the mixed
model on held-out rows and the planted model's logloss (the Bayes floor).

On the GPU the same schedule then runs a second time with the other state precision in the
same process, on the same rows: ``value_bf16_state`` / ``logloss_heldout_bf16`` (``--alt-run 0``
skips it).  ``wall_s`` breaks the process's wall time down (data generation,
setup, warmup, timed region, evaluation, the other-precision run).  ``HM_METRICS=<path>`` appends one JSON
line per timed step (device ms from per-step events read after the timed region, rows/s, mean
training loss, mixes and wire bytes) — the loss buffer is only written when it is set.
"""
from __future__ import annotations

import argparse
import json
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
    ap.add_argument("--ramp-rows", type=int, default=None,
                    help="fp32 state: the first rows (whole steps, inside the untimed warmup only) run "
                         "the atomic-update kernel, as the learner does (models/ffm.py RAMP_ROWS; "
                         "default = the learner's 2^18; 0 = off)")
    ap.add_argument("--batch", type=int, default=262144, help="rows per GPU per step")
    ap.add_argument("--hash-bits", type=int, default=20)
    ap.add_argument("--factors", type=int, default=4)
    ap.add_argument("--mix-every", type=int, default=10)
    ap.add_argument("--mix-overlap", type=int, default=0,
                    help="1: stale-by-one mixing overlapped with compute (async MixServer semantics); "
                         "0: synchronous (the FFM kernel holds every CU, so the overlap hid ~nothing: "
                         "docs/perf_notes.md)")
    ap.add_argument("--mix-wire", choices=("auto", "native", "bf16_delta"), default="auto",
                    help="bf16_delta: fp32 replicas send their step since the last mix in bf16 "
                         "(half the bytes; fp32 consensus, parallel/mix.py average_delta); auto = "
                         "bf16_delta for fp32 state, native otherwise")
    ap.add_argument("--dp-lr-power", type=float, default=None,
                    help="N > 1: every replica steps with eta0 * N^p, alpha * N^p (default: "
                         "models.ffm.DP_LR_POWER)")
    ap.add_argument("--mix-mode", choices=("mean", "sum", "touched"), default="mean",
                    help="mean: replicas averaged (Hivemall's MixServer); sum: the consensus moves "
                         "by the sum of every rank's delta since the last mix")
    ap.add_argument("--mix-power", type=float, default=1.0,
                    help="sum mode: the consensus step is mean_r(delta_r) * N**power (1 = the sum)")
    ap.add_argument("--mix-state", type=int, default=0,
                    help="1: the AdaGrad accumulators G are mixed too (delta-summed in sum mode)")
    ap.add_argument("--resident-batches", type=int, default=8,
                    help="distinct batches per rank kept in HBM and replayed in turn")
    ap.add_argument("--eval-rows", type=int, default=262144)
    ap.add_argument("--grid", type=int, default=0, help="kernel grid override (0 = auto)")
    ap.add_argument("--state", choices=("bf16", "fp32"), default="fp32",
                    help="V storage of the headline run: fp32 = Hivemall's precision (the "
                         "reported value); bf16 = stochastic-rounded storage, fp32 math")
    ap.add_argument("--alt-run", type=int, default=1,
                    help="GPU: also time the same schedule with the other state precision "
                         "(value_bf16_state / value_fp32_state)")
    ap.add_argument("--data", choices=("criteo_ffm", "criteo_like"), default="criteo_ffm",
                    help="criteo_ffm: explicit field ids + log-scaled count values on the 13 "
                         "integer fields; criteo_like: implicit fields, every value 1.0 (rounds 1-3)")
    ap.add_argument("--adagrad", choices=("slot", "element"), default="slot",
                    help="AdaGrad accumulator of V: one per (feature, field) slot (Hivemall's "
                         "AdaGradEntry; fp32) or one per V element (stored like V)")
    ap.add_argument("--layout", choices=("packed", "split"), default="packed",
                    help="V/G state layout: packed V|G slots (one 16-B access per slot) or split tables")
    ap.add_argument("--reload", type=int, default=-1,
                    help="1: re-read the own slot right before its update (short Hogwild window); "
                         "0: keep the gathered slot in registers; -1: by layout (packed -> 0)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--gen-device", choices=("auto", "cpu"), default="cpu",
                    help="where the synthetic rows are drawn: cpu (default) = the exact stream "
                         "benchmarks/ffm_seq_ref.py replays through the sequential engine, copied to "
                         "the GPU before timing (the JSON then carries logloss_seq_ref / "
                         "logloss_gap); auto = drawn on the training device (a different stream)")
    ap.add_argument("--row-order", choices=("none", "spread", "xcd"), default="none",
                    help="row order inside each resident batch (ops/ffm_sched.py, a host pass "
                         "before timing; experiment: conflict-aware scheduling, docs/perf_notes.md)")
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


def _dp_lin_mode(world: int):
    from hivemall_amd.models.ffm import dp_lin_mode
    return dp_lin_mode(world)


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
    # HM_DIST_BACKEND=gloo is the multi-rank rehearsal on fewer cards (ranks share a GPU; the
    # JSON then reports dist_backend "gloo" and rccl_world null)
    if ctx.device.type == "cuda" and torch.cuda.device_count() < args.gpus and ctx.backend != "gloo":
        bad.append(f"only {torch.cuda.device_count()} visible GPUs")
    if bad:
        print(f"[bench] --gpus {args.gpus} but " + ", ".join(bad), file=sys.stderr, flush=True)
        sys.exit(2)


def run_schedule(args, ctx, idx, fld, val, y, state: str, data, metrics=None) -> dict:
    """One full FFM schedule (fresh model, warmup, timed region, final mix, held-out logloss).

    ``state``: "bf16" or "fp32" V|G storage.  Returns the timing / quality record."""
    from hivemall_amd.models.ffm import FFMTrainer
    from hivemall_amd.ops.ffm import ffm_step, linear_mix_tensors
    from hivemall_amd.parallel.mix import ModelMixer, OverlappedMixer

    dev = ctx.device
    world, rank = ctx.world_size, ctx.rank
    F = idx.shape[1]
    NF = 1 << args.hash_bits
    B = args.batch
    nres = max(1, args.resident_batches)
    wall = {}
    t_setup = time.perf_counter()
    opts = (f"-classification -factors {args.factors} -feature_hashing {args.hash_bits} "
            f"-num_fields {F} -seed 31 -batch_size {B}" +
            (" -bf16_state" if state == "bf16" and dev.type == "cuda" else "") +
            (" -split_state" if args.layout == "split" else "") +
            (" -elementwise_adagrad" if args.adagrad == "element" else ""))
    tr = FFMTrainer(opts, device=dev)
    tr.init_state(NF, F)
    st, hyper = tr.state, tr.hyper
    sc = 1.0
    if world > 1:
        # data-parallel replicas: step size x N^p (models/ffm.py DP_LR_POWER, docs/compat.md)
        from hivemall_amd.models.ffm import DP_LR_POWER, dp_lr_scale

        sc = dp_lr_scale(world, DP_LR_POWER if args.dp_lr_power is None else args.dp_lr_power)
        hyper.eta0 *= sc
        hyper.alpha *= sc
    hyper.reload = None if args.reload < 0 else bool(args.reload)
    mixer = ModelMixer(ctx)
    # mixed: V (weights) and the FTRL (z, n) the linear weight w is computed from, w, w0;
    # AdaGrad's G stays local (parallel/mix.py)
    # (the linear {w, z, n} records in the feature blocks mix as one [NF, 4] row view)
    mix_tensors = [st["V"], *linear_mix_tensors(st), st["bias"]]
    if args.mix_state:
        mix_tensors.append(st["G"])
    overlap = OverlappedMixer(mixer, args.mix_mode, args.mix_power) if args.mix_overlap else None
    wire = args.mix_wire if args.mix_wire != "auto" else (
        "bf16_delta" if st["V"].dtype == torch.float32 and args.mix_mode == "mean" else "native")
    sync_mix = mixer.average_delta if wire == "bf16_delta" else mixer.average
    loss_buf = torch.empty(B, dtype=torch.float32, device=dev) if metrics is not None else None
    step_loss = []

    from hivemall_amd.models import ffm as ffm_model

    ramp_rows = ffm_model.RAMP_ROWS if args.ramp_rows is None else int(args.ramp_rows)
    ramp_steps = 0
    if state == "fp32" and dev.type == "cuda" and ramp_rows > 0 and ffm_model.RAMP_VARIANT >= 0:
        ramp_steps = min(args.warmup, (ramp_rows + B - 1) // B)   # never inside the timed region

    def step(i):
        s = (i % nres) * B
        ramp = i < ramp_steps
        ffm_step(st, idx[s:s + B], None if fld is None else fld[s:s + B],
                 None if val is None else val[s:s + B], y[s:s + B], hyper, train=True,
                 grid=args.grid, loss=loss_buf, variant=ffm_model.RAMP_VARIANT if ramp else None,
                 lin_mode=ffm_model.dp_lin_mode(world))
        if loss_buf is not None:
            step_loss.append(loss_buf.mean())          # device scalar, read after timing
        if world > 1 and (i + 1) % args.mix_every == 0:
            if overlap is not None:
                overlap.start(mix_tensors)   # finishes the previous mix, launches this one
            else:
                sync_mix(mix_tensors)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    sync()
    wall["setup"] = time.perf_counter() - t_setup
    t = time.perf_counter()
    for i in range(args.warmup):
        step(i)
    sync()
    ctx.barrier()
    sync()
    wall["warmup"] = time.perf_counter() - t
    calls0 = mixer.calls
    wire0 = mixer.wire_bytes
    step_loss.clear()
    ev = []
    timed_steps = range(args.warmup, args.warmup + args.steps)
    use_ev = metrics is not None and dev.type == "cuda"
    t0 = time.perf_counter()
    for i in timed_steps:
        if use_ev:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append(e)
        step(i)
    if overlap is not None:
        overlap.finish()   # the last in-flight mix is applied inside the timed region
    if use_ev:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append(e)
    sync()
    ctx.barrier()
    t1 = time.perf_counter()
    wall["timed"] = t1 - t0
    mixes_timed = mixer.calls - calls0
    wire_timed = mixer.wire_bytes - wire0
    elapsed = mixer.all_reduce_scalar(t1 - t0, "max")
    if metrics is not None:
        for k, i in enumerate(timed_steps):
            ms = ev[k].elapsed_time(ev[k + 1]) if use_ev else 1e3 * elapsed / args.steps
            mixed = world > 1 and (i + 1) % args.mix_every == 0
            metrics.log(event="step", state=state, step=i, device_ms=round(ms, 4),
                        rows_per_s=round(B / (ms * 1e-3), 1) if ms > 0 else None,
                        loss=round(float(step_loss[k].item()), 6), mix=mixed,
                        wire_bytes=(wire_timed // max(1, mixes_timed)) if mixed else 0)
    out = {"elapsed_s": elapsed, "ms_per_step": 1000.0 * elapsed / max(1, args.steps),
           "rows_per_s": float(B) * world * args.steps / elapsed, "mixes_timed": mixes_timed,
           "mixed_bytes": int(sum(t.numel() * t.element_size() for t in mix_tensors)),
           "dp_lr_scale": sc, "ramp_steps": ramp_steps}
    if os.environ.get("HM_TRACE"):
        # host + device timeline of a few extra steps (outside the timed region)
        from hivemall_amd.prof import host_trace

        with host_trace(os.environ["HM_TRACE"], name=f"bench_ffm_{state}", rank=rank):
            for i in range(3):
                step(args.warmup + args.steps + i)
            if overlap is not None:
                overlap.finish()
            sync()

    # ---- mix cost on its own (synchronous, outside the timed region); leaves the model mixed ----
    out["probe"] = mixer.probe(mix_tensors, args.mix_probe, fn=sync_mix) if world > 1 else {}
    out["mix_wire"] = wire
    # ---- quality: final mix, then held-out logloss vs the planted-model floor ----
    t = time.perf_counter()
    if world > 1:
        sync_mix(mix_tensors)
    out["ll"] = None
    if rank == 0:
        eidx, efld, evl, ey, elogit = data["eval"]
        pred = torch.empty(eidx.shape[0], dtype=torch.float32, device=dev)
        for s in range(0, eidx.shape[0], B):
            e = min(eidx.shape[0], s + B)
            ffm_step(st, eidx[s:e], None if efld is None else efld[s:e],
                     None if evl is None else evl[s:e], None, hyper, train=False, pred=pred[s:e])
        yy = (ey > 0).float()
        out["ll"] = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
        out["floor"] = torch.nn.functional.binary_cross_entropy_with_logits(elogit, yy).item()
    sync()
    wall["eval"] = time.perf_counter() - t
    out["wall"] = wall
    mixer.release()
    del tr, st
    return out


def seq_reference(args, world: int):
    """Held-out logloss of the sequential engine on this run's exact row stream, if pinned
    (resources/bench_seq_ref.json, written by benchmarks/ffm_seq_ref.py); else None."""
    if args.gen_device != "cpu" or args.data != "criteo_ffm":
        return None      # rows drawn on the device: a stream no reference was computed for
    from benchmarks.ffm_seq_ref import load_refs, ref_key

    key = ref_key(world, args.steps, args.warmup, args.batch, args.hash_bits, args.factors,
                  max(1, args.resident_batches), args.eval_rows, order=args.row_order)
    rec = load_refs().get(key)
    return None if rec is None else round(float(rec["logloss_seq"]), 5)


def main(argv=None):
    t_start = time.perf_counter()
    args = parse_args(argv)
    rc = self_launch(args, argv)
    if rc is not None:
        sys.exit(rc)
    from hivemall_amd.parallel.dist import init_distributed
    from hivemall_amd.io.synthetic import criteo_ffm, criteo_like
    from hivemall_amd.prof import MetricsWriter

    ctx = init_distributed(device=args.device)
    dev = ctx.device
    world, rank = ctx.world_size, ctx.rank
    check_world(args, ctx)
    F = 39
    B = args.batch
    nres = max(1, args.resident_batches)
    metrics = MetricsWriter(rank=rank) if os.environ.get("HM_METRICS") else None

    # per-rank shard of synthetic Criteo-shaped rows, resident in HBM
    t = time.perf_counter()
    gdev = torch.device("cpu") if args.gen_device == "cpu" else dev
    def gen(n, seed, logit=False):
        if args.data == "criteo_ffm":
            out = criteo_ffm(n, args.hash_bits, seed=seed, device=gdev, return_logit=logit)
        else:
            out = criteo_like(n, args.hash_bits, seed=seed, device=gdev, return_logit=logit)
            out = (out[0], None, None) + tuple(out[1:])
        return tuple(None if t is None else t.to(dev) for t in out)

    idx, fld, val, y = gen(B * nres, 1000 + rank)
    if args.row_order != "none":
        from hivemall_amd.ops.ffm_sched import schedule_rows

        for b in range(nres):
            sl = slice(b * B, (b + 1) * B)
            p = schedule_rows(idx[sl].cpu(), args.row_order, nf=1 << args.hash_bits).to(dev)
            for ten in (idx, fld, val, y):
                if ten is not None:
                    ten[sl] = ten[sl][p]
    data = {"eval": None}
    if rank == 0:
        data["eval"] = gen(args.eval_rows, 999_999, logit=True)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t_gen = time.perf_counter() - t

    state = args.state if dev.type == "cuda" else "fp32"
    main_run = run_schedule(args, ctx, idx, fld, val, y, state, data, metrics)
    alt_state = "fp32" if state == "bf16" else "bf16"
    alt_run = None
    if dev.type == "cuda" and args.alt_run:
        alt_run = run_schedule(args, ctx, idx, fld, val, y, alt_state, data, metrics)

    wall = {"gen": round(t_gen, 3)}
    for k, v in main_run["wall"].items():
        wall[k] = round(v, 3)
    if alt_run is not None:
        wall[f"{alt_state}_run"] = round(sum(alt_run["wall"].values()), 3)
    wall["total"] = round(time.perf_counter() - t_start, 3)
    if metrics is not None:
        metrics.log(event="summary", wall_s=wall, rows_per_s=main_run["rows_per_s"],
                    **{f"rows_per_s_{alt_state}": alt_run["rows_per_s"] if alt_run else None})
    if rank == 0:
        ll, floor = main_run["ll"], main_run.get("floor")
        seq_ref = seq_reference(args, world)
        out = {
            "metric": BASELINE_METRIC,
            "value": round(main_run["rows_per_s"], 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(main_run["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if state == "bf16" else "fp32",
            "data": ("synthetic Criteo-for-FFM field:index:value rows (39 explicit fields; 13 "
                     "integer fields hashed by log2 bucket with log-scaled count values, 26 "
                     "categorical with Kaggle-DAC cardinalities and power-law frequencies, value "
                     "1; planted FFM-style logit), random-init weights"
                     if args.data == "criteo_ffm" else
                     "synthetic (Criteo-shaped: 39 implicit fields, Kaggle-DAC cardinalities, "
                     "power-law frequencies, every value 1.0, planted FM logit), random-init weights"),
            "config": {
                "model": f"train_ffm (k={args.factors}, 2^{args.hash_bits} hashed features, "
                         f"{F} fields, AdaGrad V + FTRL w, instance L2 norm)",
                "global_batch": B * world,
                "seq_len": F,
                "nnz_per_row": F,
                "fields": "explicit" if fld is not None else "implicit (slot j = field j)",
                "values": "explicit" if val is not None else "1.0",
                "parallelism": f"dp{world}",
                "mix_every": args.mix_every,
                "state": (f"{state} V, " + ("fp32 AdaGrad accumulator per (feature, field) slot"
                                            if args.adagrad == "slot" else f"{state} AdaGrad G per element") +
                          " (fp32 math" + (", stochastic rounding)" if state == "bf16" else ")")),
                "state_layout": args.layout if dev.type == "cuda" else "split",
                "reload": (args.layout == "split") if args.reload < 0 else bool(args.reload),
                "mixed_bytes_per_mix": main_run["mixed_bytes"],
                "mixes_in_timed_region": main_run["mixes_timed"],
                "mix_overlapped": bool(args.mix_overlap),
                "mix_wire": main_run["mix_wire"],
                "dp_lr_scale": round(main_run["dp_lr_scale"], 4),
                "early_ramp_warmup_steps": main_run["ramp_steps"],
                # FTRL linear steps: hot features' (z, n) in the side table (one rank, no step lost)
                # or plain record stores (replicas that mix: the N^p step rule's calibration)
                "linear_steps": ("side-table" if _dp_lin_mode(world) is None and dev.type == "cuda"
                                 else "plain-stores"),
                "resident_batches": nres,
            },
            "rccl_world": world if ctx.backend == "nccl" else None,
            "dist_backend": ctx.backend,
            "world": world,
            **main_run["probe"],
            "logloss_heldout": round(ll, 5) if ll is not None else None,
            "logloss_planted_floor": round(floor, 5) if floor is not None else None,
            # the sequential C++ engine (Hivemall's per-row semantics, one learner over every
            # rank's rows) on this exact stream, pinned offline by benchmarks/ffm_seq_ref.py
            "logloss_seq_ref": seq_ref,
            "logloss_gap": (round(ll - seq_ref, 5) if (ll is not None and seq_ref is not None)
                            else None),
            "rows_trained_per_rank": B * (args.steps + args.warmup),
            "wall_s": wall,
        }
        if alt_run is not None:
            out[f"value_{alt_state}_state"] = round(alt_run["rows_per_s"], 1)
            out[f"ms_per_step_{alt_state}_state"] = round(alt_run["ms_per_step"], 4)
            out[f"logloss_heldout_{alt_state}"] = round(alt_run["ll"], 5)
            if seq_ref is not None:
                out[f"logloss_gap_{alt_state}"] = round(alt_run["ll"] - seq_ref, 5)
        print(json.dumps(out), flush=True)
    from hivemall_amd.parallel.dist import shutdown
    shutdown()


if __name__ == "__main__":
    main()
