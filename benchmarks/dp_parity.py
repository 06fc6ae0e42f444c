"""Logloss parity of the headline schedule at N ranks (BASELINE.json:2 "...; logloss parity").

Runs ``bench.py`` (shard-mean mixing every ``--mix-every`` steps, replicas stepping with
eta0 / alpha x N^p: the exact schedule the driver times) at world 1, 2, 4, 8 ... and, for comparison, at world 1 over
the SAME TOTAL number of distinct rows (N x steps batches on one rank).  Every batch a rank
trains on is distinct (``--resident-batches = --steps + --warmup``), so N ranks see N times the
rows of one rank, exactly as in the driver's weak-scaling run.

    python benchmarks/dp_parity.py --worlds 1 2 4 8 --device cpu            # gloo, CPU engine
    HM_DIST_BACKEND=gloo python benchmarks/dp_parity.py --device cuda ...   # N ranks on one GPU

Prints one JSON line per world: logloss_N, logloss_1 over the same total rows (``delta``) and
logloss_1 over one rank's share only (``logloss_1_same_steps``).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(world: int, steps: int, a, timeout: int) -> dict:
    """One bench.py run at ``world`` ranks, ``steps`` timed steps per rank, all rows distinct."""
    bargs = ["--gpus", str(world), "--steps", str(steps), "--warmup", str(a.warmup),
             "--batch", str(a.batch), "--hash-bits", str(a.hash_bits), "--mix-every", str(a.mix_every),
             "--mix-overlap", str(a.mix_overlap), "--eval-rows", str(a.eval_rows),
             "--resident-batches", str(steps + a.warmup), "--mix-probe", "0", "--alt-run", "0",
             "--state", a.state, "--mix-mode", a.mix_mode, "--mix-state", str(a.mix_state),
             "--mix-power", str(a.mix_power)]
    if a.dp_lr_power is not None:
        bargs += ["--dp-lr-power", str(a.dp_lr_power)]
    if a.device:
        bargs += ["--device", a.device]
    bench = os.path.join(ROOT, "bench.py")
    if world > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", bench] + bargs
    else:
        cmd = [sys.executable, bench] + bargs
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 8) // max(1, world))))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    if r.returncode != 0:
        raise RuntimeError(f"world {world}: rc {r.returncode}\n{r.stderr[-3000:]}")
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--steps", type=int, default=40, help="timed steps per rank")
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--hash-bits", type=int, default=14)
    ap.add_argument("--mix-every", type=int, default=10)
    ap.add_argument("--mix-overlap", type=int, default=0)
    ap.add_argument("--dp-lr-power", type=float, default=None)
    ap.add_argument("--eval-rows", type=int, default=65536)
    ap.add_argument("--state", default="fp32")
    ap.add_argument("--mix-mode", default="mean")
    ap.add_argument("--mix-state", type=int, default=0)
    ap.add_argument("--mix-power", type=float, default=1.0)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--timeout", type=int, default=1800)
    ap.add_argument("--same-steps", type=int, default=1,
                    help="also run one rank for --steps only (its own share of the rows)")
    a = ap.parse_args(argv)
    res = []
    for w in a.worlds:
        rn = run(w, a.steps, a, a.timeout)
        r1 = run(1, a.steps * w, a, a.timeout) if w > 1 else rn
        # one rank on its own share only (the weak-scaling comparison: what N ranks add)
        r1s = run(1, a.steps, a, a.timeout) if (w > 1 and a.same_steps) else None
        rec = {"world": w, "steps_per_rank": a.steps, "rows_per_rank": a.batch * (a.steps + a.warmup),
               "total_rows": a.batch * (a.steps + a.warmup) * w, "mix_every": a.mix_every,
               "overlap": a.mix_overlap, "mix_mode": a.mix_mode, "mix_state": a.mix_state,
               "dp_lr_scale": rn["config"].get("dp_lr_scale"),
               "mix_power": a.mix_power,
               "batch": a.batch, "hash_bits": a.hash_bits,
               "backend": rn.get("dist_backend"), "device": a.device,
               "logloss_N": rn["logloss_heldout"], "logloss_1_same_rows": r1["logloss_heldout"],
               "delta": round(rn["logloss_heldout"] - r1["logloss_heldout"], 5),
               "logloss_1_same_steps": r1s["logloss_heldout"] if r1s else None,
               "floor": rn["logloss_planted_floor"], "mixes_timed": rn["config"]["mixes_in_timed_region"]}
        res.append(rec)
        print(json.dumps(rec), flush=True)
    return res


if __name__ == "__main__":
    main()
