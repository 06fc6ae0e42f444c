"""Data-parallel FFM on one device: N replicas, the bench's exact schedule, exact mixing math.

The node metric is "rows/s at 1/2/4/8 GPUs; logloss parity" (BASELINE.json:2).  N ranks of
``bench.py`` each train their own shard (weak scaling) and mix every ``--mix-every`` steps.  This
script replays that on ONE device with N model replicas in HBM (each one a rank's replica,
stepped by the same ``hm_ffm_step`` kernel on the same rows ``bench.py`` rank r draws) and the
mixing rule applied with torch ops on the replica tensors — the collective's arithmetic without
the collective, so a mixing rule is a few lines here and N = 8 costs one card.

Reference: one replica trained on the SAME TOTAL rows (every rank's batches, interleaved),
i.e. what the node's rows/s claims to have learned from.

Mixing rules (synchronous; ``base`` = the last consensus, d_r = x_r - base):

* ``mean``     replicas averaged (Hivemall MIX / ``avg(weight) GROUP BY feature``); AdaGrad G local
* ``touched``  base + sum_r d_r / #ranks that changed the element (tail slots keep a lone rank's
               whole step; hot slots are averaged)
* ``sum``      base + N**power * mean_r d_r  (``--power``); ``gsum``: G <- Gbase + sum_r dG_r
* ``adasum``   the first-order image of ONE AdaGrad learner over the union of the ranks' rows: each
               rank's V step was taken with 1/sqrt(G0 + dG_r); the union learner's step size is
               1/sqrt(G0 + sum_r dG_r), so V <- base + sum_r d_r sqrt(G0 + dG_r + eps) /
               sqrt(G0 + sum dG + eps), G <- G0 + sum_r dG_r; FTRL (z, n) and the bias are sums of
               per-row statistics, so their deltas add and w = f(z, n)
* ``precision`` the union-optimal merge of N local optima under a quadratic model whose precision
               is AdaGrad's accumulator (argmin-KLD with the shared prior counted once): V <- base +
               sum_r (G0 + dG_r) d_r / (G0 + sum_r dG_r), G <- G0 + sum dG; a slot one rank touched
               keeps its whole step, a slot every rank drove to the same optimum from G0 ~ 0 gets
               the mean, small steps on a well-determined slot add up; the linear w the same way
               with FTRL's n as the precision (z re-derived so that f(z, n) = w)
* ``bmuf``     block momentum (Chen & Huo 2016): M <- mu M + mean_r d_r, base <- base + M, every
               replica restarts from base + mu M (Nesterov), mu = 1 - 1/N

    python benchmarks/dp_sim.py --worlds 2 4 8 --rules mean touched adasum --state fp32
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm, criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

F = 39
MIXED = ("V", "wz", "wn", "w", "bias")


def ftrl_w(z, n, h, l1=None, l2=None):
    l1 = h.lambda1 if l1 is None else l1
    l2 = h.lambda2 if l2 is None else l2
    w = -(z - torch.sign(z) * l1) / ((h.beta + n.sqrt()) / h.alpha + l2)
    return torch.where(z.abs() <= l1, torch.zeros_like(w), w)


class Sim:
    def __init__(self, a, world: int, dev):
        self.a, self.N, self.dev = a, world, dev
        B, nres = a.batch, a.resident_batches
        self.data = []
        for r in range(world):
            self.data.append(self._gen(B * nres, 1000 + r))
        self.eval = self._gen(a.eval_rows, 999_999, logit=True)

    def _gen(self, n, seed, logit=False):
        a = self.a
        if a.data == "criteo_ffm":
            out = criteo_ffm(n, a.hash_bits, seed=seed, device=self.dev, return_logit=logit)
        else:
            out = criteo_like(n, a.hash_bits, seed=seed, device=self.dev, return_logit=logit)
            out = (out[0], None, None) + tuple(out[1:])
        return out

    def trainer(self):
        a = self.a
        opts = (f"-classification -factors 4 -feature_hashing {a.hash_bits} -num_fields {F} -seed 31 "
                f"-batch_size {a.batch}" + (" -bf16_state" if a.state == "bf16" else ""))
        tr = FFMTrainer(opts, device=self.dev)
        tr.init_state(1 << a.hash_bits, F)
        return tr

    def step(self, tr, r, i):
        B = self.a.batch
        idx, fld, val, y = self.data[r]
        s = (i % self.a.resident_batches) * B
        sl = lambda t: None if t is None else t[s:s + B]  # noqa: E731
        ffm_step(tr.state, sl(idx), sl(fld), sl(val), sl(y), tr.hyper, train=True)

    def logloss(self, tr):
        eidx, efld, evl, ey, elogit = self.eval
        pred = torch.empty(eidx.shape[0], dtype=torch.float32, device=self.dev)
        B = self.a.batch
        for s in range(0, eidx.shape[0], B):
            e = min(eidx.shape[0], s + B)
            sl = lambda t: None if t is None else t[s:e]  # noqa: E731
            ffm_step(tr.state, eidx[s:e], sl(efld), sl(evl), None, tr.hyper, train=False, pred=pred[s:e])
        yy = (ey > 0).float()
        ll = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
        floor = torch.nn.functional.binary_cross_entropy_with_logits(elogit, yy).item()
        return ll, floor

    # ------------------------------------------------------------------ one rank, all rows
    def single(self, steps, lr_mult=1.0):
        tr = self.trainer()
        tr.hyper.eta0 *= lr_mult
        tr.hyper.alpha *= lr_mult
        for i in range(steps):
            for r in range(self.N):
                self.step(tr, r, i)
        return self.logloss(tr)

    # ------------------------------------------------------------------ N replicas + mixing
    def replicas(self, steps, rule, mix_every, lr_power=0.0):
        N, a = self.N, self.a
        trs = [self.trainer() for _ in range(N)]
        if lr_power:
            # every replica steps with eta0 * N**p (AdaGrad V) and alpha * N**p (FTRL w): with
            # p = 0.5 the mean of N replicas follows one learner over the union of their rows
            # (drift and noise; see docs/compat.md)
            for tr in trs:
                tr.hyper.eta0 *= float(N) ** lr_power
                tr.hyper.alpha *= float(N) ** lr_power
        h = trs[0].hyper
        keys = MIXED + ("G",)
        base = {k: trs[0].state[k].float().clone() for k in keys}
        mom = {k: torch.zeros_like(base[k]) for k in MIXED} if rule == "bmuf" else None
        glob = {k: base[k].clone() for k in MIXED} if rule == "bmuf" else None
        n_mix = 0
        t_mix = 0.0

        def mix():
            nonlocal n_mix, t_mix
            t0 = time.perf_counter()
            new = {}
            if rule == "mean":
                for k in MIXED + (("G",) if a.gsum else ()):
                    new[k] = sum(tr.state[k].float() for tr in trs) / N
            elif rule == "touched":
                for k in MIXED + (("G",) if a.gsum else ()):
                    acc = torch.zeros_like(base[k])
                    cnt = torch.zeros_like(base[k])
                    for tr in trs:
                        d = tr.state[k].float() - base[k]
                        acc += d
                        cnt += (d != 0).float()
                    new[k] = base[k] + acc / cnt.clamp_min(1.0)
            elif rule == "sum":
                sc = float(N) ** a.power / N
                for k in MIXED:
                    new[k] = base[k] + sc * sum(tr.state[k].float() - base[k] for tr in trs)
                if a.gsum:
                    new["G"] = base["G"] + sum(tr.state["G"] - base["G"] for tr in trs)
                if a.ftrl_recompute:
                    new["w"] = ftrl_w(new["wz"], new["wn"], h)
            elif rule == "adasum":
                G0 = base["G"]
                dG = [tr.state["G"] - G0 for tr in trs]
                Gn = G0 + sum(dG)
                num = torch.zeros_like(base["V"])
                for tr, g in zip(trs, dG):
                    num += (tr.state["V"].float() - base["V"]) * (G0 + g + h.eps).sqrt().unsqueeze(-1)
                new["V"] = base["V"] + num / (Gn + h.eps).sqrt().unsqueeze(-1)
                new["G"] = Gn
                for k in ("wz", "wn", "bias"):
                    new[k] = base[k] + sum(tr.state[k].float() - base[k] for tr in trs)
                new["w"] = ftrl_w(new["wz"], new["wn"], h)
                b = new["bias"]
                b[0] = -b[1] / ((h.beta + b[2].clamp_min(0).sqrt()) / h.alpha)
            elif rule == "precision":
                # union-optimal merge of N local optima under a quadratic model with the AdaGrad
                # accumulator as the precision: x = base + sum_r (G0 + dG_r) d_r / (G0 + sum dG)
                G0 = base["G"]
                dG = [tr.state["G"] - G0 for tr in trs]
                Gn = G0 + sum(dG)
                num = torch.zeros_like(base["V"])
                for tr, g in zip(trs, dG):
                    num += (tr.state["V"].float() - base["V"]) * (G0 + g + h.eps).unsqueeze(-1)
                new["V"] = base["V"] + num / (Gn + h.eps).unsqueeze(-1)
                new["G"] = Gn
                if a.lin == "mean":
                    for k in ("wz", "wn", "w", "bias"):
                        new[k] = sum(tr.state[k].float() for tr in trs) / N
                    return finish(new, t0)
                # linear term: the same merge of w with FTRL's n as the precision; z re-derived
                # so that f(z, n) = w
                n0 = base["wn"]
                dn = [tr.state["wn"] - n0 for tr in trs]
                nn = n0 + sum(dn)
                numw = sum((tr.state["w"] - base["w"]) * (n0 + d + 1e-12) for tr, d in zip(trs, dn))
                w = base["w"] + numw / (nn + 1e-12)
                D = (h.beta + nn.sqrt()) / h.alpha + h.lambda2
                new["w"] = w
                new["wn"] = nn
                new["wz"] = torch.where(w == 0, base["wz"] + sum(tr.state["wz"] - base["wz"] for tr in trs) / N,
                                        -w * D - torch.sign(w) * h.lambda1)
                # bias {w0, z0, n0}: l1 = l2 = 0
                b0 = base["bias"]
                bs = [tr.state["bias"] for tr in trs]
                dn0 = [b[2] - b0[2] for b in bs]
                n0n = b0[2] + sum(dn0)
                w0 = b0[0] + sum((b[0] - b0[0]) * (b0[2] + d + 1e-12) for b, d in zip(bs, dn0)) / (n0n + 1e-12)
                nb = b0.clone()
                nb[0], nb[2] = w0, n0n
                nb[1] = -w0 * (h.beta + n0n.sqrt()) / h.alpha
                new["bias"] = nb
            elif rule == "bmuf":
                # base = the block's start point (glob + mu M); D = mean_r x_r - start
                mu = 1.0 - 1.0 / N if a.mu < 0 else a.mu
                for k in MIXED:
                    D = sum(tr.state[k].float() - base[k] for tr in trs) / N
                    mom[k].mul_(mu).add_(D)
                    glob[k].add_(mom[k])
                    new[k] = glob[k] + mu * mom[k]
            else:
                raise ValueError(rule)
            finish(new, t0)

        def finish(new, t0):
            nonlocal n_mix, t_mix
            for k, v in new.items():
                if k == "G" and not (a.gsum or rule in ("adasum", "precision")):
                    continue
                for tr in trs:
                    tr.state[k].copy_(v)
                # the consensus as stored (bf16 V: rounded), so untouched elements compare equal
                base[k] = trs[0].state[k].float().clone()
            if dev_is_cuda:
                torch.cuda.synchronize()
            n_mix += 1
            t_mix += time.perf_counter() - t0

        dev_is_cuda = self.dev.type == "cuda"
        for i in range(steps):
            for r, tr in enumerate(trs):
                self.step(tr, r, i)
            if (i + 1) % mix_every == 0:
                mix()
        mix()                           # the final mix before the model is exported
        if rule == "bmuf":              # export the global model, not the look-ahead start
            for k in MIXED:
                trs[0].state[k].copy_(glob[k])
        ll = self.logloss(trs[0])
        del trs
        return ll, n_mix, t_mix


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--rules", nargs="*", default=["mean", "touched", "adasum"])
    ap.add_argument("--steps", type=int, default=25, help="steps per rank (driver: 20 timed + 5 warmup)")
    ap.add_argument("--mix-every", type=int, nargs="+", default=[10])
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--resident-batches", type=int, default=8)
    ap.add_argument("--hash-bits", type=int, default=20)
    ap.add_argument("--eval-rows", type=int, default=262144)
    ap.add_argument("--state", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--data", choices=("criteo_ffm", "criteo_like"), default="criteo_ffm")
    ap.add_argument("--power", type=float, default=0.5)
    ap.add_argument("--gsum", type=int, default=0)
    ap.add_argument("--ftrl-recompute", type=int, default=0)
    ap.add_argument("--mu", type=float, default=-1.0)
    ap.add_argument("--single-lr", type=float, nargs="*", default=[],
                    help="also train the one-rank reference with eta0 / alpha times these")
    ap.add_argument("--lr-power", type=float, nargs="+", default=[0.0],
                    help="replicas step with eta0 / alpha scaled by N**p")
    ap.add_argument("--lin", choices=("mean", "precision"), default="precision",
                    help="precision rule: how the linear term (w, z, n) and the bias are merged")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args(argv)
    dev = torch.device(a.device)
    for N in a.worlds:
        sim = Sim(a, N, dev)
        t0 = time.perf_counter()
        ll1, floor = sim.single(a.steps)
        rec0 = {"world": N, "rule": "single_same_rows", "steps_per_rank": a.steps, "state": a.state,
                "data": a.data, "hash_bits": a.hash_bits, "batch": a.batch, "logloss": round(ll1, 5),
                "floor": round(floor, 5), "s": round(time.perf_counter() - t0, 2)}
        print(json.dumps(rec0), flush=True)
        for m in a.single_lr:
            llm, _ = sim.single(a.steps, m)
            print(json.dumps({"world": N, "rule": "single_same_rows", "lr_mult": m, "logloss": round(llm, 5),
                              "delta_vs_default_lr": round(llm - ll1, 5)}), flush=True)
        for me, lp, rule in [(me, lp, rule) for me in a.mix_every for lp in a.lr_power for rule in a.rules]:
            if True:
                t0 = time.perf_counter()
                ll, nmix, tmix = sim.replicas(a.steps, rule, me, lp)
                rec = {"world": N, "rule": rule, "mix_every": me, "power": a.power if rule == "sum" else None,
                       "gsum": a.gsum, "lr_power": lp, "steps_per_rank": a.steps, "state": a.state, "logloss": round(ll[0], 5),
                       "single_same_rows": round(ll1, 5), "delta": round(ll[0] - ll1, 5), "mixes": nmix,
                       "mix_s": round(tmix, 3), "s": round(time.perf_counter() - t0, 2)}
                print(json.dumps(rec), flush=True)
        del sim
        if dev.type == "cuda":
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
