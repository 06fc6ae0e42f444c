"""Pure numpy per-row FFM oracle (restates the pinned train_ffm semantics, docs/compat.md).

G of shape [NF, NFLD] = one AdaGrad accumulator per (feature, field) slot (the default);
[NF, NFLD, Kp] = one per V element (-elementwise_adagrad)."""
import math

import numpy as np


def ftrl(z, n, w, g, alpha, beta, l1, l2):
    n1 = n + g * g
    sigma = (math.sqrt(n1) - math.sqrt(n)) / alpha
    z1 = z + g - sigma * w
    if abs(z1) <= l1:
        w1 = 0.0
    else:
        w1 = -(z1 - math.copysign(l1, z1)) / ((beta + math.sqrt(n1)) / alpha + l2)
    return z1, n1, w1


def ffm_train_rows(state, idx, y, hp, fld=None, val=None, train=True, cls=True, norm=True,
                   use_lin=True, use_bias=False):
    V, G, w, wz, wn, bias = (state[k] for k in ("V", "G", "w", "wz", "wn", "bias"))
    B, F = idx.shape
    losses, preds = [], []
    for r in range(B):
        ii = idx[r]
        ff = fld[r] if fld is not None else np.arange(F)
        xx = val[r].astype(np.float64) if val is not None else np.ones(F)
        sc = 1.0 / math.sqrt((xx * xx).sum()) if norm else 1.0
        snap = {(a, b): V[ii[a], ff[b]].astype(np.float64).copy() for a in range(F) for b in range(F) if a != b}
        p = 0.0
        for a in range(F):
            for b in range(a + 1, F):
                p += snap[(a, b)] @ snap[(b, a)] * xx[a] * xx[b] * sc * sc
        if use_lin:
            p += sum(w[ii[a]] * xx[a] * sc for a in range(F))
        if use_bias:
            p += bias[0]
        if cls:
            e = y[r] * p
            kappa = -y[r] / (1 + math.exp(e))
            losses.append(math.log1p(math.exp(-e)))
        else:
            kappa = p - y[r]
            losses.append(0.5 * kappa * kappa)
        preds.append(p)
        if not train:
            continue
        for a in range(F):
            for b in range(F):
                if a == b:
                    continue
                coef = kappa * sc * sc * xx[a] * xx[b]
                g = coef * snap[(b, a)] + hp["lambda_v"] * snap[(a, b)]
                if G.ndim == 2:
                    # one accumulator per (feature, field) slot: the squared gradients of its
                    # k factors are added, then every factor steps with the new total
                    G[ii[a], ff[b]] += float((g * g).sum())
                else:
                    G[ii[a], ff[b]] += g * g
                V[ii[a], ff[b]] = snap[(a, b)] - hp["eta0"] * g / np.sqrt(G[ii[a], ff[b]] + hp["eps"])
        if use_lin:
            for a in range(F):
                i = ii[a]
                wz[i], wn[i], w[i] = ftrl(wz[i], wn[i], w[i], kappa * xx[a] * sc, hp["alpha"], hp["beta"], hp["lambda1"], hp["lambda2"])
        if use_bias:
            bias[1], bias[2], bias[0] = ftrl(bias[1], bias[2], bias[0], kappa, hp["alpha"], hp["beta"], 0, 0)
    return np.array(losses), np.array(preds)
