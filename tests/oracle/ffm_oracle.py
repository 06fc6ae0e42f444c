"""Pure numpy per-row FFM oracle (restates the pinned train_ffm semantics, docs/compat.md).

G of shape [NF, NFLD] = one AdaGrad accumulator per (feature, field) slot (the default);
[NF, NFLD, Kp] = one per V element (-elementwise_adagrad).

A row updates each (feature, field) address it touches ONCE, with the gradient of the row's
loss w.r.t. that vector: when two features of the row share a field (multi-hot fields) or a
feature appears twice, every pair (a, b) with (i_a, f_b) = the address contributes its partner
term, and the L2 term lambda_v * V is added once (:func:`row_grads`)."""
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


def row_grads(snap_v, ii, ff, xx, coef_scale, lambda_v):
    """Gradient of one row's objective w.r.t. every V address the row's pairs touch.

    ``snap_v(i, f)``: the address's vector at the start of the row; ``coef_scale`` = kappa *
    scale^2.  Returns {(i, f): g} with g = sum over pairs (a, b), a != b, (i_a, f_b) = (i, f) of
    coef_scale x_a x_b V[i_b, f_a], plus lambda_v V[i, f]."""
    F = len(ii)
    out = {}
    for a in range(F):
        for b in range(F):
            if a == b or ii[a] < 0 or ii[b] < 0:
                continue
            key = (int(ii[a]), int(ff[b]))
            term = coef_scale * xx[a] * xx[b] * snap_v(ii[b], ff[a])
            out[key] = out[key] + term if key in out else term
    return {k: g + lambda_v * snap_v(*k) for k, g in out.items()}


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
        v0 = {}
        for a in range(F):
            for b in range(F):
                v0[(int(ii[a]), int(ff[b]))] = V[ii[a], ff[b]].astype(np.float64).copy()
        grads = row_grads(lambda i, f: v0[(int(i), int(f))], ii, ff, xx, kappa * sc * sc, hp["lambda_v"])
        for (i, f), g in grads.items():
            if G.ndim == 2:
                # one accumulator per (feature, field) slot: the squared gradients of its
                # k factors are added, then every factor steps with the new total
                G[i, f] += float((g * g).sum())
            else:
                G[i, f] += g * g
            V[i, f] = v0[(i, f)] - hp["eta0"] * g / np.sqrt(G[i, f] + hp["eps"])
        if use_lin:
            # one FTRL step per distinct feature of the row, with the summed gradient
            gl = {}
            for a in range(F):
                gl[int(ii[a])] = gl.get(int(ii[a]), 0.0) + kappa * xx[a] * sc
            for i, g in gl.items():
                wz[i], wn[i], w[i] = ftrl(wz[i], wn[i], w[i], g, hp["alpha"], hp["beta"], hp["lambda1"], hp["lambda2"])
        if use_bias:
            bias[1], bias[2], bias[0] = ftrl(bias[1], bias[2], bias[0], kappa, hp["alpha"], hp["beta"], 0, 0)
    return np.array(losses), np.array(preds)
