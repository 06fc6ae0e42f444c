"""Per-row numpy FM oracle (Rendle SGD, the pinned train_fm rule, docs/compat.md)."""
import math

import numpy as np


def fm_train(rows, y, dims, V0, eta0=0.05, power_t=0.1, l0=0.01, lw=0.01, lv=0.01, cls=True):
    w0 = 0.0
    w = np.zeros(dims)
    V = V0.astype(np.float64).copy()
    losses = []
    for t, (feats, yy) in enumerate(zip(rows, y), start=1):
        i = np.asarray(feats)
        x = np.ones(len(i))
        S = (V[i] * x[:, None]).sum(0)
        p = w0 + (w[i] * x).sum() + 0.5 * float((S * S).sum() - ((V[i] * x[:, None]) ** 2).sum())
        if cls:
            d = -yy / (1 + math.exp(yy * p))
            losses.append(math.log1p(math.exp(-yy * p)))
        else:
            d = p - yy
        eta = eta0 / (t ** power_t)
        for j, xi in zip(i, x):
            w[j] -= eta * (d * xi + 2 * lw * w[j])
            g = d * xi * (S - V[j] * xi) + 2 * lv * V[j]
            V[j] -= eta * g
        w0 -= eta * (d + 2 * l0 * w0)
    return w0, w, V, np.array(losses)
