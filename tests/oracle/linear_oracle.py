"""Per-example numpy restatement of a few Hivemall online learners (docs/compat.md).
Independent of csrc/kernels/linear_rules.h: used to pin the C++/HIP rules."""
import math

import numpy as np


def train(algo, rows, y, dims, r=0.1, c=1.0, eta0=0.1, power_t=0.1, eps=1e-6):
    w = np.zeros(dims)
    cov = np.ones(dims)
    G = np.zeros(dims)
    t = 0
    for feats, yy in zip(rows, y):
        t += 1
        i = np.asarray(feats, dtype=np.int64)
        x = np.ones(len(i))
        p = float((w[i] * x).sum())
        if algo == "perceptron":
            if yy * p <= 0:
                w[i] += yy * x
        elif algo == "pa1":
            loss = max(0.0, 1 - yy * p)
            if loss > 0:
                eta = min(c, loss / float((x * x).sum()))
                w[i] += eta * yy * x
        elif algo == "arow":
            m = yy * p
            var = float((cov[i] * x * x).sum())
            if m < 1:
                beta = 1.0 / (var + r)
                alpha = (1 - m) * beta
                sx = cov[i] * x
                w[i] += alpha * yy * sx
                cov[i] -= beta * sx * sx
        elif algo == "adagrad_logloss":  # train_classifier -loss logloss -opt adagrad -reg no
            z = yy * p
            d = -yy / (1 + math.exp(z))
            g = d * x
            G[i] += g * g
            eta = eta0 / (t ** power_t)
            w[i] -= eta * g / (np.sqrt(G[i]) + eps)
        else:
            raise ValueError(algo)
    return w, cov
