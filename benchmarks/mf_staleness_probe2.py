"""MF explicit SGD staleness probe 2: RMSE per grid with more epochs, and with a wider init,
to tell slow saddle escape from a race (tests/test_mf.py fixture)."""
import json, sys
import numpy as np
sys.path.insert(0, ".")
from tests.test_mf import _ratings
from hivemall_amd.models.mf import MatrixFactorization
u, i, r = _ratings()
for opts in ("-iters 20", "-iters 100", "-iters 20 -rankinit gaussian -min_init_stddev 0.5", "-iters 20 -eta0 0.003"):
    for g in (1, 2, 3):
        m = MatrixFactorization(f"-factors 10 -eta0 0.01 -update_mean -grid {g} {opts}", device="cuda").fit(u[:35000], i[:35000], r[:35000])
        pr = m.predict(u[35000:], i[35000:])
        P = m.state["P"].float()
        print(json.dumps({"opts": opts, "grid": g, "rmse": round(float(np.sqrt(((pr - r[35000:]) ** 2).mean())), 4),
                          "P_abs_mean": round(float(P.abs().mean()), 5), "hist": [round(x, 1) for x in m.cv.history[:3]] if hasattr(m.cv, "history") else None}), flush=True)
