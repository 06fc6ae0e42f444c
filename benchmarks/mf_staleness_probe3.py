"""MF explicit SGD probe 3: the same fixture with the convergence test disabled (probe 2 showed
the -cv_rate check stopping wider grids after epoch 3 while the loss was on its plateau)."""
import json, sys
import numpy as np
sys.path.insert(0, ".")
from tests.test_mf import _ratings
from hivemall_amd.models.mf import MatrixFactorization
u, i, r = _ratings()
for g in (1, 3, 9, 36):
    for it in (20, 60):
        m = MatrixFactorization(f"-factors 10 -eta0 0.01 -update_mean -disable_cv -iters {it} -grid {g}", device="cuda").fit(u[:35000], i[:35000], r[:35000])
        pr = m.predict(u[35000:], i[35000:])
        print(json.dumps({"grid": g, "iters": it, "epochs_run": len(getattr(m.cv, "history", [])),
                          "rmse": round(float(np.sqrt(((pr - r[35000:]) ** 2).mean())), 4)}), flush=True)
