import json, sys
import numpy as np
sys.path.insert(0, ".")
from tests.test_mf import _ratings
from hivemall_amd.models.mf import MatrixFactorization, MatrixFactorizationAdaGrad
u, i, r = _ratings()
for cls in (MatrixFactorization, MatrixFactorizationAdaGrad):
    for um in ("-update_mean", "-mu 3"):
        for g in (1, 3, 9, 36):
            res = {}
            for dev in ("cpu", "cuda"):
                if dev == "cpu" and g != 1:
                    continue
                m = cls(f"-factors 10 -iters 20 -eta0 0.01 {um} -grid {g}", device=dev).fit(u[:35000], i[:35000], r[:35000])
                pr = m.predict(u[35000:], i[35000:])
                res[dev] = round(float(np.sqrt(((pr - r[35000:]) ** 2).mean())), 4)
            print(json.dumps({"model": cls.NAME, "opt": um, "grid": g, **res}), flush=True)
