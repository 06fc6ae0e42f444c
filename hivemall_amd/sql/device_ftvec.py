"""Device-resident feature engineering for a learner's feature argument (SQL
executor -> ``mhash`` on the device -> fused learner kernels).

A training statement in the shape of Hivemall's tutorials::

    SELECT train_classifier(add_bias(feature_hashing(features)), label, '-loss logloss') ...

would evaluate ``feature_hashing`` and ``add_bias`` column-wise into hashed *strings* on the
host, and the learner would then parse those strings again.  On a GPU session this module
recognises a feature argument made of

    [add_bias(] feature_hashing(<column> [, '<const options>']) [)]

over an Arrow / list-of-strings column and evaluates it where the model lives: the raw strings
go up as Arrow buffers, ``hm_feat_parse`` hashes every name with Murmur3 (the same
``mhash(name, -num_features)`` the host writes as ``"h:value"``), the bias is appended on the
device, and the learner receives the CSR (``io.ingest.DeviceFeatures``).  The model table is the
string path's, bit for bit (``tests/test_sql.py``, ``benchmarks/sql_ftvec_bench.py``).

Anything else (other functions in the chain, non-constant options, a CPU session, a column
that is not a list of strings) returns None and the executor evaluates the expression as usual.
"""
from __future__ import annotations

import os

from .parser import Col, Func, Lit

DEFAULT_NUM_FEATURES = 1 << 24


def enabled() -> bool:
    return os.environ.get("HM_SQL_DEVICE_FTVEC", "1") != "0"


def _match(expr):
    """(column expr, num_features, bias) for [add_bias(]feature_hashing(col[, 'opts'])[)], else None."""
    bias = False
    e = expr
    if isinstance(e, Func) and e.name.lower() == "add_bias" and len(e.args) == 1 and e.window is None:
        bias, e = True, e.args[0]
    if not (isinstance(e, Func) and e.name.lower() == "feature_hashing" and e.window is None
            and 1 <= len(e.args) <= 2 and not e.distinct):
        return None
    nf = DEFAULT_NUM_FEATURES
    if len(e.args) == 2:
        if not (isinstance(e.args[1], Lit) and isinstance(e.args[1].value, str)):
            return None
        from ..ftvec.functions import _FH_OPTS

        cl = _FH_OPTS.parse(e.args[1].value)
        nf = int(cl["num_features"])
    col = e.args[0]
    if not isinstance(col, Col):
        return None
    return col, nf, bias


def try_device_features(session, expr, src, ctes):
    """The learner feature argument ``expr`` as ``DeviceFeatures`` when it can be evaluated on
    the session's GPU (module docstring), else None."""
    if not enabled():
        return None
    dev = getattr(session, "device", None)
    if dev is None or str(dev).split(":")[0] != "cuda":
        return None
    m = _match(expr)
    if m is None:
        return None
    col, nf, bias = m
    from ..ftvec.functions import _list_column

    s = session.eval(col, src, ctes)
    arr = _list_column(s) if hasattr(s, "dtype") else None
    if arr is None:
        return None
    from ..io.ingest import hashed_csr_device

    return hashed_csr_device(arr, nf, bias, device=dev)
