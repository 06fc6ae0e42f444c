"""Imports every function module (registering its SQL functions) and registers the learners
as table functions: ``SELECT train_xxx(features, label, '-opts') AS (...) FROM t`` trains on
the session device and returns the model table (upstream's UDTF ``close()`` -> forwardModel).
Mirrors ``resources/ddl/define-all.hive``.
"""
from __future__ import annotations

import pandas as pd

from . import registry
from .anomaly import changefinder, sst  # noqa: F401
from .ensemble import argmin_kld  # noqa: F401
from .evaluation import metrics  # noqa: F401
from .ftvec import functions as _ftvec  # noqa: F401
from .knn import cosine_similarity  # noqa: F401
from .misc import approx_count_distinct  # noqa: F401
from .models import ffm_keys  # noqa: F401
from .nlp import tokenize_ja  # noqa: F401
from .tools import functions as _tools  # noqa: F401


def _opt_arg(args, k):
    if len(args) > k and len(args[k]):
        v = args[k][0]
        return None if v is None else str(v)
    return None


def _device(session):
    return None if session is None else session.device


# learner UDTF signatures for the catalogue / DESCRIBE FUNCTION: (inputs, output columns)
_LIN_BIN = ("features, label", "feature, weight[, covar]")
_LIN_MC = ("features, label", "label, feature, weight[, covar]")
_FOREST = ("features, label", "model_id, model_weight, model, var_importance, oob_errors, oob_tests")
SIGNATURES = {
    "train_fm": ("features, target", "feature, Wi, Vif"),
    "train_ffm": ("features, label", "model_id, i, Wi, Vi"),
    "train_mf_sgd": ("user, item, rating", "idx, Pu, Qi, Bu, Bi, mu"),
    "train_mf_adagrad": ("user, item, rating", "idx, Pu, Qi, Bu, Bi, mu"),
    "train_bprmf": ("user, pos_item, neg_item", "idx, Pu, Qi, Bi"),
    "train_slim": ("i, r_i, topKRatesOfI, j, r_j", "i, nn, w"),
    "train_kpa": ("features, label", "h, hk, w0, w1, w2, w3"),
    "train_lda": ("words", "label, word, lambda"),
    "train_plsa": ("words", "label, word, prob"),
    "train_randomforest_classifier": _FOREST,
    "train_randomforest_regressor": _FOREST,
    "train_randomforest_regr": _FOREST,
    "train_gradient_tree_boosting_classifier": (
        "features, label", "iteration, pred_models, intercept, shrinkage, var_importance, oob_error_rate"),
    "train_xgboost": ("features, label", "model_id, model"),
    "train_xgboost_classifier": ("features, label", "model_id, model"),
    "train_xgboost_regr": ("features, target", "model_id, model"),
    "train_multiclass_xgboost_classifier": ("features, label", "model_id, model"),
}


def _signature(name: str):
    if name in SIGNATURES:
        return SIGNATURES[name]
    if "multiclass" in name:
        return _LIN_MC
    if name.endswith("_regr") or name in ("logress", "train_regressor"):
        return ("features, target", "feature, weight[, covar]")
    return _LIN_BIN


def _column(a, arrow_ok: bool):
    """A UDTF argument column: Arrow-backed columns stay Arrow for learners that ingest Arrow
    buffers on the device (``ARROW_INPUT``, e.g. train_ffm), everything else becomes a list."""
    import pandas as pd

    from .io.ingest import DeviceFeatures

    if isinstance(a, DeviceFeatures):
        return a
    if arrow_ok and isinstance(a, pd.Series) and isinstance(a.dtype, pd.ArrowDtype):
        arr = a.array._pa_array
        return arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    if isinstance(a, pd.Series) and isinstance(a.dtype, pd.ArrowDtype):
        return a.array._pa_array.to_pylist()
    if isinstance(a, pd.Series) and a.dtype.kind in "biuf":
        return a.to_numpy()          # labels / targets / ids: no Python object per row
    return a.tolist() if isinstance(a, pd.Series) else list(a)


def _rows(d, rank: int, world: int):
    """Rows rank, rank + world, ... of a list or an Arrow array."""
    if isinstance(d, list):
        return d[rank::world]
    if hasattr(d, "take_rows"):          # io.ingest.DeviceFeatures
        return d.take_rows(rank, world)
    import pyarrow as pa

    return d.take(pa.array(range(rank, len(d), world), type=pa.int64()))


def _dist(session):
    ctx = getattr(session, "ctx", None)
    return ctx if (ctx is not None and ctx.world_size > 1) else None


def _learner_udtf(name, cls_getter, n_data_args=2):
    """Register learner ``name`` as a table function.  In a distributed session the learner's
    ``SQL_DP`` mode decides how the ranks share the work (models/base.py Learner.SQL_DP):

    * ``shard``: rank r trains on input rows r, r + world, ... with a ModelMixer (replicas mixed
      over RCCL; all ranks end with the same model table);
    * ``union``: every rank sees all rows and builds its share of an ensemble (RandomForest
      trees t with t % world == rank); the table is the union of the ranks' tables;
    * ``replicate``: learners without a data-parallel formulation train on all rows on every
      rank (identical tables, no speed-up)."""
    def impl(*args, session=None):
        cls = cls_getter()
        opts = _opt_arg(args, n_data_args)
        data = [_column(a, getattr(cls, "ARROW_INPUT", False)) for a in args[:n_data_args]]
        ctx = _dist(session)
        if ctx is None:
            m = cls(opts, device=_device(session))
            m.fit(*data)
            return m.model_table()
        from .parallel.mix import ModelMixer

        mode = getattr(cls, "SQL_DP", "replicate")
        kw = {}
        if mode == "shard":
            data = [_rows(d, ctx.rank, ctx.world_size) for d in data]
            kw = dict(mixer=ModelMixer(ctx), rank=ctx.rank)
        elif mode == "union":
            kw = dict(mixer=ModelMixer(ctx), rank=ctx.rank)
        m = cls(opts, device=_device(session), **kw)
        m.fit(*data)
        tab = m.model_table()
        if mode == "union":
            import torch.distributed as tdist

            parts = [None] * ctx.world_size
            tdist.all_gather_object(parts, tab)
            tab = pd.concat(parts, ignore_index=True)
        return tab
    impl.wants_session = True
    impl.accepts_series = True      # argument columns arrive as Series (Arrow buffers kept)
    # the feature argument may arrive as device CSR (sql/device_ftvec.py)
    impl.device_features = bool(getattr(cls_getter(), "DEVICE_FEATURES", False))
    ins, outs = _signature(name)
    impl.__doc__ = f"{name}({ins} [, const string options]) -> table ({outs})"
    registry._register(registry.FunctionDef(name, registry.UDTF, impl, per_row=False,
                                            doc=impl.__doc__))


def _register_learners():
    from .models import linear as L
    for n in L.LEARNERS:
        _learner_udtf(n, lambda n=n: L.LEARNERS[n])
    from .models.fm import FMTrainer
    _learner_udtf("train_fm", lambda: FMTrainer)
    from .models.ffm import FFMTrainer
    _learner_udtf("train_ffm", lambda: FFMTrainer)
    _optional_learners()


def _optional_learners():
    import importlib
    for mod in ("mf", "trees", "xgboost", "topicmodel", "recommend", "fm"):
        try:
            m = importlib.import_module(f".models.{mod}", __package__)
        except ModuleNotFoundError as e:
            if e.name and e.name.endswith(f"models.{mod}"):
                continue
            raise
        reg = getattr(m, "register_sql", None)
        if reg is not None:
            reg(_learner_udtf)


_register_learners()
