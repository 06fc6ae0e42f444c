"""Sketches, geospatial, dataset generator (upstream core/src/main/java/
hivemall/{sketch/hll/ApproxCountDistinctUDAF,sketch/bloom/*,geospatial/*,
dataset/LogisticRegressionDataGeneratorUDTF}.java)."""
from __future__ import annotations

import base64
import math
import random

import numpy as np

from ..registry import udaf, udf, udtf
from ..utils.hashing import murmurhash3


# ------------------------------------------------------------------ HyperLogLog++
class HyperLogLog:
    """HyperLogLog with 2^p registers, 64-bit hashing (two murmur3 halves) and the standard
    small-range (linear counting) correction — the estimator behind approx_count_distinct."""

    def __init__(self, p: int = 15):
        self.p = int(p)
        self.m = 1 << self.p
        self.reg = np.zeros(self.m, dtype=np.uint8)

    @staticmethod
    def _h64(v) -> int:
        s = str(v)
        return ((murmurhash3(s, seed=0x9747B28C) & 0xFFFFFFFF) << 32) | (murmurhash3(s, seed=0x5BD1E995) & 0xFFFFFFFF)

    def add(self, v) -> None:
        h = self._h64(v)
        idx = h >> (64 - self.p)
        w = (h << self.p) & ((1 << 64) - 1)
        rho = 1
        while rho <= 64 - self.p and not (w & (1 << 63)):
            rho += 1
            w = (w << 1) & ((1 << 64) - 1)
        if rho > self.reg[idx]:
            self.reg[idx] = rho

    def merge(self, other: "HyperLogLog") -> None:
        np.maximum(self.reg, other.reg, out=self.reg)

    def cardinality(self) -> int:
        m = self.m
        alpha = 0.7213 / (1 + 1.079 / m)
        z = 1.0 / np.sum(np.power(2.0, -self.reg.astype(np.float64)))
        e = alpha * m * m * z
        zeros = int((self.reg == 0).sum())
        if e <= 2.5 * m and zeros:
            e = m * math.log(m / zeros)
        return int(round(e))


@udaf("approx_count_distinct")
def approx_count_distinct(values, options=None):
    p = 15
    o = options[0] if isinstance(options, (list, tuple)) and options else options
    if o:
        toks = str(o).split()
        if "-p" in toks:
            p = int(toks[toks.index("-p") + 1])
    h = HyperLogLog(p)
    for v in values:
        if v is not None:
            h.add(v)
    return h.cardinality()


# ------------------------------------------------------------------ Bloom filters
class Bloom:
    def __init__(self, m: int = 1 << 16, k: int = 4, bits: np.ndarray | None = None):
        self.m, self.k = int(m), int(k)
        self.bits = bits if bits is not None else np.zeros(self.m // 8, dtype=np.uint8)

    def _idx(self, v):
        s = str(v)
        h1 = murmurhash3(s, seed=0) & 0xFFFFFFFF
        h2 = murmurhash3(s, seed=h1) & 0xFFFFFFFF
        return [(h1 + i * h2) % self.m for i in range(self.k)]

    def add(self, v):
        for i in self._idx(v):
            self.bits[i >> 3] |= 1 << (i & 7)

    def contains(self, v) -> bool:
        return all(self.bits[i >> 3] >> (i & 7) & 1 for i in self._idx(v))

    def serialize(self) -> str:
        return f"{self.m}:{self.k}:" + base64.b64encode(self.bits.tobytes()).decode()

    @staticmethod
    def deserialize(s: str) -> "Bloom":
        m, k, b = s.split(":", 2)
        return Bloom(int(m), int(k), np.frombuffer(base64.b64decode(b), dtype=np.uint8).copy())


@udaf("bloom")
def bloom(values):
    b = Bloom()
    for v in values:
        if v is not None:
            b.add(v)
    return b.serialize()


@udf("bloom_and")
def bloom_and(a, b):
    A, B = Bloom.deserialize(a), Bloom.deserialize(b)
    return Bloom(A.m, A.k, A.bits & B.bits).serialize()


@udf("bloom_or")
def bloom_or(a, b):
    A, B = Bloom.deserialize(a), Bloom.deserialize(b)
    return Bloom(A.m, A.k, A.bits | B.bits).serialize()


@udf("bloom_not")
def bloom_not(a):
    A = Bloom.deserialize(a)
    return Bloom(A.m, A.k, ~A.bits).serialize()


@udf("bloom_contains")
def bloom_contains(a, key):
    return None if a is None else Bloom.deserialize(a).contains(key)


@udf("bloom_contains_any")
def bloom_contains_any(a, keys):
    B = Bloom.deserialize(a)
    return any(B.contains(k) for k in keys)


# ------------------------------------------------------------------ geospatial (slippy tiles)
@udf("lat2tiley")
def lat2tiley(lat, zoom):
    lat_r = math.radians(float(lat))
    n = 1 << int(zoom)
    return int((1.0 - math.log(math.tan(lat_r) + 1.0 / math.cos(lat_r)) / math.pi) / 2.0 * n)


@udf("lon2tilex")
def lon2tilex(lon, zoom):
    n = 1 << int(zoom)
    return int((float(lon) + 180.0) / 360.0 * n)


@udf("tilex2lon")
def tilex2lon(x, zoom):
    return float(x) / (1 << int(zoom)) * 360.0 - 180.0


@udf("tiley2lat")
def tiley2lat(y, zoom):
    n = math.pi - 2.0 * math.pi * float(y) / (1 << int(zoom))
    return math.degrees(math.atan(math.sinh(n)))


@udf("tile")
def tile(lat, lon, zoom):
    """Tile number ``y * 2^zoom + x``."""
    z = int(zoom)
    return lat2tiley(lat, z) * (1 << z) + lon2tilex(lon, z)


@udf("map_url")
def map_url(lat, lon, zoom, option: str = "-osm"):
    z = int(zoom)
    x, y = lon2tilex(lon, z), lat2tiley(lat, z)
    if "google" in str(option):
        return f"https://www.google.com/maps/@{lat},{lon},{z}z"
    return f"https://tile.openstreetmap.org/{z}/{x}/{y}.png"


@udf("haversine_distance")
def haversine_distance(lat1, lon1, lat2, lon2, mile: bool = False):
    R = 3958.8 if mile else 6371.0
    p1, p2 = math.radians(lat1), math.radians(lat2)
    dp, dl = p2 - p1, math.radians(lon2 - lon1)
    a = math.sin(dp / 2) ** 2 + math.cos(p1) * math.cos(p2) * math.sin(dl / 2) ** 2
    return 2 * R * math.asin(min(1.0, math.sqrt(a)))


# ------------------------------------------------------------------ dataset
@udtf("lr_datagen", per_row=False, cols=("label", "features"))
def lr_datagen(options=None):
    """Synthetic logistic-regression data (LogisticRegressionDataGeneratorUDTF):
    ``-n_examples -n_features -n_dims -eps -prob_one -seed -dense -sort -cl``."""
    import pandas as pd
    o = options[0] if isinstance(options, (list, tuple)) else options
    kv = {"n_examples": 1000, "n_features": 10, "n_dims": 200, "eps": 3.0, "prob_one": 0.6,
          "seed": 43}
    flags = set()
    if o:
        toks = str(o).split()
        i = 0
        while i < len(toks):
            k = toks[i].lstrip("-")
            if k in kv:
                kv[k] = type(kv[k])(toks[i + 1])
                i += 2
            else:
                flags.add(k)
                i += 1
    rng = np.random.default_rng(kv["seed"])
    rows = []
    for _ in range(kv["n_examples"]):
        y = 1 if rng.random() < kv["prob_one"] else 0
        if "dense" in flags:
            x = rng.normal(size=kv["n_dims"]) + (kv["eps"] if y else -kv["eps"]) / kv["n_dims"]
            feats = [float(v) for v in x]
        else:
            idx = rng.choice(kv["n_dims"], size=kv["n_features"], replace=False) + 1
            if "sort" in flags:
                idx = np.sort(idx)
            vals = rng.normal(size=kv["n_features"]) + (0.5 if y else -0.5) * kv["eps"] / 3
            feats = [f"{i}:{v:.6f}" for i, v in zip(idx, vals)]
        rows.append((y if "cl" in flags or True else float(y), feats))
    return pd.DataFrame(rows, columns=["label", "features"])
