"""Seeded pseudo-random number generators (upstream
core/src/main/java/hivemall/math/random/{PRNG,RandomNumberGeneratorFactory,JavaRandom,
SmileRandom,CommonsMathRandom}.java).

* ``JavaRandom`` reproduces ``java.util.Random`` bit for bit: the 48-bit LCG
  (multiplier 0x5DEECE66D, addend 0xB, seed scrambled with the multiplier), ``nextInt``,
  bounded ``nextInt(n)`` with Java's rejection rule in 32-bit arithmetic, ``nextLong``,
  ``nextDouble`` (26 + 27 bits), ``nextFloat`` and the polar-method ``nextGaussian`` with its
  cached second value.  ``rand_amplify`` (reservoir draws) and ``bpr_sampling`` (per-user
  negative draws) take their streams from it, so a ``-seed`` replays the same rows in every
  process.  The learners' weight init draws on the device (below), not from this class.
* ``SmileRandom`` / ``CommonsMathRandom`` are Mersenne-Twister generators upstream; here both
  wrap numpy's MT19937 seeded with the same integer (stream parity with Smile / commons-math
  is unpinned: their seeding routines differ from numpy's).

Device code does not draw from these: the GPU kernels use counter-based hashes of
(seed, row, slot) so every wave draws independently without shared state.
"""
from __future__ import annotations

from abc import ABC, abstractmethod

import math

import numpy as np

_MULT = 0x5DEECE66D
_ADD = 0xB
_MASK = (1 << 48) - 1


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def _i64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


class PRNG(ABC):
    """Interface of upstream ``hivemall.math.random.PRNG``."""

    @abstractmethod
    def next_int(self, bound: int | None = None) -> int:
        ...

    @abstractmethod
    def next_long(self) -> int:
        ...

    @abstractmethod
    def next_double(self) -> float:
        ...

    @abstractmethod
    def next_gaussian(self) -> float:
        ...

    # Java-style aliases
    def nextInt(self, bound: int | None = None) -> int:  # noqa: N802
        return self.next_int(bound)

    def nextLong(self) -> int:  # noqa: N802
        return self.next_long()

    def nextDouble(self) -> float:  # noqa: N802
        return self.next_double()

    def nextGaussian(self) -> float:  # noqa: N802
        return self.next_gaussian()


class JavaRandom(PRNG):
    """Bit-exact ``java.util.Random``."""

    def __init__(self, seed: int):
        self.set_seed(seed)

    def set_seed(self, seed: int) -> None:
        self._seed = (int(seed) ^ _MULT) & _MASK
        self._next_gaussian: float | None = None

    def _next(self, bits: int) -> int:
        self._seed = (self._seed * _MULT + _ADD) & _MASK
        return _i32(self._seed >> (48 - bits))

    def next_int(self, bound: int | None = None) -> int:
        if bound is None:
            return self._next(32)
        if bound <= 0:
            raise ValueError("bound must be positive")
        r = self._next(31)
        m = bound - 1
        if bound & m == 0:    # power of two: the high bits
            return _i32((bound * r) >> 31)
        u = r
        r = u % bound
        while _i32(u - r + m) < 0:   # Java's overflow test in int arithmetic
            u = self._next(31)
            r = u % bound
        return r

    def next_long(self) -> int:
        return _i64((self._next(32) << 32) + self._next(32))

    def next_boolean(self) -> bool:
        return self._next(1) != 0

    def next_float(self) -> float:
        return self._next(24) / float(1 << 24)

    def next_double(self) -> float:
        return ((self._next(26) << 27) + self._next(27)) * (1.0 / (1 << 53))

    def next_gaussian(self) -> float:
        if self._next_gaussian is not None:
            g, self._next_gaussian = self._next_gaussian, None
            return g
        while True:
            v1 = 2.0 * self.next_double() - 1.0
            v2 = 2.0 * self.next_double() - 1.0
            s = v1 * v1 + v2 * v2
            if 0.0 < s < 1.0:
                break
        mul = math.sqrt(-2.0 * math.log(s) / s)
        self._next_gaussian = v2 * mul
        return v1 * mul


class _MTRandom(PRNG):
    """Mersenne Twister (numpy MT19937) behind the PRNG interface."""

    def __init__(self, seed: int):
        self._rs = np.random.RandomState(int(seed) & 0xFFFFFFFF)

    def next_int(self, bound: int | None = None) -> int:
        if bound is None:
            return _i32(int(self._rs.randint(0, 1 << 32, dtype=np.uint64)))
        if bound <= 0:
            raise ValueError("bound must be positive")
        return int(self._rs.randint(0, bound))

    def next_long(self) -> int:
        return _i64(int(self._rs.randint(0, 1 << 63, dtype=np.uint64)) << 1 | int(self._rs.randint(0, 2)))

    def next_double(self) -> float:
        return float(self._rs.random_sample())

    def next_gaussian(self) -> float:
        return float(self._rs.standard_normal())


class SmileRandom(_MTRandom):
    """Stands in for Smile's ``MersenneTwister`` (used by RF/GBT bootstraps upstream)."""


class CommonsMathRandom(_MTRandom):
    """Stands in for commons-math3 ``MersenneTwister``."""


def create(kind: str = "java", seed: int | None = None) -> PRNG:
    """``RandomNumberGeneratorFactory.createPRNG``: ``java`` | ``smile`` | ``commons``;
    ``seed=None`` draws one from the OS (upstream: ``System.nanoTime()``-based)."""
    if seed is None:
        seed = int.from_bytes(np.random.default_rng().bytes(8), "little") & ((1 << 63) - 1)
    kind = kind.lower()
    if kind in ("java", "javarandom"):
        return JavaRandom(seed)
    if kind in ("smile", "smilerandom"):
        return SmileRandom(seed)
    if kind in ("commons", "commonsmath", "commonsmath3", "commonsmathrandom"):
        return CommonsMathRandom(seed)
    raise ValueError(f"unknown PRNG type {kind!r}")
