"""Scalar min / max of index tensors.  On the CPU, torch's integer reductions in this build are
~100x slower than numpy's (int32 max over 440 K a9a indices: 64 ms vs 0.5 ms), which made the
shape probes of a learner's fit cost more than its a9a epochs; device tensors reduce on the device."""
from __future__ import annotations

import torch


def tmax(t: torch.Tensor) -> int | float:
    if t.device.type == "cpu":
        return t.numpy().max().item()
    return t.max().item()


def tmin(t: torch.Tensor) -> int | float:
    if t.device.type == "cpu":
        return t.numpy().min().item()
    return t.min().item()
