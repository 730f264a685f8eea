"""Tiny models for plumbing tests and the CPU "echo" configuration (BASELINE config #1)."""
from __future__ import annotations

import torch


class ChannelMeanClassifier:
    """logits[b] = [mean(channel 0..C-1), 0, 0, 0]: deterministic, cheap, device-agnostic."""

    def __init__(self, device="cpu", extra_classes: int = 3, delay_ms: float = 0.0):
        self.device = torch.device(device)
        self.extra = extra_classes
        self.delay_s = float(delay_ms) / 1e3  # a slow "GPU" per batch (admission / overload tests)

    def __call__(self, x_u8: torch.Tensor) -> torch.Tensor:
        if self.delay_s:
            import time

            time.sleep(self.delay_s)
        m = x_u8.float().mean(dim=(1, 2))
        return torch.cat([m, torch.zeros(m.shape[0], self.extra, device=m.device)], dim=1)


def tiny_classifier(device="cpu", **kw):
    return ChannelMeanClassifier(device, **kw)


def echo(task_id: str, body: bytes, headers=None):
    """Sync echo backend (BASELINE config #1: plumbing, no GPU)."""
    return 200, body


class NullClassifier:
    """logits = zeros (never reads the pixels): a worker that costs nothing, so an ingest benchmark on CPU measures
    the front door alone (runtime/node_bench.py ingest probes)."""

    def __init__(self, device="cpu", classes: int = 4):
        self.device = torch.device(device)
        self.classes = classes

    def __call__(self, x_u8: torch.Tensor) -> torch.Tensor:
        return torch.zeros(x_u8.shape[0], self.classes, device=x_u8.device)


def null_classifier(device="cpu", **kw):
    return NullClassifier(device, **kw)
