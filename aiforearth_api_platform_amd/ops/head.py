"""Classifier head epilogue: softmax + top-k in one HIP kernel (``csrc/kernels/head.hip``).

``softmax_topk(logits, k)`` -> ``(idx int32 [N,k], prob fp32 [N,k])``, sorted by descending probability,
ties to the lower class index. Replaces cast + ``torch.softmax`` + ``torch.topk`` (+ sort + index cast):
five launches in the serving engine's graph tail. The PyTorch path is the reference.
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _ext


def softmax_topk(logits: torch.Tensor, k: int = 5) -> Tuple[torch.Tensor, torch.Tensor]:
    n, c = logits.shape
    if _ext.backend_for(logits) != "hip" or logits.dtype != torch.bfloat16 or c > 2048 or logits.stride(1) != 1:
        p, i = torch.topk(torch.softmax(logits.float(), dim=1), k, dim=1)
        return i.to(torch.int32), p
    idx = torch.empty(n, k, device=logits.device, dtype=torch.int32)
    prob = torch.empty(n, k, device=logits.device, dtype=torch.float32)
    _ext.call("ai4e_softmax_topk", logits.data_ptr(), logits.stride(0), n, c, k, idx.data_ptr(), prob.data_ptr(),
              _ext.stream_ptr(logits.device))
    return idx, prob
