"""Preprocess (K7), max-pool and global-avg-pool (K8 front half) on NHWC bf16."""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch
import torch.nn.functional as F

from . import _ext

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def preprocess_u8(img: torch.Tensor, mean: Sequence[float] = IMAGENET_MEAN, std: Sequence[float] = IMAGENET_STD,
                  scale: float = 1.0 / 255.0, out: torch.Tensor = None) -> torch.Tensor:
    """uint8 NHWC [N,H,W,Cin<=8] -> normalized bf16 NHWC [N,H,W,8] (channels >= Cin are zero)."""
    n, h, w, cin = img.shape
    if img.dtype != torch.uint8 or cin > 8:
        raise ValueError("preprocess expects uint8 NHWC with <= 8 channels")
    m8 = list(mean) + [0.0] * (8 - len(mean))
    s8 = list(std) + [1.0] * (8 - len(std))
    if out is None:
        out = torch.empty(n, h, w, 8, device=img.device, dtype=torch.bfloat16 if img.is_cuda else torch.float32)
    if _ext.backend_for(img) == "hip":
        mean_a, std_a = ctypes_floats(m8), ctypes_floats(s8)  # kept alive across the call
        _ext.call("ai4e_preprocess_u8", img.data_ptr(), out.data_ptr(), n * h * w, cin, ctypes.addressof(mean_a),
                  ctypes.addressof(std_a), scale, _ext.stream_ptr(img.device))
    else:
        x = img.float() * scale
        x = (x - torch.tensor(m8[:cin], device=img.device)) / torch.tensor(s8[:cin], device=img.device)
        out.zero_()
        out[..., :cin] = x.to(out.dtype)
    return out


def preprocess_s2d_u8(img: torch.Tensor, mean: Sequence[float] = IMAGENET_MEAN, std: Sequence[float] = IMAGENET_STD,
                      scale: float = 1.0 / 255.0, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """uint8 NHWC [N,H,W,cin<=4] -> normalized, 2x2 space-to-depth [N,H/2,W/2,16] (bf16, or fp16) for the s2d
    stem: ``out[i, j, (dy*2+dx)*cin + c] = norm(x[2i+dy-1, 2j+dx-1, c])`` (zero outside the image)."""
    n, h, w, cin = img.shape
    if img.dtype != torch.uint8 or cin > 4 or h % 2 or w % 2:
        raise ValueError("s2d preprocess expects uint8 NHWC, <= 4 channels, even H and W")
    m4 = list(mean) + [0.0] * (4 - len(mean))
    s4 = list(std) + [1.0] * (4 - len(std))
    if _ext.backend_for(img) == "hip":
        out = torch.empty(n, h // 2, w // 2, 16, device=img.device, dtype=dtype)
        ma, sa = ctypes_floats(m4), ctypes_floats(s4)
        _ext.call("ai4e_preprocess_s2d_u8_dt", img.data_ptr(), out.data_ptr(), n, h, w, cin, ctypes.addressof(ma),
                  ctypes.addressof(sa), scale, int(dtype == torch.float16), _ext.stream_ptr(img.device))
        return out
    x = (img.float() * scale - torch.tensor(m4[:cin], device=img.device)) / torch.tensor(s4[:cin], device=img.device)
    y = space_to_depth_shifted(x)
    return y.to(dtype) if img.is_cuda else y


def space_to_depth_shifted(x: torch.Tensor) -> torch.Tensor:
    """Normalized NHWC [N,H,W,C<=4] -> [N,H/2,W/2,16] with the -1 pixel shift of the s2d stem."""
    n, h, w, c = x.shape
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1, 1, 1))[:, : h, : w]   # xp[y, x] = x[y-1, x-1]
    blocks = xp.reshape(n, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 2, 4, 5).reshape(n, h // 2, w // 2, 4 * c)
    out = torch.zeros(n, h // 2, w // 2, 16, dtype=x.dtype, device=x.device)
    out[..., : 4 * c] = blocks
    return out


def ctypes_floats(vals):
    return (ctypes.c_float * len(vals))(*vals)


def maxpool2d_nhwc(x: torch.Tensor, k: int = 3, stride: int = 2, pad: int = 1) -> torch.Tensor:
    n, h, w, c = x.shape
    oh, ow = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    if _ext.backend_for(x) == "hip":
        if x.stride(3) != 1 or x.stride(1) != w * x.stride(2) or x.stride(0) != h * x.stride(1):
            x = x.contiguous()  # channel slices of an NHWC buffer are read in place
        y = torch.empty(n, oh, ow, c, device=x.device, dtype=x.dtype)
        _ext.call("ai4e_maxpool2d_dt", x.data_ptr(), y.data_ptr(), n, h, w, c, oh, ow, k, stride, pad, x.stride(2),
                  int(x.dtype == torch.float16), _ext.stream_ptr(x.device))
        return y
    y = F.max_pool2d(x.permute(0, 3, 1, 2).float(), k, stride, pad)
    return y.permute(0, 2, 3, 1).to(x.dtype).contiguous()


def global_avgpool_nhwc(x: torch.Tensor) -> torch.Tensor:
    """[N,H,W,C] -> [N,1,1,C] (kept 4-D so the classifier runs as a 1x1 conv)."""
    n, h, w, c = x.shape
    if _ext.backend_for(x) == "hip":
        x = x.contiguous()
        y = torch.empty(n, 1, 1, c, device=x.device, dtype=x.dtype)
        _ext.call("ai4e_global_avgpool_dt", x.data_ptr(), y.data_ptr(), n, h * w, c, int(x.dtype == torch.float16),
                  _ext.stream_ptr(x.device))
        return y
    return x.float().mean(dim=(1, 2), keepdim=True).to(x.dtype)
