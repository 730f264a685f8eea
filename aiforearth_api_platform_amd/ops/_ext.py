"""Loader for the in-tree gfx950 kernel library (``_lib/libai4e_kernels.so``) via a plain C ABI.

Every launcher takes raw device pointers plus the current HIP stream, so kernels compose with
PyTorch's caching allocator, streams and HIP-graph capture (``torch.cuda.graph``) with no torch
headers in the kernel translation units.

Backend policy (``AI4E_KERNEL_BACKEND``): ``auto`` runs the HIP kernels for tensors on the GPU
and the PyTorch reference ops on CPU; ``hip`` forces the kernels; ``torch`` forces the reference
ops. A GPU tensor with the library missing is a hard error — never a silent fallback.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import torch

_LIB_PATH = Path(__file__).resolve().parent.parent / "_lib" / "libai4e_kernels.so"
if os.environ.get("AI4E_KERNEL_LIB"):  # A/B of two builds of the kernel library on one GPU box
    _LIB_PATH = Path(os.environ["AI4E_KERNEL_LIB"])
_lib: Optional[ctypes.CDLL] = None

_c_int, _c_long, _c_float, _vp = ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_void_p

# name -> argtypes (all return int status)
_SIGS = {
    "ai4e_conv2d_fwd": [_vp, _vp, _vp, _vp, _vp] + [_c_int] * 19 + [_vp],
    "ai4e_conv2d_f16_fwd": [_vp, _vp, _vp, _vp, _vp] + [_c_int] * 19 + [_vp],
    "ai4e_conv2d_gn_fwd": [_vp, _vp, _vp, _vp, _vp] + [_c_int] * 19 + [_vp, _c_int, _vp],
    "ai4e_conv2d_head_fwd": [_vp, _vp, _vp, _vp, _vp] + [_c_int] * 19 + [_vp, _c_int, _vp, _vp, _vp],
    "ai4e_conv2d_sk_fwd": [_vp, _vp, _vp, _vp, _vp] + [_c_int] * 20 + [_vp, _vp, _vp],
    "ai4e_conv_chain_fwd": [_vp] * 10 + [_c_int] * 11 + [_vp, _c_int, _vp],
    "ai4e_conv_chain_f16_fwd": [_vp] * 10 + [_c_int] * 11 + [_vp, _c_int, _vp],
    "ai4e_conv_pair_fwd": [_vp] * 8 + [_c_int] * 5 + [_vp],
    "ai4e_conv_pair_f16_fwd": [_vp] * 8 + [_c_int] * 5 + [_vp],
    "ai4e_stem_pool_c1_f16_fwd": [_vp] * 7 + [_c_int] * 5 + [_vp],
    "ai4e_stem_pool_fwd": [_vp] * 4 + [_c_int] * 5 + [_vp],
    "ai4e_stem_pool_c1_fwd": [_vp] * 7 + [_c_int] * 5 + [_vp],
    "ai4e_stem_pool_c1_u8_fwd": [_vp] * 3 + [_c_float] + [_vp] * 6 + [_c_int] * 5 + [_vp],
    "ai4e_stem_stamps_read": [_vp],
    "ai4e_chain_stamps_read": [_vp],
    "ai4e_k256_stamps_read": [_vp],  # (AI4E_K256_STAMPS diagnostic builds only)
    "ai4e_pair_stamps_read": [_vp],  # (AI4E_PAIR_STAMPS diagnostic builds only)
    "ai4e_softmax_topk": [_vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp],
    "ai4e_preprocess_u8": [_vp, _vp, _c_long, _c_int, _vp, _vp, _c_float, _vp],
    "ai4e_preprocess_s2d_u8": [_vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_float, _vp],
    "ai4e_preprocess_s2d_u8_dt": [_vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_float, _c_int, _vp],
    "ai4e_maxpool2d": [_vp, _vp] + [_c_int] * 10 + [_vp],
    "ai4e_maxpool2d_dt": [_vp, _vp] + [_c_int] * 11 + [_vp],
    "ai4e_global_avgpool": [_vp, _vp, _c_int, _c_int, _c_int, _vp],
    "ai4e_global_avgpool_dt": [_vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp],
    "ai4e_groupnorm_nhwc": [_vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_float, _c_int, _c_int,
                            _c_int, _vp],
    "ai4e_groupnorm_apply_nhwc": [_vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_float, _c_int, _c_int,
                                  _c_int, _c_int, _vp],
    "ai4e_groupnorm_apply_pool_nhwc": [_vp] * 6 + [_c_int] * 5 + [_c_float] + [_c_int] * 4 + [_vp],
    "ai4e_upsample2x_bilinear": [_vp, _vp] + [_c_int] * 7 + [_vp],
    "ai4e_nms_mask": [_vp, _c_int, _c_int, _c_float, _vp, _vp],
    "ai4e_nms_reduce": [_vp, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp],
    "ai4e_rpn_decode": [_vp] * 6 + [_c_int] * 7 + [_c_float] * 5 + [_vp],
    "ai4e_row_sort_desc": [_vp, _c_int, _c_int, _vp, _vp],
    "ai4e_sort_select": [_vp, _vp, _vp, _c_int, _c_float, _c_int, _c_int] + [_vp] * 7,
    "ai4e_gather_keep": [_vp, _c_int, _c_int, _c_int] + [_vp] * 8,
    "ai4e_rpn_topk": [_vp] + [_c_int] * 5 + [_vp, _vp],
    "ai4e_det_decode": [_vp] * 6 + [_c_int] * 4 + [_vp] + [_c_float] * 4 + [_c_int, _vp],
    "ai4e_roi_align_nhwc": [_vp, _vp, _vp] + [_c_int] * 7 + [_c_float, _c_int, _c_int, _vp],
    "ai4e_roi_align_fpn_nhwc": [_vp] * 8 + [_c_int] * 6 + [_vp],
    "ai4e_crop_resize_nhwc": [_vp, _vp, _vp, _vp] + [_c_int] * 7 + [_vp],
    "ai4e_tile_stitch": [_vp, _vp, _vp] + [_c_int] * 10 + [_vp],
    "ai4e_groupnorm_finalize": [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_float, _c_int, _vp],
    "ai4e_gn_chunk_px": [],
    "ai4e_gn_relu_head8": [_vp, _c_int, _c_int, _vp, _vp, _c_int, _vp, _vp, _c_int, _c_int, _vp],
    "ai4e_conv3x3_tile_fwd": [_vp, _vp, _vp, _vp, _c_int, _vp] + [_c_int] * 10 + [_vp, _c_int, _vp],
    "ai4e_jpeg_decode": [_vp, _c_int, _c_int, _c_int, _c_long, _c_long, _c_int, _vp],
    "ai4e_crumbs_alloc": [_c_int, _vp, _vp],
    "ai4e_crumb": [_vp, _c_int, _vp],
}


class KernelError(RuntimeError):
    pass


def library_path() -> Path:
    return _LIB_PATH


def available() -> bool:
    return _LIB_PATH.exists()


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise KernelError(f"HIP kernel library not built: {_LIB_PATH} (run python -m aiforearth_api_platform_amd._build)")
        _lib = ctypes.CDLL(str(_LIB_PATH))
        for name, args in _SIGS.items():
            fn = getattr(_lib, name, None)
            if fn is not None:
                fn.argtypes = args
                fn.restype = _c_int
    return _lib


def call(name: str, *args) -> None:
    if name not in _SIGS:  # an untyped ctypes call would truncate pointers and streams to 32-bit ints
        raise KernelError(f"{name}: no argument signature registered in ops/_ext.py _SIGS")
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise KernelError(f"{name} failed with status {rc}")


def call_int(name: str, *args) -> int:
    """A library function that returns a value rather than a status (e.g. ``ai4e_gn_chunk_px``)."""
    if name not in _SIGS:
        raise KernelError(f"{name}: no argument signature registered in ops/_ext.py _SIGS")
    return int(getattr(lib(), name)(*args))


def has(name: str) -> bool:
    """Whether the loaded kernel library exports ``name`` (an A/B build of an older tree may not)."""
    return getattr(lib(), name, None) is not None


def stream_ptr(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def backend_for(t: torch.Tensor) -> str:
    mode = os.environ.get("AI4E_KERNEL_BACKEND", "auto").lower()
    if mode == "torch":
        return "torch"
    if mode == "hip":
        if not t.is_cuda:
            raise KernelError("AI4E_KERNEL_BACKEND=hip but tensor is on CPU")
        lib()
        return "hip"
    if t.is_cuda:
        lib()  # loud failure if the kernels are missing on a GPU box
        return "hip"
    return "torch"
