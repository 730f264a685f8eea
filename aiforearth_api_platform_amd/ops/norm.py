"""GroupNorm (+ReLU) [K2] and bilinear 2x upsample [K3] on NHWC tensors, with concat-slice outputs."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _ext

_GN_CHUNK = []


def _gn_chunk_px() -> int:
    """Pixels per GroupNorm statistics chunk, from the kernel library (csrc/kernels/norm_resample.hip
    GN_PIX_PER_BLOCK): the workspace of ``ai4e_groupnorm_nhwc`` is sized from it."""
    if not _GN_CHUNK:
        # a library from before the export used 1024-pixel chunks
        _GN_CHUNK.append(_ext.call_int("ai4e_gn_chunk_px") if _ext.has("ai4e_gn_chunk_px") else 1024)
    return _GN_CHUNK[0]


def _nhwc_ld(t: torch.Tensor):
    """(row stride in channels, channel offset) of an NHWC tensor that may be a channel slice."""
    n, h, w, c = t.shape
    if t.stride(3) != 1 or t.stride(1) != w * t.stride(2) or t.stride(0) != h * t.stride(1):
        raise ValueError("expected an NHWC (possibly channel-sliced) dense tensor")
    return t.stride(2), t.storage_offset() % t.stride(2)


def _base_ptr(t: torch.Tensor) -> int:
    ld, coff = _nhwc_ld(t)
    return t.untyped_storage().data_ptr() + t.element_size() * (t.storage_offset() - coff)


def group_norm_affine(stats, gamma: torch.Tensor, beta: torch.Tensor, n: int, hw: int, c: int, groups: int = 32,
                      eps: float = 1e-5) -> torch.Tensor:
    """The per-(image, channel) affine (a, b) of a GroupNorm whose statistics a conv epilogue produced (``stats`` =
    ``(partials, nchunks)``), without applying it: float32 [N, C, 2] (a view into the partials buffer) for a consumer
    that normalizes while loading (``conv.conv3x3_tile64`` ``pro``)."""
    partials, nchunks = stats
    g32 = gamma.to(partials.device, torch.float32).contiguous()
    b32 = beta.to(partials.device, torch.float32).contiguous()
    _ext.call("ai4e_groupnorm_finalize", partials.data_ptr(), g32.data_ptr(), b32.data_ptr(), n, hw, c, groups, eps,
              nchunks, _ext.stream_ptr(partials.device))
    off = n * nchunks * groups * 4
    return partials[off:off + n * c * 2].view(n, c, 2)


def gn_relu_head8_supported(z: torch.Tensor, pc) -> bool:
    """Shapes ``gn_relu_head8`` takes: bf16 NHWC z with 64 channels (may be a channel slice), H * W % 32 == 0, and a
    1x1 / stride-1 conv of 64 -> 8 output channels (the U-Net head with its classes padded to 8)."""
    n, h, w, c = z.shape
    return (_ext.backend_for(z) == "hip" and z.dtype == torch.bfloat16 and c == 64 and (h * w) % 32 == 0
            and (pc.kh, pc.kw) == (1, 1) and pc.stride == 1 and pc.pad == 0 and pc.cin_pad == 64 and pc.cout == 8
            and pc.w_packed.dtype == torch.bfloat16 and z.stride(3) == 1 and z.stride(2) % 8 == 0
            and z.stride(1) == w * z.stride(2) and z.stride(0) == h * z.stride(1))


def gn_relu_head8(z: torch.Tensor, ss: torch.Tensor, pc) -> torch.Tensor:
    """``conv1x1(relu(z * a + b)) + bias`` for 64 -> 8 channels in one pass over ``z`` (csrc/kernels/norm_resample.hip
    gn_relu_head8_kernel): ``ss`` float32 [N, 64, 2] is the GroupNorm affine from ``group_norm_affine``; the normalized
    tensor is never written. Returns [N, H, W, 8] bf16."""
    n, h, w, c = z.shape
    if not gn_relu_head8_supported(z, pc):
        raise ValueError("gn_relu_head8: unsupported shape / layout (see gn_relu_head8_supported)")
    ldz, zoff = _nhwc_ld(z)
    y = torch.empty(n, h, w, 8, device=z.device, dtype=torch.bfloat16)
    _ext.call("ai4e_gn_relu_head8", _base_ptr(z), ldz, zoff, ss.data_ptr(), pc.w_packed.data_ptr(), pc.kpad,
              pc.bias.data_ptr(), y.data_ptr(), n, h * w, _ext.stream_ptr(z.device))
    return y


def group_norm_nhwc(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, groups: int = 32, eps: float = 1e-5,
                    relu: bool = False, out: Optional[torch.Tensor] = None, stats=None,
                    pool_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``stats``: ``(partials, nchunks)`` from ``conv2d_gn_nhwc`` (the producing conv's epilogue already summed
    the groups), which skips the statistics pass. ``pool_out``: contiguous [N, H/2, W/2, C] that also receives the
    2x2/2 max-pool of the result (from the same pass when ``stats`` is given)."""
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty(n, h, w, c, device=x.device, dtype=x.dtype)
    if _ext.backend_for(x) == "hip":
        ldx, xcoff = _nhwc_ld(x)
        ldy, ycoff = _nhwc_ld(out)
        c8 = c // 8
        if (stats is not None and pool_out is not None and h % 2 == 0 and w % 2 == 0 and c % 8 == 0
                and c8 <= 256 and 256 % c8 == 0 and pool_out.is_contiguous()
                and tuple(pool_out.shape) == (n, h // 2, w // 2, c)):
            partials, nchunks = stats
            g32 = gamma.to(x.device, torch.float32).contiguous()
            b32 = beta.to(x.device, torch.float32).contiguous()
            _ext.call("ai4e_groupnorm_apply_pool_nhwc", _base_ptr(x), _base_ptr(out), g32.data_ptr(),
                      b32.data_ptr(), partials.data_ptr(), pool_out.data_ptr(), n, h, w, c, groups, eps, int(relu),
                      ldx | (ldy << 16), xcoff | (ycoff << 16), nchunks, _ext.stream_ptr(x.device))
            return out
        if pool_out is not None:
            group_norm_nhwc(x, gamma, beta, groups, eps, relu, out, stats)
            from .pool import maxpool2d_nhwc
            pool_out.copy_(maxpool2d_nhwc(out, 2, 2, 0))
            return out
        if stats is not None:
            partials, nchunks = stats
            g32 = gamma.to(x.device, torch.float32).contiguous()
            b32 = beta.to(x.device, torch.float32).contiguous()
            _ext.call("ai4e_groupnorm_apply_nhwc", _base_ptr(x), _base_ptr(out), g32.data_ptr(), b32.data_ptr(),
                      partials.data_ptr(), n, h * w, c, groups, eps, int(relu), ldx | (ldy << 16),
                      xcoff | (ycoff << 16), nchunks, _ext.stream_ptr(x.device))
            return out
        chunk = _gn_chunk_px()
        nchunks = (h * w + chunk - 1) // chunk
        # chunk partials, then the per-channel affine (scale, shift) the finalize launch writes
        partials = torch.empty(n * nchunks * groups * 4 + n * c * 2, device=x.device, dtype=torch.float32)
        g32 = gamma.to(x.device, torch.float32).contiguous()
        b32 = beta.to(x.device, torch.float32).contiguous()
        _ext.call("ai4e_groupnorm_nhwc", _base_ptr(x), _base_ptr(out), g32.data_ptr(), b32.data_ptr(),
                  partials.data_ptr(), n, h * w, c, groups, eps, int(relu), ldx | (ldy << 16), xcoff | (ycoff << 16),
                  _ext.stream_ptr(x.device))
        return out
    y = F.group_norm(x.permute(0, 3, 1, 2).float(), groups, gamma.float().to(x.device), beta.float().to(x.device), eps)
    if relu:
        y = F.relu(y)
    out.copy_(y.permute(0, 2, 3, 1).to(out.dtype))
    if pool_out is not None:
        pool_out.copy_(F.max_pool2d(out.permute(0, 3, 1, 2).float(), 2, 2).permute(0, 2, 3, 1).to(pool_out.dtype))
    return out


def upsample2x_nhwc(x: torch.Tensor, out: Optional[torch.Tensor] = None, out_coff: int = 0) -> torch.Tensor:
    """Bilinear x2 (align_corners=False). ``out`` may be a wider concat buffer; writes channels
    [out_coff, out_coff + C)."""
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty(n, 2 * h, 2 * w, c, device=x.device, dtype=x.dtype)
        out_coff = 0
    if _ext.backend_for(x) == "hip":
        x = x.contiguous()
        if out.stride(3) != 1:
            raise ValueError("bad output buffer")
        _ext.call("ai4e_upsample2x_bilinear", x.data_ptr(), out.data_ptr(), n, h, w, c, out.stride(2), out_coff, 0,
                  _ext.stream_ptr(x.device))
        return out
    y = F.interpolate(x.permute(0, 3, 1, 2).float(), scale_factor=2, mode="bilinear", align_corners=False)
    out[..., out_coff:out_coff + c] = y.permute(0, 2, 3, 1).to(out.dtype)
    return out
