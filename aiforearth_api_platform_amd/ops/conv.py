"""Fused NHWC conv2d (+folded BN bias, +residual, +ReLU) — HIP implicit-GEMM kernel K1.

``PackedConv`` holds one layer's weights in the kernel layout ``[rows_pad, Kpad]`` bf16 with
``k = (kh, kw, c)`` (c innermost, C padded to a multiple of 8, K to a multiple of 32, rows to the
tile height) and an fp32 bias, plus the reference fp32 weights for the PyTorch path.

``conv2d_nhwc(x, pc, residual=None, relu=False, out=None, out_coff=0)`` runs on NHWC tensors.
``out``/``out_coff`` let a layer write a channel slice of a wider buffer (U-Net skip concat without
a copy). ``x`` may itself be a channel slice view of a wider buffer.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import _ext

K_ALIGN = 64  # K steps of 32 come in pairs: the K1 main loop is unrolled by two
ROW_ALIGN = 256
C_ALIGN = 8


def _round_up(a: int, b: int) -> int:
    return (a + b - 1) // b * b


@dataclass
class PackedConv:
    w_ref: torch.Tensor      # [Cout, Cin, KH, KW] fp32 (BN folded)
    b_ref: torch.Tensor      # [Cout] fp32
    w_packed: torch.Tensor   # [rows_pad, Kpad] bf16
    bias: torch.Tensor       # [rows_pad] fp32
    cin: int
    cin_pad: int
    cout: int
    kh: int
    kw: int
    stride: int
    pad: int
    pad_hi: Optional[int] = None   # bottom/right padding when it differs from the top/left `pad`

    @property
    def kpad(self) -> int:
        return self.w_packed.shape[1]

    def to(self, device) -> "PackedConv":
        return PackedConv(self.w_ref.to(device), self.b_ref.to(device), self.w_packed.to(device), self.bias.to(device),
                          self.cin, self.cin_pad, self.cout, self.kh, self.kw, self.stride, self.pad, self.pad_hi)

    def cast(self, dtype: torch.dtype) -> "PackedConv":
        """The same layer with its packed weights in ``dtype`` (fp16 for the f16 K1 path), re-rounded from the
        fp32 weights (``w_ref``; the packed layout is [Cout, (kh, kw, c)] with zero padding, as pack_conv)."""
        if dtype == self.w_packed.dtype:
            return self
        w = torch.zeros(self.cout, self.kh, self.kw, self.cin_pad, device=self.w_ref.device)
        w[..., :self.w_ref.shape[1]] = self.w_ref.float().permute(0, 2, 3, 1)
        k = self.kh * self.kw * self.cin_pad
        wp = torch.zeros_like(self.w_packed, dtype=dtype)
        wp[:self.cout, :k] = w.reshape(self.cout, k).to(dtype)
        return PackedConv(self.w_ref, self.b_ref, wp, self.bias, self.cin, self.cin_pad, self.cout, self.kh, self.kw,
                          self.stride, self.pad, self.pad_hi)

    def out_hw(self, h: int, w: int):
        hi = self.pad if self.pad_hi is None else self.pad_hi
        return ((h + self.pad + hi - self.kh) // self.stride + 1, (w + self.pad + hi - self.kw) // self.stride + 1)


def pack_conv(weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int = 1, pad: int = 0,
              cin_pad: Optional[int] = None) -> PackedConv:
    """Pack an OIHW fp32 weight (+bias) into the K1 layout."""
    weight = weight.detach().float().cpu()
    cout, cin, kh, kw = weight.shape
    cin_pad = cin_pad or _round_up(cin, C_ALIGN)
    w = torch.zeros(cout, kh, kw, cin_pad)
    w[..., :cin] = weight.permute(0, 2, 3, 1)
    k = kh * kw * cin_pad
    kp = _round_up(k, K_ALIGN)
    rows = _round_up(cout, ROW_ALIGN)
    wp = torch.zeros(rows, kp, dtype=torch.bfloat16)
    wp[:cout, :k] = w.reshape(cout, k).to(torch.bfloat16)
    b = torch.zeros(rows, dtype=torch.float32)
    bref = torch.zeros(cout) if bias is None else bias.detach().float().cpu()
    b[:cout] = bref
    return PackedConv(weight, bref, wp, b, cin, cin_pad, cout, kh, kw, stride, pad)


def fold_bn(weight: torch.Tensor, bn_weight, bn_bias, running_mean, running_var, eps: float = 1e-5,
            conv_bias: Optional[torch.Tensor] = None):
    """Fold inference BatchNorm into the preceding conv: returns (w', b')."""
    scale = bn_weight / torch.sqrt(running_var + eps)
    w = weight * scale.reshape(-1, 1, 1, 1)
    b = bn_bias - running_mean * scale
    if conv_bias is not None:
        b = b + conv_bias * scale
    return w, b


_TILES = None


def tile_key(pc: PackedConv, n: int, h: int, w: int, residual: bool) -> str:
    return f"{pc.kh}x{pc.kw}s{pc.stride}p{pc.pad}c{pc.cin_pad}k{pc.cout}n{n}h{h}w{w}r{int(residual)}"


def tuned_tile(pc: PackedConv, n: int, h: int, w: int, residual: bool) -> int:
    """Measured per-shape tile config (bench/conv_tune.py -> ops/conv_tiles.json, or the table named by
    ``AI4E_CONV_TILES`` for A/B runs); 0 = kernel default."""
    global _TILES
    if _TILES is None:
        import json
        import os

        path = os.environ.get("AI4E_CONV_TILES") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                 "conv_tiles.json")
        try:
            with open(path) as f:
                _TILES = json.load(f)
        except (OSError, ValueError):
            _TILES = {}
    cfg = _TILES.get(tile_key(pc, n, h, w, residual))
    if cfg is None and 224 <= n <= 288:  # batch sizes near the tuned 256 share its tile choices
        cfg = _TILES.get(tile_key(pc, 256, h, w, residual))
    if cfg is None and n > 250 and n % 250 == 0:  # whole multiples of the serving batch: its grids, more rounds
        cfg = _TILES.get(tile_key(pc, 250, h, w, residual))
    return int(cfg or 0)


def split_cfg(tile_cfg: int) -> Tuple[int, int]:
    """Tile-table entry -> (K split, tile config): entries ``cfg | ks << 4`` (ks 2..4) run a 256-wide config (6, 9,
    10) with split-K over ``ks`` workgroups per output tile (``ai4e_conv2d_sk_fwd``): layer4's 3x3 convs at batch 250
    are 96-128 tiles of K 2304-4608, a quarter to a half of the chip's 256 CUs. Other paths (fp16, fused GroupNorm
    statistics / head) run the plain config."""
    ks = tile_cfg >> 4
    if ks < 2 or (tile_cfg & 15) not in (6, 9, 10):
        return 1, tile_cfg & 15 if ks else tile_cfg
    return ks, tile_cfg & 15


def conv2d_nhwc(x: torch.Tensor, pc: PackedConv, residual: Optional[torch.Tensor] = None, relu: bool = False,
                out: Optional[torch.Tensor] = None, out_coff: int = 0, tile_cfg: int = -1,
                residual_up2: bool = False) -> torch.Tensor:
    """``residual_up2``: ``residual`` is [N, OH/2, OW/2, Cout] and is added nearest-neighbour upsampled 2x
    (the FPN top-down merge), read straight from the half-resolution tensor by the kernel epilogue."""
    n, h, w, c = x.shape
    if tile_cfg < 0:
        tile_cfg = tuned_tile(pc, n, h, w, residual is not None)
    if c != pc.cin_pad:
        raise ValueError(f"conv expects C={pc.cin_pad} (padded), got {c}")
    oh, ow = pc.out_hw(h, w)
    if out is None:
        out = torch.empty(n, oh, ow, pc.cout, device=x.device, dtype=x.dtype)
        out_coff = 0
    if _ext.backend_for(x) == "hip":
        _conv_hip(x, pc, residual, relu, out, out_coff, tile_cfg, residual_up2)
    else:
        if residual is not None and residual_up2:
            residual = residual.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)
        y = _conv_torch(x, pc, residual, relu)
        out[..., out_coff:out_coff + pc.cout] = y.to(out.dtype)
    return out


# (measured and removed in round 5: hipBLASLt routes for the wide-K 1x1 convs, the classifier FC and the detector's
# box-head FCs — flat or slower inside the captured forwards than K1; patch in profiles/r5_pruned/)


def _conv_hip(x, pc, residual, relu, out, out_coff, tile_cfg, residual_up2=False, gn=None):
    n, h, w, c = x.shape
    oh, ow = pc.out_hw(h, w)
    f16 = x.dtype == torch.float16
    if x.dtype not in (torch.bfloat16, torch.float16) or out.dtype != x.dtype or pc.w_packed.dtype != x.dtype or \
            (residual is not None and residual.dtype != x.dtype) or (f16 and gn is not None):
        raise TypeError("HIP conv path: bf16 or fp16 activations, weights (PackedConv.cast) and residual alike")
    # x may be a channel-slice view of a wider NHWC buffer: rows stride = x.stride(2)
    if x.stride(3) != 1 or x.stride(2) * w != x.stride(1) or x.stride(1) * h != x.stride(0):
        raise ValueError("conv input must be an NHWC (possibly channel-sliced) dense tensor")
    ldx = x.stride(2)
    base = x.untyped_storage().data_ptr()
    xoff = x.storage_offset()
    if out.stride(3) != 1 or out.shape[1] != oh or out.shape[2] != ow:
        raise ValueError("bad conv output buffer")
    ldy = out.stride(2)
    ldres = 0
    if residual is not None:
        rshape = (n, oh // 2, ow // 2, pc.cout) if residual_up2 else (n, oh, ow, pc.cout)
        if residual.shape != rshape or not residual.is_contiguous() or (residual_up2 and (oh % 2 or ow % 2)):
            raise ValueError(f"residual must be contiguous {list(rshape)}")
        ldres = pc.cout
    ksplit, tile_cfg = split_cfg(tile_cfg)
    args = (base + 2 * (xoff - xoff % ldx), pc.w_packed.data_ptr(), pc.bias.data_ptr(), _ext.ptr(residual),
            out.data_ptr(), n, h, w, c, ldx, xoff % ldx, pc.kh, pc.kw, pc.stride, pc.pad, oh, ow, pc.cout, pc.kpad, ldy,
            out_coff, ldres, int(relu) | (2 if residual_up2 else 0), tile_cfg)
    if ksplit > 1 and gn is None and not f16:
        # split-K workspace per call (stream-ordered allocator; a captured graph keeps its own): the parked fp32
        # partials and the arrival / ready counters, which must be zero at launch (the kernel leaves them zero)
        tiles = -(-n * oh * ow // (256 if tile_cfg == 6 else 192)) * -(-pc.cout // 256)
        park = torch.empty(tiles * ksplit * (256 if tile_cfg == 6 else 192) * 256, device=x.device,
                           dtype=torch.float32)
        sems = torch.zeros(2 * tiles, device=x.device, dtype=torch.int32)
        diag = int(os.environ.get("AI4E_SPLITK_DIAG", "0"))  # hand-off A/B variants (timing only)
        _ext.call("ai4e_conv2d_sk_fwd", *args, ksplit | diag << 8, park.data_ptr(), sems.data_ptr(), _ext.stream_ptr(x.device))
        return
    if gn is None:
        _ext.call("ai4e_conv2d_f16_fwd" if f16 else "ai4e_conv2d_fwd", *args, _ext.stream_ptr(x.device))
    else:
        _ext.call("ai4e_conv2d_gn_fwd", *args, gn[0].data_ptr(), gn[1], _ext.stream_ptr(x.device))


def conv2d_head_nhwc(x: torch.Tensor, pc: PackedConv, head: PackedConv, relu: bool = True,
                     tile_cfg: int = -1) -> torch.Tensor:
    """``conv2d_nhwc(conv2d_nhwc(x, pc, relu=relu), head)`` for a 256-channel conv followed by a 1x1 conv to 16
    channels whose input is used nowhere else (the FPN RPN conv and its objectness / box-delta head). On a 256-wide
    tile config the head runs inside the conv's epilogue on the staged output tile (``ai4e_conv2d_head_fwd``): the
    256-channel intermediate is never written and the head's separate pass over it disappears. Other shapes run the
    two convs. Returns [N, OH, OW, 16]. ``tile_cfg`` overrides the tuned tile of the first conv (tests)."""
    n, h, w, c = x.shape
    oh, ow = pc.out_hw(h, w)
    cfg = tuned_tile(pc, n, h, w, False) if tile_cfg < 0 else tile_cfg
    fused = (_ext.backend_for(x) == "hip" and cfg in (6, 9, 10) and pc.cout == 256 and head.cout == 16
             and (head.kh, head.kw, head.stride, head.pad) == (1, 1, 1, 0) and head.cin_pad == 256
             and head.kpad >= 256 and x.dtype == torch.bfloat16 and pc.w_packed.dtype == torch.bfloat16
             and head.w_packed.dtype == torch.bfloat16 and c == pc.cin_pad and x.is_contiguous()
             and _ext.has("ai4e_conv2d_head_fwd"))
    if not fused:
        return conv2d_nhwc(conv2d_nhwc(x, pc, relu=relu, tile_cfg=tile_cfg), head)
    y = torch.empty(n, oh, ow, 16, device=x.device, dtype=x.dtype)
    _ext.call("ai4e_conv2d_head_fwd", x.data_ptr(), pc.w_packed.data_ptr(), pc.bias.data_ptr(), None, None, n, h, w,
              c, c, 0, pc.kh, pc.kw, pc.stride, pc.pad, oh, ow, pc.cout, pc.kpad, pc.cout, 0, 0, int(relu), cfg,
              head.w_packed.data_ptr(), head.kpad, head.bias.data_ptr(), y.data_ptr(), _ext.stream_ptr(x.device))
    return y


def conv2d_gn_nhwc(x: torch.Tensor, pc: PackedConv, groups: int, out: Optional[torch.Tensor] = None,
                   out_coff: int = 0):
    """``conv2d_nhwc(x, pc)`` that also produces the GroupNorm statistics of its output from the same epilogue
    (per image, tile-row chunk and group: sum and sum of squares of the stored bf16 values), so the norm that
    follows skips its statistics pass over the tensor. Returns ``(y, stats)``; ``stats`` = ``(partials,
    nchunks)`` for ``group_norm_nhwc(..., stats=stats)``, or ``None`` when the shape or the tuned tile cannot
    fuse (then the norm computes its own statistics)."""
    n, h, w, c = x.shape
    oh, ow = pc.out_hw(h, w)
    cfg = tuned_tile(pc, n, h, w, False) or (2 if pc.cout <= 64 else 1)
    # statistics tile (pixels, channels) of each config: the 256-wide ping-pong configs (6: 256 x 256, 9 / 10:
    # 192 x 256) emit them from their epilogue too (round 5: the U-Net's deep-level convs lost their stats pass)
    bm, bn = {2: (256, 64), 5: (256, 64), 8: (256, 64), 6: (256, 256), 9: (192, 256), 10: (192, 256)}.get(cfg, (128, 128))
    cg = pc.cout // groups if groups > 0 else 0
    ok = (_ext.backend_for(x) == "hip" and cfg in (1, 2, 4, 5, 6, 7, 8, 9, 10) and groups > 0 and pc.cout % groups == 0
          and (oh * ow) % bm == 0 and pc.cout % 8 == 0 and bn % cg == 0 and out_coff % 8 == 0
          and (cfg not in (6, 9, 10) or cg & (cg - 1) == 0)
          and (out is None or out.stride(2) % 8 == 0) and x.dtype == torch.bfloat16 and c == pc.cin_pad)
    if not ok:
        return conv2d_nhwc(x, pc, out=out, out_coff=out_coff), None
    if out is None:
        out = torch.empty(n, oh, ow, pc.cout, device=x.device, dtype=x.dtype)
        out_coff = 0
    nchunks = oh * ow // bm
    # chunk sums, then room for the per-channel affine the norm's finalize launch writes
    partials = torch.empty(n * nchunks * groups * 4 + n * pc.cout * 2, device=x.device, dtype=torch.float32)
    _conv_hip(x, pc, None, False, out, out_coff, cfg, gn=(partials, groups))
    return out, (partials, nchunks)


def _tile_rows(cout: int) -> int:
    return 8  # output tile rows (x 32 columns); the input channels run as 64-channel k-slices


def tile64_supported(x: torch.Tensor, pc: PackedConv) -> bool:
    """Shapes K1t (``conv3x3_tile64``, csrc/kernels/conv_tile3x3.hip) takes: 3x3 / stride 1 / pad 1, bf16, 64 or 128
    -> 64 channels (8 x 32 output tiles, H % 8 == 0, W % 32 == 0). AI4E_CONV_TILE64: "1" default; "64" the 64 -> 64
    instance only; "0" off (K1 everywhere: the A/B reference). 128-output-channel instances were measured 1.4 % slower
    than K1 at level 1 and removed (profiles/r4_k1t/cout128/, patch in profiles/r5_pruned/)."""
    n, h, w, c = x.shape
    # the 64-channel instances beat K1 (profiles/r4_k1t/: 558 vs 670 us and 829 vs 1022 us per conv over 16 tiles of
    # 512^2; U-Net 24.4 vs 22.5 mosaics/s with K1)
    mode = os.environ.get("AI4E_CONV_TILE64", "1")
    ok_c = pc.cout == 64 and pc.cin_pad in (64, 128)
    return (mode != "0" and (mode != "64" or (c == 64 and pc.cout == 64)) and _ext.backend_for(x) == "hip"
            and x.dtype == torch.bfloat16 and pc.w_packed.dtype == torch.bfloat16 and (pc.kh, pc.kw) == (3, 3)
            and pc.stride == 1 and pc.pad == 1 and (pc.pad if pc.pad_hi is None else pc.pad_hi) == 1
            and ok_c and c == pc.cin_pad and pc.w_packed.shape[0] >= pc.cout
            and h % _tile_rows(pc.cout) == 0 and w % 32 == 0 and x.stride(3) == 1 and x.stride(2) % 8 == 0
            and x.stride(2) * w == x.stride(1) and x.stride(1) * h == x.stride(0))


def conv3x3_tile64(x: torch.Tensor, pc: PackedConv, pro: Optional[torch.Tensor] = None, pro_relu: bool = True,
                   gn_groups: int = 0) -> Tuple[torch.Tensor, Optional[tuple]]:
    """K1t: ``conv3x3(pro(x)) + bias`` (see ``tile64_supported``), one 8 x 32 output tile at a time per persistent
    workgroup from an LDS input patch. ``pro``: float32 [N, C, 2] per-(image, channel) affine applied to the input as
    it is loaded (``x * a + b``, then ReLU with ``pro_relu``): the previous GroupNorm, which then needs no apply pass
    (``norm.group_norm_affine``). Returns ``(y, stats)`` with ``stats`` = ``(partials, nchunks)`` GroupNorm
    statistics of y (as ``conv2d_gn_nhwc``) when ``gn_groups``, else None."""
    n, h, w, c = x.shape
    if not tile64_supported(x, pc):
        raise ValueError("conv3x3_tile64: unsupported shape / dtype / layout")
    if pro is not None and (pro.dtype != torch.float32 or not pro.is_contiguous() or tuple(pro.shape) != (n, c, 2)):
        raise ValueError(f"conv3x3_tile64: pro must be contiguous float32 [N, {c}, 2]")
    cout = pc.cout
    ldx = x.stride(2)
    xoff = x.storage_offset()
    base = x.untyped_storage().data_ptr() + 2 * (xoff - xoff % ldx)
    out = torch.empty(n, h, w, cout, device=x.device, dtype=x.dtype)
    nchunks = (h // _tile_rows(cout)) * (w // 32)
    partials = None
    if gn_groups:
        partials = torch.empty(n * nchunks * gn_groups * 4 + n * cout * 2, device=x.device, dtype=torch.float32)
    _ext.call("ai4e_conv3x3_tile_fwd", base, pc.w_packed.data_ptr(), pc.bias.data_ptr(), _ext.ptr(pro),
              int(pro_relu), out.data_ptr(), n, h, w, c, cout, ldx, xoff % ldx, pc.kpad, cout, 0, _ext.ptr(partials),
              gn_groups, _ext.stream_ptr(x.device))
    return out, ((partials, nchunks) if gn_groups else None)


def chain_kernel_builds(mid: int, midn: int = 0) -> bool:
    """Shapes the fused bottleneck-chain kernel K1c is built for (csrc/kernels/conv_chain.hip); ``midn`` is
    the chained 1x1's output width (0 = no chained 1x1)."""
    return (mid, midn) in ((64, 0), (64, 64), (64, 128), (128, 0), (128, 128))


def chain_supported(mid: int, midn: int = 0) -> bool:
    """Shapes ``conv_chain`` routes to K1c by default."""
    return chain_kernel_builds(mid, midn)


def _down_pack(c3: PackedConv, down: PackedConv) -> Tuple[torch.Tensor, torch.Tensor]:
    """[W3 | Wd] along K and b3 + bd: the downsample 1x1 folded into c3 (K1c DOWN mode), cached on c3."""
    cached = getattr(c3, "_down_pack", None)
    if cached is not None and cached[0] is down:
        return cached[1], cached[2]
    k3, kd = c3.cin_pad, down.cin_pad
    w = torch.cat([c3.w_packed[:, :k3], down.w_packed[:, :kd]], dim=1).contiguous()
    b = (c3.bias + down.bias).contiguous()
    c3._down_pack = (down, w, b)
    return w, b


def conv_chain(t1: torch.Tensor, c2: PackedConv, c3: PackedConv, residual: Optional[torch.Tensor],
               c1n: Optional[PackedConv] = None, out: Optional[torch.Tensor] = None, force: bool = False,
               tile_cfg: int = -1, down: Optional[PackedConv] = None, x0: Optional[torch.Tensor] = None,
               t1n_out: Optional[torch.Tensor] = None):
    """Fused bottleneck tail (K1c): ``y = relu(c3(relu(c2(t1))) + residual)`` and, with ``c1n`` (the next
    block's 1x1 reduce), ``t1n = relu(c1n(y))`` from the same kernel. Returns ``(y, t1n or None)``.

    ``out`` / ``t1n_out`` are optional preallocated outputs (micro-batch slices of full-batch buffers).
    ``t1``: NHWC ``[N,H,W,mid]`` bf16 (c1's output), ``c2`` 3x3/pad 1 (stride 1 or 2) mid->mid, ``c3`` 1x1
    mid->4*mid, ``residual`` ``[N,OH,OW,4*mid]``, ``c1n`` 1x1 4*mid->mid. With ``residual=None`` and
    ``down``/``x0`` the residual is ``down(x0)`` (a stage's first block); for mid 64, stride 1 and a chained
    64-wide c1n the kernel folds that projection into c3's K (no residual tensor at all). Shapes the kernel does not cover
    (``chain_supported``; ``force`` = every shape the kernel builds) and the PyTorch backend run the
    three convs separately.
    """
    n, h, w, mid = t1.shape
    if residual is None:
        if down is None or x0 is None:
            raise ValueError("conv_chain: residual or (down, x0) required")
        dmode = (_ext.backend_for(t1) == "hip" and mid == 64 and c2.stride == 1 and c1n is not None
                 and c1n.cout == 64 and down.kh == 1 and down.stride == 1 and down.cin_pad == 64
                 and x0.is_contiguous() and x0.shape[:3] == t1.shape[:3])
        if not dmode:
            residual = conv2d_nhwc(x0, down)
    if (c2.kh, c2.kw, c2.pad, c2.cin_pad, c2.cout) != (3, 3, 1, mid, mid) or c3.kh != 1 or c3.cin_pad != mid \
            or c3.cout != 4 * mid or (c1n is not None and (c1n.kh != 1 or c1n.stride != 1 or c1n.cin_pad != 4 * mid)):
        raise ValueError("conv_chain: layer shapes do not form a bottleneck chain")
    oh, ow = c2.out_hw(h, w)
    if out is None:
        out = torch.empty(n, oh, ow, 4 * mid, device=t1.device, dtype=t1.dtype)
    ok = chain_kernel_builds if force else chain_supported
    midn = c1n.cout if c1n is not None else 0
    if _ext.backend_for(t1) != "hip" or not ok(mid, midn):
        y2 = conv2d_nhwc(t1, c2, relu=True)
        if c1n is not None and _ext.backend_for(t1) == "hip" and residual is not None and pair_route(mid, c3.cout, midn):
            return conv_pair(y2, c3, residual, c1n, out=out, t1n_out=t1n_out)  # K1p: c3 + residual + next c1
        conv2d_nhwc(y2, c3, residual=residual, relu=True, out=out)
        return out, (conv2d_nhwc(out, c1n, relu=True, out=t1n_out) if c1n is not None else None)
    f16 = t1.dtype == torch.float16  # (the f16-MFMA instantiation: the ensemble's fp16 crop classifier)
    if t1.dtype not in (torch.bfloat16, torch.float16) or not t1.is_contiguous() or not out.is_contiguous():
        raise ValueError("conv_chain: contiguous bf16 or fp16 NHWC tensors required")
    if any(c is not None and c.w_packed.dtype != t1.dtype for c in (c2, c3, c1n, down)) or \
            (residual is not None and residual.dtype != t1.dtype) or out.dtype != t1.dtype:
        raise TypeError("conv_chain: activations, weights (PackedConv.cast) and residual in one dtype")
    if residual is not None and (residual.shape != (n, oh, ow, 4 * mid) or not residual.is_contiguous()):
        raise ValueError("conv_chain: residual must be contiguous [N,OH,OW,4*mid]")
    w3, b3, kpad3 = c3.w_packed, c3.bias, c3.kpad
    if residual is None:
        w3, b3 = _down_pack(c3, down)
        kpad3 = w3.shape[1]
    t1n = None
    if c1n is not None:
        t1n = torch.empty(n, oh, ow, midn, device=t1.device, dtype=t1.dtype) if t1n_out is None else t1n_out
        if t1n.shape != (n, oh, ow, midn) or not t1n.is_contiguous():
            raise ValueError("conv_chain: bad t1n_out buffer")
    _ext.call("ai4e_conv_chain_f16_fwd" if f16 else "ai4e_conv_chain_fwd", t1.data_ptr(), c2.w_packed.data_ptr(),
              c2.bias.data_ptr(),
              w3.data_ptr(), b3.data_ptr(), _ext.ptr(residual), out.data_ptr(),
              _ext.ptr(c1n.w_packed if c1n is not None else None), _ext.ptr(c1n.bias if c1n is not None else None),
              _ext.ptr(t1n), n, h, w, mid, mid, midn, c2.stride, c2.kpad, kpad3, c1n.kpad if c1n is not None else 0,
              CHAIN_TILE.get(mid, 0) if tile_cfg < 0 else tile_cfg, _ext.ptr(x0 if residual is None else None),
              x0.shape[-1] if residual is None else 0, _ext.stream_ptr(t1.device))
    return out, t1n


def pack_mfma_frags(w: torch.Tensor) -> torch.Tensor:
    """[R, K] bf16 (R % 16 == 0, K % 32 == 0) -> the MFMA fragment order the K1p pair kernel streams:
    [R/16][K/32][64 lanes][8], lane l holding row 16 rb + (l & 15), K elements 32 ks + 8 (l >> 4) .. +8
    (the B-operand fragment of v_mfma_f32_16x16x32_bf16), so each fragment is one contiguous 1-KB wave load."""
    r, k = w.shape
    if r % 16 or k % 32:
        raise ValueError(f"pack_mfma_frags: [{r}, {k}] is not a whole number of 16x32 fragments")
    return w.reshape(r // 16, 16, k // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(r // 16, k // 32, 64, 8)


def pair_supported(mid: int, c4: int, midn: int, dtype: torch.dtype = torch.bfloat16) -> bool:
    """Shapes the fused 1x1 pair kernel K1p (csrc/kernels/conv_pair.hip) is built for (fp16: the layer3 pair)."""
    if dtype == torch.float16:
        return (mid, c4, midn) == (256, 1024, 256)
    return (mid, c4, midn) in ((256, 1024, 256), (128, 512, 256), (256, 1024, 512), (512, 2048, 512))


def pair_route(mid: int, c4: int, midn: int) -> bool:
    """Whether ``conv_chain`` runs this c3 + residual + next-c1 shape as K1p by default (env switches below)."""
    if not PAIR or not pair_supported(mid, c4, midn):
        return False
    if mid == 128:
        return False  # the last layer2 block stays a K1c chain (K1 3x3 + K1p measured slower, removed in round 5)
    if mid == 512:
        return PAIR_L4
    return midn == mid or PAIR_X


def _pair_pack(c3: PackedConv, c1n: PackedConv):
    cached = getattr(c3, "_pair_pack", None)
    if cached is not None and cached[0] is c1n:
        return cached[1], cached[2]
    w3p = pack_mfma_frags(c3.w_packed[:c3.cout, :c3.cin_pad])
    w1p = pack_mfma_frags(c1n.w_packed[:c1n.cout, :c1n.cin_pad])
    c3._pair_pack = (c1n, w3p, w1p)
    return w3p, w1p


def conv_pair(t2: torch.Tensor, c3: PackedConv, residual: torch.Tensor, c1n: PackedConv,
              out: Optional[torch.Tensor] = None, t1n_out: Optional[torch.Tensor] = None, tile_cfg: int = -1):
    """K1p: ``y = relu(c3(t2) + residual)`` and the next block's ``t1n = relu(c1n(y))`` in one launch (c3, c1n
    1x1 convs; ``t2`` [N,H,W,mid], ``residual`` [N,H,W,4*mid]); Y is read back from LDS instead of HBM.
    Returns ``(y, t1n)``. Other backends/shapes: the two K1 convs."""
    n, h, w, mid = t2.shape
    c4, midn = c3.cout, c1n.cout
    if out is None:
        out = torch.empty(n, h, w, c4, device=t2.device, dtype=t2.dtype)
    t1n = torch.empty(n, h, w, midn, device=t2.device, dtype=t2.dtype) if t1n_out is None else t1n_out
    ok = (_ext.backend_for(t2) == "hip" and pair_supported(mid, c4, midn, t2.dtype) and c3.kh == 1 and c3.stride == 1
          and c1n.kh == 1 and c1n.stride == 1 and c3.cin_pad == mid and c1n.cin_pad == c4 and t2.is_contiguous()
          and residual.is_contiguous() and residual.shape == (n, h, w, c4) and out.is_contiguous()
          and t1n.is_contiguous() and t1n.shape == (n, h, w, midn) and t2.dtype in (torch.bfloat16, torch.float16)
          and c3.w_packed.dtype == t2.dtype and c1n.w_packed.dtype == t2.dtype and residual.dtype == t2.dtype)
    if not ok:
        conv2d_nhwc(t2, c3, residual=residual, relu=True, out=out)
        conv2d_nhwc(out, c1n, relu=True, out=t1n)
        return out, t1n
    w3p, w1p = _pair_pack(c3, c1n)
    _ext.call("ai4e_conv_pair_f16_fwd" if t2.dtype == torch.float16 else "ai4e_conv_pair_fwd", t2.data_ptr(),
              w3p.data_ptr(), c3.bias.data_ptr(), residual.data_ptr(),
              out.data_ptr(), w1p.data_ptr(), c1n.bias.data_ptr(), t1n.data_ptr(), n * h * w, mid, c4, midn,
              (PAIR_TILE if (mid, midn) == (256, 256) else 0) if tile_cfg < 0 else tile_cfg, _ext.stream_ptr(t2.device))
    return out, t1n


# K1p: on by default for the ResNet layer3 pairs (AI4E_PAIR=0 runs c3 + residual and the next c1 as two K1
# launches); AI4E_PAIR_TILE picks the tile height (0 = kernel default)
PAIR = os.environ.get("AI4E_PAIR", "1") not in ("0", "off", "")
PAIR_TILE = int(os.environ.get("AI4E_PAIR_TILE", "0"))
# layer4 (mid 512): a 32-pixel tile streams 4 MB of weights per tile through L2, so it stays opt-in (AI4E_PAIR_L4=1)
PAIR_L4 = os.environ.get("AI4E_PAIR_L4", "0") not in ("0", "off", "")
# the last layer3 block's c3 + residual with layer4's first (512-wide) c1, opt-in (AI4E_PAIR_X=1): 110 vs 124 us in
# isolation, but -1 to -7 % images/s in the serving worker (profiles/r2_pair/README.md)
PAIR_X = os.environ.get("AI4E_PAIR_X", "0") not in ("0", "off", "")


# K1c tile config per bottleneck width: 3 = 128-pixel tiles with phase A from the LDS input patch wherever the
# shape allows it (stride 1, patch fits), else the LDS-DMA ring (bench/chain_patch_ab.py: layer1 chains 14-17 %,
# layer2 6 % faster at batch 250); conv_chain(tile_cfg=0) runs the ring everywhere (the A/B reference and its tests)
CHAIN_TILE = {64: 3, 128: 3}

# K1s variant: 0 = direct conv from the LDS input footprint (default), 1 = DMA-gather implicit GEMM
STEM_VARIANT = int(os.environ.get("AI4E_STEM_VARIANT", "0"))


def stem_pool(x: torch.Tensor, pc: PackedConv, variant: int = -1) -> torch.Tensor:
    """Fused s2d stem (K1s): ``maxpool3x3/2(relu(conv4x4(x) + b))`` in one kernel; ``x`` = the
    ``[N,H,W,16]`` space-to-depth input, ``pc`` from ``pack_stem_s2d``. PyTorch backend: the two ops."""
    from .pool import maxpool2d_nhwc

    n, h, w, c = x.shape
    if _ext.backend_for(x) != "hip" or pc.cout != 64 or c != 16 or (pc.kh, pc.kw, pc.pad, pc.pad_hi) != (4, 4, 1, 2):
        return maxpool2d_nhwc(conv2d_nhwc(x, pc, relu=True), 3, 2, 1)
    if x.dtype != torch.bfloat16 or not x.is_contiguous():
        raise ValueError("stem_pool: contiguous bf16 [N,H,W,16] input required")
    y = torch.empty(n, (h - 1) // 2 + 1, (w - 1) // 2 + 1, 64, device=x.device, dtype=x.dtype)
    _ext.call("ai4e_stem_pool_fwd", x.data_ptr(), pc.w_packed.data_ptr(), pc.bias.data_ptr(), y.data_ptr(), n, h, w,
              pc.kpad, STEM_VARIANT if variant < 0 else variant, _ext.stream_ptr(x.device))
    return y


def stem_u8_supported(img: torch.Tensor, pc: PackedConv, c1: PackedConv) -> bool:
    """Shapes ``stem_pool_c1_u8`` runs as ONE launch from the uint8 images (else: preprocess + ``stem_pool_c1``)."""
    return (_ext.backend_for(img) == "hip" and img.dtype == torch.uint8 and img.dim() == 4 and img.shape[-1] == 3
            and img.shape[1] % 2 == 0 and img.shape[2] % 2 == 0 and img.is_contiguous() and pc.cout == 64
            and (pc.kh, pc.kw, pc.pad, pc.pad_hi) == (4, 4, 1, 2) and pc.cin_pad == 16
            and (c1.kh, c1.kw, c1.stride, c1.pad, c1.cin_pad, c1.cout) == (1, 1, 1, 0, 64, 64) and STEM_VARIANT == 0
            and pc.w_packed.dtype == torch.bfloat16 and c1.w_packed.dtype == torch.bfloat16
            and _ext.has("ai4e_stem_pool_c1_u8_fwd"))


def stem_pool_c1_u8(img: torch.Tensor, pc: PackedConv, c1: PackedConv, mean=None, std=None, scale: float = 1.0 / 255.0):
    """``stem_pool_c1(preprocess_s2d_u8(img, mean, std, scale), pc, c1)`` in ONE launch: the direct stem kernel builds
    its input footprint from the uint8 RGB images (the same normalization arithmetic, so the result is identical),
    and the normalized space-to-depth tensor (100 MB bf16 at batch 250) is never written or read."""
    from .pool import IMAGENET_MEAN, IMAGENET_STD, ctypes_floats, preprocess_s2d_u8
    mean = IMAGENET_MEAN if mean is None else mean
    std = IMAGENET_STD if std is None else std
    if not stem_u8_supported(img, pc, c1):
        return stem_pool_c1(preprocess_s2d_u8(img, mean, std, scale), pc, c1)
    import ctypes
    n, h, w, _ = img.shape
    ph, pw = (h // 2 - 1) // 2 + 1, (w // 2 - 1) // 2 + 1
    y = torch.empty(n, ph, pw, 64, device=img.device, dtype=torch.bfloat16)
    t1 = torch.empty(n, ph, pw, 64, device=img.device, dtype=torch.bfloat16)
    ma, sa = ctypes_floats(list(mean)[:3]), ctypes_floats(list(std)[:3])
    _ext.call("ai4e_stem_pool_c1_u8_fwd", img.data_ptr(), ctypes.addressof(ma), ctypes.addressof(sa), scale,
              pc.w_packed.data_ptr(), pc.bias.data_ptr(), y.data_ptr(), c1.w_packed.data_ptr(), c1.bias.data_ptr(),
              t1.data_ptr(), c1.kpad, n, h, w, pc.kpad, _ext.stream_ptr(img.device))
    return y, t1


def stem_pool_c1(x: torch.Tensor, pc: PackedConv, c1: PackedConv):
    """K1s followed by the first bottleneck's 1x1 c1 (64 -> 64, + bias, ReLU) computed from the pooled tile
    while it is still in LDS: returns ``(y, relu(c1(y)))`` from ONE launch (no re-read of y). Other backends /
    shapes: ``stem_pool`` then a K1 conv."""
    n, h, w, c = x.shape
    f16 = x.dtype == torch.float16
    if (_ext.backend_for(x) != "hip" or pc.cout != 64 or c != 16 or (pc.kh, pc.kw, pc.pad, pc.pad_hi) != (4, 4, 1, 2)
            or (c1.kh, c1.kw, c1.stride, c1.pad, c1.cin_pad, c1.cout) != (1, 1, 1, 0, 64, 64) or STEM_VARIANT != 0
            or x.dtype not in (torch.bfloat16, torch.float16) or pc.w_packed.dtype != x.dtype
            or c1.w_packed.dtype != x.dtype or not x.is_contiguous()):
        if f16:  # (K1s is built for bf16 and fp16; other shapes: K1 conv + the max-pool kernel)
            from .pool import maxpool2d_nhwc
            y = maxpool2d_nhwc(conv2d_nhwc(x, pc, relu=True), 3, 2, 1)
        else:
            y = stem_pool(x, pc)
        return y, conv2d_nhwc(y, c1, relu=True)
    ph, pw = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    y = torch.empty(n, ph, pw, 64, device=x.device, dtype=x.dtype)
    t1 = torch.empty(n, ph, pw, 64, device=x.device, dtype=x.dtype)
    _ext.call("ai4e_stem_pool_c1_f16_fwd" if f16 else "ai4e_stem_pool_c1_fwd", x.data_ptr(), pc.w_packed.data_ptr(),
              pc.bias.data_ptr(), y.data_ptr(),
              c1.w_packed.data_ptr(), c1.bias.data_ptr(), t1.data_ptr(), c1.kpad, n, h, w, pc.kpad,
              _ext.stream_ptr(x.device))
    return y, t1


def _conv_torch(x, pc, residual, relu):
    cdt = torch.float32 if not x.is_cuda else x.dtype
    xin = x[..., :pc.cin].permute(0, 3, 1, 2).to(cdt)
    pad = pc.pad
    if pc.pad_hi is not None and pc.pad_hi != pc.pad:
        xin = F.pad(xin, (pc.pad, pc.pad_hi, pc.pad, pc.pad_hi))
        pad = 0
    y = F.conv2d(xin, pc.w_ref.to(x.device, cdt), pc.b_ref.to(x.device, cdt), stride=pc.stride, padding=pad)
    y = y.permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual.to(cdt)
    if relu:
        y = F.relu(y)
    return y


def pack_stem_s2d(weight: torch.Tensor, bias: Optional[torch.Tensor]) -> PackedConv:
    """7x7/2 pad-3 stem -> equivalent 4x4/1 conv on the 2x2 space-to-depth input.

    With ``X'[i, j, (dy, dx, c)] = x[2i + dy - 1, 2j + dx - 1, c]`` (built by ``preprocess_s2d``),
    ``conv7x7s2(x)[oh, ow] = sum_{a,b<4} W'[a, b] . X'[oh - 1 + a, ow - 1 + b]`` where
    ``W'[a, b, dy, dx, c] = W[2a + dy, 2b + dx, c]`` (zero for taps beyond 6). The GEMM K drops from
    49 taps x 8 padded channels (416) to 16 taps x 16 channels (256) and every tap is a contiguous
    32-byte run, so the stem runs in 8 instead of 13 K-steps.
    """
    weight = weight.detach().float().cpu()
    cout, cin, kh, kw = weight.shape
    if (kh, kw) != (7, 7) or cin * 4 > 16:
        raise ValueError("s2d stem expects a 7x7 kernel with <= 4 input channels")
    w = torch.zeros(cout, 4, 4, 2, 2, cin)  # [cout, a, b, dy, dx, c]
    wt = weight.permute(0, 2, 3, 1)          # [cout, kh, kw, c]
    for a in range(4):
        for dy in range(2):
            r = 2 * a + dy
            if r > 6:
                continue
            for b in range(4):
                for dx in range(2):
                    q = 2 * b + dx
                    if q <= 6:
                        w[:, a, b, dy, dx] = wt[:, r, q]
    w16 = torch.zeros(cout, 4, 4, 16)
    w16[..., : 4 * cin] = w.reshape(cout, 4, 4, 4 * cin)
    pc = pack_conv(w16.permute(0, 3, 1, 2).contiguous(), bias, stride=1, pad=1, cin_pad=16)
    pc.pad_hi = 2
    return pc


def conv_flops(pc: PackedConv, n: int, h: int, w: int) -> int:
    oh, ow = pc.out_hw(h, w)
    return 2 * n * oh * ow * pc.cout * pc.kh * pc.kw * pc.cin


def kaiming_conv(cout: int, cin: int, k: int, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    std = math.sqrt(2.0 / (cin * k * k))
    return torch.randn(cout, cin, k, k, generator=generator) * std
