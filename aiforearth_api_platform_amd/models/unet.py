"""Land-cover U-Net (BASELINE config #4): 4-band (RGB+NIR) tiles -> per-pixel class logits.

Architecture: the bilinear-upsampling U-Net (64-128-256-512-512 encoder, GroupNorm(32)+ReLU after
every 3x3 conv, 2x2 max-pool down, bilinear x2 up + skip concat), ~17M parameters; the reference's
land-cover API exposes classify / tile operations (``APIManagement/create_sync_api_management_api.sh:9-92``).

``UNet`` is the plain NCHW fp32 ``torch.nn`` reference. ``FusedUNet`` is the serving graph on NHWC
bf16 built from the hand-written kernels, arranged so that skip-concat costs no copy:

* each decoder level owns one concat buffer ``[N, H, W, C_skip + C_up]``;
* the encoder's last GroupNorm of that level writes its output straight into channels
  ``[0, C_skip)`` of the buffer (K2 with an output channel slice), and the next max-pool reads that
  slice in place;
* the decoder's bilinear upsample (K3) writes channels ``[C_skip, C_skip + C_up)``;
* the decoder's first conv (K1) reads the whole buffer.
"""
from __future__ import annotations

import os

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.conv import conv2d_gn_nhwc, conv2d_nhwc, conv3x3_tile64, pack_conv, tile64_supported
from ..ops.norm import (gn_relu_head8, gn_relu_head8_supported, group_norm_affine, group_norm_nhwc,
                        upsample2x_nhwc)
from ..ops.pool import maxpool2d_nhwc, preprocess_u8

# per-band normalisation for uint8 RGB+NIR imagery (NAIP-style); NIR uses the same scale
LANDCOVER_MEAN = (0.40, 0.42, 0.38, 0.45)
LANDCOVER_STD = (0.20, 0.18, 0.18, 0.22)


class DoubleConv(nn.Module):
    def __init__(self, cin, cout, mid=None, groups=32):
        super().__init__()
        mid = mid or cout
        self.c1 = nn.Conv2d(cin, mid, 3, padding=1, bias=False)
        self.n1 = nn.GroupNorm(groups, mid)
        self.c2 = nn.Conv2d(mid, cout, 3, padding=1, bias=False)
        self.n2 = nn.GroupNorm(groups, cout)

    def forward(self, x):
        return F.relu(self.n2(self.c2(F.relu(self.n1(self.c1(x))))))


class UNet(nn.Module):
    def __init__(self, in_ch: int = 4, n_classes: int = 7, width: int = 64):
        super().__init__()
        w = width
        self.n_classes = n_classes
        self.inc = DoubleConv(in_ch, w)
        self.d1 = DoubleConv(w, 2 * w)
        self.d2 = DoubleConv(2 * w, 4 * w)
        self.d3 = DoubleConv(4 * w, 8 * w)
        self.d4 = DoubleConv(8 * w, 8 * w)
        self.u1 = DoubleConv(16 * w, 4 * w, 8 * w)
        self.u2 = DoubleConv(8 * w, 2 * w, 4 * w)
        self.u3 = DoubleConv(4 * w, w, 2 * w)
        self.u4 = DoubleConv(2 * w, w, w)
        self.outc = nn.Conv2d(w, n_classes, 1)

    def forward(self, x):
        x1 = self.inc(x)
        x2 = self.d1(F.max_pool2d(x1, 2))
        x3 = self.d2(F.max_pool2d(x2, 2))
        x4 = self.d3(F.max_pool2d(x3, 2))
        x5 = self.d4(F.max_pool2d(x4, 2))
        up = lambda t: F.interpolate(t, scale_factor=2, mode="bilinear", align_corners=False)  # noqa: E731
        y = self.u1(torch.cat([x4, up(x5)], 1))
        y = self.u2(torch.cat([x3, up(y)], 1))
        y = self.u3(torch.cat([x2, up(y)], 1))
        y = self.u4(torch.cat([x1, up(y)], 1))
        return self.outc(y)


def unet_landcover(n_classes: int = 7, in_ch: int = 4, seed: int = 0, width: int = 64) -> UNet:
    g = torch.Generator().manual_seed(seed)
    m = UNet(in_ch, n_classes, width)
    for mod in m.modules():
        if isinstance(mod, nn.Conv2d):
            nn.init.kaiming_normal_(mod.weight, nonlinearity="relu", generator=g)
            if mod.bias is not None:
                nn.init.normal_(mod.bias, 0, 0.1, generator=g)
        elif isinstance(mod, nn.GroupNorm):
            mod.weight.data = 0.75 + 0.5 * torch.rand(mod.num_channels, generator=g)
            mod.bias.data = 0.1 * torch.randn(mod.num_channels, generator=g)
    return m.eval()


class _FusedDouble:
    def __init__(self, dc: DoubleConv, device, cin_pad=None):
        self.c1 = pack_conv(dc.c1.weight.data, None, stride=1, pad=1, cin_pad=cin_pad).to(device)
        self.c2 = pack_conv(dc.c2.weight.data, None, stride=1, pad=1).to(device)
        self.g1 = (dc.n1.weight.data.float().to(device), dc.n1.bias.data.float().to(device), dc.n1.num_groups)
        self.g2 = (dc.n2.weight.data.float().to(device), dc.n2.bias.data.float().to(device), dc.n2.num_groups)

    @staticmethod
    def _k1t_groups(g: int, cout: int = 64) -> bool:  # K1t's epilogue sums whole groups within a lane's 4 channels
        return cout % g == 0 and cout // g <= 4 and g <= 64

    def __call__(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                 pool_out: Optional[torch.Tensor] = None, head=None):
        """``head``: a 1x1 PackedConv to apply after the final GroupNorm + ReLU; then returns ``(y, headed)`` where
        ``headed`` says whether ``y`` is already the head's output (fused: csrc/kernels/norm_resample.hip
        gn_relu_head8_kernel) or still the block output."""
        # GroupNorm statistics come out of the conv epilogues (conv2d_gn_nhwc, K1t) where the tile allows
        if tile64_supported(x, self.c1) and self._k1t_groups(self.g1[2], self.c1.cout):
            y, st = conv3x3_tile64(x, self.c1, gn_groups=self.g1[2])  # e.g. the last decoder's 128 -> 64 c1
        else:
            y, st = conv2d_gn_nhwc(x, self.c1, self.g1[2])
        if st is not None and tile64_supported(y, self.c2) and self._k1t_groups(self.g2[2], self.c2.cout):
            # 64 -> 64 at full resolution (K1t): c1's GroupNorm + ReLU is applied while c2 loads its input patch, so
            # the normalized c1 output is never written (csrc/kernels/conv_tile3x3.hip)
            n, h, w, c = y.shape
            ss = group_norm_affine(st, *self.g1[:2], n=n, hw=h * w, c=c, groups=self.g1[2])
            z, st = conv3x3_tile64(y, self.c2, pro=ss, pro_relu=True, gn_groups=self.g2[2])
            if head is not None and pool_out is None and gn_relu_head8_supported(z, head):
                # the last decoder: GroupNorm + ReLU + the 1x1 head in one pass over z (the normalized tensor is
                # never written, and the head conv does not read it back)
                ss2 = group_norm_affine(st, *self.g2[:2], n=n, hw=h * w, c=c, groups=self.g2[2])
                return gn_relu_head8(z, ss2, head), True
            r = group_norm_nhwc(z, *self.g2[:2], groups=self.g2[2], relu=True, out=out if out is not None else z,
                                stats=st, pool_out=pool_out)
            return (r, False) if head is not None else r
        y = group_norm_nhwc(y, *self.g1[:2], groups=self.g1[2], relu=True, out=y, stats=st)
        z, st = conv2d_gn_nhwc(y, self.c2, self.g2[2])
        r = group_norm_nhwc(z, *self.g2[:2], groups=self.g2[2], relu=True, out=out if out is not None else z,
                            stats=st, pool_out=pool_out)
        return (r, False) if head is not None else r


class FusedUNet:
    def __init__(self, model: UNet, device="cpu", mean=LANDCOVER_MEAN, std=LANDCOVER_STD):
        self.device = torch.device(device)
        self.mean, self.std = mean, std
        d = self.device
        self.inc = _FusedDouble(model.inc, d, cin_pad=8)
        self.down = [_FusedDouble(m, d) for m in (model.d1, model.d2, model.d3, model.d4)]
        self.up = [_FusedDouble(m, d) for m in (model.u1, model.u2, model.u3, model.u4)]
        self.n_classes = model.n_classes
        kout = (model.n_classes + 3) // 4 * 4
        w = torch.zeros(kout, model.outc.in_channels, 1, 1)
        b = torch.full((kout,), -1e4)
        w[: model.n_classes] = model.outc.weight.data
        b[: model.n_classes] = model.outc.bias.data
        self.outc = pack_conv(w, b).to(d)
        self.out_channels = kout
        self.fused_pool = os.environ.get("AI4E_UNET_FUSED_POOL", "1") != "0"
        # the last decoder's GroupNorm + ReLU and the 1x1 head in one pass (AI4E_UNET_FUSED_HEAD=0: apply, then conv)
        self.fused_head = os.environ.get("AI4E_UNET_FUSED_HEAD", "1") != "0"

    def tensors(self) -> List[torch.Tensor]:
        """Every weight tensor (packed convs + GroupNorm affine), for ``parallel.dist.broadcast_tensors``."""
        out = []
        for dc in [self.inc] + self.down + self.up:
            for pc in (dc.c1, dc.c2):
                out += [pc.w_packed, pc.bias, pc.w_ref]
            out += [dc.g1[0], dc.g1[1], dc.g2[0], dc.g2[1]]
        return out + [self.outc.w_packed, self.outc.bias, self.outc.w_ref, self.outc.b_ref]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: normalized NHWC [N,H,W,8] (H, W multiples of 16) -> logits NHWC [N,H,W,kout]."""
        n, h, w, _ = x.shape
        enc_c = [self.inc.c2.cout] + [d.c2.cout for d in self.down[:3]]   # skip channels per level
        up_c = [self.down[3].c2.cout] + [u.c2.cout for u in self.up[:3]]  # upsampled channels per level (deepest first)
        cat = []
        for lvl in range(4):
            s = 2 ** lvl
            cat.append(torch.empty(n, h // s, w // s, enc_c[lvl] + up_c[3 - lvl], device=x.device, dtype=x.dtype))
        # each encoder level's GN apply also writes the 2x2 max-pool the next level reads (no pool pass)
        if not self.fused_pool:
            return self._forward_unfused(x, cat, enc_c)
        pooled = torch.empty(n, h // 2, w // 2, enc_c[0], device=x.device, dtype=x.dtype)
        self.inc(x, out=cat[0][..., : enc_c[0]], pool_out=pooled)
        for lvl in range(1, 5):
            if lvl < 4:
                s = 2 ** (lvl + 1)
                nxt = torch.empty(n, h // s, w // s, enc_c[lvl], device=x.device, dtype=x.dtype)
                self.down[lvl - 1](pooled, out=cat[lvl][..., : enc_c[lvl]], pool_out=nxt)
                pooled = nxt
            else:
                y = self.down[3](pooled)
        for i, lvl in enumerate((3, 2, 1, 0)):
            buf = cat[lvl]
            upsample2x_nhwc(y, out=buf, out_coff=enc_c[lvl])
            if i == 3 and self.fused_head:
                y, headed = self.up[i](buf, head=self.outc)
                if headed:
                    return y
            else:
                y = self.up[i](buf)
        return conv2d_nhwc(y, self.outc)

    def _forward_unfused(self, x, cat, enc_c):
        """Encoder with a separate max-pool pass (AI4E_UNET_FUSED_POOL=0, for A/B)."""
        skip = self.inc(x, out=cat[0][..., : enc_c[0]])
        for lvl in range(1, 5):
            pooled = maxpool2d_nhwc(skip, 2, 2, 0)
            if lvl < 4:
                skip = self.down[lvl - 1](pooled, out=cat[lvl][..., : enc_c[lvl]])
            else:
                y = self.down[3](pooled)
        for i, lvl in enumerate((3, 2, 1, 0)):
            buf = cat[lvl]
            upsample2x_nhwc(y, out=buf, out_coff=enc_c[lvl])
            y = self.up[i](buf)
        return conv2d_nhwc(y, self.outc)

    def forward_u8(self, img_u8: torch.Tensor) -> torch.Tensor:
        return self.forward(preprocess_u8(img_u8, self.mean, self.std))

    __call__ = forward_u8

    def classify(self, img_u8: torch.Tensor) -> torch.Tensor:
        """Per-pixel class map [N,H,W] uint8."""
        return self.forward_u8(img_u8)[..., : self.n_classes].argmax(-1).to(torch.uint8)
