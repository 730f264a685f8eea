"""ResNet-50 (v1.5, torchvision layout) — the headline ResNet-50 224x224 classification API model.

Two forms:

* ``ResNet`` — a plain ``torch.nn`` NCHW definition (fp32), the numerics reference and the
  weight source (``load_state_dict`` accepts torchvision-style keys; weights are random-init here
  because no checkpoint is available offline).
* ``FusedResNet`` — the serving form: BatchNorm folded into the convs, NHWC bf16 activations, every
  conv (+bias +ReLU +residual add) one K1 HIP kernel, preprocess (K7, fused 2x2 space-to-depth so
  the 7x7/2 stem runs as a dense 4x4/1 conv), max-pool, global avg-pool and the classifier (a 1x1
  conv through K1) — 57 kernel launches per forward, capturable in a HIP graph.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.conv import (PackedConv, chain_supported, conv2d_nhwc, conv_chain, fold_bn, pack_conv, pack_stem_s2d,
                        pair_route, pair_supported, stem_pool, stem_pool_c1, stem_pool_c1_u8, stem_u8_supported)
from ..ops.head import softmax_topk
from ..ops.pool import global_avgpool_nhwc, maxpool2d_nhwc, preprocess_s2d_u8, space_to_depth_shifted


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return F.relu(out + idt)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000, in_ch: int = 3):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(in_ch, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make(64, layers[0], 1)
        self.layer2 = self._make(128, layers[1], 2)
        self.layer3 = self._make(256, layers[2], 2)
        self.layer4 = self._make(512, layers[3], 2)
        self.fc = nn.Linear(2048, num_classes)

    def _make(self, planes, blocks, stride):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                                 nn.BatchNorm2d(planes * 4))
        mods = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        mods += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def features(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        return self.layer4(self.layer3(self.layer2(self.layer1(x))))

    def forward(self, x):
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(self.features(x), 1), 1))


def randomize_bn_(model: nn.Module, generator: Optional[torch.Generator] = None) -> nn.Module:
    """Random-init weights with realistic inference BN statistics (so folding is exercised)."""
    g = generator
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu", generator=g)
        elif isinstance(m, nn.BatchNorm2d):
            c = m.num_features
            m.weight.data = 0.5 + 0.5 * torch.rand(c, generator=g)
            m.bias.data = 0.1 * torch.randn(c, generator=g)
            m.running_mean.data = 0.1 * torch.randn(c, generator=g)
            m.running_var.data = 0.5 + torch.rand(c, generator=g)
        elif isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0, 0.01, generator=g)
            nn.init.zeros_(m.bias)
    # keep the residual stream bounded through 16 blocks with random weights (zero-init-residual
    # style damping of the last BN in every block)
    for m in model.modules():
        if isinstance(m, Bottleneck):
            m.bn3.weight.data *= 0.2
    return model.eval()


def resnet50(num_classes: int = 1000, seed: int = 0) -> ResNet:
    g = torch.Generator().manual_seed(seed)
    return randomize_bn_(ResNet((3, 4, 6, 3), num_classes), g)


def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d, cin_pad: Optional[int] = None) -> PackedConv:
    w, b = fold_bn(conv.weight.data.float(), bn.weight.data.float(), bn.bias.data.float(), bn.running_mean.float(),
                   bn.running_var.float(), bn.eps)
    return pack_conv(w, b, stride=conv.stride[0], pad=conv.padding[0], cin_pad=cin_pad)


def _env_chunk() -> Optional[Tuple[int, int]]:
    """``AI4E_RESNET_CHUNK=mb:nblocks`` (``0`` / ``off`` disables); default from ``DEFAULT_CHUNK``."""
    v = os.environ.get("AI4E_RESNET_CHUNK")
    if v is None:
        return DEFAULT_CHUNK
    if v in ("", "0", "off"):
        return None
    mb, nb = v.split(":")
    return int(mb), int(nb)


DEFAULT_CHUNK: Optional[Tuple[int, int]] = None


def _env_chain() -> bool:
    """``AI4E_RESNET_CHAIN=0`` runs every conv as its own K1 launch instead of the K1c bottleneck chains."""
    return os.environ.get("AI4E_RESNET_CHAIN", "1") not in ("0", "off", "")


class FusedResNet:
    """Inference graph over packed, BN-folded layers (NHWC bf16)."""

    def __init__(self, model: ResNet, device="cpu", in_ch: Optional[int] = None,
                 chunk: Optional[Tuple[int, int]] = None, dtype: torch.dtype = torch.bfloat16):
        """``dtype``: bf16 or fp16 (the ensemble's crop classifier, weights re-rounded from fp32): the same fused
        serving graph (K1s stem with the fused c1, K1c chains, K1p pairs, K1 elsewhere) on bf16 or f16 MFMA."""
        model = model.eval()
        self.device = torch.device(device)
        self.dtype = dtype
        self.in_ch = in_ch or model.conv1.in_channels
        w, b = fold_bn(model.conv1.weight.data.float(), model.bn1.weight.data.float(), model.bn1.bias.data.float(),
                       model.bn1.running_mean.float(), model.bn1.running_var.float(), model.bn1.eps)
        self.stem = pack_stem_s2d(w, b).to(self.device)  # 7x7/2 stem as a 4x4/1 conv on space-to-depth input
        self.blocks: List[Tuple[PackedConv, PackedConv, PackedConv, Optional[PackedConv]]] = []
        for layer in (model.layer1, model.layer2, model.layer3, model.layer4):
            for blk in layer:
                down = None
                if blk.downsample is not None:
                    down = _fold(blk.downsample[0], blk.downsample[1]).to(self.device)
                self.blocks.append((_fold(blk.conv1, blk.bn1).to(self.device), _fold(blk.conv2, blk.bn2).to(self.device),
                                    _fold(blk.conv3, blk.bn3).to(self.device), down))
        # the classifier FC runs on K1, whose output rows are whole 8-channel vectors: classes padded to a multiple
        # of 8 with zero rows, the logits sliced back to num_classes
        self.num_classes = model.fc.out_features
        ncp = -(-self.num_classes // 8) * 8
        fcw = torch.zeros(ncp, model.fc.in_features, 1, 1)
        fcw[:self.num_classes] = model.fc.weight.data.float().reshape(self.num_classes, -1, 1, 1)
        fcb = torch.zeros(ncp)
        fcb[:self.num_classes] = model.fc.bias.data.float()
        self.fc = pack_conv(fcw, fcb).to(self.device)
        self.chunk = chunk if chunk is not None else _env_chunk()
        self.chain = _env_chain()
        if dtype == torch.float16:  # K1 / K1s / K1c / K1p all have f16-MFMA instantiations
            self.stem = self.stem.cast(dtype)
            self.blocks = [tuple(c.cast(dtype) if c is not None else None for c in blk) for blk in self.blocks]
            self.fc = self.fc.cast(dtype)
            self.chunk = None
        elif dtype != torch.bfloat16:
            raise ValueError(f"FusedResNet dtype must be bf16 or fp16, got {dtype}")
        self.fold_down = os.environ.get("AI4E_RESNET_FOLD_DOWN", "1") not in ("0", "off", "")
        # the first bottleneck's 1x1 c1 fused into the stem kernel (computed from the pooled tile in LDS)
        self.stem_c1 = os.environ.get("AI4E_STEM_C1", "1") not in ("0", "off", "")
        # opt-in (AI4E_STEM_U8=1): the stem builds its input from the uint8 images itself (no preprocess launch, no
        # s2d tensor, and the exact 7x7/2 conv at the bottom / right edge, which the [N, H/2, W/2, 16] s2d tensor of
        # the default path leaves out), but its per-byte footprint loads cost more than they save: 3.306 vs 3.231 ms
        # per forward, same process (profiles/r6_stem_u8/)
        self.stem_u8 = os.environ.get("AI4E_STEM_U8", "0") not in ("0", "off", "")
        # classifier FC on K1 (1x1 conv over the pooled features) by default: parity-or-better with hipBLASLt in
        # the captured forward (80.7/80.7k vs 81.3/80.9k images/s same-box A/B) and no library kernel left
        # stage entry: the downsample projection on a side stream, concurrent with the stage's first c1 (both read
        # the previous stage's output, both are latency-bound short-K GEMMs); forked and joined inside the caller's
        # stream, so a captured HIP graph holds the two as parallel branches. Opt-in (AI4E_PAR_DOWN=1): -27 us on a
        # lone forward but -2.2 % images/s in the serving worker, whose two compute streams already fill the chip
        # (profiles/r2_pair/README.md)
        self.par_down = os.environ.get("AI4E_PAR_DOWN", "0") not in ("0", "off", "")
        self._side: dict = {}
        self._side_pool: List[torch.cuda.Stream] = []  # created on first use outside a graph capture
        # stages: runs of blocks starting at a block with a downsample conv
        self.stages: List[List[Tuple[PackedConv, PackedConv, PackedConv, Optional[PackedConv]]]] = []
        for blk in self.blocks:
            if blk[3] is not None or not self.stages:
                self.stages.append([])
            self.stages[-1].append(blk)

    def tensors(self) -> List[torch.Tensor]:
        """Every weight tensor of the packed model (for ``parallel.dist.broadcast_tensors``: load on one rank,
        replicate over xGMI). Call before the first forward: derived caches (folded downsample weights, the
        library-GEMM FC views) are built lazily from these."""
        out = []
        for pc in self.layers():
            out += [pc.w_packed, pc.bias, pc.w_ref, pc.b_ref]
        return out

    def layers(self) -> List[PackedConv]:
        out = [self.stem]
        for c1, c2, c3, d in self.blocks:
            out += [c1, c2, c3] + ([d] if d is not None else [])
        return out + [self.fc]

    def flops(self, n: int, h: int = 224, w: int = 224) -> int:
        from ..ops.conv import conv_flops

        total = 2 * n * (h // 2) * (w // 2) * 64 * 7 * 7 * self.in_ch  # true 7x7/2 stem FLOPs
        h, w = h // 2, w // 2
        h, w = (h + 1) // 2, (w + 1) // 2
        for c1, c2, c3, d in self.blocks:
            total += conv_flops(c1, n, h, w) + conv_flops(c2, n, h, w)
            h2, w2 = c2.out_hw(h, w)
            total += conv_flops(c3, n, h2, w2)
            if d is not None:
                total += conv_flops(d, n, h, w)
            h, w = h2, w2
        return total + conv_flops(self.fc, n, 1, 1)

    def stem_input(self, x: torch.Tensor) -> torch.Tensor:
        """Normalized NHWC input -> the s2d stem's [N,H/2,W/2,16] layout (no-op if already s2d)."""
        if x.shape[-1] == 16:
            return x
        return space_to_depth_shifted(x[..., : self.in_ch])

    def _stem(self, x: torch.Tensor) -> torch.Tensor:
        if self.dtype == torch.float16:  # K1 s2d conv + the max-pool kernel (the stem-only K1s is bf16-only)
            return maxpool2d_nhwc(conv2d_nhwc(self.stem_input(x), self.stem, relu=True))
        return stem_pool(self.stem_input(x), self.stem)  # K1s: conv + bias + ReLU + 3x3/2 max-pool

    def _stem_t1(self, x: torch.Tensor):
        """(stem output, first bottleneck's c1 output): one K1s launch with the 1x1 fused (AI4E_STEM_C1=0: two)."""
        if self.stem_c1:
            return stem_pool_c1(self.stem_input(x), self.stem, self.stages[0][0][0])
        return self._stem(x), None

    @staticmethod
    def _block(x: torch.Tensor, blk, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        c1, c2, c3, down = blk
        idt = x if down is None else conv2d_nhwc(x, down)
        y = conv2d_nhwc(x, c1, relu=True)
        y = conv2d_nhwc(y, c2, relu=True)
        return conv2d_nhwc(y, c3, residual=idt, relu=True, out=out)

    def _stages_chained(self, y: torch.Tensor, collect: bool = False, t1: Optional[torch.Tensor] = None,
                        s0: int = 0, s1: Optional[int] = None):
        """Stages ``s0 .. s1-1`` with the K1c chains: the first block's downsample runs as a K1 conv, then every
        block is ONE kernel (c2 -> c3 + residual -> the next block's c1, across stage boundaries too: the
        last block of a stage computes the next stage's first c1). Shapes K1c does not build fall back to
        separate K1 convs inside ``conv_chain``. ``collect`` returns every stage's output (FPN backbones).
        ``t1`` is stage ``s0``'s first c1 output when a previous call already computed it; with ``s1`` short
        of the last stage the call returns ``(y, t1)`` for the next call (``tools/chain_stamps.py`` times
        the stages one at a time that way)."""
        s1 = len(self.stages) if s1 is None else s1
        outs = []
        for si in range(s0, s1):
            blocks = self.stages[si]
            c1, _, _, down = blocks[0]
            # the first block's downsample: folded into the chain kernel where it can be (layer1), else a K1 conv
            x0, dn = (y, down) if down is not None and down.stride == 1 and self.fold_down else (None, None)
            if t1 is None and dn is None and down is not None and self._side_ok(y):
                t1, idt = self._c1_down_parallel(y, c1, down)
            else:
                if t1 is None:
                    t1 = conv2d_nhwc(y, c1, relu=True)
                idt = None if dn is not None else (y if down is None else conv2d_nhwc(y, down))
            for i, (_, c2, c3, _) in enumerate(blocks):
                if i + 1 < len(blocks):
                    nxt = blocks[i + 1][0]
                elif si + 1 < len(self.stages):
                    nxt = self.stages[si + 1][0][0]
                else:
                    nxt = None
                if (nxt is not None and not chain_supported(c2.cout, nxt.cout) and chain_supported(c2.cout)
                        and not pair_route(c2.cout, c3.cout, nxt.cout)):
                    nxt = None  # keep the chain, run the next c1 as its own K1 launch
                if (nxt is not None and i + 1 == len(blocks) and not chain_supported(c2.cout, nxt.cout)
                        and not pair_supported(c2.cout, c3.cout, nxt.cout) and self._side_ok(t1)):
                    nxt = None  # the next stage's c1 runs at its entry, beside its downsample
                idt, t1 = conv_chain(t1, c2, c3, idt, c1n=nxt, down=dn, x0=x0)
                x0 = dn = None
            y = idt
            outs.append(y)
        if s1 < len(self.stages):
            return y, t1
        return outs if collect else y

    def _side_ok(self, t: torch.Tensor) -> bool:
        if not (self.par_down and t.is_cuda):
            return False
        if not self._side_pool and not torch.cuda.is_current_stream_capturing():
            self._side_pool = [torch.cuda.Stream(device=t.device) for _ in range(4)]
        return bool(self._side_pool)

    def _c1_down_parallel(self, y: torch.Tensor, c1: PackedConv, down: PackedConv):
        """(relu(c1(y)), down(y)) with the downsample forked onto a side stream of the current stream."""
        main = torch.cuda.current_stream(y.device)
        side = self._side.get(main.cuda_stream)
        if side is None:  # pre-created streams only: no stream creation inside a graph capture
            side = self._side[main.cuda_stream] = self._side_pool[len(self._side) % len(self._side_pool)]
        side.wait_stream(main)
        with torch.cuda.stream(side):
            idt = conv2d_nhwc(y, down)
        t1 = conv2d_nhwc(y, c1, relu=True)
        main.wait_stream(side)
        idt.record_stream(main)
        return t1, idt

    def stage_features(self, x_s2d: torch.Tensor):
        """Space-to-depth input -> the four stage outputs (C2..C5) through K1s + the K1c chains; the
        per-conv K1 graph when chains are off."""
        if self.chain:
            y, t1 = self._stem_t1(x_s2d)
            return self._stages_chained(y, collect=True, t1=t1)
        y = self._stem(x_s2d)
        outs, ends, start = [], [], 0
        for st in self.stages:
            start += len(st)
            ends.append(start - 1)
        for i, blk in enumerate(self.blocks):
            y = self._block(y, blk)
            if i in ends:
                outs.append(y)
        return outs

    def _prefix_shape(self, n: int, h: int, w: int, nblocks: int) -> Tuple[int, int, int, int]:
        """Output shape after the stem, max-pool and the first ``nblocks`` bottlenecks."""
        h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1  # maxpool 3/2/1 on the (H/2, W/2) stem output
        c = self.stem.cout
        for c1, c2, c3, d in self.blocks[:nblocks]:
            h, w = c2.out_hw(h, w)
            c = c3.cout
        return n, h, w, c

    def forward_features(self, x: torch.Tensor, preprocess=None) -> torch.Tensor:
        """x: normalized NHWC [N,H,W,8] (or space-to-depth [N,H/2,W/2,16]; or uint8 images when
        ``preprocess`` is given) -> [N,h,w,2048].

        Cache-resident micro-batching: at batch 256 a layer1 activation is 411 MB, so every conv of
        the high-resolution stages streams its input, residual and output through HBM. With
        ``chunk = (mb, nblocks)`` the stem and the first ``nblocks`` bottlenecks run ``mb`` images
        at a time (a layer1 tensor of 32 images is 51 MB, so producer -> consumer traffic stays in
        the 256 MB Infinity Cache) and write their output straight into the full-batch buffer; the
        low-resolution stages then run on the whole batch, where they need it to fill 256 CUs.
        """
        n = x.shape[0]
        mb, nblocks = self.chunk if self.chunk else (n, 0)
        pre = preprocess or (lambda t: t)
        if mb < n and nblocks > 0:
            s2d = preprocess is None and x.shape[-1] == 16
            h, w = (x.shape[1], x.shape[2]) if s2d else (x.shape[1] // 2, x.shape[2] // 2)  # stem output
            feats = torch.empty(self._prefix_shape(n, h, w, nblocks), device=x.device, dtype=torch.bfloat16)
            for n0 in range(0, n, mb):
                y = self._stem(pre(x[n0:n0 + mb]))
                for i in range(nblocks):
                    y = self._block(y, self.blocks[i], out=feats[n0:n0 + mb] if i == nblocks - 1 else None)
            y = feats
        elif self.chain:
            if (preprocess is preprocess_s2d_u8 and self.stem_c1 and self.stem_u8
                    and stem_u8_supported(x, self.stem, self.stages[0][0][0])):
                y, t1 = stem_pool_c1_u8(x, self.stem, self.stages[0][0][0])  # preprocess inside the stem launch
            else:
                y, t1 = self._stem_t1(pre(x))
            return self._stages_chained(y, t1=t1)
        else:
            y, nblocks = self._stem(pre(x)), 0
        if self.chain and nblocks == 0:
            return self._stages_chained(y)
        for blk in self.blocks[nblocks:]:
            y = self._block(y, blk)
        return y

    def logits(self, x: torch.Tensor, preprocess=None) -> torch.Tensor:
        """Logits [N, classes] in the model dtype (bf16 / fp16)."""
        return self._head_logits(self.forward_features(x, preprocess))

    def _head_logits(self, feats: torch.Tensor) -> torch.Tensor:
        f = global_avgpool_nhwc(feats)
        y = conv2d_nhwc(f, self.fc).reshape(f.shape[0], -1)
        return y if y.shape[1] == self.num_classes else y[:, :self.num_classes].contiguous()

    def forward(self, x: torch.Tensor, preprocess=None) -> torch.Tensor:
        return self.logits(x, preprocess).float()

    def topk_u8(self, img_u8: torch.Tensor, k: int = 5):
        """uint8 NHWC images -> (top-k class ids int32, probabilities fp32): the serving head, with softmax
        and top-k fused into one kernel (ops/head.py)."""
        return softmax_topk(self.logits(img_u8, preprocess=self._pre()), k)

    def _pre(self):
        if self.dtype == torch.float16:
            return lambda img: preprocess_s2d_u8(img, dtype=torch.float16)
        return preprocess_s2d_u8

    def forward_u8(self, img_u8: torch.Tensor) -> torch.Tensor:
        """uint8 NHWC images -> fp32 logits (preprocess fused into the first kernel launch)."""
        return self.forward(img_u8, preprocess=self._pre())

    __call__ = forward_u8
