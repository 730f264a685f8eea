"""On-GPU JPEG reconstruction for camera-trap ingest (survey §5.8(4) / §7.5.4).

Camera-trap clients post multi-megapixel JPEG frames (the reference's detection API takes image files:
``APIs/Charts/camera-trap/detection-async/prod-values.yaml``; ``APIs/2.0/camera-trap/detection-sync``). On the CPU path
(:func:`runtime.decode.decode_image`) a frame costs ~8 ms of a core (PIL: DCT-domain draft decode + bilinear
resize), so a node's CPUs, not its GPUs, set the ingest ceiling. Here the CPU only parses the headers and copies the
entropy-coded bytes (``_ai4e_core.jpeg_scan_prepare``, ~0.2 ms); everything else runs as HIP kernels
(``csrc/kernels/jpeg.hip``): parallel Huffman decoding over self-synchronising spans, dequantisation + libjpeg's
scaled IDCTs, YCbCr -> RGB and PIL's two-pass bilinear resize, straight into the model's uint8 HWC input.

The output is bit-identical to ``decode_image`` (the CPU path the endpoints use): the same draft scale PIL picks,
libjpeg's per-component IDCT sizes (chroma scaled up in the IDCT instead of upsampled), libjpeg's integer IDCTs and
colour tables, and PIL's fixed-point resample coefficients, computed here with PIL's own double arithmetic.
Frames outside that envelope (progressive, restart intervals, CMYK, chroma that would need upsampling, a resize with
PIL's ``reducing_gap`` pre-reduction) and frames whose decode reports an error are decoded on the CPU instead.
"""
from __future__ import annotations

import functools
import math
import struct
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

SCAN_MAGIC = 0x3153434A  # "JCS1" (csrc/core/jpeg_layout.h)
COEF_MAGIC = 0x314F434A  # "JCO1"
PRECISION_BITS = 22      # PIL Resample.c (32 - 8 - 2)
DEFAULT_SPAN_BITS = 2048  # bits per decoder thread: 85-95 % of speculative spans synchronise inside their own span; a pass
# costs ~one span's decode latency, so shorter spans finish sooner (4096: 12.8k frames/s, 2048: 15.1k, 1024: 14.8k)
DEFAULT_SYNC_PASSES = 8  # parallel passes; 2048-bit spans settle in 3-8 on the frames tested, the fix-up kernel finishes the rest
ST_OK, ST_UNSUPPORTED, ST_CORRUPT, ST_NOROOM = 0, 1, 2, 3


# ---------------------------------------------------------------------------------------------------------------- plan
@dataclass(frozen=True)
class FramePlan:
    width: int
    height: int
    ncomp: int
    hmax: int
    vmax: int
    comp: Tuple[Tuple[int, ...], ...]  # per component: h, v, blocks_w, blocks_h, first, tq
    scale: int                         # PIL draft scale (1, 2, 4, 8)
    ssize: Tuple[int, ...]             # IDCT output size per component
    src_w: int                         # decoded (draft) size
    src_h: int
    out_w: int
    out_h: int
    nblocks: int

    @property
    def plane_dims(self) -> List[Tuple[int, int]]:
        """(pitch, rows) of each component plane at the output scale."""
        return [(c[2] * s, c[3] * s) for c, s in zip(self.comp, self.ssize)]


def draft_scale(width: int, height: int, out_w: int, out_h: int) -> int:
    """The scale ``decode_image`` decodes at: PIL's ``draft()`` when the frame is >= 2x the model input."""
    if not (width >= 2 * out_w or height >= 2 * out_h):
        return 1
    scale = min(width // out_w, height // out_h)
    for s in (8, 4, 2, 1):
        if scale >= s:
            return s
    return 1


def component_ssize(hmax: int, vmax: int, h: int, v: int, scale: int) -> Tuple[int, int, int]:
    """libjpeg-turbo jdmaster.c: the IDCT size of a component when decoding at 1/scale (chroma is scaled up through the
    IDCT where the subsampling allows, instead of upsampled). Returns (ssize, h_expand, v_expand)."""
    min_s = 8 // scale
    ss = min_s
    while ss < 8 and (hmax * min_s) % (h * ss * 2) == 0 and (vmax * min_s) % (v * ss * 2) == 0:
        ss *= 2
    return ss, (hmax * min_s) // (h * ss), (vmax * min_s) // (v * ss)


_HDR = struct.Struct("<40I")


def parse_header(buf) -> dict:
    """The fixed part of a prepared frame (JpegScanHeader or JpegCoefHeader)."""
    u32 = _HDR.unpack_from(buf)
    magic, W, H, nc, hmax, vmax, nb, nbytes = u32[:8]
    nc = min(nc, 3)
    comp = tuple(u32[8 + 8 * c: 16 + 8 * c] for c in range(nc))
    d = dict(magic=magic, width=W, height=H, ncomp=nc, hmax=hmax, vmax=vmax, nblocks=nb, data_bytes=nbytes, comp=comp)
    if magic == SCAN_MAGIC:
        d.update(mcux=u32[32], mcuy=u32[33], bpm=u32[34], total_bits=u32[36])
    return d


def plan_frame(hdr: dict, out_w: int, out_h: int, out_c: int = 3) -> Optional[FramePlan]:
    """The GPU plan of a frame for a (out_h, out_w, out_c) model input, or None when the CPU path must decode it."""
    return _plan(hdr["width"], hdr["height"], hdr["ncomp"], hdr["hmax"], hdr["vmax"],
                 tuple(tuple(c[:6]) for c in hdr["comp"]), hdr["nblocks"], out_w, out_h, out_c)


@functools.lru_cache(maxsize=1024)
def _plan(W, H, ncomp, hmax, vmax, comps, nblocks, out_w, out_h, out_c) -> Optional[FramePlan]:
    hdr = dict(width=W, height=H, ncomp=ncomp, hmax=hmax, vmax=vmax, comp=comps, nblocks=nblocks)
    if out_c != 3:
        return None
    s = draft_scale(W, H, out_w, out_h)
    src_w, src_h = -(-W // s), -(-H // s)
    # Image.resize(reducing_gap=2.0) pre-reduces by box averaging when the size is >= 4x the target: CPU path
    if max(int(src_w / out_w / 2.0), 1) > 1 or max(int(src_h / out_h / 2.0), 1) > 1:
        return None
    ss = []
    for c in hdr["comp"]:
        size, he, ve = component_ssize(hdr["hmax"], hdr["vmax"], c[0], c[1], s)
        if he != 1 or ve != 1:
            return None  # would need libjpeg's fancy upsampling
        ss.append(size)
    return FramePlan(W, H, hdr["ncomp"], hdr["hmax"], hdr["vmax"], tuple(c[:6] for c in hdr["comp"]), s, tuple(ss),
                     src_w, src_h, out_w, out_h, hdr["nblocks"])


# ---------------------------------------------------------------------------------------- PIL resample coefficients
def pil_bilinear_coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray]:
    """PIL ``precompute_coeffs`` + ``normalize_coeffs_8bpc`` for the bilinear filter over the box (0, in_size), in the
    same double arithmetic: (bounds int32 [out, 2] = (first, count), coefficients int32 [out, ksize])."""
    if in_size == out_size:  # PIL skips the pass; an identity table gives the same bytes
        return (np.stack([np.arange(out_size), np.ones(out_size, np.int64)], 1).astype(np.int32),
                np.full((out_size, 1), 1 << PRECISION_BITS, np.int32))
    scale = float(in_size) / out_size
    filterscale = scale if scale >= 1.0 else 1.0
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    one = float(1 << PRECISION_BITS)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = (x + xmin - center + 0.5) * ss
            if t < 0.0:
                t = -t
            v = 1.0 - t if t < 1.0 else 0.0
            w.append(v)
            ww += v
        for x in range(xmax):
            v = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + v * one) if v < 0 else int(0.5 + v * one)
        bounds[xx] = (xmin, xmax)
    return bounds, kk


# ------------------------------------------------------------------------------------------- numpy reference (tests)
_ISLOW = dict(a=2446, b=3196, c=4433, d=6270, e=7373, f=9633, g=12299, h=15137, i=16069, j=16819, k=20995, l=25172)


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def _range_limit(x):
    y = (x + 128) & 1023
    return np.where(y < 256, y, np.where(y < 640, 255, 0))


def _islow_1d(x, shift):
    K = _ISLOW
    z1 = (x[2] + x[6]) * K["c"]
    tmp2, tmp3 = z1 - x[6] * K["h"], z1 + x[2] * K["d"]
    tmp0, tmp1 = (x[0] + x[4]) << 13, (x[0] - x[4]) << 13
    t10, t13, t11, t12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
    o0, o1, o2, o3 = x[7], x[5], x[3], x[1]
    z1, z2, z3, z4 = o0 + o3, o1 + o2, o0 + o2, o1 + o3
    z5 = (z3 + z4) * K["f"]
    o0, o1, o2, o3 = o0 * K["a"], o1 * K["j"], o2 * K["l"], o3 * K["g"]
    z1, z2, z3, z4 = -z1 * K["e"], -z2 * K["k"], -z3 * K["i"] + z5, -z4 * K["b"] + z5
    o0, o1, o2, o3 = o0 + z1 + z3, o1 + z2 + z4, o2 + z2 + z3, o3 + z1 + z4
    s = shift
    return [_descale(t10 + o3, s), _descale(t11 + o2, s), _descale(t12 + o1, s), _descale(t13 + o0, s),
            _descale(t13 - o0, s), _descale(t12 - o1, s), _descale(t11 - o2, s), _descale(t10 - o3, s)]


def _red4_1d(x, shift):
    t0 = x[0] << 14
    t2 = x[2] * 15137 - x[6] * 6270
    t10, t12 = t0 + t2, t0 - t2
    e0 = -x[7] * 1730 + x[5] * 11893 - x[3] * 17799 + x[1] * 8697
    e2 = -x[7] * 4176 - x[5] * 4926 + x[3] * 7373 + x[1] * 20995
    return [_descale(t10 + e2, shift), _descale(t12 + e0, shift), _descale(t12 - e0, shift), _descale(t10 - e2, shift)]


def _red2_1d(x, shift):
    t10 = x[0] << 15
    t0 = -x[7] * 5906 + x[5] * 6967 - x[3] * 10426 + x[1] * 29692
    return [_descale(t10 + t0, shift), _descale(t10 - t0, shift)]


def idct_reference(d: np.ndarray, size: int) -> np.ndarray:
    """libjpeg's IDCT of dequantised int64 blocks [n, 8, 8] (rows = vertical frequency) to uint8 [n, size, size]."""
    n = d.shape[0]
    if size == 1:
        return _range_limit(_descale(d[:, 0, 0], 3)).astype(np.uint8).reshape(n, 1, 1)
    fn = {8: (_islow_1d, 11, 18), 4: (_red4_1d, 12, 19), 2: (_red2_1d, 13, 20)}[size][0]
    s1, s2 = {8: (11, 18), 4: (12, 19), 2: (13, 20)}[size]
    used = {8: range(1, 8), 4: (1, 2, 3, 5, 6, 7), 2: (1, 3, 5, 7)}[size]
    ws = np.zeros((n, size, 8), np.int64)
    for c in range(8):
        x = [d[:, r, c] for r in range(8)]
        zero = np.all([x[r] == 0 for r in used], 0)
        o = fn(x, s1)
        for r in range(size):
            ws[:, r, c] = np.where(zero, x[0] << 2, o[r])
    out = np.zeros((n, size, size), np.int64)
    for r in range(size):
        x = [ws[:, r, c] for c in range(8)]
        zero = np.all([x[c] == 0 for c in used], 0)
        o = fn(x, s2)
        for c in range(size):
            out[:, r, c] = np.where(zero, _descale(x[0], 5), o[c])
    return _range_limit(out).astype(np.uint8)


def coef_planes(buf) -> Tuple[dict, List[np.ndarray]]:
    """Dense dequantisation-ready blocks per component from the CPU coefficient decoder's layout (JpegCoefHeader)."""
    from aiforearth_api_platform_amd import _ai4e_core as core

    hdr = parse_header(buf)
    quant = np.frombuffer(buf, np.uint16, 256, 128).reshape(4, 64).astype(np.int64)
    hb = core.JPEG_COEF_HEADER_BYTES
    nb = hdr["nblocks"]
    offs = np.frombuffer(buf, np.uint32, nb, hb).astype(np.int64)
    data = np.frombuffer(buf, np.uint8, hdr["data_bytes"], hb + 4 * nb)
    coefs = np.zeros((nb, 64), np.int64)
    cnt = offs >> 24
    start = offs & 0xFFFFFF
    idx = np.repeat(np.arange(nb), cnt)
    pos = np.repeat(start, cnt) + 3 * (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    val = (data[pos + 1].astype(np.int16) | (data[pos + 2].astype(np.int16) << 8)).astype(np.int64)
    coefs[idx, data[pos]] = val
    blocks = []
    for c in hdr["comp"]:
        bw, bh, first, tq = c[2], c[3], c[4], c[5]
        blocks.append((coefs[first:first + bw * bh] * quant[tq][None]).reshape(bh, bw, 8, 8))
    return hdr, blocks


def reconstruct_reference(blocks: List[np.ndarray], plan: FramePlan) -> np.ndarray:
    """Dequantised blocks per component ([bh, bw, 8, 8] each) -> uint8 [out_h, out_w, 3]: the kernels' IDCT, colour
    and resize steps in numpy."""
    h_out, w_out = plan.out_h, plan.out_w
    planes = []
    for b, s in zip(blocks, plan.ssize):
        bh, bw = b.shape[:2]
        px = idct_reference(b.reshape(-1, 8, 8), s).reshape(bh, bw, s, s).transpose(0, 2, 1, 3).reshape(bh * s, bw * s)
        planes.append(px[:plan.src_h, :plan.src_w].astype(np.int64))
    if plan.ncomp == 3:
        y, cb, cr = planes[0], planes[1] - 128, planes[2] - 128
        rgb = np.stack([y + ((91881 * cr + 32768) >> 16), y + ((-22554 * cb - 46802 * cr + 32768) >> 16),
                        y + ((116130 * cb + 32768) >> 16)], -1)
        rgb = np.clip(rgb, 0, 255)
    else:
        rgb = np.repeat(planes[0][..., None], 3, -1)
    hb_, hk = pil_bilinear_coeffs(plan.src_w, w_out)
    vb_, vk = pil_bilinear_coeffs(plan.src_h, h_out)
    rows = np.zeros((plan.src_h, w_out, 3), np.int64)
    for xo in range(w_out):
        x0, n = hb_[xo]
        rows[:, xo] = np.clip(((1 << 21) + np.einsum("k,hkc->hc", hk[xo, :n].astype(np.int64), rgb[:, x0:x0 + n]))
                              >> PRECISION_BITS, 0, 255)
    out = np.zeros((h_out, w_out, 3), np.int64)
    for yo in range(h_out):
        y0, n = vb_[yo]
        out[yo] = np.clip(((1 << 21) + np.einsum("k,kwc->wc", vk[yo, :n].astype(np.int64), rows[y0:y0 + n]))
                          >> PRECISION_BITS, 0, 255)
    return out.astype(np.uint8)


def reference_decode(body: bytes, shape: Tuple[int, int, int]) -> Optional[np.ndarray]:
    """The GPU pipeline in numpy over the CPU Huffman decoder's coefficients (tests: bit-exact vs ``decode_image``)."""
    from aiforearth_api_platform_amd import _ai4e_core as core

    h_out, w_out, c_out = shape
    buf = np.zeros(max(8 << 20, 8 * len(body)), np.uint8)
    st, used = core.jpeg_coef_decode(body, buf.ctypes.data, buf.nbytes)
    if st != ST_OK:
        return None
    hdr, blocks = coef_planes(buf[:used].tobytes())
    plan = plan_frame(hdr, w_out, h_out, c_out)
    if plan is None:
        return None
    return reconstruct_reference(blocks, plan)


def decode_prepared_cpu(prepared: np.ndarray, shape: Tuple[int, int, int]) -> Optional[np.ndarray]:
    """Decode a prepared frame (uint8 array holding a JpegScanHeader + scan) on the CPU: the kernels' span decoder run
    sequentially (``_ai4e_core.jpeg_scan_coefs``) + the numpy reconstruction. Workers on CPU devices; None if the frame
    is corrupt or outside the plan."""
    from aiforearth_api_platform_amd import _ai4e_core as core

    prepared = np.ascontiguousarray(prepared)
    hdr = parse_header(prepared[:160].tobytes())
    plan = plan_frame(hdr, shape[1], shape[0], shape[2])
    if hdr["magic"] != SCAN_MAGIC or plan is None:
        return None
    coef = np.zeros((hdr["nblocks"], 64), np.int16)
    if core.jpeg_scan_coefs(prepared.ctypes.data, prepared.nbytes, coef.ctypes.data) != 0:
        return None
    u8 = prepared[:core.JPEG_SCAN_HEADER_BYTES]
    bc, bdy, bdx = u8[160:176].astype(np.int64), u8[176:192].astype(np.int64), u8[192:208].astype(np.int64)
    quant = u8[224:736].view(np.uint16).reshape(4, 64).astype(np.int64)
    q = np.arange(hdr["nblocks"])
    m, k = q // hdr["bpm"], q % hdr["bpm"]
    blocks = []
    for c, comp in enumerate(hdr["comp"]):
        h, v, bw, bh, _, tq = comp[:6]
        sel = bc[k] == c
        row = (m[sel] // hdr["mcux"]) * v + bdy[k[sel]]
        col = (m[sel] % hdr["mcux"]) * h + bdx[k[sel]]
        blk = np.zeros((bh, bw, 64), np.int64)
        blk[row, col] = coef[sel].astype(np.int64) * quant[tq][None]
        blocks.append(blk.reshape(bh, bw, 8, 8))
    return reconstruct_reference(blocks, plan)


# ------------------------------------------------------------------------------------------------ payload-ring slots
# A request's JPEG body can be prepared straight into its payload-ring slot (front-ends: model_endpoint.py,
# csrc/ingest/ingestd.cpp); the slot then ends with a JpegSlotTrailer holding the ring's key, and the worker decodes
# it on the GPU into the model input (engine.py). csrc/core/jpeg_layout.h.
SLOT_MAGIC = 0x3153504A45344941  # "AI4EJPS1"
RING_TAIL_MAGIC = 0x474E495245344941  # "AI4ERING"
RING_TAIL_BYTES = 64
TRAILER_BYTES = 32
JPEG_TYPES = ("image/jpeg", "image/jpg", "image/pjpeg")


def init_ring_tail(shm_buf, nbytes: int, enabled: bool) -> int:
    """Write the ring's tail (after ``nbytes`` of slots): magic + a random key (0 = prepared frames disabled)."""
    import secrets

    key = (secrets.randbits(63) | 1) if enabled else 0
    np.frombuffer(shm_buf, np.uint64, 2, nbytes)[:] = (RING_TAIL_MAGIC, key)
    return key


def ring_key(shm_buf, nbytes: int) -> int:
    """The key of a ring whose shared memory holds a tail, else 0."""
    if len(shm_buf) < nbytes + RING_TAIL_BYTES:
        return 0
    magic, key = (int(x) for x in np.frombuffer(shm_buf, np.uint64, 2, nbytes))
    return key if magic == RING_TAIL_MAGIC else 0


def prepare_into_slot(body: bytes, slot_addr: int, item_bytes: int, shape: Tuple[int, int, int], key: int) -> bool:
    """Prepare a JPEG body into a slot (address ``slot_addr``) and mark it; False (slot untouched as far as the
    trailer goes) when the frame must be decoded on the CPU instead."""
    from aiforearth_api_platform_amd import _ai4e_core as core

    if not key or item_bytes <= core.JPEG_SCAN_HEADER_BYTES + TRAILER_BYTES + 64:
        return False
    st, used = core.jpeg_scan_prepare(body, slot_addr, item_bytes - TRAILER_BYTES)
    if st != ST_OK:
        return False
    import ctypes

    hdr = parse_header(ctypes.string_at(slot_addr, 160))
    if plan_frame(hdr, shape[1], shape[0], shape[2]) is None:
        return False
    trailer = np.array([SLOT_MAGIC, key, used], np.uint64)
    ctypes.memmove(slot_addr + item_bytes - TRAILER_BYTES, trailer.ctypes.data, 24)
    return True


def slot_frames(ring_u8: np.ndarray, slots: Sequence[int], key: int) -> List[Tuple[int, int]]:
    """[(index in ``slots``, prepared bytes)] of the slots that hold prepared frames (``ring_u8``: [nslots, item])."""
    if not key or len(slots) == 0:
        return []
    tail = ring_u8[np.asarray(slots, np.int64), -TRAILER_BYTES:]
    words = np.ascontiguousarray(tail).view(np.uint64)
    hit = np.nonzero((words[:, 0] == np.uint64(SLOT_MAGIC)) & (words[:, 1] == np.uint64(key)))[0]
    item = ring_u8.shape[1]
    return [(int(j), int(words[j, 2])) for j in hit if 0 < int(words[j, 2]) <= item - TRAILER_BYTES]


# ----------------------------------------------------------------------------------------------------- GPU decoder
_DESC_FIELDS = ([("scan", "u8"), ("coef", "u8"), ("blen", "u8"), ("exit0", "u8"), ("exit1", "u8"), ("chg0", "u8"), ("chg1", "u8"),
                 ("counts", "u8"), ("planes", "u8"), ("rows", "u8"), ("out", "u8"), ("hk", "u8"), ("hb", "u8"),
                 ("vk", "u8"), ("vb", "u8"), ("status", "u8"), ("nthreads", "i4"), ("span_bits", "i4"), ("hks", "i4"),
                 ("vks", "i4")] + [(f"ssize{i}", "i4") for i in range(3)] + [(f"plane_off{i}", "i4") for i in range(3)]
                + [(f"plane_pitch{i}", "i4") for i in range(3)]
                + [(k, "i4") for k in ("src_w", "src_h", "out_w", "out_h", "out_c", "kbase1", "kbase2")])
DESC_DTYPE = np.dtype(_DESC_FIELDS)
assert DESC_DTYPE.itemsize == 208  # sizeof(JpegFrameDesc)


def _align(n: int, a: int = 256) -> int:
    return (n + a - 1) // a * a


def header_sane(hdr: dict, used: int) -> bool:
    """Consistency of a prepared frame's header with its own geometry and size (the worker checks what the front-end
    wrote before any kernel reads it)."""
    from aiforearth_api_platform_amd import _ai4e_core as core

    try:
        W, H, nc, hm, vm = hdr["width"], hdr["height"], hdr["ncomp"], hdr["hmax"], hdr["vmax"]
        if hdr["magic"] != SCAN_MAGIC or nc not in (1, 3) or not (0 < W <= 65535 and 0 < H <= 65535):
            return False
        if core.JPEG_SCAN_HEADER_BYTES + hdr["data_bytes"] + 64 > used or hdr["total_bits"] > 8 * hdr["data_bytes"]:
            return False
        if nc == 1:
            mcux, mcuy, bpm = -(-W // 8), -(-H // 8), 1
        else:
            mcux, mcuy = -(-W // (8 * hm)), -(-H // (8 * vm))
            bpm = sum(c[0] * c[1] for c in hdr["comp"])
        if (hdr["mcux"], hdr["mcuy"], hdr["bpm"]) != (mcux, mcuy, bpm) or bpm > 10:
            return False
        nb = 0
        for c in hdr["comp"]:
            h, v, bw, bh, first, tq = c[:6]
            if nc == 3 and (bw != mcux * h or bh != mcuy * v):
                return False
            if first != nb or tq > 3 or c[6] > 1 or c[7] > 1:
                return False
            nb += bw * bh
        return nb == hdr["nblocks"] == mcux * mcuy * bpm
    except (KeyError, IndexError, TypeError):
        return False


class JpegLauncher:
    """Device work areas + frame descriptors + one ``ai4e_jpeg_decode`` launch for a batch of prepared frames that are
    already on the device. Launches on one stream are ordered, so the work areas and the coefficient array (zero
    between batches: the IDCT clears what it reads) are reused batch after batch."""

    def __init__(self, device, span_bits: int = DEFAULT_SPAN_BITS, sync_passes: int = DEFAULT_SYNC_PASSES):
        import torch

        from aiforearth_api_platform_amd.ops import _ext

        self.torch, self._ext = torch, _ext
        _ext.lib()  # loud failure when the kernel library is missing
        self.device = torch.device(device)
        self.span_bits = int(span_bits)
        self.sync_passes = int(sync_passes)
        self._work = None
        self._coef = None
        self._blen = None
        self._coeff_cache = {}
        self._templates = {}

    def _resample(self, n_in: int, n_out: int):
        t = self._coeff_cache.get((n_in, n_out))
        if t is None:
            bounds, kk = pil_bilinear_coeffs(n_in, n_out)
            torch = self.torch
            t = (torch.from_numpy(bounds).to(self.device), torch.from_numpy(kk).to(self.device), kk.shape[1])
            self._coeff_cache[(n_in, n_out)] = t
        return t

    def grow(self, cur, nbytes: int):
        """A uint8 device area of at least ``nbytes`` (``cur`` when it is large enough)."""
        return self._buf(cur, nbytes)

    def _buf(self, cur, nbytes: int, zero: bool = False):
        torch = self.torch
        if cur is not None and cur.numel() * cur.element_size() >= nbytes:
            return cur
        n = _align(max(int(nbytes * 1.25), 1), 1 << 20)
        if zero:
            return torch.zeros(n // 2, dtype=torch.int16, device=self.device)
        return torch.empty(n, dtype=torch.uint8, device=self.device)

    def _template(self, plan: FramePlan):
        """The plan-dependent part of a descriptor (+ its planes / rows bytes), built once per plan."""
        t = self._templates.get(plan)
        if t is None:
            d = np.zeros(1, DESC_DTYPE)[0]
            dims = plan.plane_dims
            poff = 0
            for c in range(3):
                if c < plan.ncomp:
                    d[f"ssize{c}"], d[f"plane_off{c}"], d[f"plane_pitch{c}"] = plan.ssize[c], poff, dims[c][0]
                    poff += dims[c][0] * dims[c][1]
                else:
                    d[f"ssize{c}"], d[f"plane_off{c}"], d[f"plane_pitch{c}"] = 1, 0, dims[0][0]
            d["span_bits"] = self.span_bits
            d["src_w"], d["src_h"], d["out_w"], d["out_h"], d["out_c"] = plan.src_w, plan.src_h, plan.out_w, plan.out_h, 3
            hv = [c[0] * c[1] for c in plan.comp]
            d["kbase1"] = hv[0]
            d["kbase2"] = hv[0] + (hv[1] if len(hv) > 1 else 0)
            hb, hk, hks = self._resample(plan.src_w, plan.out_w)
            vb, vk, vks = self._resample(plan.src_h, plan.out_h)
            d["hb"], d["hk"], d["hks"] = hb.data_ptr(), hk.data_ptr(), hks
            d["vb"], d["vk"], d["vks"] = vb.data_ptr(), vk.data_ptr(), vks
            t = (d, poff, plan.src_h * plan.out_w * 3)
            self._templates[plan] = t
        return t

    def launch(self, frames, stream):
        """``frames``: [(hdr, plan, device address of the prepared bytes, device address of the uint8 HWC output)].
        Returns the per-frame status (int32 device tensor: 0 ok, bit 1 corrupt data) and what must stay alive until
        the launch has run. Descriptors are built column-wise (one template per distinct plan)."""
        torch = self.torch
        n = len(frames)
        with torch.cuda.stream(stream):
            tmpl = [self._template(p) for _, p, _, _ in frames]
            descs = np.array([t[0] for t in tmpl], DESC_DTYPE)
            nthr = np.array([max(1, -(-h["total_bits"] // self.span_bits)) for h, _, _, _ in frames], np.int64)
            nblk = np.array([h["nblocks"] for h, _, _, _ in frames], np.int64)
            al = lambda x: (x + 255) // 256 * 256  # noqa: E731
            e8, c4, c16 = al(8 * nthr), al(4 * nthr), al(16 * nthr)
            pl = al(np.array([t[1] for t in tmpl], np.int64))
            rw = al(np.array([t[2] for t in tmpl], np.int64))
            per = 2 * e8 + 2 * c4 + c16 + pl + rw
            fbase = np.concatenate([[0], np.cumsum(per)[:-1]])
            cbytes = nblk * 128
            cb = np.concatenate([[0], np.cumsum(cbytes)[:-1]])
            self._work = self._buf(self._work, int(per.sum()))
            self._coef = self._buf(self._coef, int(cbytes.sum()), zero=True)
            self._blen = self._buf(self._blen, int(nblk.sum()) + 2, zero=True)  # (int16 storage, byte offsets)
            status = torch.zeros(n, dtype=torch.int32, device=self.device)
            w = self._work.data_ptr() + fbase
            descs["exit0"], descs["exit1"] = w, w + e8
            descs["chg0"], descs["chg1"] = w + 2 * e8, w + 2 * e8 + c4
            descs["counts"] = w + 2 * e8 + 2 * c4
            descs["planes"] = w + 2 * e8 + 2 * c4 + c16
            descs["rows"] = w + 2 * e8 + 2 * c4 + c16 + pl
            descs["coef"] = self._coef.data_ptr() + cb
            descs["blen"] = self._blen.data_ptr() + np.concatenate([[0], np.cumsum(nblk)[:-1]])
            descs["scan"] = np.array([f[2] for f in frames], np.uint64)
            descs["out"] = np.array([f[3] for f in frames], np.uint64)
            descs["status"] = status.data_ptr() + 4 * np.arange(n, dtype=np.uint64)
            descs["nthreads"] = nthr
            max_rows = int(max(t[0]["src_h"] for t in tmpl)) * int(max(t[0]["out_w"] for t in tmpl))
            max_out = int(max(t[0]["out_h"] * t[0]["out_w"] for t in tmpl)) * 3
            self.last_descs = descs  # (debugging: device addresses of the last batch's work areas)
            ddesc = torch.from_numpy(descs.view(np.uint8)).pin_memory().to(self.device, non_blocking=True)
            self._ext.call("ai4e_jpeg_decode", ddesc.data_ptr(), n, int(nthr.max()), int(nblk.max()), max_rows, max_out,
                           self.sync_passes, stream.cuda_stream)
        return status, ddesc


@dataclass
class Pending:
    """A submitted batch: ``finish()`` reads its statuses and decodes the frames the GPU did not on the CPU."""
    bodies: Sequence[bytes]
    out: object
    gpu: List[int]
    cpu: List[int]
    status: object = None
    keep: tuple = ()


class JpegGpuDecoder:
    """Batched on-GPU decode of JPEG bodies to uint8 [B, H, W, 3] on ``device`` (bit-identical to ``decode_image``).

    ``submit(bodies)`` prepares the frames on ``threads`` CPU threads (header parse + unstuffed copy into pinned
    staging, laid out back to back so one copy moves the batch), copies them to the GPU and launches the kernels on the
    current stream without waiting; ``finish(pending)`` reads the per-frame statuses (one small read per batch) and
    decodes on the CPU (``decode_image``) the frames the GPU path does not cover or whose data is corrupt. Two batches
    may be in flight (double-buffered staging), so a caller overlaps preparing batch i+1 with the GPU decoding batch i.
    ``errors`` holds the message of each frame that could not be decoded at all (its output is left zero).
    """

    def __init__(self, shape: Tuple[int, int, int], device="cuda", threads: int = 8, span_bits: int = DEFAULT_SPAN_BITS,
                 sync_passes: int = DEFAULT_SYNC_PASSES):
        import torch

        from aiforearth_api_platform_amd import _ai4e_core as core

        self.torch, self.core = torch, core
        self.shape = tuple(shape)
        self.device = torch.device(device)
        self.launcher = JpegLauncher(self.device, span_bits, sync_passes)
        self.hdr_bytes = int(core.JPEG_SCAN_HEADER_BYTES)
        self.threads = max(1, int(threads))
        self.pool = ThreadPoolExecutor(self.threads, thread_name_prefix="jpeg-prep")
        self._staging: List = [None, None]  # pinned host staging, double-buffered across batches
        self._staging_evt: List = [None, None]
        self._scan: List = [None, None]
        self._scan_done: List = [None, None]
        self.copy_stream = torch.cuda.Stream(self.device)
        self._flip = 0
        self._lock = threading.Lock()
        self.errors = {}
        self.stats = dict(frames=0, gpu_frames=0, cpu_frames=0, unsupported=0, failed=0)
        self.host_s = dict(staging_wait=0.0, prepare=0.0, plan=0.0, launch=0.0, finish=0.0)  # host seconds by step

    def _pinned(self, nbytes: int):
        torch = self.torch
        i = self._flip
        if self._staging_evt[i] is not None:
            self._staging_evt[i].synchronize()  # the copy out of this staging buffer (two batches ago) is done
        buf = self._staging[i]
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(_align(int(nbytes * 1.25), 1 << 20), dtype=torch.uint8, pin_memory=True)
            self._staging[i] = buf
        return buf

    def decode(self, bodies: Sequence[bytes], out=None):
        """uint8 [len(bodies), H, W, 3] on the device (``out`` if given), all frames decoded."""
        return self.finish(self.submit(bodies, out))

    def submit(self, bodies: Sequence[bytes], out=None) -> Pending:
        torch = self.torch
        h_out, w_out, c_out = self.shape
        B = len(bodies)
        if out is None:
            out = torch.empty((B, h_out, w_out, c_out), dtype=torch.uint8, device=self.device)
        if B == 0:
            return Pending(bodies, out, [], [])
        # frame i's prepared bytes fit in header + its body + padding: back-to-back offsets known before preparing
        caps = [_align(self.hdr_bytes + len(b) + 128) for b in bodies]
        offs = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64)
        t0 = time.perf_counter()
        staging = self._pinned(int(offs[-1]))
        t1 = time.perf_counter()
        base = staging.data_ptr()
        nt = min(self.threads, B)

        def chunk(k):  # one task per thread (a future per frame costs more than the frame's header parse)
            return [self.core.jpeg_scan_prepare(bodies[i], base + int(offs[i]), caps[i]) for i in range(k, B, nt)]

        parts = list(self.pool.map(chunk, range(nt)))
        results = [parts[i % nt][i // nt] for i in range(B)]
        t2 = time.perf_counter()
        host = staging.numpy()
        frames, gpu, cpu = [], [], []
        for i, (st, used) in enumerate(results):
            if st == ST_OK:
                hdr = parse_header(host[offs[i]:offs[i] + 160])
                plan = plan_frame(hdr, w_out, h_out, c_out)
                if plan is not None:
                    frames.append((hdr, plan, int(offs[i]), out[i].data_ptr()))
                    gpu.append(i)
                    continue
            cpu.append(i)
        pending = Pending(bodies, out, gpu, cpu)
        t3 = time.perf_counter()
        if gpu:
            k = self._flip
            stream = torch.cuda.current_stream(self.device)
            total = int(offs[gpu[-1] + 1])
            # the batch's bytes go up on a copy stream, under the previous batch's kernels; scan area k is rewritten
            # only once the decode that read it (two batches ago) is done
            cs = self.copy_stream
            with torch.cuda.stream(cs):
                if self._scan_done[k] is not None:
                    cs.wait_event(self._scan_done[k])
                self._scan[k] = self.launcher._buf(self._scan[k], total)
                self._scan[k][:total].copy_(staging[:total], non_blocking=True)  # the whole batch in one copy
            evt = torch.cuda.Event()
            evt.record(cs)
            self._staging_evt[k] = evt
            stream.wait_event(evt)
            self._scan[k].record_stream(stream)
            sbase = self._scan[k].data_ptr()
            frames = [(h, p, sbase + o, dst) for h, p, o, dst in frames]
            status, keep = self.launcher.launch(frames, stream)
            # statuses into pinned memory behind the decode: finish() waits for this batch only, not for batches
            # submitted after it (a .cpu() on the stream would)
            host = torch.empty(status.numel(), dtype=torch.int32, pin_memory=True)
            with torch.cuda.stream(stream):
                host.copy_(status, non_blocking=True)
            done = torch.cuda.Event()
            done.record(stream)
            self._scan_done[k] = done
            pending.status = (host, done)
            pending.keep = (keep, self._scan[k], status)
        self._flip ^= 1
        t4 = time.perf_counter()
        with self._lock:
            self.stats["frames"] += B
            self.stats["unsupported"] += len(cpu)
            h = self.host_s
            h["staging_wait"] += t1 - t0
            h["prepare"] += t2 - t1
            h["plan"] += t3 - t2
            h["launch"] += t4 - t3
        return pending

    def finish(self, p: Pending):
        torch = self.torch
        t0 = time.perf_counter()
        cpu = list(p.cpu)
        if p.status is not None:
            host, done = p.status
            done.synchronize()
            st = host.numpy()
            bad = [p.gpu[j] for j in np.nonzero(st)[0]]
            with self._lock:
                self.stats["failed"] += len(bad)
                self.stats["gpu_frames"] += len(p.gpu) - len(bad)
            cpu = sorted(cpu + bad)
        if cpu:
            from aiforearth_api_platform_amd.runtime.decode import decode_image

            def one(i):
                try:
                    return decode_image(p.bodies[i], "image/jpeg", self.shape)
                except Exception as e:  # noqa: BLE001 - a bad frame must not fail its batch
                    return e

            for i, a in zip(cpu, self.pool.map(one, cpu)):
                if isinstance(a, Exception):
                    self.errors[id(p.bodies[i])] = str(a)
                    p.out[i].zero_()
                else:
                    p.out[i].copy_(torch.from_numpy(np.require(a, requirements="W")))
            with self._lock:
                self.stats["cpu_frames"] += len(cpu)
        self.host_s["finish"] += time.perf_counter() - t0
        return p.out

    def close(self):
        self.pool.shutdown(wait=True)
