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

import math
import threading
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

SCAN_MAGIC = 0x3153434A  # "JCS1" (csrc/core/jpeg_layout.h)
COEF_MAGIC = 0x314F434A  # "JCO1"
PRECISION_BITS = 22      # PIL Resample.c (32 - 8 - 2)
DEFAULT_SPAN_BITS = 4096  # bits per decoder thread: ~99 % of speculative spans synchronise inside their own span
DEFAULT_SYNC_PASSES = 8  # 4096-bit spans settle in <= 4 passes on every frame tested (tests/test_jpeg_gpu.py)
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


def parse_header(buf) -> dict:
    """The fixed part of a prepared frame (JpegScanHeader or JpegCoefHeader)."""
    u32 = np.frombuffer(buf, np.uint32, 40)
    magic, W, H, nc, hmax, vmax, nb, nbytes = (int(x) for x in u32[:8])
    comp = tuple(tuple(int(x) for x in u32[8 + 8 * c: 16 + 8 * c]) for c in range(nc))
    d = dict(magic=magic, width=W, height=H, ncomp=nc, hmax=hmax, vmax=vmax, nblocks=nb, data_bytes=nbytes, comp=comp)
    if magic == SCAN_MAGIC:
        d.update(mcux=int(u32[32]), mcuy=int(u32[33]), bpm=int(u32[34]), total_bits=int(u32[36]))
    return d


def plan_frame(hdr: dict, out_w: int, out_h: int, out_c: int = 3) -> Optional[FramePlan]:
    """The GPU plan of a frame for a (out_h, out_w, out_c) model input, or None when the CPU path must decode it."""
    if out_c != 3:
        return None
    W, H = hdr["width"], hdr["height"]
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


# ----------------------------------------------------------------------------------------------------- GPU decoder
_DESC_FIELDS = ([("scan", "u8"), ("coef", "u8"), ("exit0", "u8"), ("exit1", "u8"), ("chg0", "u8"), ("chg1", "u8"),
                 ("counts", "u8"), ("planes", "u8"), ("rows", "u8"), ("out", "u8"), ("hk", "u8"), ("hb", "u8"),
                 ("vk", "u8"), ("vb", "u8"), ("status", "u8"), ("nthreads", "i4"), ("span_bits", "i4"), ("hks", "i4"),
                 ("vks", "i4")] + [(f"ssize{i}", "i4") for i in range(3)] + [(f"plane_off{i}", "i4") for i in range(3)]
                + [(f"plane_pitch{i}", "i4") for i in range(3)]
                + [(k, "i4") for k in ("src_w", "src_h", "out_w", "out_h", "out_c", "kbase1", "kbase2")])
DESC_DTYPE = np.dtype(_DESC_FIELDS)
assert DESC_DTYPE.itemsize == 200  # sizeof(JpegFrameDesc)


def _align(n: int, a: int = 256) -> int:
    return (n + a - 1) // a * a


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
    staging, laid out back to back so one copy moves the batch), copies them to the GPU and launches
    ``ai4e_jpeg_decode`` on the current stream without waiting; ``finish(pending)`` reads the per-frame statuses (one
    small read per batch) and decodes on the CPU (``decode_image``) the frames the GPU path does not cover or whose
    decode reported an error. Two batches may be in flight (double-buffered staging), so a caller overlaps preparing
    batch i+1 with the GPU decoding batch i. ``errors`` holds the message of each frame that could not be decoded at
    all (its output is left zero).
    """

    def __init__(self, shape: Tuple[int, int, int], device="cuda", threads: int = 8, span_bits: int = DEFAULT_SPAN_BITS,
                 sync_passes: int = DEFAULT_SYNC_PASSES):
        import torch

        from aiforearth_api_platform_amd import _ai4e_core as core
        from aiforearth_api_platform_amd.ops import _ext

        self.torch, self.core, self._ext = torch, core, _ext
        _ext.lib()  # loud failure when the kernel library is missing
        self.shape = tuple(shape)
        self.device = torch.device(device)
        self.span_bits = int(span_bits)
        self.sync_passes = int(sync_passes)
        self.hdr_bytes = int(core.JPEG_SCAN_HEADER_BYTES)
        self.pool = ThreadPoolExecutor(max(1, threads), thread_name_prefix="jpeg-prep")
        self._staging: List = [None, None]  # pinned host staging, double-buffered across batches
        self._staging_evt: List = [None, None]
        self._flip = 0
        self._coef = torch.zeros(0, dtype=torch.int16, device=self.device)  # zero between batches (the IDCT clears it)
        self._work = [torch.empty(0, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self._scan = [torch.empty(0, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self._coeff_cache = {}
        self._lock = threading.Lock()
        self.errors = {}
        self.stats = dict(frames=0, gpu_frames=0, cpu_frames=0, unsupported=0, failed=0)

    # -- helpers
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

    def _resample(self, n_in: int, n_out: int):
        key = (n_in, n_out)
        t = self._coeff_cache.get(key)
        if t is None:
            bounds, kk = pil_bilinear_coeffs(n_in, n_out)
            torch = self.torch
            t = (torch.from_numpy(bounds).to(self.device), torch.from_numpy(kk).to(self.device), kk.shape[1])
            self._coeff_cache[key] = t
        return t

    def _device_buf(self, cur, nbytes: int, zero: bool = False):
        torch = self.torch
        if cur.numel() * cur.element_size() >= nbytes:
            return cur
        n = _align(int(nbytes * 1.25), 1 << 20)
        if zero:
            return torch.zeros(n // 2, dtype=torch.int16, device=self.device)
        return torch.empty(n, dtype=torch.uint8, device=self.device)

    # -- API
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
        staging = self._pinned(int(offs[-1]))
        base = staging.data_ptr()
        results = list(self.pool.map(lambda i: self.core.jpeg_scan_prepare(bodies[i], base + int(offs[i]), caps[i]),
                                     range(B)))
        host = staging.numpy()
        plans: List = []
        for i, (st, used) in enumerate(results):
            plan = None
            if st == ST_OK:
                hdr = parse_header(host[offs[i]:offs[i] + 160])
                p = plan_frame(hdr, w_out, h_out, c_out)
                if p is not None:
                    plan = (p, hdr, used)
            plans.append(plan)
        gpu = [i for i, p in enumerate(plans) if p is not None]
        cpu = [i for i, p in enumerate(plans) if p is None]
        pending = Pending(bodies, out, gpu, cpu)
        if gpu:
            pending.status, pending.keep = self._launch(gpu, plans, staging, offs, out)
        self._flip ^= 1
        with self._lock:
            self.stats["frames"] += B
            self.stats["unsupported"] += len(cpu)
        return pending

    def finish(self, p: Pending):
        torch = self.torch
        cpu = list(p.cpu)
        if p.status is not None:
            st = p.status.cpu().numpy()
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
        return p.out

    def _launch(self, gpu: List[int], plans, staging, offs, out):
        torch = self.torch
        h_out, w_out, c_out = self.shape
        k = self._flip
        total = int(offs[gpu[-1] + 1])
        dscan = self._scan[k] = self._device_buf(self._scan[k], total)
        dscan[:total].copy_(staging[:total], non_blocking=True)  # the whole batch in one copy
        evt = torch.cuda.Event()
        evt.record(torch.cuda.current_stream(self.device))
        self._staging_evt[k] = evt
        descs = np.zeros(len(gpu), DESC_DTYPE)
        work_off = coef_off = 0
        layout = []
        max_threads = max_blocks = max_rows = max_out = 0
        for j, i in enumerate(gpu):
            plan, hdr, used = plans[i]
            nthreads = max(1, -(-hdr["total_bits"] // self.span_bits))
            dims = plan.plane_dims
            sizes = dict(exit0=8 * nthreads, exit1=8 * nthreads, chg0=4 * nthreads, chg1=4 * nthreads,
                         counts=16 * nthreads, planes=sum(pp * r for pp, r in dims), rows=plan.src_h * w_out * c_out)
            fo = {}
            for name, v in sizes.items():
                fo[name] = work_off
                work_off += _align(v)
            layout.append((fo, coef_off))
            coef_off += hdr["nblocks"] * 128
            max_threads = max(max_threads, nthreads)
            max_blocks = max(max_blocks, hdr["nblocks"])
            max_rows = max(max_rows, plan.src_h * w_out)
            max_out = max(max_out, h_out * w_out * c_out)
            d = descs[j]
            d["nthreads"], d["span_bits"] = nthreads, self.span_bits
            poff = 0
            for c in range(3):
                if c < plan.ncomp:
                    d[f"ssize{c}"], d[f"plane_off{c}"], d[f"plane_pitch{c}"] = plan.ssize[c], poff, dims[c][0]
                    poff += dims[c][0] * dims[c][1]
                else:
                    d[f"ssize{c}"], d[f"plane_off{c}"], d[f"plane_pitch{c}"] = 1, 0, dims[0][0]
            d["src_w"], d["src_h"], d["out_w"], d["out_h"], d["out_c"] = plan.src_w, plan.src_h, w_out, h_out, c_out
            hv = [c[0] * c[1] for c in plan.comp]
            d["kbase1"] = hv[0]
            d["kbase2"] = hv[0] + (hv[1] if len(hv) > 1 else 0)
        work = self._work[k] = self._device_buf(self._work[k], work_off)
        self._coef = self._device_buf(self._coef, coef_off, zero=True)
        wbase, cbase, sbase = work.data_ptr(), self._coef.data_ptr(), dscan.data_ptr()
        status = torch.zeros(len(gpu), dtype=torch.int32, device=self.device)
        for j, i in enumerate(gpu):
            plan = plans[i][0]
            fo, coff = layout[j]
            d = descs[j]
            d["scan"] = sbase + int(offs[i])
            d["coef"] = cbase + coff
            for name in ("exit0", "exit1", "chg0", "chg1", "counts", "planes", "rows"):
                d[name] = wbase + fo[name]
            d["status"] = status.data_ptr() + 4 * j
            d["out"] = out[i].data_ptr()
            hb, hk, hks = self._resample(plan.src_w, w_out)
            vb, vk, vks = self._resample(plan.src_h, h_out)
            d["hb"], d["hk"], d["hks"] = hb.data_ptr(), hk.data_ptr(), hks
            d["vb"], d["vk"], d["vks"] = vb.data_ptr(), vk.data_ptr(), vks
        ddesc = torch.from_numpy(descs.view(np.uint8)).pin_memory().to(self.device, non_blocking=True)
        self._ext.call("ai4e_jpeg_decode", ddesc.data_ptr(), len(gpu), max_threads, max_blocks, max_rows, max_out,
                       self.sync_passes, self._ext.stream_ptr(self.device))
        return status, (ddesc, dscan, work)

    def close(self):
        self.pool.shutdown(wait=True)
