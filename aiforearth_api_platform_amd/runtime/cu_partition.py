"""CU-partitioned HIP streams (csrc/kernels/cu_partition.hip): a stream whose kernels may only occupy a chosen
subset of the device's CUs, wrapped as a ``torch.cuda.ExternalStream`` so graph replays and eager launches
can target it. The serving engine uses two of them (AI4E_ENGINE_CU_SPLIT) to run a batch pipeline's front and
back stages on disjoint CU sets (runtime/engine.py).

CU numbering: bit ``i`` of the mask is the runtime's CU ``i``. Which XCD (and so which L2) a CU belongs to is
learned from a census launch (``census``: the XCC id every workgroup of a launch ran on), so a partition can
take the same share of every XCD (``balanced``)."""
from __future__ import annotations

import ctypes
from collections import Counter
from typing import Dict, List, Optional, Sequence

import torch

from ..ops import _ext

_streams: List[int] = []  # raw handles kept alive for the process lifetime (ExternalStream does not own them)


def cu_count(device: Optional[torch.device] = None) -> int:
    return torch.cuda.get_device_properties(device or torch.cuda.current_device()).multi_processor_count


def mask_words(cus: Sequence[int], total: int) -> List[int]:
    words = [0] * ((total + 31) // 32)
    for c in cus:
        if not 0 <= c < total:
            raise ValueError(f"CU {c} outside 0..{total - 1}")
        words[c // 32] |= 1 << (c % 32)
    return words


def masked_stream(cus: Sequence[int], device: Optional[torch.device] = None) -> torch.cuda.ExternalStream:
    """A stream restricted to the CUs ``cus`` (runtime numbering) of ``device``."""
    device = torch.device(device or "cuda")
    total = cu_count(device)
    words = mask_words(cus, total)
    arr = (ctypes.c_uint32 * len(words))(*words)
    out = ctypes.c_void_p()
    with torch.cuda.device(device):
        _ext.call("ai4e_stream_create_cu_mask", ctypes.cast(arr, ctypes.c_void_p), len(words), ctypes.byref(out))
    _streams.append(out.value)
    return torch.cuda.ExternalStream(out.value, device=device)


def stream_mask(stream: torch.cuda.Stream, total: int) -> List[int]:
    """The CU indices the runtime reports as enabled for ``stream``."""
    n = (total + 31) // 32
    arr = (ctypes.c_uint32 * n)()
    _ext.call("ai4e_stream_get_cu_mask", stream.cuda_stream, ctypes.cast(arr, ctypes.c_void_p), n)
    return [32 * w + b for w in range(n) for b in range(32) if (arr[w] >> b) & 1 and 32 * w + b < total]


def census(stream: torch.cuda.Stream, nblocks: int = 4096, spin_cycles: int = 20000) -> Dict[str, object]:
    """Where ``nblocks`` one-wave workgroups launched on ``stream`` ran: per-XCC workgroup counts and the number
    of distinct (XCC, HW_ID SE/SH/CU) slots seen."""
    out = torch.full((nblocks, 2), -1, dtype=torch.int32, device=stream.device)
    with torch.cuda.stream(stream):
        _ext.call("ai4e_cu_census", out.data_ptr(), nblocks, spin_cycles, stream.cuda_stream)
    stream.synchronize()
    o = out.cpu().tolist()
    xcc = Counter(r[0] for r in o)
    # HW_ID (gfx9): CU_ID bits 11:8, SH_ID bit 12, SE_ID bits 15:13
    slots = {(r[0], (r[1] >> 8) & 0xFF) for r in o}
    return {"per_xcc": dict(sorted(xcc.items())), "cu_slots": len(slots)}


def xcc_of_cus(device: Optional[torch.device] = None) -> List[int]:
    """XCC id of every CU in the runtime's numbering. Two censuses decide between the two layouts a mask can
    have on an 8-XCD part: CUs 0..31 on one XCD (blocked: XCD = c // (total / 8)) or spread over all eight
    (interleaved: XCD = c % 8)."""
    device = torch.device(device or "cuda")
    total = cu_count(device)
    per = total // 8
    first = census(masked_stream(range(per), device), nblocks=8 * per, spin_cycles=20000)["per_xcc"]
    if len(first) == 1:
        return [c // per for c in range(total)]
    if len(first) == 8:
        return [c % 8 for c in range(total)]
    raise RuntimeError(f"unrecognised CU -> XCD layout: CUs 0..{per - 1} ran on XCCs {first}")


def balanced(n: int, xcc: Sequence[int], exclude: Sequence[int] = ()) -> List[int]:
    """``n`` CUs taking (as near as possible) the same number from every XCD, skipping ``exclude``."""
    ex = set(exclude)
    by: Dict[int, List[int]] = {}
    for c, x in enumerate(xcc):
        if c not in ex:
            by.setdefault(x, []).append(c)
    groups = [by[k] for k in sorted(by)]
    out: List[int] = []
    i = 0
    while len(out) < n and any(groups):
        for g in groups:
            if i < len(g) and len(out) < n:
                out.append(g[i])
        i += 1
    return sorted(out)
