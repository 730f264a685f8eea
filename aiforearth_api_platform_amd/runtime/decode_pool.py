"""Decode worker processes: image request bodies decoded straight into payload-ring slots.

JPEG/PNG decoding of real uploads (camera-trap frames are 2-6 MP) costs milliseconds of CPU per image,
orders of magnitude more than everything else the gateway does per request, and Pillow holds the GIL
for part of it. With ``decode_processes: N`` the gateway's image endpoints hand (slot, body) to N
spawned processes that map the node's shared payload ring and write the decoded uint8 image into the
slot themselves, so decode throughput scales with the node's cores (``bench/jpeg_ingest_bench.py``).
The reference decodes inside its single Flask container process (``APIs/1.0/base-py/ai4e_service.py``).
"""
from __future__ import annotations

import multiprocessing as mp
from concurrent.futures import ProcessPoolExecutor
from typing import Optional, Sequence, Tuple

import numpy as np

_RING: Optional[np.ndarray] = None
_SHM = None


def _init(shm_name: str, nslots: int, item_shape: Tuple[int, ...]) -> None:
    global _RING, _SHM
    from multiprocessing import shared_memory

    # spawned from the ring's owner: same resource tracker, so no unregister (worker_pool.SharedPayloadRing)
    _SHM = shared_memory.SharedMemory(name=shm_name)
    _RING = np.ndarray((nslots, *item_shape), dtype=np.uint8, buffer=_SHM.buf)


def _decode_into(slot: int, body: bytes, content_type: str) -> Optional[Tuple[int, str]]:
    """Decode into ring slot ``slot``; returns None, or (HTTP status, message) for a bad payload."""
    from .decode import PayloadError, decode_image

    try:
        _RING[slot] = decode_image(body, content_type, _RING.shape[1:])
    except PayloadError as e:
        return e.status, str(e)
    return None


def _ping() -> int:
    return 0


class DecodePool:
    def __init__(self, processes: int, shm_name: str, nslots: int, item_shape: Sequence[int]):
        self.processes = int(processes)
        self.ex = ProcessPoolExecutor(self.processes, mp_context=mp.get_context("spawn"), initializer=_init,
                                      initargs=(shm_name, int(nslots), tuple(int(x) for x in item_shape)))
        # start every process now (the executor spawns one per submit while none is idle), not under load
        for f in [self.ex.submit(_ping) for _ in range(self.processes)]:
            f.result()

    def decode_into(self, slot: int, body: bytes, content_type: str) -> None:
        """Blocking (call from an executor thread); raises PayloadError for undecodable bodies."""
        from .decode import PayloadError

        err = self.ex.submit(_decode_into, int(slot), body, content_type).result()
        if err is not None:
            raise PayloadError(err[1], err[0])

    def close(self) -> None:
        self.ex.shutdown(wait=True, cancel_futures=True)
