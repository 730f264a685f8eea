"""Python side of the scheduler <-> GPU worker wire protocol (``csrc/core/scheduler.h``).

Frames travel over a ``multiprocessing.connection.Connection`` (a socketpair for spawned workers,
TCP for ``torchrun`` ranks), so framing is Connection's own 4-byte length prefix and the native
scheduler reads/writes the same bytes on the raw fd. Payload = u32 type + little-endian fields.
"""
from __future__ import annotations

import json
import struct
import threading
from typing import List, Sequence, Tuple

import numpy as np

F_READY, F_HB, F_DONE, F_BATCH, F_STOP, F_SUBMIT, F_FREE, F_STAGE, F_SUBMIT_IDS, F_SUBMITTED = range(1, 11)
IT_OK, IT_INVALID, IT_ERROR, IT_RETRY = 0, 1, 2, 3

_U32 = struct.Struct("<I")
_READY = struct.Struct("<Iii")
_HB = struct.Struct("<IdQQdQQQdd")
_DONE_HDR = struct.Struct("<IQII5d")
_BATCH_HDR = struct.Struct("<IQII")
_SLOTS_HDR = struct.Struct("<III")
_STAGE = struct.Struct("<IQII")
_SUBMIT_IDS_HDR = struct.Struct("<IIIIIQ")
_SUBMITTED = struct.Struct("<IQII")


class FrameConn:
    """Thread-safe sender + single-reader receiver over a Connection."""

    def __init__(self, conn):
        self.conn = conn
        self._mu = threading.Lock()

    def send(self, payload) -> None:
        with self._mu:
            self.conn.send_bytes(payload)

    def recv(self) -> bytes:
        return self.conn.recv_bytes()

    def poll(self, timeout: float) -> bool:
        return self.conn.poll(timeout)

    def close(self) -> None:
        try:
            self.conn.close()
        except OSError:
            pass

    # ---------------------------------------------------------------- worker -> scheduler
    def ready(self, rank: int, pinned: bool, info: dict) -> None:
        self.send(_READY.pack(F_READY, rank, int(pinned)) + json.dumps(info).encode())

    def heartbeat(self, t: float, hbm_used: int, hbm_total: int, busy_ms: float, batches: int, xgmi_tx: int = 0,
                  xgmi_rx: int = 0, gfx_mhz: float = 0.0, power_w: float = 0.0) -> None:
        self.send(_HB.pack(F_HB, t, hbm_used, hbm_total, busy_ms, batches, xgmi_tx, xgmi_rx, gfx_mhz, power_w))

    def done(self, bid: int, status: np.ndarray, rows: bytes, row_bytes: int, stage: Sequence[float]) -> None:
        n = int(status.shape[0])
        pad = (n + 7) // 8 * 8
        st = np.zeros(pad, np.uint8)
        st[:n] = status
        self.send(b"".join((_DONE_HDR.pack(F_DONE, bid, n, row_bytes, *stage), st.tobytes(), rows)))

    def submit(self, slots: Sequence[int]) -> None:
        a = np.asarray(slots, dtype=np.int64)
        self.send(_SLOTS_HDR.pack(F_SUBMIT, a.shape[0], 0) + a.tobytes())

    def stage(self, bid: int, stage: int) -> None:
        self.send(_STAGE.pack(F_STAGE, bid, stage, 0))

    def submit_ids(self, slots: Sequence[int], ids: Sequence[str], trace: str = "", token: int = 0,
                   ack: bool = True) -> None:
        """Ingest front-end: enqueue payloads under task ids minted here (all ids the same length)."""
        a = np.asarray(slots, dtype=np.int64)
        enc = [i.encode("ascii") for i in ids]  # ids are validated ASCII (frontend.valid_task_id)
        il = len(enc[0]) if enc else 0
        if any(len(e) != il for e in enc):
            raise ValueError("submit_ids: all task ids must have the same byte length")
        tb = trace.encode()
        self.send(b"".join((_SUBMIT_IDS_HDR.pack(F_SUBMIT_IDS, a.shape[0], len(tb), il, int(ack), token),
                            a.tobytes(), b"".join(enc), tb)))


def frame_type(buf: bytes) -> int:
    return _U32.unpack_from(buf, 0)[0]


def parse_batch(buf: bytes) -> Tuple[int, np.ndarray]:
    _, bid, n, _ = _BATCH_HDR.unpack_from(buf, 0)
    return bid, np.frombuffer(buf, dtype=np.int64, count=n, offset=_BATCH_HDR.size)


def parse_slots(buf: bytes) -> np.ndarray:
    _, n, _ = _SLOTS_HDR.unpack_from(buf, 0)
    return np.frombuffer(buf, dtype=np.int64, count=n, offset=_SLOTS_HDR.size)


def parse_submitted(buf: bytes) -> Tuple[int, int]:
    """SUBMITTED -> (token, tasks created)."""
    _, token, n, _ = _SUBMITTED.unpack_from(buf, 0)
    return token, n


def parse_ready_info(buf: bytes) -> dict:
    return json.loads(buf[_READY.size:].decode() or "{}")


def batch_frame(bid: int, slots: Sequence[int]) -> bytes:
    """Scheduler-side BATCH frame (used by the pure-Python tests of the worker loop)."""
    a = np.asarray(slots, dtype=np.int64)
    return _BATCH_HDR.pack(F_BATCH, bid, a.shape[0], 0) + a.tobytes()


def parse_done(buf: bytes) -> Tuple[int, np.ndarray, bytes, int, List[float]]:
    _, bid, n, row_bytes, *stage = _DONE_HDR.unpack_from(buf, 0)
    pad = (n + 7) // 8 * 8
    off = _DONE_HDR.size
    status = np.frombuffer(buf, np.uint8, count=n, offset=off)
    return bid, status, buf[off + pad: off + pad + n * row_bytes], row_bytes, list(stage)
