"""Launcher of the native ingest front-ends (``csrc/ingest/ingestd.cpp``, built to ``_lib/ai4e_ingestd``).

Same role and same admission rules as the Python front-ends of :mod:`runtime.frontend` — a process on the
public port beside the serving process (SO_REUSEPORT), its own partition of every pool endpoint's payload
ring, SUBMIT_IDS / SUBMITTED / FREE with the node scheduler over its own ingest connection — but written in
C++: a binary batch or a raw single payload is ``recv()``'d straight into ring slots (one kernel->ring copy,
no interpreter on the path), one thread per client connection. Requests it does not ingest itself (encoded
images, task API, sync routes, upstream ``taskId`` requests, chunked bodies) are proxied to the serving
process. With a certificate configured (``security["tls_cert"]`` / ``["tls_key"]``) every client connection is a
TLS session terminated in the native process (OpenSSL); the body is decrypted straight into the ring slots.

The scheduler connection is the socket end of a ``multiprocessing.Pipe`` (a socketpair) inherited by the
child; the config is a small line-oriented file (``ingestd.cpp`` ``parse_config``).
"""
from __future__ import annotations

import os
import subprocess
import tempfile
import time
from typing import Dict, List, Optional

from .. import _build


class NativeFrontend:
    """Handle of one ``ai4e_ingestd`` process (``terminate`` / ``join`` / ``is_alive`` like a Process)."""

    def __init__(self, proc: subprocess.Popen, cfg_path: str):
        self.proc, self.cfg_path = proc, cfg_path
        self.pid = proc.pid

    def terminate(self) -> None:
        if self.proc.poll() is None:
            self.proc.terminate()

    def kill(self) -> None:
        if self.proc.poll() is None:
            self.proc.kill()

    def join(self, timeout: Optional[float] = None) -> None:
        try:
            self.proc.wait(timeout)
        except subprocess.TimeoutExpired:
            pass
        if self.proc.poll() is not None and os.path.exists(self.cfg_path):
            os.unlink(self.cfg_path)

    def is_alive(self) -> bool:
        return self.proc.poll() is None

    @property
    def exitcode(self) -> Optional[int]:
        return self.proc.poll()


def available() -> bool:
    try:
        _build.build_tools()
    except Exception:
        return False
    return _build.INGESTD.exists()


def _token(v) -> str:
    s = str(v)
    if not s or any(c.isspace() for c in s):
        raise ValueError(f"native front-end config value must be a non-empty token without spaces: {s!r}")
    return s


def spawn_native_frontends(n: int, pools: Dict[str, object], routes: List[dict], host: str, port: int,
                           internal_url: str, security: Optional[dict] = None,
                           ack_timeout_s: float = 30.0, max_queue_ms: float = 0.0,
                           wait_ready_s: float = 30.0) -> List[NativeFrontend]:
    """Start ``n`` native front-ends; arguments as :func:`runtime.frontend.spawn_frontends`.

    Each front-end attaches to every control-plane shard of every pool endpoint (one ``shard`` line per shard: its
    ring partition, scheduler connection and the task-store digits its ids end in); a route lists its endpoint's
    shards and the front-end picks the least-loaded one per request. ``max_queue_ms`` > 0: latency-budgeted
    admission (429 + Retry-After once a request's projected queue wait exceeds the budget). Returns once every
    front-end listens on the public port (each writes one byte to a ready pipe after ``listen``), so the caller
    can hand the port over (:func:`handover_public_port`)."""
    import multiprocessing as mp

    if not n or not pools:
        return []
    sec = security or {}
    if bool(sec.get("tls_cert")) != bool(sec.get("tls_key")):
        raise ValueError("TLS needs both a certificate (AI4E_TLS_CERT) and a private key (AI4E_TLS_KEY)")
    _build.build_tools()
    ihost, iport = internal_url.split("://", 1)[1].rsplit(":", 1)
    names = list(pools)
    procs, readies = [], []
    for i in range(n):
        lines = [f"listen {_token(host)} {int(port)}", f"internal {_token(ihost)} {int(iport)}",
                 f"ack_timeout {float(ack_timeout_s)}", f"frontend_index {i}"]
        if max_queue_ms and max_queue_ms > 0:
            lines.append(f"max_queue_ms {float(max_queue_ms)}")
        lines += [f"key {_token(k)}" for k in sec.get("keys") or []]
        if sec.get("tls_cert"):
            lines.append(f"tls {_token(os.path.abspath(sec['tls_cert']))} {_token(os.path.abspath(sec['tls_key']))}")
        ready_r, ready_w = os.pipe()
        lines.append(f"ready {ready_w}")
        child_ends, fds = [], [ready_w]
        shard_lines: Dict[str, List[int]] = {}  # endpoint name -> its shard line indices
        for name in names:
            ep = pools[name]
            for pool in getattr(ep.worker, "control_shards", [ep.worker]):
                base, length, rank = pool.frontend_partitions[i]
                parent, child = mp.Pipe(duplex=True)
                pool.attach_ingest(rank, parent)
                child_ends.append(child)
                fds.append(child.fileno())
                item = 1
                for v in ep.item_shape:
                    item *= int(v)
                shape = "(" + ",".join(str(int(v)) for v in ep.item_shape) + ")"
                si = sum(len(v) for v in shard_lines.values())
                shard_lines.setdefault(name, []).append(si)
                digits = pool.mint_digits() if hasattr(pool, "mint_digits") else "-"
                stat = getattr(pool, "stat_name", "") or "-"  # the shard's load counters (admission)
                mb = int(getattr(getattr(pool, "spec", None), "max_batch", 0) or 0)  # (admission: full-batch capacity)
                lines.append(f"shard {si} {child.fileno()} {_token(ep.ring.name)} {int(ep.ring.nslots)} {item} "
                             f"{int(base)} {int(length)} {_token(ep.endpoint)} {shape} {_token(digits)} {_token(stat)} "
                             f"{mb}")
        for r in routes:
            si = ",".join(map(str, shard_lines[r["endpoint"]])) if r.get("endpoint") in pools else "-1"
            types = ",".join(_token(t) for t in r.get("content_types") or []) or "-"
            keys = ",".join(_token(k) for k in r.get("keys") or []) or "-"
            mc = r.get("max_concurrent")
            lines.append(f"route {_token(r['prefix'])} {_token(r.get('mode', 'async'))} {si} "
                         f"{int(r.get('max_content_length') or 0)} {-1 if mc is None else int(mc)} {types} {keys}")
        fd, cfg_path = tempfile.mkstemp(prefix="ai4e_ingestd_", suffix=".conf")
        with os.fdopen(fd, "w") as f:
            f.write("\n".join(lines) + "\n")
        os.chmod(cfg_path, 0o600)  # (subscription keys)
        binary = os.environ.get("AI4E_INGESTD") or str(_build.INGESTD)  # (a sanitizer build in the race tests)
        p = subprocess.Popen([binary, cfg_path], pass_fds=fds, close_fds=True)
        for c in child_ends:
            c.close()
        os.close(ready_w)
        procs.append(NativeFrontend(p, cfg_path))
        readies.append(ready_r)
    import select

    deadline = time.time() + wait_ready_s
    for fd in readies:
        try:
            r, _, _ = select.select([fd], [], [], max(0.0, deadline - time.time()))
            if not r or not os.read(fd, 1):
                raise RuntimeError("a native ingest front-end did not start listening")
        finally:
            os.close(fd)
    return procs


def handover_public_port(socks: list, frontends: list) -> list:
    """With native front-ends listening (they run the latency-budgeted admission), the serving process stops
    accepting on the shared public port: a connection a 429 closed reconnects to a front-end, never drifting onto a
    path without admission. Returns the sockets the gateway keeps serving (the internal one)."""
    if frontends and len(socks) > 1 and all(isinstance(p, NativeFrontend) for p in frontends):
        socks[0].close()
        return socks[1:]
    return socks
