"""HTTP load generator processes for the REST benchmarks (no torch import).

The clients run in their own processes so the server under test does not share an interpreter (and a GIL)
with its load. ``run_native_clients`` (the default of the benchmarks) starts ``procs`` processes of the C++
generator ``_lib/ai4e_http_load`` (csrc/ingest/http_load.cpp: one thread per keep-alive connection, one
writev per request), which report their own CPU time; ``run_clients`` is the aiohttp form. Both return every
TaskId the server handed out plus the wall-clock window the requests covered.
"""
from __future__ import annotations

import multiprocessing as mp
import time
from typing import List, Tuple


def _client(url: str, seconds: float, conc: int, body: bytes, content_type: str, batch: bool, start_at: float,
            out) -> None:
    import asyncio

    import aiohttp

    async def main():
        ids: List[str] = []
        errors = 0
        while time.time() < start_at:
            await asyncio.sleep(0.001)
        t_end = time.perf_counter() + seconds
        conn = aiohttp.TCPConnector(limit=conc)
        async with aiohttp.ClientSession(connector=conn) as s:
            async def one():
                nonlocal errors
                while time.perf_counter() < t_end:
                    async with s.post(url, data=body, headers={"Content-Type": content_type}) as r:
                        if r.status != 200:
                            errors += 1
                            await r.read()
                            continue
                        js = await r.json()
                        if batch:
                            ids.extend(js["TaskIds"])
                        else:
                            ids.append(js["TaskId"])

            t0 = time.time()
            await asyncio.gather(*(one() for _ in range(conc)))
            t1 = time.time()
        return ids, t0, t1, errors

    try:
        out.send(asyncio.run(main()))
    except Exception as e:  # reported to the parent, which raises
        out.send(repr(e))
    finally:
        out.close()


def run_clients(url: str, seconds: float, conc: int, body: bytes, content_type: str, batch: bool,
                procs: int = 2) -> Tuple[List[str], float, float, int]:
    ctx = mp.get_context("spawn")
    start_at = time.time() + 3.0  # all clients start together once their interpreters are up
    pipes, ps = [], []
    for _ in range(procs):
        r, w = ctx.Pipe(duplex=False)
        p = ctx.Process(target=_client, args=(url, seconds, conc, body, content_type, batch, start_at, w), daemon=True)
        p.start()
        w.close()
        pipes.append(r)
        ps.append(p)
    ids: List[str] = []
    t0, t1, errors = float("inf"), 0.0, 0
    for r in pipes:
        res = r.recv()
        if isinstance(res, str):
            raise RuntimeError(f"HTTP load client failed: {res}")
        i, a, b, e = res
        ids.extend(i)
        t0, t1, errors = min(t0, a), max(t1, b), errors + e
    for p in ps:
        p.join(30)
    return ids, t0, t1, errors


def run_native_clients(url: str, seconds: float, conc: int, body: bytes, content_type: str, procs: int = 2,
                       headers=()) -> dict:
    """``procs`` C++ load processes x ``conc`` connections each. Returns {ids, t0, t1, errors, busy, requests,
    bytes_sent, client_cpu_s (user + system, all client processes), client_processes, connections}."""
    import json
    import os
    import subprocess
    import tempfile
    from urllib.parse import urlparse

    from .. import _build

    _build.build_tools()
    u = urlparse(url)
    tmp = tempfile.mkdtemp(prefix="ai4e_load_")
    body_path = os.path.join(tmp, "body.bin")
    with open(body_path, "wb") as f:
        f.write(body)
    start_at = time.time() + 1.0
    ps = []
    for i in range(procs):
        host = ("tls:" if u.scheme == "https" else "") + u.hostname  # (https: TLS sessions, no cert verification)
        cmd = [str(_build.HTTP_LOAD), host, str(u.port), u.path + (("?" + u.query) if u.query else ""),
               content_type, body_path, str(conc), str(seconds), f"{start_at:.6f}", os.path.join(tmp, f"ids{i}.txt"),
               *headers]
        ps.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    out = {"ids": [], "t0": float("inf"), "t1": 0.0, "errors": 0, "busy": 0, "requests": 0, "bytes_sent": 0.0,
           "client_cpu_s": 0.0, "client_processes": procs, "connections": procs * conc}
    for i, p in enumerate(ps):
        try:
            so, se = p.communicate(timeout=seconds + 90)
        except subprocess.TimeoutExpired:
            for q in ps:
                q.kill()
            raise
        if p.returncode != 0:
            raise RuntimeError(f"ai4e_http_load failed ({p.returncode}): {se[-500:]}")
        st = json.loads(so.strip().splitlines()[-1])
        out["t0"], out["t1"] = min(out["t0"], st["t0"]), max(out["t1"], st["t1"])
        out["errors"] += st["errors"]
        out["busy"] += st.get("busy", 0)  # 429 answers of the latency-budgeted admission (retried by the client)
        out["requests"] += st["requests"]
        out["bytes_sent"] += st["bytes_sent"]
        out["client_cpu_s"] += st["cpu_user_s"] + st["cpu_sys_s"]
        with open(os.path.join(tmp, f"ids{i}.txt")) as f:
            out["ids"] += [l.strip() for l in f if l.strip()]
        lp = os.path.join(tmp, f"ids{i}.txt.lat")
        if os.path.exists(lp):
            with open(lp) as f:
                out.setdefault("request_latency_ms", []).extend(float(l) for l in f if l.strip())
    for name in os.listdir(tmp):
        os.unlink(os.path.join(tmp, name))
    os.rmdir(tmp)
    return out
