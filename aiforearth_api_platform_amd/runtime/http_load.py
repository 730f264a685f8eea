"""HTTP load generator processes for the REST benchmarks (no torch import).

The clients run in their own spawned processes so the server under test does not share an
interpreter (and a GIL) with its load: ``run_clients`` starts ``procs`` processes, each driving
``conc`` keep-alive connections for ``seconds``, and returns every TaskId the server handed out
plus the wall-clock window the requests covered.
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
