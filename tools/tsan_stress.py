"""Threaded stress of the native core, meant to run under ThreadSanitizer (tools/tsan_check.sh)."""
import os
import sys
import threading
import time

sys.path.insert(0, sys.argv[1])  # dir holding the TSAN-built _ai4e_core
import _ai4e_core as c  # noqa: E402

s = c.TaskStore()
q = c.DispatchQueue("q", 3, 0.05, 0)
N, P = 400, 4
done = []


def producer():
    for _ in range(N // 40):
        ids = s.create_many("http://h/v1/x", 40)
        q.send_many(ids, [])
        s.incrby("CURRENT_REQUESTS/c/v1/x", 1)


stop = threading.Event()


def consumer():
    got = 0
    while not stop.is_set():
        ms = q.receive(32, 0.05, 0.0005)
        if not ms:
            continue
        ids = [m.task_id for m in ms]
        s.transition_many(ids, "running", "r")
        if got % 3 == 0 and ms:
            q.abandon(ms[0].seq, 0.0)
            ms = ms[1:]
            ids = ids[1:]
        s.transition_many(ids, "completed", "ok")
        q.complete([m.seq for m in ms])
        got += len(ms)
        s.zcard("/v1/x_completed")
        s.get(ids[0]) if ids else None
    done.append(got)


prods = [threading.Thread(target=producer) for _ in range(P)]
cons = [threading.Thread(target=consumer) for _ in range(2)]
[t.start() for t in prods + cons]
[t.join(120) for t in prods]
deadline = time.time() + 60
while time.time() < deadline:
    st = q.stats()
    if st["ready"] == 0 and st["scheduled"] == 0 and st["inflight"] == 0:
        break
    time.sleep(0.05)
stop.set()
[t.join(30) for t in cons]

# ---- node scheduler: dispatcher + reader threads against fake workers on socketpairs (threads here)
import socket  # noqa: E402
import struct  # noqa: E402

sched_store = c.TaskStore("", 4)
sq = c.DispatchQueue("sq", 5, 30.0, 0)
ring = c.SlotRing(64, 0)
sched = c.NodeScheduler(sched_store, sq, "http://h/v1/s", 64, max_batch=8, linger_s=0.0005, depth=2,
                        hb_timeout_s=30.0, poll_s=0.002)
sched.add_local_ring(ring)


def fake_worker(sock, rank):
    f = sock.makefile("rwb", buffering=0)

    def send(payload):
        f.write(struct.pack("!i", len(payload)) + payload)

    send(struct.pack("<Iii", 1, rank, 0) + b"{}")
    while True:
        hdr = f.read(4)
        if len(hdr) < 4:
            return
        (n,) = struct.unpack("!i", hdr)
        buf = f.read(n)
        t = struct.unpack_from("<I", buf)[0]
        if t == 5:
            return
        if t == 4:
            _, bid, k, _ = struct.unpack_from("<IQII", buf)
            pad = (k + 7) // 8 * 8
            send(struct.pack("<IQII5d", 3, bid, k, 4, 0, 0, 0, 0, 0) + bytes(pad) + bytes(4 * k))


threads = []
for r in range(3):
    a, b = socket.socketpair()
    t = threading.Thread(target=fake_worker, args=(b, r), daemon=True)
    t.start()
    threads.append((t, b))
    sched.attach(r, os.dup(a.fileno()), True)
    a.close()
total = 0
for _ in range(40):
    slots = ring.alloc(8, 5.0)
    sched.submit(slots, "")
    total += 8
deadline = time.time() + 60
while time.time() < deadline and sched.images_done() < total:
    time.sleep(0.01)
sched.worker_stats()
sched.detach(0, 5.0)
sched.stop()
assert sched.images_done() == total, (sched.images_done(), total)
print("tsan stress ok", sum(done), s.size(), q.stats(), "scheduler", sched.images_done())
