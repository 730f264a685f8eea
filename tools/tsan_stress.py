"""Threaded stress of the native core, meant to run under ThreadSanitizer (tools/tsan_check.sh)."""
import sys
import threading

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
import time  # noqa: E402
deadline = time.time() + 60
while time.time() < deadline:
    st = q.stats()
    if st["ready"] == 0 and st["scheduled"] == 0 and st["inflight"] == 0:
        break
    time.sleep(0.05)
stop.set()
[t.join(30) for t in cons]
print("tsan stress ok", sum(done), s.size(), q.stats())
