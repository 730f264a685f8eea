"""Race detection: the native core under ThreadSanitizer (survey §5.2). CPU-only, ~30 s."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with -fsanitize=thread")
def test_native_core_is_tsan_clean(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "tsan_check.sh")], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "tsan stress ok" in r.stdout


@pytest.mark.slow
@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with -fsanitize=thread")
@pytest.mark.parametrize("san", ["thread", "address"])
def test_native_ingest_frontend_sanitizers(tmp_path, san):
    """ai4e_ingestd built with -fsanitize=thread / address behind the CPU platform: concurrent keep-alive
    batch + single-image ingest from the C++ load generator, proxied task queries and fresh-connection admission
    errors; the sanitizer must report nothing."""
    import sys
    import time

    import numpy as np
    import requests
    import yaml

    from aiforearth_api_platform_amd.runtime.http_load import run_native_clients

    binary = str(tmp_path / f"ingestd_{san}")
    r = subprocess.run(["g++", "-O1", "-g", f"-fsanitize={san}", "-std=c++17", "-pthread",
                        os.path.join(ROOT, "csrc", "ingest", "ingestd.cpp"), "-o", binary, "-lrt"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    doc = yaml.safe_load(open(os.path.join(ROOT, "examples", "platform_cpu.yaml")))
    doc["endpoints"]["tiny"]["max_batch"] = 64
    cfgp = tmp_path / "platform.yaml"
    cfgp.write_text(yaml.safe_dump(doc))
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    log = tmp_path / "serve.log"
    env = dict(os.environ, PYTHONPATH=ROOT, AI4E_FRONTEND_PROCESSES="2", AI4E_FRONTEND_IMPL="native",
               AI4E_INGESTD=binary, TSAN_OPTIONS="report_signal_unsafe=0", ASAN_OPTIONS="detect_leaks=0")
    proc = subprocess.Popen([sys.executable, "-m", "aiforearth_api_platform_amd.serve", "--config", str(cfgp),
                             "--port", str(port)], cwd=ROOT, env=env, stdout=open(log, "w"), stderr=subprocess.STDOUT)
    base = f"http://127.0.0.1:{port}"
    try:
        for _ in range(600):
            try:
                if requests.get(base + "/", timeout=1).status_code == 200:
                    break
            except requests.ConnectionError:
                time.sleep(0.1)
        time.sleep(1.5)
        img = np.zeros((4, 4, 3), np.uint8)
        url = base + "/v1/tiny/async"
        a = run_native_clients(url, 1.5, 6, np.repeat(img[None], 16, 0).tobytes(), "application/x-ai4e-batch", procs=2)
        b = run_native_clients(url, 1.5, 8, img.tobytes(), "application/octet-stream", procs=2)
        assert a["errors"] == 0 and b["errors"] == 0 and a["ids"] and b["ids"]
        for _ in range(20):  # fresh connections: proxied queries and admission errors through any listener
            assert requests.get(f"{base}/v1/taskmanagement/task/{b['ids'][0]}",
                                headers={"Connection": "close"}).status_code == 200
            assert requests.post(url, data=b"\x00" * 50, headers={"Content-Type": "application/x-ai4e-batch",
                                                                  "Connection": "close"}).status_code == 400
    finally:
        proc.terminate()
        try:
            proc.wait(20)
        except subprocess.TimeoutExpired:
            proc.kill()
    out = log.read_text()
    assert "ai4e_ingestd pid" in out
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]
