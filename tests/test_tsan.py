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
@pytest.mark.parametrize("san,tls", [("thread", False), ("address", False), ("thread", True), ("address", True)])
def test_native_ingest_frontend_sanitizers(tmp_path, san, tls):
    """ai4e_ingestd built with -fsanitize=thread / address behind the CPU platform: concurrent keep-alive
    batch + single-image ingest from the C++ load generator, proxied task queries, fresh-connection admission
    errors and an oversized Content-Length (413); plain HTTP and TLS (OpenSSL sessions in the connection threads);
    the sanitizer must report nothing."""
    import sys
    import time

    import numpy as np
    import requests
    import yaml

    from aiforearth_api_platform_amd.runtime.http_load import run_native_clients

    binary = str(tmp_path / f"ingestd_{san}")
    r = subprocess.run(["g++", "-O1", "-g", f"-fsanitize={san}", "-std=c++17", "-pthread",
                        os.path.join(ROOT, "csrc", "ingest", "ingestd.cpp"), "-o", binary, "-lrt", "-lssl", "-lcrypto"],
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
    if tls:
        fx = os.path.join(ROOT, "tests", "fixtures")
        env.update(AI4E_TLS_CERT=os.path.join(fx, "tls_test_cert.pem"), AI4E_TLS_KEY=os.path.join(fx, "tls_test_key.pem"))
    proc = subprocess.Popen([sys.executable, "-m", "aiforearth_api_platform_amd.serve", "--config", str(cfgp),
                             "--port", str(port)], cwd=ROOT, env=env, stdout=open(log, "w"), stderr=subprocess.STDOUT)
    base = f"{'https' if tls else 'http'}://127.0.0.1:{port}"
    import ssl
    import urllib3

    urllib3.disable_warnings()
    ctx = ssl.create_default_context()
    ctx.check_hostname, ctx.verify_mode = False, ssl.CERT_NONE

    def oversized() -> bytes:
        raw = socket.create_connection(("127.0.0.1", port), timeout=10)
        c = ctx.wrap_socket(raw) if tls else raw
        with c:
            c.sendall(b"POST /v1/tiny/async HTTP/1.1\r\nHost: x\r\nContent-Type: application/octet-stream\r\n"
                      b"Content-Length: 999999999999\r\n\r\n")
            return c.recv(256)
    try:
        for _ in range(600):
            try:
                if requests.get(base + "/", timeout=1, verify=False).status_code == 200:
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
            assert requests.get(f"{base}/v1/taskmanagement/task/{b['ids'][0]}", verify=False,
                                headers={"Connection": "close"}).status_code == 200
            assert requests.post(url, data=b"\x00" * 50, verify=False,
                                 headers={"Content-Type": "application/x-ai4e-batch",
                                          "Connection": "close"}).status_code == 400
            assert b" 413 " in oversized()
    finally:
        proc.terminate()
        try:
            proc.wait(20)
        except subprocess.TimeoutExpired:
            proc.kill()
    out = log.read_text()
    assert "ai4e_ingestd pid" in out
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]
