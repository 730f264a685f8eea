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
