"""The ctypes signatures in ops/_ext.py must match the C ABI of csrc/kernels/*.hip (CPU check)."""
import pytest
import re
from pathlib import Path

from aiforearth_api_platform_amd.ops import _ext

ROOT = Path(__file__).resolve().parent.parent


def _c_signatures():
    sigs = {}
    for f in (ROOT / "csrc" / "kernels").glob("*.hip"):
        src = f.read_text()
        for m in re.finditer(r"AI4E_API\s+int\s+(\w+)\s*\(([^)]*)\)", src):
            args = [a.strip() for a in m.group(2).split(",") if a.strip()]
            sigs[m.group(1)] = args
    return sigs


def _kind(c_arg: str):
    c_arg = re.sub(r"\s+\w+$", "", c_arg.strip())  # drop the parameter name
    if "*" in c_arg or "hipStream_t" in c_arg:
        return "p"
    if "float" in c_arg:
        return "f"
    if "long" in c_arg:
        return "l"
    return "i"


def test_every_launcher_signature_matches():
    import ctypes
    csigs = _c_signatures()
    assert csigs, "no AI4E_API launchers found"
    pykind = {ctypes.c_void_p: "p", ctypes.c_int: "i", ctypes.c_long: "l", ctypes.c_float: "f"}
    for name, c_args in csigs.items():
        if not c_args:
            continue
        assert name in _ext._SIGS, f"{name} missing from _ext._SIGS"
        py = [pykind[t] for t in _ext._SIGS[name]]
        c = [_kind(a) for a in c_args]
        assert py == c, f"{name}: python {py} != C {c}"


def test_gn_chunk_px_exported():
    """ops/norm.py sizes the GroupNorm workspace from the library's statistics chunk (ai4e_gn_chunk_px)."""
    from aiforearth_api_platform_amd.ops import _ext, norm
    if not _ext.available():
        pytest.skip("kernel library not built")
    assert _ext.has("ai4e_gn_chunk_px")
    assert norm._gn_chunk_px() == _ext.call_int("ai4e_gn_chunk_px") > 0
