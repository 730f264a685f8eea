"""In-tree native build: the C++ control-plane core and the gfx950 HIP kernel library.

Both artefacts land inside the package directory so they travel with the repo snapshot to
the GPU box (see README "Build"):

* ``_ai4e_core<EXT_SUFFIX>`` — pybind11 module (task store + dispatch queue), g++ -O3.
* ``_lib/libai4e_kernels.so`` — hand-written CDNA4 kernels (``csrc/kernels/*.hip``) built
  with ``hipcc --offload-arch=gfx950`` and exposed through a plain C ABI consumed via ctypes
  (no torch headers in the kernel TU => seconds per file, no JIT cache under ~/.cache).
* ``_lib/ai4e_ingestd`` / ``_lib/ai4e_http_load`` — the native ingest front-end and the REST load
  generator (``csrc/ingest/*.cpp``), g++ -O2.

Rebuilds are decided by CONTENT: every artefact has a ``<artefact>.sha`` manifest next to it holding the sha256 of
its sources, headers, compiler and flags; an artefact whose manifest does not match what the tree would build now is
rebuilt, whatever the file times say (a snapshot pushed to a GPU box never runs a stale library, and a fresh checkout
with a matching manifest never rebuilds).  ``python -m aiforearth_api_platform_amd._build``.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = ROOT / "csrc"
LIBDIR = PKG / "_lib"
OBJDIR = ROOT / "build" / "obj"
ARCH = os.environ.get("AI4E_OFFLOAD_ARCH", "gfx950")

CORE_SO = PKG / ("_ai4e_core" + sysconfig.get_config_var("EXT_SUFFIX"))
KERNEL_SO = LIBDIR / "libai4e_kernels.so"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the gfx950 kernels)")


def _digest(deps, cmd) -> str:
    h = hashlib.sha256()
    for part in cmd:
        h.update(str(part).encode() + b"\0")
    for d in sorted(map(str, deps)):
        h.update(d.rsplit("/", 1)[-1].encode() + b"\0")
        h.update(Path(d).read_bytes())
    return h.hexdigest()


def _manifest(out: Path) -> Path:
    return out.with_name(out.name + ".sha")


def _stale(out: Path, deps, cmd=()) -> bool:
    """True unless ``out`` exists and its manifest holds the digest of ``deps`` + ``cmd`` (content, not mtime)."""
    if not out.exists():
        return True
    m = _manifest(out)
    return not m.exists() or m.read_text().strip() != _digest(deps, cmd)


def _stamp(out: Path, deps, cmd=()) -> None:
    _manifest(out).write_text(_digest(deps, cmd) + "\n")


def _run(cmd, verbose):
    if verbose:
        print(" ".join(map(str, cmd)), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def build_core(verbose: bool = False, force: bool = False) -> Path:
    src = sorted((CSRC / "core").glob("*.cpp"))
    headers = sorted((CSRC / "core").glob("*.h"))
    cxx = os.environ.get("CXX", "g++")
    extra = os.environ.get("AI4E_CORE_CXXFLAGS", "")  # e.g. "-fsanitize=thread -g" for the TSAN build
    key = [cxx, "-O3", "-std=c++17", extra]
    if not force and not _stale(CORE_SO, [*src, *headers], key):
        return CORE_SO
    import pybind11

    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall",
           f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}",
           *map(str, src), "-o", str(CORE_SO), "-lpthread"]
    if extra:
        cmd[1:1] = extra.split()
    _run(cmd, verbose)
    _stamp(CORE_SO, [*src, *headers], key)
    return CORE_SO


def _kernel_sources():
    return sorted((CSRC / "kernels").glob("*.hip"))


def build_kernels(verbose: bool = False, force: bool = False, jobs: int = 8, defines=(), variant: str = "") -> Path:
    """``defines`` + ``variant``: an A/B build of the library (``_lib/libai4e_kernels_<variant>.so``, objects in
    their own directory), loaded with AI4E_KERNEL_LIB=<path> (ops/_ext.py)."""
    srcs = _kernel_sources()
    # + the layout / span-decoder headers the JPEG kernels share with the CPU preparer
    headers = sorted((CSRC / "kernels").glob("*.h")) + [CSRC / "core" / "jpeg_layout.h", CSRC / "core" / "jpeg_span.h"]
    objdir = OBJDIR if not variant else OBJDIR.parent / f"obj_{variant}"
    out_so = KERNEL_SO if not variant else LIBDIR / f"libai4e_kernels_{variant}.so"
    LIBDIR.mkdir(parents=True, exist_ok=True)
    objdir.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    # -amdgpu-mfma-vgpr-form: MFMA accumulators in arch VGPRs (gfx950 has one unified 512-entry
    # file per SIMD); with AGPR accumulators hipcc shuttled them AGPR<->VGPR inside the K1 loop.
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-Wno-unused-result", f"-I{CSRC / 'kernels'}",
             *[f"-D{d}" for d in defines]]

    key = [hipcc, *flags]
    if not force and not _stale(out_so, [*srcs, *headers], key):
        return out_so  # the library matches the tree: no object is needed

    def one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        if force or _stale(obj, [src, *headers], key):
            _run([hipcc, *flags, "-c", str(src), "-o", str(obj)], verbose)
            _stamp(obj, [src, *headers], key)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs) or 1))) as ex:
        objs = list(ex.map(one, srcs))
    _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(out_so)], verbose)
    _stamp(out_so, [*srcs, *headers], key)
    return out_so


INGESTD = LIBDIR / "ai4e_ingestd"
HTTP_LOAD = LIBDIR / "ai4e_http_load"


def build_tools(verbose: bool = False, force: bool = False) -> None:
    """The native executables of the ingest path (``csrc/ingest``)."""
    LIBDIR.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    headers = sorted((CSRC / "core").glob("*.h"))
    for src, out in ((CSRC / "ingest" / "ingestd.cpp", INGESTD), (CSRC / "ingest" / "http_load.cpp", HTTP_LOAD)):
        key = [cxx, "-O2"]
        if force or _stale(out, [src, *headers], key):
            # OpenSSL (TLS termination in ai4e_ingestd, HTTPS load generation in ai4e_http_load)
            _run([cxx, "-O2", "-std=c++17", "-Wall", "-pthread", str(src), "-o", str(out), "-lrt", "-lssl", "-lcrypto"],
                 verbose)
            _stamp(out, [src, *headers], key)


def build_all(verbose: bool = False, force: bool = False) -> None:
    build_core(verbose=verbose, force=force)
    build_kernels(verbose=verbose, force=force)
    build_tools(verbose=verbose, force=force)


if __name__ == "__main__":
    build_all(verbose=True, force="--force" in sys.argv)
    print("built:", CORE_SO, KERNEL_SO, INGESTD, HTTP_LOAD)
