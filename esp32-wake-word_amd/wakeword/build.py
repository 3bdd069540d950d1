"""Build libwakeword.so (all HIP kernels + the C ABI) for gfx950, in-tree.

    python -m wakeword.build          (from esp32-wake-word_amd/)

hipcc cross-compiles for gfx950 without a GPU.  Objects are compiled in
parallel and linked into ``wakeword/libwakeword.so`` next to this file, so
the library travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                       # esp32-wake-word_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG, "libwakeword.so")
HOST_LIB = os.path.join(PKG, "libwakeword_host.so")      # the host-CPU library (wk_host.cpp, no HIP)
HOST_SOURCES = ["wk_host.cpp", "wk_wav.cpp"]   # (wk_wav.cpp is host C++ in both libraries)
OBJDIR = os.path.join(ROOT, "build")
SOURCES = ["wk_frontend.hip", "wk_fused.hip", "wk_fused_xdl.hip", "wk_misc.hip", "wk_api.hip", "wk_ctc.hip", "wk_wav.cpp", "wk_int8.hip", "wk_esp_mfcc.hip"]
LIBS = ["-Wl,-rpath,/opt/rocm/lib"]   # HIP runtime only: every GEMM is a hand-written kernel (no rocBLAS)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("WK_OFFLOAD_ARCH", "gfx950")
CFLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-fno-signed-zeros", "-ffp-contract=fast", "-fno-slp-vectorize",
          "-Wall", "-Wno-unused-function", "-I", INCLUDE, "-I", CSRC]


def _compile(src: str, extra) -> str:
    obj = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
    cmd = [HIPCC, *CFLAGS, *extra, "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip():
        sys.stderr.write(r.stderr)
    return obj


def _stale(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(INCLUDE, h) for h in os.listdir(INCLUDE)]
    return any(os.path.getmtime(d) > t for d in deps + [__file__])


def build_host(force: bool = False) -> str:
    """libwakeword_host.so: the host-CPU path (include/wakeword_host.h), plain
    g++ -- it links no HIP and is what a caller without a GPU loads."""
    if not force and not _stale(HOST_LIB):
        return HOST_LIB
    cxx = os.environ.get("CXX", "g++")
    tmp = HOST_LIB + ".tmp"
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", "-I", INCLUDE, "-I", CSRC,
           *[os.path.join(CSRC, f) for f in HOST_SOURCES], "-Wl,--no-undefined", "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"host library build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, HOST_LIB)
    return HOST_LIB


def build(force: bool = False, extra=()) -> str:
    """libwakeword.so.  The host library is built alongside, but a host-compiler
    failure there is reported and does not block the GPU library (which does
    not need it); wakeword.host / the --cpu CLI build it on demand and raise."""
    try:
        build_host(force)
    except (RuntimeError, OSError) as e:
        sys.stderr.write(f"warning: host library not built: {e}\n")
    if not force and not _stale():
        return LIB
    if shutil.which(HIPCC) is None and not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found ({HIPCC})")
    os.makedirs(OBJDIR, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(s, list(extra)), SOURCES))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, *LIBS, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
