"""Build the in-tree HIP library for gfx950 (``hipcc --offload-arch=gfx950``).

``python -m xtddft_amd.build`` or ``xtddft_amd.build.build()``; the result
``xtddft_amd/_lib/libxtddft_amd.so`` travels with the repository snapshot.
Each translation unit compiles to its own object (in parallel, only when it or
a header changed), then one link step produces the shared library.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
OBJ_DIR = os.path.join(OUT_DIR, "obj")
OUT = os.path.join(OUT_DIR, "libxtddft_amd.so")
SOURCES = ["xt_gemm.hip", "xt_kernels.hip", "xt_chol.hip", "xt_ctx.hip"]
HEADERS = ["xt_internal.h", "xt_kernels.h", "../../include/xtddft_amd.h"]
ARCH = os.environ.get("XT_OFFLOAD_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _obj(src):
    return os.path.join(OBJ_DIR, src.replace(".hip", ".o"))


def _stale_sources(force):
    hdr = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS)
    out = []
    for s in SOURCES:
        o = _obj(s)
        if force or _mtime(o) < max(hdr, _mtime(os.path.join(CSRC, s))):
            out.append(s)
    return out


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = _mtime(OUT)
    if any(_mtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS):
        return True
    return False


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(OBJ_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    todo = _stale_sources(force)

    def compile_one(src):
        cmd = [hipcc] + FLAGS + ["-c", os.path.join(CSRC, src), "-o", _obj(src) + ".tmp"]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        os.replace(_obj(src) + ".tmp", _obj(src))

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(todo)))) as ex:
        list(ex.map(compile_one, todo))
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp"] + \
        [_obj(s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
