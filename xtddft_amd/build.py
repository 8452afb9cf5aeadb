"""Build the in-tree HIP library for gfx950 (``hipcc --offload-arch=gfx950``).

``python -m xtddft_amd.build`` or ``xtddft_amd.build.build()``; the result
``xtddft_amd/_lib/libxtddft_amd.so`` travels with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
OUT = os.path.join(OUT_DIR, "libxtddft_amd.so")
SOURCES = ["xt_gemm.hip", "xt_kernels.hip", "xt_chol.hip", "xt_ctx.hip"]
HEADERS = ["xt_internal.h", "xt_kernels.h", "../../include/xtddft_amd.h"]
ARCH = os.environ.get("XT_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    for f in SOURCES + HEADERS:
        if os.path.getmtime(os.path.join(CSRC, f)) > t:
            return True
    return False


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(OUT_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17",
           "-Wno-unused-result", "-o", OUT + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{r.stdout}\n{r.stderr}")
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
