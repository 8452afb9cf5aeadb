"""Build the in-tree HIP library for gfx950 (``hipcc --offload-arch=gfx950``).

``python -m xtddft_amd.build`` or ``xtddft_amd.build.build()``; the result
``xtddft_amd/_lib/libxtddft_amd.so`` travels with the repository snapshot.
Each translation unit compiles to its own object (in parallel, only when it or
a header changed), then one link step produces the shared library.

The library is bound to its sources: ``source_hash()`` (SHA-256 over every
source and header, the compiler flags and the target) is compiled into it and
exported as ``xt_build_id()``; ``build()`` rebuilds whenever the hash of the
tree differs from the one in the library, and ``_capi.lib()`` refuses to load a
library built from other sources.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
OBJ_DIR = os.path.join(OUT_DIR, "obj")
OUT = os.path.join(OUT_DIR, "libxtddft_amd.so")
SOURCES = ["xt_gemm.hip", "xt_exch.hip", "xt_xcm.hip", "xt_xcw.hip", "xt_xcws.hip", "xt_kernels.hip", "xt_chol.hip", "xt_int.hip",
           "xt_ctx.hip"]
HEADERS = ["xt_internal.h", "xt_kernels.h", "../../include/xtddft_amd.h"]
ARCH = os.environ.get("XT_OFFLOAD_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result"]


def source_hash() -> str | None:
    """SHA-256 (hex, 32 chars) of the sources, headers, flags and target; None
    when the sources are not present (an installed library without its tree)."""
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        p = os.path.join(CSRC, f)
        if not os.path.exists(p):
            return None
        h.update(f.encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:32]


_ID_TAG = b"XT_BUILD_ID:"


def library_build_id(path: str = OUT) -> str | None:
    """The source hash compiled into a built library, read from the file (no
    dlopen: a library already loaded in this process would shadow a rebuilt one)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    i = data.find(_ID_TAG)
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + len(_ID_TAG):j].decode()


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
    want = source_hash()
    return want is not None and library_build_id() != want


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(OBJ_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    todo = _stale_sources(force)
    # an id mismatch with up-to-date objects (e.g. objects from another tree): recompile all
    if not todo and not force:
        todo = list(SOURCES)

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
    # the build id: one tiny C unit carrying the source hash
    bid_c = os.path.join(OBJ_DIR, "xt_build_id.c")
    bid_o = os.path.join(OBJ_DIR, "xt_build_id.o")
    with open(bid_c, "w") as f:
        f.write('static const char id[] = "%s%s";\n'
                'const char* xt_build_id(void) { return id + %d; }\n'
                % (_ID_TAG.decode(), source_hash(), len(_ID_TAG)))
    r = subprocess.run(["gcc", "-O2", "-fPIC", "-c", bid_c, "-o", bid_o], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"gcc failed on the build id:\n{r.stderr}")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp"] + \
        [_obj(s) for s in SOURCES] + [bid_o]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
