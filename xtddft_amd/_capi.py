"""ctypes binding of the C ABI declared in ``include/xtddft_amd.h``.

The shared library is built in-tree (``xtddft_amd/_lib/libxtddft_amd.so``,
see ``xtddft_amd.build``).  There is no fallback: if the library is missing
or cannot be loaded, every operator raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_long, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libxtddft_amd.so")

XT_PTR_HOST = 0
XT_PTR_DEVICE = 1
KIND = {"XTDA": 0, "UTDA": 1, "SF_DOWN": 2, "SF_UP": 3, "XSF": 4}
XC = {"HF": 0, "LDA": 1, "GGA": 2, "MGGA": 3}
K_MODE = {"auto": 0, "direct": 1, "stored": 2}
SF_KERNEL = {"alda0": 0, "mc": 1}
K_MODE_NAME = {v: k for k, v in K_MODE.items()}

ERRORS = {-1: ValueError, -2: MemoryError, -3: RuntimeError, -4: RuntimeError, -5: RuntimeError}

EXPORTS = [
    "xt_create", "xt_destroy", "xt_set_stream", "xt_last_error", "xt_abi_version",
    "xt_set_orbitals", "xt_set_fock_mo", "xt_set_orbital_energies", "xt_set_jk_df",
    "xt_set_jk_eri8", "xt_naux",
    "xt_set_grid", "xt_set_oo_basis", "xt_apply", "xt_dim", "xt_last_timings",
    "xt_xsf_j_diagonals", "xt_set_exchange_mode", "xt_prepare", "xt_exchange_plan", "xt_set_partition", "xt_set_profile",
    "xt_profile_stats", "xt_profile_bytes", "xt_dgemm", "xt_dgemm_strided", "xt_precond", "xt_row_norms2", "xt_row_scale", "xt_build_id",
    "xt_int3c2e_cart", "xt_int2e_cart", "xt_eval_ao",
]


class XtDesc(ctypes.Structure):
    _fields_ = [
        ("kind", c_int), ("restricted", c_int), ("nao", c_int), ("nmo", c_int),
        ("nc", c_int), ("no", c_int), ("nv", c_int), ("naux", c_int), ("ngrid", c_int),
        ("xctype", c_int), ("hyb", c_double), ("alpha", c_double), ("omega", c_double),
        ("si", c_double), ("sa", c_int), ("foo", c_double), ("fglobal", c_double),
        ("remove", c_int), ("add_local", c_int), ("device", c_int), ("sf_kernel", c_int),
    ]


ABI_VERSION = 7   # include/xtddft_amd.h XT_ABI_VERSION


class LibraryMissing(RuntimeError):
    pass


_lib = None


def lib():
    """Load the HIP library (raises LibraryMissing -- no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LibraryMissing(f"{LIB_PATH} not built; run xtddft_amd.build.build()")
    # PyTorch-ROCm ships its own libamdhip64 (same SONAME).  Load it first so the
    # library binds to that single HIP runtime instead of a second copy from
    # /opt/rocm (two HIP/HSA runtimes in one process cannot share the device).
    try:
        import torch  # noqa: F401
    except Exception:   # pragma: no cover -- plain C-ABI use without torch
        pass
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:   # pragma: no cover
        raise LibraryMissing(f"cannot load {LIB_PATH}: {e}") from e
    vp = c_void_p
    dp = c_void_p   # double* passed as raw addresses (host numpy or device)
    L.xt_create.argtypes = [POINTER(XtDesc), POINTER(vp)]
    L.xt_destroy.argtypes = [vp]
    L.xt_set_stream.argtypes = [vp, vp]
    L.xt_last_error.restype = ctypes.c_char_p
    L.xt_build_id.restype = ctypes.c_char_p
    L.xt_set_orbitals.argtypes = [vp, dp, dp, c_int]
    L.xt_set_fock_mo.argtypes = [vp, dp, dp, dp, dp, c_int]
    L.xt_set_orbital_energies.argtypes = [vp, dp, dp, c_int]
    L.xt_set_jk_df.argtypes = [vp, dp, c_int, c_int]
    L.xt_set_jk_eri8.argtypes = [vp, dp, c_int, c_double, c_int, c_int, c_int]
    L.xt_naux.argtypes = [vp, POINTER(c_int), POINTER(c_int)]
    L.xt_set_grid.argtypes = [vp, dp, dp, dp, c_int]
    L.xt_set_oo_basis.argtypes = [vp, dp, c_int]
    L.xt_apply.argtypes = [vp, c_int, dp, dp, c_int]
    L.xt_dim.argtypes = [vp]
    L.xt_last_timings.argtypes = [vp, dp]
    L.xt_xsf_j_diagonals.argtypes = [vp, dp, dp, c_int]
    L.xt_set_exchange_mode.argtypes = [vp, c_int, c_double]
    L.xt_prepare.argtypes = [vp, POINTER(c_int), POINTER(c_double)]
    L.xt_exchange_plan.argtypes = [vp, POINTER(c_int), POINTER(c_double)]
    L.xt_set_partition.argtypes = [vp, c_int, c_int, c_int, c_int]
    L.xt_set_profile.argtypes = [vp, c_int]
    L.xt_profile_stats.argtypes = [vp, c_int, dp]
    L.xt_profile_bytes.argtypes = [vp, c_int, dp]
    L.xt_dgemm.argtypes = [c_int, c_int, c_int, c_int, c_int, c_double, dp, c_long, dp, c_long,
                           c_double, dp, c_long, vp]
    L.xt_dgemm_strided.argtypes = [c_int, c_int, c_int, c_int, c_int, c_double, dp, c_long, c_long, c_long, c_long,
                                   dp, c_long, c_long, c_long, c_long, c_double, dp, c_long, c_long, vp]
    L.xt_precond.argtypes = [c_int, c_int, dp, dp, c_double, dp, dp, vp]
    L.xt_row_norms2.argtypes = [c_int, c_int, dp, dp, vp]
    L.xt_row_scale.argtypes = [c_int, c_int, dp, dp, vp]
    L.xt_int3c2e_cart.argtypes = [c_int, vp, dp, dp, c_int, vp, dp, dp, c_int, c_int, c_double, dp, c_long, vp]
    L.xt_int2e_cart.argtypes = [c_int, vp, dp, dp, c_int, vp, dp, dp, c_int, c_int, c_double, dp, dp, c_double,
                                c_int, dp, c_long, vp]
    L.xt_eval_ao.argtypes = [c_int, dp, c_int, vp, dp, dp, dp, c_int, dp, c_long, c_long, vp]
    for name in EXPORTS:
        if not hasattr(L, name):
            raise LibraryMissing(f"{LIB_PATH} lacks symbol {name}")
    if L.xt_abi_version() != ABI_VERSION:
        raise LibraryMissing(f"{LIB_PATH} has ABI {L.xt_abi_version()}, expected {ABI_VERSION}; rebuild")
    # the library must have been built from THIS tree's sources (xtddft_amd.build.source_hash)
    from .build import source_hash
    want, have = source_hash(), L.xt_build_id().decode()
    if want is not None and have != want:
        raise LibraryMissing(f"{LIB_PATH} was built from other sources (build id {have}, tree {want}); "
                             f"run xtddft_amd.build.build()")
    _lib = L
    return L


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().xt_last_error().decode(errors="replace")
        raise ERRORS.get(rc, RuntimeError)(f"{what}: {msg} (code {rc})")
