"""Stored 4-index ERIs in PySCF's 8-fold packed order (jk_mode 'ERI8').

The reference's incore path keeps ``mf._eri`` packed with ``ao2mo.restore(8,
eri, nao)`` and hands it to ``get_jk`` (XTDA.py:518-543 via PySCF).  Pair
index ij = i(i+1)/2 + j for i >= j; (ij|kl) lives at ij(ij+1)/2 + kl for
ij >= kl.  The device factorises the packed array itself
(``xt_set_jk_eri8``); these host helpers only build and inspect packed arrays.
"""
from __future__ import annotations

import numpy as np


def npair(nao: int) -> int:
    return nao * (nao + 1) // 2


def pair_indices(nao: int):
    """(i, j) with i >= j in pair order ij = i(i+1)/2 + j."""
    i, j = np.tril_indices(nao)
    return i, j


def pack_s8(eri_full: np.ndarray) -> np.ndarray:
    """(nao, nao, nao, nao) with 8-fold symmetry -> packed (npair(npair+1)/2,)."""
    nao = eri_full.shape[0]
    i, j = pair_indices(nao)
    v = eri_full[i[:, None], j[:, None], i[None, :], j[None, :]]   # (npair, npair)
    a, b = np.tril_indices(v.shape[0])
    return np.ascontiguousarray(v[a, b])


def unpack_s8(packed: np.ndarray, nao: int) -> np.ndarray:
    """Packed 8-fold -> full (nao, nao, nao, nao) (small nao only)."""
    n = npair(nao)
    v = np.zeros((n, n))
    a, b = np.tril_indices(n)
    v[a, b] = packed
    v[b, a] = packed
    i, j = pair_indices(nao)
    pair = np.zeros((nao, nao), dtype=np.int64)
    pair[i, j] = np.arange(n)
    pair[j, i] = np.arange(n)
    return v[pair[:, :, None, None], pair[None, None, :, :]]


def eri_from_cderi(cderi) -> np.ndarray:
    """Packed (mu nu|la si) = sum_P B_P[mu,nu] B_P[la,si] from a symmetric DF factor."""
    b = np.asarray(cderi, dtype=np.float64)
    nao = b.shape[1]
    i, j = pair_indices(nao)
    bp = b[:, i, j]                  # (naux, npair)
    v = bp.T @ bp
    a, c = np.tril_indices(v.shape[0])
    return np.ascontiguousarray(v[a, c])
