"""Integral-direct pivoted Cholesky factorisation of the ERIs on the GPU.

The reference's default mean field is direct-SCF with exact J/K
(``mf.get_jk`` / ``get_k``, XTDA.py:518-543) and exact MO integrals
(``ao2mo.general``, XTDA.py:120).  The hot path consumes any exact factor
(mu nu|la si) = sum_P L_P[mu nu] L_P[la si] through the same MO-route engine as a
DF factor (``xt_set_jk_df``), so the exact ERIs are handed over as their pivoted
Cholesky vectors -- computed here without the 4-index array ever existing
(SURVEY.md 7.3.3 / 8(f)1):

* the diagonal (mu nu|mu nu) and per-shell-pair Schwarz bounds from the integral
  kernel (``dints.eri_diag_device``);
* while the largest residual diagonal D_max exceeds ``tol``: take the shell pairs
  whose residual exceeds ``spread`` x D_max (at most ``batch`` of them, largest
  first), evaluate their columns (all pairs | those pairs) with the integral kernel
  (Schwarz-screened), subtract the existing vectors' contribution with one GEMM
  (``xt_dgemm``), then pivot inside the batch -- new vectors are taken while the
  batch's residual diagonal exceeds max(tol, spread x D_max).  The pivoting runs on
  the batch's own (ncols x ncols) residual block on the host (``_batch_pivots``: the
  pivot order and the new vectors' values at the batch pairs), then every new vector
  at once on the device by one triangular solve, V_new^T = Lp^-1 M[:, piv]^T, and the
  diagonal by one sum of squares -- the same vectors as a rank-one update of the
  (npack x ncols) columns per pivot (C60 / cc-pVDZ: 11 954 of them, 9.5 s), in a few
  device calls per batch.

The result is exact to ``tol``: every residual diagonal is <= tol at exit, so by
Cauchy-Schwarz every |(mu nu|la si) - sum_P L L| <= tol.  Vectors live in the
packed pair index mu (mu+1)/2 + nu; ``cholesky_eri`` returns them unpacked as
the (naux, nao, nao) factor the operator and the SCF take.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

from .. import _capi
from .dints import eri_columns_device, eri_diag_device, pair_table

SCREEN = 1e-15        # Schwarz threshold (absolute), far below any factorisation tol
TRSM_COLS = 8192      # packed columns per triangular solve


def _gemm_tn_sub(L, a, b, c, device):
    """c -= a^T b on device (a (k, m), b (k, n), c (m, n) contiguous) via xt_dgemm."""
    import torch
    st = torch.cuda.current_stream(torch.device(f"cuda:{device}")).cuda_stream
    k, m = a.shape
    n = b.shape[1]
    _capi.check(L.xt_dgemm(1, 0, m, n, k, -1.0, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), 1.0,
                           c.data_ptr(), c.stride(0), ctypes.c_void_p(st)), "xt_dgemm")


def _batch_pivots(C: np.ndarray, d: np.ndarray, cut: float):
    """Pivoted Cholesky of one batch's residual block C (ncols x ncols, symmetric) with
    residual diagonal d: pivots are taken largest-first while d > cut.  Returns the
    pivot columns and Lb (ncols x r), the new vectors' values at the batch pairs
    (column k = vector k)."""
    n = d.size
    d = d.astype(np.float64, copy=True)
    Lb = np.zeros((n, n))
    piv = []
    for k in range(n):
        iq = int(np.argmax(d))
        dk = d[iq]
        if dk <= cut:
            break
        col = (C[:, iq] - Lb[:, :k] @ Lb[iq, :k]) / math.sqrt(dk)
        Lb[:, k] = col
        d -= col * col
        d[iq] = 0.0
        piv.append(iq)
    return np.asarray(piv, dtype=np.int64), Lb[:, :len(piv)]


def cholesky_packed(mol, tol: float = 1e-12, device: int = 0, batch: int = 24, spread: float = 0.01,
                    omega: float = 0.0, stats: dict | None = None):
    """Packed Cholesky vectors (naux, npack) of the ERIs (omega > 0: the
    erf(omega r12)/r12 ERIs) on GPU ``device``."""
    import time
    import torch
    L = _capi.lib()
    tab = pair_table(mol)
    dv = torch.device(f"cuda:{device}")
    t0 = time.perf_counter()
    split = dict(diag=0.0, columns=0.0, gemm=0.0, pivot=0.0)

    def lap(name, t):
        torch.cuda.synchronize(dv)
        now = time.perf_counter()
        split[name] += now - t
        return now
    with torch.cuda.device(dv):
        D, q = eri_diag_device(mol, device, omega)
        D = D.clone()
        pack_pair = tab.dev(device)["pack_pair"]
        npack = tab.npack
        cap = min(npack, max(64, 4 * mol.nao))
        V = torch.empty((cap, npack), dtype=torch.float64, device=dv)
        nvec = 0
        nbatch = ncols = 0
        pmax = torch.empty(tab.npair, dtype=torch.float64, device=dv)
        t = lap("diag", t0)
        while True:
            dmax = float(D.max())
            if dmax <= tol:
                break
            pmax.fill_(0.0)
            pmax.scatter_reduce_(0, pack_pair, D, reduce="amax")
            cut = max(spread * dmax, tol)
            cand = torch.nonzero(pmax > cut).flatten()
            cand = cand[torch.argsort(pmax[cand], descending=True)][:batch].cpu().numpy()
            cols, M = eri_columns_device(mol, cand, q, SCREEN, device, omega)
            t = lap("columns", t)
            nbatch += 1
            ncols += len(cols)
            tcols = torch.as_tensor(cols, device=dv)
            if nvec:
                _gemm_tn_sub(L, V[:nvec], V[:nvec][:, tcols].contiguous(), M, device)
            t = lap("gemm", t)
            piv, Lb = _batch_pivots(M[tcols].cpu().numpy(), D[tcols].cpu().numpy(), cut)
            r = piv.size
            if r:
                while nvec + r > V.shape[0]:
                    grow = min(npack, 2 * V.shape[0]) - V.shape[0]
                    if grow <= 0:
                        raise RuntimeError("Cholesky rank exceeds the number of pairs")
                    V = torch.cat([V, torch.empty((grow, npack), dtype=torch.float64, device=dv)])
                # vector k = (M[:, piv_k] - sum_{j<k} v_j Lb[piv_k, j]) / Lb[piv_k, k]:
                # Lp V_new^T = M[:, piv]^T with Lp = Lb[piv] lower triangular
                tp = torch.as_tensor(piv, device=dv)
                Lp = torch.as_tensor(Lb[piv], device=dv)
                # (column blocks: one rocBLAS trsm over all npack columns asks for more
                # workspace than torch hands hipBLAS and fails with ALLOC_FAILED)
                vn = V[nvec:nvec + r]
                for c0 in range(0, npack, TRSM_COLS):
                    c1 = min(c0 + TRSM_COLS, npack)
                    vn[:, c0:c1] = torch.linalg.solve_triangular(Lp, M[c0:c1, tp].T.contiguous(), upper=False)
                nvec += r
                D -= (vn * vn).sum(0)
                D[tcols[tp]] = 0.0
            D.clamp_(min=0.0)
            if r == 0 and float(D[tcols].max()) > cut:
                raise RuntimeError("pivoted Cholesky made no progress on a batch")
            t = lap("pivot", t)
        torch.cuda.synchronize(dv)
    if stats is not None:
        stats.update(naux=nvec, batches=nbatch, columns=ncols, seconds=time.perf_counter() - t0,
                     npack=npack, tol=tol, split_s={k: round(v, 3) for k, v in split.items()})
    return V[:nvec]


def unpack(vecs, mol, device: int = 0):
    """(naux, npack) packed vectors -> (naux, nao, nao) symmetric factor (device)."""
    tab = pair_table(mol)
    n = mol.nao
    return vecs[:, tab.dev(device)["packidx"]].reshape(-1, n, n)


def cholesky_eri(mol, tol: float = 1e-12, device: int = 0, omega: float = 0.0, stats: dict | None = None, **kw):
    """Exact-ERI factor B (naux, nao, nao) on the GPU with
    |(mu nu|la si) - sum_P B[P,mu,nu] B[P,la,si]| <= tol for every element."""
    return unpack(cholesky_packed(mol, tol, device, omega=omega, stats=stats, **kw), mol, device)


def eri_from_packed(vecs, mol, device: int = 0):
    """(mu nu|la si) reassembled from packed vectors (testing, small molecules)."""
    b = unpack(vecs, mol, device).reshape(vecs.shape[0], -1)
    n = mol.nao
    return (b.T @ b).reshape(n, n, n, n).cpu().numpy()

