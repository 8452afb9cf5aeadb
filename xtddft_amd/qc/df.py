"""Density fitting: auxiliary basis, 3-index factor, DF J/K (PySCF ``mf.density_fit()``).

Replaces ``df.DF`` / ``df_jk.get_jk`` on the reference's DF path (the mean
field whose ``get_jk`` XTDA.py:518-543 calls, and ``ao2mo`` of XTDA.py:120 via
the same factor): ``cderi[P] = sum_Q (L^-1)_PQ (Q|mu nu)`` with (P|Q) = L L^T
(``df.incore.cholesky_eri``), so (mu nu|la si) ~ sum_P cderi[P,mu,nu] cderi[P,la,si].

The auxiliary basis is either given by the caller ({element: shells}, PySCF
format) or generated even-tempered per element from the orbital basis in the
manner of PySCF's ``df.addons.aug_etb`` (exponent range of the products of the
element's orbital primitives per total angular momentum, ratio ``beta``):
no JK-fitting basis data can be loaded offline.  DF results are therefore
unpinned against the reference (whose notebooks use the exact 4-index ERIs);
the fitting error itself is tested against the exact ERIs.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg

ETB_BETA = 2.0


def make_auxbasis(mol, beta: float = ETB_BETA):
    """Even-tempered auxiliary basis {element: [[l, [exp, 1.0]], ...]}."""
    from . import basis as _basis
    out = {}
    for el in sorted(set(mol.elements)):
        emin = {}
        emax = {}
        for sh in _basis.load(mol.basis, el):
            l = int(sh[0])
            prim = np.array(sh[1:], dtype=np.float64)
            es = prim[np.abs(prim[:, 1:]).max(axis=1) > 1e-3, 0]
            if es.size == 0:
                continue
            emin[l] = min(emin.get(l, np.inf), es.min())
            emax[l] = max(emax.get(l, 0.0), es.max())
        lmax = max(emin)
        ranges = []
        for L in range(2 * lmax + 1):                # product angular momenta
            lo, hi = np.inf, 0.0
            for li in emin:
                for lj in emin:
                    if li + lj == L:
                        lo = min(lo, math.sqrt(emin[li] * emin[lj]))
                        hi = max(hi, math.sqrt(emax[li] * emax[lj]))
            if np.isfinite(lo):
                ranges.append((L, 2.0 * lo, 2.0 * hi))   # alpha + alpha on one centre
        # one polarisation level above the products, with the top product range (a
        # two-centre product needs higher l on each centre; measured on HF/6-31G:
        # max |(ij|kl) - fit| 2.4e-3 without it, 1.1e-4 with it)
        ranges.append((ranges[-1][0] + 1, ranges[-1][1], ranges[-1][2]))
        shells = []
        for L, lo, hi in ranges:
            n = int(math.ceil(math.log((hi + lo) / lo) / math.log(beta)))
            for i in reversed(range(max(n, 1))):
                shells.append([L, [lo * beta ** i, 1.0]])
        out[el] = shells
    return out


def aux_mole(mol, auxbasis=None):
    from .gto import Mole
    if auxbasis is None:
        auxbasis = make_auxbasis(mol)
    return Mole(mol.atom, basis=auxbasis, charge=0, spin=_aux_spin(mol, auxbasis), unit=mol.unit)


def _aux_spin(mol, auxbasis):
    # the aux "molecule" only carries functions; pick the spin parity its charge needs
    return int(round(sum(mol._charges))) % 2


def cholesky_cderi(j3: np.ndarray, j2: np.ndarray, lindep: float = 1e-12) -> np.ndarray:
    """cderi = L^-1 (P|mu nu) with (P|Q) = L L^T; a numerically singular (P|Q) is
    handled by its eigendecomposition with eigenvalues below ``lindep`` dropped."""
    naux, n, _ = j3.shape
    flat = j3.reshape(naux, n * n)
    try:
        low = np.linalg.cholesky(j2)
        out = scipy.linalg.solve_triangular(low, flat, lower=True)
    except np.linalg.LinAlgError:
        w, v = np.linalg.eigh(j2)
        keep = w > lindep * w.max()
        out = (v[:, keep] / np.sqrt(w[keep])).T @ flat
    return out.reshape(-1, n, n)


class DF:
    """``mf.with_df``: auxiliary Mole and the 3-index factor."""

    def __init__(self, mol, auxbasis=None, device=None):
        self.mol = mol
        self.auxbasis = auxbasis
        self.device = device            # GPU for the 3-index integrals (None: host)
        self.auxmol = None
        self._cderi = None
        self._cderi_lr = {}

    def build(self):
        if self._cderi is None:
            self.auxmol = aux_mole(self.mol, self.auxbasis)
            j3 = self.mol.int3c2e(self.auxmol, device=self.device)
            j2 = self.auxmol.int2c2e()
            self._cderi = cholesky_cderi(j3, j2)
        return self

    @property
    def cderi(self):
        return self.build()._cderi

    def cderi_lr(self, omega: float):
        """The long-range factor of erf(omega r12)/r12 (PySCF ``with_df.range_coulomb``:
        3-index and 2-index integrals both attenuated), the ``cderi_lr`` of a
        range-separated mean field (MeanField, XTDA.py:527-539): the SCF's long-range
        exchange of CAM-B3LYP (``xc._RSH``) and the factor ``_meanfield`` hands the
        operator.  Cached per omega."""
        self.build()
        key = float(omega)
        if key not in self._cderi_lr:
            j3 = self.mol.int3c2e(self.auxmol, device=self.device, omega=omega)
            self._cderi_lr[key] = cholesky_cderi(j3, self.auxmol.int2c2e(omega=omega))
        return self._cderi_lr[key]

    def get_k_lr(self, dms, omega: float):
        """Long-range K[D] = sum_P L_P D L_P with the erf(omega r12)/r12 factor."""
        return self.get_jk(dms, with_j=False, factor=self.cderi_lr(omega))[1]

    def get_jk(self, dms, with_j=True, with_k=True, factor=None):
        """J[D] = sum_P B_P <B_P, D>, K[D] = sum_P B_P D B_P (PySCF convention)."""
        b = self.cderi if factor is None else factor
        naux, n, _ = b.shape
        d = np.asarray(dms, dtype=np.float64)
        shape = d.shape
        d = d.reshape(-1, n, n)
        vj = vk = None
        if with_j:
            gam = b.reshape(naux, n * n) @ d.reshape(-1, n * n).T          # (naux, nset)
            vj = (gam.T @ b.reshape(naux, n * n)).reshape(shape)
        if with_k:
            vk = np.empty_like(d)
            for x in range(d.shape[0]):
                t = (b.reshape(-1, n) @ d[x]).reshape(naux, n, n)          # B_P D
                vk[x] = np.einsum('pml,pln->mn', t, b, optimize=True)
            vk = vk.reshape(shape)
        return vj, vk
