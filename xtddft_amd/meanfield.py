"""Mean-field duck types consumed by the TDA operators.

The reference drives every operator from a PySCF ``mol`` / ``mf`` pair
(``XTDA.py:21-37``, ``SF_TDA.py:26-37``, ``XSF_TDA.py:147-213``).  PySCF is not
part of this framework, so the data the hot path actually reads from ``mf`` is
carried by the two plain containers below:

* ``Mole``      -- ``spin`` and ``nao_nr()`` (``XTDA.py:283,613``).
* ``MeanField`` -- orbitals / occupations / energies, the KS and pure-HF
  effective potentials at the SCF density (``XTDA.py:588-613``,
  ``XSF_TDA.py:1070-1114``), the hybrid coefficients of
  ``ni.rsh_and_hybrid_coeff`` (``XTDA.py:501``), the density-fitting factor
  ``B[P,mu,nu]`` that defines ``(mu nu|la si) = sum_P B B`` for ``get_jk``
  (``XTDA.py:518-543``), and the cached XC kernel on the grid that
  ``ni.cache_xc_kernel`` / ``cache_xc_kernel_sf`` produce once per solve
  (``XTDA.py:504``, ``SF_TDA.py:39-88``).

No arithmetic lives here: the containers only validate shapes/orderings and
expose the reference attribute names.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np


@dataclass
class Mole:
    """Minimal ``gto.Mole`` stand-in: what the TDA operators read."""
    nao: int
    spin: int
    nelectron: int = 0
    symmetry: bool = False

    def nao_nr(self) -> int:
        return self.nao


@dataclass
class Grid:
    """AO values on the integration grid (``ni.block_loop`` output, whole grid).

    ao      : (ncomp, ngrid, nao)  ncomp = 1 (LDA) or 4 (GGA: value, d/dx, d/dy, d/dz)
    weights : (ngrid,)
    """
    ao: np.ndarray
    weights: np.ndarray

    @property
    def ngrid(self) -> int:
        return int(self.weights.shape[0])

    @property
    def ncomp(self) -> int:
        return int(self.ao.shape[0])


def _pad_rows(b, n):
    """b (naux, nao, nao) with zero rows appended up to n (NumPy or a torch tensor)."""
    if int(b.shape[0]) == n:
        return b
    if type(b).__module__.startswith("torch"):
        import torch
        return torch.cat([b, b.new_zeros((n - b.shape[0],) + tuple(b.shape[1:]))])
    return np.concatenate([np.asarray(b), np.zeros((n - b.shape[0],) + b.shape[1:])])


@dataclass
class MeanField:
    """``mf`` duck type (ROKS when ``mo_coeff.ndim == 2``, UKS when 3).

    Attributes mirror PySCF names so the reference call sites read the same:
    ``mo_coeff``, ``mo_occ``, ``mo_energy``, ``xc``, ``level_shift``,
    ``get_hcore()``, ``get_veff()``, ``make_rdm1()``.

    veff     : (2, nao, nao)  KS effective potential at the SCF density.
    veff_hf  : (2, nao, nao)  pure-HF potential at the same density
               (``scf.ROHF(mol).get_veff(mol, dm)``, XTDA.py:608-612).
    cderi    : (naux, nao, nao) symmetric DF factor, full-range Coulomb
               (jk_mode 'DF').
    cderi_lr : optional (naux, nao, nao) factor of the long-range
               erf(omega r)/r operator for range-separated hybrids.
    eri      : stored 4-index ERIs in PySCF 8-fold packed order (the incore
               ``mf._eri``, ``ao2mo.restore(8, ...)``) -- jk_mode 'ERI8',
               used when ``cderi`` is None.  ``eri_lr`` likewise for the
               long-range operator; ``chol_tol`` the device Cholesky
               tolerance (0: 1e-13 x largest diagonal).
    fxc      : (2, ncomp, 2, ncomp, ngrid) un-weighted UKS second derivative
               kernel (``cache_xc_kernel`` output, XTDA.py:504); ncomp 1 / 4 / 5
               for LDA / GGA / MGGA (rho, grad rho, tau -- PySCF's MGGA layout).
    fxc_sf   : (ngrid,) ALDA0 spin-flip kernel already multiplied by the grid
               weight (``cache_xc_kernel_sf``, SF_TDA.py:82-84).
    fxc_sf_mc: optional (nk, nk, ngrid) multicollinear spin-flip kernel (method=1,
               ``cache_xc_kernel_sf_mc``, SF_TDA.py:942-974), un-weighted, over the spin
               variables (s, grad s[, tau_s]); None: computed on demand from the SCF
               density (``xtddft_amd.mcol.sf_mc_kernel``).
    xctype   : 'HF' | 'LDA' | 'GGA' | 'MGGA'
    omega, alpha, hyb : ``ni.rsh_and_hybrid_coeff`` (XTDA.py:501).
    """
    mol: Mole
    mo_coeff: np.ndarray
    mo_occ: np.ndarray
    mo_energy: np.ndarray
    h1e: np.ndarray
    veff: np.ndarray
    veff_hf: np.ndarray
    cderi: Optional[np.ndarray] = None
    grids: Optional[Grid] = None
    fxc: Optional[np.ndarray] = None
    fxc_sf: Optional[np.ndarray] = None
    fxc_sf_mc: Optional[np.ndarray] = None
    nlc: bool = False          # the SCF functional carries a VV10 non-local term (mf.do_nlc())
    cderi_lr: Optional[np.ndarray] = None
    xc: str = "synthetic"
    xctype: str = "GGA"
    omega: float = 0.0
    alpha: float = 0.0
    hyb: float = 0.0
    level_shift: float = 0.0
    eri: Optional[np.ndarray] = None
    eri_lr: Optional[np.ndarray] = None
    chol_tol: float = 0.0
    e_tot: float = 0.0
    max_memory: int = 4000
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        self.mo_coeff = np.asarray(self.mo_coeff, dtype=np.float64)
        self.mo_occ = np.asarray(self.mo_occ)
        self.mo_energy = np.asarray(self.mo_energy, dtype=np.float64)
        if self.xctype not in ("HF", "LDA", "GGA", "MGGA"):
            raise ValueError(f"unsupported xctype {self.xctype!r}")
        if self.is_rohf:
            occ = self.mo_occ
            # core | open | virtual ordering (PySCF ROHF _finalize sorts this way);
            # the reference's block slicing (XTDA.py:636, XSF_TDA.py:1078) assumes it.
            nc = int(np.count_nonzero(occ == 2))
            no = int(np.count_nonzero(occ == 1))
            expect = np.concatenate([np.full(nc, 2), np.full(no, 1),
                                     np.zeros(occ.size - nc - no)])
            if not np.array_equal(occ, expect):
                raise ValueError("ROKS mo_occ must be ordered core|open|virtual")
        if self.cderi is None and self.eri is None:
            raise ValueError("need a DF factor (cderi) or stored ERIs (eri)")
        if self.cderi is not None and (self.cderi.ndim != 3 or self.cderi.shape[1:] != (self.nao, self.nao)):
            raise ValueError("cderi must be (naux, nao, nao)")
        if self.cderi is not None and self.cderi_lr is not None:
            if self.cderi_lr.ndim != 3 or tuple(self.cderi_lr.shape[1:]) != (self.nao, self.nao):
                raise ValueError("cderi_lr must be (naux_lr, nao, nao)")
            # the operator streams both factors over one aux window: a common row count,
            # zero rows padding the shorter factor (they add nothing to J or K)
            n = max(int(self.cderi.shape[0]), int(self.cderi_lr.shape[0]))
            self.cderi, self.cderi_lr = _pad_rows(self.cderi, n), _pad_rows(self.cderi_lr, n)
        npair = self.nao * (self.nao + 1) // 2
        for name in ("eri", "eri_lr"):
            e = getattr(self, name)
            if e is not None and np.asarray(e).size != npair * (npair + 1) // 2:
                raise ValueError(f"{name} must be 8-fold packed: npair*(npair+1)/2 = "
                                 f"{npair * (npair + 1) // 2} elements for nao = {self.nao}")

    # ---- reference attribute surface -------------------------------------
    @property
    def is_rohf(self) -> bool:
        return self.mo_coeff.ndim == 2

    @property
    def nao(self) -> int:
        return int(self.mo_coeff.shape[-2])

    @property
    def jk_mode(self) -> str:
        return "DF" if self.cderi is not None else "ERI8"

    @property
    def naux(self) -> int:
        return int(self.cderi.shape[0]) if self.cderi is not None else 0

    def get_hcore(self):
        return self.h1e

    def get_ovlp(self):
        """AO overlap (the SCF's when it supplied one; synthetic problems have S = I)."""
        s = self.extra.get("s1e")
        return np.eye(self.nao) if s is None else s

    def get_veff(self, mol=None, dm=None):
        return self.veff

    def get_veff_hf(self):
        return self.veff_hf

    def make_rdm1(self):
        if self.is_rohf:
            c = self.mo_coeff
            da = c[:, self.mo_occ >= 1] @ c[:, self.mo_occ >= 1].T
            db = c[:, self.mo_occ >= 2] @ c[:, self.mo_occ >= 2].T
        else:
            ca, cb = self.mo_coeff
            da = ca[:, self.mo_occ[0] > 0] @ ca[:, self.mo_occ[0] > 0].T
            db = cb[:, self.mo_occ[1] > 0] @ cb[:, self.mo_occ[1] > 0].T
        return np.asarray([da, db])

    def rsh_and_hybrid_coeff(self):
        return self.omega, self.alpha, self.hyb

    def spin_square(self):
        """<S^2> and 2S+1 as PySCF returns them: the pure-state value for ROKS; for a
        UKS determinant the SCF driver's value when it supplied one."""
        if "spin_square" in self.extra:
            return self.extra["spin_square"]
        s = 0.5 * self.mol.spin
        return s * (s + 1), 2 * s + 1

    # ---- occupation helpers (XTDA.py:565-586, SF_TDA.py:26-37) ------------
    def spin_occupations(self):
        """(mo_coeff_a, mo_coeff_b, occ_a, occ_b) as 0/1 arrays per spin."""
        if self.is_rohf:
            occ = np.zeros((2, self.mo_occ.size))
            occ[0][self.mo_occ >= 1] = 1
            occ[1][self.mo_occ >= 2] = 1
            return self.mo_coeff, self.mo_coeff, occ[0], occ[1]
        return self.mo_coeff[0], self.mo_coeff[1], self.mo_occ[0], self.mo_occ[1]

    def fock_mo(self):
        """KS Fock in the MO basis per spin: C^T (h1e + veff[s]) C (XTDA.py:589-595)."""
        ca, cb, _, _ = self.spin_occupations()
        return (ca.T @ (self.h1e + self.veff[0]) @ ca,
                cb.T @ (self.h1e + self.veff[1]) @ cb)

    def fock_mo_hf(self):
        """Pure-HF Fock in the MO basis (XTDA.py:608-612, XSF_TDA.py:1110-1113)."""
        ca, cb, _, _ = self.spin_occupations()
        return (ca.T @ (self.h1e + self.veff_hf[0]) @ ca,
                cb.T @ (self.h1e + self.veff_hf[1]) @ cb)

    def shape_info(self):
        """nc / no / nv in the reference's convention (utils.get_cov, utils.py:6-41)."""
        _, _, oa, ob = self.spin_occupations()
        nocc_a, nocc_b = int(oa.sum()), int(ob.sum())
        nmo = oa.size
        return dict(nc=min(nocc_a, nocc_b), no=abs(nocc_a - nocc_b),
                    nv=min(nmo - nocc_a, nmo - nocc_b), nocc_a=nocc_a,
                    nocc_b=nocc_b, nvir_a=nmo - nocc_a, nvir_b=nmo - nocc_b, nmo=nmo)
