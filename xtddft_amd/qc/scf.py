"""ROKS / UKS (and ROHF / UHF) self-consistent field, producing the ``mf`` the
TDA drivers consume (the reference runs ``dft.ROKS(mol)`` / ``dft.UKS(mol)``
with ``mf.irrep_nelec``, ``mf.xc = 'bhandhlyp'``, ``mf.kernel()``,
``example/XSF_TDA.ipynb`` cells 1 and 5).

Conventions kept from PySCF because the TDA operators read them:

* ROKS energy = UKS energy functional of (D_a, D_b) built from ROHF orbitals;
  orbitals from Roothaan's effective Fock (PySCF ``rohf.get_roothaan_fock``),
  ``mo_energy`` = its eigenvalues, ``mo_occ`` in {2, 1, 0}, orbitals sorted
  core | open | virtual after convergence (``rohf_symm._finalize``).
* Occupations: aufbau with PySCF's ROHF rule (core by Roothaan energy, open
  shells by alpha energy) or, with ``irrep_nelec = {irrep: (n_a, n_b)}``, the
  same rule inside each C2v irrep (``mol.ao_irreps``).
* Energy pieces as PySCF prints them: E1 = sum_s tr(D_s h), Ecoul =
  tr(D J)/2, Exc = E_xc[DFT] - hyb/2 sum_s tr(D_s K_s) (``uks.get_veff``); a
  range-separated hybrid (CAM-B3LYP) adds (alpha - hyb) K_LR[D] to hyb K[D], K_LR
  from the erf(omega r12)/r12 ERIs of the same route (stored, DF or the device
  Cholesky factor), as ``rks.get_veff`` does with ``get_k(omega=omega)``.

Convergence: Pulay DIIS on (effective) Fock matrices, stop when |dE| <
``conv_tol`` and the orbital-rotation gradient norm < ``conv_tol_grad``.
"""
from __future__ import annotations

import dataclasses

import numpy as np
import scipy.linalg

from . import xc as _xc
from .grid import gen_grids
from .gto import C2V_IRREPS

XC_BLOCK = 16384
INCORE_MAX_NAO = 200      # eri_mode 'auto' on a GPU: stored ERIs up to this size, Cholesky above


class _SCFBase:
    restricted_open = True

    def __init__(self, mol, xc: str = "HF"):
        self.mol = mol
        self.xc = xc
        self.irrep_nelec = None
        self.conv_tol = 1e-10
        self.conv_tol_grad = None
        self.max_cycle = 100
        self.diis_space = 8
        self.grids = None
        self.verbose = 0
        self.converged = False
        self.e_tot = 0.0
        self.scf_summary = {}
        self.mo_coeff = self.mo_occ = self.mo_energy = None
        self.with_df = None
        self.eri_mode = "auto"          # 'incore' | 'cholesky' | 'auto' (see build)
        self.chol_tol = 1e-12
        self.cderi_exact = None
        self.cderi_exact_lr = None
        self.eri_lr = None
        self.timings = {}
        self.device_engine = None
        self._device = None
        self._built = False

    def to_device(self, device: int = 0):
        """Evaluate J/K and XC (and the cached TDA kernels) on the GPU through the
        library's GEMM engine (``qc.device.DeviceEngine``)."""
        self._device = device
        self.device_engine = None
        self._built = False
        df = getattr(self, "with_df", None)
        if df is not None and df._cderi is None:
            df.device = device          # the 3-index integrals on the same GPU
        return self

    def density_fit(self, auxbasis=None):
        """J/K from a 3-index factor instead of the 4-index ERIs (PySCF
        ``mf.density_fit()``; the reference's DF mean fields, XTDA.py:518-543).
        ``auxbasis``: {element: shells} or None for the even-tempered default."""
        from .df import DF
        self.with_df = DF(self.mol, auxbasis, device=getattr(self, "_device", None))
        self._built = False
        return self

    def cholesky(self, tol: float = 1e-12):
        """Exact J/K from the integral-direct pivoted Cholesky factor of the ERIs,
        computed on the GPU without the 4-index array (``qc.dchol``; the direct-SCF
        mean field the reference defaults to, XTDA.py:518-543).  Needs to_device()."""
        self.eri_mode = "cholesky"
        self.chol_tol = float(tol)
        self._built = False
        return self

    def _use_cholesky(self):
        if self.with_df is not None:
            return False
        if self.eri_mode == "cholesky":
            if self._device is None:
                raise ValueError("the integral-direct Cholesky factor is computed on the GPU: call to_device() first")
            return True
        return self.eri_mode == "auto" and self._device is not None and self.mol.nao > INCORE_MAX_NAO

    # ----------------------------------------------------------- set-up
    def build(self):
        if self._built:
            return self
        import time
        mol = self.mol
        dev = getattr(self, "_device", None)
        self.comps, self.hyb, self.xctype = _xc.parse_xc(self.xc)
        self.omega, self.alpha = _xc.rsh_and_hybrid_coeff(self.xc)[:2] if self.xctype != "HF" else (0.0, 1.0)
        t0 = time.perf_counter()
        self.s1e = mol.intor("int1e_ovlp")
        self.h1e = mol.intor("int1e_kin") + mol.intor("int1e_nuc", device=dev)
        self.timings["int1e_s"] = time.perf_counter() - t0
        self.eri = self.eri_lr = None
        self._eri_k = self._eri_k_lr = None
        self.cderi_exact = self.cderi_exact_lr = None
        t0 = time.perf_counter()
        rsh = self.omega != 0
        if self._use_cholesky():
            from .dchol import cholesky_eri
            st = {}
            self.cderi_exact = cholesky_eri(mol, self.chol_tol, dev, stats=st)
            self.timings["cholesky"] = st
            if rsh:
                self.cderi_exact_lr = cholesky_eri(mol, self.chol_tol, dev, omega=self.omega)
        elif self.with_df is None:
            self.eri = mol.eri_full(device=dev)
            if rsh:
                self.eri_lr = mol.eri_full(device=dev, omega=self.omega)
        else:
            self.with_df.build()
            if rsh:
                self.with_df.cderi_lr(self.omega)
        self.timings["int2e_s"] = time.perf_counter() - t0
        if self.xctype != "HF":
            t0 = time.perf_counter()
            if self.grids is None:
                self.grids = gen_grids(mol, device=dev)
            self.timings["grid_s"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            self.ao = mol.eval_ao(self.grids.coords, deriv=1 if self.xctype in ("GGA", "MGGA") else 0,
                                  device=dev)
            if self.ao.ndim == 2:
                self.ao = self.ao[None]
            if dev is not None:
                import torch
                torch.cuda.synchronize(dev)
            self.timings["eval_ao_s"] = time.perf_counter() - t0
        if self._device is not None:
            from .device import DeviceEngine
            self.device_engine = DeviceEngine(self, self._device)
        if mol.symmetry is not None:
            self.ao_irrep = mol.ao_irreps()
        else:
            self.ao_irrep = np.zeros(mol.nao, dtype=np.int64)
        self._built = True
        return self

    def get_hcore(self):
        return self.h1e

    def get_ovlp(self):
        return self.s1e

    def energy_nuc(self):
        return self.mol.energy_nuc()

    # -------------------------------------------------------- potentials
    def _factored(self, dms, factors):
        """dms built as C_s C_s^T from orbitals: remember the factors for the device
        exchange (K[D] = sum_P (B_P C)(B_P C)^T, no eigendecomposition of D)."""
        self._dm_factors = (dms, factors, float(np.sum(dms)))
        return dms

    def _factors_of(self, dm):
        """The factors of exactly that density array, unless it was changed in place since."""
        f = getattr(self, "_dm_factors", None)
        return f[1] if f is not None and f[0] is dm and float(np.sum(dm)) == f[2] else None

    def get_jk(self, mol=None, dm=None, hermi=1, with_j=True, with_k=True):
        """PySCF incore convention: vj = (ij|kl) D_kl, vk = (ij|kl) D_jk -> [i,l]."""
        if self.device_engine is not None:
            return self.device_engine.get_jk(dm, with_j, with_k, factors=self._factors_of(dm))
        if self.with_df is not None:
            return self.with_df.get_jk(dm, with_j, with_k)
        d = np.asarray(dm, dtype=np.float64)
        shape = d.shape
        n = shape[-1]
        d = d.reshape(-1, n * n)
        eri = self.eri.reshape(n * n, n * n)
        vj = (eri @ d.T).T.reshape(shape) if with_j else None
        vk = None
        if with_k:
            if getattr(self, "_eri_k", None) is None:
                self._eri_k = np.ascontiguousarray(self.eri.transpose(0, 3, 1, 2)).reshape(n * n, n * n)
            vk = (self._eri_k @ d.T).T.reshape(shape)
        return vj, vk

    def get_k_lr(self, dm):
        """Long-range exchange K_LR[D] with the erf(omega r12)/r12 operator
        (``mf.get_k(mol, dm, hermi, omega=omega)``, XTDA.py:534-539)."""
        if self.omega == 0:
            raise ValueError(f"{self.xc} is not range-separated")
        if self.device_engine is not None:
            return self.device_engine.get_k(dm, lr=True, factors=self._factors_of(dm))
        if self.with_df is not None:
            return self.with_df.get_k_lr(dm, self.omega)
        d = np.asarray(dm, dtype=np.float64)
        shape = d.shape
        n = shape[-1]
        if self._eri_k_lr is None:
            self._eri_k_lr = np.ascontiguousarray(self.eri_lr.transpose(0, 3, 1, 2)).reshape(n * n, n * n)
        return (self._eri_k_lr @ d.reshape(-1, n * n).T).T.reshape(shape)

    def _rho(self, dm):
        """rho (4, ngrid) (or (1, ngrid); MGGA (5, ngrid) with tau = 1/2 sum_c
        grad_c phi D grad_c phi) of a symmetric density matrix."""
        ao = self.ao
        c0 = ao[0] @ dm
        nc = 5 if self.xctype == "MGGA" else ao.shape[0]
        rho = np.empty((nc, ao.shape[1]))
        rho[0] = np.einsum('gp,gp->g', ao[0], c0)
        for k in range(1, ao.shape[0]):
            rho[k] = 2.0 * np.einsum('gp,gp->g', ao[k], c0)
        if nc == 5:
            rho[4] = 0.5 * sum(np.einsum('gp,gp->g', ao[k], ao[k] @ dm) for k in range(1, 4))
        return rho

    def _vxc(self, dms):
        """(E_xc[DFT], V_xc (2, nao, nao)) at spin densities dms."""
        if self.device_engine is not None:
            return self.device_engine.vxc(dms)
        nao = dms.shape[-1]
        vmat = np.zeros((2, nao, nao))
        exc_tot = 0.0
        ng = self.grids.size
        for g0 in range(0, ng, XC_BLOCK):
            g1 = min(ng, g0 + XC_BLOCK)
            ao = self.ao[:, g0:g1]
            w = self.grids.weights[g0:g1]
            saved, self.ao = self.ao, ao
            rho = np.asarray([self._rho(dms[0]), self._rho(dms[1])])
            self.ao = saved
            exc, vxc, _ = _xc.eval_xc_eff(self.xc, rho, deriv=1)
            exc_tot += float(np.sum(w * exc * (rho[0, 0] + rho[1, 0])))
            for s in range(2):
                wv = vxc[s] * w
                if self.xctype in ("GGA", "MGGA"):
                    wv[0] *= 0.5
                    aow = np.einsum('yg,ygp->gp', wv[:4], ao[:4])
                    v = ao[0].T @ aow
                    vmat[s] += v + v.T
                    if self.xctype == "MGGA":    # tau part: 1/2 sum_c grad_c phi^T w_tau grad_c phi
                        for k in range(1, 4):
                            vmat[s] += 0.5 * ao[k].T @ (wv[4][:, None] * ao[k])
                else:
                    vmat[s] += ao[0].T @ (wv[0][:, None] * ao[0])
        return exc_tot, vmat

    def get_veff(self, mol=None, dm=None):
        """KS (or HF) potential per spin and the energy pieces (ecoul, exc)."""
        dms = np.asarray(dm)
        vj, vk = self.get_jk(dm=dms)
        vj = vj[0] + vj[1]
        if self.xctype == "HF":
            veff = vj[None] - vk
            exc = -0.5 * (np.sum(dms[0] * vk[0]) + np.sum(dms[1] * vk[1]))
        else:
            exc, vxc = self._vxc(dms)
            veff = vxc + vj[None]
            if self.omega != 0:     # hyb K + (alpha - hyb) K_LR (XTDA.py:537-539)
                vk = self.hyb * vk + (self.alpha - self.hyb) * self.get_k_lr(dms)
                veff = veff - vk
                exc -= 0.5 * (np.sum(dms[0] * vk[0]) + np.sum(dms[1] * vk[1]))
            elif self.hyb != 0:
                veff = veff - self.hyb * vk
                exc -= 0.5 * self.hyb * (np.sum(dms[0] * vk[0]) + np.sum(dms[1] * vk[1]))
        ecoul = 0.5 * np.sum((dms[0] + dms[1]) * vj)
        return veff, float(ecoul), float(exc)

    def get_veff_hf(self, dm):
        """Pure-HF potential J - K at dm (``scf.ROHF(mol).get_veff``, XTDA.py:608-612)."""
        vj, vk = self.get_jk(dm=np.asarray(dm))
        return (vj[0] + vj[1])[None] - vk

    def energy_elec(self, dms, veff_parts):
        _, ecoul, exc = veff_parts
        e1 = float(np.sum(dms[0] * self.h1e) + np.sum(dms[1] * self.h1e))
        return e1 + ecoul + exc, e1, ecoul, exc

    # ----------------------------------------------------- diagonalisation
    def _eig_sym(self, f):
        """Generalised eigenproblem per irrep; returns (e, C, irrep labels) sorted by e."""
        n = f.shape[0]
        es, cs, labels = [], [], []
        for ir in np.unique(self.ao_irrep):
            idx = np.where(self.ao_irrep == ir)[0]
            e, c = scipy.linalg.eigh(f[np.ix_(idx, idx)], self.s1e[np.ix_(idx, idx)])
            full = np.zeros((n, idx.size))
            full[idx] = c
            es.append(e)
            cs.append(full)
            labels.append(np.full(idx.size, ir))
        e = np.concatenate(es)
        c = np.concatenate(cs, axis=1)
        lab = np.concatenate(labels)
        order = np.argsort(e, kind="stable")
        return e[order], c[:, order], lab[order]

    def _irrep_counts(self):
        """{irrep index: (n_a, n_b)} or None."""
        if self.irrep_nelec is None:
            return None
        if self.mol.symmetry is None:
            raise ValueError("irrep_nelec needs mol.symmetry")
        out = {}
        na = nb = 0
        for name, n in self.irrep_nelec.items():
            ir = C2V_IRREPS.index(name)
            if np.isscalar(n):
                raise ValueError("irrep_nelec entries must be (n_alpha, n_beta)")
            out[ir] = (int(n[0]), int(n[1]))
            na += int(n[0])
            nb += int(n[1])
        if (na, nb) != tuple(self.mol.nelec):
            raise ValueError(f"irrep_nelec gives {(na, nb)} electrons, mol has {self.mol.nelec}")
        return out


class ROHF(_SCFBase):
    """Restricted open-shell HF; ``ROKS`` sets a functional."""

    def __init__(self, mol, xc: str = "HF"):
        super().__init__(mol, xc)

    @staticmethod
    def get_roothaan_fock(fa, fb, dma, dmb, s):
        fc = 0.5 * (fa + fb)
        n = s.shape[0]
        pc = dmb @ s
        po = (dma - dmb) @ s
        pv = np.eye(n) - dma @ s
        f = 0.5 * (pc.T @ fc @ pc) + 0.5 * (po.T @ fc @ po) + 0.5 * (pv.T @ fc @ pv)
        f += po.T @ fb @ pc
        f += po.T @ fa @ pv
        f += pv.T @ fc @ pc
        return f + f.T

    def _occ(self, e, c, lab, fa):
        """ROHF occupations: core by Roothaan energy, open shells by alpha energy."""
        ea = np.sum(c * (fa @ c), axis=0)              # diag(C^T F_a C) by one GEMM
        occ = np.zeros(e.size)
        counts = self._irrep_counts()
        groups = ([(np.arange(e.size), self.mol.nelec)] if counts is None else
                  [(np.where(lab == ir)[0], nab) for ir, nab in counts.items()])
        for idx, (na, nb) in groups:
            core = idx[np.argsort(e[idx], kind="stable")[:nb]]
            rest = np.setdiff1d(idx, core)
            opn = rest[np.argsort(ea[rest], kind="stable")[:na - nb]]
            occ[core] = 2
            occ[opn] = 1
        return occ

    def _dms(self, c, occ):
        ca = c[:, occ >= 1]
        cb = c[:, occ >= 2]
        return self._factored(np.asarray([ca @ ca.T, cb @ cb.T]), [ca, cb])

    def _grad(self, c, occ, fa, fb):
        fam = c.T @ fa @ c
        fbm = c.T @ fb @ c
        occa, occb = occ >= 1, occ >= 2
        g = np.zeros_like(fam)
        g[np.ix_(~occa, occa)] += fam[np.ix_(~occa, occa)]
        g[np.ix_(~occb, occb)] += fbm[np.ix_(~occb, occb)]
        return g

    def kernel(self, dm0=None):
        self.build()
        s = self.s1e
        tol_grad = self.conv_tol_grad or np.sqrt(self.conv_tol)
        if dm0 is None:
            e, c, lab = self._eig_sym(self.h1e)
            occ = self._occ(e, c, lab, self.h1e)
            dms = self._dms(c, occ)
        else:
            dms = np.asarray(dm0)
        diis_f, diis_e = [], []
        e_last = None
        for cycle in range(self.max_cycle):
            parts = self.get_veff(dm=dms)
            fa, fb = self.h1e + parts[0][0], self.h1e + parts[0][1]
            e_tot = self.energy_elec(dms, parts)[0] + self.energy_nuc()
            f = self.get_roothaan_fock(fa, fb, dms[0], dms[1], s)
            dt = dms[0] + dms[1]
            err = f @ dt @ s - s @ dt @ f
            diis_f.append(f)
            diis_e.append(err)
            diis_f, diis_e = diis_f[-self.diis_space:], diis_e[-self.diis_space:]
            f_use = _diis(diis_f, diis_e) if cycle >= 1 else f
            e, c, lab = self._eig_sym(f_use)
            occ = self._occ(e, c, lab, fa)
            gnorm = np.linalg.norm(self._grad(c, occ, fa, fb)) if cycle else np.inf
            dms_new = self._dms(c, occ)
            if self.verbose:
                print(f"cycle {cycle} E= {e_tot:.12f} |g|= {gnorm:.2e}")
            if e_last is not None and abs(e_tot - e_last) < self.conv_tol and gnorm < tol_grad:
                self.converged = True
                dms = dms_new
                break
            e_last = e_tot
            dms = dms_new
        self._finalize(dms)
        return self.e_tot

    def _finalize(self, dms):
        """One more Fock build at the final density; canonical orbitals core|open|virtual."""
        parts = self.get_veff(dm=dms)
        fa, fb = self.h1e + parts[0][0], self.h1e + parts[0][1]
        f = self.get_roothaan_fock(fa, fb, dms[0], dms[1], self.s1e)
        e, c, lab = self._eig_sym(f)
        occ = self._occ(e, c, lab, fa)
        order = np.concatenate([np.where(occ == 2)[0], np.where(occ == 1)[0], np.where(occ == 0)[0]])
        self.mo_energy, self.mo_coeff, self.mo_occ = e[order], c[:, order], occ[order]
        self.orbsym = lab[order]
        dms = self._dms(self.mo_coeff, self.mo_occ)
        parts = self.get_veff(dm=dms)
        etot, e1, ecoul, exc = self.energy_elec(dms, parts)
        self.e_tot = etot + self.energy_nuc()
        self.scf_summary = dict(e1=e1, coul=ecoul, exc=exc, nuc=self.energy_nuc())
        self._veff = parts[0]
        self._dm = dms

    def make_rdm1(self):
        return self._dm.copy()

    def to_meanfield(self, chol_tol: float = 1e-14):
        return _meanfield(self, chol_tol)


class UHF(_SCFBase):
    """Unrestricted HF; ``UKS`` sets a functional."""
    restricted_open = False

    def __init__(self, mol, xc: str = "HF"):
        super().__init__(mol, xc)

    def _occ(self, es, labs):
        counts = self._irrep_counts()
        occ = np.zeros((2, es[0].size))
        for s in range(2):
            if counts is None:
                occ[s][np.argsort(es[s], kind="stable")[:self.mol.nelec[s]]] = 1
            else:
                for ir, nab in counts.items():
                    idx = np.where(labs[s] == ir)[0]
                    occ[s][idx[np.argsort(es[s][idx], kind="stable")[:nab[s]]]] = 1
        return occ

    def _uhf_dms(self, cs, occ):
        f = [cs[t][:, occ[t] > 0] for t in range(2)]
        return self._factored(np.asarray([f[t] @ f[t].T for t in range(2)]), f)

    def kernel(self, dm0=None):
        self.build()
        s = self.s1e
        tol_grad = self.conv_tol_grad or np.sqrt(self.conv_tol)
        if dm0 is None:
            e, c, lab = self._eig_sym(self.h1e)
            occ = self._occ((e, e), (lab, lab))
            cs = (c, c)
        else:
            cs = None
        dms = (self._uhf_dms(cs, occ) if dm0 is None else np.asarray(dm0))
        diis_f, diis_e = [], []
        e_last = None
        for cycle in range(self.max_cycle):
            parts = self.get_veff(dm=dms)
            f = self.h1e[None] + parts[0]
            e_tot = self.energy_elec(dms, parts)[0] + self.energy_nuc()
            err = np.asarray([f[t] @ dms[t] @ s - s @ dms[t] @ f[t] for t in range(2)])
            diis_f.append(f)
            diis_e.append(err)
            diis_f, diis_e = diis_f[-self.diis_space:], diis_e[-self.diis_space:]
            f_use = _diis(diis_f, diis_e) if cycle >= 1 else f
            res = [self._eig_sym(f_use[t]) for t in range(2)]
            occ = self._occ((res[0][0], res[1][0]), (res[0][2], res[1][2]))
            gnorm = np.inf
            if cycle:
                g = 0.0
                for t in range(2):
                    ct = res[t][1]
                    fm = ct.T @ f[t] @ ct
                    o = occ[t] > 0
                    g += np.sum(fm[np.ix_(~o, o)] ** 2)
                gnorm = np.sqrt(g)
            dms_new = self._uhf_dms([res[0][1], res[1][1]], occ)
            if self.verbose:
                print(f"cycle {cycle} E= {e_tot:.12f} |g|= {gnorm:.2e}")
            if e_last is not None and abs(e_tot - e_last) < self.conv_tol and gnorm < tol_grad:
                self.converged = True
                dms = dms_new
                break
            e_last = e_tot
            dms = dms_new
        self._finalize(dms)
        return self.e_tot

    def _finalize(self, dms):
        parts = self.get_veff(dm=dms)
        f = self.h1e[None] + parts[0]
        res = [self._eig_sym(f[t]) for t in range(2)]
        occ = self._occ((res[0][0], res[1][0]), (res[0][2], res[1][2]))
        mo_e, mo_c, mo_o, sym = [], [], [], []
        for t in range(2):
            e, c, lab = res[t]
            order = np.concatenate([np.where(occ[t] > 0)[0], np.where(occ[t] == 0)[0]])
            mo_e.append(e[order])
            mo_c.append(c[:, order])
            mo_o.append(occ[t][order])
            sym.append(lab[order])
        self.mo_energy = np.asarray(mo_e)
        self.mo_coeff = np.asarray(mo_c)
        self.mo_occ = np.asarray(mo_o)
        self.orbsym = np.asarray(sym)
        dms = np.asarray([self.mo_coeff[t][:, self.mo_occ[t] > 0] @ self.mo_coeff[t][:, self.mo_occ[t] > 0].T
                          for t in range(2)])
        parts = self.get_veff(dm=dms)
        etot, e1, ecoul, exc = self.energy_elec(dms, parts)
        self.e_tot = etot + self.energy_nuc()
        self.scf_summary = dict(e1=e1, coul=ecoul, exc=exc, nuc=self.energy_nuc())
        self._veff = parts[0]
        self._dm = dms

    def make_rdm1(self):
        return self._dm.copy()

    def spin_square(self):
        """<S^2> and 2S+1 of the UHF/UKS determinant (PySCF ``uhf.spin_square``)."""
        ca = self.mo_coeff[0][:, self.mo_occ[0] > 0]
        cb = self.mo_coeff[1][:, self.mo_occ[1] > 0]
        na, nb = ca.shape[1], cb.shape[1]
        ovl = ca.T @ self.s1e @ cb
        ssxy = (na + nb) * 0.5 - np.sum(ovl ** 2)
        ssz = 0.25 * (na - nb) ** 2
        ss = ssxy + ssz
        return ss, 2 * np.sqrt(ss + 0.25)

    def to_meanfield(self, chol_tol: float = 1e-14):
        return _meanfield(self, chol_tol)


def ROKS(mol, xc: str = "LDA"):
    """``dft.ROKS(mol)``; set ``.xc`` before ``kernel()`` (default kept as PySCF's 'LDA,VWN'
    is not implemented: pass the functional explicitly)."""
    return ROHF(mol, xc)


def UKS(mol, xc: str = "LDA"):
    return UHF(mol, xc)


def _diis(fs, errs):
    n = len(fs)
    B = np.empty((n + 1, n + 1))
    B[-1, :] = B[:, -1] = -1.0
    B[-1, -1] = 0.0
    for i in range(n):
        for j in range(i + 1):
            B[i, j] = B[j, i] = float(np.sum(errs[i] * errs[j]))
    rhs = np.zeros(n + 1)
    rhs[-1] = -1.0
    try:
        c = np.linalg.solve(B, rhs)[:n]
    except np.linalg.LinAlgError:
        c = np.linalg.lstsq(B, rhs, rcond=None)[0][:n]
    return sum(ci * fi for ci, fi in zip(c, fs))


# ------------------------------------------------------------ MeanField
def pivoted_cholesky(m: np.ndarray, tol: float):
    """Rows L (naux, n) with L^T L ~ m for a PSD matrix m (stops at diag < tol)."""
    n = m.shape[0]
    d = np.diag(m).copy()
    vecs = []
    for _ in range(n):
        p = int(np.argmax(d))
        if d[p] <= tol:
            break
        v = m[:, p].copy()
        for u in vecs:
            v -= u * u[p]
        v /= np.sqrt(d[p])
        vecs.append(v)
        d -= v * v
    return np.asarray(vecs)


def _meanfield(mf, chol_tol):
    """Package a converged SCF as the ``MeanField`` the TDA operators read.

    Contents mirror what the reference pulls out of PySCF's ``mf``:
    ``get_veff`` at the SCF density (XTDA.py:588-590), the pure-HF potential
    (XTDA.py:608-612, XSF_TDA.py:1104-1114), the incore ERIs (jk_mode ERI8,
    8-fold packed) and their exact Cholesky factor (cderi; the oracle's J/K
    engine), the grid with AO values/gradients, the UKS ``fxc`` of
    ``cache_xc_kernel`` (XTDA.py:504) and the ALDA0 ``fxc_ab`` of
    ``cache_xc_kernel_sf`` (SF_TDA.py:39-88).
    """
    from ..eri import pack_s8
    from ..meanfield import Grid, MeanField, Mole as MFMole
    if mf.mo_coeff is None:
        raise RuntimeError("run kernel() first")
    mol = mf.mol
    nao = mol.nao
    dms = mf._dm
    omega, alpha, hyb = (0.0, 0.0, 1.0) if mf.xctype == "HF" else _xc.rsh_and_hybrid_coeff(mf.xc)
    eri8_lr = cderi_lr = None
    if mf.with_df is not None:      # DF mean field: the fitted factor, no 4-index ERIs
        eri8 = None
        cderi = mf.with_df.cderi
        if omega != 0:
            cderi_lr = mf.with_df.cderi_lr(omega)
    elif mf.cderi_exact is not None:   # integral-direct Cholesky: the exact factor, on the device
        eri8 = None
        cderi = mf.cderi_exact
        cderi_lr = mf.cderi_exact_lr
    else:
        eri8 = pack_s8(mf.eri)
        cderi = pivoted_cholesky(mf.eri.reshape(nao * nao, nao * nao), chol_tol).reshape(-1, nao, nao)
        if omega != 0:
            eri8_lr = pack_s8(mf.eri_lr)
            cderi_lr = pivoted_cholesky(mf.eri_lr.reshape(nao * nao, nao * nao), chol_tol).reshape(-1, nao, nao)
    veff_hf = mf.get_veff_hf(dms)
    grids = fxc = fxc_sf = None
    if mf.xctype != "HF":
        ao = mf.ao
        w = mf.grids.weights
        if mf.device_engine is not None:
            fxc, fxc_sf = mf.device_engine.kernels(dms)
        else:
            rho = np.asarray([mf._rho(dms[0]), mf._rho(dms[1])])
            fxc = _xc.eval_xc_eff(mf.xc, rho, deriv=2)[2]
            # ALDA0 (SF_TDA.py:69-85): density-only rho, vxc weighted, divided by rho_a - rho_b + 1e-9
            rho0 = np.zeros_like(rho)
            rho0[:, 0] = rho[:, 0]
            vxc0 = _xc.eval_xc_eff(mf.xc, rho0, deriv=1)[1]
            fxc_sf = (vxc0[0, 0] * w - vxc0[1, 0] * w) / (rho[0, 0] - rho[1, 0] + 1e-9)
        grids = Grid(ao=ao if _is_tensor(ao) else np.ascontiguousarray(ao), weights=np.ascontiguousarray(w))
    mfmol = MFMole(nao=nao, spin=mol.spin, nelectron=mol.nelectron, symmetry=mol.symmetry is not None)
    out = MeanField(mol=mfmol, mo_coeff=mf.mo_coeff, mo_occ=mf.mo_occ, mo_energy=mf.mo_energy,
                    h1e=mf.h1e, veff=np.asarray(mf._veff), veff_hf=np.asarray(veff_hf),
                    cderi=cderi, grids=grids, fxc=fxc, fxc_sf=fxc_sf, xc=mf.xc,
                    xctype=mf.xctype, omega=omega, alpha=alpha, hyb=hyb, eri=eri8,
                    cderi_lr=cderi_lr, eri_lr=eri8_lr, e_tot=mf.e_tot)
    out.extra.update(dict(s1e=mf.s1e, orbsym=getattr(mf, "orbsym", None), qc_mol=mol))
    if not mf.restricted_open:
        out.extra["spin_square"] = mf.spin_square()
    return out


def _is_tensor(x):
    return type(x).__module__.startswith("torch")


def as_device_eri8(mfield):
    """The same MeanField in jk_mode 'ERI8' (device factorises the stored ERIs)."""
    return dataclasses.replace(mfield, cderi=None)
