"""Spin-adapted spin-flip TDA (XSF-TDA) with the reference's API
(``xtddft/XSF_TDA.py``).

``XSF_TDA(mf, SA=None, davidson=True, method=0, collinear_samples=60,
calculate_sp=False)`` (XSF_TDA.py:146-213) and
``kernel(nstates=1, remove=None, frozen=None, foo=1.0, d_lda=0.3,
fglobal=None, fit=True)`` -> ``(e * 27.21138505, v)`` (XSF_TDA.py:1501-1554).

* ``gen_tda_operation_sf(foo, fglobal)`` -> ``(vind, hdiag)`` (1029-1277):
  the device operator (SF-down response + Fock + Delta-A of level ``SA``)
  on cv|co|ov|oo vectors, OO compressed when ``remove``.
* the preconditioner (915-961) takes its J diagonals from the device:
  ``co_j[i,u] = sum_P B[P,i,u]^2`` -- one pass over the MO DF factor instead
  of the reference's (nc*no + no*nv) unit-density J builds (859-913).
* ``davidson_process`` uses the reference criteria tol 1e-8, lindep 1e-9,
  max_cycle 1000 (1467-1470) on the device solver.
* ``method``: 0 ALDA0, 1 multicollinear (``collinear_samples`` Gauss-Legendre samples,
  ``xtddft_amd.mcol``; fglobal fitted by 4 (cx - 1/2)^2, XSF_TDA.py:1517-1518), 2 collinear.
* ``calculate_sp=True`` runs ``get_sp`` (XSF_TDA.py:215-262): the spin-polarisation
  integrals of a triplet reference, <LH|HL> and <iH|Ha>, <iL|La>, as elements of the
  device operator's response to the unit H->H / L->L spin flips.
* ``kernel(frozen=...)`` drops frozen core orbitals from the explicit matrix
  (``frozen_A``, XSF_TDA.py:1483-1499, 1544-1545: davidson=False without OO removal).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg

from . import davidson as _dav
from .meanfield import MeanField
from .parallel import require_group
from .sf_tda import _check_method, _dense, mf_info, sf_operator
from .utils import HA2EV_XSF, nlc_check


def get_vect(no):
    """OO compression basis vects (no^2, no^2-1) (XSF_TDA.py:397-414)."""
    tmp_v = np.zeros((no - 1, no))
    for i in range(1, no):
        factor = 1 / np.sqrt((no - i + 1) * (no - i))
        tmp_v[i - 1][i - 1:] = np.array([no - i] + [-1] * (no - i)) * factor
    vect = tmp_v.T
    vects = np.eye(no * no)[:, :-1]
    index = [0] + [i * (no + 1) for i in range(1, no)]
    for i in range(vect.shape[1]):
        vects[0::no + 1, index[i]] = vect[:, i]
    return vects


def split_xsf_vector(value, nc, no, nv, vects=None):
    """cv (nc,nv), co (nc,no), ov (no,nv), oo (no,no) blocks of one XSF vector in
    the reference's order; a compressed OO block is expanded with ``vects``
    (XSF_TDA.py:728-734)."""
    d1, d2, d3 = nc * nv, nc * nv + nc * no, nc * nv + nc * no + no * nv
    oo = value[d3:]
    oo = (vects @ oo).reshape(no, no) if vects is not None else oo.reshape(no, no)
    return (value[:d1].reshape(nc, nv), value[d1:d2].reshape(nc, no),
            value[d2:d3].reshape(no, nv), oo)


def delta_s2_u(mf, value, nc, no, nv):
    """XSF_TDA.deltaS2_U (XSF_TDA.py:613-649): the <S^2> term P_ab of a spin-flip
    vector on a UKS reference, from the alpha/beta MO overlaps."""
    mo, occ = mf.mo_coeff, mf.mo_occ
    s = mf.get_ovlp()
    mooa = mo[0][:, occ[0] > 0]
    moob = mo[1][:, occ[1] > 0]
    movb = mo[1][:, occ[1] == 0]
    sba_oo = moob.T @ s @ mooa
    sba_vo = movb.T @ s @ mooa
    cv, co, ov, oo = split_xsf_vector(value, nc, no, nv)
    x_ba = np.vstack([np.hstack([co, cv]), np.hstack([oo, ov])]).T    # (no+nv, nc+no)
    t1 = np.einsum('ai,aj,jk,ki->', x_ba, x_ba, sba_oo.T, sba_oo)
    t2 = np.einsum('ai,bi,kb,ak->', x_ba, x_ba, sba_vo.T, sba_vo)
    t3 = np.einsum('ai,ai->', x_ba, sba_vo) ** 2
    return t1 - t2 + t3


class XSF_TDA:
    def __init__(self, mf: MeanField, SA=None, davidson=True, method=0, collinear_samples=60,
                 calculate_sp=False, device=0, shard=(0, 1)):
        _check_method(method)
        self.mf = mf
        self.type_u = not mf.is_rohf
        self.SA = (0 if self.type_u else 3) if SA is None else SA
        self.davidson = davidson
        self.method = method
        self.collinear_samples = collinear_samples
        self.device = device
        self.shard = tuple(shard)
        require_group(self.shard[1])
        nlc_check(mf)
        info = mf.shape_info()
        self.nc, self.no, self.nv = info['nc'], info['no'], info['nv']
        self.nocc_a, self.nocc_b = info['nocc_a'], info['nocc_b']
        self.mo_energy, self.mo_occ, self.mo_coeff = mf_info(mf)
        if mf.xctype == 'HF':
            self.omega, self.alpha, self.hyb = 0.0, 0.0, 1.0
        else:
            self.omega, self.alpha, self.hyb = mf.omega, mf.alpha, mf.hyb
        _, dsp1 = mf.spin_square()
        self.ground_s = (dsp1 - 1) / 2
        self.re = None
        self.calculate_sp = calculate_sp
        if calculate_sp:   # J. Chem. Theory Comput. 2023, 19, 7606-7616 (XSF_TDA.py:211-213)
            self.sp = self.get_sp()

    # ------------------------------------------------------------ helpers
    def get_sp(self, verbose=True):
        """Spin-polarisation analysis of a triplet ROKS reference (XSF_TDA.py:215-262): the
        response V[|H><H|] of the spin-flip kernel (XC of ``method`` + hybrid exchange,
        ``gen_response_sf``) at MO element (nc + no, nc + no) -- what the reference prints as
        <LH|HL> -- and the pure exchange integrals <iH|Ha> = K[|H><H|]_ia, <iL|La> =
        K[|L><L|]_ia (core i, virtual a; H, L the two open shells).  Each is read off one
        device A.x on a unit spin-flip vector: <iH|Ha>, <iL|La> from an exchange-only
        operator, the response element from one whose occupied space is widened by one
        orbital so that (nc + no, nc + no) is a spin-flip pair (the Fock terms vanish at
        all these elements).  Returns dict(lhhl, homo (nc, nv), lumo (nc, nv)) and prints
        the reference's top-10 tables."""
        import dataclasses
        from .operator import DeviceOperator
        from .sf_tda import _collinear
        if self.type_u or self.no != 2:
            raise ValueError("get_sp analyses a triplet ROKS reference (two open shells)")
        nc, no, nv = self.nc, self.no, self.nv
        mf = self.mf

        def unit(dim, nvb, i, a):   # SF-down vector in PySCF order (occ_a x vir_b)
            z = np.zeros((1, dim))
            z[0, i * nvb + a] = 1.0
            return z
        # response at (nc + no, nc + no): occupations widened by that orbital (order kept:
        # core | open | virtual), kernel and orbitals unchanged
        occ = np.array(mf.mo_occ, dtype=np.float64)
        occ[nc + no] = 1.0
        wide = dataclasses.replace(mf, mo_occ=occ)
        if self.method == 1:
            from .mcol import sf_mc_kernel
            resp = DeviceOperator(wide, "SF_DOWN", device=self.device, sf_kernel="mc",
                                  mc_kernel=sf_mc_kernel(mf, self.collinear_samples, device=self.device))
        else:
            resp = DeviceOperator(_collinear(wide) if self.method == 2 else wide, "SF_DOWN", device=self.device)
        nvb = no + 1 + nv - 1
        lhhl = float(resp.apply(unit(resp.dim, nvb, nc, 0))[0, (nc + no) * nvb + no])
        resp.close()
        kmf = dataclasses.replace(mf, xctype="HF", hyb=1.0, alpha=0.0, omega=0.0, grids=None, fxc=None,
                                  fxc_sf=None, fxc_sf_mc=None, cderi_lr=None, eri_lr=None)
        kop = DeviceOperator(kmf, "SF_DOWN", device=self.device)
        nvb = no + nv
        homo = -kop.apply(unit(kop.dim, nvb, nc, 0))[0].reshape(nc + no, nvb)[:nc, no:]
        lumo = -kop.apply(unit(kop.dim, nvb, nc + 1, 1))[0].reshape(nc + no, nvb)[:nc, no:]
        kop.close()

        def top10(m):
            idx = np.argsort(-np.abs(m), axis=None)[:10]
            return [(float(m.flat[k]),) + tuple(int(t) for t in np.unravel_index(k, m.shape)) for k in idx]
        lines = ["=================================================", f"<LH|HL> is {lhhl:9.6f}"]
        for title, m in (("<iH|Ha>", homo), ("<iL|La>", lumo), ("<iH|Ha>-<iL|La>", homo - lumo),
                         ("<iH|Ha>*<iL|La>", homo * lumo)):
            lines.append(f"Top 10 value in {title}:")
            for n, (v, i, a) in enumerate(top10(m)):
                lines.append(f"{n + 1} {v:9.6f}, CV is {(i + 1, a + nc + no + 1)}")
        lines.append("=================================================")
        if verbose:
            print("\n".join(lines))
        return dict(lhhl=lhhl, homo=homo, lumo=lumo, lines=lines)

    def frozen_A(self, frozen):
        """Drop frozen core orbitals from the un-compressed cv|co|ov|oo matrix
        (XSF_TDA.py:1483-1499): ``frozen=True`` drops the innermost core orbital, an
        integer n > 0 the n innermost (the reference's integer branch reads ``f`` before
        assigning it; n is what it means)."""
        f = frozen if (isinstance(frozen, (int, np.integer)) and not isinstance(frozen, bool)
                       and frozen > 0) else 1
        nc, no, nv = self.nc, self.no, self.nv
        if f > nc:
            raise ValueError(f"cannot freeze {f} of {nc} core orbitals")
        minus_cv = self.A[f * nv:, f * nv:]
        dim = minus_cv.shape[0]
        kept = np.r_[0:(nc - f) * nv, (nc - f) * nv + f * no:dim]
        return minus_cv[np.ix_(kept, kept)]

    def get_vect(self):
        return get_vect(self.no)

    def default_fglobal(self, d_lda=0.3, fit=True):
        cx = self.hyb if self.omega == 0 else self.hyb + (self.alpha - self.hyb) * math.erf(self.omega)
        f = (1 - d_lda) * cx + d_lda
        if self.method == 1 and fit:
            f = f * 4 * (cx - 0.5) ** 2
        return f

    def _operator(self, foo, fglobal):
        # method 1: the multicollinear response (XSF_TDA.py:1097-1098) with collinear_samples
        op = sf_operator(self.mf, 'XSF', self.method, self.collinear_samples, device=self.device,
                         shard=self.shard, sa=self.SA, foo=foo, fglobal=fglobal, remove=bool(self.re))
        if self.re:
            op.set_oo_basis(self.vects)
        return op

    def _build_preconditioner_hdiag(self, fglobal, op):
        mf = self.mf
        fockA, fockB = mf.fock_mo()
        nc, no = self.nc, self.no
        si = no / 2.0
        hdiag = fockB.diagonal()[self.nocc_b:][None, :] - fockA.diagonal()[:self.nocc_a, None]
        if self.SA > 0:
            fa_hf, fb_hf = mf.fock_mo_hf()
            diag_s = ((fb_hf - fa_hf) * 0.5).diagonal()
            co_j, ov_j = op.xsf_j_diagonals()
            hdiag[:nc, no:] += fglobal * (diag_s[nc + no:] + diag_s[:nc, None]) / si
            hdiag[:nc, :no] += fglobal * (2.0 * diag_s[:nc, None] - co_j) / (2 * si - 1)
            hdiag[nc:, no:] += fglobal * (2.0 * diag_s[nc + no:] - ov_j) / (2 * si - 1)
        return np.hstack([hdiag[:nc, no:].ravel(), hdiag[:nc, :no].ravel(),
                          hdiag[nc:, no:].ravel(), hdiag[nc:, :no].ravel()])

    def _compress_removed_hdiag(self, hdiag):
        d3 = self.nc * self.nv + self.nc * self.no + self.no * self.nv
        out = np.empty(hdiag.size - 1)
        out[:d3] = hdiag[:d3]
        out[d3:] = np.einsum("x,xy,xy->y", hdiag[d3:], self.vects, self.vects)
        return out

    def gen_tda_operation_sf(self, foo=1.0, fglobal=None):
        if self.re is None:
            self.re = not self.type_u
        if self.re:
            self.vects = self.get_vect()
        if fglobal is None:
            fglobal = self.default_fglobal()
        op = self._operator(foo, fglobal)
        self._op = op
        hdiag = self._build_preconditioner_hdiag(fglobal, op)
        if self.re:
            hdiag = self._compress_removed_hdiag(hdiag)

        def vind(zs0):
            if isinstance(zs0, (list, tuple)):
                zs0 = np.asarray(zs0)
            return op.apply_full(zs0)
        vind.operator = op
        return vind, hdiag

    def init_guess(self, nstates, hdiag):
        gaps = np.asarray(hdiag)
        nroots = min(nstates, gaps.size)
        if nroots < 1:
            raise ValueError("No spin-flip excitation space is available.")
        thr = np.sort(gaps)[nroots - 1] + 1e-5
        idx = np.where(gaps <= thr)[0]
        x0 = np.zeros((idx.size, gaps.size))
        x0[np.arange(idx.size), idx] = 1.0
        return x0

    def davidson_process(self, foo, fglobal):
        vind, hdiag = self.gen_tda_operation_sf(foo, fglobal)
        x0 = self.init_guess(self.nstates, hdiag)
        self.converged, self.e, x1, self.icyc = _dav.davidson1(
            vind, x0, hdiag, tol=1e-8, lindep=1e-9, nroots=self.nstates, max_cycle=1000,
            device=self.device, lockstep=self.shard[1] > 1)
        self.v = np.array(x1).T

    def deltaS2_U(self, nstate):
        """P_ab of root ``nstate`` (XSF_TDA.py:613-649), UKS references."""
        return delta_s2_u(self.mf, np.asarray(self.v)[:, nstate], self.nc, self.no, self.nv)

    def analyse(self, threshold=0.05, verbose=False):
        """Delta<S^2> per root and the dominant-amplitude lines (XSF_TDA.py:709-793):
        UKS: P_ab - no + 1; ROKS with SA = 0: -2 S + 1 + sum cv^2 - sum oo^2 +
        (tr oo)^2; spin-adapted ROKS roots are pure spin states (no value, None).
        Returns (Ds, lines); irrep labels need the point-group tables of PySCF
        and are not reproduced."""
        nc, no, nv = self.nc, self.no, self.nv
        vects = self.vects if self.re else None
        Ds, lines = [], []
        for n in range(self.nstates):
            value = np.asarray(self.v)[:, n]
            cv, co, ov, oo = split_xsf_vector(value, nc, no, nv, vects)
            for tag, blk, (o0, v0) in (("CV", cv, (0, nc + no)), ("CO", co, (0, nc)),
                                       ("OV", ov, (nc, nc + no)), ("OO", oo, (nc, nc))):
                for o, v in zip(*np.where(abs(blk) > threshold)):
                    lines.append(f"{100 * blk[o, v] ** 2:5.2f}% {tag}(ab) {o + 1 + o0}a -> "
                                 f"{v + 1 + v0}b {blk[o, v]:10.5f}")
            if self.type_u:
                ds2 = self.deltaS2_U(n) - no + 1
            elif self.SA == 0:
                ds2 = -2 * self.ground_s + 1 + (cv * cv).sum() - (oo * oo).sum() + np.trace(oo) ** 2
            else:
                ds2 = None
            Ds.append(ds2)
            lines.append(f"Excited state {n + 1} {self.e[n] * HA2EV_XSF:10.5f} eV "
                         f"{self.e[n] + self.mf.e_tot:11.8f} Hartree"
                         + (f" D<S^2>={ds2:3.2f}" if ds2 is not None else ""))
        if verbose:
            print("\n".join(lines))
        return Ds, lines

    def get_Amat(self, foo=1.0, fglobal=None):
        """Explicit (remove-compressed when self.re) A through the device operator."""
        vind, _ = self.gen_tda_operation_sf(foo, fglobal)
        return _dense(vind.operator)

    def kernel(self, nstates=1, remove=None, frozen=None, foo=1.0, d_lda=0.3, fglobal=None, fit=True):
        self.re = (not self.type_u) if remove is None else bool(remove)
        if self.re and self.no < 1:
            raise ValueError("OO compression needs an open shell")
        nov = (self.nc + self.no) * (self.no + self.nv)
        self.nstates = min(nstates, nov)
        if fglobal is None:
            fglobal = self.default_fglobal(d_lda, fit)
        self.fglobal = fglobal
        if self.davidson:
            self.davidson_process(foo=foo, fglobal=fglobal)
        else:
            self.A = self.get_Amat(foo=foo, fglobal=fglobal)
            if frozen is not None and not self.re:   # XSF_TDA.py:1544-1545 (the un-removed branch)
                self.A = self.frozen_A(frozen)
            e, v = scipy.linalg.eigh(self.A)
            self.e = e[:self.nstates]
            self.v = v[:, :self.nstates]
        return np.asarray(self.e) * HA2EV_XSF, self.v
