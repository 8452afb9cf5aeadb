"""XSF-TDA oracle (spin-adapted spin-flip down).  TEST INFRASTRUCTURE ONLY.

Restates ``XSF_TDA`` (XSF_TDA.py:146-1554):
* ``get_vect``                       XSF_TDA.py:397-414  (OO compression basis)
* ``build_preconditioner_hdiag``     XSF_TDA.py:915-961 + ``_response_j_diagonals`` 859-913
* ``compress_removed_hdiag``         XSF_TDA.py:999-1009
* ``split_block_vectors`` / ``join`` XSF_TDA.py:1011-1027, 1279-1290
* ``gen_tda_operation_sf`` / vind    XSF_TDA.py:1029-1277
* ``get_amat`` + ``remove``          XSF_TDA.py:265-395, 416-427
* ``default_fglobal``                XSF_TDA.py:1511-1518
(the full-width comma at XSF_TDA.py:1137 is read as the ASCII comma it means).
"""
from __future__ import annotations

import math

import numpy as np

from . import engines
from .sf_tda import amat_down, mf_info


def default_fglobal(mf, d_lda=0.3, method=0, fit=True):
    if mf.xctype == 'HF':
        cx = 1.0
    elif mf.omega == 0:
        cx = mf.hyb
    else:
        cx = mf.hyb + (mf.alpha - mf.hyb) * math.erf(mf.omega)
    f = (1 - d_lda) * cx + d_lda
    if method == 1 and fit:
        f = f * 4 * (cx - 0.5) ** 2
    return f


def get_vect(no):
    tmp_v = np.zeros((no - 1, no))
    for i in range(1, no):
        factor = 1 / np.sqrt((no - i + 1) * (no - i))
        tmp = [no - i] + [-1] * (no - i)
        tmp_v[i - 1][i - 1:] = np.array(tmp) * factor
    vect = tmp_v.T
    vects = np.eye(no * no)[:, :-1]
    index = [0] + [i * (no + 1) for i in range(1, no)]
    for i in range(vect.shape[1]):
        vects[0::no + 1, index[i]] = vect[:, i]
    return vects


class XSFOracle:
    def __init__(self, mf, SA=None, method=0):
        self.mf = mf
        self.mo_energy, self.mo_occ, self.mo_coeff = mf_info(mf)
        self.type_u = not mf.is_rohf
        self.SA = (0 if self.type_u else 3) if SA is None else SA
        self.method = method
        self.occidx_a = np.where(self.mo_occ[0] == 1)[0]
        self.viridx_a = np.where(self.mo_occ[0] == 0)[0]
        self.occidx_b = np.where(self.mo_occ[1] == 1)[0]
        self.viridx_b = np.where(self.mo_occ[1] == 0)[0]
        self.nocc_a = len(self.occidx_a)
        self.nocc_b = len(self.occidx_b)
        self.nvir_a = len(self.viridx_a)
        self.nvir_b = len(self.viridx_b)
        self.nc = self.nocc_b
        self.nv = self.nvir_a
        self.no = self.nocc_a - self.nocc_b
        self.re = not self.type_u
        self.vects = get_vect(self.no) if self.no > 1 else np.zeros((self.no ** 2, 0))

    # ---------------------------------------------------------------- hdiag
    def _response_j_diagonals(self):
        mo_coeff = self.mo_coeff
        nc, no, nv = self.nc, self.no, self.nv
        orbca = mo_coeff[0][:, self.occidx_a[:nc]]
        orboa_open = mo_coeff[0][:, self.occidx_a[nc:nc + no]]
        orbbo = mo_coeff[1][:, self.viridx_b[:no]]
        orbvv = mo_coeff[1][:, self.viridx_b[no:]]

        def diag_j(orbo, orbv, n_o, n_v):
            n = n_o * n_v
            out = np.zeros(n)
            for p0 in range(0, n, 64):
                idx = np.arange(p0, min(n, p0 + 64))
                trial = np.zeros((idx.size, n))
                trial[np.arange(idx.size), idx] = 1
                trial = trial.reshape(idx.size, n_o, n_v)
                dms = np.einsum("xov,qv,po->xpq", trial, orbv, orbo)
                vj = engines.jk(self.mf, dms, with_k=False)[0]
                blk = np.einsum("xpq,pi,qu->xiu", vj, orbo, orbv).reshape(idx.size, n)
                out[idx] = blk[np.arange(idx.size), idx]
            return out.reshape(n_o, n_v)

        return diag_j(orbca, orbbo, nc, no), diag_j(orboa_open, orbvv, no, nv)

    def build_preconditioner_hdiag(self, fglobal):
        mf = self.mf
        fockA, fockB = mf.fock_mo()
        nc, no = self.nc, self.no
        si = no / 2.0
        diag_a, diag_b = fockA.diagonal(), fockB.diagonal()
        hdiag = diag_b[self.nocc_b:, None].T - diag_a[:self.nocc_a, None]
        if self.SA > 0:
            fockA_hf, fockB_hf = mf.fock_mo_hf()
            diag_s = ((fockB_hf - fockA_hf) * 0.5).diagonal()
            hdiag[:nc, no:] += fglobal * (diag_s[nc + no:] + diag_s[:nc, None]) / si
            co_j, ov_j = self._response_j_diagonals()
            hdiag[:nc, :no] += fglobal * (2.0 * diag_s[:nc, None] - co_j) / (2 * si - 1)
            hdiag[nc:, no:] += fglobal * (2.0 * diag_s[nc + no:] - ov_j) / (2 * si - 1)
        return np.hstack([hdiag[:nc, no:].reshape(-1), hdiag[:nc, :no].reshape(-1),
                          hdiag[nc:, no:].reshape(-1), hdiag[nc:, :no].reshape(-1)])

    def compress_removed_hdiag(self, hdiag):
        nc, no, nv = self.nc, self.no, self.nv
        dim3 = nc * nv + nc * no + no * nv
        new_oo = np.einsum("x,xy,xy->y", hdiag[dim3:], self.vects, self.vects)
        out = np.zeros(hdiag.size - 1)
        out[:dim3] = hdiag[:dim3]
        out[dim3:] = new_oo
        return out

    # ---------------------------------------------------------------- blocks
    def split_block_vectors(self, data, expand_oo=True):
        data = np.asarray(data)
        if data.ndim == 1:
            data = data.reshape(1, -1)
        nc, no, nv = self.nc, self.no, self.nv
        d1 = nc * nv; d2 = d1 + nc * no; d3 = d2 + no * nv
        n = data.shape[0]
        cv = data[:, :d1].reshape(n, nc, nv)
        co = data[:, d1:d2].reshape(n, nc, no)
        ov = data[:, d2:d3].reshape(n, no, nv)
        oo = data[:, d3:]
        if self.re and expand_oo:
            oo = np.einsum("xy,ny->nx", self.vects, oo)
        return cv, co, ov, oo.reshape(n, no, no)

    def join_block_vectors(self, cv, co, ov, oo, compress_oo=True):
        oo = oo.reshape(oo.shape[0], -1)
        if compress_oo:
            oo = np.einsum("xy,nx->ny", self.vects, oo)
        return np.hstack([cv.reshape(cv.shape[0], -1), co.reshape(co.shape[0], -1),
                          ov.reshape(ov.shape[0], -1), oo])

    # ---------------------------------------------------------------- vind
    def gen_tda_operation_sf(self, foo=1.0, fglobal=None, with_hdiag=True):
        """with_hdiag=False skips the preconditioner's J diagonals (one J build per
        64 unit vectors; setup, not part of A.x) and returns the Fock-difference
        diagonal only -- for timing vind alone (bench.py cpu_baseline)."""
        mf = self.mf
        if fglobal is None:
            fglobal = default_fglobal(mf, method=self.method)
        mo_coeff = self.mo_coeff
        nc, no, nv = self.nc, self.no, self.nv
        si = no / 2.0
        orboa = mo_coeff[0][:, self.occidx_a]
        orbvb = mo_coeff[1][:, self.viridx_b]
        fockA, fockB = mf.fock_mo()
        orbca = orboa[:, :nc]
        orboa_open = orboa[:, nc:nc + no]
        orbbo = orbvb[:, :no]
        orbvv = orbvb[:, no:]
        fa_cc = fockA[:nc, :nc]; fa_co = fockA[:nc, nc:nc + no]
        fa_oc = fockA[nc:nc + no, :nc]; fa_oo = fockA[nc:nc + no, nc:nc + no]
        fb_oo = fockB[nc:nc + no, nc:nc + no]; fb_ov = fockB[nc:nc + no, nc + no:]
        fb_vo = fockB[nc + no:, nc:nc + no]; fb_vv = fockB[nc + no:, nc + no:]

        if with_hdiag:
            hdiag = self.build_preconditioner_hdiag(fglobal)
        else:
            fa, fb = mf.fock_mo()
            hd = fb.diagonal()[self.nocc_b:][None, :] - fa.diagonal()[:self.nocc_a, None]
            hdiag = np.hstack([hd[:nc, no:].reshape(-1), hd[:nc, :no].reshape(-1),
                               hd[nc:, no:].reshape(-1), hd[nc:, :no].reshape(-1)])
        if self.re:
            hdiag = self.compress_removed_hdiag(hdiag)
        vresp = engines.gen_response_sf(mf, method=self.method)
        if self.SA > 0:
            fockA_hf, fockB_hf = mf.fock_mo_hf()
            fockS_hf = (fockB_hf - fockA_hf) * 0.5
            factor1 = np.sqrt((2 * si + 1) / (2 * si)) - 1
            factor2 = np.sqrt((2 * si + 1) / (2 * si - 1))
            factor3 = np.sqrt((2 * si) / (2 * si - 1)) - 1
            factor4 = 1 / np.sqrt(2 * si * (2 * si - 1))
            fs_cc = fockS_hf[:nc, :nc]
            fs_vv = fockS_hf[nc + no:, nc + no:]
            fs_cv = fockS_hf[:nc, nc + no:]
        iden_O = np.eye(no)
        c = np.einsum

        def proj(v1ao):
            return (c("xpq,pi,qa->xia", v1ao, orbca, orbvv, optimize=True),
                    c("xpq,pi,qu->xiu", v1ao, orbca, orbbo, optimize=True),
                    c("xpq,pu,qa->xua", v1ao, orboa_open, orbvv, optimize=True),
                    c("xpq,pu,qv->xuv", v1ao, orboa_open, orbbo, optimize=True))

        def vind(zs0):
            zs0 = np.asarray(zs0)
            cv, co, ov, oo = self.split_block_vectors(zs0, expand_oo=self.re)
            d_cv = c("xia,qa,pi->xpq", cv, orbvv, orbca, optimize=True)
            d_co = c("xiu,qu,pi->xpq", co, orbbo, orbca, optimize=True)
            d_ov = c("xua,qa,pu->xpq", ov, orbvv, orboa_open, optimize=True)
            d_oo = c("xuv,qv,pu->xpq", oo, orbbo, orboa_open, optimize=True)
            v1ao = vresp(d_cv + d_co + d_ov + d_oo)
            vs_cv, vs_co, vs_ov, vs_oo = proj(v1ao)
            vs_cv = vs_cv + (c("xiu,ua->xia", co, fb_ov) + c("xib,ba->xia", cv, fb_vv)
                             - c("ij,xja->xia", fa_cc, cv) - c("iu,xua->xia", fa_co, ov))
            vs_co = vs_co + (c("xiv,vu->xiu", co, fb_oo) + c("xia,au->xiu", cv, fb_vo)
                             - c("ij,xju->xiu", fa_cc, co) - c("iv,xvu->xiu", fa_co, oo))
            vs_ov = vs_ov + (c("xuv,va->xua", oo, fb_ov) + c("xub,ba->xua", ov, fb_vv)
                             - c("ui,xia->xua", fa_oc, cv) - c("uv,xva->xua", fa_oo, ov))
            vs_oo = vs_oo + (c("xuw,wv->xuv", oo, fb_oo) + c("xua,av->xuv", ov, fb_vo)
                             - c("ui,xiv->xuv", fa_oc, co) - c("uw,xwv->xuv", fa_oo, oo))
            if self.SA > 0:
                dcv = np.zeros_like(cv); dco = np.zeros_like(co)
                dov = np.zeros_like(ov); doo = np.zeros_like(oo)
                nb = cv.shape[0]
                dm_hf = np.concatenate([d_cv, d_co, d_ov, d_oo], axis=0)
                v1_j, v1_k = engines.jk(mf, dm_hf)
                v1_cv_k = v1_k[:nb]
                v1_co_j, v1_co_k = v1_j[nb:2 * nb], v1_k[nb:2 * nb]
                v1_ov_j, v1_ov_k = v1_j[2 * nb:3 * nb], v1_k[2 * nb:3 * nb]
                v1_oo_k = v1_k[3 * nb:]
                cv_co_j, co_co_j, ov_co_j, oo_co_j = proj(v1_co_j)
                cv_ov_j, co_ov_j, ov_ov_j, oo_ov_j = proj(v1_ov_j)
                cv_cv_k, co_cv_k, ov_cv_k, oo_cv_k = proj(v1_cv_k)
                cv_co_k, co_co_k, ov_co_k, oo_co_k = proj(v1_co_k)
                cv_ov_k, co_ov_k, ov_ov_k, oo_ov_k = proj(v1_ov_k)
                cv_oo_k, co_oo_k, ov_oo_k, oo_oo_k = proj(v1_oo_k)
                dcv += (c("ab,xib->xia", fs_vv, cv) + c("ji,xja->xia", fs_cc, cv)) / si
                dco += -co_co_j / (2 * si - 1) + 2.0 * c("ji,xju->xiu", fs_cc, co) / (2 * si - 1)
                dov += -ov_ov_j / (2 * si - 1) + 2.0 * c("ab,xub->xua", fs_vv, ov) / (2 * si - 1)
                if self.SA > 1:
                    fB_vo = fockB_hf[nc + no:, nc:nc + no]
                    fA_oc = fockA_hf[nc:nc + no, :nc]
                    dcv += factor1 * (-cv_co_k + c("av,xiv->xia", fB_vo, co))
                    dco += factor1 * (-co_cv_k + c("av,xja->xjv", fB_vo, cv))
                    dcv += factor1 * (-cv_ov_k - c("vi,xva->xia", fA_oc, ov))
                    dov += factor1 * (-ov_cv_k - c("vi,xib->xvb", fA_oc, cv))
                    dco += (co_ov_j - co_ov_k) / (2 * si - 1)
                    dov += (ov_co_j - ov_co_k) / (2 * si - 1)
                if self.SA > 2:
                    fA_co = fockA_hf[:nc, nc:nc + no]
                    fB_co = fockB_hf[:nc, nc:nc + no]
                    fB_vo = fockB_hf[nc + no:, nc:nc + no]
                    fA_vo = fockA_hf[nc + no:, nc:nc + no]
                    dcv += foo * (-(factor2 - 1) * cv_oo_k
                                  + (factor2 / si) * c("ia,xvv->xia", fs_cv, oo))
                    doo += foo * (-(factor2 - 1) * oo_cv_k
                                  + (factor2 / si) * c("vw,ia,xia->xvw", iden_O, fs_cv, cv))
                    dco += foo * (factor3 * (-co_oo_k - c("iw,xwu->xiu", fA_co, oo))
                                  + factor4 * c("vw,iu,xvw->xiu", iden_O, fB_co, oo))
                    doo += foo * (factor3 * (-oo_co_k - c("iw,xiv->xwv", fA_co, co))
                                  + factor4 * c("vw,iu,xiu->xvw", iden_O, fB_co, co))
                    dov += foo * (factor3 * (-ov_oo_k + c("av,xuv->xua", fB_vo, oo))
                                  - factor4 * c("vw,au,xvw->xua", iden_O, fA_vo, oo))
                    doo += foo * (factor3 * (-oo_ov_k + c("av,xwa->xwv", fB_vo, ov))
                                  - factor4 * c("vw,au,xua->xwv", iden_O, fA_vo, ov))
                vs_cv = vs_cv + fglobal * dcv
                vs_co = vs_co + fglobal * dco
                vs_ov = vs_ov + fglobal * dov
                vs_oo = vs_oo + fglobal * doo
            return self.join_block_vectors(vs_cv, vs_co, vs_ov, vs_oo, self.re)

        return vind, hdiag

    def init_guess(self, nstates, hdiag):
        """XSF_TDA._build_initial_guess_from_gaps (XSF_TDA.py:964-982)."""
        gaps = np.asarray(hdiag)
        nov = gaps.size
        nroots = min(nstates, nov)
        thr = np.sort(gaps)[nroots - 1] + 1e-5
        idx = np.where(gaps <= thr)[0]
        x0 = np.zeros((idx.size, nov))
        x0[np.arange(idx.size), idx] = 1.0
        return x0

    # ---------------------------------------------------------------- explicit
    def get_amat(self, foo=1.0, fglobal=None, SA=None):
        """XSF_TDA.get_Amat (XSF_TDA.py:265-395), un-compressed cv|co|ov|oo."""
        mf = self.mf
        SA = self.SA if SA is None else SA
        if fglobal is None:
            fglobal = default_fglobal(mf, method=self.method)
        nc, nv, no = self.nc, self.nv, self.no
        sf_A = amat_down(mf, method=self.method)
        if self.type_u:
            return sf_A
        Amat = np.zeros_like(sf_A)
        d1 = nc * nv; d2 = d1 + nc * no; d3 = d2 + no * nv
        si = 1.e10 if SA == 0 else no / 2
        fockA_hf, fockB_hf = mf.fock_mo_hf()
        fockS = (fockB_hf - fockA_hf) / 2
        fS_C, fS_V = fockS[:nc, :nc], fockS[nc + no:, nc + no:]
        fS_CV = fockS[:nc, nc + no:]
        c = mf.mo_coeff
        bmo = np.einsum('pmn,mi,nj->pij', mf.cderi, c, c, optimize=True)
        eri = np.einsum('pij,pkl->ijkl', bmo, bmo, optimize=True)
        iC, iO, iV = np.eye(nc), np.eye(no), np.eye(nv)
        e = np.einsum
        Amat[:d1, :d1] += (e('ij,ab->iajb', iC, fS_V).reshape(d1, d1)
                           + e('ji,ab->iajb', fS_C, iV).reshape(d1, d1)) / si
        Amat[d1:d2, d1:d2] += (e('ji,uv->iujv', fS_C, iO).reshape(no * nc, no * nc) * 2 / (2 * si - 1)
                               - e('uijv->iujv', eri[nc:nc + no, :nc, :nc, nc:nc + no]).reshape(no * nc, no * nc) / (2 * si - 1))
        Amat[d2:d3, d2:d3] += (e('uv,ab->uavb', iO, fS_V).reshape(nv * no, nv * no) * 2 / (2 * si - 1)
                               - e('auvb->uavb', eri[nc + no:, nc:nc + no, nc:nc + no, nc + no:]).reshape(nv * no, nv * no) / (2 * si - 1))
        if SA > 1:
            t = (np.sqrt(1 + 1 / (2 * si)) - 1) * (e('ij,av->iajv', iC, fockB_hf[nc + no:, nc:nc + no])
                                                   - e('avji->iajv', eri[nc + no:, nc:nc + no, :nc, :nc])).reshape(nv * nc, no * nc)
            Amat[:d1, d1:d2] += t; Amat[d1:d2, :d1] += t.T
            t = (np.sqrt(1 + 1 / (2 * si)) - 1) * (-e('iv,ab->iavb', fockA_hf[:nc, nc:nc + no], iV)
                                                   - e('abvi->iavb', eri[nc + no:, nc + no:, nc:nc + no, :nc])).reshape(nv * nc, nv * no)
            Amat[:d1, d2:d3] += t; Amat[d2:d3, :d1] += t.T
            t = (1 / (2 * si - 1)) * (e('uivb->iuvb', eri[nc:nc + no, :nc, nc:nc + no, nc + no:])
                                      - e('ubvi->iuvb', eri[nc:nc + no, nc + no:, nc:nc + no, :nc])).reshape(no * nc, nv * no)
            Amat[d1:d2, d2:d3] += t; Amat[d2:d3, d1:d2] += t.T
        factor = np.sqrt((2 * si + 1) / (2 * si - 1))
        if SA > 2:
            t = (-(factor - 1) * e('avwi->iawv', eri[nc + no:, nc:nc + no, nc:nc + no, :nc]).reshape(nv * nc, no * no)
                 + (1 / si) * factor * e('ia,wv->iawv', fS_CV, iO).reshape(nv * nc, no * no))
            Amat[:d1, d3:] += foo * t; Amat[d3:, :d1] += foo * t.T
            t = ((np.sqrt(2 * si / (2 * si - 1)) - 1) * (-e('wi,uv->iuwv', fockA_hf[nc:nc + no, :nc], iO).reshape(no * nc, no * no)
                                                         - e('uvwi->iuwv', eri[nc:nc + no, nc:nc + no, nc:nc + no, :nc]).reshape(no * nc, no * no))
                 + (1 / np.sqrt(2 * si * (2 * si - 1))) * e('iu,wv->iuwv', fockB_hf[:nc, nc:nc + no], iO).reshape(no * nc, no * no))
            Amat[d1:d2, d3:] += foo * t; Amat[d3:, d1:d2] += foo * t.T
            t = ((np.sqrt(2 * si / (2 * si - 1)) - 1) * (e('wu,av->uawv', iO, fockB_hf[nc + no:, nc:nc + no]).reshape(nv * no, no * no)
                                                         - e('avwu->uawv', eri[nc + no:, nc:nc + no, nc:nc + no, nc:nc + no]).reshape(nv * no, no * no))
                 - (1 / np.sqrt(2 * si * (2 * si - 1))) * e('ua,wv->uawv', fockA_hf[nc:nc + no, nc + no:], iO).reshape(nv * no, no * no))
            Amat[d2:d3, d3:] += foo * t; Amat[d3:, d2:d3] += foo * t.T
        return sf_A + fglobal * Amat

    def remove(self, A):
        d3 = self.nc * self.nv + self.nc * self.no + self.no * self.nv
        dim = A.shape[0]
        V = self.vects
        out = np.zeros((dim - 1, dim - 1))
        out[:d3, :d3] = A[:d3, :d3]
        out[:d3, d3:] = A[:d3, d3:] @ V
        out[d3:, :d3] = V.T @ A[d3:, :d3]
        out[d3:, d3:] = V.T @ A[d3:, d3:] @ V
        return out
