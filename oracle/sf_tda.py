"""SF-TDA oracle (spin-flip up / down, ALDA0 or collinear).  TEST INFRASTRUCTURE ONLY.

* ``gen_tda_operation_sf`` restates SF_TDA.py:162-244 (isf = -1 down, +1 up).
* ``init_guess`` restates SF_TDA.py:348-380.
* ``amat_down`` / ``amat_up`` restate the explicit matrices of
  ``SF_TDA_down.get_Amat`` (SF_TDA.py:624-804) and ``SF_TDA_up.get_Amat``
  (SF_TDA.py:448-560) using MO integrals from the same DF factor and the
  ALDA0 kernel ``fxc_sf`` on the grid; ``method=1`` swaps in the multicollinear
  block of ``get_ab_sf`` (SF_TDA.py:1051-1276, ``oracle.mcol``).
"""
from __future__ import annotations

import numpy as np

from . import engines


def mf_info(mf):
    """SF_TDA.mf_info (SF_TDA.py:26-37)."""
    if not mf.is_rohf:
        return mf.mo_energy, mf.mo_occ, mf.mo_coeff
    mo_energy = np.array([mf.mo_energy, mf.mo_energy])
    mo_coeff = np.array([mf.mo_coeff, mf.mo_coeff])
    mo_occ = np.zeros((2, len(mf.mo_coeff)))
    mo_occ[0][np.where(mf.mo_occ >= 1)[0]] = 1
    mo_occ[1][np.where(mf.mo_occ >= 2)[0]] = 1
    return mo_energy, mo_occ, mo_coeff


def gen_tda_operation_sf(mf, isf, method=0):
    mo_energy, mo_occ, mo_coeff = mf_info(mf)
    occidxa = np.where(mo_occ[0] == 1)[0]
    occidxb = np.where(mo_occ[1] == 1)[0]
    viridxa = np.where(mo_occ[0] == 0)[0]
    viridxb = np.where(mo_occ[1] == 0)[0]
    nocca, noccb = len(occidxa), len(occidxb)
    nvira, nvirb = len(viridxa), len(viridxb)
    orboa = mo_coeff[0][:, occidxa]
    orbob = mo_coeff[1][:, occidxb]
    orbva = mo_coeff[0][:, viridxa]
    orbvb = mo_coeff[1][:, viridxb]
    fockA, fockB = mf.fock_mo()
    if isf == -1:
        e_ia = (mo_energy[1][viridxb, None] - mo_energy[0][occidxa]).T
        ndim = (nocca, nvirb)
        orbo, orbv = orboa, orbvb
    else:
        e_ia = (mo_energy[0][viridxa, None] - mo_energy[1][occidxb]).T
        ndim = (noccb, nvira)
        orbo, orbv = orbob, orbva
    hdiag = e_ia.ravel()
    vresp = engines.gen_response_sf(mf, method=method)

    def vind(zs0):
        zs = np.asarray(zs0).reshape(-1, ndim[0], ndim[1])
        dmov = np.einsum('xov,qv,po->xpq', zs, orbv, orbo, optimize=True)
        v1ao = vresp(dmov)
        vs = np.einsum('xpq,po,qv->xov', v1ao, orbo, orbv, optimize=True)
        if isf == -1:
            vs += (np.einsum('ab,xib->xia', fockB[noccb:, noccb:], zs)
                   - np.einsum('ij,xja->xia', fockA[:nocca, :nocca], zs))
        else:
            vs += (np.einsum('ab,xib->xia', fockA[nocca:, nocca:], zs)
                   - np.einsum('ij,xja->xia', fockB[:noccb, :noccb], zs))
        return vs.reshape(zs.shape[0], -1)

    return vind, hdiag


def init_guess(mf, nstates, isf=-1):
    """SF_TDA.init_guess (SF_TDA.py:348-380)."""
    mo_energy, mo_occ, _ = mf_info(mf)
    occidxa = np.where(mo_occ[0] > 0)[0]
    occidxb = np.where(mo_occ[1] > 0)[0]
    viridxa = np.where(mo_occ[0] == 0)[0]
    viridxb = np.where(mo_occ[1] == 0)[0]
    if isf == 1:
        e = (mo_energy[0][viridxa, None] - mo_energy[1][occidxb]).T.ravel()
    else:
        e = (mo_energy[1][viridxb, None] - mo_energy[0][occidxa]).T.ravel()
    nov = e.size
    nstates = min(nstates, nov)
    thr = np.sort(e)[nstates - 1] + 1e-5
    idx = np.where(e <= thr)[0]
    x0 = np.zeros((idx.size, nov))
    for i, j in enumerate(idx):
        x0[i, j] = 1
    return x0


def _sf_xc_kernel_block(mf, orbo, orbv, method=0):
    """sum_g fxc_sf(g) (phi_o phi_v)(phi_o phi_v) over the grid (SF_TDA.py:509-556);
    method 1: the multicollinear block of get_ab_sf (SF_TDA.py:1179-1272)."""
    if mf.xctype == 'HF':
        return 0.0
    if method == 1:
        from .mcol import sf_mc_block
        return sf_mc_block(mf, mf.fxc_sf_mc, orbo, orbv)
    ao0 = mf.grids.ao[0]
    ro = ao0 @ orbo
    rv = ao0 @ orbv
    rov = np.einsum('ri,ra->ria', ro, rv)
    return np.einsum('ria,rjb->iajb', rov, rov * mf.fxc_sf[:, None, None], optimize=True)


def _exchange_block(mf, orbo, orbv, hyb):
    b_oo = np.einsum('pmn,mi,nj->pij', mf.cderi, orbo, orbo, optimize=True)
    b_vv = np.einsum('pmn,ma,nb->pab', mf.cderi, orbv, orbv, optimize=True)
    a = -hyb * np.einsum('pij,pba->iajb', b_oo, b_vv, optimize=True)
    if mf.omega != 0:
        l_oo = np.einsum('pmn,mi,nj->pij', mf.cderi_lr, orbo, orbo, optimize=True)
        l_vv = np.einsum('pmn,ma,nb->pab', mf.cderi_lr, orbv, orbv, optimize=True)
        a -= (mf.alpha - mf.hyb) * np.einsum('pij,pba->iajb', l_oo, l_vv, optimize=True)
    return a


def amat_down(mf, method=0):
    """SF_TDA_down.get_Amat in cv|co|ov|oo order (SF_TDA.py:624-804)."""
    _, mo_occ, mo_coeff = mf_info(mf)
    orbo_a = mo_coeff[0][:, mo_occ[0] == 1]
    orbv_b = mo_coeff[1][:, mo_occ[1] == 0]
    nocc_a, nvir_b = orbo_a.shape[1], orbv_b.shape[1]
    nc = int((mo_occ[1] == 1).sum())
    no = nocc_a - nc
    nv = nvir_b - no
    hyb = 1.0 if mf.xctype == 'HF' else mf.hyb
    a = _exchange_block(mf, orbo_a, orbv_b, hyb) if (hyb != 0 or mf.omega != 0) else \
        np.zeros((nocc_a, nvir_b, nocc_a, nvir_b))
    if method != 2:
        a = a + _sf_xc_kernel_block(mf, orbo_a, orbv_b, method)
    fockA, fockB = mf.fock_mo()
    e = np.einsum
    iC, iO, iV = np.eye(nc), np.eye(no), np.eye(nv)
    fA_C, fA_O = fockA[:nc, :nc], fockA[nc:nc + no, nc:nc + no]
    fB_O, fB_V = fockB[nc:nc + no, nc:nc + no], fockB[nc + no:, nc + no:]
    dim = (nc + no) * (nv + no)
    d1 = nc * nv; d2 = d1 + nc * no; d3 = d2 + no * nv
    A = np.zeros((dim, dim))
    A[:d1, :d1] = (e('ij,ab->iajb', iC, fB_V).reshape(d1, d1)
                   - e('ji,ab->iajb', fA_C, iV).reshape(d1, d1)
                   + a[:nc, no:, :nc, no:].reshape(d1, d1))
    A[d1:d2, d1:d2] = (e('ij,xy->ixjy', iC, fB_O).reshape(nc * no, nc * no)
                       - e('ji,xy->ixjy', fA_C, iO).reshape(nc * no, nc * no)
                       + a[:nc, :no, :nc, :no].reshape(nc * no, nc * no))
    A[d2:d3, d2:d3] = (e('xy,ab->xayb', iO, fB_V).reshape(no * nv, no * nv)
                       - e('yx,ab->xayb', fA_O, iV).reshape(no * nv, no * nv)
                       + a[nc:, no:, nc:, no:].reshape(no * nv, no * nv))
    A[d3:, d3:] = (e('uv,tw->utvw', iO, fB_O).reshape(no * no, no * no)
                   - e('vu,tw->utvw', fA_O, iO).reshape(no * no, no * no)
                   + a[nc:nc + no, :no, nc:nc + no, :no].reshape(no * no, no * no))
    t = (e('ij,ay->iajy', iC, fockB[nc + no:, nc:nc + no]).reshape(d1, nc * no)
         + a[:nc, no:, :nc, :no].reshape(d1, nc * no))
    A[:d1, d1:d2] = t; A[d1:d2, :d1] = t.T
    t = (-e('yi,ab->iayb', fockA[nc:nc + no, :nc], iV).reshape(d1, no * nv)
         + a[:nc, no:, nc:nc + no, no:].reshape(d1, no * nv))
    A[:d1, d2:d3] = t; A[d2:d3, :d1] = t.T
    t = a[:nc, :no, nc:nc + no, no:].reshape(nc * no, no * nv)
    A[d1:d2, d2:d3] = t; A[d2:d3, d1:d2] = t.T
    t = a[:nc, no:, nc:nc + no, :no].reshape(d1, no * no)
    A[:d1, d3:] = t; A[d3:, :d1] = t.T
    t = (-e('yi,WZ->iWyZ', fockA[nc:nc + no, :nc], iO).reshape(nc * no, no * no)
         + a[:nc, :no, nc:nc + no, :no].reshape(nc * no, no * no))
    A[d1:d2, d3:] = t; A[d3:, d1:d2] = t.T
    t = (e('yx,aZ->xayZ', iO, fockB[nc + no:, nc:nc + no]).reshape(no * nv, no * no)
         + a[nc:, no:, nc:, :no].reshape(no * nv, no * no))
    A[d2:d3, d3:] = t; A[d3:, d2:d3] = t.T
    return A


def amat_up(mf, method=0):
    """SF_TDA_up.get_Amat (SF_TDA.py:448-560): (nc*nv)^2, beta-core -> alpha-virtual."""
    _, mo_occ, mo_coeff = mf_info(mf)
    orbo_b = mo_coeff[1][:, mo_occ[1] == 1]
    orbv_a = mo_coeff[0][:, mo_occ[0] == 0]
    nc, nv = orbo_b.shape[1], orbv_a.shape[1]
    no = int((mo_occ[0] == 1).sum()) - nc
    hyb = 1.0 if mf.xctype == 'HF' else mf.hyb
    a = _exchange_block(mf, orbo_b, orbv_a, hyb) if (hyb != 0 or mf.omega != 0) else \
        np.zeros((nc, nv, nc, nv))
    if method != 2:
        a = a + _sf_xc_kernel_block(mf, orbo_b, orbv_a, method)
    fockA, fockB = mf.fock_mo()
    d_ij = np.eye(nc + no)
    d_ab = np.eye(nv + no)
    A = (a + np.einsum('ij,ab->iajb', d_ij[no:, no:], fockA[nc + no:, nc + no:])
         - np.einsum('ij,ab->iajb', fockB[:nc, :nc], d_ab[no:, no:]))
    return A.reshape(nc * nv, nc * nv)
