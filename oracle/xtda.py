"""X-TDA / U-TDA oracle.  TEST INFRASTRUCTURE ONLY.

* ``gen_tda_operation`` restates ``XTDA._gen_tda_operation`` + ``vind``
  (XTDA.py:558-692): MO->AO transition densities, AO response
  (``engines.gen_response``), AO->MO projection, ROKS Fock terms and the
  spin-adaptation Delta-A terms with coefficients from ``si = spin/2``.
* ``get_init_guess`` restates XTDA.py:700-734, ``get_precond`` XTDA.py:736-744.
* ``full_diag_matrix`` restates the explicit A of ``XTDA.full_diag``
  (XTDA.py:56-400) with MO integrals from the same DF factor and the
  explicit XC kernel loops (LDA XTDA.py:178-207, GGA 208-238, MGGA 239-276) -- an
  independent code path used to pin ``vind``.
"""
from __future__ import annotations

import numpy as np

from . import engines


def _orbitals(mf):
    if mf.is_rohf:
        c = mf.mo_coeff
        occ = np.zeros((2, mf.mo_occ.size))
        occ[0][mf.mo_occ >= 1] = 1
        occ[1][mf.mo_occ >= 2] = 1
        mo_coeff = (c, c)
        mo_energy = (mf.mo_energy, mf.mo_energy)
    else:
        mo_coeff = (mf.mo_coeff[0], mf.mo_coeff[1])
        mo_energy = (mf.mo_energy[0], mf.mo_energy[1])
        occ = mf.mo_occ
    return mo_coeff, mo_energy, occ


def gen_tda_operation(mf):
    """(vind, hdiag) exactly as XTDA._gen_tda_operation builds them."""
    X = mf.is_rohf
    mo_coeff, mo_energy, mo_occ = _orbitals(mf)
    occidxa = np.where(mo_occ[0] > 0)[0]
    occidxb = np.where(mo_occ[1] > 0)[0]
    viridxa = np.where(mo_occ[0] == 0)[0]
    viridxb = np.where(mo_occ[1] == 0)[0]
    nocca, noccb = len(occidxa), len(occidxb)
    nvira, nvirb = len(viridxa), len(viridxb)
    orboa = mo_coeff[0][:, occidxa]
    orbob = mo_coeff[1][:, occidxb]
    orbva = mo_coeff[0][:, viridxa]
    orbvb = mo_coeff[1][:, viridxb]

    if X:
        focka_mo, fockb_mo = mf.fock_mo()
        e_ia_a = focka_mo.diagonal()[viridxa] - focka_mo.diagonal()[occidxa, None]
        e_ia_b = fockb_mo.diagonal()[viridxb] - fockb_mo.diagonal()[occidxb, None]
    else:
        e_ia_a = mo_energy[0][viridxa] - mo_energy[0][occidxa, None]
        e_ia_b = mo_energy[1][viridxb] - mo_energy[1][occidxb, None]
    hdiag = np.hstack((e_ia_a.reshape(-1), e_ia_b.reshape(-1)))
    vresp = engines.gen_response(mf)

    if X:
        focka_mo_hf, fockb_mo_hf = mf.fock_mo_hf()
        si = 0.5 * mf.mol.spin
        c_p = 0.5 * (1 - np.sqrt((si + 1) / si) + 1 / (2 * si))
        c_m = 0.5 * (-1 + np.sqrt((si + 1) / si) + 1 / (2 * si))
        c_x = 0.5 * 1 / (2 * si)

    def vind(zs):
        zs = np.asarray(zs)
        nz = len(zs)
        za = zs[:, :nocca * nvira].reshape(nz, nocca, nvira)
        zb = zs[:, nocca * nvira:].reshape(nz, noccb, nvirb)
        dmsa = np.einsum('xov,pv,qo->xpq', za, orbva, orboa, optimize=True)
        dmsb = np.einsum('xov,pv,qo->xpq', zb, orbvb, orbob, optimize=True)
        v1ao = vresp(np.asarray((dmsa, dmsb)))
        v1a = np.einsum('xpq,qo,pv->xov', v1ao[0], orboa, orbva, optimize=True)
        v1b = np.einsum('xpq,qo,pv->xov', v1ao[1], orbob, orbvb, optimize=True)
        if X:
            v1a += (np.einsum('xib,ab->xia', za, focka_mo[nocca:, nocca:])
                    - np.einsum('xja,ij->xia', za, focka_mo[:nocca, :nocca]))
            zac = za[:, :noccb, :]
            zbv = zb[:, :, -nvira:]
            dv = fockb_mo_hf[nocca:, nocca:] - focka_mo_hf[nocca:, nocca:]
            do = fockb_mo_hf[:noccb, :noccb] - focka_mo_hf[:noccb, :noccb]
            # CV(aa)-CV(aa)  (XTDA.py:636-645)
            v1a[:, :noccb, :] += (c_p * np.einsum('xib,ab->xia', zac, dv)
                                  + c_m * np.einsum('xja,ij->xia', zac, do))
            # CV(aa)-CV(bb)  (XTDA.py:649-656)
            v1a[:, :noccb, :] -= c_x * (np.einsum('xib,ab->xia', zbv, dv)
                                        + np.einsum('xja,ij->xia', zbv, do))
            v1b += (np.einsum('xib,ab->xia', zb, fockb_mo[noccb:, noccb:])
                    - np.einsum('xja,ij->xia', zb, fockb_mo[:noccb, :noccb]))
            # CV(bb)-CV(aa)  (XTDA.py:664-671)
            v1b[:, :, -nvira:] -= c_x * (np.einsum('xib,ab->xia', zac, dv)
                                         + np.einsum('xja,ij->xia', zac, do))
            # CV(bb)-CV(bb)  (XTDA.py:675-684)
            v1b[:, :, -nvira:] += (c_m * np.einsum('xib,ab->xia', zbv, dv)
                                   + c_p * np.einsum('xja,ij->xia', zbv, do))
        else:
            v1a += np.einsum('xia,ia->xia', za, e_ia_a)
            v1b += np.einsum('xia,ia->xia', zb, e_ia_b)
        return np.hstack((v1a.reshape(nz, -1), v1b.reshape(nz, -1)))

    return vind, hdiag


def get_init_guess(mf, nstates):
    """Koopmans unit vectors (XTDA.py:700-734)."""
    _, mo_energy, mo_occ = _orbitals(mf)
    occidxa = np.where(mo_occ[0] > 0)[0]
    occidxb = np.where(mo_occ[1] > 0)[0]
    viridxa = np.where(mo_occ[0] == 0)[0]
    viridxb = np.where(mo_occ[1] == 0)[0]
    e_ia_a = mo_energy[0][viridxa] - mo_energy[0][occidxa, None]
    e_ia_b = mo_energy[1][viridxb] - mo_energy[1][occidxb, None]
    nov = e_ia_a.size + e_ia_b.size
    nstates = min(nstates, nov)
    e_ia = np.append(e_ia_a.ravel(), e_ia_b.ravel())
    e_threshold = np.partition(e_ia, nstates - 1)[nstates - 1] + 0.001
    idx = np.where(e_ia <= e_threshold)[0]
    x0 = np.zeros((idx.size, nov))
    for i, j in enumerate(idx):
        x0[i, j] = 1
    return x0


def get_precond(mf, hdiag):
    """XTDA.get_precond (XTDA.py:736-744)."""
    def precond(x, e, *args):
        if isinstance(e, np.ndarray):
            e = e[0]
        diagd = hdiag - (e - mf.level_shift)
        diagd[abs(diagd) < 1e-8] = 1e-8
        return x / diagd
    return precond


def pickeig(w, v, nroots, envs):
    """XTDA.Davidson.pickeig (XTDA.py:769-772)."""
    idx = np.where(w > 0.001)[0]
    return w[idx], v[:, idx], idx


# ---------------------------------------------------------------------------
# explicit A (XTDA.full_diag, XTDA.py:56-400), in PySCF order
# ---------------------------------------------------------------------------
def _mo_eri(cderi, c1, c2, c3, c4):
    b12 = np.einsum('pmn,mi,nj->pij', cderi, c1, c2, optimize=True)
    b34 = np.einsum('pmn,mk,nl->pkl', cderi, c3, c4, optimize=True)
    return np.einsum('pij,pkl->ijkl', b12, b34, optimize=True)


def full_diag_matrix(mf):
    """Explicit ROKS X-TDA matrix in the reference's "my order"
    CV(aa), OV(aa), CO(bb), CV(bb) (XTDA.py:278-398)."""
    assert mf.is_rohf
    mo_coeff = mf.mo_coeff
    mo_occ = mf.mo_occ
    occidx_a = np.where(mo_occ >= 1)[0]
    viridx_a = np.where(mo_occ == 0)[0]
    occidx_b = np.where(mo_occ >= 2)[0]
    viridx_b = np.where(mo_occ != 2)[0]
    nocc_a, nvir_a = len(occidx_a), len(viridx_a)
    nocc_b, nvir_b = len(occidx_b), len(viridx_b)
    orbo_a, orbv_a = mo_coeff[:, occidx_a], mo_coeff[:, viridx_a]
    orbo_b, orbv_b = mo_coeff[:, occidx_b], mo_coeff[:, viridx_b]
    mo_a = np.hstack((orbo_a, orbv_a))
    nmo_a = mo_a.shape[1]
    fock_a, fock_b = mf.fock_mo()
    focka2, fockb2 = mf.fock_mo_hf()
    fab_a2 = focka2[nocc_a:, nocc_a:]
    fab_b2 = fockb2[nocc_b:, nocc_b:]
    fij_a2 = focka2[:nocc_a, :nocc_a]
    fij_b2 = fockb2[:nocc_b, :nocc_b]
    hyb = mf.hyb if mf.xctype != 'HF' else 1.0

    eri = _mo_eri(mf.cderi, orbo_a, mo_a, orbv_b, mo_a)   # (nocc_a, nmo, nvir_b, nmo)
    aa = np.zeros((nocc_a, nvir_a, nocc_a, nvir_a))
    ab = np.zeros((nocc_a, nvir_a, nocc_b, nvir_b))
    bb = np.zeros((nocc_b, nvir_b, nocc_b, nvir_b))
    aa += np.einsum('iabj->iajb', eri[:nocc_a, nocc_a:, nocc_a - nocc_b:, :nocc_a])
    aa -= np.einsum('ijba->iajb', eri[:nocc_a, :nocc_a, nocc_a - nocc_b:, nocc_a:]) * hyb
    bb += np.einsum('iabj->iajb', eri[:nocc_b, nocc_b:, 0:, :nocc_b])
    bb -= np.einsum('ijba->iajb', eri[:nocc_b, :nocc_b, 0:, nocc_b:]) * hyb
    ab += np.einsum('iabj->iajb', eri[:nocc_a, nocc_a:, 0:, :nocc_b])
    if mf.omega != 0:
        c_lr = engines._k_coeffs(mf)[1]
        # full_diag (XTDA.py:150-158) only treats the hyb + (alpha-hyb)*LR case
        eri_aa = _mo_eri(mf.cderi_lr, orbo_a, mo_a, mo_a, mo_a)
        mo_b = np.hstack((orbo_b, orbv_b))
        eri_bb = _mo_eri(mf.cderi_lr, orbo_b, mo_b, mo_b, mo_b)
        aa -= np.einsum('ijba->iajb', eri_aa[:nocc_a, :nocc_a, nocc_a:, nocc_a:]) * c_lr
        bb -= np.einsum('ijba->iajb', eri_bb[:nocc_b, :nocc_b, nocc_b:, nocc_b:]) * c_lr

    if mf.xctype in ('LDA', 'GGA', 'MGGA'):
        # XTDA.py:178-276, summed over grid blocks (the whole-grid rho_ov of a 200-AO
        # molecule would take tens of GB); each block's contraction as one GEMM
        ng = mf.grids.ngrid
        for g0 in range(0, ng, engines.GRID_BLOCK):
            g1 = min(ng, g0 + engines.GRID_BLOCK)
            ao = mf.grids.ao[:, g0:g1]
            w = mf.grids.weights[g0:g1]
            fxc = mf.fxc[..., g0:g1]
            if mf.xctype == 'LDA':
                wfxc = fxc[:, 0, :, 0] * w
                rho_ov_a = np.einsum('ri,ra->ria', ao[0] @ orbo_a, ao[0] @ orbv_a)[None]
                rho_ov_b = np.einsum('ri,ra->ria', ao[0] @ orbo_b, ao[0] @ orbv_b)[None]
                wfxc = wfxc[:, None, :, None]
            else:
                wfxc = fxc * w
                rho_o_a = np.einsum('xrp,pi->xri', ao, orbo_a)
                rho_v_a = np.einsum('xrp,pi->xri', ao, orbv_a)
                rho_o_b = np.einsum('xrp,pi->xri', ao, orbo_b)
                rho_v_b = np.einsum('xrp,pi->xri', ao, orbv_b)
                rho_ov_a = np.einsum('xri,ra->xria', rho_o_a, rho_v_a[0])
                rho_ov_b = np.einsum('xri,ra->xria', rho_o_b, rho_v_b[0])
                rho_ov_a[1:4] += np.einsum('ri,xra->xria', rho_o_a[0], rho_v_a[1:4])
                rho_ov_b[1:4] += np.einsum('ri,xra->xria', rho_o_b[0], rho_v_b[1:4])
                if mf.xctype == 'MGGA':     # tau_ov = 1/2 sum_c d_c phi_i d_c phi_a (XTDA.py:256-259)
                    tau_ov_a = np.einsum('xri,xra->ria', rho_o_a[1:4], rho_v_a[1:4]) * .5
                    tau_ov_b = np.einsum('xri,xra->ria', rho_o_b[1:4], rho_v_b[1:4]) * .5
                    rho_ov_a = np.vstack([rho_ov_a, tau_ov_a[np.newaxis]])
                    rho_ov_b = np.vstack([rho_ov_b, tau_ov_b[np.newaxis]])
            w_ov_aa = np.einsum('xyr,xria->yria', wfxc[0, :, 0], rho_ov_a)
            w_ov_ab = np.einsum('xyr,xria->yria', wfxc[0, :, 1], rho_ov_a)
            w_ov_bb = np.einsum('xyr,xria->yria', wfxc[1, :, 1], rho_ov_b)
            ra = rho_ov_a.reshape(-1, nocc_a * nvir_a)       # (x r, i a)
            rb = rho_ov_b.reshape(-1, nocc_b * nvir_b)
            aa += (w_ov_aa.reshape(ra.shape).T @ ra).reshape(aa.shape)
            bb += (w_ov_bb.reshape(rb.shape).T @ rb).reshape(bb.shape)
            ab += (w_ov_ab.reshape(ra.shape).T @ rb).reshape(ab.shape)

    nc = min(nocc_a, nocc_b)
    no = abs(nocc_a - nocc_b)
    nv = min(nvir_a, nvir_b)
    dim = (nc + no) * nv + nc * (nv + no)
    A = np.zeros((dim, dim))
    si = 0.5 * mf.mol.spin
    d_ij = np.eye(nocc_b)
    d_ab = np.eye(nvir_a)
    d_ij_a = np.eye(nocc_a)
    d_ij_b = np.eye(nocc_b)
    d_ab_a = np.eye(nvir_a)
    d_ab_b = np.eye(nvir_b)
    e = np.einsum
    s1 = nc * nv
    s2 = (nc + no) * nv
    s3 = s2 + nc * no
    A[:s1, :s1] = (e('ij,ab->iajb', d_ij_a[:nc, :nc], fock_a[nc + no:, nc + no:])
                   - e('ij,ab->iajb', fock_a[:nc, :nc], d_ab_a)
                   + aa[:nc, :, :nc, :]).reshape(s1, s1)
    dvv = fab_b2[no:, no:] - fab_a2
    doo = fij_b2 - fij_a2[:-no, :-no]
    A[:s1, :s1] += (0.5 * (1 - np.sqrt((si + 1) / si) + 1 / (2 * si)) * e('ij,ab->iajb', d_ij, dvv)
                    + 0.5 * (-1 + np.sqrt((si + 1) / si) + 1 / (2 * si)) * e('ab,ij->iajb', d_ab, doo)
                    ).reshape(s1, s1)
    A_cv_ov = (e('ij,ab->iajb', d_ij_a[:nc, nc:nc + no], fock_a[nc + no:, nc + no:])
               - e('ij,ab->iajb', fock_a[:nc, nc:nc + no], d_ab_a)
               + aa[:nc, :, nc:nc + no, :]).reshape(s1, no * nv)
    A[:s1, s1:s2] = A_cv_ov
    A_cv_co = ab[:nc, :, :, :no].reshape(s1, nc * no)
    A[:s1, s2:s3] = A_cv_co
    A_cv_cvb = ab[:nc, :, :, no:no + nv].reshape(s1, s1).copy()
    A_cv_cvb -= (0.5 / (2 * si) * (e('ij,ab->iajb', d_ij, dvv) + e('ab,ij->iajb', d_ab, doo))).reshape(s1, s1)
    A[:s1, s3:] = A_cv_cvb
    A[s1:s2, :s1] = A_cv_ov.T
    A[s1:s2, s1:s2] = (e('ij,ab->iajb', d_ij_a[nc:nc + no, nc:nc + no], fock_a[nc + no:, nc + no:])
                       - e('ij,ab->iajb', fock_a[nc:nc + no, nc:nc + no], d_ab_a)
                       + aa[nc:nc + no, :, nc:nc + no, :]).reshape(no * nv, no * nv)
    A_ov_co = ab[nc:nc + no, :, :, :no].reshape(no * nv, nc * no)
    A[s1:s2, s2:s3] = A_ov_co
    A_ov_cvb = ab[nc:nc + no, :, :, no:no + nv].reshape(no * nv, s1)
    A[s1:s2, s3:] = A_ov_cvb
    A[s2:s3, :s1] = A_cv_co.T
    A[s2:s3, s1:s2] = A_ov_co.T
    A[s2:s3, s2:s3] = (e('ij,ab->iajb', d_ij_b, fock_b[nc:nc + no, nc:nc + no])
                       - e('ij,ab->iajb', fock_b[:nc, :nc], d_ab_b[:no, :no])
                       + bb[:, :no, :, :no]).reshape(nc * no, nc * no)
    A_co_cvb = (e('ij,ab->iajb', d_ij_b, fock_b[nc:nc + no, nc + no:])
                - e('ij,ab->iajb', fock_b[:nc, :nc], d_ab_b[:no, no:])
                + bb[:, :no, :, no:]).reshape(nc * no, s1)
    A[s2:s3, s3:] = A_co_cvb
    A[s3:, :s1] = A_cv_cvb.T
    A[s3:, s1:s2] = A_ov_cvb.T
    A[s3:, s2:s3] = A_co_cvb.T
    A[s3:, s3:] = (e('ij,ab->iajb', d_ij_b, fock_b[nc + no:, nc + no:])
                   - e('ij,ab->iajb', fock_b[:nc, :nc], d_ab_b[no:, no:])
                   + bb[:, no:, :, no:]).reshape(s1, s1)
    A[s3:, s3:] += (0.5 * (-1 + np.sqrt((si + 1) / si) + 1 / (2 * si)) * e('ij,ab->iajb', d_ij, dvv)
                    + 0.5 * (1 - np.sqrt((si + 1) / si) + 1 / (2 * si)) * e('ab,ij->iajb', d_ab, doo)
                    ).reshape(s1, s1)
    return A
