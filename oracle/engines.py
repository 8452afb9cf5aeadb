"""AO-route response engines (oracle).  TEST INFRASTRUCTURE ONLY.

Restates what PySCF computes inside the reference's ``vresp`` closures:

* ``get_jk``  -- ``mf.get_jk / get_j / get_k`` with the density-fitted ERI
  ``(mu nu|la si) = sum_P B[P,mu,nu] B[P,la,si]`` in PySCF's convention
  ``vk = einsum('ijkl,jk->il', eri, dm)`` (call sites XTDA.py:518-543,
  SF_TDA.py:273-281, XSF_TDA.py:996).
* ``nr_uks_fxc`` -- ``ni.nr_uks_fxc`` for hermi=0 densities (XTDA.py:514):
  rho1 from ``eval_rho`` (GGA gradient terms both ways for non-hermitian dm; MGGA
  tau1 = 1/2 sum_c d_c phi D d_c phi, V += 1/2 sum_c d_c phi^T w_tau d_c phi),
  ``wv = w * einsum('axg,axbyg->byg', rho1, fxc)``, then for GGA
  ``wv[0]*=.5; V = ao0^T (sum_y ao_y wv_y); V += V^T``.
* ``nr_uks_fxc_sf_tda`` -- the reference's own ALDA0 spin-flip kernel
  (SF_TDA.py:90-160): density-only rho1, ``wv = rho1 * fxc_sf`` (weighted).
* ``gen_response`` (XTDA.py:482-556) and ``gen_response_sf``
  (SF_TDA.py:246-286) closures built on those.
"""
from __future__ import annotations

import numpy as np

GRID_BLOCK = 8192


def _k_coeffs(mf):
    """(c_full, c_lr) such that vk = c_full*K(B) + c_lr*K(B_lr) (XTDA.py:522-539)."""
    omega, alpha, hyb = mf.omega, mf.alpha, mf.hyb
    if omega == 0:
        return hyb, 0.0
    if mf.cderi_lr is None:
        raise ValueError("range-separated hybrid needs cderi_lr")
    if alpha == 0:      # SR only: K_sr = K - K_lr
        return hyb, -hyb
    if hyb == 0:        # LR only
        return 0.0, alpha
    return hyb, alpha - hyb


def get_jk(cderi, dms, with_j=True, with_k=True):
    """J[D] = sum_P B_P <B_P, D>;  K[D] = sum_P B_P D B_P  (dms: (..., nao, nao))."""
    dms = np.asarray(dms, dtype=np.float64)
    shape = dms.shape
    d = dms.reshape(-1, shape[-2], shape[-1])
    vj = vk = None
    if with_j:
        gam = np.einsum('pmn,xmn->xp', cderi, d, optimize=True)
        vj = np.einsum('xp,pmn->xmn', gam, cderi, optimize=True).reshape(shape)
    if with_k:
        # chunked over P so the (P, nao, nao) intermediate stays bounded at large naux
        naux, nao = cderi.shape[0], shape[-1]
        pc = max(1, min(naux, (1 << 29) // (8 * nao * nao)))
        vk = np.zeros_like(d)
        for x in range(d.shape[0]):
            for p0 in range(0, naux, pc):
                b = cderi[p0:p0 + pc]
                # B_P D for the whole chunk as one GEMM, then sum_P (B_P D) B_P
                t = (b.reshape(-1, nao) @ d[x]).reshape(b.shape)
                for q in range(b.shape[0]):
                    vk[x] += t[q] @ b[q]
        vk = vk.reshape(shape)
    return vj, vk


def unpack_eri_s8(packed, nao):
    """PySCF 8-fold packed ERIs -> full (nao,)*4, written out with explicit
    loops over the pair indices (ao2mo.restore(1, eri, nao) semantics):
    ij = i(i+1)/2 + j (i >= j), (ij|kl) at ij(ij+1)/2 + kl (ij >= kl)."""
    full = np.empty((nao, nao, nao, nao))
    pairs = [(i, j) for i in range(nao) for j in range(i + 1)]
    for ij, (i, j) in enumerate(pairs):
        for kl, (k, l) in enumerate(pairs[:ij + 1]):
            v = packed[ij * (ij + 1) // 2 + kl]
            for a, b in ((i, j), (j, i)):
                for c, d in ((k, l), (l, k)):
                    full[a, b, c, d] = v
                    full[c, d, a, b] = v
    return full


def get_jk_eri(eri_full, dms, with_j=True, with_k=True, eri_k=None):
    """PySCF incore get_jk convention on a full 4-index tensor:
    vj = einsum('ijkl,kl->ij', eri, dm), vk = einsum('ijkl,jk->il', eri, dm),
    as matrix products over the pair index (eri_k: the (i,l),(j,k) re-layout,
    built here when not cached by the caller)."""
    dms = np.asarray(dms, dtype=np.float64)
    shape = dms.shape
    n = shape[-1]
    d = dms.reshape(-1, n * n)
    vj = vk = None
    if with_j:
        vj = (eri_full.reshape(n * n, n * n) @ d.T).T.reshape(shape)
    if with_k:
        if eri_k is None:
            eri_k = eri_k_layout(eri_full)
        vk = (eri_k @ d.T).T.reshape(shape)
    return vj, vk


def eri_k_layout(eri_full):
    """(i l),(j k) matrix of (ij|kl) for the exchange contraction."""
    n = eri_full.shape[0]
    return np.ascontiguousarray(eri_full.transpose(0, 3, 1, 2)).reshape(n * n, n * n)


def eri_full_from_cderi(cderi):
    """(ij|kl) = sum_P B[P,i,j] B[P,k,l] as a full 4-index array."""
    naux, n, _ = cderi.shape
    b = cderi.reshape(naux, n * n)
    return (b.T @ b).reshape(n, n, n, n)


def jk(mf, dms, with_j=True, with_k=True, lr=False):
    """get_jk on the mean field's J/K model: stored 4-index ERIs when the caller
    attached them (mf.extra['eri_full'], the incore mf._eri route), else the
    DF factor."""
    key = "eri_full_lr" if lr else "eri_full"
    eri = mf.extra.get(key) if getattr(mf, "extra", None) else None
    if eri is None:
        return get_jk(mf.cderi_lr if lr else mf.cderi, dms, with_j, with_k)
    kk = key + "_k"
    if with_k and kk not in mf.extra:
        mf.extra[kk] = eri_k_layout(eri)
    return get_jk_eri(eri, dms, with_j, with_k, eri_k=mf.extra.get(kk))


def get_k_total(mf, dms):
    """Exchange with the functional's hybrid coefficients (already scaled)."""
    c_full, c_lr = _k_coeffs(mf)
    vk = np.zeros_like(np.asarray(dms, dtype=np.float64))
    if c_full != 0:
        vk += c_full * jk(mf, dms, with_j=False)[1]
    if c_lr != 0:
        vk += c_lr * jk(mf, dms, with_j=False, lr=True)[1]
    return vk


def _eval_rho(ao, dm, xctype):
    """PySCF eval_rho for a non-hermitian dm (hermi=0); MGGA adds
    tau = 1/2 sum_c sum_pq d_c phi_p D_pq d_c phi_q."""
    c0 = ao[0] @ dm                       # c0[g,q] = sum_p phi_p D_pq
    rho0 = np.einsum('gq,gq->g', ao[0], c0)
    if xctype == 'LDA':
        return rho0[None]
    c1 = ao[0] @ dm.T                     # c1[g,q] = sum_p phi_p D_qp
    rho = np.empty((5 if xctype == 'MGGA' else 4, ao.shape[1]))
    rho[0] = rho0
    for i in range(1, 4):
        rho[i] = np.einsum('gq,gq->g', ao[i], c0) + np.einsum('gq,gq->g', c1, ao[i])
    if xctype == 'MGGA':
        rho[4] = 0.5 * sum(np.einsum('gq,gq->g', ao[i] @ dm, ao[i]) for i in range(1, 4))
    return rho


def _wv_to_vmat(ao, wv, xctype):
    """V_mu,nu from weighted potential wv (PySCF _dot_ao_ao / hermi_sum for GGA;
    MGGA adds 1/2 sum_c d_c phi^T w_tau d_c phi)."""
    if xctype == 'LDA':
        return ao[0].T @ (wv[0][:, None] * ao[0])
    wv = wv.copy()
    wv[0] *= .5
    aow = np.einsum('yg,ygq->gq', wv[:4], ao[:4])
    v = ao[0].T @ aow
    v = v + v.T
    if xctype == 'MGGA':
        for i in range(1, 4):
            v += 0.5 * ao[i].T @ (wv[4][:, None] * ao[i])
    return v


def nr_uks_fxc(mf, dms):
    """UKS XC response V[s] for densities dms (2, nz, nao, nao), hermi=0."""
    grids, fxc, xctype = mf.grids, mf.fxc, mf.xctype
    dms = np.asarray(dms)
    nz, nao = dms.shape[1], dms.shape[-1]
    ncomp = {'LDA': 1, 'GGA': 4, 'MGGA': 5}[xctype]
    nao_c = min(ncomp, 4)                 # AO values + gradients (tau needs no more)
    vmat = np.zeros((2, nz, nao, nao))
    ng = grids.ngrid
    for g0 in range(0, ng, GRID_BLOCK):
        g1 = min(ng, g0 + GRID_BLOCK)
        ao = grids.ao[:nao_c, g0:g1]
        w = grids.weights[g0:g1]
        f = fxc[:, :ncomp, :, :ncomp, g0:g1]
        for i in range(nz):
            rho1 = np.asarray([_eval_rho(ao, dms[s, i], xctype) for s in range(2)])
            wv = np.einsum('axg,axbyg->byg', rho1, f) * w
            for s in range(2):
                vmat[s, i] += _wv_to_vmat(ao, wv[s], xctype)
    return vmat


def nr_uks_fxc_sf_tda(mf, dms):
    """ALDA0 spin-flip XC response (SF_TDA.py:90-160); dms (nz, nao, nao)."""
    grids, vxc = mf.grids, mf.fxc_sf
    dms = np.asarray(dms)
    nz, nao = dms.shape[0], dms.shape[-1]
    vmat = np.zeros((nz, nao, nao))
    ng = grids.ngrid
    for g0 in range(0, ng, GRID_BLOCK):
        g1 = min(ng, g0 + GRID_BLOCK)
        ao0 = grids.ao[0, g0:g1]
        v = vxc[g0:g1]
        for i in range(nz):
            rho1 = np.einsum('gp,pq,gq->g', ao0, dms[i], ao0, optimize=True)
            wv = rho1 * v
            # LDA: _dot_ao_ao(ao, ao, wv); GGA: wv[0]*=.5, ao0^T(ao0 wv) + h.c. == same
            vmat[i] += ao0.T @ (wv[:, None] * ao0)
    return vmat


def gen_response(mf, with_j=True):
    """Restates XTDA.gen_response (XTDA.py:482-556) for hermi=0."""
    def vind(dm1):
        dm1 = np.asarray(dm1, dtype=np.float64)
        if mf.xctype == 'HF':
            vj, vk = jk(mf, dm1)
            return vj[0] + vj[1] - vk
        v1 = nr_uks_fxc(mf, dm1)
        hybrid = (mf.hyb != 0) or (mf.omega != 0)
        if not hybrid:
            if with_j:
                vj = jk(mf, dm1, with_k=False)[0]
                v1 += vj[0] + vj[1]
            return v1
        vk = get_k_total(mf, dm1)
        if with_j:
            vj = jk(mf, dm1, with_k=False)[0]
            v1 += vj[0] + vj[1] - vk
        else:
            v1 -= vk
        return v1
    return vind


def gen_response_sf(mf, method=0):
    """Restates SF_TDA.gen_response_sf (SF_TDA.py:246-286): no J in spin flip.
    method 1: the multicollinear response of _gen_uhf_tda_response_sf (SF_TDA.py:855-904)
    with the kernel mf.fxc_sf_mc (oracle.mcol.cache_xc_kernel_sf_mc)."""
    if method == 1 and mf.xctype != 'HF' and mf.fxc_sf_mc is None:
        raise ValueError("method 1 needs mf.fxc_sf_mc (the multicollinear kernel)")

    def vind(dm1):
        dm1 = np.asarray(dm1, dtype=np.float64)
        if mf.xctype == 'HF':
            return -jk(mf, dm1, with_j=False)[1]
        if method == 0:
            v1 = nr_uks_fxc_sf_tda(mf, dm1)
        elif method == 1:
            from .mcol import nr_uks_fxc_sf_tda_mc
            v1 = nr_uks_fxc_sf_tda_mc(mf, mf.fxc_sf_mc, dm1)
        else:
            v1 = np.zeros_like(dm1)
        hybrid = (mf.hyb != 0) or (mf.omega != 0)
        if hybrid:
            vk = mf.hyb * jk(mf, dm1, with_j=False)[1]
            if mf.omega > 1e-10:
                vk += (mf.alpha - mf.hyb) * jk(mf, dm1, with_j=False, lr=True)[1]
            v1 -= vk
        return v1
    return vind
