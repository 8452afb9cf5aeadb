"""Multicollinear spin-flip XC kernel (oracle).  TEST INFRASTRUCTURE ONLY.

The reference's ``method=1`` (SF_TDA.py:855-1047, called from XSF_TDA.py:217-218,
1097-1098 and SF_TDA.py:218-219) delegates the kernel to the third-party library
``mcfun`` (Pu, Li, Sun et al.; unpinned in the reference, absent here), through
``numint2c.NumInt2C`` with ``collinear='mcol'``.  This module restates:

* ``make_paxis_samples``      -- mcfun's principal-axis samples: Gauss-Legendre
                                 nodes / weights mapped to [0, 1].
* ``eval_xc_eff_sf``          -- mcfun ``eval_xc_eff_sf`` for deriv = 2 (the published
                                 multicollinear spin-flip kernel): with the collinear
                                 functional e(rho_t, s) in (total, spin) variables,
                                 E^MC[rho, m] = int dOmega/4pi (e + s . de/ds)(rho, n.m);
                                 its transverse second derivative at a collinear
                                 reference is  f_sf[x, y] = int_0^1 dt d2e/ds_x ds_y (rho, t s)
                                 over every spin variable (s, grad s[, tau_s]).  The
                                 functional is evaluated in (alpha, beta) variables and
                                 its derivatives rotated to (t, s) as PySCF's
                                 ``xc_deriv.ud2ts`` does (SF_TDA.py:907-912).
* ``cache_xc_kernel_sf_mc``   -- SF_TDA.py:942-974: rho_tmz = 1e-11 + (rho_a + rho_b,
                                 rho_a - rho_b) on every component, then the kernel above.
* ``nr_uks_fxc_sf_tda_mc``    -- SF_TDA.py:976-1047: ``wv = einsum('bg,abg->ag', rho1sf,
                                 2 fxc) * w``, then PySCF's GGA / MGGA potential assembly.
* ``sf_mc_block``             -- the multicollinear XC block of the explicit matrix
                                 ``get_ab_sf`` (SF_TDA.py:1179-1272).

Parity of the whole kernel is pinned by the reference's stored multicollinear runs
(example/XSF_TDA.ipynb cells 3 and 7, tests/test_qc.py).
"""
from __future__ import annotations

import numpy as np

from .engines import GRID_BLOCK, _eval_rho, _wv_to_vmat

NCOMP = {"LDA": 1, "GGA": 4, "MGGA": 5}


def make_paxis_samples(n):
    """Samples on the principal axis between [0, 1] (Gauss-Legendre)."""
    t, w = np.polynomial.legendre.leggauss(n)
    return 0.5 * t + 0.5, 0.5 * w


def ud2ts_fxc(f):
    """(2, n, 2, n, g) second derivatives in (alpha, beta) variables -> (total, spin),
    rho_a = (t + s) / 2, rho_b = (t - s) / 2 on every component."""
    u = 0.5 * np.array([[1.0, 1.0], [1.0, -1.0]])      # d(rho_a, rho_b) / d(t, s)
    return np.einsum('ia,axbyg,jb->ixjyg', u, f, u)


def eval_xc_eff_sf(eval_xc, rho_tmz, collinear_samples):
    """fxc_sf (nvar, nvar, ngrid) of the multicollinear kernel; rho_tmz (2, nvar, ngrid)
    = (total density, m_z) and their derivatives; eval_xc(rho_ud, deriv) returns
    (exc, vxc, fxc) of the collinear functional on (2, nvar, ngrid) spin densities."""
    rho_tmz = np.asarray(rho_tmz, dtype=np.float64)
    nvar, ng = rho_tmz.shape[1], rho_tmz.shape[2]
    ts, ws = make_paxis_samples(collinear_samples)
    out = np.zeros((nvar, nvar, ng))
    nb = max(1, (1 << 20) // max(ng, 1))          # samples per functional call
    for k0 in range(0, len(ts), nb):
        t = ts[k0:k0 + nb]
        tot = np.repeat(rho_tmz[0][:, None, :], len(t), axis=1)
        spin = rho_tmz[1][:, None, :] * t[None, :, None]
        rho_ud = np.asarray([0.5 * (tot + spin), 0.5 * (tot - spin)]).reshape(2, nvar, -1)
        f = eval_xc(rho_ud, 2)[2].reshape(2, nvar, 2, nvar, len(t), ng)
        for j in range(len(t)):
            out += ws[k0 + j] * ud2ts_fxc(f[..., j, :])[1, :, 1, :]
    return out


def cache_xc_kernel_sf_mc(eval_xc, rho_ab, collinear_samples):
    """SF_TDA.py:942-974 from the SCF spin densities rho_ab (2, nvar, ngrid)."""
    rho_ab = np.asarray(rho_ab, dtype=np.float64)
    rho_tmz = np.zeros_like(rho_ab) + 1e-11
    rho_tmz[0] += rho_ab[0] + rho_ab[1]
    rho_tmz[1] += rho_ab[0] - rho_ab[1]
    return eval_xc_eff_sf(eval_xc, rho_tmz, collinear_samples)


def nr_uks_fxc_sf_tda_mc(mf, fxc_mc, dms):
    """SF_TDA.py:976-1047: V for spin-flip transition densities dms (nz, nao, nao)."""
    xctype = mf.xctype
    dms = np.asarray(dms)
    nz, nao = dms.shape[0], dms.shape[-1]
    vmat = np.zeros((nz, nao, nao))
    ng = mf.grids.ngrid
    for g0 in range(0, ng, GRID_BLOCK):
        g1 = min(ng, g0 + GRID_BLOCK)
        ao = mf.grids.ao[:min(NCOMP[xctype], 4), g0:g1]
        w = mf.grids.weights[g0:g1]
        f = fxc_mc[..., g0:g1]
        for i in range(nz):
            rho1 = _eval_rho(ao, dms[i], xctype)
            if xctype == 'LDA':
                wv = (rho1[0] * f[0, 0] * 2.0 * w)[None]
            else:
                wv = np.einsum('bg,abg->ag', rho1, f * 2.0) * w
            vmat[i] += _wv_to_vmat(ao, wv, xctype)
    return vmat


def _rho_ov(ao, orbo, orbv, xctype):
    """Transition densities phi_i phi_a (+ gradients, + tau) on a grid block (SF_TDA.py:1214-1260)."""
    if xctype == 'LDA':
        return np.einsum('ri,ra->ria', ao[0] @ orbo, ao[0] @ orbv)[None]
    ro = np.einsum('xrp,pi->xri', ao[:4], orbo)
    rv = np.einsum('xrp,pi->xri', ao[:4], orbv)
    r = np.einsum('xri,ra->xria', ro, rv[0])
    r[1:4] += np.einsum('ri,xra->xria', ro[0], rv[1:4])
    if xctype == 'MGGA':
        tau = 0.5 * np.einsum('xri,xra->ria', ro[1:4], rv[1:4])
        r = np.concatenate([r, tau[None]])
    return r


def sf_mc_block(mf, fxc_mc, orbo, orbv):
    """sum_g rho_ov[x] (2 w fxc[x, y]) rho_ov[y] -> (no, nv, no, nv) (SF_TDA.py:1179-1272)."""
    xctype = mf.xctype
    no, nv = orbo.shape[1], orbv.shape[1]
    out = np.zeros((no, nv, no, nv))
    ng = mf.grids.ngrid
    for g0 in range(0, ng, GRID_BLOCK):
        g1 = min(ng, g0 + GRID_BLOCK)
        ao = mf.grids.ao[:, g0:g1]
        w = mf.grids.weights[g0:g1]
        r = _rho_ov(ao, orbo, orbv, xctype)
        wf = fxc_mc[..., g0:g1] * w * 2.0
        w_ov = np.einsum('xyr,xria->yria', wf, r)
        out += np.einsum('xria,xrjb->iajb', w_ov, r, optimize=True)
    return out
