"""Multicollinear spin-flip XC kernel (the reference's ``method=1``).

Replaces ``cache_xc_kernel_sf_mc`` (SF_TDA.py:942-974), which evaluates the
third-party ``mcfun.eval_xc_eff_sf`` through PySCF's ``NumInt2C(collinear='mcol')``
(SF_TDA.py:865-867, 914-939).  The multicollinear functional of a collinear
functional e(rho_t, s) (total / spin variables) is

    E^MC[rho, m] = int dOmega/4pi  (e + s . de/ds)(rho, n . m),

and its transverse (spin-flip) second derivative at the collinear SCF density is

    fxc_sf[x, y](r) = int_0^1 dt  d2e / ds_x ds_y (rho(r), t s(r))

over every spin variable x, y of the functional (s, grad s for GGA, + tau_s for
MGGA), integrated with ``collinear_samples`` Gauss-Legendre points on [0, 1]
(mcfun's principal-axis samples).  The result is the un-weighted (nk, nk, ngrid)
kernel that ``nr_uks_fxc_sf_tda_mc`` contracts as ``wv = einsum('bg,abg->ag',
rho1sf, 2 fxc) * w`` (SF_TDA.py:997-1003) -- on the device, the GGA / MGGA
response engine with one spin-flip channel (``xt_desc.sf_kernel = XT_SF_MC``).

This is once-per-solve setup (the ``cache_xc_kernel`` analogue), evaluated with the
functional library of ``xtddft_amd.qc.xc`` by autograd, all samples of a grid
block in one batch, on the GPU when one is present.  Sample counts follow the
reference's call sites: XSF_TDA ``collinear_samples`` (default 60, XSF_TDA.py:147,
217-218, 302), the module-level SF-TDA Davidson path 50 (SF_TDA.py:219), the
explicit matrix ``get_ab_sf`` 30 (SF_TDA.py:1051).
"""
from __future__ import annotations

import numpy as np

RHO_SHIFT = 1e-11      # SF_TDA.py:969: added to every component of (rho_t, m_z)
NCOMP = {"LDA": 1, "GGA": 4, "MGGA": 5}


def _torch_device(mf, device):
    import torch
    ao = mf.grids.ao
    if isinstance(ao, torch.Tensor) and ao.is_cuda:
        return ao.device
    if device is not None and torch.cuda.is_available():
        return torch.device(f"cuda:{device}")
    return torch.device("cpu")


def ground_state_rho(mf, dev):
    """(2, nk, ngrid) spin densities (rho, grad rho[, tau]) of the SCF density on the grid
    (``ni.eval_rho2`` of each spin's occupied orbitals, SF_TDA.py:963-966)."""
    import torch
    nk = NCOMP[mf.xctype]
    ao = torch.as_tensor(mf.grids.ao, device=dev)
    dms = torch.as_tensor(np.asarray(mf.make_rdm1()), device=dev)
    out = []
    for s in range(2):
        c0 = ao[0] @ dms[s]
        comps = [(ao[0] * c0).sum(1)]
        if nk >= 4:
            comps += [2.0 * (ao[k] * c0).sum(1) for k in range(1, 4)]
        if nk == 5:
            comps.append(0.5 * sum((ao[k] * (ao[k] @ dms[s])).sum(1) for k in range(1, 4)))
        out.append(torch.stack(comps))
    return torch.stack(out)


def sf_mc_kernel(mf, collinear_samples: int = 60, device=None, max_points: int = 1 << 21, rho=None):
    """The multicollinear kernel fxc_sf (nk, nk, ngrid) of mean field ``mf``.

    ``mf.fxc_sf_mc`` when set (synthetic problems); otherwise computed from the SCF
    density and cached in ``mf.extra`` per sample count and orbital set (the cache is
    keyed on the identity of ``mo_coeff`` / ``mo_occ``: a mean field copied with new
    orbitals shares ``extra`` but not the kernel), or from the given spin densities
    ``rho`` (2, nk, ngrid), never cached.  Returns a host array, or a device tensor when
    the grid's AO values live in HBM.
    """
    import torch
    from .qc import xc as _xc
    if mf.fxc_sf_mc is not None:
        return mf.fxc_sf_mc
    if mf.xctype == "HF":
        return None
    key = ("fxc_sf_mc", int(collinear_samples))
    ident = (id(mf.mo_coeff), id(mf.mo_occ))
    cache = rho is None
    if cache and key in mf.extra and mf.extra.get(key + ("orbitals",)) == ident:
        return mf.extra[key]
    dev = _torch_device(mf, device)
    rho = ground_state_rho(mf, dev) if rho is None else torch.as_tensor(rho, device=dev)
    nk, ng = rho.shape[1], rho.shape[2]
    tot = rho[0] + rho[1] + RHO_SHIFT
    spin = rho[0] - rho[1] + RHO_SHIFT
    t, w = np.polynomial.legendre.leggauss(int(collinear_samples))
    t, w = 0.5 * t + 0.5, 0.5 * w
    out = torch.zeros((nk, nk, ng), dtype=torch.float64, device=dev)
    gb = max(1, min(ng, max_points))                       # grid points per batch
    sb = max(1, min(len(t), max_points // gb))              # samples per batch
    for g0 in range(0, ng, gb):
        g1 = min(ng, g0 + gb)
        tt, ss = tot[:, g0:g1], spin[:, g0:g1]
        for k0 in range(0, len(t), sb):
            k1 = min(len(t), k0 + sb)
            tk = torch.as_tensor(t[k0:k1], dtype=torch.float64, device=dev)
            sk = ss[:, None, :] * tk[None, :, None]                       # (nk, ns, g)
            ud = torch.stack([0.5 * (tt[:, None, :] + sk), 0.5 * (tt[:, None, :] - sk)])
            f = _xc.eval_xc_eff_torch(mf.xc, ud.reshape(2, nk, -1), deriv=2)[2]
            f = f.reshape(2, nk, 2, nk, k1 - k0, g1 - g0)
            # d2e/ds ds in (t, s) variables: rho_a = (t + s)/2, rho_b = (t - s)/2
            fss = 0.25 * (f[0, :, 0] - f[0, :, 1] - f[1, :, 0] + f[1, :, 1])
            wk = torch.as_tensor(w[k0:k1], dtype=torch.float64, device=dev)
            out[:, :, g0:g1] += torch.einsum("xyng,n->xyg", fss, wk)
    out = 0.5 * (out + out.transpose(0, 1))      # exact symmetry (the (t, s) rotation's round-off)
    ao = mf.grids.ao
    res = out if (isinstance(ao, torch.Tensor) and ao.is_cuda) else out.cpu().numpy()
    if cache:
        mf.extra[key] = res
        mf.extra[key + ("orbitals",)] = ident
    return res
