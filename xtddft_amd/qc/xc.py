"""Exchange-correlation functionals with first and second derivatives.

Replaces the libxc calls on the reference's path (``ni.eval_xc_eff``,
``SF_TDA.py:81``; ``ni.cache_xc_kernel``, ``XTDA.py:504``): energy density,
``vxc`` (2, 4, ngrid) and ``fxc`` (2, 4, 2, 4, ngrid) with respect to
(rho_s, grad rho_s) -- PySCF's ``eval_xc_eff`` layout for spin-polarised GGA
(the LDA layout is (2, 1, ngrid) / (2, 1, 2, 1, ngrid)).

The functionals are written as plain float64 torch expressions of
(rho_a, grad rho_a, rho_b, grad rho_b); derivatives come from autograd (exact
to round-off, no finite differences).  Forms follow libxc 7.0's definitions:

* Slater exchange   e = -(3/2)(3/4pi)^(1/3) sum_s rho_s^(4/3)
* B88 exchange      e = -sum_s rho_s^(4/3) [C_x + beta x_s^2 / (1 + 6 beta x_s asinh x_s)],
                    x_s = |grad rho_s| / rho_s^(4/3), beta = 0.0042
* LYP correlation   Miehlich-Savin-Stoll-Preuss form (CPL 157, 200 (1989)),
                    a = 0.04918, b = 0.132, c = 0.2533, d = 0.349
* VWN correlation   Vosko-Wilk-Nusair, Can. J. Phys. 58, 1200 (1980):
                    VWN5 (libxc LDA_C_VWN: paramagnetic / ferromagnetic / spin
                    stiffness fits, e = e_P + a_c f(z)(1 - z^4)/f''(0) + (e_F - e_P) f(z) z^4)
                    and VWN_RPA (libxc LDA_C_VWN_RPA: the RPA fits interpolated by
                    f(z) alone, e = e_P (1 - f(z)) + e_F f(z)).

Hybrids: BHandHLYP = 0.5 HF + 0.5 B88 + LYP (libxc HYB_GGA_XC_BHANDHLYP), the
reference's functional in every stored example (``example/XSF_TDA.ipynb``,
``spin up.ipynb``); B3LYP = 0.2 HF + 0.08 Slater + 0.72 B88 + 0.19 VWN_RPA +
0.81 LYP (libxc HYB_GGA_XC_B3LYP, which PySCF >= 2.3 calls B3LYP: the
reference's default functional, XTDA.py:1526, and the one of example/TDA.ipynb)
and B3LYP5 (same with VWN5); BLYP; SVWN (Slater + VWN5); HF (no DFT part).
Points whose total density is below ``DENS_THRESHOLD`` contribute nothing
(libxc's density screening).  The stored reference outputs pin BHandHLYP only
(B3LYP's example needs cc-pVDZ, not available offline): VWN is unpinned.
"""
from __future__ import annotations

import math

import numpy as np

DENS_THRESHOLD = 1e-14

_CX = 1.5 * (3.0 / (4.0 * math.pi)) ** (1.0 / 3.0)

# name -> (list of (component, coefficient), hybrid fraction, xctype)
_FUNCTIONALS = {
    "HF": ([], 1.0, "HF"),
    "SLATER": ([("slater", 1.0)], 0.0, "LDA"),
    "B88": ([("b88", 1.0)], 0.0, "GGA"),
    "BLYP": ([("b88", 1.0), ("lyp", 1.0)], 0.0, "GGA"),
    "BHANDHLYP": ([("b88", 0.5), ("lyp", 1.0)], 0.5, "GGA"),
    "SVWN": ([("slater", 1.0), ("vwn5", 1.0)], 0.0, "LDA"),
    "B3LYP": ([("slater", 0.08), ("b88", 0.72), ("vwn_rpa", 0.19), ("lyp", 0.81)], 0.2, "GGA"),
    "B3LYPG": ([("slater", 0.08), ("b88", 0.72), ("vwn_rpa", 0.19), ("lyp", 0.81)], 0.2, "GGA"),
    "B3LYP5": ([("slater", 0.08), ("b88", 0.72), ("vwn5", 0.19), ("lyp", 0.81)], 0.2, "GGA"),
}


def parse_xc(xc: str):
    """(components, hyb, xctype); ``rsh_and_hybrid_coeff`` gives (0, hyb, hyb) for these."""
    key = xc.upper().replace("-", "").replace(" ", "")
    if key not in _FUNCTIONALS:
        raise KeyError(f"functional {xc!r} not implemented (available: {sorted(_FUNCTIONALS)})")
    return _FUNCTIONALS[key]


def rsh_and_hybrid_coeff(xc: str):
    """(omega, alpha, hyb) as PySCF returns them for a global hybrid
    (the reference prints "Omega, alpha, hyb 0.0 0.5 0.5" for BHandHLYP)."""
    _, hyb, _ = parse_xc(xc)
    return 0.0, hyb, hyb


def xc_type(xc: str) -> str:
    return parse_xc(xc)[2]


# ----------------------------------------------------------------- pieces
def _x_asinh_x(y, torch):
    """sqrt(y) asinh(sqrt(y)) as a smooth function of y = x^2 >= 0."""
    big = y > 1e-6
    ys = torch.where(big, y, torch.ones_like(y))
    sq = torch.sqrt(ys)
    direct = sq * torch.asinh(sq)
    ysm = torch.where(big, torch.zeros_like(y), y)
    series = ysm - ysm * ysm / 6.0 + 3.0 * ysm ** 3 / 40.0
    return torch.where(big, direct, series)


def _slater(ra, rb, saa, sab, sbb, torch):
    return -_CX * (ra ** (4.0 / 3.0) + rb ** (4.0 / 3.0))


def _b88(ra, rb, saa, sab, sbb, torch):
    beta = 0.0042
    out = 0.0
    for r, s in ((ra, saa), (rb, sbb)):
        r43 = r ** (4.0 / 3.0)
        y = s / (r43 * r43)
        out = out - r43 * (_CX + beta * y / (1.0 + 6.0 * beta * _x_asinh_x(y, torch)))
    return out


def _lyp(ra, rb, saa, sab, sbb, torch):
    a, b, c, d = 0.04918, 0.132, 0.2533, 0.349
    rho = ra + rb
    rm13 = rho ** (-1.0 / 3.0)
    dd = 1.0 + d * rm13
    omega = torch.exp(-c * rm13) / dd * rho ** (-11.0 / 3.0)
    delta = c * rm13 + d * rm13 / dd
    cf = 0.3 * (3.0 * math.pi ** 2) ** (2.0 / 3.0)
    s = saa + 2.0 * sab + sbb
    t1 = -a * 4.0 / dd * ra * rb / rho
    inner = (2.0 ** (11.0 / 3.0) * cf * (ra ** (8.0 / 3.0) + rb ** (8.0 / 3.0))
             + (47.0 / 18.0 - 7.0 / 18.0 * delta) * s
             - (2.5 - delta / 18.0) * (saa + sbb)
             - (delta - 11.0) / 9.0 * (ra / rho * saa + rb / rho * sbb))
    br = (ra * rb * inner - 2.0 / 3.0 * rho * rho * s
          + (2.0 / 3.0 * rho * rho - ra * ra) * sbb + (2.0 / 3.0 * rho * rho - rb * rb) * saa)
    return t1 - a * b * omega * br


# VWN fits (A in Hartree): index 0 paramagnetic, 1 ferromagnetic, 2 spin stiffness
_VWN5 = dict(A=(0.0310907, 0.01554535, -1.0 / (6.0 * math.pi ** 2)), b=(3.72744, 7.06042, 1.13107),
             c=(12.9352, 18.0578, 13.0045), x0=(-0.10498, -0.32500, -0.0047584))
_VWN_RPA = dict(A=(0.0310907, 0.01554535, -1.0 / (6.0 * math.pi ** 2)), b=(13.0720, 20.1231, 1.06835),
                c=(42.7198, 101.578, 11.4813), x0=(-0.409286, -0.743294, -0.228344))
_FPP = 4.0 / (9.0 * (2.0 ** (1.0 / 3.0) - 1.0))           # f''(0)


def _vwn_fit(prm, i, x, torch):
    """VWN interpolation formula (eq. 4.4 of the paper) in x = sqrt(rs)."""
    A, b, c, x0 = prm["A"][i], prm["b"][i], prm["c"][i], prm["x0"][i]
    q = math.sqrt(4.0 * c - b * b)
    X = x * x + b * x + c
    X0 = x0 * x0 + b * x0 + c
    at = torch.atan(q / (2.0 * x + b))
    return A * (torch.log(x * x / X) + 2.0 * b / q * at
                - b * x0 / X0 * (torch.log((x - x0) ** 2 / X) + 2.0 * (b + 2.0 * x0) / q * at))


def _vwn_parts(ra, rb, torch):
    rho = ra + rb
    x = (3.0 / (4.0 * math.pi * rho)) ** (1.0 / 6.0)
    z = (ra - rb) / rho
    fz = ((1.0 + z) ** (4.0 / 3.0) + (1.0 - z) ** (4.0 / 3.0) - 2.0) / (2.0 ** (4.0 / 3.0) - 2.0)
    return rho, x, z, fz


def _vwn5(ra, rb, saa, sab, sbb, torch):
    rho, x, z, fz = _vwn_parts(ra, rb, torch)
    ep, ef = _vwn_fit(_VWN5, 0, x, torch), _vwn_fit(_VWN5, 1, x, torch)
    ac = _vwn_fit(_VWN5, 2, x, torch)
    z4 = z ** 4
    return rho * (ep + ac * fz * (1.0 - z4) / _FPP + (ef - ep) * fz * z4)


def _vwn_rpa(ra, rb, saa, sab, sbb, torch):
    rho, x, z, fz = _vwn_parts(ra, rb, torch)
    ep, ef = _vwn_fit(_VWN_RPA, 0, x, torch), _vwn_fit(_VWN_RPA, 1, x, torch)
    return rho * (ep * (1.0 - fz) + ef * fz)


_PIECES = {"slater": _slater, "b88": _b88, "lyp": _lyp, "vwn5": _vwn5, "vwn_rpa": _vwn_rpa}


def eval_xc_eff(xc: str, rho: np.ndarray, deriv: int = 1):
    """Spin-polarised XC on a grid.

    rho : (2, 4, ngrid) for GGA (rho, d/dx, d/dy, d/dz per spin) or (2, ngrid) /
          (2, 1, ngrid) for LDA.
    Returns (exc, vxc, fxc): exc (ngrid,) energy per particle, vxc (2, ncomp, ngrid),
    fxc (2, ncomp, 2, ncomp, ngrid) or None when deriv < 2.
    """
    import torch
    nthreads = torch.get_num_threads()
    torch.set_num_threads(1)       # element-wise graphs: intra-op threading only adds overhead
    try:
        return _eval_xc_eff(torch, xc, rho, deriv)
    finally:
        torch.set_num_threads(nthreads)


def _eval_xc_eff(torch, xc, rho, deriv):
    comps, _, xctype = parse_xc(xc)
    rho = np.asarray(rho, dtype=np.float64)
    if rho.ndim == 2:
        rho = rho[:, None, :]
    ncomp = 4 if xctype == "GGA" else 1
    ng = rho.shape[-1]
    exc = np.zeros(ng)
    vxc = np.zeros((2, ncomp, ng))
    fxc = np.zeros((2, ncomp, 2, ncomp, ng)) if deriv >= 2 else None
    if not comps:
        return exc, vxc, fxc
    rtot = rho[0, 0] + rho[1, 0]
    mask = rtot > DENS_THRESHOLD
    if not np.any(mask):
        return exc, vxc, fxc
    x = torch.tensor(rho[:, :ncomp, mask].reshape(2 * ncomp, -1), dtype=torch.float64,
                     requires_grad=True)
    rs = x.reshape(2, ncomp, -1)
    ra = torch.clamp(rs[0, 0], min=1e-30)
    rb = torch.clamp(rs[1, 0], min=1e-30)
    if ncomp == 4:
        ga, gb = rs[0, 1:], rs[1, 1:]
        saa = (ga * ga).sum(0)
        sab = (ga * gb).sum(0)
        sbb = (gb * gb).sum(0)
    else:
        saa = sab = sbb = torch.zeros_like(ra)
    eps = 0.0
    for name, coef in comps:
        eps = eps + coef * _PIECES[name](ra, rb, saa, sab, sbb, torch)
    g = torch.autograd.grad(eps.sum(), x, create_graph=deriv >= 2)[0]
    exc[mask] = (eps / (ra + rb)).detach().numpy()
    vxc[:, :, mask] = g.detach().numpy().reshape(2, ncomp, -1)
    if deriv >= 2:
        n = 2 * ncomp
        H = np.empty((n, n, int(mask.sum())))
        for k in range(n):
            H[k] = torch.autograd.grad(g[k].sum(), x, retain_graph=k < n - 1)[0].numpy()
        H = 0.5 * (H + H.transpose(1, 0, 2))       # exact symmetry (autograd round-off)
        fxc[..., mask] = H.reshape(2, ncomp, 2, ncomp, -1)
    return exc, vxc, fxc


def eval_xc_eff_torch(xc: str, rho, deriv: int = 1):
    """``eval_xc_eff`` on a torch tensor rho (2, ncomp, ngrid) wherever it lives
    (the device SCF engine evaluates the functional on the GPU): returns torch
    (exc (ngrid,), vxc (2, ncomp, ngrid), fxc (2, ncomp, 2, ncomp, ngrid) or None)
    with the same density screening and derivative layout."""
    import torch
    comps, _, xctype = parse_xc(xc)
    ncomp = 4 if xctype == "GGA" else 1
    if rho.dim() == 2:
        rho = rho[:, None, :]
    rho = rho[:, :ncomp].to(torch.float64)
    ng = rho.shape[-1]
    kw = dict(dtype=torch.float64, device=rho.device)
    exc = torch.zeros(ng, **kw)
    vxc = torch.zeros((2, ncomp, ng), **kw)
    fxc = torch.zeros((2, ncomp, 2, ncomp, ng), **kw) if deriv >= 2 else None
    if not comps:
        return exc, vxc, fxc
    mask = (rho[0, 0] + rho[1, 0]) > DENS_THRESHOLD
    idx = torch.nonzero(mask).squeeze(1)
    if idx.numel() == 0:
        return exc, vxc, fxc
    x = rho[:, :, idx].reshape(2 * ncomp, -1).clone().requires_grad_(True)
    rs = x.reshape(2, ncomp, -1)
    ra = torch.clamp(rs[0, 0], min=1e-30)
    rb = torch.clamp(rs[1, 0], min=1e-30)
    if ncomp == 4:
        ga, gb = rs[0, 1:], rs[1, 1:]
        saa, sab, sbb = (ga * ga).sum(0), (ga * gb).sum(0), (gb * gb).sum(0)
    else:
        saa = sab = sbb = torch.zeros_like(ra)
    eps = 0.0
    for name, coef in comps:
        eps = eps + coef * _PIECES[name](ra, rb, saa, sab, sbb, torch)
    g = torch.autograd.grad(eps.sum(), x, create_graph=deriv >= 2)[0]
    exc[idx] = (eps / (ra + rb)).detach()
    vxc[:, :, idx] = g.detach().reshape(2, ncomp, -1)
    if deriv >= 2:
        n = 2 * ncomp
        H = torch.empty((n, n, idx.numel()), **kw)
        for k in range(n):
            H[k] = torch.autograd.grad(g[k].sum(), x, retain_graph=k < n - 1)[0]
        H = 0.5 * (H + H.transpose(0, 1))
        fxc[..., idx] = H.reshape(2, ncomp, 2, ncomp, -1)
    return exc, vxc, fxc
