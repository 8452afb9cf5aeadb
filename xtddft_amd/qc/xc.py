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

Meta-GGA (the reference's MGGA branches, XTDA.py:239-276 and nr_uks_fxc, XTDA.py:514):
inputs (rho_s, grad rho_s, tau_s) per spin, PySCF's 5-component layout (2, 5, ngrid)
with tau = 1/2 sum |grad phi|^2 (no Laplacian):

* TPSS exchange     Tao, Perdew, Staroverov, Scuseria, PRL 91, 146401 (2003), eqs. 4-10,
                    spin scaling E_x[n_a, n_b] = (E_x[2 n_a] + E_x[2 n_b]) / 2
* TPSS correlation  revPKZB (eqs. 11-14) on PBE correlation (PRL 77, 3865 (1996)) over
                    PW92 (libxc's PW_MOD parameters), d = 2.8 Ha^-1

Range separation (the reference's RSH branches: ``rsh_and_hybrid_coeff``, XTDA.py:82, 501;
long-range K at XTDA.py:150-151, 527-539):

* ITYH short-range B88 exchange  Iikura, Tsuneda, Yanai, Hirao, JCP 115, 3540 (2001):
                    per spin e = -C_x rho_s^(4/3) F_B88(x_s) att(a_s), a_s = omega / (2 k_s),
                    k_s = sqrt(9 pi / K_s) rho_s^(1/3), K_s = 2 C_x F_B88(x_s) (libxc GGA_X_ITYH
                    with the B88 enhancement), att(a) = 1 - 8/3 a [sqrt(pi) erf(1/(2a))
                    + (2a - 4a^3) exp(-1/(4a^2)) - 3a + 4a^3] (libxc attenuation_erf), its
                    large-a series past a = 0.6 (the closed form cancels there)
* CAM-B3LYP         libxc HYB_GGA_XC_CAM_B3LYP: 0.35 B88 + 0.46 ITYH-B88(omega) + 0.19 VWN5
                    + 0.81 LYP, omega = 0.33, HF exchange 0.19 short-range + 0.65 long-range:
                    PySCF's (omega, alpha, hyb) = (0.33, 0.65, 0.19), K = hyb K + (alpha - hyb) K_LR.
                    Parity unpinned (no reference printout); checked by att's limits (omega -> 0
                    gives B88, omega -> inf gives zero), the series / closed-form match, and the
                    SCF's energy stationarity (tests/test_qc.py).

PBE family (the reference's demo list, XTDA.py:1524-1531: 'pbe0', 'pbe38'):

* PBE exchange      Perdew, Burke, Ernzerhof, PRL 77, 3865 (1996): per spin (spin scaling)
                    e = -C_x (2 rho_s)^(4/3) F(s) / 2, F = 1 + kappa - kappa / (1 + mu s^2 / kappa),
                    kappa = 0.804, mu = 0.2195149727645171, s = |grad n| / (2 (3 pi^2)^(1/3) n^(4/3))
* PBE correlation   PW92 (PW_MOD) + H(rs, zeta, t) -- the same expression TPSS builds on
PBE = PBE x + PBE c, PBE0 = 0.25 HF + 0.75 PBE x + PBE c, PBE38 = 0.375 HF + 0.625 PBE x +
PBE c.  Pinned by the hydrogen atom (tests/test_qc.py): E_x^PBE = -0.3059 and E_c^PBE = -0.0060 Ha
on the exact density (Perdew, Burke, Ernzerhof's table), E_x^LDA = -0.2680.

omegaB97X-D (Chai and Head-Gordon, PCCP 10, 6615 (2008); the reference's 'wb97xd', XTDA.py:1528):
B97-type power series in u = gamma s^2 / (1 + gamma s^2), s_s^2 = |grad rho_s|^2 / rho_s^(8/3):

* exchange          sum_s e_x,s^LSDA att(a_s) g_x(u_s), a_s = omega / (2 (6 pi^2 rho_s)^(1/3)), gamma 0.004
                    (short-range LSDA: the erf attenuation of the ITYH piece with the LDA Fermi wave vector)
* correlation       same-spin PW92(rho_s, 0) g_ss(u_s) (gamma 0.2) + opposite-spin
                    [n PW92(n, zeta) - sum_s PW92(rho_s, 0)] g_os(u_avg), s_avg^2 = (s_a^2 + s_b^2) / 2
                    (gamma 0.006), the Stoll partition
* coefficients      c_x = 0.777964, 0.661160, 0.574541, -5.25671, 11.6386;
                    c_ss = 1, -6.90539, 31.3343, -51.0533, 26.4423;
                    c_os = 1, 1.79413, -12.0477, 14.0847, -8.50809;
                    HF exchange 0.222036 short-range + 1.0 long-range, omega = 0.2:
                    PySCF's (omega, alpha, hyb) = (0.2, 1.0, 0.222036).
The empirical -D dispersion energy depends on the nuclei only: it shifts E_tot and nothing else
(no orbital, no response term) and is not added.  Parity unpinned (no reference printout);
checked by its limits: the uniform-gas limit of the series (g(0) = c_0) and omega -> 0.

TPSS = TPSS x + TPSS c, TPSSh = 0.1 HF + 0.9 TPSS x + TPSS c.  Pinned by two exact
properties of the functional (tests/test_qc.py): the hydrogen-atom exchange energy is
exactly -5/16 Ha and the correlation energy of any one-electron density is zero.

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
_ZETA_MAX = 1.0 - 1e-10          # |zeta| cap (libxc's zeta threshold): (1 -+ zeta)^(-4/3) stays finite
# spin-separable exchange pieces: each spin channel's half is screened on its own
# density, as libxc does for exchange; correlation sees both channels unscreened
_EXCHANGE = ("slater", "b88", "tpss_x", "pbe_x")

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
    "TPSS": ([("tpss_x", 1.0), ("tpss_c", 1.0)], 0.0, "MGGA"),
    "TPSSH": ([("tpss_x", 0.9), ("tpss_c", 1.0)], 0.1, "MGGA"),
    "CAMB3LYP": ([("b88", 0.35), ("ityh_b88@0.33", 0.46), ("vwn5", 0.19), ("lyp", 0.81)], 0.19, "GGA"),
    "PBE": ([("pbe_x", 1.0), ("pbe_c", 1.0)], 0.0, "GGA"),
    "PBE0": ([("pbe_x", 0.75), ("pbe_c", 1.0)], 0.25, "GGA"),
    "PBE38": ([("pbe_x", 0.625), ("pbe_c", 1.0)], 0.375, "GGA"),
    "WB97XD": ([("wb97x_x@0.2", 1.0), ("wb97x_c", 1.0)], 0.222036, "GGA"),
}
# range-separated hybrids: name -> (omega, alpha) with PySCF's meaning (hyb from the table above)
_RSH = {"CAMB3LYP": (0.33, 0.65), "WB97XD": (0.2, 1.0)}
NCOMP = {"HF": 1, "LDA": 1, "GGA": 4, "MGGA": 5}


def parse_xc(xc: str):
    """(components, hyb, xctype); ``rsh_and_hybrid_coeff`` gives (0, hyb, hyb) for these."""
    key = xc.upper().replace("-", "").replace(" ", "")
    if key not in _FUNCTIONALS:
        raise KeyError(f"functional {xc!r} not implemented (available: {sorted(_FUNCTIONALS)})")
    return _FUNCTIONALS[key]


def rsh_and_hybrid_coeff(xc: str):
    """(omega, alpha, hyb) as PySCF returns them: (0, hyb, hyb) for a global hybrid (the
    reference prints "Omega, alpha, hyb 0.0 0.5 0.5" for BHandHLYP); for a range-separated
    hybrid K = hyb K + (alpha - hyb) K_LR(omega) (XTDA.py:537-539)."""
    _, hyb, _ = parse_xc(xc)
    key = xc.upper().replace("-", "").replace(" ", "")
    if key in _RSH:
        omega, alpha = _RSH[key]
        return omega, alpha, hyb
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
    z = torch.clamp((ra - rb) / rho, -_ZETA_MAX, _ZETA_MAX)     # libxc's zeta threshold
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


# ---------------------------------------------------------------- TPSS (meta-GGA)
_TAU_MIN = 1e-30


def _tpss_x_unpol(n, sigma, tau, torch):
    """TPSS exchange energy density of a spin-unpolarised density n (PRL 91, 146401)."""
    kappa, b, c, e, mu = 0.804, 0.40, 1.59096, 1.537, 0.21951
    kf2 = (3.0 * math.pi ** 2 * n) ** (2.0 / 3.0)
    p = sigma / (4.0 * kf2 * n * n)
    tauw = sigma / (8.0 * n)
    z = torch.clamp(tauw / torch.clamp(tau, min=_TAU_MIN), max=1.0)
    alpha = (5.0 / 3.0) * p * (1.0 / torch.clamp(z, min=1e-300) - 1.0)
    qb = 0.45 * (alpha - 1.0) / torch.sqrt(1.0 + b * alpha * (alpha - 1.0)) + 2.0 * p / 3.0
    se = math.sqrt(e)
    num = ((10.0 / 81.0 + c * z * z / (1.0 + z * z) ** 2) * p + 146.0 / 2025.0 * qb * qb
           - 73.0 / 405.0 * qb * torch.sqrt(0.5 * (0.6 * z) ** 2 + 0.5 * p * p + 1e-40)
           + (10.0 / 81.0) ** 2 * p * p / kappa + 2.0 * se * (10.0 / 81.0) * (0.6 * z) ** 2 + e * mu * p ** 3)
    x = num / (1.0 + se * p) ** 2
    fx = 1.0 + kappa - kappa / (1.0 + x / kappa)
    return -0.75 * (3.0 / math.pi) ** (1.0 / 3.0) * n ** (4.0 / 3.0) * fx


def _tpss_x(ra, rb, saa, sab, sbb, ta, tb, torch):
    return 0.5 * (_tpss_x_unpol(2.0 * ra, 4.0 * saa, 2.0 * ta, torch)
                  + _tpss_x_unpol(2.0 * rb, 4.0 * sbb, 2.0 * tb, torch))


# PW92 with libxc's PW_MOD parameters: (A, alpha1, beta1..beta4) for ec(rs, 0), ec(rs, 1), -alpha_c
_PW92 = ((0.0310907, 0.21370, 7.5957, 3.5876, 1.6382, 0.49294),
         (0.01554535, 0.20548, 14.1189, 6.1977, 3.3662, 0.62517),
         (0.0168869, 0.11125, 10.357, 3.6231, 0.88026, 0.49671))
_FZ20 = 1.709920934161365617563962776245


def _pw92_g(rs, prm, torch):
    A, a1, b1, b2, b3, b4 = prm
    srs = torch.sqrt(rs)
    den = 2.0 * A * (b1 * srs + b2 * rs + b3 * rs * srs + b4 * rs * rs)
    return -2.0 * A * (1.0 + a1 * rs) * torch.log1p(1.0 / den)


def _ec_pw92(n, zeta, torch):
    """PW92 correlation energy per particle."""
    rs = (3.0 / (4.0 * math.pi * n)) ** (1.0 / 3.0)
    ec0, ec1, mac = (_pw92_g(rs, prm, torch) for prm in _PW92)
    fz = ((1.0 + zeta) ** (4.0 / 3.0) + (1.0 - zeta) ** (4.0 / 3.0) - 2.0) / (2.0 ** (4.0 / 3.0) - 2.0)
    z4 = zeta ** 4
    return ec0 - mac * fz * (1.0 - z4) / _FZ20 + (ec1 - ec0) * fz * z4


def _ec_pbe(n, zeta, sigma, torch):
    """PBE correlation energy per particle (PW92 + H)."""
    beta, gamma = 0.06672455060314922, (1.0 - math.log(2.0)) / math.pi ** 2
    ec = _ec_pw92(n, zeta, torch)
    phi = 0.5 * ((1.0 + zeta) ** (2.0 / 3.0) + (1.0 - zeta) ** (2.0 / 3.0))
    kf = (3.0 * math.pi ** 2 * n) ** (1.0 / 3.0)
    ks2 = 4.0 * kf / math.pi
    t2 = sigma / (4.0 * phi * phi * ks2 * n * n)
    phi3 = phi ** 3
    A = beta / gamma / torch.expm1(-ec / (gamma * phi3))
    at2 = A * t2
    return ec + gamma * phi3 * torch.log1p(beta / gamma * t2 * (1.0 + at2) / (1.0 + at2 + at2 * at2))


def _tpss_c(ra, rb, saa, sab, sbb, ta, tb, torch):
    n = ra + rb
    zeta = torch.clamp((ra - rb) / n, -_ZETA_MAX, _ZETA_MAX)
    stot = saa + 2.0 * sab + sbb
    e_pbe = _ec_pbe(n, zeta, stot, torch)
    one = torch.full_like(n, _ZETA_MAX)
    e_a = torch.maximum(_ec_pbe(ra, one, saa, torch), e_pbe)       # fully polarised n_s alone
    e_b = torch.maximum(_ec_pbe(rb, one, sbb, torch), e_pbe)
    # xi = |grad zeta| / (2 (3 pi^2 n)^(1/3)), |grad zeta|^2 = 4 (rb^2 saa - 2 ra rb sab + ra^2 sbb) / n^4
    gz2 = 4.0 * torch.clamp(rb * rb * saa - 2.0 * ra * rb * sab + ra * ra * sbb, min=0.0) / n ** 4
    xi2 = gz2 / (4.0 * (3.0 * math.pi ** 2 * n) ** (2.0 / 3.0))
    z2 = zeta * zeta
    cnum = 0.53 + 0.87 * z2 + 0.50 * z2 * z2 + 2.26 * z2 ** 3
    cden = (1.0 + 0.5 * xi2 * ((1.0 + zeta) ** (-4.0 / 3.0) + (1.0 - zeta) ** (-4.0 / 3.0))) ** 4
    cc = cnum / cden
    tauw = stot / (8.0 * n)
    z = torch.clamp(tauw / torch.clamp(ta + tb, min=_TAU_MIN), max=1.0)
    zz = z * z
    e_rev = e_pbe * (1.0 + cc * zz) - (1.0 + cc) * zz * (ra / n * e_a + rb / n * e_b)
    return n * e_rev * (1.0 + 2.8 * e_rev * zz * z)


# attenuation of the erf-screened (short-range) LDA exchange hole, att(a) (libxc attenuation_erf)
_ATT_SWITCH = 0.6
_ATT_NSER = 24
_ATT_C = [(-1.0) ** k * (2.0 / (math.factorial(k) * (2 * k + 1)) - 1.0 / math.factorial(k + 1)
                         - 0.5 / math.factorial(k + 2)) for k in range(_ATT_NSER + 1)]


def _att_erf(a, torch):
    """1 - 8/3 a [sqrt(pi) erf(1/(2a)) + (2a - 4a^3) exp(-1/(4a^2)) - 3a + 4a^3].  Past a = 0.6
    the bracket cancels to ~1/a: there the series att = -4/3 sum_k c_k u^k in u = 1/(4a^2)
    (c_k from the erf and exp series; c_1 = -1/12 gives the 1/(36 a^2) tail)."""
    small = a < _ATT_SWITCH
    ad = torch.where(small, a, torch.full_like(a, _ATT_SWITCH))
    direct = 1.0 - 8.0 / 3.0 * ad * (math.sqrt(math.pi) * torch.erf(0.5 / ad)
                                     + (2.0 * ad - 4.0 * ad ** 3) * torch.exp(-0.25 / (ad * ad))
                                     - 3.0 * ad + 4.0 * ad ** 3)
    as_ = torch.where(small, torch.full_like(a, _ATT_SWITCH), a)
    u = 0.25 / (as_ * as_)
    ser = 0.0
    for k in range(_ATT_NSER, 0, -1):          # Horner in u
        ser = (ser + _ATT_C[k]) * u
    return torch.where(small, direct, -4.0 / 3.0 * ser)


def _ityh_b88(ra, rb, saa, sab, sbb, torch, omega):
    """Short-range B88 exchange of Iikura-Tsuneda-Yanai-Hirao (libxc GGA_X_ITYH)."""
    beta = 0.0042
    out = 0.0
    for r, s in ((ra, saa), (rb, sbb)):
        r13 = r ** (1.0 / 3.0)
        r43 = r * r13
        y = s / (r43 * r43)
        fx = 1.0 + beta / _CX * y / (1.0 + 6.0 * beta * _x_asinh_x(y, torch))
        k = torch.sqrt(9.0 * math.pi / (2.0 * _CX * fx)) * r13
        out = out - _CX * r43 * fx * _att_erf(omega / (2.0 * k), torch)
    return out


def _pbe_x(ra, rb, saa, sab, sbb, torch):
    """PBE exchange, spin-scaled: sum_s E_x^unpol[2 rho_s] / 2."""
    kappa, mu = 0.804, 0.2195149727645171
    out = 0.0
    for r, sg in ((ra, saa), (rb, sbb)):
        n, sig = 2.0 * r, 4.0 * sg
        s2 = sig / (4.0 * (3.0 * math.pi ** 2) ** (2.0 / 3.0) * n ** (8.0 / 3.0))
        fx = 1.0 + kappa - kappa / (1.0 + mu * s2 / kappa)
        out = out - 0.5 * _CX * 2.0 ** (-1.0 / 3.0) * n ** (4.0 / 3.0) * fx
    return out


def _pbe_c(ra, rb, saa, sab, sbb, torch):
    n = ra + rb
    zeta = torch.clamp((ra - rb) / n, -_ZETA_MAX, _ZETA_MAX)
    return n * _ec_pbe(n, zeta, saa + 2.0 * sab + sbb, torch)


_WB97XD = dict(cx=(0.777964, 0.661160, 0.574541, -5.25671, 11.6386),
               css=(1.0, -6.90539, 31.3343, -51.0533, 26.4423),
               cos=(1.0, 1.79413, -12.0477, 14.0847, -8.50809))


def _b97_g(c, gamma, s2):
    u = gamma * s2 / (1.0 + gamma * s2)
    out = 0.0
    for ci in reversed(c):
        out = out * u + ci
    return out


def _wb97x_x(ra, rb, saa, sab, sbb, torch, omega):
    """omegaB97X short-range exchange: sum_s e_x,s^LSDA att(omega / 2 k_F,s) g_x(s_s^2)."""
    out = 0.0
    for r, sg in ((ra, saa), (rb, sbb)):
        r13 = r ** (1.0 / 3.0)
        r43 = r * r13
        kf = (6.0 * math.pi ** 2) ** (1.0 / 3.0) * r13
        out = out - _CX * r43 * _att_erf(omega / (2.0 * kf), torch) * _b97_g(_WB97XD["cx"], 0.004, sg / (r43 * r43))
    return out


def _wb97x_c(ra, rb, saa, sab, sbb, torch):
    """omegaB97X correlation: same-spin and opposite-spin PW92 (Stoll partition) x B97 series."""
    n = ra + rb
    zeta = torch.clamp((ra - rb) / n, -_ZETA_MAX, _ZETA_MAX)
    one = torch.full_like(n, _ZETA_MAX)
    ess = 0.0
    s2 = []
    for r, sg in ((ra, saa), (rb, sbb)):
        e_s = r * _ec_pw92(r, one, torch)
        x2 = sg / r ** (8.0 / 3.0)
        s2.append(x2)
        ess = ess + e_s * _b97_g(_WB97XD["css"], 0.2, x2)
    e_os = n * _ec_pw92(n, zeta, torch) - ra * _ec_pw92(ra, one, torch) - rb * _ec_pw92(rb, one, torch)
    return ess + e_os * _b97_g(_WB97XD["cos"], 0.006, 0.5 * (s2[0] + s2[1]))


_PIECES = {"slater": _slater, "b88": _b88, "lyp": _lyp, "vwn5": _vwn5, "vwn_rpa": _vwn_rpa,
           "pbe_x": _pbe_x, "pbe_c": _pbe_c, "wb97x_c": _wb97x_c}
_MPIECES = {"tpss_x": _tpss_x, "tpss_c": _tpss_c}


def _piece(name, ra, rb, saa, sab, sbb, ta, tb, torch):
    if name.startswith("ityh_b88@"):
        return _ityh_b88(ra, rb, saa, sab, sbb, torch, float(name.split("@")[1]))
    if name.startswith("wb97x_x@"):
        return _wb97x_x(ra, rb, saa, sab, sbb, torch, float(name.split("@")[1]))
    if name in _MPIECES:
        return _MPIECES[name](ra, rb, saa, sab, sbb, ta, tb, torch)
    return _PIECES[name](ra, rb, saa, sab, sbb, torch)


def _energy_density(comps, ra, rb, saa, sab, sbb, ta, tb, torch, on=None):
    """Sum of the functional's pieces.  ``on`` = (on_a, on_b): 0/1 constants marking
    where each channel's density exceeds DENS_THRESHOLD; an exchange piece's half of a
    channel below it is dropped (with the other channel's arguments replaced by inert
    constants, so no derivative reaches the vanishing channel)."""
    eps = 0.0
    for name, coef in comps:
        if on is not None and (name in _EXCHANGE or name.startswith(("ityh_b88@", "wb97x_x@"))):
            tiny = torch.full_like(ra, 1e-30).detach()
            zero = torch.zeros_like(ra).detach()
            half_a = _piece(name, ra, tiny, saa, zero, zero, ta, None if tb is None else tiny, torch)
            half_b = _piece(name, tiny, rb, zero, zero, sbb, None if ta is None else tiny, tb, torch)
            eps = eps + coef * (on[0] * half_a + on[1] * half_b)
        else:
            eps = eps + coef * _piece(name, ra, rb, saa, sab, sbb, ta, tb, torch)
    return eps


def eval_xc_eff(xc: str, rho: np.ndarray, deriv: int = 1):
    """Spin-polarised XC on a grid.

    rho : (2, 4, ngrid) for GGA (rho, d/dx, d/dy, d/dz per spin), (2, 5, ngrid) for
          MGGA (+ tau), or (2, ngrid) / (2, 1, ngrid) for LDA.
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
    ncomp = NCOMP[xctype]
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
    if ncomp >= 4:
        ga, gb = rs[0, 1:4], rs[1, 1:4]
        saa = (ga * ga).sum(0)
        sab = (ga * gb).sum(0)
        sbb = (gb * gb).sum(0)
    else:
        saa = sab = sbb = torch.zeros_like(ra)
    ta, tb = (rs[0, 4], rs[1, 4]) if ncomp == 5 else (None, None)
    on = ((rs[0, 0] > DENS_THRESHOLD).to(torch.float64).detach(),
          (rs[1, 0] > DENS_THRESHOLD).to(torch.float64).detach())
    eps = _energy_density(comps, ra, rb, saa, sab, sbb, ta, tb, torch, on)
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
    if xctype == "MGGA":
        _screen_spin(rho, vxc, fxc, np)
    return exc, vxc, fxc


def _screen_spin(rho, vxc, fxc, xp):
    """Meta-GGA only: a spin channel without density at a point (below DENS_THRESHOLD)
    carries no potential or kernel there (TPSS correlation's fully polarised terms are
    singular in a vanishing channel).  LDA / GGA functionals screen only their
    exchange halves per channel (``_energy_density``), as libxc does."""
    for s in range(2):
        off = rho[s, 0] < DENS_THRESHOLD
        if not bool(off.any()):
            continue
        vxc[s, :, off] = 0.0
        if fxc is not None:
            fxc[s, :, :, :, off] = 0.0
            fxc[:, :, s, :, off] = 0.0


def eval_xc_eff_torch(xc: str, rho, deriv: int = 1):
    """``eval_xc_eff`` on a torch tensor rho (2, ncomp, ngrid) wherever it lives
    (the device SCF engine evaluates the functional on the GPU): returns torch
    (exc (ngrid,), vxc (2, ncomp, ngrid), fxc (2, ncomp, 2, ncomp, ngrid) or None)
    with the same density screening and derivative layout."""
    import torch
    comps, _, xctype = parse_xc(xc)
    ncomp = NCOMP[xctype]
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
    if ncomp >= 4:
        ga, gb = rs[0, 1:4], rs[1, 1:4]
        saa, sab, sbb = (ga * ga).sum(0), (ga * gb).sum(0), (gb * gb).sum(0)
    else:
        saa = sab = sbb = torch.zeros_like(ra)
    ta, tb = (rs[0, 4], rs[1, 4]) if ncomp == 5 else (None, None)
    on = ((rs[0, 0] > DENS_THRESHOLD).to(torch.float64).detach(),
          (rs[1, 0] > DENS_THRESHOLD).to(torch.float64).detach())
    eps = _energy_density(comps, ra, rb, saa, sab, sbb, ta, tb, torch, on)
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
    if xctype == "MGGA":
        _screen_spin(rho, vxc, fxc, torch)
    return exc, vxc, fxc
