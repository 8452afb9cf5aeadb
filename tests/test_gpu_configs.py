"""GPU: every BASELINE.json configuration (bench.CONFIGS, SURVEY.md 8 shape table)
through the C ABI.

* C1 CH2 / 6-31G shape (X-TDA, 5 roots): A.x vs the oracle at full size, device
  Davidson vs the oracle's explicit-A eigenvalues (XTDA.full_diag route).
* C2 naphthalene+ / SVP shape (X-TDA, nao 180, 20 roots) and C5 [Cu2O2]2+ / TZVP
  shape (X-TDA, nao 152, 50 roots, EXACT K = stored 8-fold ERIs): A.x vs the
  oracle (C5: the oracle contracts the same tensor as a DF factor, ERI = B^T B),
  and the device Davidson vs the oracle Davidson at reduced naux / ngrid.
* C3 Fe(II)P / TZVP shape (SF-up, nao 861, 30 roots) and C4 C60 / SVP shape (XSF,
  nao 840, 40 roots, as the quartet at SA = 3 and the doublet at SA = 0, OO
  compressed) at FULL size: symmetry, linearity and batch invariance of A, the
  reference drivers' Davidson converged for every root, and each root's
  residual |A v - w v| re-checked by a separate A.x call.
* H, the headline shape (X-TDA, nao 1000, 20 roots, stored exchange) at FULL size: the
  same properties, Davidson and residual checks.
Tolerances: 1e-12 relative on sigma (FP64 round-off of a different summation
order), 1e-9 Ha on Davidson-vs-Davidson / explicit-A eigenvalues.
"""
import numpy as np
import pytest

import bench
from oracle import davidson as odav
from oracle import xtda as oxtda
from xtddft_amd.synthetic import as_eri8, make_mf, make_trial_vectors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch(hiplib):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.fixture(autouse=True)
def _release_memory(torch):
    """The library allocates with hipMalloc beside torch's caching allocator: hand
    torch's cached blocks back between the large configurations."""
    yield
    import gc
    gc.collect()
    torch.cuda.empty_cache()


def _shape(name):
    c = bench.CONFIGS[name]
    return dict(nao=c["nao"], nc=c["nc"], no=c["no"], hyb=c["hyb"]), c


def _rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


def test_c1_ch2_xtda(torch):
    from xtddft_amd import XTDA
    from xtddft_amd.operator import DeviceOperator
    sh, c = _shape("C1")
    mf = make_mf(naux=3 * sh["nao"], ngrid=c["ngrid"], xctype="GGA", **sh)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(7, hdiag.size)
    assert _rel(DeviceOperator(mf, "XTDA").apply(z), vind(z)) < 1e-12
    a = oxtda.full_diag_matrix(mf)                    # independent explicit-A route
    w = np.linalg.eigvalsh(a)[:c["nroots"]]
    x = XTDA(mf.mol, mf, nstates=c["nroots"])
    e = x.kernel()
    assert x.converged.all() and np.abs(e - w).max() < 1e-9


def _xtda_davidson_vs_oracle(torch, mf, nroots):
    from xtddft_amd.davidson import DiagPrecond, davidson1
    from xtddft_amd.operator import DeviceOperator
    vind, hdiag = oxtda.gen_tda_operation(mf)
    x0 = oxtda.get_init_guess(mf, nroots)
    c1, e1, _, _ = odav.davidson1(vind, x0, oxtda.get_precond(mf, hdiag), tol_residual=1e-6,
                                  lindep=1e-12, nroots=nroots, pick=oxtda.pickeig, max_cycle=100)
    op = DeviceOperator(mf, "XTDA")
    c2, e2, _, _ = davidson1(op.apply, x0, DiagPrecond(hdiag, 0.0), tol_residual=1e-6,
                             lindep=1e-12, nroots=nroots, pick=oxtda.pickeig, max_cycle=100)
    op.close()
    assert c1.all() and c2.all()
    assert np.abs(np.asarray(e1) - np.asarray(e2)).max() < 1e-9


def test_c2_naphthalene_shape_sigma(torch):
    from xtddft_amd.operator import DeviceOperator
    sh, _ = _shape("C2")
    mf = make_mf(naux=3 * sh["nao"], ngrid=12000, xctype="GGA", **sh)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(3, hdiag.size)
    for mode in ("stored", "direct"):
        op = DeviceOperator(mf, "XTDA", k_mode=mode)
        assert _rel(op.apply(z), vind(z)) < 1e-12, mode
        op.close()


def test_c2_naphthalene_shape_davidson(torch):
    sh, c = _shape("C2")
    _xtda_davidson_vs_oracle(torch, make_mf(naux=90, ngrid=6000, xctype="GGA", **sh), c["nroots"])


def test_c5_exact_k_sigma(torch):
    """The stored 8-fold ERIs (mf._eri route; device pivoted Cholesky) against the
    oracle contracting the same ERI tensor as its DF factor."""
    from xtddft_amd.operator import DeviceOperator
    sh, _ = _shape("C5")
    mf = make_mf(naux=3 * sh["nao"], ngrid=8000, xctype="GGA", **sh)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(3, hdiag.size)
    op = DeviceOperator(as_eri8(mf), "XTDA")
    naux, rank = op.naux()
    assert rank <= 3 * sh["nao"]
    assert _rel(op.apply(z), vind(z)) < 1e-12


def test_c5_exact_k_davidson(torch):
    sh, c = _shape("C5")
    mf = make_mf(naux=100, ngrid=4000, xctype="GGA", **sh)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    x0 = oxtda.get_init_guess(mf, c["nroots"])
    from xtddft_amd.davidson import DiagPrecond, davidson1
    from xtddft_amd.operator import DeviceOperator
    c1, e1, _, _ = odav.davidson1(vind, x0, oxtda.get_precond(mf, hdiag), tol_residual=1e-6,
                                  lindep=1e-12, nroots=c["nroots"], pick=oxtda.pickeig, max_cycle=100)
    op = DeviceOperator(as_eri8(mf), "XTDA")
    c2, e2, _, _ = davidson1(op.apply, x0, DiagPrecond(hdiag, 0.0), tol_residual=1e-6,
                             lindep=1e-12, nroots=c["nroots"], pick=oxtda.pickeig, max_cycle=100)
    assert c1.all() and c2.all()
    assert np.abs(np.asarray(e1) - np.asarray(e2)).max() < 1e-9


# ---- full-size configurations: properties + converged reference drivers ------
def _properties(torch, op):
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn((3, op.dim), dtype=torch.float64, device="cuda", generator=g)
    y = torch.randn((3, op.dim), dtype=torch.float64, device="cuda", generator=g)
    ax, ay = op.apply(x), op.apply(y)
    lhs, rhs = y @ ax.T, ay @ x.T                          # <y, A x> = <A y, x>
    assert float((lhs - rhs).abs().max() / lhs.abs().max()) < 1e-11
    comb = op.apply(0.3 * x - 1.7 * y)                     # linearity
    assert float((comb - (0.3 * ax - 1.7 * ay)).abs().max() / comb.abs().max()) < 1e-12
    single = op.apply(x[1:2].contiguous())                 # batch invariance
    assert float((single - ax[1:2]).abs().max() / single.abs().max()) < 1e-13


def _residuals(torch, op, e_ha, v):
    """|A v - w v| of each root from a fresh A.x call (not the solver's images)."""
    vt = torch.as_tensor(np.ascontiguousarray(np.asarray(v).T), device="cuda")
    av = op.apply(vt)
    r = av - torch.as_tensor(np.asarray(e_ha), device="cuda")[:, None] * vt
    return (r.norm(dim=1) / vt.norm(dim=1)).cpu().numpy()


def _device_mf(name):
    from xtddft_amd.synthetic import make_device_mf
    sh, c = _shape(name)
    return make_device_mf(xctype="GGA", **sh), c


def test_c3_fe_porphyrin_sf_up_full_size(torch):
    from xtddft_amd.sf_tda import SF_TDA
    mf, c = _device_mf("C3")
    sf = SF_TDA(mf, isf=1)
    e_ev, v = sf.kernel(nstates=c["nroots"])
    _properties(torch, sf._op)
    assert sf.converged.all()
    r = _residuals(torch, sf._op, np.asarray(sf.e)[:c["nroots"]], v)
    assert r.max() < 1e-3, r           # SF_TDA.py:392 tol 1e-7 -> residual <= sqrt(tol)
    sf._op.close()


@pytest.mark.parametrize("name,sa", [("C4", 3), ("C4d", 0)])
def test_c4_c60_xsf_full_size(torch, name, sa):
    from xtddft_amd.xsf_tda import XSF_TDA
    mf, c = _device_mf(name)
    x = XSF_TDA(mf, SA=sa)
    e_ev, v = x.kernel(nstates=c["nroots"], remove=True)
    assert v.shape == (x._op.dim, c["nroots"])
    assert x._op.dim == (c["nc"] + c["no"]) * (c["nao"] - c["nc"]) - 1
    _properties(torch, x._op)
    assert x.converged.all()
    r = _residuals(torch, x._op, np.asarray(x.e), v)
    assert r.max() < 1e-4, r           # XSF_TDA.py:1467 tol 1e-8 -> residual <= sqrt(tol)
    x._op.close()


def test_h_headline_xtda_full_size(torch):
    """The headline shape itself (bench config H: nao 1000, 101 / 99 occupied, naux 3000,
    ngrid 1.2 M, GGA, the 62 GiB stored exchange): symmetry, linearity and batch
    invariance of A, the 20-root X-TDA Davidson converged, and every root's residual
    re-checked by a separate A.x (XTDA.py:769-777 criteria: |r| < 1e-5)."""
    from xtddft_amd import XTDA
    mf, c = _device_mf("H")
    x = XTDA(None, mf, nstates=c["nroots"])
    e = x.kernel()
    op = x.operator()
    assert op.k_mode == "stored"
    _properties(torch, op)
    assert np.all(x.converged) and len(e) == c["nroots"]
    v = np.empty_like(x.v)
    v[x.order] = x.v                                       # back to the operator's order
    r = _residuals(torch, op, np.asarray(e), v)
    assert r.max() < 1e-4, r
    op.close()
