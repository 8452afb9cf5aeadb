"""CPU: the oracle against itself across two reference code paths, and against
the committed golden fixtures (no GPU)."""
import numpy as np
import pytest

from golden_io import list_cases, load
from oracle import davidson as odav
from oracle import sf_tda as osf
from oracle import xsf_tda as oxsf
from oracle import xtda as oxtda
from oracle.utils import order_pyscf2my as order_literal
from xtddft_amd.synthetic import make_mf, make_trial_vectors
from xtddft_amd.utils import order_pyscf2my


def dense(vind, dim):
    return vind(np.eye(dim)).T


@pytest.mark.parametrize("xct,omega", [("HF", 0.0), ("LDA", 0.0), ("GGA", 0.0), ("GGA", 0.33)])
def test_xtda_vind_matches_full_diag(xct, omega):
    """vind (XTDA.py:615-690, AO route) == full_diag's explicit A (XTDA.py:56-400, MO route)."""
    mf = make_mf(nao=14, nc=3, no=2, xctype=xct, hyb=0.19 if omega else 0.2, omega=omega,
                 alpha=0.65 if omega else 0.0)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    a = dense(vind, hdiag.size)
    o = order_pyscf2my(3, 2, 9)
    assert np.abs(a - a.T).max() < 1e-14
    assert np.abs(a[o][:, o] - oxtda.full_diag_matrix(mf)).max() < 1e-13


def test_utda_symmetric_with_orbital_energy_diagonal():
    mf = make_mf(nao=14, nc=3, no=2, kind="U", xctype="GGA")
    vind, hdiag = oxtda.gen_tda_operation(mf)
    a = dense(vind, hdiag.size)
    assert np.abs(a - a.T).max() < 1e-14
    assert np.linalg.eigvalsh(a).min() > 0


@pytest.mark.parametrize("kind", ["RO", "U"])
@pytest.mark.parametrize("xct", ["HF", "LDA", "GGA"])
def test_sf_vind_matches_get_amat(kind, xct):
    mf = make_mf(nao=14, nc=3, no=2, xctype=xct, hyb=0.5, kind=kind)
    vind, hdiag = osf.gen_tda_operation_sf(mf, 1)
    assert np.abs(dense(vind, hdiag.size) - osf.amat_up(mf)).max() < 1e-13
    vind, hdiag = osf.gen_tda_operation_sf(mf, -1)
    nc, no, nv = 3, 2, 9
    idx = np.arange((nc + no) * (no + nv)).reshape(nc + no, no + nv)
    perm = np.concatenate([idx[:nc, no:].ravel(), idx[:nc, :no].ravel(),
                           idx[nc:, no:].ravel(), idx[nc:, :no].ravel()])
    a = dense(vind, hdiag.size)[perm][:, perm]
    assert np.abs(a - osf.amat_down(mf)).max() < 1e-13


@pytest.mark.parametrize("sa", [1, 2, 3])
@pytest.mark.parametrize("no", [2, 3])
def test_xsf_vind_matches_get_amat_removed(sa, no):
    mf = make_mf(nao=15, nc=3, no=no, xctype="GGA", hyb=0.5)
    o = oxsf.XSFOracle(mf, SA=sa)
    vind, hdiag = o.gen_tda_operation_sf()
    a = dense(vind, hdiag.size)
    assert np.abs(a - o.remove(o.get_amat())).max() < 1e-13
    assert np.abs(a - a.T).max() < 1e-14


def test_xsf_unrestricted_is_sf_down():
    mf = make_mf(nao=14, nc=3, no=2, xctype="LDA", hyb=0.5, kind="U")
    o = oxsf.XSFOracle(mf)
    vind, hdiag = o.gen_tda_operation_sf()
    assert not o.re and o.SA == 0
    assert np.abs(dense(vind, hdiag.size) - o.get_amat()).max() < 1e-13


def test_oracle_davidson_matches_eigh():
    mf = make_mf(nao=24, nc=5, no=2, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    x0 = oxtda.get_init_guess(mf, 6)
    conv, e, x, icyc = odav.davidson1(vind, x0, oxtda.get_precond(mf, hdiag), tol_residual=1e-6,
                                      lindep=1e-12, nroots=6, pick=oxtda.pickeig, max_cycle=100)
    assert conv.all()
    w = np.linalg.eigvalsh(dense(vind, hdiag.size))
    assert np.abs(e - w[:6]).max() < 1e-10


def test_order_closed_form_matches_reference_loop():
    for nc, no, nv in [(3, 2, 8), (5, 1, 4), (4, 3, 6), (2, 4, 3), (1, 1, 1)]:
        assert np.array_equal(order_pyscf2my(nc, no, nv), order_literal(nc, no, nv))


@pytest.mark.parametrize("case", list_cases())
def test_golden_fixture_reproduced(case):
    """The oracle reproduces its committed fixture bit-for-bit-ish (drift guard)."""
    mf, ex = load(case)
    kind = str(ex["in_kind"])
    if kind in ("XTDA", "UTDA"):
        vind, hdiag = oxtda.gen_tda_operation(mf)
    elif kind == "SF_DOWN":
        vind, hdiag = osf.gen_tda_operation_sf(mf, -1)
    elif kind == "SF_UP":
        vind, hdiag = osf.gen_tda_operation_sf(mf, 1)
    else:
        o = oxsf.XSFOracle(mf, SA=3)
        vind, hdiag = o.gen_tda_operation_sf(fglobal=oxsf.default_fglobal(mf))
    s = vind(ex["in_z"])
    assert np.abs(s - ex["out_sigma"]).max() <= 1e-13 * np.abs(ex["out_sigma"]).max()
    assert np.abs(hdiag - ex["out_hdiag"]).max() < 1e-13


def test_trial_vectors_normalised():
    z = make_trial_vectors(4, 50)
    assert np.allclose(np.linalg.norm(z, axis=1), 1.0)


def test_oracle_stored_eri_route_equals_df():
    """The oracle's incore-ERI J/K route (mf.extra['eri_full'], PySCF mf._eri
    convention) gives the DF route's sigma for ERI = B^T B: the CPU baseline of
    the exact-K configuration times it."""
    import dataclasses
    from oracle.engines import eri_full_from_cderi
    mf = make_mf(nao=14, nc=3, no=2, naux=30, ngrid=500, xctype="GGA", hyb=0.3, omega=0.4, alpha=0.7)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    m2 = dataclasses.replace(mf, extra=dict(eri_full=eri_full_from_cderi(mf.cderi),
                                            eri_full_lr=eri_full_from_cderi(mf.cderi_lr)))
    vind2, _ = oxtda.gen_tda_operation(m2)
    z = make_trial_vectors(3, hdiag.size)
    ref = vind(z)
    assert np.abs(vind2(z) - ref).max() < 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("nz", [1, 3])
def test_mgga_vind_equals_explicit_a(nz):
    """MGGA: the AO-route response (nr_uks_fxc restated with tau) and the explicit-A
    kernel loop (XTDA.py:239-276 restated) are two reference code paths for the same
    operator: equal to round-off on a synthetic ROKS problem."""
    from oracle import xtda as ox
    from xtddft_amd.synthetic import make_mf, make_trial_vectors
    from xtddft_amd.utils import order_pyscf2my
    mf = make_mf(nao=20, nc=4, no=2, ngrid=600, xctype="MGGA", hyb=0.2)
    vind, hdiag = ox.gen_tda_operation(mf)
    A = ox.full_diag_matrix(mf)
    info = mf.shape_info()
    order = order_pyscf2my(info['nc'], info['no'], info['nv'])
    z = make_trial_vectors(nz, hdiag.size)
    zm = z[:, order]
    assert np.abs(vind(z)[:, order] - zm @ A.T).max() < 1e-13 * np.abs(A).max()
