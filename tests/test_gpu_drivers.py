"""GPU: reference-driver conventions beyond the operator.

* SF_TDA_down returns eigenvectors in the reference's cv|co|ov|oo block order
  (deal_v_davidson, SF_TDA.py:304-345; get_Amat block order, SF_TDA.py:746-801),
  on both the Davidson and the explicit-A path: compared with the oracle's
  block-ordered explicit A.
* XSF_TDA on a ROKS doublet (no = 1) with the OO element removed at SA = 0
  (XSF_TDA.py:397-414, 1519-1523): A.x and eigenvalues vs the oracle.
* UKS X-TDA: "my order", Delta<S^2> and analyze() (XTDA.py:796-822).
* A driver sharded over ranks refuses to run without a process group.
"""
import numpy as np
import pytest

from oracle import sf_tda as osf
from oracle import xsf_tda as oxsf
from oracle import xtda as oxtda
from xtddft_amd.synthetic import make_mf, make_trial_vectors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch(hiplib):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _block_overlap(v, w):
    """|<v_k, w_k>| per root for unit eigenvectors (sign-free comparison)."""
    return np.abs(np.einsum("ik,ik->k", v, w))


@pytest.mark.parametrize("davidson", [True, False])
def test_sf_down_vectors_in_block_order(torch, davidson):
    from xtddft_amd.sf_tda import SF_TDA
    mf = make_mf(nao=22, nc=4, no=2, xctype="GGA", hyb=0.5)
    a = osf.amat_down(mf)                       # cv|co|ov|oo order
    w, u = np.linalg.eigh(a)
    sf = SF_TDA(mf, isf=-1, davidson=davidson)
    e_ev, v = sf.kernel(nstates=4)
    assert np.abs(np.asarray(sf.e)[:4] - w[:4]).max() < 1e-8
    ov = _block_overlap(np.asarray(v)[:, :4], u[:, :4])
    assert np.all(ov > 1 - 1e-6), ov
    if not davidson:
        assert np.abs(sf.A - a).max() < 1e-12 * np.abs(a).max()
    ds, lines = sf.analyse(verbose=False)
    assert len(ds) == 4 and lines


def test_xsf_doublet_remove(torch):
    from xtddft_amd.xsf_tda import XSF_TDA
    mf = make_mf(nao=20, nc=5, no=1, xctype="GGA", hyb=0.5)
    o = oxsf.XSFOracle(mf, SA=0)
    o.re = True
    fg = oxsf.default_fglobal(mf)
    vind, hdiag = o.gen_tda_operation_sf(fglobal=fg)
    dim = hdiag.size
    assert dim == (5 + 1) * (1 + 14) - 1
    x = XSF_TDA(mf, SA=0)
    e_ev, v = x.kernel(nstates=5, remove=True, fglobal=fg)
    z = make_trial_vectors(4, dim)
    s = x._op.apply(z)
    ref = vind(z)
    assert np.abs(s - ref).max() < 1e-12 * np.abs(ref).max()
    wref = np.linalg.eigvalsh(vind(np.eye(dim)).T)[:5]
    assert x.converged.all() and np.abs(np.asarray(x.e) - wref).max() < 1e-7
    # explicit-A path too
    e2, _ = XSF_TDA(mf, SA=0, davidson=False).kernel(nstates=5, remove=True, fglobal=fg)
    assert np.abs(e2 / 27.21138505 - wref).max() < 1e-9


def test_utda_order_and_analyze(torch):
    from xtddft_amd import XTDA
    mf = make_mf(nao=24, nc=5, no=2, xctype="GGA", hyb=0.2, kind="U")
    vind, hdiag = oxtda.gen_tda_operation(mf)
    x = XTDA(mf.mol, mf, nstates=4)
    e = x.kernel()
    w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)[:4]
    assert x.converged.all() and np.abs(e - w).max() < 1e-9
    assert x.v.shape == (hdiag.size, 4) and x.dS2.shape == (4,)
    assert np.all(np.asarray(x.order)[:5] == np.arange(5))
    lines = x.analyze(verbose=False)
    assert any("w:" in ln for ln in lines)


def test_sharded_driver_needs_group(torch):
    from xtddft_amd import XTDA
    from xtddft_amd.xsf_tda import XSF_TDA
    mf = make_mf(nao=20, nc=4, no=2, xctype="GGA", hyb=0.2)
    with pytest.raises(ValueError):
        XTDA(mf.mol, mf, shard=(0, 2))
    with pytest.raises(ValueError):
        XSF_TDA(mf, shard=(1, 2))
