"""GPU: the kernel paths each context selects for the fused XC classes, against the
oracle, and the XSF exchange through the stored matrix at the row counts that take
its 160-row streaming tile and its batching.

Automatic selection (xt_ctx.hip): the dedicated M-backward kernel (xt_xcm.hip) for
O <= 128 and the generic engine's fused mode 2 above; the dedicated rho-forward
kernel (xt_xcw.hip) for O > 64, the small-O rho-forward kernel (xt_xcws.hip) for
O <= 48 from 8 trial pairs, and the engine's fused mode 1 in between.
The two test hooks (environment, read once at xt_create) force either side outside
its automatic range so each path is checked at every occupied-row shape:

* XT_M_KERNEL=0 -> XC M-backward through the engine's mode 2
* XT_W_KERNEL=0 / 1 / 3 -> XC rho-forward through the engine's mode 1 / the O > 64
  kernel / the small-O kernel (every pair count; O <= 48)

Tolerance: 1e-12 relative max-norm on sigma (FP64 round-off of a different
summation order), as in test_gpu_parity.py.
"""
import os

import numpy as np
import pytest

from oracle import xsf_tda as oxsf
from oracle import xtda as oxtda
from xtddft_amd.synthetic import make_mf, make_trial_vectors

pytestmark = pytest.mark.gpu
RTOL = 1e-12


def rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


@pytest.fixture
def env():
    saved = {}

    def set_(**kw):
        for k, v in kw.items():
            saved.setdefault(k, os.environ.get(k))
            os.environ[k] = str(v)
    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("knobs", [dict(), dict(XT_M_KERNEL=0), dict(XT_W_KERNEL=0), dict(XT_M_KERNEL=0, XT_W_KERNEL=0),
                                   dict(XT_M_KERNEL=1, XT_W_KERNEL=1), dict(XT_W_KERNEL=3)])
@pytest.mark.parametrize("nc,no,nao", [(2, 1, 20), (9, 2, 40), (5, 2, 26), (33, 1, 60), (35, 2, 70), (40, 1, 72),
                                      (45, 2, 80), (95, 2, 130), (99, 2, 140), (120, 3, 150)])
def test_xc_kernel_variants(hiplib, env, knobs, nc, no, nao):
    """O = 3, 11, 7, 34, 37, 41, 47, 97, 101 and 123: one to eight 16-row sub-tiles of the
    dedicated kernels, with (34, 37, 41, 47, 97, 101) and without a VALU remainder-row block;
    the small-O rho-forward with 1, 3, 9, 11 (odd: one single k-step) and 2, 10, 12 k-steps."""
    from xtddft_amd.operator import DeviceOperator
    env(**knobs)
    mf = make_mf(nao=nao, nc=nc, no=no, ngrid=3000, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(7, hdiag.size)
    op = DeviceOperator(mf, "XTDA")
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("nz", [13, 30, 41])
@pytest.mark.parametrize("sa", [2, 3])
def test_xsf_stored_exchange_blocks(hiplib, nz, sa):
    """4 nz = 52 rows (96-row image), 120 rows (128-row image) and 41 vectors (one
    40-vector batch, 160 rows, + 1)."""
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=30, nc=6, no=3, xctype="GGA", hyb=0.5)
    o = oxsf.XSFOracle(mf, SA=sa)
    fg = oxsf.default_fglobal(mf)
    vind, hdiag = o.gen_tda_operation_sf(foo=0.7, fglobal=fg)
    z = make_trial_vectors(nz, hdiag.size)
    op = DeviceOperator(mf, "XSF", sa=sa, fglobal=fg, foo=0.7, remove=o.re, k_mode="stored")
    op.set_oo_basis(o.vects)
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("nz", [17, 20, 23, 25, 48, 49, 64, 65])
def test_stored_exchange_row_shapes(hiplib, nz):
    """2 nz = 34 / 40 rows: the 32 MFMA rows + VALU remainder shape of the streaming
    exchange kernel; 46 rows: the 48-row MFMA shape; 50 / 96 rows the 96-row image, 98 / 128
    the 128-row image, 130 the 160-row image."""
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=40, nc=8, no=2, ngrid=2000, xctype="GGA", hyb=0.25)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(nz, hdiag.size)
    op = DeviceOperator(mf, "XTDA", k_mode="stored")
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("kind,nz", [("XTDA", 1), ("XTDA", 8), ("XTDA", 9), ("XTDA", 16), ("SF_UP", 16),
                                     ("SF_UP", 30)])
def test_stored_exchange_small_row_counts(hiplib, kind, nz):
    """The 16- and 32-row images of the streaming exchange kernel (M = 2 nz for X-TDA,
    nz for SF-up: 2, 16 | 18, 32 | 16 | 30 rows) against the oracle."""
    from oracle import sf_tda as osf
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=40, nc=8, no=2, ngrid=2000, xctype="GGA", hyb=0.25)
    if kind == "XTDA":
        vind, hdiag = oxtda.gen_tda_operation(mf)
    else:
        vind, hdiag = osf.gen_tda_operation_sf(mf, isf=1)
    z = make_trial_vectors(nz, hdiag.size)
    op = DeviceOperator(mf, kind, k_mode="stored")
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("nz", [1, 2, 3, 5, 7, 13])
@pytest.mark.parametrize("nc,no,nao", [(5, 2, 26), (33, 1, 60), (95, 2, 130), (99, 2, 140), (120, 3, 150)])
@pytest.mark.parametrize("knobs", [dict(), dict(XT_W_KERNEL=1), dict(XT_W_KERNEL=3)])
def test_xc_kernels_small_batches(hiplib, env, knobs, nz, nc, no, nao):
    """Davidson steps with few new vectors: nx = 2 nz = 2, 4, 6, 10, 14, 26 trial pairs
    take the dedicated kernels' small-batch shapes (rho-forward: 8, 4, 2 or 1 pairs per
    block with a pair's k-steps split over 8 / PB waves; M-backward: blocks of 8, 4, 2 or
    1 waves) -- against the oracle."""
    from xtddft_amd.operator import DeviceOperator
    env(**knobs)
    mf = make_mf(nao=nao, nc=nc, no=no, ngrid=3000, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(nz, hdiag.size)
    op = DeviceOperator(mf, "XTDA")
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("nz", [3, 5, 8, 11])
def test_xc_small_o_tail_split(hiplib, env, nz):
    """The small-O rho-forward on a grid of more 64-point blocks than the chip has CUs
    (20 000 points: 313 blocks = 256 + 57 on 256 CUs): the last round's blocks split their
    trial pairs 4 ways (nx = 16, 22), 2 ways (nx = 10) or not at all (nx = 6) -- against the
    oracle."""
    from xtddft_amd.operator import DeviceOperator
    env(XT_W_KERNEL=3)
    mf = make_mf(nao=60, nc=33, no=1, ngrid=20000, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(nz, hdiag.size)
    op = DeviceOperator(mf, "XTDA")
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("nz", [1, 3, 30])
def test_sf_up_single_channel_small_batches(hiplib, nz):
    """SF-up (one channel: nx = nz, odd counts) through the same small-batch shapes."""
    from oracle import sf_tda as osf
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=130, nc=95, no=4, ngrid=3000, xctype="GGA", hyb=0.5)
    vind, hdiag = osf.gen_tda_operation_sf(mf, isf=1)
    z = make_trial_vectors(nz, hdiag.size)
    op = DeviceOperator(mf, "SF_UP")
    assert rel(op.apply(z), vind(z)) < RTOL
