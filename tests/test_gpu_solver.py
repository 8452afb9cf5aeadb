"""GPU: the FP64-MFMA GEMM engine, the device Davidson and the reference-style
drivers, plus size-independent properties at larger sizes."""
import ctypes

import numpy as np
import pytest

from oracle import davidson as odav
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


@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (17, 33, 5), (128, 128, 16), (200, 301, 257),
                                   (40, 7, 100000), (513, 129, 64), (3, 1000, 0)])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_dgemm_layouts(torch, hiplib, m, n, k, ta, tb):
    from xtddft_amd import _capi
    g = torch.Generator(device="cuda").manual_seed(m * 7 + n * 13 + k)
    a = torch.randn((k, m) if ta else (m, k), dtype=torch.float64, device="cuda", generator=g)
    b = torch.randn((n, k) if tb else (k, n), dtype=torch.float64, device="cuda", generator=g)
    c = torch.randn((m, n), dtype=torch.float64, device="cuda", generator=g)
    ref = 0.7 * ((a.T if ta else a) @ (b.T if tb else b)) - 0.3 * c
    st = torch.cuda.current_stream().cuda_stream
    _capi.check(hiplib.xt_dgemm(ta, tb, m, n, k, 0.7, a.data_ptr(), a.shape[1], b.data_ptr(),
                                b.shape[1], -0.3, c.data_ptr(), n, ctypes.c_void_p(st)), "dgemm")
    torch.cuda.synchronize()
    scale = max(1.0, float(ref.abs().max()))
    assert float((c - ref).abs().max()) / scale < 1e-13 * max(1, k) ** 0.5


@pytest.mark.parametrize("m,n,k,r,nb", [(200, 301, 77, 3, 1), (128, 96, 40, 2, 2), (97, 130, 33, 1, 1),
                                         (300, 250, 1000, 4, 1)])
@pytest.mark.parametrize("ak,bk", [(False, False), (True, False), (False, True), (True, True)])
def test_dgemm_strided_reduce_index(torch, hiplib, m, n, k, r, nb, ak, bk):
    """xt_dgemm_strided: C[b] = alpha sum_r A[b,r] B[b,r] + beta C[b] against torch for
    every operand layout (ak: A k-contiguous, bk: B k-contiguous), a reduce index
    r > 1 and ragged K (K % 32 != 0) -- (False, False) with M, N >= 96 is the BK-32
    rows-on-SIMD tile and its masked ragged-K instantiation."""
    from xtddft_amd import _capi
    g = torch.Generator(device="cuda").manual_seed(m + 3 * n + 7 * k + r)
    # A as (nb, r, m, k) k-contiguous or (nb, r, k, m) m-contiguous; B as (nb, r, k, n) or (nb, r, n, k)
    a = torch.randn((nb, r, m, k) if ak else (nb, r, k, m), dtype=torch.float64, device="cuda", generator=g)
    b = torch.randn((nb, r, n, k) if bk else (nb, r, k, n), dtype=torch.float64, device="cuda", generator=g)
    c = torch.randn((nb, m, n), dtype=torch.float64, device="cuda", generator=g)
    am = a if ak else a.transpose(2, 3)
    bm = b.transpose(2, 3) if bk else b
    ref = 0.7 * torch.einsum("brmk,brkn->bmn", am, bm) - 0.3 * c
    sAm, sAk = (k, 1) if ak else (1, m)
    sBk, sBn = (1, k) if bk else (n, 1)
    st = torch.cuda.current_stream().cuda_stream
    _capi.check(hiplib.xt_dgemm_strided(m, n, k, r, nb, 0.7, a.data_ptr(), sAm, sAk, m * k, r * m * k,
                                        b.data_ptr(), sBk, sBn, k * n, r * k * n, -0.3, c.data_ptr(), n, m * n,
                                        ctypes.c_void_p(st)), "dgemm_strided")
    torch.cuda.synchronize()
    scale = max(1.0, float(ref.abs().max()))
    assert float((c - ref).abs().max()) / scale < 1e-13 * (r * k) ** 0.5


def test_davidson_checkpoint_and_restart(torch, tmp_path):
    """davidson.checkpoint saves the Ritz vectors every iteration; a solve restarted from
    the file (x0 = restart_guess) converges to the same roots in fewer iterations."""
    from xtddft_amd import XTDA
    from xtddft_amd.davidson import checkpoint, restart_guess
    mf = make_mf(nao=40, nc=8, no=2, xctype="GGA", hyb=0.2)
    path = str(tmp_path / "dav.npz")
    x = XTDA(None, mf, nstates=6)
    x.callback = checkpoint(path)
    x.max_cycle = 4                       # interrupted before convergence
    x.kernel()
    x0, e_ck, icyc = restart_guess(path)
    assert x0.shape == (6, x.operator().dim) and icyc >= 1
    y = XTDA(None, mf, nstates=6)
    e_full = y.kernel()
    z = XTDA(None, mf, nstates=6)
    e_re = z.Davidson(x0=x0)
    assert np.all(z.converged) and np.abs(np.asarray(e_re) - np.asarray(e_full)).max() < 1e-9
    assert z.icyc < y.icyc


def test_davidson_matches_oracle_davidson(torch):
    from xtddft_amd.davidson import DiagPrecond, davidson1
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=40, nc=8, no=2, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    x0 = oxtda.get_init_guess(mf, 8)
    # (tol_residual 1e-7 with lindep 1e-12 makes the reference algorithm exit early on
    #  linear dependence -- both solvers do -- so the comparison runs at 1e-6)
    c1, e1, _, _ = odav.davidson1(vind, x0, oxtda.get_precond(mf, hdiag), tol_residual=1e-6,
                                  lindep=1e-12, nroots=8, pick=oxtda.pickeig, max_cycle=100)
    op = DeviceOperator(mf, "XTDA")
    c2, e2, x2, _ = davidson1(op.apply, x0, DiagPrecond(hdiag, 0.0), tol_residual=1e-6, lindep=1e-12,
                              nroots=8, pick=oxtda.pickeig, max_cycle=100)
    assert c1.all() and c2.all()
    assert np.abs(e1 - e2).max() < 1e-9
    x2 = np.asarray(x2)
    assert np.allclose(x2 @ x2.T, np.eye(8), atol=1e-8)


def test_xtda_driver_davidson_and_full_diag(torch):
    from xtddft_amd import XTDA
    mf = make_mf(nao=36, nc=7, no=2, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)
    x = XTDA(mf.mol, mf, nstates=6)
    e = x.kernel()
    assert x.converged.all() and np.abs(e - w[:6]).max() < 1e-9
    assert x.v.shape == (hdiag.size, 6) and x.dS2.shape == (6,)
    y = XTDA(mf.mol, mf, nstates=6, use_Davidson=False)
    assert np.abs(y.kernel() - w[:6]).max() < 1e-12
    lines = y.analyze(verbose=False)
    assert lines[0].startswith("D1")


def test_sf_and_xsf_drivers(torch):
    from xtddft_amd import SF_TDA, XSF_TDA
    mf = make_mf(nao=36, nc=7, no=3, xctype="GGA", hyb=0.5)
    for isf in (-1, 1):
        e, v = SF_TDA(mf, isf=isf).kernel(nstates=4)
        vind, hdiag = osf.gen_tda_operation_sf(mf, isf)
        w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)
        assert np.abs(e - w[:4] * 27.2113834).max() < 1e-5       # tol 1e-7 (SF_TDA.py:392)
        e2, _ = SF_TDA(mf, isf=isf, davidson=False).kernel(nstates=4)
        assert np.abs(e2 - w[:4] * 27.2113834).max() < 1e-9
    x = XSF_TDA(mf)
    e, v = x.kernel(nstates=5)
    o = oxsf.XSFOracle(mf)
    vind, hdiag = o.gen_tda_operation_sf()
    w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)
    assert x.converged.all() and np.abs(e - w[:5] * 27.21138505).max() < 1e-5
    e2, _ = XSF_TDA(mf, davidson=False).kernel(nstates=5)
    assert np.abs(e2 - w[:5] * 27.21138505).max() < 1e-9


@pytest.mark.parametrize("kind", ["XTDA", "SF_DOWN"])
def test_properties_at_larger_size(torch, kind):
    """Symmetry <y, A x> = <A y, x> and linearity at nao = 240 (oracle too slow here)."""
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=240, nc=40, no=2, naux=600, ngrid=20000, xctype="GGA", hyb=0.3,
                 omega=0.3, alpha=0.6)
    op = DeviceOperator(mf, kind)
    x = make_trial_vectors(4, op.dim, seed=1)
    y = make_trial_vectors(4, op.dim, seed=2)
    ax, ay = op.apply(x), op.apply(y)
    lhs, rhs = y @ ax.T, ay @ x.T
    assert np.abs(lhs - rhs).max() < 1e-12 * np.abs(lhs).max()
    comb = op.apply(0.3 * x - 1.7 * y)
    assert np.abs(comb - (0.3 * ax - 1.7 * ay)).max() < 1e-12 * np.abs(comb).max()
    # the batch size does not change a vector's image
    single = op.apply(x[2:3])
    assert np.abs(single - ax[2:3]).max() < 1e-13 * np.abs(single).max()


def test_davidson_follow_state_and_lessio_accepted(torch):
    """follow_state (Davidson.py:246-253) restarts from the previous Ritz vectors
    only on a residual blow-up; on a regular problem it leaves the roots unchanged.
    lessio has no effect with the subspace in memory, as in the reference."""
    from xtddft_amd.davidson import DiagPrecond, davidson1
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=30, nc=6, no=2, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    x0 = oxtda.get_init_guess(mf, 4)
    op = DeviceOperator(mf, "XTDA")
    kw = dict(tol_residual=1e-6, lindep=1e-12, nroots=4, pick=oxtda.pickeig, max_cycle=100)
    c1, e1, _, _ = davidson1(op.apply, x0, DiagPrecond(hdiag, 0.0), **kw)
    c2, e2, _, _ = davidson1(op.apply, x0, DiagPrecond(hdiag, 0.0), follow_state=True, lessio=True, **kw)
    assert c1.all() and c2.all() and np.abs(np.asarray(e1) - np.asarray(e2)).max() < 1e-10


def _mgs_host(x, lindep):
    """PySCF _qr on the host (modified Gram-Schmidt, drop norm**2 <= lindep)."""
    q = []
    for row in x:
        v = row.copy()
        for u in q:
            v -= u * (u @ v)
        for u in q:
            v -= u * (u @ v)
        n2 = v @ v
        if n2 > lindep:
            q.append(v / np.sqrt(n2))
    return np.asarray(q)


@pytest.mark.parametrize("eps", [1e-3, 1e-5, 1e-6])
def test_qr_near_collinear_rows(torch, eps):
    """Blocks with nearly collinear rows at lindep 1e-14 (the SF drivers' value,
    SF_TDA.py:392): the block QR keeps the same rows as the vector-by-vector
    reference rule and its output is orthonormal to round-off (the
    Gram-matrix route squares the conditioning; nearly dependent blocks take the
    vector-wise path)."""
    from xtddft_amd.davidson import _Dev, _qr, _qr_vectorwise
    rng = np.random.default_rng(11)
    dim = 600
    base = rng.normal(size=(5, dim))
    rows = [base[0], base[1], base[0] + eps * rng.normal(size=dim), base[2],
            base[1] + eps * rng.normal(size=dim), 0.5 * base[0] + 2 * base[2],      # exactly dependent
            base[3], base[2] + eps * rng.normal(size=dim), base[4]]
    x = np.asarray(rows)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    dev = _Dev(0)
    xt = torch.as_tensor(x, device="cuda")
    q = _qr(dev, xt, 1e-14).cpu().numpy()
    qv = _qr_vectorwise(dev, xt, 1e-14).cpu().numpy()
    ref = _mgs_host(x, 1e-14)
    assert q.shape[0] == qv.shape[0] == ref.shape[0] == 8
    for a in (q, qv):
        assert np.abs(a @ a.T - np.eye(a.shape[0])).max() < 1e-12
        # same span as the reference
        assert np.abs(a @ ref.T @ ref - a).max() < 1e-9


def test_davidson_follow_state_restart_branch(torch):
    """An aop that corrupts one step's images (a residual blow-up) makes follow_state restart
    from the previous Ritz vectors (Davidson.py:246-253): the next block lies in the
    span of the subspace before the corrupted step, and the solver still converges
    to the uncorrupted roots."""
    from xtddft_amd.davidson import DiagPrecond, davidson1
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=30, nc=6, no=2, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    x0 = oxtda.get_init_guess(mf, 3)
    op = DeviceOperator(mf, "XTDA")
    w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)
    blocks, state = [], dict(calls=0, hit=None)

    def aop(xt):
        blocks.append(xt.cpu().numpy().copy())
        s = op.apply(xt)
        state["calls"] += 1
        if state["calls"] == 4:
            # add a direction outside the subspace to every image: the subspace matrix is
            # unchanged, the residuals of this step blow up
            state["hit"] = len(blocks) - 1
            span, _ = np.linalg.qr(np.concatenate(blocks).T)
            u = np.random.default_rng(5).normal(size=span.shape[0])
            u -= span @ (span.T @ u)
            u /= np.linalg.norm(u)
            s = s + 200.0 * torch.as_tensor(np.broadcast_to(u, s.shape).copy(), device=s.device)
        return s
    c, e, _, _ = davidson1(aop, x0, DiagPrecond(hdiag, 0.0), tol_residual=1e-6, lindep=1e-12, nroots=3,
                           pick=oxtda.pickeig, max_cycle=100, follow_state=True, max_space=30)
    k = state["hit"]
    assert k is not None and len(blocks) > k + 1
    before = np.concatenate(blocks[:k])
    qb, _ = np.linalg.qr(before.T)
    nxt = blocks[k + 1]
    assert np.abs(nxt.T - qb @ (qb.T @ nxt.T)).max() < 1e-8      # restarted inside the old span
    assert c.all() and np.abs(np.asarray(e) - w[:3]).max() < 1e-8
