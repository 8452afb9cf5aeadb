"""GPU: the HIP path (through the C ABI) against the CPU oracle and the golden
fixtures.  FP64 throughout; tolerance: relative max-norm 1e-12 on sigma, 1e-9 Ha
on Davidson eigenvalues (BASELINE target 1e-6 Ha)."""
import numpy as np
import pytest

from golden_io import list_cases, load
from oracle import sf_tda as osf
from oracle import xsf_tda as oxsf
from oracle import xtda as oxtda
from xtddft_amd.synthetic import make_mf, make_trial_vectors

pytestmark = pytest.mark.gpu
RTOL = 1e-12


def rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


@pytest.fixture(scope="module", params=["direct", "stored"])
def dev(hiplib, request):
    """DeviceOperator with the exchange forced to the DF sandwich or the stored MO matrix."""
    import functools
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from xtddft_amd.operator import DeviceOperator

    def make(*a, **kw):
        op = DeviceOperator(*a, k_mode=request.param, **kw)
        assert op.k_mode == (request.param if _has_k(op.mf) else "direct")
        return op
    return make


def _has_k(mf):
    return mf.xctype == "HF" or mf.hyb != 0 or mf.omega != 0


def test_exchange_mode_auto_respects_cap(hiplib):
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=26, nc=5, no=2, xctype="GGA", hyb=0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(3, hdiag.size)
    big = DeviceOperator(mf, "XTDA")
    small = DeviceOperator(mf, "XTDA", k_max_gib=1e-6)
    assert big.k_mode == "stored" and big.k_gib > 0
    assert small.k_mode == "direct" and small.k_gib == 0
    assert rel(big.apply(z), vind(z)) < RTOL and rel(small.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("case", list_cases())
def test_golden_fixtures(dev, case):
    mf, ex = load(case)
    kind = str(ex["in_kind"])
    kw = {}
    if kind == "XSF":
        o = oxsf.XSFOracle(mf, SA=3)
        kw = dict(sa=3, fglobal=oxsf.default_fglobal(mf), foo=1.0, remove=True)
    op = dev(mf, kind, **kw)
    if kind == "XSF":
        op.set_oo_basis(o.vects)
    assert rel(op.apply(ex["in_z"]), ex["out_sigma"]) < RTOL


@pytest.mark.parametrize("xct,omega,kind", [("GGA", 0.0, "RO"), ("LDA", 0.0, "RO"), ("HF", 0.0, "RO"),
                                            ("GGA", 0.33, "RO"), ("GGA", 0.0, "U"), ("LDA", 0.33, "U"),
                                            ("HF", 0.0, "U"), ("MGGA", 0.0, "RO"), ("MGGA", 0.0, "U")])
@pytest.mark.parametrize("nz", [1, 7, 41])
def test_xtda_utda(dev, xct, omega, kind, nz):
    mf = make_mf(nao=26, nc=5, no=2, xctype=xct, kind=kind, omega=omega,
                 alpha=0.65 if omega else 0.0, hyb=0.19 if omega else 0.2)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(nz, hdiag.size)
    op = dev(mf, "XTDA" if kind == "RO" else "UTDA")
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("nc,no", [(14, 2), (29, 3), (47, 2), (60, 1), (140, 2)])
def test_xtda_many_occupied(dev, nc, no):
    """Occupied counts O = nc + no spanning 1..4 K-tiles of the fused XC kernels
    (K = O there) and the point kernel's register chunks (O > 128), with V not a
    multiple of the 16-wide virtual blocks."""
    mf = make_mf(nao=nc + no + 53, nc=nc, no=no, xctype="GGA", hyb=0.2, ngrid=3000)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(9, hdiag.size)
    op = dev(mf, "XTDA")
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("kind", ["RO", "U"])
@pytest.mark.parametrize("xct", ["GGA", "LDA", "HF"])
@pytest.mark.parametrize("isf", [-1, 1])
def test_sf(dev, kind, xct, isf):
    mf = make_mf(nao=26, nc=5, no=2, xctype=xct, kind=kind, hyb=0.5)
    vind, hdiag = osf.gen_tda_operation_sf(mf, isf)
    z = make_trial_vectors(6, hdiag.size)
    op = dev(mf, "SF_DOWN" if isf == -1 else "SF_UP")
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("sa", [0, 1, 2, 3])
@pytest.mark.parametrize("no", [2, 3, 4])
def test_xsf(dev, sa, no):
    mf = make_mf(nao=28, nc=5, no=no, xctype="GGA", hyb=0.5)
    o = oxsf.XSFOracle(mf, SA=sa)
    fg = oxsf.default_fglobal(mf)
    vind, hdiag = o.gen_tda_operation_sf(foo=0.7, fglobal=fg)
    z = make_trial_vectors(5, hdiag.size)
    op = dev(mf, "XSF", sa=sa, fglobal=fg, foo=0.7, remove=o.re)
    op.set_oo_basis(o.vects)
    assert rel(op.apply(z), vind(z)) < RTOL
    co, ov = op.xsf_j_diagonals()
    co_ref, ov_ref = o._response_j_diagonals()
    assert np.abs(co - co_ref).max() < 1e-13 and np.abs(ov - ov_ref).max() < 1e-13


def test_device_pointers_and_host_pointers_agree(dev):
    import torch
    mf = make_mf(nao=30, nc=6, no=2, xctype="GGA", hyb=0.2)
    op = dev(mf, "XTDA")
    z = make_trial_vectors(9, op.dim)
    s_host = op.apply(z)
    s_dev = op.apply(torch.as_tensor(z, device="cuda")).cpu().numpy()
    assert np.abs(s_host - s_dev).max() == 0.0


def test_ragged_edges(dev):
    """nv = 1, no = 1 (X-TDA doublet), a single vector, and wrong lengths raise."""
    mf = make_mf(nao=9, nc=6, no=2, xctype="LDA", hyb=0.3)          # nv = 1
    vind, hdiag = oxtda.gen_tda_operation(mf)
    op = dev(mf, "XTDA")
    z = make_trial_vectors(3, hdiag.size)
    assert rel(op.apply(z), vind(z)) < RTOL
    mf = make_mf(nao=20, nc=5, no=1, xctype="GGA", hyb=0.2)         # doublet
    vind, hdiag = oxtda.gen_tda_operation(mf)
    op = dev(mf, "XTDA")
    z = make_trial_vectors(1, hdiag.size)
    assert rel(op.apply(z[0]), vind(z)) < RTOL
    with pytest.raises(ValueError):
        op.apply(np.zeros((2, hdiag.size + 1)))


def test_xsf_doublet_rejected(dev):
    mf = make_mf(nao=20, nc=5, no=1, xctype="GGA", hyb=0.5)
    with pytest.raises(ValueError):
        dev(mf, "XSF", sa=3, fglobal=0.65, remove=True)


def test_sharded_contexts_sum_to_full_operator(dev):
    """The multi-GPU decomposition on one GPU: sum over 3 shard contexts == full."""
    mf = make_mf(nao=40, nc=8, no=2, xctype="GGA", hyb=0.2, omega=0.3, alpha=0.6)
    full = dev(mf, "XTDA")
    z = make_trial_vectors(5, full.dim)
    s = sum(dev(mf, "XTDA", shard=(r, 3)).apply(z) for r in range(3))
    assert rel(s, full.apply(z)) < RTOL
    mf = make_mf(nao=40, nc=8, no=3, xctype="GGA", hyb=0.5)
    o = oxsf.XSFOracle(mf, SA=3)
    fg = oxsf.default_fglobal(mf)
    parts = []
    for r in range(2):
        op = dev(mf, "XSF", sa=3, fglobal=fg, remove=True, shard=(r, 2))
        op.set_oo_basis(o.vects)
        parts.append(op)
    vind, hdiag = o.gen_tda_operation_sf(fglobal=fg)
    z = make_trial_vectors(4, hdiag.size)
    assert rel(parts[0].apply(z) + parts[1].apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("replicate", [False, True])
@pytest.mark.parametrize("case", ["xtda_rsh", "utda", "sf_up_u", "sf_down", "xsf_sa3", "xtda_eri8"])
def test_partitioned_contexts_sum_to_full_operator(dev, case, replicate):
    """Every kind: sum over 3 rank contexts == full operator, with the factor
    aux-sliced or replicated + partitioned (aux window, stored-exchange rows)."""
    from xtddft_amd.synthetic import as_eri8
    kw, o = {}, None
    if case == "xtda_rsh":
        mf, kind = make_mf(nao=30, nc=6, no=2, xctype="GGA", hyb=0.2, omega=0.3, alpha=0.6), "XTDA"
    elif case == "utda":
        mf, kind = make_mf(nao=30, nc=6, no=2, xctype="LDA", kind="U", hyb=0.25), "UTDA"
    elif case == "sf_up_u":
        mf, kind = make_mf(nao=30, nc=6, no=2, xctype="GGA", kind="U", hyb=0.5), "SF_UP"
    elif case == "sf_down":
        mf, kind = make_mf(nao=30, nc=6, no=2, xctype="GGA", hyb=0.5), "SF_DOWN"
    elif case == "xtda_eri8":
        mf, kind = as_eri8(make_mf(nao=24, nc=5, no=2, xctype="GGA", hyb=0.2)), "XTDA"
    else:
        mf, kind = make_mf(nao=30, nc=6, no=3, xctype="GGA", hyb=0.5), "XSF"
        o = oxsf.XSFOracle(mf, SA=3)
        kw = dict(sa=3, fglobal=oxsf.default_fglobal(mf), remove=True)
    full = dev(mf, kind, **kw)
    parts = [dev(mf, kind, shard=(r, 3), replicate_df=replicate, **kw) for r in range(3)]
    if o is not None:
        for op in [full] + parts:
            op.set_oo_basis(o.vects)
    z = make_trial_vectors(4, full.dim)
    assert all(p.replicate_df == replicate for p in parts)
    assert rel(sum(p.apply(z) for p in parts), full.apply(z)) < RTOL


# ---- stored ERIs (jk_mode ERI8): device pivoted Cholesky + the DF engine ----
ERI8_TOL = 1e-11   # Cholesky to 1e-13 x max diagonal: exact to round-off at these sizes


@pytest.mark.parametrize("case", ["xtda_gga", "xtda_rsh", "utda_lda", "sf_down", "sf_up", "xsf_sa"])
def test_eri8_equals_df(dev, case):
    """ERI8 (the packed ERIs sum_P B B) and DF (B) on the same tensor agree, and
    both match the oracle (the two modes test each other)."""
    from xtddft_amd.synthetic import as_eri8
    kw, o = {}, None
    if case == "xtda_gga":
        mf, kind = make_mf(nao=24, nc=4, no=2, xctype="GGA"), "XTDA"
        vind = oxtda.gen_tda_operation(mf)[0]
    elif case == "xtda_rsh":
        mf, kind = make_mf(nao=24, nc=4, no=2, xctype="GGA", omega=0.33, alpha=0.65, hyb=0.19), "XTDA"
        vind = oxtda.gen_tda_operation(mf)[0]
    elif case == "utda_lda":
        mf, kind = make_mf(nao=24, nc=4, no=2, xctype="LDA", kind="U"), "UTDA"
        vind = oxtda.gen_tda_operation(mf)[0]
    elif case in ("sf_down", "sf_up"):
        mf = make_mf(nao=24, nc=4, no=2, xctype="GGA", hyb=0.5)
        isf = -1 if case == "sf_down" else 1
        kind = "SF_DOWN" if isf == -1 else "SF_UP"
        vind = osf.gen_tda_operation_sf(mf, isf)[0]
    else:
        mf, kind = make_mf(nao=24, nc=4, no=3, xctype="GGA", hyb=0.5), "XSF"
        o = oxsf.XSFOracle(mf, SA=2)
        kw = dict(sa=2, fglobal=oxsf.default_fglobal(mf), foo=0.7, remove=o.re)
        vind = o.gen_tda_operation_sf(foo=0.7, fglobal=kw["fglobal"])[0]
    op_df, op_eri = dev(mf, kind, **kw), dev(as_eri8(mf), kind, **kw)
    if o is not None:
        op_df.set_oo_basis(o.vects)
        op_eri.set_oo_basis(o.vects)
    z = make_trial_vectors(5, op_df.dim)
    s_df, s_eri = op_df.apply(z), op_eri.apply(z)
    assert rel(s_eri, s_df) < ERI8_TOL
    assert rel(s_eri, vind(z)) < ERI8_TOL
    naux, rank = op_eri.naux()
    assert rank == mf.naux and naux == mf.naux   # synthetic B has full column rank naux < npair
    if kind == "XSF":
        co, ov = op_eri.xsf_j_diagonals()
        co_ref, ov_ref = op_df.xsf_j_diagonals()
        assert np.abs(co - co_ref).max() < 1e-12 and np.abs(ov - ov_ref).max() < 1e-12


def test_eri8_sharded_cholesky_sums_to_full(dev):
    """Aux sharding of the Cholesky vectors (multi-GPU): the
    per-rank partial sigma (one-electron terms on rank 0) sum to the full sigma."""
    from xtddft_amd.synthetic import as_eri8
    mf = as_eri8(make_mf(nao=24, nc=4, no=2, xctype="GGA", omega=0.33, alpha=0.65, hyb=0.19))
    z = make_trial_vectors(4, dev(mf, "XTDA").dim)
    full = dev(mf, "XTDA").apply(z)
    parts = [dev(mf, "XTDA", shard=(r, 3)).apply(z) for r in range(3)]
    assert rel(sum(parts), full) < 1e-13


def test_apply_boundary_checks(hiplib):
    """DeviceOperator.apply at the C-ABI boundary: an empty batch returns an empty result
    (host and device) without a launch; a zero vector maps to exactly zero; float32 input,
    a wrong length, or an `out` of the wrong shape / dtype is refused before any kernel
    could read or write past a buffer."""
    import torch
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=26, nc=5, no=2, xctype="GGA", hyb=0.2)
    op = DeviceOperator(mf, "XTDA")
    assert op.apply(np.zeros((0, op.dim))).shape == (0, op.dim)
    z0 = torch.zeros((0, op.dim), dtype=torch.float64, device="cuda")
    assert tuple(op.apply(z0).shape) == (0, op.dim)
    zero = torch.zeros((2, op.dim), dtype=torch.float64, device="cuda")
    assert float(op.apply(zero).abs().max()) == 0.0
    z = torch.randn((3, op.dim), dtype=torch.float64, device="cuda")
    with pytest.raises(TypeError):
        op.apply(z.float())
    with pytest.raises(ValueError):
        op.apply(z[:, :-1])
    with pytest.raises(ValueError):
        op.apply(z, out=torch.empty((2, op.dim), dtype=torch.float64, device="cuda"))
    with pytest.raises(ValueError):
        op.apply(z, out=torch.empty((3, op.dim), dtype=torch.float32, device="cuda"))
    out = torch.empty_like(z)
    assert op.apply(z, out=out) is out
    assert rel(out.cpu().numpy(), op.apply(z.cpu().numpy())) < 1e-14
    op.close()


# ---- multicollinear spin-flip kernel (method=1, SF_TDA.py:855-1047) ----------
@pytest.mark.parametrize("kind", ["RO", "U"])
@pytest.mark.parametrize("xct", ["GGA", "LDA", "MGGA"])
@pytest.mark.parametrize("op_kind", ["SF_DOWN", "SF_UP", "XSF"])
@pytest.mark.parametrize("nz", [1, 5, 13])
def test_sf_multicollinear(dev, kind, xct, op_kind, nz):
    """Device spin-flip response with the multicollinear kernel (the one-channel GGA /
    MGGA point kernels, the LDA scalar path) against the oracle's AO route of
    nr_uks_fxc_sf_tda_mc (SF_TDA.py:976-1047) on the same synthetic kernel."""
    mf = make_mf(nao=26, nc=5, no=2, xctype=xct, kind=kind, hyb=0.5)
    kw = {}
    if op_kind == "XSF":
        o = oxsf.XSFOracle(mf, method=1)
        kw = dict(sa=o.SA, fglobal=0.4, foo=0.8, remove=o.re)
        vind, hdiag = o.gen_tda_operation_sf(foo=0.8, fglobal=0.4)
    else:
        vind, hdiag = osf.gen_tda_operation_sf(mf, -1 if op_kind == "SF_DOWN" else 1, method=1)
    z = make_trial_vectors(nz, hdiag.size)
    op = dev(mf, op_kind, sf_kernel="mc", mc_kernel=mf.fxc_sf_mc, **kw)
    if op_kind == "XSF":
        op.set_oo_basis(o.vects)
    assert rel(op.apply(z), vind(z)) < RTOL
    if nz == 5 and op_kind == "SF_DOWN":   # the kernel changes the operator: ALDA0 differs
        alda0 = dev(mf, op_kind)
        assert rel(alda0.apply(z), vind(z)) > 1e-3


@pytest.mark.parametrize("nc", [60, 140, 270])
def test_sf_multicollinear_many_occupied(dev, nc):
    """The one-channel GGA point kernel's other variants: O > 128 (one vector per
    reduction, 4 register chunks) and O > 256 (the LDS block kernel)."""
    mf = make_mf(nao=nc + 2 + 21, nc=nc, no=2, xctype="GGA", hyb=0.5, ngrid=1500)
    vind, hdiag = osf.gen_tda_operation_sf(mf, -1, method=1)
    z = make_trial_vectors(3, hdiag.size)
    op = dev(mf, "SF_DOWN", sf_kernel="mc", mc_kernel=mf.fxc_sf_mc)
    assert rel(op.apply(z), vind(z)) < RTOL


@pytest.mark.parametrize("nranks", [4, 5, 8])
def test_partitioned_operator_at_driver_rank_counts(hiplib, nranks):
    """The headline's O = 101 occupied rows over 4, 5 and 8 ranks (replicated factor: aux
    windows + stored-exchange rows, and the direct aux-window partition): the parts sum to
    the full operator and the oracle at every rank count the scaling run uses."""
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=130, nc=99, no=2, xctype="GGA", hyb=0.25, ngrid=3000)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(4, hdiag.size)
    ref = vind(z)
    for rep in (True, False):
        parts = [DeviceOperator(mf, "XTDA", k_mode="stored" if rep else "direct", shard=(r, nranks),
                                replicate_df=rep) for r in range(nranks)]
        assert rel(sum(p.apply(z) for p in parts), ref) < RTOL
        del parts


@pytest.mark.parametrize("nz", [4, 30])
@pytest.mark.parametrize("nranks", [2, 3])
def test_partitioned_stored_exchange_many_rows(hiplib, nranks, nz):
    """Stored exchange over a replicated factor with >= 2 KX_FOLD chunks of occupied rows
    per rank (O = 48 over 2 and 3 ranks): the symmetric build's mirror runs for row blocks
    that start past 0 (i0 > 0), and each partitioned context drops the factor rows outside
    its aux window after the build (xt_prepare).  The summed parts equal the full operator
    and the oracle; 2 nz = 8 and 60 stream rows (the 16- and 96-row images)."""
    from xtddft_amd.operator import DeviceOperator
    mf = make_mf(nao=80, nc=46, no=2, xctype="GGA", hyb=0.25, ngrid=2000)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(nz, hdiag.size)
    full = DeviceOperator(mf, "XTDA", k_mode="stored")
    parts = [DeviceOperator(mf, "XTDA", k_mode="stored", shard=(r, nranks), replicate_df=True)
             for r in range(nranks)]
    assert all(p.k_mode == "stored" for p in parts)
    rows = [p.partition["exchange_rows"] for p in parts]
    assert all(i1 - i0 >= 2 * 8 for i0, i1 in rows) and rows[-1][0] > 0
    win = [p.partition["aux"] for p in parts]
    assert [p.naux()[0] for p in parts] == [p1 - p0 for p0, p1 in win]   # factor trimmed to the window
    s = sum(p.apply(z) for p in parts)
    assert rel(s, full.apply(z)) < RTOL
    assert rel(s, vind(z)) < RTOL
