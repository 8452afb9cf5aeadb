"""CPU: host-side logic of the framework (no GPU, no compute calls)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import sf_tda as osf
from oracle import xsf_tda as oxsf
from oracle import xtda as oxtda
from xtddft_amd import meanfield, parallel, utils
from xtddft_amd.synthetic import make_mf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "xtddft_amd.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(xt_\w+)\s*\(", txt, re.M)))


def test_library_builds_and_exports_every_header_symbol(hiplib):
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(hiplib, s), s
    from xtddft_amd._capi import ABI_VERSION
    assert hiplib.xt_abi_version() == ABI_VERSION == 7


def test_desc_layout_matches_c_header(tmp_path):
    """ctypes XtDesc has the same size/offsets as the C struct (gcc on the header)."""
    from xtddft_amd._capi import XtDesc
    fields = [f for f, _ in XtDesc._fields_]
    src = tmp_path / "t.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "xtddft_amd.h"\nint main(){'
                   'printf("%zu", sizeof(xt_desc));' +
                   "".join(f'printf(" %zu", offsetof(xt_desc, {f}));' for f in fields) + "return 0;}")
    exe = tmp_path / "t"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)])
    out = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    assert out[0] == ctypes.sizeof(XtDesc)
    assert out[1:] == [getattr(XtDesc, f).offset for f in fields]


def test_create_rejects_bad_descriptor_without_gpu(hiplib):
    """Argument validation happens before any HIP call (reference ValueError, XTDA.py:37)."""
    from xtddft_amd import _capi
    d = _capi.XtDesc(kind=0, restricted=1, nao=10, nmo=10, nc=3, no=2, nv=4)   # nc+no+nv != nmo
    h = ctypes.c_void_p()
    rc = hiplib.xt_create(ctypes.byref(d), ctypes.byref(h))
    assert rc == -1
    with pytest.raises(ValueError):
        _capi.check(rc, "xt_create")
    d = _capi.XtDesc(kind=0, restricted=0, nao=10, nmo=10, nc=3, no=2, nv=5, si=1.0)  # XTDA needs ROKS
    assert hiplib.xt_create(ctypes.byref(d), ctypes.byref(h)) == -1
    d = _capi.XtDesc(kind=2, restricted=1, nao=10, nmo=10, nc=3, no=2, nv=5, sf_kernel=7)  # no such kernel
    assert hiplib.xt_create(ctypes.byref(d), ctypes.byref(h)) == -1
    assert b"sf_kernel" in hiplib.xt_last_error()
    d = _capi.XtDesc(kind=4, restricted=1, nao=10, nmo=10, nc=3, no=1, nv=6, sa=3)   # 2S-1 = 0
    assert hiplib.xt_create(ctypes.byref(d), ctypes.byref(h)) == -1
    assert b"2S-1" in hiplib.xt_last_error()


def test_meanfield_requires_core_open_virtual_order():
    mf = make_mf(nao=10, nc=2, no=2)
    occ = mf.mo_occ.copy()
    occ[[1, 2]] = occ[[2, 1]]
    with pytest.raises(ValueError):
        meanfield.MeanField(mol=mf.mol, mo_coeff=mf.mo_coeff, mo_occ=occ, mo_energy=mf.mo_energy,
                            h1e=mf.h1e, veff=mf.veff, veff_hf=mf.veff_hf, cderi=mf.cderi)


def test_synthetic_is_seeded():
    a = make_mf(nao=12, nc=3, no=2, seed=5)
    b = make_mf(nao=12, nc=3, no=2, seed=5)
    assert np.array_equal(a.cderi, b.cderi) and np.array_equal(a.grids.ao, b.grids.ao)


def test_product_init_guess_and_hdiag_match_oracle():
    from xtddft_amd.xtda import XTDA
    for kind in ("RO", "U"):
        mf = make_mf(nao=16, nc=4, no=2, kind=kind)
        x = XTDA(mf.mol, mf, nstates=5)
        vind, hdiag = oxtda.gen_tda_operation(mf)
        assert np.abs(x._hdiag() - hdiag).max() == 0
        assert np.array_equal(x.get_init_guess(mf, 5), oxtda.get_init_guess(mf, 5))
        pre = oxtda.get_precond(mf, hdiag)
        r = np.random.default_rng(0).standard_normal(hdiag.size)
        assert np.allclose(pre(r.copy(), 0.3), r / (hdiag - 0.3))


def test_sf_and_xsf_host_pieces_match_oracle():
    from xtddft_amd import sf_tda, xsf_tda
    mf = make_mf(nao=16, nc=4, no=3, xctype="GGA", hyb=0.5)
    for isf in (-1, 1):
        assert np.array_equal(sf_tda.init_guess(mf, 4, isf), osf.init_guess(mf, 4, isf))
    for no in (2, 3, 4):
        v = xsf_tda.get_vect(no)
        assert np.array_equal(v, oxsf.get_vect(no))
        assert np.allclose(v.T @ v, np.eye(no * no - 1))
    x = xsf_tda.XSF_TDA.__new__(xsf_tda.XSF_TDA)
    x.hyb, x.alpha, x.omega, x.method = 0.5, 0.0, 0.0, 0
    assert abs(x.default_fglobal() - oxsf.default_fglobal(mf)) < 1e-15


def test_so2st_roundtrip():
    v = np.random.default_rng(1).standard_normal((3 * 5 + 2 * 5 + 3 * 2 + 3 * 5, 4))
    assert np.allclose(utils.st2so(utils.so2st(v, 3, 2, 5), 3, 2, 5), v)


def test_shard_ranges_cover_exactly():
    for n in (1, 7, 3000, 1200000):
        for nr in (1, 2, 3, 8):
            rs = [parallel.shard_range(n, r, nr) for r in range(nr)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(nr - 1))


def test_no_cpu_fallback_in_product():
    """The product package never imports the oracle (test infrastructure only)."""
    pkg = os.path.join(ROOT, "xtddft_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert "import oracle" not in src and "from oracle" not in src, f


# ---- stored-ERI (jk_mode ERI8) host side -----------------------------------
def test_eri_s8_packing_matches_pyscf_convention():
    """xtddft_amd.eri packing == the loop-written ao2mo 's8' convention of the oracle."""
    from oracle.engines import unpack_eri_s8
    from xtddft_amd import eri as E
    rng = np.random.default_rng(3)
    nao = 6
    b = rng.standard_normal((9, nao, nao))
    b = b + b.transpose(0, 2, 1)
    full = np.einsum('pij,pkl->ijkl', b, b)
    packed = E.pack_s8(full)
    assert packed.size == E.npair(nao) * (E.npair(nao) + 1) // 2
    assert np.array_equal(unpack_eri_s8(packed, nao), E.unpack_s8(packed, nao))
    assert np.abs(unpack_eri_s8(packed, nao) - full).max() < 1e-13
    assert np.abs(E.eri_from_cderi(b) - packed).max() < 1e-12


def test_oracle_eri_jk_equals_df_jk():
    """The stored-ERI J/K (PySCF get_jk convention) on sum_P B B equals the DF J/K on B,
    for non-symmetric densities (hermi = 0, XTDA.py:518-543)."""
    from oracle.engines import get_jk, get_jk_eri, unpack_eri_s8
    from xtddft_amd.synthetic import as_eri8, make_mf
    mf = make_mf(nao=10, nc=3, no=2, xctype="HF")
    full = unpack_eri_s8(as_eri8(mf).eri, 10)
    dms = np.random.default_rng(4).standard_normal((3, 10, 10))
    vj, vk = get_jk(mf.cderi, dms)
    vj2, vk2 = get_jk_eri(full, dms)
    assert np.abs(vj - vj2).max() < 1e-13 and np.abs(vk - vk2).max() < 1e-13


def test_meanfield_eri_validation():
    import dataclasses
    from xtddft_amd.synthetic import as_eri8, make_mf
    mf = as_eri8(make_mf(nao=8, nc=2, no=2, xctype="HF"))
    assert mf.jk_mode == "ERI8" and mf.naux == 0
    with pytest.raises(ValueError):
        dataclasses.replace(mf, eri=mf.eri[:-1])
    with pytest.raises(ValueError):
        dataclasses.replace(mf, eri=None)


@pytest.mark.skipif(os.environ.get("XT_ASAN") != "1",
                    reason="host AddressSanitizer build of the whole library takes ~3 min: XT_ASAN=1")
def test_host_asan_build_of_the_c_abi():
    """SURVEY.md section 5 (race detection / sanitizers): every csrc file built with
    -Xarch_host -fsanitize=address, and tests/asan/asan_driver.cpp drives the C ABI's
    validation and error paths under ASan (no GPU needed; tools/asan_host.sh)."""
    r = subprocess.run(["bash", "tools/asan_host.sh"], cwd=ROOT, capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "asan driver: ok" in r.stdout


def test_device_mf_shards_concatenate_to_the_unsharded_tensors():
    """make_device_mf generates the DF factor and the grid in fixed blocks, each from its
    own seed: the shards of 2 and 3 ranks concatenate to the 1-rank tensors exactly, so a
    sharded bench run solves the same operator as N = 1 (torch CPU generator here; the
    device generator has the same block structure)."""
    import torch
    from xtddft_amd.synthetic import make_device_mf
    kw = dict(nao=20, nc=4, no=2, naux=150, ngrid=140000, torch_device="cpu", sf_mc=True)
    full = make_device_mf(**kw)
    for n in (2, 3):
        parts = [make_device_mf(shard=(r, n), **kw) for r in range(n)]
        assert torch.equal(torch.cat([p.grids.ao for p in parts], 1), full.grids.ao)
        assert torch.equal(torch.cat([p.grids.weights for p in parts]), full.grids.weights)
        assert torch.equal(torch.cat([p.cderi for p in parts], 0), full.cderi)
        assert torch.equal(torch.cat([p.fxc for p in parts], -1), full.fxc)
        assert torch.equal(torch.cat([p.fxc_sf_mc for p in parts], -1), full.fxc_sf_mc)
        assert torch.equal(make_device_mf(shard=(1, n), full_aux=True, **kw).cderi, full.cderi)


def test_nlc_functional_follows_the_reference():
    """VV10 (NLC): the reference adds get_vnlc_resp in the X-TDA Davidson response only
    (XTDA.py:515-517) -- not built here, so that path refuses instead of silently differing;
    the explicit A and the SF / XSF paths leave it out with the reference's warning
    (XTDA.py:166-169, SF_TDA.py:490-493, 869-872)."""
    from xtddft_amd.sf_tda import SF_TDA_up
    from xtddft_amd.synthetic import make_mf
    from xtddft_amd.xsf_tda import XSF_TDA
    from xtddft_amd.xtda import XTDA
    mf = make_mf(nao=20, nc=4, no=2, ngrid=500, xctype="GGA", hyb=0.2)
    mf.nlc = True
    with pytest.raises(NotImplementedError, match="get_vnlc_resp"):
        XTDA(None, mf).kernel()
    with pytest.warns(RuntimeWarning, match="NLC functional"):
        SF_TDA_up(mf)
    with pytest.warns(RuntimeWarning, match="NLC functional"):
        XSF_TDA(mf)


def test_cholesky_batch_pivots_reproduce_the_block():
    """qc/dchol.py _batch_pivots (the host half of the blocked in-batch pivoting): on a
    rank-12 PSD block the pivots run largest-residual-first until the residual diagonal
    is below the cut, and the factor's outer product reproduces the block; with a cut
    above the smaller residuals it stops early and every skipped diagonal is <= cut."""
    from xtddft_amd.qc.dchol import _batch_pivots
    rng = np.random.default_rng(3)
    g = rng.normal(size=(30, 12)) * 0.4 ** np.arange(12)      # decaying spectrum
    c = g @ g.T
    piv, lb = _batch_pivots(c, np.diag(c).copy(), 1e-10)
    assert piv.size == 12 and piv[0] == int(np.argmax(np.diag(c)))
    assert np.abs(lb @ lb.T - c).max() < 1e-9 * np.abs(c).max()
    cut = 1e-3 * np.diag(c).max()
    piv2, lb2 = _batch_pivots(c, np.diag(c).copy(), cut)
    assert 0 < piv2.size < 12
    assert np.array_equal(piv2, piv[:piv2.size])
    assert (np.diag(c - lb2 @ lb2.T) <= cut * (1 + 1e-12)).all()


def test_scf_density_factors_follow_the_array():
    """qc/scf.py: the orbital factors handed to the device exchange belong to the exact
    density array they were built with, and are dropped once it is changed in place."""
    from xtddft_amd.qc import ROKS
    from molecules import hf_mol
    mf = ROKS(hf_mol(), "HF")
    c = np.linalg.qr(np.random.default_rng(0).normal(size=(mf.mol.nao, mf.mol.nao)))[0]
    occ = np.zeros(mf.mol.nao)
    occ[:4], occ[4] = 2, 1
    dms = mf._dms(c, occ)
    f = mf._factors_of(dms)
    assert f is not None and np.allclose(f[0] @ f[0].T, dms[0]) and np.allclose(f[1] @ f[1].T, dms[1])
    assert mf._factors_of(dms.copy()) is None
    dms *= 0.5
    assert mf._factors_of(dms) is None
