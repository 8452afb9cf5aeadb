"""Seeded synthetic open-shell problems.

PySCF (integrals, grids, libxc, SCF) is not part of this framework, so the
operators are exercised on synthetic mean fields of the exact shapes and
structure the reference consumes:

* orthonormal MO coefficients (overlap = I), ROKS ordering core|open|virtual;
* per-spin KS Fock matrices ``diag(eps) + 1e-3 sym(N)`` and pure-HF Fock
  matrices ``F + 1e-2 sym(N)`` (the Delta-A inputs, XTDA.py:607-613);
* a symmetric DF factor ``B[P,mu,nu] = sym(N) * exp(-|mu-nu|/50)`` whose
  ``sum_P B B`` is a PSD, 8-fold symmetric ERI tensor;
* a grid with AO values/gradients, weights and an ``fxc`` kernel symmetric
  under (s,x) <-> (t,y); an ALDA0 ``fxc_sf`` kernel (weighted) and a multicollinear
  spin-flip kernel ``fxc_sf_mc`` (nk, nk, ngrid), symmetric, un-weighted (drawn from
  its own stream, so the other tensors do not depend on it).

Magnitudes are calibrated so that the response part of A is ~0.05-0.1 Ha
against orbital gaps >= 0.25 Ha, giving a positive spectrum that the
reference's Davidson criteria (pick w > 1e-3) handle the way they do for
real molecules.  Seed 20261015 is the default.
"""
from __future__ import annotations

import numpy as np

from .meanfield import Grid, MeanField, Mole

DEFAULT_SEED = 20261015


def _sym(rng, n, scale=1.0):
    g = rng.standard_normal((n, n))
    return (g + g.T) * (scale / np.sqrt(2.0))


def _orthonormal(rng, n):
    q, r = np.linalg.qr(rng.standard_normal((n, n)))
    return q * np.sign(np.diag(r))


def df_scale(nao, naux, nocc, nvir, target=0.08, decay=50.0):
    """Entry scale for B so that the Coulomb block of A has norm ~ target."""
    k = np.arange(nao)
    d2 = np.exp(-2.0 * np.abs(k[:, None] - k[None, :]) / decay)
    std_mo = np.sqrt(d2.mean())
    sigma = np.sqrt(target) / (np.sqrt(naux) + np.sqrt(max(1, nocc * nvir)))
    return sigma / std_mo


def grid_scale(ngrid, nocc, nvir, target=0.05):
    """AO-value scale so the XC block of A has norm ~ target."""
    mean_wf = 0.275 / ngrid
    return (target / (mean_wf * (np.sqrt(ngrid) + np.sqrt(max(1, nocc * nvir))) ** 2)) ** 0.25


def make_df_tensor(rng, nao, naux, scale, decay=50.0):
    k = np.arange(nao)
    dmat = np.exp(-np.abs(k[:, None] - k[None, :]) / decay)
    b = np.empty((naux, nao, nao))
    # generated in P chunks (the same random stream as one draw) to bound the temporaries
    pc = max(1, (1 << 28) // (8 * nao * nao))
    for p0 in range(0, naux, pc):
        t = rng.standard_normal((min(pc, naux - p0), nao, nao))
        b[p0:p0 + t.shape[0]] = (t + t.transpose(0, 2, 1)) * (scale / np.sqrt(2.0)) * dmat[None]
    return b


def make_grid(rng, nao, ngrid, ncomp, scale):
    ao = rng.standard_normal((ncomp, ngrid, nao)) * scale
    w = rng.uniform(0.0, 1.0, ngrid) / ngrid
    return Grid(ao=ao, weights=w)


def make_fxc(rng, ngrid, ncomp):
    """UKS kernel (2,ncomp,2,ncomp,ngrid) symmetric under (s,x)<->(t,y)."""
    n = 2 * ncomp
    f = rng.standard_normal((n, n, ngrid)) * 0.01
    f = 0.5 * (f + f.transpose(1, 0, 2))
    for s in range(2):
        for t in range(2):
            v = -rng.uniform(0.1, 1.0, ngrid)
            f[s * ncomp, t * ncomp] = v
            f[t * ncomp, s * ncomp] = v
    return f.reshape(2, ncomp, 2, ncomp, ngrid)


def make_fxc_sf_mc(rng, ngrid, nk):
    """Multicollinear spin-flip kernel (nk, nk, ngrid) symmetric in (x, y); its (s, s)
    entry negative like the collinear-limit kernel (v_a - v_b) / (2 s)."""
    f = rng.standard_normal((nk, nk, ngrid)) * 0.01
    f = 0.5 * (f + f.transpose(1, 0, 2))
    f[0, 0] = -0.5 * rng.uniform(0.1, 1.0, ngrid)
    return f


def make_mf(nao=24, nc=5, no=2, naux=None, ngrid=None, xctype="GGA", hyb=0.2,
            omega=0.0, alpha=0.0, kind="RO", seed=DEFAULT_SEED,
            jk_target=0.08, xc_target=0.05) -> MeanField:
    """Build a seeded synthetic ROKS ('RO') or UKS ('U') mean field.

    nc / no are the closed / open shell counts (2S = no); nvir = nao-nc-no.
    ``xctype='HF'`` gives a pure Hartree-Fock response (no grid).
    ``omega != 0`` adds a long-range DF factor (range-separated hybrid).
    """
    rng = np.random.default_rng(seed)
    nmo = nao
    nv = nmo - nc - no
    if nv < 1 or nc < 1:
        raise ValueError("need at least one core and one virtual orbital")
    naux = naux if naux is not None else 3 * nao
    ngrid = ngrid if ngrid is not None else 60 * nao
    ncomp = 4 if xctype in ("GGA", "MGGA") else 1     # AO values (+ gradients) on the grid

    eps_c = np.sort(rng.uniform(-1.0, -0.5, nc))
    eps_o = np.sort(rng.uniform(-0.45, -0.25, no))
    eps_v = np.sort(rng.uniform(0.05, 3.0, nv))
    eps = np.concatenate([eps_c, eps_o, eps_v])

    def fock_pair(shift_o_a, shift_o_b):
        ea = eps.copy(); eb = eps.copy()
        ea[nc:nc + no] += shift_o_a
        eb[nc:nc + no] += shift_o_b
        eb[:nc] += 0.02
        eb[nc + no:] += 0.02
        fa = np.diag(ea) + _sym(rng, nmo, 1e-3)
        fb = np.diag(eb) + _sym(rng, nmo, 1e-3)
        return fa, fb

    fa_mo, fb_mo = fock_pair(-0.05, 0.15)
    fa_hf = fa_mo + _sym(rng, nmo, 1e-2)
    fb_hf = fb_mo + _sym(rng, nmo, 1e-2)

    if kind == "RO":
        c = _orthonormal(rng, nao)
        mo_coeff = c
        mo_occ = np.concatenate([np.full(nc, 2.0), np.full(no, 1.0), np.zeros(nv)])
        mo_energy = eps.copy()
        ca = cb = c
    elif kind == "U":
        ca = _orthonormal(rng, nao)
        rot = _orthonormal(rng, nao)
        # beta orbitals: a small rotation of the alpha set
        cb = ca @ (np.eye(nao) + 0.05 * (rot - rot.T))
        cb, r = np.linalg.qr(cb)
        cb = cb * np.sign(np.diag(r))
        mo_coeff = np.asarray([ca, cb])
        occa = np.zeros(nmo); occa[:nc + no] = 1
        occb = np.zeros(nmo); occb[:nc] = 1
        mo_occ = np.asarray([occa, occb])
        mo_energy = np.asarray([np.diag(fa_mo).copy(), np.diag(fb_mo).copy()])
    else:
        raise ValueError("kind must be 'RO' or 'U'")

    h1e = _sym(rng, nao, 0.1)
    fa_ao = ca @ fa_mo @ ca.T
    fb_ao = cb @ fb_mo @ cb.T
    veff = np.asarray([fa_ao - h1e, fb_ao - h1e])
    veff_hf = np.asarray([ca @ fa_hf @ ca.T - h1e, cb @ fb_hf @ cb.T - h1e])

    nocc, nvir = nc + no, no + nv
    cderi = make_df_tensor(rng, nao, naux, df_scale(nao, naux, nocc, nvir, jk_target))
    cderi_lr = None
    if omega != 0.0:
        cderi_lr = make_df_tensor(rng, nao, naux, 0.5 * df_scale(nao, naux, nocc, nvir, jk_target))

    grids = fxc = fxc_sf = None
    if xctype != "HF":
        grids = make_grid(rng, nao, ngrid, ncomp, grid_scale(ngrid, nocc, nvir, xc_target))
        fxc = make_fxc(rng, ngrid, 5 if xctype == "MGGA" else ncomp)
        fxc_sf = -rng.uniform(0.1, 1.0, ngrid) * grids.weights
    else:
        hyb, alpha, omega = 1.0, 0.0, 0.0

    fxc_sf_mc = None
    if xctype != "HF":
        fxc_sf_mc = make_fxc_sf_mc(np.random.default_rng(seed + 17), ngrid, 5 if xctype == "MGGA" else ncomp)
    mol = Mole(nao=nao, spin=no, nelectron=2 * nc + no)
    return MeanField(mol=mol, mo_coeff=mo_coeff, mo_occ=mo_occ, mo_energy=mo_energy,
                     h1e=h1e, veff=veff, veff_hf=veff_hf, cderi=cderi, grids=grids,
                     fxc=fxc, fxc_sf=fxc_sf, fxc_sf_mc=fxc_sf_mc, cderi_lr=cderi_lr, xctype=xctype,
                     omega=omega, alpha=alpha, hyb=hyb)


def as_eri8(mf: MeanField, chol_tol: float = 0.0) -> MeanField:
    """The same mean field in jk_mode 'ERI8': the DF factor(s) replaced by the
    8-fold packed ERIs they define, (mu nu|la si) = sum_P B B (SURVEY.md 8(d):
    DF and ERI8 are fed the same tensor so the two modes test each other)."""
    import dataclasses
    from .eri import eri_from_cderi
    eri_lr = eri_from_cderi(mf.cderi_lr) if mf.cderi_lr is not None else None
    return dataclasses.replace(mf, cderi=None, cderi_lr=None, eri=eri_from_cderi(mf.cderi),
                               eri_lr=eri_lr, chol_tol=chol_tol)


GRID_BLOCK = 65536     # grid points per generator block (make_device_mf)
AUX_BLOCK = 64         # DF rows per generator block


def _block_generator(dev, seed, stream, index):
    """A generator for block ``index`` of stream ``stream`` (0: DF factor, 1: grid, 2: the
    multicollinear kernel): every block has its own seed, so a block's values do not depend
    on which rank generates it or on how the global range is split."""
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed((int(seed) * 1000003 + 7919 * (stream + 1) + 104729 * int(index)) % (1 << 62))
    return g


def make_device_mf(nao=1000, nc=99, no=2, naux=None, ngrid=None, xctype="GGA", hyb=0.2,
                   seed=DEFAULT_SEED, device=0, shard=(0, 1), full_aux=False, sf_mc=False,
                   torch_device=None) -> MeanField:
    """Synthetic ROKS problem whose big tensors are generated directly in HBM.

    Same distributions as ``make_mf`` (torch RNG, so not bitwise equal).  The DF factor
    is generated in blocks of AUX_BLOCK rows and the grid in blocks of GRID_BLOCK points,
    each block from its own seed (``_block_generator``): a rank generates only the blocks
    of its shard (aux rows / grid points of ``shard = (rank, nranks)``) and the shards of
    any rank count concatenate to the SAME global tensors -- a sharded run solves the
    operator of the 1-GPU run.  Small per-orbital data (C, Fock, energies) come from
    ``make_mf`` and are identical on every rank.  full_aux: every rank holds the whole DF
    factor (the replicated-factor partition).  sf_mc: also a multicollinear spin-flip
    kernel ``fxc_sf_mc`` (nk, nk, ngrid).  torch_device: generate on that torch device
    instead of ``cuda:device`` (the shard-invariance test runs on the CPU).
    """
    import torch
    naux = naux if naux is not None else 3 * nao
    ngrid = ngrid if ngrid is not None else 1200 * nao
    rank, nranks = shard
    small = make_mf(nao=nao, nc=nc, no=no, naux=1, ngrid=1, xctype=xctype, hyb=hyb, seed=seed)
    dev = torch.device(torch_device) if torch_device is not None else torch.device(f"cuda:{device}")
    nv = nao - nc - no

    def split(n):
        base, rem = divmod(n, nranks)
        lo = rank * base + min(rank, rem)
        return lo, lo + base + (1 if rank < rem else 0)
    p0, p1 = (0, naux) if full_aux else split(naux)
    g0, g1 = split(ngrid)
    nocc, nvir = nc + no, no + nv
    f64 = dict(dtype=torch.float64, device=dev)
    k = torch.arange(nao, **f64)
    dmat = torch.exp(-torch.abs(k[:, None] - k[None, :]) / 50.0)
    sdf = df_scale(nao, naux, nocc, nvir) / np.sqrt(2.0)
    cderi = torch.empty((p1 - p0, nao, nao), **f64)
    for b in range(p0 // AUX_BLOCK, -(-p1 // AUX_BLOCK)):
        b0, b1 = b * AUX_BLOCK, min(naux, (b + 1) * AUX_BLOCK)
        t = torch.randn((b1 - b0, nao, nao), generator=_block_generator(dev, seed, 0, b), **f64)
        lo, hi = max(b0, p0), min(b1, p1)
        cderi[lo - p0:hi - p0] = (t[lo - b0:hi - b0] + t[lo - b0:hi - b0].transpose(1, 2)) * sdf * dmat
        del t
    ncomp = 4 if xctype in ("GGA", "MGGA") else 1
    nf = 5 if xctype == "MGGA" else ncomp              # kernel components (+ tau)
    ng = g1 - g0
    scale = grid_scale(ngrid, nocc, nvir)
    ao = torch.empty((ncomp, ng, nao), **f64)
    w = torch.empty(ng, **f64)
    fxc = torch.empty((2, nf, 2, nf, ng), **f64)
    fxc_sf = torch.empty(ng, **f64)
    fmc = torch.empty((nf, nf, ng), **f64) if sf_mc else None
    n = 2 * nf
    for b in range(g0 // GRID_BLOCK, -(-g1 // GRID_BLOCK)):
        b0, b1 = b * GRID_BLOCK, min(ngrid, (b + 1) * GRID_BLOCK)
        lo, hi = max(b0, g0), min(b1, g1)
        nb, s0, s1, d0, d1 = b1 - b0, lo - b0, hi - b0, lo - g0, hi - g0
        g = _block_generator(dev, seed, 1, b)
        ao[:, d0:d1] = (torch.randn((ncomp, nb, nao), generator=g, **f64) * scale)[:, s0:s1]
        wb = torch.rand(nb, generator=g, **f64) / ngrid
        w[d0:d1] = wb[s0:s1]
        f = torch.randn((n, n, nb), generator=g, **f64) * 0.01
        f = 0.5 * (f + f.transpose(0, 1))
        for sa in range(2):
            for sb in range(2):
                v = -(0.1 + 0.9 * torch.rand(nb, generator=g, **f64))
                f[sa * nf, sb * nf] = v
                f[sb * nf, sa * nf] = v
        fxc[..., d0:d1] = f.reshape(2, nf, 2, nf, nb)[..., s0:s1]
        fxc_sf[d0:d1] = (-(0.1 + 0.9 * torch.rand(nb, generator=g, **f64)) * wb)[s0:s1]
        if sf_mc:
            gm = _block_generator(dev, seed, 2, b)
            m = torch.randn((nf, nf, nb), generator=gm, **f64) * 0.01
            m = 0.5 * (m + m.transpose(0, 1))
            m[0, 0] = -0.5 * (0.1 + 0.9 * torch.rand(nb, generator=gm, **f64))
            fmc[..., d0:d1] = m[..., s0:s1]
        del f
    small.cderi = cderi
    small.grids = Grid(ao=ao, weights=w)
    small.fxc = fxc
    small.fxc_sf = fxc_sf
    small.fxc_sf_mc = fmc
    small.extra = dict(shard=shard, aux_range=(p0, p1), grid_range=(g0, g1), naux_global=naux,
                       ngrid_global=ngrid)
    return small


def make_trial_vectors(nz, dim, seed=DEFAULT_SEED + 1):
    """Row-normalised N(0,1) trial vectors."""
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((nz, dim))
    return z / np.linalg.norm(z, axis=1, keepdims=True)
