"""Spin-flip TDA with the reference's API (``xtddft/SF_TDA.py``).

* ``SF_TDA(mf, isf=-1, davidson=True, method=0)`` factory (SF_TDA.py:17-23)
  returning ``SF_TDA_down`` / ``SF_TDA_up`` (588-849 / 408-585) whose
  ``kernel(nstates)`` returns ``(e * ha2eV, v)``.
* module functions ``gen_tda_operation_sf(mf, isf, method)`` (162-244),
  ``init_guess(mf, nstates, isf)`` (348-380) and
  ``davidson_process(mf, nstates, method, isf)`` (382-406, PySCF
  ``lib.davidson1`` with tol 1e-7, lindep 1e-14, max_cycle 3000).

``method=0`` is the ALDA0 collinear-limit kernel (``mf.fxc_sf``), ``method=1``
the multicollinear kernel (``_gen_uhf_tda_response_sf``, SF_TDA.py:855-1047; kernel
from ``xtddft_amd.mcol.sf_mc_kernel``, response on the device's GGA / MGGA engine
with one spin-flip channel), ``method=2`` the collinear (no XC) response.
``collinear_samples`` defaults to the reference's per-path counts: 50 on the
Davidson path (SF_TDA.py:219), 30 for the explicit matrix (``get_ab_sf``,
SF_TDA.py:1051, 570, 843).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

from . import davidson as _dav
from .meanfield import MeanField
from .operator import DeviceOperator
from .parallel import require_group
from .utils import nlc_check, order_sf_down

HA2EV = 27.2113834   # SF_TDA.py:15


def mf_info(mf: MeanField):
    """(mo_energy, mo_occ, mo_coeff) per spin (SF_TDA.py:26-37)."""
    if not mf.is_rohf:
        return mf.mo_energy, mf.mo_occ, mf.mo_coeff
    occ = np.zeros((2, mf.mo_occ.size))
    occ[0][mf.mo_occ >= 1] = 1
    occ[1][mf.mo_occ >= 2] = 1
    return np.array([mf.mo_energy, mf.mo_energy]), occ, np.array([mf.mo_coeff, mf.mo_coeff])


DAVIDSON_SAMPLES = 50    # SF_TDA.py:219
EXPLICIT_SAMPLES = 30    # get_ab_sf default, SF_TDA.py:1051


def _check_method(method):
    if method not in (0, 1, 2):
        raise ValueError("method must be 0 (ALDA0), 1 (multicollinear) or 2 (collinear)")


def sf_operator(mf, kind, method, collinear_samples, device=0, shard=(0, 1), **kw):
    """The device operator of a spin-flip kind with the XC kernel of ``method``."""
    if method == 1:
        from .mcol import sf_mc_kernel
        kern = sf_mc_kernel(mf, collinear_samples, device=device)
        return DeviceOperator(mf, kind, device=device, shard=shard, sf_kernel="mc", mc_kernel=kern, **kw)
    return DeviceOperator(_collinear(mf) if method == 2 else mf, kind, device=device, shard=shard, **kw)


def _collinear(mf):
    """Collinear response (method=2): exchange only, no XC kernel (SF_TDA.py:265-266)."""
    import copy
    m = copy.copy(mf)
    m.grids = None
    m.fxc_sf = None
    m.extra = dict(mf.extra, collinear=True)
    return m


def sf_hdiag(mf, isf):
    """Orbital-energy gaps of the spin-flip space (SF_TDA.py:208-217)."""
    mo_energy, mo_occ, _ = mf_info(mf)
    occa = np.where(mo_occ[0] == 1)[0]; occb = np.where(mo_occ[1] == 1)[0]
    vira = np.where(mo_occ[0] == 0)[0]; virb = np.where(mo_occ[1] == 0)[0]
    if isf == -1:
        return (mo_energy[1][virb, None] - mo_energy[0][occa]).T.ravel()
    if isf == 1:
        return (mo_energy[0][vira, None] - mo_energy[1][occb]).T.ravel()
    raise ValueError("isf must be -1 (down) or +1 (up)")


def gen_tda_operation_sf(mf, isf, method=0, device=0, shard=(0, 1), collinear_samples=DAVIDSON_SAMPLES):
    _check_method(method)
    hdiag = sf_hdiag(mf, isf)
    kind = 'SF_DOWN' if isf == -1 else 'SF_UP'
    op = sf_operator(mf, kind, method, collinear_samples, device=device, shard=shard)

    def vind(zs0):
        if isinstance(zs0, (list, tuple)):
            zs0 = np.asarray(zs0)
        return op.apply_full(zs0)
    vind.operator = op
    return vind, hdiag


def init_guess(mf, nstates, isf=-1):
    mo_energy, mo_occ, _ = mf_info(mf)
    occa = mo_occ[0] > 0; occb = mo_occ[1] > 0
    vira = mo_occ[0] == 0; virb = mo_occ[1] == 0
    if isf == 1:
        e = (mo_energy[0][vira, None] - mo_energy[1][occb]).T.ravel()
    else:
        e = (mo_energy[1][virb, None] - mo_energy[0][occa]).T.ravel()
    nstates = min(nstates, e.size)
    thr = np.sort(e)[nstates - 1] + 1e-5
    idx = np.where(e <= thr)[0]
    x0 = np.zeros((idx.size, e.size))
    x0[np.arange(idx.size), idx] = 1
    return x0


def _sf_shape(mf):
    info = mf.shape_info()
    return info['nc'], info['no'], info['nv']


def deal_v_davidson(mf, v):
    """Spin-flip-down eigenvectors (columns, PySCF occ_a x vir_b order) -> the
    reference's cv|co|ov|oo block order (SF_TDA.py:304-345)."""
    return np.asarray(v)[order_sf_down(*_sf_shape(mf))]


def davidson_process(mf, nstates, method, isf=-1, device=0, shard=(0, 1), return_operator=False,
                     collinear_samples=DAVIDSON_SAMPLES):
    vind, hdiag = gen_tda_operation_sf(mf, isf, method, device=device, shard=shard,
                                       collinear_samples=collinear_samples)
    x0 = init_guess(mf, nstates, isf)
    conv, e, x1, icyc = _dav.davidson1(vind, x0, hdiag, tol=1e-7, lindep=1e-14, nroots=nstates,
                                       max_cycle=3000, device=device,
                                       lockstep=shard[1] > 1)
    v = np.array(x1).T
    if isf == -1:   # SF_TDA.py:400-401
        v = deal_v_davidson(mf, v)
    if return_operator:
        return e, v, conv, vind.operator
    return e, v, conv


def _dense(op):
    dim = op.dim
    A = np.empty((dim, dim))
    for j0 in range(0, dim, 256):
        j1 = min(dim, j0 + 256)
        eye = np.zeros((j1 - j0, dim))
        eye[np.arange(j1 - j0), np.arange(j0, j1)] = 1.0
        A[:, j0:j1] = op.apply_full(eye).T
    return A


class _SFBase:
    isf = 0

    def __init__(self, mf, method=0, davidson=True, device=0, shard=(0, 1), collinear_samples=None):
        _check_method(method)
        self.mf = mf
        self.method = method
        self.collinear_samples = collinear_samples
        self.davidson = davidson
        self.device = device
        self.shard = tuple(shard)
        require_group(self.shard[1])
        nlc_check(mf)
        self.nc, self.no, self.nv = _sf_shape(mf)

    def get_Amat(self):
        """Explicit A through the device operator; SF-down in the reference's
        cv|co|ov|oo block order (SF_TDA_down.get_Amat, SF_TDA.py:746-801)."""
        vind, _ = gen_tda_operation_sf(self.mf, self.isf, self.method, device=self.device,
                                       shard=self.shard,
                                       collinear_samples=self.collinear_samples or EXPLICIT_SAMPLES)
        A = _dense(vind.operator)
        if self.isf == -1:
            order = order_sf_down(self.nc, self.no, self.nv)
            A = A[order][:, order]
        return A

    def kernel(self, nstates=1):
        self.nstates = nstates
        if self.davidson:
            self.e, self.v, self.converged, self._op = davidson_process(
                self.mf, nstates, self.method, self.isf, self.device, self.shard, return_operator=True,
                collinear_samples=self.collinear_samples or DAVIDSON_SAMPLES)
        else:
            self.A = self.get_Amat()
            self.e, self.v = scipy.linalg.eigh(self.A)
        return self.e[:nstates] * HA2EV, self.v[:, :nstates]


class SF_TDA_up(_SFBase):
    isf = 1


class SF_TDA_down(_SFBase):
    isf = -1

    def analyse(self, threshold=0.1, verbose=True):
        """Delta<S^2> per root and dominant amplitudes from the cv|co|ov|oo
        blocks (SF_TDA_down.analyse, SF_TDA.py:806-836; the <S^2> expression
        holds for a ROKS reference)."""
        nc, no, nv = self.nc, self.no, self.nv
        d1, d2, d3 = nc * nv, nc * nv + nc * no, nc * nv + nc * no + no * nv
        Ds, lines = [], []
        for n in range(self.nstates):
            value = np.asarray(self.v)[:, n]
            cv = value[:d1].reshape(nc, nv)
            co = value[d1:d2].reshape(nc, no)
            ov = value[d2:d3].reshape(no, nv)
            oo = value[d3:].reshape(no, no)
            dp = (cv * cv).sum() - (oo * oo).sum() + np.trace(oo) ** 2
            Ds.append(-no + 1 + dp)
            lines.append(f'Excited state {n + 1} {self.e[n] * HA2EV:10.5f} eV D<S^2>={-no + 1 + dp:5.2f}')
            for tag, blk, (o0, v0) in (('CV', cv, (0, nc + no)), ('CO', co, (0, nc)),
                                       ('OV', ov, (nc, nc + no)), ('OO', oo, (nc, nc))):
                for o, v in zip(*np.where(abs(blk) > threshold)):
                    lines.append(f'{100 * blk[o, v] ** 2:3.0f}% {tag}(ab) {o + 1 + o0}a -> '
                                 f'{v + 1 + v0}b {blk[o, v]:10.5f}')
        if verbose:
            print("\n".join(lines))
        return Ds, lines


def SF_TDA(mf, isf=-1, davidson=True, method=0, device=0, shard=(0, 1), collinear_samples=None):
    if isf == -1:
        return SF_TDA_down(mf, method, davidson, device, shard, collinear_samples)
    if isf == 1:
        return SF_TDA_up(mf, method, davidson, device, shard, collinear_samples)
    raise ValueError("isf must be -1 or 1")
