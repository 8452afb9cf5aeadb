"""Spin-flip TDA with the reference's API (``xtddft/SF_TDA.py``).

* ``SF_TDA(mf, isf=-1, davidson=True, method=0)`` factory (SF_TDA.py:17-23)
  returning ``SF_TDA_down`` / ``SF_TDA_up`` (588-849 / 408-585) whose
  ``kernel(nstates)`` returns ``(e * ha2eV, v)``.
* module functions ``gen_tda_operation_sf(mf, isf, method)`` (162-244),
  ``init_guess(mf, nstates, isf)`` (348-380) and
  ``davidson_process(mf, nstates, method, isf)`` (382-406, PySCF
  ``lib.davidson1`` with tol 1e-7, lindep 1e-14, max_cycle 3000).

``method=0`` is the ALDA0 collinear-limit kernel (``mf.fxc_sf``), ``method=2``
the collinear (no XC) response; ``method=1`` (multicollinear, needs mcfun)
is outside the hot-path scope and raises.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

from . import davidson as _dav
from .meanfield import MeanField
from .operator import DeviceOperator

HA2EV = 27.2113834   # SF_TDA.py:15


def mf_info(mf: MeanField):
    """(mo_energy, mo_occ, mo_coeff) per spin (SF_TDA.py:26-37)."""
    if not mf.is_rohf:
        return mf.mo_energy, mf.mo_occ, mf.mo_coeff
    occ = np.zeros((2, mf.mo_occ.size))
    occ[0][mf.mo_occ >= 1] = 1
    occ[1][mf.mo_occ >= 2] = 1
    return np.array([mf.mo_energy, mf.mo_energy]), occ, np.array([mf.mo_coeff, mf.mo_coeff])


def _check_method(method):
    if method == 1:
        raise NotImplementedError("multicollinear kernel (method=1) needs mcfun; outside hot-path scope")
    if method not in (0, 2):
        raise ValueError("method must be 0 (ALDA0), 1 (multicollinear) or 2 (collinear)")


def _collinear(mf):
    """Collinear response (method=2): exchange only, no XC kernel (SF_TDA.py:265-266)."""
    import copy
    m = copy.copy(mf)
    m.grids = None
    m.fxc_sf = None
    m.extra = dict(mf.extra, collinear=True)
    return m


def gen_tda_operation_sf(mf, isf, method=0, device=0, shard=(0, 1)):
    _check_method(method)
    mo_energy, mo_occ, _ = mf_info(mf)
    occa = np.where(mo_occ[0] == 1)[0]; occb = np.where(mo_occ[1] == 1)[0]
    vira = np.where(mo_occ[0] == 0)[0]; virb = np.where(mo_occ[1] == 0)[0]
    if isf == -1:
        hdiag = (mo_energy[1][virb, None] - mo_energy[0][occa]).T.ravel()
        kind = 'SF_DOWN'
    elif isf == 1:
        hdiag = (mo_energy[0][vira, None] - mo_energy[1][occb]).T.ravel()
        kind = 'SF_UP'
    else:
        raise ValueError("isf must be -1 (down) or +1 (up)")
    op = DeviceOperator(_collinear(mf) if method == 2 else mf, kind, device=device, shard=shard)

    def vind(zs0):
        if isinstance(zs0, (list, tuple)):
            zs0 = np.asarray(zs0)
        return op.apply(zs0)
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


def davidson_process(mf, nstates, method, isf=-1, device=0):
    vind, hdiag = gen_tda_operation_sf(mf, isf, method, device=device)
    x0 = init_guess(mf, nstates, isf)
    conv, e, x1, icyc = _dav.davidson1(vind, x0, hdiag, tol=1e-7, lindep=1e-14, nroots=nstates,
                                       max_cycle=3000, device=device)
    v = np.array(x1).T
    return e, v, conv


def _dense(op):
    dim = op.dim
    A = np.empty((dim, dim))
    for j0 in range(0, dim, 256):
        j1 = min(dim, j0 + 256)
        eye = np.zeros((j1 - j0, dim))
        eye[np.arange(j1 - j0), np.arange(j0, j1)] = 1.0
        A[:, j0:j1] = op.apply(eye).T
    return A


class _SFBase:
    isf = 0

    def __init__(self, mf, method=0, davidson=True, device=0):
        _check_method(method)
        self.mf = mf
        self.method = method
        self.davidson = davidson
        self.device = device
        info = mf.shape_info()
        self.nc, self.no, self.nv = info['nc'], info['no'], info['nv']

    def kernel(self, nstates=1):
        self.nstates = nstates
        if self.davidson:
            self.e, self.v, self.converged = davidson_process(self.mf, nstates, self.method,
                                                              self.isf, self.device)
        else:
            vind, _ = gen_tda_operation_sf(self.mf, self.isf, self.method, device=self.device)
            self.A = _dense(vind.operator)
            self.e, self.v = scipy.linalg.eigh(self.A)
        return self.e[:nstates] * HA2EV, self.v[:, :nstates]


class SF_TDA_up(_SFBase):
    isf = 1


class SF_TDA_down(_SFBase):
    isf = -1


def SF_TDA(mf, isf=-1, davidson=True, method=0, device=0):
    if isf == -1:
        return SF_TDA_down(mf, method, davidson, device)
    if isf == 1:
        return SF_TDA_up(mf, method, davidson, device)
    raise ValueError("isf must be -1 or 1")
