"""Davidson oracle.  TEST INFRASTRUCTURE ONLY.

Restates ``xtddft/utils/Davidson.py:davidson1`` (Davidson.py:21-298) with the
PySCF ``lib.linalg_helper`` helpers it imports (Davidson.py:7-9):
``_qr`` (modified Gram-Schmidt, drop below lindep), ``_fill_heff_hermitian``,
``_outprod_to_subspace`` (= ``_gen_x0``), ``_sort_elast``,
``_normalize_xt_`` (project out xs, drop below lindep) and
``make_diag_precond`` (level shift 1e-3, clamp |d| < 1e-8).
The CuPy ``.get()`` calls (Davidson.py:104-105,175) are dropped and the
intended 4-tuple ``(conv, e, x, icyc)`` of the callers (XTDA.py:775) is
returned.  ``lib.davidson1`` as used by SF/XSF (SF_TDA.py:392,
XSF_TDA.py:1467) is the same algorithm returning the first three.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg


class LinearDependenceError(RuntimeError):
    pass


def make_diag_precond(diag, level_shift=1e-3):
    def precond(dx, e, *args):
        diagd = diag - (e - level_shift)
        diagd[abs(diagd) < 1e-8] = 1e-8
        return dx / diagd
    return precond


def _qr(xs, lindep=1e-14):
    nvec = len(xs)
    qs = np.empty((nvec, xs[0].size))
    nv = 0
    for i in range(nvec):
        xi = np.array(xs[i], copy=True)
        for j in range(nv):
            xi -= qs[j] * np.dot(qs[j], xi)
        innerprod = np.dot(xi, xi)
        if innerprod > lindep:
            qs[nv] = xi / np.sqrt(innerprod)
            nv += 1
    return qs[:nv]


def _fill_heff_hermitian(heff, xs, ax, xt, axt):
    nrow = len(axt)
    row1 = len(ax)
    row0 = row1 - nrow
    for ip, i in enumerate(range(row0, row1)):
        for jp, j in enumerate(range(row0, i)):
            heff[i, j] = np.dot(xt[ip], axt[jp])
            heff[j, i] = heff[i, j]
        heff[i, i] = np.dot(xt[ip], axt[ip])
    for i in range(row0):
        axi = np.asarray(ax[i])
        for jp, j in enumerate(range(row0, row1)):
            heff[j, i] = np.dot(xt[jp], axi)
            heff[i, j] = heff[j, i]
    return heff


def _gen_x0(v, xs):
    return np.dot(np.asarray(v).T, np.asarray(xs))


def _sort_elast(elast, conv_last, vlast, v):
    head, nroots = vlast.shape
    ovlp = abs(np.dot(v[:head].T, vlast))
    mapidx = np.argmax(ovlp, axis=1)
    return elast[mapidx], conv_last[mapidx]


def _normalize_xt_(xt, xs, threshold):
    norm_min = 1
    out = []
    for xi in xt:
        if xi is None:
            continue
        for xsi in xs:
            xi -= xsi * np.dot(xsi, xi)
        norm = np.sqrt(np.dot(xi, xi))
        if norm ** 2 > threshold:
            xi *= 1 / norm
            out.append(xi)
            norm_min = min(norm_min, norm)
    return out, norm_min


def davidson1(aop, x0, precond, tol=1e-12, max_cycle=50, max_space=12,
              lindep=1e-14, nroots=1, pick=None, tol_residual=None):
    toloose = np.sqrt(tol) if tol_residual is None else tol_residual
    if not callable(precond):
        precond = make_diag_precond(precond)
    x0 = np.asarray(x0, dtype=np.float64)
    if x0.ndim == 1:
        x0 = x0[None]
    max_space = max_space + (nroots - 1) * 4
    heff = None
    fresh_start = True
    e = v = None
    conv = np.zeros(nroots, dtype=bool)
    icyc = 0
    for icyc in range(max_cycle):
        if fresh_start:
            xs, ax = [], []
            space = 0
            xt = _qr(list(x0), lindep)
            if len(xt) == 0:
                raise LinearDependenceError('Initial guess is empty or zero' if icyc == 0
                                            else 'No more linearly independent basis were found.')
            x0 = None
        elif len(xt) > 1:
            xt = _qr(xt, lindep)
            xt = xt[:40]
        axt = np.asarray(aop(np.asarray(xt)))
        for k in range(len(xt)):
            xs.append(np.asarray(xt[k]))
            ax.append(axt[k])
        space += len(xt)
        if heff is None:
            heff = np.empty((max_space + nroots, max_space + nroots))
        elast, vlast, conv_last = e, v, conv
        _fill_heff_hermitian(heff, xs, ax, xt, axt)
        xt = axt = None
        w, v = scipy.linalg.eigh(heff[:space, :space])
        if callable(pick):
            w, v, idx = pick(w, v, nroots, locals())
            if len(w) == 0:
                raise RuntimeError(f'Not enough eigenvalues found by {pick}')
        e = w[:nroots]
        v = v[:, :nroots]
        conv = np.zeros(e.size, dtype=bool)
        if not fresh_start:
            elast, conv_last = _sort_elast(elast, conv_last, vlast, v)
        if elast is None or elast.size != e.size:
            de = e
        else:
            de = e - elast
        x0 = _gen_x0(v, xs)
        ax0 = _gen_x0(v, ax)
        dx_norm = np.zeros(e.size)
        xt = [None] * nroots
        for k, ek in enumerate(e):
            xt[k] = ax0[k] - ek * x0[k]
            dx_norm[k] = np.sqrt(np.dot(xt[k], xt[k]))
            conv[k] = abs(de[k]) < tol and dx_norm[k] < toloose
        ax0 = None
        if all(conv):
            break
        for k, ek in enumerate(e):
            if (not conv[k]) and dx_norm[k] ** 2 > lindep:
                xt[k] = precond(xt[k], e[0], x0[k])
                xt[k] *= np.dot(xt[k], xt[k]) ** -.5
            else:
                xt[k] = None
        xt, norm_min = _normalize_xt_(xt, xs, lindep)
        if len(xt) == 0:
            conv = dx_norm < toloose
            break
        fresh_start = space + nroots > max_space
    return np.asarray(conv), e, list(x0), icyc
