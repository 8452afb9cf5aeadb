"""Block Davidson with the trial subspace resident in HBM.

Same algorithm and control flow as the reference solver
``xtddft/utils/Davidson.py:davidson1`` (Davidson.py:21-298, itself PySCF's
``lib.davidson1`` plus a CuPy ``.get()`` and a ``tol_residual`` argument) and
returning the 4-tuple ``(conv, e, x, icyc)`` its callers unpack
(XTDA.py:775).  Differences are only where the data lives:

* ``xs`` / ``ax`` (the subspace and its images) are device matrices; every
  O(space x dim) operation -- the heff rows (``_fill_heff_hermitian``), the
  Ritz vectors (``_gen_x0``), residuals, projections -- is an FP64-MFMA GEMM
  through ``xt_dgemm``; preconditioning and norms are device kernels.
* ``_qr`` orthonormalises a block with two host round trips: Gram-Schmidt
  on the host in the coefficient space of the Gram matrix (same order and
  drop rule ``norm**2 > lindep`` as the reference's vector-by-vector
  modified Gram-Schmidt), then one Cholesky-QR pass on the device; nearly
  dependent blocks fall back to the vector-by-vector form on the device;
  ``_normalize_xt_`` projects out the subspace with two passes of classical
  Gram-Schmidt as GEMMs (CGS2).  Equal in exact arithmetic to the
  reference's orthogonalisation, orthogonal to round-off.
* only the small ``heff`` (<= (max_space+nroots)^2) crosses to the host for
  ``scipy.linalg.eigh`` (Davidson.py:199), as in the reference.

``aop`` receives and returns device tensors of shape (n, dim).  For the replicated
solver of a sharded operator (``lockstep=True``, which the drivers pass when their
shard spans more than one rank) every iteration's decisions are gathered and compared
across the ranks of ``group`` (``parallel.lockstep_check``): a divergence raises on all
ranks instead of leaving some waiting in the next all-reduce.  An unsharded solve
never communicates, whatever process group exists.

Host cost per iteration (the part that does not shrink with more GPUs): three device ->
host round trips (heff rows, residual norms, the Gram matrix of the new block -- its
diagonal is the drop test of ``_normalize_xt_`` and it seeds the next ``_qr``; a fourth,
the Cholesky-QR pass, only for nearly dependent blocks), and the small host LAPACK (heff
``eigh`` by divide and conquer, the coefficient-space Gram-Schmidt) on one BLAS thread: a
multithreaded BLAS is slower on matrices of this size (measured: eigh of 70 x 70 at 0.6 ms
on one thread, up to 8 ms on eight).  ``stats`` returns the per-phase split.  ``precond``
may be a diagonal (array or device tensor: PySCF ``make_diag_precond`` with
level shift 1e-3), a ``DiagPrecond`` (device kernel), or any host callable
``precond(dx, e, x0)`` (evaluated on host copies).
"""
from __future__ import annotations

import ctypes
import logging

import numpy as np
import scipy.linalg

from . import _capi

log = logging.getLogger("xtddft_amd.davidson")


class LinearDependenceError(RuntimeError):
    pass


def _torch():
    import torch
    return torch


_BLAS_CTL = None


def _one_blas_thread():
    """Context limiting the host BLAS to one thread (cached controller: ~15 us per use)."""
    global _BLAS_CTL
    if _BLAS_CTL is None:
        from threadpoolctl import ThreadpoolController
        _BLAS_CTL = ThreadpoolController()
    return _BLAS_CTL.limit(limits=1, user_api="blas")


class DiagPrecond:
    """x / clamp(diag - (e - level_shift)) on device (XTDA.py:736-744 with
    ``level_shift = mf.level_shift``; PySCF make_diag_precond uses 1e-3)."""

    def __init__(self, diag, level_shift=1e-3, device=0):
        torch = _torch()
        self.diag_host = np.asarray(diag.cpu().numpy() if hasattr(diag, "cpu") else diag, dtype=np.float64)
        self.diag = torch.as_tensor(self.diag_host, device=f"cuda:{device}")
        self.level_shift = float(level_shift)

    def __call__(self, x, e, *args):
        """Host-compatible form (numpy in, numpy out)."""
        if isinstance(e, np.ndarray):
            e = e[0]
        d = self.diag_host - (e - self.level_shift)
        d[abs(d) < 1e-8] = 1e-8
        return x / d

    def apply_device(self, r, e0, stream):
        torch = _torch()
        out = torch.empty_like(r)
        e = torch.full((r.shape[0],), float(e0), dtype=torch.float64, device=r.device)
        _capi.check(_capi.lib().xt_precond(r.shape[0], r.shape[1], self.diag.data_ptr(), e.data_ptr(),
                                           self.level_shift, r.data_ptr(), out.data_ptr(),
                                           ctypes.c_void_p(stream)), "xt_precond")
        return out


class _Dev:
    """Thin GEMM / vector-op helpers on one stream."""

    def __init__(self, device):
        torch = _torch()
        self.torch = torch
        self.device = torch.device(f"cuda:{device}")
        self.stream = torch.cuda.current_stream(self.device).cuda_stream
        self.L = _capi.lib()

    def gemm(self, ta, tb, m, n, k, alpha, a, lda, b, ldb, beta, c, ldc):
        if m == 0 or n == 0:
            return
        with self.torch.cuda.device(self.device):   # xt_dgemm keys its workspace by the current device
            _capi.check(self.L.xt_dgemm(ta, tb, m, n, k, alpha, a.data_ptr(), lda, b.data_ptr(), ldb,
                                        beta, c.data_ptr(), ldc, ctypes.c_void_p(self.stream)), "xt_dgemm")

    def norms2(self, x):
        out = self.torch.empty(x.shape[0], dtype=self.torch.float64, device=self.device)
        if x.shape[0]:
            _capi.check(self.L.xt_row_norms2(x.shape[0], x.shape[1], x.data_ptr(), out.data_ptr(),
                                             ctypes.c_void_p(self.stream)), "xt_row_norms2")
        return out

    def scale_rows(self, x, s):
        s = self.torch.as_tensor(np.asarray(s, dtype=np.float64), device=self.device)
        if x.shape[0]:
            _capi.check(self.L.xt_row_scale(x.shape[0], x.shape[1], x.data_ptr(), s.data_ptr(),
                                            ctypes.c_void_p(self.stream)), "xt_row_scale")

    def project_out(self, xt, xs, space):
        """xt -= (xt xs^T) xs, twice (CGS2)."""
        if space == 0 or xt.shape[0] == 0:
            return
        n, dim = xt.shape
        coef = self.torch.empty((n, space), dtype=self.torch.float64, device=self.device)
        for _ in range(2):
            self.gemm(0, 1, n, space, dim, 1.0, xt, dim, xs, dim, 0.0, coef, space)
            self.gemm(0, 0, n, dim, space, -1.0, coef, space, xs, dim, 1.0, xt, dim)


def _gram_gs(g, lindep):
    """Gram-Schmidt in coefficient space: rows of C (kept x n) with C x
    orthonormal, processing the rows of x in order and dropping a row whose
    residual norm**2 <= lindep (PySCF _qr's rule) -- from the Gram matrix
    g = x x^T alone.  Returns (C, smallest kept norm**2, smallest kept norm**2 relative to
    the row's own norm**2)."""
    n = g.shape[0]
    c = np.zeros((n, n))
    kept = 0
    nmin = rmin = np.inf
    for i in range(n):
        r = np.zeros(n)
        r[i] = 1.0
        if kept:
            prod = c[:kept] @ g[:, i]
            r -= prod @ c[:kept]
        nrm2 = float(r @ g @ r)
        if nrm2 > lindep:
            c[kept] = r / np.sqrt(nrm2)
            kept += 1
            nmin = min(nmin, nrm2)
            rmin = min(rmin, nrm2 / g[i, i])
    return c[:kept], nmin, rmin


# Below this residual norm**2 the Gram-matrix route loses the accuracy the drop rule
# needs (its rounding grows like eps / norm**2): orthonormalise vector by vector instead.
GRAM_SAFE_NORM2 = 1e-8
# Above this smallest kept residual norm**2 (relative to the row's norm**2) one Gram-Schmidt
# pass is orthogonal to ~eps / ratio <= 1e-14 (the reference's one-pass modified Gram-Schmidt is no better): the
# Cholesky-QR second pass and its host round trip are skipped.
QR_ONE_PASS_NORM2 = 1e-2


def _qr_vectorwise(dev, x, lindep):
    """PySCF _qr row by row on the device: each row has the kept rows projected out
    (two classical Gram-Schmidt passes), is dropped when its residual norm**2 <=
    lindep and normalised otherwise.  One host round trip per row."""
    torch = dev.torch
    n, dim = x.shape
    out = torch.empty_like(x)
    kept = 0
    for i in range(n):
        v = x[i:i + 1].clone()
        dev.project_out(v, out[:kept], kept)
        nrm2 = float(dev.norms2(v)[0])
        if nrm2 > lindep:
            out[kept] = v[0] / np.sqrt(nrm2)
            kept += 1
    return out[:kept]


def _qr(dev, x, lindep, gram=None):
    """Orthonormalise the rows of x in order, dropping dependent ones (PySCF
    _qr, Davidson.py:152,172).  Block form with two host round trips instead
    of one per vector: the Gram matrix x x^T (device GEMM) drives Gram-Schmidt
    on the host in coefficient space (same order, same drop rule), Q1 = C x on
    the device, then one Cholesky-QR pass Q = L^-1 Q1 (L L^T = Q1 Q1^T)
    restores orthogonality to round-off (CholQR2 pattern).  Nearly dependent
    rows (a kept residual norm**2 below GRAM_SAFE_NORM2) or a failed Cholesky take
    the vector-by-vector path (``_qr_vectorwise``).  ``gram``: x x^T when the caller
    already holds it on the host (saves one round trip)."""
    torch = dev.torch
    n, dim = x.shape
    if n == 0:
        return x
    x = x.contiguous()
    if gram is None:
        g = torch.empty((n, n), dtype=torch.float64, device=dev.device)
        dev.gemm(0, 1, n, n, dim, 1.0, x, dim, x, dim, 0.0, g, n)
        gram = g.cpu().numpy()
    with _one_blas_thread():
        c, nmin, rmin = _gram_gs(gram, lindep)
    k = c.shape[0]
    if k == 0:
        return x[:0]
    if nmin < GRAM_SAFE_NORM2:
        return _qr_vectorwise(dev, x, lindep)
    ct = torch.as_tensor(np.ascontiguousarray(c), device=dev.device)
    q = torch.empty((k, dim), dtype=torch.float64, device=dev.device)
    dev.gemm(0, 0, k, dim, n, 1.0, ct, n, x, dim, 0.0, q, dim)
    if rmin > QR_ONE_PASS_NORM2:
        return q
    g2 = torch.empty((k, k), dtype=torch.float64, device=dev.device)
    dev.gemm(0, 1, k, k, dim, 1.0, q, dim, q, dim, 0.0, g2, k)
    g2h = g2.cpu().numpy()
    try:
        with _one_blas_thread():
            low = np.linalg.cholesky(0.5 * (g2h + g2h.T))
            linv = scipy.linalg.solve_triangular(low, np.eye(k), lower=True)
    except np.linalg.LinAlgError:
        return _qr_vectorwise(dev, x, lindep)
    lt = torch.as_tensor(np.ascontiguousarray(linv), device=dev.device)
    out = torch.empty_like(q)
    dev.gemm(0, 0, k, dim, k, 1.0, lt, k, q, dim, 0.0, out, dim)
    return out


def _sort_elast(elast, conv_last, vlast, v):
    head, nroots = vlast.shape
    ovlp = abs(np.dot(v[:head].T, vlast))
    mapidx = np.argmax(ovlp, axis=1)
    return elast[mapidx], conv_last[mapidx]


def checkpoint(path: str, every: int = 1):
    """A ``davidson1`` callback that saves the current Ritz vectors, Ritz values, the
    convergence flags and the iteration to ``path`` (NumPy ``.npz``, written to a temporary
    file and renamed, so an interrupted write never leaves a torn file) every ``every``
    iterations.  Resume with ``x0 = restart_guess(path)[0]`` (the reference Davidson takes
    any x0, Davidson.py:21-298; SURVEY.md section 5 "checkpoint / resume")."""
    import os

    def cb(envs):
        icyc = int(envs["icyc"])
        if icyc % max(1, int(every)):
            return
        tmp = path + ".tmp"
        with open(tmp, "wb") as fh:
            np.savez(fh, x=envs["x0r"].cpu().numpy(), e=np.asarray(envs["e"]),
                     conv=np.asarray(envs["conv"]), icyc=icyc)
        os.replace(tmp, path)
    return cb


def restart_guess(path: str):
    """(x0, e, icyc) from a ``checkpoint`` file (x0: Ritz vectors as rows)."""
    with np.load(path) as f:
        return f["x"], f["e"], int(f["icyc"])


def davidson1(aop, x0, precond, tol=1e-12, max_cycle=50, max_space=12, lindep=1e-14,
              max_memory=4000, dot=None, callback=None, nroots=1, lessio=False, pick=None,
              verbose=None, follow_state=False, tol_residual=None, fill_heff=None, device=0,
              return_device=False, lockstep=False, group=None, stats=None):
    """lockstep: compare every iteration's decisions across the ranks of ``group`` (the
    replicated solver of a sharded operator); off for an unsharded solve.
    stats: a dict that receives the wall seconds per solver phase (qr, aop, heff, eigh,
    ritz, lockstep, precond, other) -- the phases end at host round trips, so no
    synchronisation is added."""
    import time
    from .parallel import lockstep_check
    torch = _torch()
    t_last = [time.perf_counter()]

    def tick(name):
        if stats is not None:
            t = time.perf_counter()
            stats[name] = stats.get(name, 0.0) + t - t_last[0]
            t_last[0] = t
    if not torch.cuda.is_available():
        raise RuntimeError("xtddft_amd.davidson1 runs on the GPU; no device is visible")
    dev = _Dev(device)
    toloose = np.sqrt(tol) if tol_residual is None else tol_residual
    if callable(x0):
        x0 = x0()
    if not (hasattr(x0, "is_cuda") and x0.is_cuda):
        x0 = np.asarray(x0, dtype=np.float64)
        if x0.ndim == 1:
            x0 = x0[None]
        x0 = torch.as_tensor(x0, device=dev.device)
    x0 = x0.to(torch.float64)
    if x0.dim() == 1:
        x0 = x0[None]
    dim = x0.shape[1]
    if isinstance(precond, DiagPrecond):
        pre = precond
    elif callable(precond):
        pre = None
    else:
        pre = DiagPrecond(precond, 1e-3, device)

    max_space = max_space + (nroots - 1) * 4
    cap = max_space + nroots + 40
    xs = torch.empty((cap, dim), dtype=torch.float64, device=dev.device)
    ax = torch.empty_like(xs)
    heff = np.empty((max_space + nroots + 40, max_space + nroots + 40))
    fresh_start = True
    e = v = None
    conv = np.zeros(nroots, dtype=bool)
    space = 0
    xt = None
    xt_gram = None          # host Gram matrix of xt, from _normalize_xt_'s round trip
    icyc = 0
    x0r = None
    max_dx_last = 1e9
    for icyc in range(max_cycle):
        if fresh_start:
            space = 0
            xt = _qr(dev, x0, lindep)
            if xt.shape[0] == 0:
                raise LinearDependenceError('Initial guess is empty or zero' if icyc == 0 else
                                            'No more linearly independent basis were found.')
            x0 = None
            max_dx_last = 1e9            # Davidson.py:168
        elif xt.shape[0] > 1:
            xt = _qr(dev, xt, lindep, gram=xt_gram)[:40]
        tick("qr")
        axt = aop(xt)
        if not (hasattr(axt, "is_cuda") and axt.is_cuda):
            axt = torch.as_tensor(np.asarray(axt, dtype=np.float64), device=dev.device)
        tick("aop")
        nnew = xt.shape[0]
        if space + nnew > cap:
            raise RuntimeError("Davidson subspace overflow")
        row0, space = space, space + nnew
        xs[row0:space] = xt
        ax[row0:space] = axt
        elast, vlast, conv_last = e, v, conv
        # _fill_heff_hermitian: heff[i, j] = xt_i . ax_j for new i, j <= i (Davidson.py:197)
        h = torch.empty((nnew, space), dtype=torch.float64, device=dev.device)
        dev.gemm(0, 1, nnew, space, dim, 1.0, xs[row0:space], dim, ax, dim, 0.0, h, space)
        hh = h.cpu().numpy()
        for ip in range(nnew):
            i = row0 + ip
            heff[i, :i + 1] = hh[ip, :i + 1]
            heff[:i + 1, i] = hh[ip, :i + 1]
        xt = axt = None
        tick("heff")
        with _one_blas_thread():     # divide and conquer: the fastest LAPACK driver at these sizes
            w, vv = scipy.linalg.eigh(heff[:space, :space], driver="evd")
        tick("eigh")
        if callable(pick):
            w, vv, idx = pick(w, vv, nroots, locals())
            if len(w) == 0:
                raise RuntimeError(f'Not enough eigenvalues found by {pick}')
        e = w[:nroots]
        v = vv[:, :nroots]
        conv = np.zeros(e.size, dtype=bool)
        if not fresh_start:
            elast, conv_last = _sort_elast(elast, conv_last, vlast, v)
        de = e if (elast is None or elast.size != e.size) else e - elast
        nr = e.size
        # v^T and -(v e)^T in one upload
        vv2 = torch.as_tensor(np.ascontiguousarray(np.concatenate([v.T, -(v * e).T])), device=dev.device)
        vt, vte = vv2[:nr], vv2[nr:]                                                # (nr, space) each
        x0r = torch.empty((nr, dim), dtype=torch.float64, device=dev.device)
        dev.gemm(0, 0, nr, dim, space, 1.0, vt, space, xs, dim, 0.0, x0r, dim)     # x0 = v^T xs
        # ax0 = v^T ax.  (lessio recomputes A x0 only when the subspace is not held
        # in memory -- lessio = lessio and not _incore, Davidson.py:128; here it
        # always is, in HBM, so lessio has no effect, as in the reference.)
        r = torch.empty_like(x0r)
        dev.gemm(0, 0, nr, dim, space, 1.0, vt, space, ax, dim, 0.0, r, dim)
        dev.gemm(0, 0, nr, dim, space, 1.0, vte, space, xs, dim, 1.0, r, dim)      # r = ax0 - e x0
        dx_norm = np.sqrt(dev.norms2(r).cpu().numpy())
        for k in range(nr):
            conv[k] = abs(de[k]) < tol and dx_norm[k] < toloose
        tick("ritz")
        if lockstep:   # every break / restart decision below follows from these
            lockstep_check(np.concatenate([[icyc, space, nnew, float(np.sum(heff[:space, :space]))],
                                           e, dx_norm, conv]), f"iteration {icyc}", group)
        tick("lockstep")
        log.debug("davidson %d %d |r|=%.3g e=%s max|de|=%.3g", icyc, space, dx_norm.max(), e,
                  np.abs(de).max())
        if all(conv):
            break
        max_dx = float(dx_norm.max())
        if (follow_state and max_dx > 1 and max_dx / max_dx_last > 3 and space > nroots + 2):
            # large |r|: restart from the previous Ritz vectors (Davidson.py:246-253)
            log.debug("davidson %d: large |r| %.3g, restoring the previous x0", icyc, max_dx)
            k = vlast.shape[0]
            vl = torch.as_tensor(np.ascontiguousarray(vlast.T), device=dev.device)
            x0 = torch.empty((vlast.shape[1], dim), dtype=torch.float64, device=dev.device)
            dev.gemm(0, 0, vlast.shape[1], dim, k, 1.0, vl, k, xs, dim, 0.0, x0, dim)
            fresh_start = True
            continue
        keep = [k for k in range(nr) if (not conv[k]) and dx_norm[k] ** 2 > lindep]
        if keep:
            rk = r[keep].contiguous()
            if pre is not None:
                rk = pre.apply_device(rk, e[0], dev.stream)
            else:
                host = rk.cpu().numpy()
                x0h = x0r[keep].cpu().numpy()
                host = np.asarray([precond(host[j], e[0], x0h[j]) for j in range(len(keep))])
                rk = torch.as_tensor(host, device=dev.device)
            rk = rk * torch.rsqrt(dev.norms2(rk))[:, None]          # normalise on the device
            # _normalize_xt_: project out xs, drop if norm**2 <= lindep, normalise; the Gram
            # matrix of the block gives the norms and seeds the next _qr in one round trip
            dev.project_out(rk, xs[:space], space)
            nk = rk.shape[0]
            g = torch.empty((nk, nk), dtype=torch.float64, device=dev.device)
            dev.gemm(0, 1, nk, nk, dim, 1.0, rk, dim, rk, dim, 0.0, g, nk)
            gh = g.cpu().numpy()
            nrm2 = np.diag(gh).copy()
            ok = np.where(nrm2 > lindep)[0]
            sc = 1.0 / np.sqrt(nrm2[ok])
            if ok.size == nk:        # nothing dropped: scale by the device copy of the diagonal
                rk = rk * torch.rsqrt(torch.diagonal(g))[:, None]
            else:
                rk = rk[torch.as_tensor(ok, device=dev.device)].contiguous()
                dev.scale_rows(rk, sc)
            xt_gram = gh[np.ix_(ok, ok)] * sc[:, None] * sc[None, :]
            xt = rk
        else:
            xt = torch.empty((0, dim), dtype=torch.float64, device=dev.device)
        tick("precond")
        if lockstep:
            lockstep_check([icyc, xt.shape[0]], f"iteration {icyc} new vectors", group)
        if xt.shape[0] == 0:
            conv = dx_norm < toloose
            break
        max_dx_last = max_dx
        fresh_start = space + nroots > max_space
        if fresh_start:
            x0 = x0r
        if callable(callback):
            callback(locals())
        tick("other")
    if return_device:
        return np.asarray(conv), e, x0r, icyc
    x_host = x0r.cpu().numpy()
    return np.asarray(conv), e, [x_host[k] for k in range(x_host.shape[0])], icyc
