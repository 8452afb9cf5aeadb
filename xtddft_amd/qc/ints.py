"""Gaussian integrals by the McMurchie-Davidson scheme (replaces libcint for the
hot path's inputs: ``int1e_ovlp``, ``int1e_kin``, ``int1e_nuc``, ``int1e_r``,
``int2e`` as PySCF's ``mol.intor`` returns them, XTDA.py:120,848,869).

Cartesian primitives x^i y^j z^k exp(-a r^2) are expanded in Hermite Gaussians
(E coefficients, one recursion per Cartesian direction); Coulomb-type
integrals use the Hermite integrals R_tuv built by the standard downward
recursion from Boys functions.  Everything is vectorised over primitive pairs
(bra) x primitive pairs (ket); the Python loops run over shells only.
The spherical transform and AO normalisation are applied by ``gto.Mole``.
"""
from __future__ import annotations

from functools import lru_cache

import numpy as np
from scipy.special import gamma as _gamma, gammainc as _gammainc


# --------------------------------------------------------------------------- Boys
def boys(nmax: int, t: np.ndarray) -> np.ndarray:
    """F_n(T) for n = 0..nmax (shape (nmax+1,) + T.shape), ~1e-15 relative.

    F_nmax from the positive series e^-T sum_k (2T)^k / ((2n+1)(2n+3)...(2n+2k+1))
    for T < 12 and from the incomplete gamma function above; lower orders by the
    stable downward recursion F_n = (2T F_{n+1} + e^-T) / (2n+1).
    """
    t = np.asarray(t, dtype=np.float64)
    out = np.empty((nmax + 1,) + t.shape)
    et = np.exp(-t)
    small = t < 12.0
    fn = np.empty(t.shape)
    if np.any(small):
        ts = t[small]
        term = np.full(ts.shape, 1.0 / (2 * nmax + 1))
        acc = term.copy()
        for k in range(1, 80):
            term = term * (2.0 * ts) / (2 * nmax + 2 * k + 1)
            acc += term
        fn[small] = et[small] * acc
    if np.any(~small):
        tl = t[~small]
        a = nmax + 0.5
        fn[~small] = _gamma(a) * _gammainc(a, tl) / (2.0 * tl ** a)
    out[nmax] = fn
    for n in range(nmax - 1, -1, -1):
        out[n] = (2.0 * t * out[n + 1] + et) / (2 * n + 1)
    return out


# --------------------------------------------------------------- index helpers
@lru_cache(maxsize=None)
def cart_comps(l: int):
    """Cartesian components of a shell in PySCF/libcint order (xx, xy, xz, yy, yz, zz ...)."""
    out = []
    for ix in range(l, -1, -1):
        for iy in range(l - ix, -1, -1):
            out.append((ix, iy, l - ix - iy))
    return tuple(out)


@lru_cache(maxsize=None)
def hermite_index(L: int):
    """All (t,u,v) with t+u+v <= L and a dict (t,u,v) -> position."""
    tuv = [(t, u, v) for n in range(L + 1) for t in range(n, -1, -1)
           for u in range(n - t, -1, -1) for v in [n - t - u]]
    return tuple(tuv), {k: i for i, k in enumerate(tuv)}


@lru_cache(maxsize=None)
def _sum_table(lab: int, lcd: int):
    """idx[i_ab, i_cd] of (t+tau, u+nu, v+phi) in hermite_index(lab+lcd), and (-1)^(tau+nu+phi)."""
    tab, _ = hermite_index(lab)
    tcd, _ = hermite_index(lcd)
    _, pos = hermite_index(lab + lcd)
    idx = np.empty((len(tab), len(tcd)), dtype=np.int64)
    for i, (t, u, v) in enumerate(tab):
        for j, (a, b, c) in enumerate(tcd):
            idx[i, j] = pos[(t + a, u + b, v + c)]
    sign = np.array([(-1.0) ** (a + b + c) for (a, b, c) in tcd])
    return idx, sign


# ------------------------------------------------------------ E coefficients
def hermite_e(la: int, lb: int, a: np.ndarray, b: np.ndarray, xab: float) -> np.ndarray:
    """E^{ij}_t for one Cartesian direction: shape (la+1, lb+1, la+lb+1) + a.shape.

    a, b broadcast to the primitive-pair shape; xab = A_x - B_x.
    """
    p = a + b
    xpa = -b * xab / p
    xpb = a * xab / p
    oo2p = 0.5 / p
    tmax = la + lb
    E = np.zeros((la + 1, lb + 1, tmax + 1) + p.shape)
    E[0, 0, 0] = np.exp(-(a * b / p) * xab * xab)
    for i in range(la + 1):
        for j in range(lb + 1):
            if i == 0 and j == 0:
                continue
            if i > 0:
                src, x = E[i - 1, j], xpa
                top = i - 1 + j
            else:
                src, x = E[i, j - 1], xpb
                top = i + j - 1
            for t in range(i + j + 1):
                v = x * src[t] if t <= top else 0.0
                if t > 0:
                    v = v + oo2p * src[t - 1]
                if t + 1 <= top:
                    v = v + (t + 1) * src[t + 1]
                E[i, j, t] = v
    return E


# ------------------------------------------------------------ R integrals
def hermite_r(L: int, alpha: np.ndarray, X: np.ndarray, Y: np.ndarray, Z: np.ndarray) -> np.ndarray:
    """R^0_{tuv}(alpha, X, Y, Z) for every (t,u,v) of hermite_index(L): (ntuv,) + X.shape."""
    F = boys(L, alpha * (X * X + Y * Y + Z * Z))
    m2a = -2.0 * alpha
    prev = {(0, 0, 0): m2a ** L * F[L]}
    for n in range(L - 1, -1, -1):
        cur = {(0, 0, 0): m2a ** n * F[n]}
        for tot in range(1, L - n + 1):
            for t in range(tot, -1, -1):
                for u in range(tot - t, -1, -1):
                    v = tot - t - u
                    if t > 0:
                        val = X * prev[(t - 1, u, v)]
                        if t > 1:
                            val = val + (t - 1) * prev[(t - 2, u, v)]
                    elif u > 0:
                        val = Y * prev[(0, u - 1, v)]
                        if u > 1:
                            val = val + (u - 1) * prev[(0, u - 2, v)]
                    else:
                        val = Z * prev[(0, 0, v - 1)]
                        if v > 1:
                            val = val + (v - 1) * prev[(0, 0, v - 2)]
                    cur[(t, u, v)] = val
        prev = cur
    tuv, _ = hermite_index(L)
    return np.stack([prev[k] for k in tuv])


def _attenuate(alpha, omega):
    """erf(omega r)/r instead of 1/r: the Hermite integrals of the attenuated operator
    are sqrt(a'/alpha) R_tuv(a') with 1/a' = 1/alpha + 1/omega^2 (the Fourier factor
    exp(-k^2 / 4 omega^2) folded into the Gaussian product's exponent).  Returns
    (exponent for R, prefactor scale); omega = 0 is the full Coulomb operator."""
    if not omega:
        return alpha, 1.0
    w2 = omega * omega
    a2 = alpha * w2 / (alpha + w2)
    return a2, np.sqrt(a2 / alpha)


# ------------------------------------------------------------ shell pairs, batched
class ShellPairBatch:
    """ShellPair for many pairs (sa_k, sb_k) of one class -- equal angular momenta and
    primitive counts -- with every table vectorised over the pairs (P leading axis):
    the one-electron integrals and the device pair tables of large molecules (65k pairs
    at 840 AOs) without a Python loop per pair.  Same formulas as ShellPair."""

    def __init__(self, sas, sbs, kin: bool = False, hermite: bool = True):
        la, lb = sas[0].l, sbs[0].l
        self.la, self.lb = la, lb
        a = np.stack([s.exps for s in sas])[:, :, None]           # (P, na, 1)
        b = np.stack([s.exps for s in sbs])[:, None, :]           # (P, 1, nb)
        A = np.stack([s.center for s in sas])
        B = np.stack([s.center for s in sbs])
        AB = A - B
        ext = 2 if kin else 0
        self.E = [hermite_e(la, lb + ext, a, b, AB[:, d][:, None, None]) for d in range(3)]
        p = a + b                                                 # (P, na, nb)
        self.p = p.reshape(p.shape[0], -1)
        self.bexp = np.broadcast_to(b, p.shape)
        self.P = ((a[..., None] * A[:, None, None, :] + b[..., None] * B[:, None, None, :])
                  / p[..., None]).reshape(p.shape[0], -1, 3)
        ca = np.stack([s.coefs for s in sas])
        cb = np.stack([s.coefs for s in sbs])
        self.cc = ca[:, :, None] * cb[:, None, :]                 # (P, na, nb)
        self._sq = np.sqrt(np.pi / p)
        if hermite:
            L = la + lb
            tuv, _ = hermite_index(L)
            cA, cB = cart_comps(la), cart_comps(lb)
            npair, npp = self.p.shape
            Eab = np.zeros((npair, len(cA), len(cB), len(tuv), npp))
            Ex, Ey, Ez = (e.reshape(e.shape[:4] + (-1,)) for e in self.E)
            ccf = self.cc.reshape(npair, -1)
            for i, (ax, ay, az) in enumerate(cA):
                for j, (bx, by, bz) in enumerate(cB):
                    for k, (t, u, v) in enumerate(tuv):
                        if t > ax + bx or u > ay + by or v > az + bz:
                            continue
                        Eab[:, i, j, k] = Ex[ax, bx, t] * Ey[ay, by, u] * Ez[az, bz, v] * ccf
            self.Eab = Eab

    def _s1d(self, d):
        return self.E[d][:, :, 0] * self._sq                      # (la+1, lb+ext+1, P, na, nb)

    def overlap(self):
        S = [self._s1d(d) for d in range(3)]
        cA, cB = cart_comps(self.la), cart_comps(self.lb)
        out = np.empty((self.cc.shape[0], len(cA), len(cB)))
        for i, (ax, ay, az) in enumerate(cA):
            for j, (bx, by, bz) in enumerate(cB):
                out[:, i, j] = np.sum(self.cc * S[0][ax, bx] * S[1][ay, by] * S[2][az, bz], axis=(1, 2))
        return out

    def kinetic(self):
        """Needs kin=True (E tables extended to lb + 2)."""
        S = [self._s1d(d) for d in range(3)]
        b = self.bexp

        def t1d(Sd, i, j):
            v = -2.0 * b * b * Sd[i, j + 2] + b * (2 * j + 1) * Sd[i, j]
            if j >= 2:
                v = v - 0.5 * j * (j - 1) * Sd[i, j - 2]
            return v
        cA, cB = cart_comps(self.la), cart_comps(self.lb)
        out = np.empty((self.cc.shape[0], len(cA), len(cB)))
        for i, (ax, ay, az) in enumerate(cA):
            for j, (bx, by, bz) in enumerate(cB):
                tx = t1d(S[0], ax, bx) * S[1][ay, by] * S[2][az, bz]
                ty = S[0][ax, bx] * t1d(S[1], ay, by) * S[2][az, bz]
                tz = S[0][ax, bx] * S[1][ay, by] * t1d(S[2], az, bz)
                out[:, i, j] = np.sum(self.cc * (tx + ty + tz), axis=(1, 2))
        return out


def pair_classes(shells, chunk: int = 4096):
    """Shell pairs (i, j), i >= j, grouped by class (l_i, l_j, nprim_i, nprim_j): yields
    (class pair indices into the i >= j enumeration, i array, j array) in chunks."""
    groups = {}
    k = 0
    for i, si in enumerate(shells):
        for j in range(i + 1):
            sj = shells[j]
            groups.setdefault((si.l, sj.l, si.exps.size, sj.exps.size), []).append((k, i, j))
            k += 1
    for members in groups.values():
        arr = np.asarray(members, dtype=np.int64)
        for c0 in range(0, len(arr), chunk):
            blk = arr[c0:c0 + chunk]
            yield blk[:, 0], blk[:, 1], blk[:, 2]


# ------------------------------------------------------------ shell pairs
class ShellPair:
    """Primitive-pair data of two contracted Cartesian shells (A, B).

    Eab[ca, cb, i_tuv, q]  Hermite expansion coefficients with contraction
                           coefficients folded in (q runs over na*nb pairs),
    p[q], P[q, 3]          combined exponents / centres.
    """

    def __init__(self, sa, sb, kin: bool = False, hermite: bool = True):
        self.sa, self.sb = sa, sb
        la, lb = sa.l, sb.l
        a = sa.exps[:, None]
        b = sb.exps[None, :]
        AB = sa.center - sb.center
        ext = 2 if kin else 0
        self.E = [hermite_e(la, lb + ext, a, b, AB[d]) for d in range(3)]
        p = a + b
        self.p = p.ravel()
        self.P = ((a[..., None] * sa.center + b[..., None] * sb.center) / p[..., None]).reshape(-1, 3)
        cc = (sa.coefs[:, None] * sb.coefs[None, :]).ravel()
        self.cc = cc
        L = la + lb
        self.L = L
        if not hermite:          # one-electron overlap-type integrals need only the 1D tables
            return
        tuv, _ = hermite_index(L)
        ca, cb = cart_comps(la), cart_comps(lb)
        Eab = np.zeros((len(ca), len(cb), len(tuv), self.p.size))
        Ex, Ey, Ez = (e.reshape(e.shape[:3] + (-1,)) for e in self.E)
        for i, (ax, ay, az) in enumerate(ca):
            for j, (bx, by, bz) in enumerate(cb):
                for k, (t, u, v) in enumerate(tuv):
                    if t > ax + bx or u > ay + by or v > az + bz:
                        continue
                    Eab[i, j, k] = Ex[ax, bx, t] * Ey[ay, by, u] * Ez[az, bz, v] * cc
        self.Eab = Eab

    # 1D overlap table S[i, j] over primitive pairs, with the sqrt(pi/p) factor
    def _s1d(self, d):
        e = self.E[d].reshape(self.E[d].shape[:3] + (-1,))
        return e[:, :, 0] * np.sqrt(np.pi / self.p)

    def overlap(self):
        la, lb = self.sa.l, self.sb.l
        S = [self._s1d(d) for d in range(3)]
        out = np.empty((len(cart_comps(la)), len(cart_comps(lb))))
        for i, (ax, ay, az) in enumerate(cart_comps(la)):
            for j, (bx, by, bz) in enumerate(cart_comps(lb)):
                out[i, j] = np.sum(self.cc * S[0][ax, bx] * S[1][ay, by] * S[2][az, bz])
        return out

    def kinetic(self):
        """Needs kin=True (E tables extended to lb+2)."""
        la, lb = self.sa.l, self.sb.l
        b = np.broadcast_to(self.sb.exps[None, :], (self.sa.exps.size, self.sb.exps.size)).ravel()
        S = [self._s1d(d) for d in range(3)]

        def t1d(Sd, i, j):
            v = -2.0 * b * b * Sd[i, j + 2] + b * (2 * j + 1) * Sd[i, j]
            if j >= 2:
                v = v - 0.5 * j * (j - 1) * Sd[i, j - 2]
            return v
        out = np.empty((len(cart_comps(la)), len(cart_comps(lb))))
        for i, (ax, ay, az) in enumerate(cart_comps(la)):
            for j, (bx, by, bz) in enumerate(cart_comps(lb)):
                tx = t1d(S[0], ax, bx) * S[1][ay, by] * S[2][az, bz]
                ty = S[0][ax, bx] * t1d(S[1], ay, by) * S[2][az, bz]
                tz = S[0][ax, bx] * S[1][ay, by] * t1d(S[2], az, bz)
                out[i, j] = np.sum(self.cc * (tx + ty + tz))
        return out

    # ket-side 1D tables (need kin=True: E extended to lb + 2):
    #   D[i, j] = <i| d/dx |j> = j S[i, j-1] - 2 b S[i, j+1]
    #   X[i, j] = <i| x - O |j> = S[i, j+1] + (B - O) S[i, j]
    def _d1d(self, Sd):
        b = np.broadcast_to(self.sb.exps[None, :], (self.sa.exps.size, self.sb.exps.size)).ravel()
        la, lb = self.sa.l, self.sb.l
        D = np.empty((la + 1, lb + 1, b.size))
        for i in range(la + 1):
            for j in range(lb + 1):
                D[i, j] = -2.0 * b * Sd[i, j + 1] + (j * Sd[i, j - 1] if j >= 1 else 0.0)
        return D

    def deriv1(self):
        """<a| d/dr_d |b> for d = x, y, z: (3, nca, ncb).  Needs kin=True."""
        la, lb = self.sa.l, self.sb.l
        S = [self._s1d(d) for d in range(3)]
        D = [self._d1d(S[d]) for d in range(3)]
        out = np.empty((3, len(cart_comps(la)), len(cart_comps(lb))))
        for i, a in enumerate(cart_comps(la)):
            for j, b in enumerate(cart_comps(lb)):
                for d in range(3):
                    f = D[d][a[d], b[d]]
                    for e in range(3):
                        if e != d:
                            f = f * S[e][a[e], b[e]]
                    out[d, i, j] = np.sum(self.cc * f)
        return out

    def angmom(self, origin):
        """<a| ((r - origin) x nabla)_d |b>: (3, nca, ncb).  Needs kin=True."""
        la, lb = self.sa.l, self.sb.l
        S = [self._s1d(d) for d in range(3)]
        D = [self._d1d(S[d]) for d in range(3)]
        B = self.sb.center
        X = []
        for d in range(3):
            Xd = np.empty((la + 1, lb + 1, self.p.size))
            for i in range(la + 1):
                for j in range(lb + 1):
                    Xd[i, j] = S[d][i, j + 1] + (B[d] - origin[d]) * S[d][i, j]
            X.append(Xd)
        out = np.empty((3, len(cart_comps(la)), len(cart_comps(lb))))
        for i, a in enumerate(cart_comps(la)):
            for j, b in enumerate(cart_comps(lb)):
                for d, (u, v) in enumerate(((1, 2), (2, 0), (0, 1))):
                    w = 3 - u - v            # the untouched direction
                    t1 = X[u][a[u], b[u]] * D[v][a[v], b[v]]     # (r-O)_u d_v
                    t2 = X[v][a[v], b[v]] * D[u][a[u], b[u]]     # (r-O)_v d_u
                    out[d, i, j] = np.sum(self.cc * (t1 - t2) * S[w][a[w], b[w]])
        return out

    def multipole1(self, origin):
        """<a| (r - origin)_d |b> for d = x, y, z: (3, nca, ncb)."""
        la, lb = self.sa.l, self.sb.l
        S = [self._s1d(d) for d in range(3)]
        M = []
        for d in range(3):
            e = self.E[d].reshape(self.E[d].shape[:3] + (-1,))
            xpc = self.P[:, d] - origin[d]
            M.append(((e[:, :, 1] if e.shape[2] > 1 else 0.0) + xpc * e[:, :, 0]) * np.sqrt(np.pi / self.p))
        out = np.empty((3, len(cart_comps(la)), len(cart_comps(lb))))
        for i, (ax, ay, az) in enumerate(cart_comps(la)):
            for j, (bx, by, bz) in enumerate(cart_comps(lb)):
                out[0, i, j] = np.sum(self.cc * M[0][ax, bx] * S[1][ay, by] * S[2][az, bz])
                out[1, i, j] = np.sum(self.cc * S[0][ax, bx] * M[1][ay, by] * S[2][az, bz])
                out[2, i, j] = np.sum(self.cc * S[0][ax, bx] * S[1][ay, by] * M[2][az, bz])
        return out

    def nuclear(self, charges, coords):
        """sum_C -Z_C <a| 1/|r - C| |b> (point nuclei)."""
        acc = np.zeros(self.Eab.shape[:2])
        for z, c in zip(charges, coords):
            d = self.P - c
            R = hermite_r(self.L, self.p, d[:, 0], d[:, 1], d[:, 2])      # (ntuv, q)
            acc += -z * np.einsum('abtq,tq->ab', self.Eab, R * (2.0 * np.pi / self.p))
        return acc


def eri_quartet(bra: ShellPair, ket: ShellPair, omega: float = 0.0) -> np.ndarray:
    """(ab|cd) over Cartesian components: (nca, ncb, ncc, ncd); omega > 0: the
    long-range operator erf(omega r12)/r12."""
    p = bra.p[:, None]
    q = ket.p[None, :]
    alpha, scale = _attenuate(p * q / (p + q), omega)
    d = bra.P[:, None, :] - ket.P[None, :, :]
    L = bra.L + ket.L
    R = hermite_r(L, alpha, d[..., 0], d[..., 1], d[..., 2])          # (ntuv_L, P, Q)
    pref = 2.0 * np.pi ** 2.5 / (p * q * np.sqrt(p + q)) * scale
    idx, sign = _sum_table(bra.L, ket.L)
    Rm = R[idx] * pref                                                 # (ntab, ntcd, P, Q)
    X = np.einsum('tsPQ,s,cdsQ->tcdP', Rm, sign, ket.Eab, optimize=True)
    return np.einsum('abtP,tcdP->abcd', bra.Eab, X, optimize=True)


# ------------------------------------------------------------ 3-index (DF)
class AuxShellSet:
    """All auxiliary shells of one angular momentum, primitives stacked (for the
    3-index Coulomb integrals (ab|P) of density fitting).

    Each primitive of shell k is a one-centre Hermite expansion (the ket of a
    pair whose second function is the unit s function exp(0 r^2)); ``seg``
    maps stacked primitives to shells so the contraction is one product."""

    def __init__(self, shells):
        self.l = shells[0].l
        self.shells = shells
        self.p = np.concatenate([s.exps for s in shells])
        self.P = np.concatenate([np.repeat(s.center[None], s.exps.size, 0) for s in shells])
        self.coef = np.concatenate([s.coefs for s in shells])
        self.seg = np.zeros((self.p.size, len(shells)))
        q = 0
        for k, s in enumerate(shells):
            self.seg[q:q + s.exps.size, k] = 1.0
            q += s.exps.size
        # one-centre Hermite coefficients E^{i0}_t (b = 0): x^i e^{-p x^2} = sum_t E_t Lambda_t
        l = self.l
        tuv, _ = hermite_index(l)
        E1 = hermite_e(l, 0, self.p, np.zeros_like(self.p), 0.0)       # (l+1, 1, l+1, Q)
        comps = cart_comps(l)
        Ek = np.zeros((len(comps), len(tuv), self.p.size))
        for i, (ax, ay, az) in enumerate(comps):
            for k, (t, u, v) in enumerate(tuv):
                if t > ax or u > ay or v > az:
                    continue
                Ek[i, k] = E1[ax, 0, t] * E1[ay, 0, u] * E1[az, 0, v] * self.coef
        self.Ek = Ek


def eri3c(bra: ShellPair, aux: AuxShellSet, omega: float = 0.0) -> np.ndarray:
    """(ab|P) over Cartesian components for every shell of ``aux``:
    (nca, ncb, nshell_aux, ncart_aux); omega > 0: erf(omega r12)/r12."""
    p = bra.p[:, None]
    q = aux.p[None, :]
    alpha, scale = _attenuate(p * q / (p + q), omega)
    d = bra.P[:, None, :] - aux.P[None, :, :]
    L = bra.L + aux.l
    R = hermite_r(L, alpha, d[..., 0], d[..., 1], d[..., 2])          # (ntuv_L, P, Q)
    pref = 2.0 * np.pi ** 2.5 / (p * q * np.sqrt(p + q)) * scale
    idx, sign = _sum_table(bra.L, aux.l)
    Rm = R[idx] * pref                                                 # (ntab, ntc, P, Q)
    X = np.einsum('tsPQ,s,csQ->tcPQ', Rm, sign, aux.Ek, optimize=True)
    X = X @ aux.seg                                                    # (ntab, nc, P, nshell)
    return np.einsum('abtP,tcPk->abkc', bra.Eab, X, optimize=True)


def eri2c(auxa: AuxShellSet, auxb: AuxShellSet, omega: float = 0.0) -> np.ndarray:
    """(P|Q) over Cartesian components: (nshell_a, nca, nshell_b, ncb); omega > 0:
    erf(omega r12)/r12."""
    p = auxa.p[:, None]
    q = auxb.p[None, :]
    alpha, scale = _attenuate(p * q / (p + q), omega)
    d = auxa.P[:, None, :] - auxb.P[None, :, :]
    L = auxa.l + auxb.l
    R = hermite_r(L, alpha, d[..., 0], d[..., 1], d[..., 2])
    pref = 2.0 * np.pi ** 2.5 / (p * q * np.sqrt(p + q)) * scale
    idx, sign = _sum_table(auxa.l, auxb.l)
    Rm = R[idx] * pref
    X = np.einsum('tsPQ,s,csQ->tcPQ', Rm, sign, auxb.Ek, optimize=True) @ auxb.seg   # (nta, ncb, Pprim, kb)
    Y = np.einsum('atP,tcPk->aPck', auxa.Ek, X, optimize=True)                      # (nca, Pprim, ncb, kb)
    Y = np.einsum('aPck,Pj->jakc', Y, auxa.seg, optimize=True)
    return Y
