"""Two-electron integrals on the GPU (the device integral path):
the 3-index DF integrals and the 4-index ERIs of the exact-exchange path.

``int3c2e_device(mol, auxmol)`` returns the same (naux, nao, nao) tensor as
``Mole.int3c2e`` (PySCF ``df.incore.aux_e2(mol, auxmol, 'int3c2e')``, aux-major):

* per shell pair (i >= j) and per auxiliary shell the host prepares the Hermite
  expansion coefficients (``ints.ShellPair.Eab``, ``ints.AuxShellSet.Ek``: O(primitives)
  work);
* ``xt_int3c2e_cart`` (``csrc/xt_int.hip``) evaluates the quartic part on the
  device -- Boys functions, Hermite integrals, both contractions -- into one
  Cartesian matrix (pair components x auxiliary components);
* the spherical transforms are two ``xt_dgemm`` products with block-diagonal
  Cartesian -> solid-harmonic matrices; the (mu nu) <-> (nu mu) fill is one gather
  of pair rows and the AO / auxiliary normalisation element-wise, on the device.

``eri_full_device(mol)`` returns ``Mole.eri_full`` (PySCF ``mol.intor('int2e')``)
the same way, the ket given to the kernel as the same shell pairs.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _capi
from .gto import _sph_transform
from .ints import AuxShellSet, ShellPair


def _block_transform(shells):
    """Block-diagonal (n_sph_total, n_cart_total) Cartesian -> spherical matrix."""
    ns = sum(s.nsph for s in shells)
    nc = sum(s.ncart for s in shells)
    T = np.zeros((ns, nc))
    r = c = 0
    for s in shells:
        T[r:r + s.nsph, c:c + s.ncart] = _sph_transform(s.l)
        r += s.nsph
        c += s.ncart
    return T


def int3c2e_device(mol, auxmol, device: int = 0, omega: float = 0.0):
    """(P|mu nu) over normalised spherical functions, (naux, nao, nao), on the GPU
    (omega > 0: erf(omega r12)/r12)."""
    import torch
    L = _capi.lib()
    dev = torch.device(f"cuda:{device}")
    sh, ash = mol.shells, auxmol.shells
    n, naux = mol.nao, auxmol.nao
    pinfo, pprim, eab, prow, nrow = _pairs(mol)
    tp, sel = _pair_sph(mol, prow, nrow)
    # auxiliary shells
    ainfo, aprim, ek = [], [], []
    col = r0 = e0 = 0
    for s in ash:
        a = AuxShellSet([s])
        ainfo.append([s.l, s.exps.size, r0, e0, col, s.ncart, 0, 0])
        aprim.append(np.column_stack([a.p, a.P]))
        ek.append(a.Ek.ravel())
        col += s.ncart
        r0 += s.exps.size
        e0 += a.Ek.size
    ncol = col

    def dt(x, dtype=torch.float64):
        return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=dev)
    t_pinfo, t_pprim, t_eab = dt(pinfo, torch.int32), dt(pprim), dt(eab)
    t_ainfo = dt(np.array(ainfo, dtype=np.int32), torch.int32)
    t_aprim, t_ek = dt(np.concatenate(aprim)), dt(np.concatenate(ek))
    cart = torch.zeros((nrow, ncol), dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        st = torch.cuda.current_stream(dev).cuda_stream
        _capi.check(L.xt_int3c2e_cart(len(prow), t_pinfo.data_ptr(), t_pprim.data_ptr(), t_eab.data_ptr(),
                                      len(ash), t_ainfo.data_ptr(), t_aprim.data_ptr(), t_ek.data_ptr(),
                                      max(s.l for s in sh), max(s.l for s in ash), float(omega), cart.data_ptr(),
                                      ncol, ctypes.c_void_p(st)), "xt_int3c2e_cart")
        # spherical on both sides (pair blocks Ti (x) Tj, aux blocks Ta), then the
        # (mu nu) fill as one gather of pair rows
        ysph = _mm(L, st, dev, _mm(L, st, dev, dt(tp), cart), dt(_block_transform(ash)), tb=1)   # (npair_sph, naux)
        out = ysph.index_select(0, dt(sel, torch.int64)).t().reshape(naux, n, n)
        nrm = dt(mol._norm)
        out *= dt(auxmol._norm)[:, None, None] * nrm[None, :, None] * nrm[None, None, :]
        return out.cpu().numpy()


def _mm(L, st, dev, a, b, ta=0, tb=0):
    """op(a) @ op(b) for 2-D contiguous device tensors through the library's FP64 MFMA GEMM."""
    import torch
    m = a.shape[1] if ta else a.shape[0]
    k = a.shape[0] if ta else a.shape[1]
    nn = b.shape[0] if tb else b.shape[1]
    c = torch.empty((m, nn), dtype=torch.float64, device=dev)
    _capi.check(L.xt_dgemm(ta, tb, m, nn, k, 1.0, a.data_ptr(), a.shape[1], b.data_ptr(), b.shape[1],
                           0.0, c.data_ptr(), nn, ctypes.c_void_p(st)), "xt_dgemm")
    return c


def _pair_sph(mol, prow, ncart_tot):
    """Block-diagonal pair Cartesian -> spherical matrix (Ti (x) Tj per pair) and, per
    full index mu * n + nu, the spherical pair row that holds it (either order)."""
    sh, n = mol.shells, mol.nao
    nsph_tot = sum(sh[i].nsph * sh[j].nsph for i, j, _ in prow)
    tp = np.zeros((nsph_tot, ncart_tot))
    sel = np.empty(n * n, dtype=np.int64)
    r = 0
    for i, j, c0 in prow:
        si, sj = sh[i], sh[j]
        tp[r:r + si.nsph * sj.nsph, c0:c0 + si.ncart * sj.ncart] = np.kron(_sph_transform(si.l),
                                                                          _sph_transform(sj.l))
        mu = mol.ao_loc[i] + np.arange(si.nsph)[:, None]
        nu = mol.ao_loc[j] + np.arange(sj.nsph)[None, :]
        rows = r + np.arange(si.nsph * sj.nsph).reshape(si.nsph, sj.nsph)
        sel[(mu * n + nu).ravel()] = rows.ravel()
        sel[(nu * n + mu).ravel()] = rows.ravel()
        r += si.nsph * sj.nsph
    return tp, sel


def _pairs(mol):
    """Shell pairs i >= j: kernel tables (pair_info, pair_prim, eab) and per pair
    (i, j, first Cartesian row)."""
    sh = mol.shells
    pinfo, pprim, eab, prow = [], [], [], []
    row = q0 = e0 = 0
    for i in range(len(sh)):
        for j in range(i + 1):
            sp = ShellPair(sh[i], sh[j])
            nca, ncb, _, npp = sp.Eab.shape
            pinfo.append([sh[i].l, sh[j].l, npp, q0, e0, row, 0, 0])
            pprim.append(np.column_stack([sp.p, sp.P]))
            eab.append(sp.Eab.ravel())
            prow.append((i, j, row))
            row += nca * ncb
            q0 += npp
            e0 += sp.Eab.size
    return np.array(pinfo, dtype=np.int32), np.concatenate(pprim), np.concatenate(eab), prow, row


def eri_full_device(mol, device: int = 0, omega: float = 0.0):
    """(mu nu|la si) over normalised spherical AOs, all 8 symmetry copies (as
    ``Mole.eri_full``, PySCF ``mol.intor('int2e')``), on the GPU: the bra and the
    ket are the same shell-pair tables, the Cartesian (pair x pair) matrix comes
    from ``xt_int3c2e_cart`` with the ket given as pairs, the spherical transform
    is two ``xt_dgemm`` products and the symmetric fill one gather."""
    import torch
    L = _capi.lib()
    dev = torch.device(f"cuda:{device}")
    sh = mol.shells
    n = mol.nao
    pinfo, pprim, eab, prow, ncart_tot = _pairs(mol)
    ainfo = np.zeros_like(pinfo)                 # the ket: the same pairs
    ainfo[:, 0] = pinfo[:, 0] + pinfo[:, 1]
    ainfo[:, 1:5] = pinfo[:, 2:6]
    ainfo[:, 5] = [sh[i].ncart * sh[j].ncart for i, j, _ in prow]

    def dt(x, dtype=torch.float64):
        return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=dev)
    t_pinfo, t_ainfo = dt(pinfo, torch.int32), dt(ainfo, torch.int32)
    t_pprim, t_eab = dt(pprim), dt(eab)
    lmax = max(s.l for s in sh)
    cart = torch.zeros((ncart_tot, ncart_tot), dtype=torch.float64, device=dev)
    tp, sel = _pair_sph(mol, prow, ncart_tot)
    with torch.cuda.device(dev):
        st = torch.cuda.current_stream(dev).cuda_stream
        _capi.check(L.xt_int3c2e_cart(len(prow), t_pinfo.data_ptr(), t_pprim.data_ptr(), t_eab.data_ptr(),
                                      len(prow), t_ainfo.data_ptr(), t_pprim.data_ptr(), t_eab.data_ptr(),
                                      lmax, 2 * lmax, float(omega), cart.data_ptr(), ncart_tot, ctypes.c_void_p(st)),
                    "xt_int3c2e_cart (4-index)")
        t_tp = dt(tp)
        s_ = _mm(L, st, dev, _mm(L, st, dev, t_tp, cart), t_tp, tb=1)          # (nsph_tot, nsph_tot)
        # AO normalisation per pair row, then (ab|cd) = (cd|ab) exactly (the two come
        # from different threads' summation orders): every symmetry copy is one element
        w = np.zeros(s_.shape[0])
        w[sel] = np.outer(mol._norm, mol._norm).ravel()
        t_w = dt(w)
        s_ *= t_w[:, None] * t_w[None, :]
        s_ = 0.5 * (s_ + s_.t())
        idx = dt(sel, torch.int64)
        return s_.index_select(0, idx).index_select(1, idx).reshape(n, n, n, n).cpu().numpy()
