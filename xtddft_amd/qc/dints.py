"""3-index DF integrals on the GPU (the device integral path).

``int3c2e_device(mol, auxmol)`` returns the same (naux, nao, nao) tensor as
``Mole.int3c2e`` (PySCF ``df.incore.aux_e2(mol, auxmol, 'int3c2e')``, aux-major):

* per shell pair (i >= j) and per auxiliary shell the host prepares the Hermite
  expansion coefficients (``ints.ShellPair.Eab``, ``ints.AuxShellSet.Ek``: O(primitives)
  work);
* ``xt_int3c2e_cart`` (``csrc/xt_int.hip``) evaluates the quartic part on the
  device -- Boys functions, Hermite integrals, both contractions -- into one
  Cartesian matrix (pair components x auxiliary components);
* the spherical transforms are two ``xt_dgemm`` products with block-diagonal
  Cartesian -> solid-harmonic matrices; the AO / auxiliary normalisation and the
  (mu nu) <-> (nu mu) fill are element-wise on the device.
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


def int3c2e_device(mol, auxmol, device: int = 0):
    """(P|mu nu) over normalised spherical functions, (naux, nao, nao), on the GPU."""
    import torch
    L = _capi.lib()
    dev = torch.device(f"cuda:{device}")
    sh, ash = mol.shells, auxmol.shells
    # ---- shell pairs i >= j: Hermite coefficients and primitive-pair centres
    pinfo, pprim, eab, prow = [], [], [], []
    row = q0 = e0 = 0
    for i in range(len(sh)):
        for j in range(i + 1):
            sp = ShellPair(sh[i], sh[j])
            nca, ncb, _, npp = sp.Eab.shape
            pinfo += [sh[i].l, sh[j].l, npp, q0, e0, row, 0, 0]
            pprim.append(np.column_stack([sp.p, sp.P]))
            eab.append(sp.Eab.ravel())
            prow.append((i, j, row))
            row += nca * ncb
            q0 += npp
            e0 += sp.Eab.size
    nrow = row
    # ---- auxiliary shells
    ainfo, aprim, ek = [], [], []
    col = r0 = e0 = 0
    for s in ash:
        a = AuxShellSet([s])
        ainfo += [s.l, s.exps.size, r0, e0, col, 0, 0, 0]
        aprim.append(np.column_stack([a.p, a.P]))
        ek.append(a.Ek.ravel())
        col += s.ncart
        r0 += s.exps.size
        e0 += a.Ek.size
    ncol = col

    def dt(x, dtype=torch.float64):
        return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=dev)
    t_pinfo = dt(np.array(pinfo, dtype=np.int32), torch.int32)
    t_pprim = dt(np.concatenate(pprim))
    t_eab = dt(np.concatenate(eab))
    t_ainfo = dt(np.array(ainfo, dtype=np.int32), torch.int32)
    t_aprim = dt(np.concatenate(aprim))
    t_ek = dt(np.concatenate(ek))
    cart = torch.zeros((nrow, ncol), dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        st = torch.cuda.current_stream(dev).cuda_stream
        _capi.check(L.xt_int3c2e_cart(len(prow), t_pinfo.data_ptr(), t_pprim.data_ptr(), t_eab.data_ptr(),
                                      len(ash), t_ainfo.data_ptr(), t_aprim.data_ptr(), t_ek.data_ptr(),
                                      max(s.l for s in sh), max(s.l for s in ash), cart.data_ptr(), ncol,
                                      ctypes.c_void_p(st)), "xt_int3c2e_cart")

        def mm(a, b, tb=0):        # a @ op(b) through the library's FP64 MFMA GEMM
            m, k = a.shape
            n = b.shape[0] if tb else b.shape[1]
            c = torch.empty((m, n), dtype=torch.float64, device=dev)
            _capi.check(L.xt_dgemm(0, tb, m, n, k, 1.0, a.data_ptr(), a.shape[1], b.data_ptr(), b.shape[1],
                                   0.0, c.data_ptr(), n, ctypes.c_void_p(st)), "xt_dgemm")
            return c
        # auxiliary Cartesian -> spherical for every row at once: (nrow, naux)
        ta = dt(_block_transform(ash))
        y = mm(cart, ta, tb=1)
        naux, n = auxmol.nao, mol.nao
        out = torch.zeros((naux, n, n), dtype=torch.float64, device=dev)
        yt = y.t().contiguous()                                  # (naux, nrow)
        tcache = {}
        for i, j, r in prow:
            si, sj = sh[i], sh[j]
            a0, a1 = int(mol.ao_loc[i]), int(mol.ao_loc[i + 1])
            b0, b1 = int(mol.ao_loc[j]), int(mol.ao_loc[j + 1])
            key = (si.l, sj.l)
            if key not in tcache:       # Ti (x) Tj over the pair's Cartesian components
                tcache[key] = dt(np.kron(_sph_transform(si.l), _sph_transform(sj.l)))
            blk = mm(yt[:, r:r + si.ncart * sj.ncart].contiguous(), tcache[key], tb=1)
            blk = blk.reshape(naux, si.nsph, sj.nsph)
            out[:, a0:a1, b0:b1] = blk
            out[:, b0:b1, a0:a1] = blk.transpose(1, 2)
        nrm = dt(mol._norm)
        out *= dt(auxmol._norm)[:, None, None] * nrm[None, :, None] * nrm[None, None, :]
        return out.cpu().numpy()
