"""Integrals on the GPU (the device integral path).

Everything here goes through two library kernels (``csrc/xt_int.hip``):

* ``xt_int2e_cart`` -- McMurchie-Davidson Coulomb integrals between shell pairs
  (the bra) and a ket table (auxiliary shells, shell pairs, or point charges),
  orbital shells up to f;
* ``xt_eval_ao`` -- AO values and gradients on grid points.

The host prepares only per-shell-pair data (``ints.ShellPair.Eab``: Hermite
coefficients, O(primitives) work) once per molecule (``PairTable``, cached on the
``Mole``).  The Cartesian -> spherical transform is block-sparse: pairs are grouped
by (l_i, l_j) class and each class is one batched product with kron(T_li, T_lj) --
no dense transform matrix exists, so the memory stays O(pairs) at any size.

Entry points (all return what the host routines of ``gto.Mole`` return; tests
compare them to 1e-12):

* ``int3c2e_device``   -- (P|mu nu), PySCF ``df.incore.aux_e2`` (aux-major);
* ``eri_full_device``  -- (mu nu|la si), PySCF ``mol.intor('int2e')`` (small molecules);
* ``eri_diag_device`` / ``eri_columns_device`` -- the diagonal (mu nu|mu nu) and the
  columns (all pairs | chosen shell pairs) in the packed pair index
  mu (mu+1)/2 + nu, mu >= nu: the two integral requests of the integral-direct
  Cholesky factorisation (``qc/dchol.py``);
* ``int1e_nuc_device`` -- sum_C -Z_C <mu|1/|r-C||nu> (point charges as s shells of
  exponent 1e24 with coefficient (s/pi)^1.5: the kernel's prefactor then tends to
  PySCF's 2 pi / p to 1e-20 relative);
* ``eval_ao_device``   -- AO values (+ gradients) on grid points (PySCF ``eval_ao``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _capi
from .gto import _sph_transform
from .ints import AuxShellSet, ShellPair, ShellPairBatch, pair_classes

POINT_CHARGE_EXP = 1e24
AO_MAX_L = 4
PRIM_SCREEN = 1e-18       # primitive pairs below this bound are dropped (PairTable)


def _torch():
    import torch
    return torch


class PairTable:
    """Shell pairs i >= j of a Mole: the kernel tables, the block-sparse spherical
    transform and the index maps (spherical pair rows, packed pair index)."""

    def __init__(self, mol):
        sh = mol.shells
        n = mol.nao
        self.nao = n
        pinfo, pprim, eab, pairs = [], [], [], []
        c0s, s0s = [], []
        crow = srow = q0 = e0 = 0
        self.nprim_pairs = self.nprim_pairs_kept = 0
        # Hermite tables of every pair, vectorised over the pairs of a class (ShellPairBatch)
        tabs = [None] * (len(sh) * (len(sh) + 1) // 2)
        for kk, ii, jj in pair_classes(sh):
            bt = ShellPairBatch([sh[i] for i in ii], [sh[j] for j in jj])
            # primitive-pair screening: a primitive pair whose Hermite coefficients are
            # negligible (the Gaussian product factor exp(-ab/(a+b) |AB|^2) of two tight
            # primitives on different atoms) contributes below PRIM_SCREEN to every
            # integral -- its overlap-scale magnitude bounds its share of any (ab|cd),
            # (ab|P) or <a|V|b> (the max(1, sqrt p) covers the 1/p of the Coulomb kernel
            # against point charges); dropped from the kernels' loops
            bound = (np.abs(bt.Eab).reshape(len(ii), -1, bt.p.shape[1]).max(axis=1)
                     * (np.pi / bt.p) ** 1.5 * np.maximum(1.0, np.sqrt(bt.p)))
            for m, k in enumerate(kk):
                keep = bound[m] >= PRIM_SCREEN
                tabs[k] = (np.ascontiguousarray(bt.Eab[m][..., keep]), bt.p[m][keep], bt.P[m][keep])
                self.nprim_pairs += keep.size
                self.nprim_pairs_kept += int(keep.sum())
        # pair order: by total angular momentum, then by primitive pairs (most first) -- the
        # integral kernel runs one thread per (bra pair, ket) with the bra index fastest, so
        # a wave's bras share their class and loop trip counts
        tri = [(i, j) for i in range(len(sh)) for j in range(i + 1)]
        order = sorted(range(len(tri)), key=lambda kk: (sh[tri[kk][0]].l + sh[tri[kk][1]].l,
                                                        -tabs[kk][1].size, kk))
        for kk in order:
            i, j = tri[kk]
            eab_k, p_k, P_k = tabs[kk]
            tabs[kk] = None
            nca, ncb, _, npp = eab_k.shape
            pinfo.append([sh[i].l, sh[j].l, npp, q0, e0, crow, 0, 0])
            pprim.append(np.column_stack([p_k, P_k]))
            eab.append(eab_k.ravel())
            pairs.append((i, j))
            c0s.append(crow)
            s0s.append(srow)
            crow += nca * ncb
            srow += sh[i].nsph * sh[j].nsph
            q0 += npp
            e0 += eab_k.size
        self.pinfo = np.array(pinfo, dtype=np.int32)
        self.pprim = np.concatenate(pprim) if any(x.size for x in pprim) else np.zeros((1, 4))
        self.eab = np.concatenate(eab) if any(x.size for x in eab) else np.zeros(1)
        self.pairs = pairs
        self.npair = len(pairs)
        self.c0 = np.array(c0s, dtype=np.int64)
        self.s0 = np.array(s0s, dtype=np.int64)
        self.ncart_tot, self.nsph_tot = crow, srow
        self.lmax = max(s.l for s in sh)
        # spherical row of every (mu, nu) (either order), row norms, pair of each row
        sel = np.empty(n * n, dtype=np.int64)
        wrow = np.empty(srow)
        self.nab = np.empty(self.npair, dtype=np.int64)
        self.nsab = np.empty(self.npair, dtype=np.int64)
        nrm = mol._norm
        classes = {}
        for k, (i, j) in enumerate(pairs):
            si, sj = sh[i], sh[j]
            mu = mol.ao_loc[i] + np.arange(si.nsph)[:, None]
            nu = mol.ao_loc[j] + np.arange(sj.nsph)[None, :]
            rows = s0s[k] + np.arange(si.nsph * sj.nsph).reshape(si.nsph, sj.nsph)
            sel[(mu * n + nu).ravel()] = rows.ravel()
            sel[(nu * n + mu).ravel()] = rows.ravel()
            wrow[rows.ravel()] = (nrm[mu] * nrm[nu]).ravel()
            self.nab[k] = si.ncart * sj.ncart
            self.nsab[k] = si.nsph * sj.nsph
            classes.setdefault((si.l, sj.l), []).append(k)
        self.sel = sel
        self.wrow = wrow
        self.classes = {key: np.array(v, dtype=np.int64) for key, v in classes.items()}
        # packed pair index p = mu (mu + 1) / 2 + nu (mu >= nu) -> spherical row, pair id
        iu, ju = np.tril_indices(n)
        self.npack = iu.size
        packidx = np.empty(n * n, dtype=np.int64)
        pidx = iu * (iu + 1) // 2 + ju
        packidx[iu * n + ju] = pidx
        packidx[ju * n + iu] = pidx
        order = np.argsort(pidx)
        self.upack = sel[(iu * n + ju)[order]]                 # spherical row of packed index p
        self.packidx = packidx                                 # (mu, nu) -> packed index
        row_pair = np.empty(srow, dtype=np.int64)
        for k in range(self.npair):
            row_pair[s0s[k]:s0s[k] + self.nsab[k]] = k
        self.pack_pair = row_pair[self.upack]                  # shell pair of packed index p
        self._dev = {}

    # ------------------------------------------------------------ device copies
    def dev(self, device):
        """Kernel tables and transform blocks on GPU ``device`` (cached)."""
        if device in self._dev:
            return self._dev[device]
        torch = _torch()
        dv = torch.device(f"cuda:{device}")

        def t(x, dtype=torch.float64):
            return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=dv)
        d = dict(dev=dv, pinfo=t(self.pinfo, torch.int32), pprim=t(self.pprim), eab=t(self.eab),
                 wrow=t(self.wrow), upack=t(self.upack, torch.int64), sel=t(self.sel, torch.int64),
                 packidx=t(self.packidx, torch.int64), pack_pair=t(self.pack_pair, torch.int64))
        cls = []
        for (li, lj), ks in self.classes.items():
            Tk = np.kron(_sph_transform(li), _sph_transform(lj))
            ns, nc = Tk.shape
            cidx = self.c0[ks][:, None] + np.arange(nc)[None, :]
            sidx = self.s0[ks][:, None] + np.arange(ns)[None, :]
            cls.append((t(Tk), t(cidx, torch.int64), t(sidx, torch.int64), ks))
        d["classes"] = cls
        self._dev[device] = d
        return d

    # ------------------------------------------------------------ transforms
    def rows_to_sph(self, x, device):
        """(ncart_tot, m) Cartesian pair rows -> (nsph_tot, m) normalised spherical rows."""
        torch = _torch()
        d = self.dev(device)
        y = torch.empty((self.nsph_tot, x.shape[1]), dtype=torch.float64, device=d["dev"])
        for Tk, cidx, sidx, _ in d["classes"]:
            y[sidx.reshape(-1)] = torch.matmul(Tk, x[cidx]).reshape(-1, x.shape[1])
        y *= d["wrow"][:, None]
        return y

    def ket_info_pairs(self, ks, col_offsets=None):
        """Ket table (8 ints per entry) giving shell pairs ``ks`` as kets, output
        columns from ``col_offsets`` (default: consecutive Cartesian blocks)."""
        p = self.pinfo[ks]
        out = np.zeros((len(ks), 8), dtype=np.int32)
        out[:, 0] = p[:, 0] + p[:, 1]
        out[:, 1:4] = p[:, 2:5]
        nab = self.nab[ks]
        out[:, 4] = np.concatenate([[0], np.cumsum(nab)[:-1]]) if col_offsets is None else col_offsets
        out[:, 5] = nab
        return out


def pair_table(mol) -> PairTable:
    tab = getattr(mol, "_pair_table", None)
    if tab is None:
        tab = PairTable(mol)
        mol._pair_table = tab
    return tab


def _stream(device):
    torch = _torch()
    return ctypes.c_void_p(torch.cuda.current_stream(torch.device(f"cuda:{device}")).cuda_stream)


def _launch(L, tab, d, nket, kinfo, kprim, ek, lket, omega, out, ldo, device, qb=None, qk=None, thr=0.0,
            diag=0):
    _capi.check(L.xt_int2e_cart(tab.npair, d["pinfo"].data_ptr(), d["pprim"].data_ptr(), d["eab"].data_ptr(),
                                nket, kinfo.data_ptr(), kprim.data_ptr(), ek.data_ptr(), tab.lmax, int(lket),
                                float(omega), None if qb is None else qb.data_ptr(),
                                None if qk is None else qk.data_ptr(), float(thr), int(diag), out.data_ptr(),
                                int(ldo), _stream(device)), "xt_int2e_cart")


# ---------------------------------------------------------------- 3-index DF
def int3c2e_device(mol, auxmol, device: int = 0, omega: float = 0.0, as_tensor: bool = False):
    """(P|mu nu) over normalised spherical functions, (naux, nao, nao), on the GPU
    (omega > 0: erf(omega r12)/r12)."""
    torch = _torch()
    L = _capi.lib()
    tab = pair_table(mol)
    d = tab.dev(device)
    dv = d["dev"]
    ash = auxmol.shells
    n, naux = mol.nao, auxmol.nao
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

    def t(x, dtype=torch.float64):
        return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=dv)
    with torch.cuda.device(dv):
        cart = torch.zeros((tab.ncart_tot, ncol), dtype=torch.float64, device=dv)
        _launch(L, tab, d, len(ash), t(np.array(ainfo, dtype=np.int32), torch.int32), t(np.concatenate(aprim)),
                t(np.concatenate(ek)), max(s.l for s in ash), omega, cart, ncol, device)
        y = tab.rows_to_sph(cart, device)                                   # (nsph_tot, ncart_aux)
        del cart
        ta = torch.block_diag(*[t(_sph_transform(s.l)) for s in ash])       # (naux, ncart_aux)
        ysph = torch.matmul(y, ta.T)                                        # (nsph_tot, naux)
        out = ysph.index_select(0, d["sel"]).T.reshape(naux, n, n)
        out = out * t(auxmol._norm)[:, None, None]
        return out if as_tensor else out.cpu().numpy()


# ---------------------------------------------------------------- 4-index
def eri_full_device(mol, device: int = 0, omega: float = 0.0):
    """(mu nu|la si) over normalised spherical AOs, all 8 symmetry copies (as
    ``Mole.eri_full``, PySCF ``mol.intor('int2e')``), on the GPU: bra and ket are
    the same shell-pair table; exact (ab|cd) = (cd|ab) by symmetrising."""
    torch = _torch()
    L = _capi.lib()
    tab = pair_table(mol)
    d = tab.dev(device)
    dv = d["dev"]
    n = mol.nao
    kinfo = torch.as_tensor(tab.ket_info_pairs(np.arange(tab.npair), tab.c0.astype(np.int32)), device=dv)
    with torch.cuda.device(dv):
        cart = torch.zeros((tab.ncart_tot, tab.ncart_tot), dtype=torch.float64, device=dv)
        _launch(L, tab, d, tab.npair, kinfo, d["pprim"], d["eab"], 2 * tab.lmax, omega, cart, tab.ncart_tot, device)
        y = tab.rows_to_sph(tab.rows_to_sph(cart, device).T.contiguous(), device)   # (nsph, nsph), symmetric
        y = 0.5 * (y + y.T)
        return y.index_select(0, d["sel"]).index_select(1, d["sel"]).reshape(n, n, n, n).cpu().numpy()


def _diag_blocks(tab, device, omega=0.0):
    """Cartesian diagonal blocks (ab|ab) of every shell pair: (ncart_tot, maxnab)."""
    torch = _torch()
    L = _capi.lib()
    d = tab.dev(device)
    ldo = int(tab.nab.max())
    kinfo = torch.as_tensor(tab.ket_info_pairs(np.arange(tab.npair), np.zeros(tab.npair, dtype=np.int32)),
                            device=d["dev"])
    out = torch.zeros((tab.ncart_tot, ldo), dtype=torch.float64, device=d["dev"])
    _launch(L, tab, d, tab.npair, kinfo, d["pprim"], d["eab"], 2 * tab.lmax, omega, out, ldo, device, diag=1)
    return out


def eri_diag_device(mol, device: int = 0, omega: float = 0.0):
    """(diag, q): the packed ERI diagonal (mu nu|mu nu), mu >= nu, (npack,) and the
    per-shell-pair Schwarz bound q[k] >= |(mu nu|la si)| / q[k'] for normalised
    spherical AOs of pairs k, k' (device tensors)."""
    torch = _torch()
    tab = pair_table(mol)
    d = tab.dev(device)
    dv = d["dev"]
    with torch.cuda.device(dv):
        blk = _diag_blocks(tab, device, omega)
        dsph = torch.empty(tab.nsph_tot, dtype=torch.float64, device=dv)
        q = torch.empty(tab.npair, dtype=torch.float64, device=dv)
        wmax = torch.zeros(tab.npair, dtype=torch.float64, device=dv)
        wmax.scatter_reduce_(0, torch.as_tensor(np.repeat(np.arange(tab.npair), tab.nsab), device=dv),
                             d["wrow"], reduce="amax")
        for Tk, cidx, sidx, ks in d["classes"]:
            nc = cidx.shape[1]
            b = blk[cidx][:, :, :nc]                                          # (npc, nc, nc)
            dsph[sidx.reshape(-1)] = torch.einsum('sa,kab,sb->ks', Tk, b, Tk).reshape(-1)
            cmax = torch.diagonal(b, dim1=1, dim2=2).clamp(min=0).amax(dim=1)
            q[torch.as_tensor(ks, device=dv)] = torch.sqrt(cmax) * Tk.abs().sum(1).max()
        dsph *= d["wrow"] ** 2
        q *= wmax
        return dsph[d["upack"]], q


def eri_columns_device(mol, kets, q=None, thr: float = 0.0, device: int = 0, omega: float = 0.0):
    """Columns (all packed pairs | packed pairs of shell pairs ``kets``):
    returns (packed column indices (m,), (npack, m) tensor).  With Schwarz bounds
    ``q`` (eri_diag_device) blocks whose bound is below ``thr`` are skipped."""
    torch = _torch()
    L = _capi.lib()
    tab = pair_table(mol)
    d = tab.dev(device)
    dv = d["dev"]
    kets = np.asarray(kets, dtype=np.int64)
    nab = tab.nab[kets]
    ncol = int(nab.sum())
    kinfo = torch.as_tensor(tab.ket_info_pairs(kets), device=dv)
    with torch.cuda.device(dv):
        cart = torch.zeros((tab.ncart_tot, ncol), dtype=torch.float64, device=dv)
        qk = None if q is None else q[torch.as_tensor(kets, device=dv)].contiguous()
        _launch(L, tab, d, len(kets), kinfo, d["pprim"], d["eab"], 2 * tab.lmax, omega, cart, ncol, device,
                qb=q, qk=qk, thr=thr)
        rows = tab.rows_to_sph(cart, device)[d["upack"]]                    # (npack, ncol) packed rows
        del cart
        # ket side: Cartesian -> spherical, one batched product per (l_i, l_j) class of the
        # kets, then the unique (mu >= nu) columns times their norms -- a few uploads per
        # batch instead of several per ket
        cstart = np.concatenate([[0], np.cumsum(nab)[:-1]])
        by_class = {}
        for pos, k in enumerate(kets):
            i, j = tab.pairs[k]
            by_class.setdefault((mol.shells[i].l, mol.shells[j].l), []).append(pos)
        tks = d.setdefault("ket_tk", {})
        blocks, cols, sel, wts = [], [], [], []
        off = 0
        for (li, lj), poss in by_class.items():
            if (li, lj) not in tks:
                tks[(li, lj)] = torch.as_tensor(np.kron(_sph_transform(li), _sph_transform(lj)), device=dv)
            Tk = tks[(li, lj)]
            ns, nc = Tk.shape
            cidx = torch.as_tensor((cstart[poss][:, None] + np.arange(nc)[None, :]).ravel(), device=dv)
            blocks.append(torch.matmul(rows[:, cidx].reshape(-1, len(poss), nc), Tk.T).reshape(-1, len(poss) * ns))
            for m, pos in enumerate(poss):
                i, j = tab.pairs[kets[pos]]
                si, sj = mol.shells[i], mol.shells[j]
                mu = mol.ao_loc[i] + np.arange(si.nsph)[:, None]
                nu = mol.ao_loc[j] + np.arange(sj.nsph)[None, :]
                keep = np.where((mu >= nu).ravel())[0]
                sel.append(off + m * ns + keep)
                wts.append((mol._norm[mu] * mol._norm[nu]).ravel()[keep])
                mm = np.broadcast_to(mu, (si.nsph, sj.nsph)).ravel()[keep]
                nn = np.broadcast_to(nu, (si.nsph, sj.nsph)).ravel()[keep]
                cols.append(mm * (mm + 1) // 2 + nn)
            off += len(poss) * ns
        allb = torch.cat(blocks, dim=1) if len(blocks) > 1 else blocks[0]
        tsel = torch.as_tensor(np.concatenate(sel), device=dv)
        tw = torch.as_tensor(np.concatenate(wts), device=dv)
        return np.concatenate(cols), allb[:, tsel] * tw[None, :]


# ---------------------------------------------------------------- 1-electron
def int1e_nuc_device(mol, device: int = 0):
    """Nuclear attraction sum_C -Z_C <mu|1/|r - C||nu> (PySCF int1e_nuc) on the GPU."""
    torch = _torch()
    L = _capi.lib()
    tab = pair_table(mol)
    d = tab.dev(device)
    dv = d["dev"]
    natm = mol.natm
    s = POINT_CHARGE_EXP
    kinfo = np.zeros((natm, 8), dtype=np.int32)
    kinfo[:, 1] = 1
    kinfo[:, 2] = np.arange(natm)
    kinfo[:, 3] = np.arange(natm)
    kinfo[:, 4] = np.arange(natm)
    kinfo[:, 5] = 1
    kprim = np.column_stack([np.full(natm, s), mol.atom_coords()])
    ek = -mol._charges * (s / np.pi) ** 1.5
    with torch.cuda.device(dv):
        cart = torch.zeros((tab.ncart_tot, natm), dtype=torch.float64, device=dv)
        _launch(L, tab, d, natm, torch.as_tensor(kinfo, device=dv), torch.as_tensor(kprim, device=dv),
                torch.as_tensor(ek, device=dv), 0, 0.0, cart, natm, device)
        v = tab.rows_to_sph(cart.sum(1, keepdim=True).contiguous(), device)[:, 0]
        n = mol.nao
        return v[d["sel"]].reshape(n, n).cpu().numpy()


# ---------------------------------------------------------------- AO on the grid
_SPH_TAB = None


def _sph_table():
    global _SPH_TAB
    if _SPH_TAB is None:
        _SPH_TAB = np.concatenate([_sph_transform(l).ravel() for l in range(AO_MAX_L + 1)])
    return _SPH_TAB


def ao_shell_tables(mol):
    """(shell_info (nshell, 8) int32, shell_data) for xt_eval_ao."""
    info, dat = [], []
    off = 0
    for s, p0 in zip(mol.shells, mol.ao_loc[:-1]):
        if s.l > AO_MAX_L:
            raise ValueError(f"xt_eval_ao handles l <= {AO_MAX_L}, got {s.l}")
        info.append([s.l, s.exps.size, off, int(p0), 0, 0, 0, 0])
        dat.append(np.concatenate([s.exps, s.coefs, s.center]))
        off += 2 * s.exps.size + 3
    return np.array(info, dtype=np.int32), np.concatenate(dat)


def eval_ao_device(mol, coords, deriv: int = 0, device: int = 0, out=None, block: int = 1 << 17):
    """AO values (deriv 0: (ngrid, nao)) or values + gradients (deriv 1:
    (4, ngrid, nao)) on the GPU as a device tensor; evaluated in grid blocks of
    ``block`` points into one resident array (or ``out``)."""
    torch = _torch()
    L = _capi.lib()
    dv = torch.device(f"cuda:{device}")
    c = coords if isinstance(coords, torch.Tensor) else torch.as_tensor(np.ascontiguousarray(coords), device=dv)
    c = c.to(dv, torch.float64).contiguous()
    ng, n = c.shape[0], mol.nao
    ncomp = 4 if deriv else 1
    info, dat = ao_shell_tables(mol)
    with torch.cuda.device(dv):
        t_info = torch.as_tensor(info, device=dv)
        t_dat = torch.as_tensor(dat, device=dv)
        t_sph = torch.as_tensor(_sph_table(), device=dv)
        t_nrm = torch.as_tensor(mol._norm, device=dv)
        if out is None:
            out = torch.empty((ncomp, ng, n), dtype=torch.float64, device=dv)
        st = _stream(device)
        for g0 in range(0, ng, block):
            g1 = min(ng, g0 + block)
            _capi.check(L.xt_eval_ao(g1 - g0, c[g0:g1].data_ptr(), len(mol.shells), t_info.data_ptr(),
                                     t_dat.data_ptr(), t_sph.data_ptr(), t_nrm.data_ptr(), int(bool(deriv)),
                                     out[0, g0:g1].data_ptr(), n, ng * n, st), "xt_eval_ao")
    return out if deriv else out[0]
