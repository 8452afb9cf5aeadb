"""``Mole``: atoms + spherical Gaussian basis, the ``gto.M(...)`` the reference's
drivers start from (``example/XSF_TDA.ipynb`` cell 1, ``XTDA.py:1486-1556``).

Conventions follow PySCF/libcint so that AO-basis quantities are directly
comparable with the reference:

* coordinates in Bohr, ``BOHR = 0.52917721092`` Angstrom (PySCF ``param.BOHR``);
* spherical AOs, shell by shell in input order; p shells ordered (px, py, pz),
  d shells (xy, yz, z^2, xz, x^2-y^2);
* primitive coefficients scaled by the radial norm of r^l exp(-a r^2) and each
  AO normalised to one (PySCF ``NORMALIZE_GTO``), so ``diag(S) = 1``.

Point-group symmetry is supported for the case the reference examples use:
linear or planar molecules whose symmetry planes are the xz / yz planes
(C2v with the z axis as C2; ``Coov`` is run in its C2v subgroup, as PySCF does,
``example/XSF_TDA.ipynb``: "point group symmetry = Coov, use subgroup C2v").
Each AO then belongs to one irrep (``ao_irreps``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from . import basis as _basis
from .ints import AuxShellSet, ShellPair, cart_comps, eri2c, eri3c, eri_quartet

BOHR = 0.52917721092

ELEMENTS = ["X", "H", "He", "Li", "Be", "B", "C", "N", "O", "F", "Ne", "Na", "Mg", "Al", "Si",
            "P", "S", "Cl", "Ar", "K", "Ca", "Sc", "Ti", "V", "Cr", "Mn", "Fe", "Co", "Ni", "Cu",
            "Zn", "Ga", "Ge", "As", "Se", "Br", "Kr"]
CHARGE = {s: i for i, s in enumerate(ELEMENTS)}

C2V_IRREPS = ("A1", "A2", "B1", "B2")     # PySCF order; B1 ~ x, B2 ~ y


def _sph_transform(l: int) -> np.ndarray:
    """(n_sph, n_cart) un-normalised real solid harmonics in libcint order:
    p as (x, y, z); l >= 2 as m = -l..l (d: xy, yz, z^2, xz, x^2-y^2), each the
    Helgaker-Joergensen-Olsen expansion (eq. 6.4.48) of S_lm in Cartesian
    monomials x^i y^j z^k (the AO normalisation is applied afterwards)."""
    if l == 0:
        return np.ones((1, 1))
    if l == 1:
        return np.eye(3)
    return _solid_harmonics(l)


def _solid_harmonics(l: int) -> np.ndarray:
    from math import comb
    comps = cart_comps(l)
    pos = {c: i for i, c in enumerate(comps)}
    out = np.zeros((2 * l + 1, len(comps)))
    for row, m in enumerate(range(-l, l + 1)):
        am = abs(m)
        vm2 = 0 if m >= 0 else 1                     # 2 v_m
        for t in range((l - am) // 2 + 1):
            for u in range(t + 1):
                # v = v_m .. floor(|m|/2 - v_m) + v_m, stored as 2v
                v2 = vm2
                while v2 <= 2 * ((am - vm2) // 2) + vm2 and v2 <= am:
                    c = ((-1) ** (t + (v2 - vm2) // 2) * 0.25 ** t * comb(l, t) * comb(l - t, am + t)
                         * comb(t, u) * comb(am, v2))
                    ix = 2 * t + am - 2 * u - v2
                    iy = 2 * u + v2
                    iz = l - 2 * t - am
                    out[row, pos[(ix, iy, iz)]] += c
                    v2 += 2
    return out


def gto_norm(l: int, a: np.ndarray) -> np.ndarray:
    """Radial norm of r^l exp(-a r^2) (PySCF gto.gto_norm)."""
    return np.sqrt(2.0 * (2.0 * a) ** (l + 1.5) / math.gamma(l + 1.5))


@dataclass
class Shell:
    atom: int
    l: int
    center: np.ndarray
    exps: np.ndarray
    coefs: np.ndarray          # primitive coefficients x radial norms (one contraction)

    @property
    def ncart(self):
        return (self.l + 1) * (self.l + 2) // 2

    @property
    def nsph(self):
        return 2 * self.l + 1


def _parse_atoms(atom) -> List[tuple]:
    if isinstance(atom, str):
        items = []
        for line in atom.replace(";", "\n").splitlines():
            f = line.split()
            if not f:
                continue
            items.append((f[0], tuple(float(x) for x in f[1:4])))
        return items
    return [(a[0], tuple(float(x) for x in a[1])) for a in atom]


class Mole:
    """Minimal ``gto.Mole``: geometry, basis, electron count, integrals."""

    def __init__(self, atom, basis="6-31G", charge: int = 0, spin: int = 0,
                 unit: str = "Angstrom", symmetry=False, verbose: int = 0):
        self.atom = atom
        self.basis = basis
        self.charge = int(charge)
        self.spin = int(spin)
        self.unit = unit
        self.verbose = verbose
        atoms = _parse_atoms(atom)
        scale = 1.0 / BOHR if unit.lower().startswith("a") else 1.0
        self.elements = [a[0].capitalize() for a in atoms]
        self._coords = np.array([a[1] for a in atoms], dtype=np.float64) * scale
        self._charges = np.array([CHARGE[e] for e in self.elements], dtype=np.float64)
        self.nelectron = int(round(self._charges.sum())) - self.charge
        if (self.nelectron + self.spin) % 2:
            raise ValueError(f"electron number {self.nelectron} and spin {self.spin} are inconsistent")
        self.shells: List[Shell] = []
        for ia, el in enumerate(self.elements):
            for sh in _basis.load(basis, el):
                l = int(sh[0])
                prim = np.array(sh[1:], dtype=np.float64)
                exps = prim[:, 0]
                for ic in range(1, prim.shape[1]):
                    c = prim[:, ic] * gto_norm(l, exps)
                    self.shells.append(Shell(ia, l, self._coords[ia].copy(), exps.copy(), c))
        self.ao_loc = np.cumsum([0] + [s.nsph for s in self.shells])
        self._nao = int(self.ao_loc[-1])
        self.symmetry = self._check_symmetry(symmetry)
        self._norm = None
        self._int1e = {}
        # AO norms need only the diagonal shell blocks <a|a>
        diag = np.empty(self._nao)
        for s, p0 in zip(self.shells, self.ao_loc[:-1]):
            T = _sph_transform(s.l)
            diag[p0:p0 + s.nsph] = np.diag(T @ ShellPair(s, s, hermite=False).overlap() @ T.T)
        self._norm = 1.0 / np.sqrt(diag)

    # -------------------------------------------------------------- basics
    def nao_nr(self) -> int:
        return self._nao

    @property
    def nao(self) -> int:
        return self._nao

    @property
    def natm(self) -> int:
        return len(self.elements)

    @property
    def nelec(self):
        return ((self.nelectron + self.spin) // 2, (self.nelectron - self.spin) // 2)

    def atom_coords(self) -> np.ndarray:
        return self._coords.copy()

    def atom_charges(self) -> np.ndarray:
        return self._charges.astype(np.int64)

    def energy_nuc(self) -> float:
        e = 0.0
        for i in range(self.natm):
            for j in range(i):
                e += self._charges[i] * self._charges[j] / np.linalg.norm(self._coords[i] - self._coords[j])
        return e

    def ao_atom(self) -> np.ndarray:
        out = np.empty(self._nao, dtype=np.int64)
        for s, p0, p1 in zip(self.shells, self.ao_loc[:-1], self.ao_loc[1:]):
            out[p0:p1] = s.atom
        return out

    # ------------------------------------------------------------ symmetry
    def _check_symmetry(self, symmetry):
        if not symmetry:
            return None
        group = str(symmetry)
        if group is True or group.lower() in ("true", "c2v", "coov"):
            xy = self._coords[:, :2]
            if np.abs(xy).max() > 1e-8:
                raise NotImplementedError("symmetry is supported for molecules on the z axis "
                                          "(C2v / Coov run in C2v)")
            return "C2v"
        raise NotImplementedError(f"point group {symmetry!r} not supported (C2v / Coov only)")

    def ao_irreps(self) -> np.ndarray:
        """Irrep index (into C2V_IRREPS) of every AO under C2v (z = C2 axis)."""
        if self.symmetry is None:
            raise ValueError("mol.symmetry is off")
        out = np.empty(self._nao, dtype=np.int64)
        for s, p0 in zip(self.shells, self.ao_loc[:-1]):
            T = _sph_transform(s.l)
            comps = cart_comps(s.l)
            for m in range(s.nsph):
                nz = [comps[c] for c in range(len(comps)) if abs(T[m, c]) > 0]
                px = {c[0] % 2 for c in nz}
                py = {c[1] % 2 for c in nz}
                assert len(px) == 1 and len(py) == 1
                odd_x, odd_y = px.pop(), py.pop()
                out[p0 + m] = {(0, 0): 0, (1, 1): 1, (1, 0): 2, (0, 1): 3}[(odd_x, odd_y)]
        return out

    # ----------------------------------------------------------- integrals
    def _ovlp_kin(self):
        """int1e_ovlp and int1e_kin in one pass over the shell pairs, vectorised over the
        pairs of each class (``ints.ShellPairBatch``; the pair's Hermite tables, extended
        for the kinetic operator, serve both); cached."""
        if "kin" not in self._int1e:
            from .ints import ShellPairBatch, pair_classes
            n = self._nao
            S, T = np.zeros((n, n)), np.zeros((n, n))
            sh = self.shells
            loc = self.ao_loc
            for _, ii, jj in pair_classes(sh):
                batch = ShellPairBatch([sh[i] for i in ii], [sh[j] for j in jj], kin=True, hermite=False)
                Ti, Tj = _sph_transform(sh[ii[0]].l), _sph_transform(sh[jj[0]].l)
                mi, nj = Ti.shape[0], Tj.shape[0]
                rows = loc[ii][:, None, None] + np.arange(mi)[None, :, None]
                cols = loc[jj][:, None, None] + np.arange(nj)[None, None, :]
                rows, cols = np.broadcast_arrays(rows, cols)
                for out, blk in ((S, batch.overlap()), (T, batch.kinetic())):
                    blk = np.einsum('mi,pij,nj->pmn', Ti, blk, Tj)
                    out[rows, cols] = blk
                    out[cols, rows] = blk
            nrm = self._norm[:, None] * self._norm[None, :]
            self._int1e["ovlp"], self._int1e["kin"] = S * nrm, T * nrm
        return self._int1e["ovlp"].copy(), self._int1e["kin"].copy()

    def _intor_raw(self, kind, origin=(0.0, 0.0, 0.0)):
        n = self._nao
        if kind in ("ovlp", "kin") and self._norm is not None:
            return self._ovlp_kin()[0 if kind == "ovlp" else 1]
        if kind in ("r", "ipovlp", "irxp"):
            out = np.zeros((3, n, n))
        else:
            out = np.zeros((n, n))
        sh = self.shells
        for i, si in enumerate(sh):
            Ti = _sph_transform(si.l)
            for j in range(i + 1):
                sj = sh[j]
                Tj = _sph_transform(sj.l)
                pair = ShellPair(si, sj, kin=kind in ("kin", "ipovlp", "irxp"))
                if kind == "ovlp":
                    blk = pair.overlap()
                elif kind == "kin":
                    blk = pair.kinetic()
                elif kind == "nuc":
                    blk = pair.nuclear(self._charges, self._coords)
                elif kind == "r":
                    blk = pair.multipole1(np.asarray(origin, dtype=np.float64))
                elif kind == "ipovlp":     # <nabla a | b> = -<a | nabla b>
                    blk = -pair.deriv1()
                elif kind == "irxp":       # <a | (r - O) x nabla | b>
                    blk = pair.angmom(np.asarray(origin, dtype=np.float64))
                else:
                    raise KeyError(kind)
                three = kind in ("r", "ipovlp", "irxp")
                blk = np.einsum('mi,dij,nj->dmn', Ti, blk, Tj) if three else Ti @ blk @ Tj.T
                a0, a1 = self.ao_loc[i], self.ao_loc[i + 1]
                b0, b1 = self.ao_loc[j], self.ao_loc[j + 1]
                if three:
                    sign = 1.0 if kind == "r" else -1.0   # hermitian / anti-hermitian
                    out[:, b0:b1, a0:a1] = sign * blk.transpose(0, 2, 1)
                    out[:, a0:a1, b0:b1] = blk
                else:
                    out[a0:a1, b0:b1] = blk
                    out[b0:b1, a0:a1] = blk.T
        if self._norm is not None:
            nrm = self._norm
            out = out * (nrm[:, None] * nrm[None, :])
        return out

    def intor_symmetric(self, name: str, comp=None, origin=(0.0, 0.0, 0.0)):
        """PySCF ``Mole.intor_symmetric`` (the one-electron integrals here are all hermitian)."""
        return self.intor(name, comp=comp, origin=origin)

    def intor(self, name: str, comp=None, hermi=0, origin=(0.0, 0.0, 0.0), device=None):
        """PySCF names: int1e_ovlp, int1e_kin, int1e_nuc, int1e_r, int1e_ipovlp,
        int1e_cg_irxp (comp 3; common gauge origin = ``origin``, PySCF's default 0), int2e.
        ``device=k``: int1e_nuc and int2e through the GPU integral kernel (``qc.dints``)."""
        key = name.replace("_sph", "")
        if device is not None and key == "int1e_nuc":
            from .dints import int1e_nuc_device
            return int1e_nuc_device(self, device)
        if device is not None and key == "int2e":
            return self.eri_full(device=device)
        if key == "int1e_ovlp":
            return self._intor_raw("ovlp")
        if key == "int1e_kin":
            return self._intor_raw("kin")
        if key == "int1e_nuc":
            return self._intor_raw("nuc")
        if key == "int1e_r":
            return self._intor_raw("r", origin)
        if key == "int1e_ipovlp":       # (nabla i | j), anti-hermitian
            return self._intor_raw("ipovlp")
        if key == "int1e_cg_irxp":      # i (r - common origin) x p = (r - O) x nabla, anti-hermitian
            return self._intor_raw("irxp", origin)
        if key == "int2e":
            return self.eri_full()
        raise KeyError(name)

    # -------------------------------------------------- density fitting
    def _aux_groups(self):
        """{l: (AuxShellSet, AO offsets of its shells)} in shell order."""
        groups = {}
        for k, sh in enumerate(self.shells):
            groups.setdefault(sh.l, []).append(k)
        return {l: (AuxShellSet([self.shells[k] for k in ks]), [int(self.ao_loc[k]) for k in ks])
                for l, ks in groups.items()}

    def int3c2e(self, auxmol, device=None, omega: float = 0.0) -> np.ndarray:
        """(P|mu nu) over normalised spherical functions: (naux, nao, nao) -- PySCF
        ``df.incore.aux_e2(mol, auxmol, 'int3c2e')`` transposed to aux-major.
        ``device=k``: evaluated on GPU k (``qc.dints``, the HIP integral kernel);
        ``omega > 0``: the long-range operator erf(omega r12)/r12 (PySCF
        ``mol.with_range_coulomb(omega)``)."""
        if device is not None:
            from .dints import int3c2e_device
            return int3c2e_device(self, auxmol, device, omega=omega)
        n, naux = self._nao, auxmol.nao
        out = np.zeros((naux, n, n))
        aux = auxmol._aux_groups()
        Ta = {l: _sph_transform(l) for l in aux}
        sh = self.shells
        for i in range(len(sh)):
            Ti = _sph_transform(sh[i].l)
            a = slice(self.ao_loc[i], self.ao_loc[i + 1])
            for j in range(i + 1):
                Tj = _sph_transform(sh[j].l)
                b = slice(self.ao_loc[j], self.ao_loc[j + 1])
                pair = ShellPair(sh[i], sh[j])
                for l, (aset, offs) in aux.items():
                    blk = eri3c(pair, aset, omega)                   # (ca, cb, k, cP)
                    blk = np.einsum('mi,nj,ijkc,pc->kpmn', Ti, Tj, blk, Ta[l], optimize=True)
                    for k, o in enumerate(offs):
                        out[o:o + 2 * l + 1, a, b] = blk[k]
                        out[o:o + 2 * l + 1, b, a] = blk[k].transpose(0, 2, 1)
        nrm = self._norm
        out *= auxmol._norm[:, None, None] * nrm[None, :, None] * nrm[None, None, :]
        return out

    def int2c2e(self, omega: float = 0.0) -> np.ndarray:
        """(P|Q) of this (auxiliary) basis over normalised spherical functions
        (omega > 0: erf(omega r12)/r12)."""
        n = self._nao
        out = np.zeros((n, n))
        groups = self._aux_groups()
        for la, (sa, oa) in groups.items():
            for lb, (sb, ob) in groups.items():
                blk = eri2c(sa, sb, omega)                           # (ka, ca, kb, cb)
                blk = np.einsum('pa,kalc,qc->kplq', _sph_transform(la), blk, _sph_transform(lb),
                                optimize=True)
                for k, o1 in enumerate(oa):
                    for m, o2 in enumerate(ob):
                        out[o1:o1 + 2 * la + 1, o2:o2 + 2 * lb + 1] = blk[k, :, m, :]
        nrm = self._norm
        return out * (nrm[:, None] * nrm[None, :])

    def eri_full(self, device=None, omega: float = 0.0) -> np.ndarray:
        """(mu nu|la si) over normalised spherical AOs, all 8 symmetry copies filled.
        ``device=k``: evaluated on GPU k (``qc.dints``, the HIP integral kernel);
        ``omega > 0``: erf(omega r12)/r12 (the long-range ERIs of ``eri_lr``)."""
        if device is not None:
            from .dints import eri_full_device
            return eri_full_device(self, device, omega=omega)
        n = self._nao
        sh = self.shells
        nsh = len(sh)
        T = [_sph_transform(s.l) for s in sh]
        pairs = {}
        for i in range(nsh):
            for j in range(i + 1):
                pairs[(i, j)] = ShellPair(sh[i], sh[j])
        eri = np.zeros((n, n, n, n))
        keys = list(pairs)
        for ij, (i, j) in enumerate(keys):
            bra = pairs[(i, j)]
            for (k, l) in keys[:ij + 1]:
                ket = pairs[(k, l)]
                blk = eri_quartet(bra, ket, omega)
                blk = np.einsum('ai,bj,ijkl,ck,dl->abcd', T[i], T[j], blk, T[k], T[l], optimize=True)
                a = slice(self.ao_loc[i], self.ao_loc[i + 1])
                b = slice(self.ao_loc[j], self.ao_loc[j + 1])
                c = slice(self.ao_loc[k], self.ao_loc[k + 1])
                d = slice(self.ao_loc[l], self.ao_loc[l + 1])
                for (x, y, bx) in ((a, b, blk), (b, a, blk.transpose(1, 0, 2, 3))):
                    for (z, w, bz) in ((c, d, bx), (d, c, bx.transpose(0, 1, 3, 2))):
                        eri[x, y, z, w] = bz
                        eri[z, w, x, y] = bz.transpose(2, 3, 0, 1)
        nrm = self._norm
        eri *= (nrm[:, None, None, None] * nrm[None, :, None, None]
                * nrm[None, None, :, None] * nrm[None, None, None, :])
        return eri

    # ----------------------------------------------------- AO on the grid
    def eval_ao(self, coords: np.ndarray, deriv: int = 0, device=None):
        """AO values (deriv 0: (ngrid, nao)) or values + gradients (deriv 1: (4, ngrid, nao)).
        ``device=k``: evaluated on GPU k in grid blocks (``xt_eval_ao``), returned as a
        device tensor that stays in HBM."""
        if device is not None:
            from .dints import eval_ao_device
            return eval_ao_device(self, coords, deriv, device)
        coords = np.asarray(coords, dtype=np.float64)
        ng = coords.shape[0]
        ncomp = 4 if deriv else 1
        out = np.empty((ncomp, ng, self._nao))
        for s, p0, p1 in zip(self.shells, self.ao_loc[:-1], self.ao_loc[1:]):
            d = coords - s.center
            r2 = np.einsum('gx,gx->g', d, d)
            ex = np.exp(-np.outer(r2, s.exps))            # (ng, nprim)
            g0 = ex @ s.coefs
            comps = cart_comps(s.l)
            cart = np.empty((ncomp, ng, len(comps)))
            if deriv:
                g1 = ex @ (-2.0 * s.exps * s.coefs)         # d/d(r^2) part: grad = g1 * d
            for c, (ix, iy, iz) in enumerate(comps):
                poly = d[:, 0] ** ix * d[:, 1] ** iy * d[:, 2] ** iz
                cart[0, :, c] = poly * g0
                if deriv:
                    for k, e in enumerate((ix, iy, iz)):
                        if e > 0:
                            pe = list((ix, iy, iz))
                            pe[k] -= 1
                            dpoly = e * d[:, 0] ** pe[0] * d[:, 1] ** pe[1] * d[:, 2] ** pe[2]
                        else:
                            dpoly = 0.0
                        cart[1 + k, :, c] = dpoly * g0 + poly * d[:, k] * g1
            T = _sph_transform(s.l)
            out[:, :, p0:p1] = np.einsum('xgc,mc->xgm', cart, T) * self._norm[p0:p1]
        return out if deriv else out[0]


def M(atom, basis="6-31G", charge=0, spin=0, unit="Angstrom", symmetry=False, verbose=0) -> Mole:
    """``gto.M`` equivalent."""
    return Mole(atom, basis=basis, charge=charge, spin=spin, unit=unit, symmetry=symmetry,
                verbose=verbose)


def chiral_mol(mol, tol: float = 1e-4) -> bool:
    """``pyscf.gto.mole.chiral_mol(mol)``: True when the molecule cannot be
    superimposed on its mirror image by a proper rotation (XTDA.py:818 gates the
    rotatory strengths on it).

    Mirror = reflection z -> -z about the charge centroid.  Candidate rotations
    come from Kabsch fits of one non-collinear reference triple of the mirror
    onto every charge- and distance-compatible triple of the original; the
    molecule is achiral if one of them maps every atom onto an atom of equal
    charge.  Linear and planar molecules are achiral outright.
    """
    x = np.asarray(mol.atom_coords(), dtype=np.float64)
    z = np.asarray(mol.atom_charges())
    n = len(z)
    if n < 4:
        return False
    x = x - (z[:, None] * x).sum(0) / z.sum()
    if np.linalg.svd(x, compute_uv=False)[-1] < tol * max(1.0, np.abs(x).max()):
        return False                       # planar (or linear): the plane is a mirror
    y = x * np.array([1.0, 1.0, -1.0])
    dx = np.linalg.norm(x[:, None] - x[None], axis=-1)
    # reference triple of the mirror: atoms 0, the farthest from it, then the one
    # farthest from their line (non-collinear)
    i0 = 0
    i1 = int(np.argmax(dx[i0]))
    u = (y[i1] - y[i0]) / np.linalg.norm(y[i1] - y[i0])
    off = y - y[i0] - np.outer((y - y[i0]) @ u, u)
    i2 = int(np.argmax(np.linalg.norm(off, axis=1)))
    ref = [i0, i1, i2]
    dref = dx[np.ix_(ref, ref)]          # mirror distances equal the original's

    def kabsch(p, q):                      # proper rotation R with R p ~ q
        h = p.T @ q
        uu, _, vt = np.linalg.svd(h)
        d = np.sign(np.linalg.det(vt.T @ uu.T))
        return vt.T @ np.diag([1.0, 1.0, d]) @ uu.T

    for a in np.where(z == z[i0])[0]:
        for b in np.where((z == z[i1]) & (np.abs(dx[a] - dref[0, 1]) < 1e-3))[0]:
            for c in np.where((z == z[i2]) & (np.abs(dx[a] - dref[0, 2]) < 1e-3)
                              & (np.abs(dx[b] - dref[1, 2]) < 1e-3))[0]:
                r = kabsch(y[ref], x[[a, b, c]])
                yr = y @ r.T
                d = np.linalg.norm(yr[:, None] - x[None], axis=-1)
                d[z[:, None] != z[None, :]] = np.inf
                if np.all(d.min(axis=1) < 1e-3):
                    return False
    return True
