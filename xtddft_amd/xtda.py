"""X-TDA / U-TDA driver with the reference's API (``xtddft/XTDA.py``).

``XTDA(mol, mf, nstates=10, basis='orbital', so2st=True, use_Davidson=True)``
(XTDA.py:21-37) with ``kernel`` (39-54), ``gen_vind`` (694-698),
``get_init_guess`` (700-734), ``get_precond`` (736-744), ``Davidson``
(746-829), ``full_diag`` (explicit A, 56-450), ``deltaS2`` (831-836),
``osc_str`` (838-858) and ``analyze`` (893-937).

The operator behind ``gen_vind`` is the device ``DeviceOperator``
(MO-route FP64-MFMA A.x, xtddft_amd/csrc); the Davidson subspace lives in
HBM (``xtddft_amd.davidson``).  ``full_diag`` assembles A column-block by
column-block through the same device operator and diagonalises on the host.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

from . import davidson as _dav
from .meanfield import MeanField
from .operator import DeviceOperator
from .parallel import require_group
from .utils import HA2EV, EVXNM, nlc_check, order_pyscf2my, so2st as _so2st

CGS2AU = 1 / (235.7220 * 2)    # xtddft/utils/unit.py:9 (rotatory strength a.u. -> cgs)

# PySCF TDBase defaults the reference copies (XTDA.py:29-31)
CONV_TOL = 1e-5
LINDEP = 1e-12
MAX_CYCLE = 100


class XTDA:
    def __init__(self, mol, mf: MeanField, nstates=10, basis='orbital', so2st=True,
                 use_Davidson=True, device=0, shard=(0, 1)):
        self.mol = mol
        self.mf = mf
        self.nstates = nstates
        self.basis = basis
        self.so2st = so2st
        self.use_Davidson = use_Davidson
        self.conv_tol = CONV_TOL
        self.lindep = LINDEP
        self.max_cycle = MAX_CYCLE
        self.device = device
        self.shard = tuple(shard)
        require_group(self.shard[1])
        if not isinstance(mf, MeanField):
            raise ValueError("mf must be a ROKS or UKS mean field")
        self.X = bool(mf.is_rohf)
        self._op = None
        self.callback = None      # davidson1 callback, e.g. davidson.checkpoint(path)

    # ------------------------------------------------------------------ API
    def kernel(self):
        if self.basis == 'tensor':
            raise NotImplementedError("tensor-basis X_TDA (XTDA.py:947-1483) is outside the hot path")
        if self.basis != 'orbital':
            raise ValueError('basis must be tensor or orbital')
        nlc_check(self.mf, davidson_xtda=self.use_Davidson)
        if self.use_Davidson:
            return self.Davidson()
        return self.full_diag()

    def operator(self):
        if self._op is None:
            self._op = DeviceOperator(self.mf, 'XTDA' if self.X else 'UTDA', device=self.device,
                                      shard=self.shard)
        return self._op

    def _occ(self):
        mf = self.mf
        if self.X:
            occ = np.zeros((2, mf.mo_occ.size))
            occ[0][mf.mo_occ >= 1] = 1
            occ[1][mf.mo_occ >= 2] = 1
            mo_energy = (mf.mo_energy, mf.mo_energy)
        else:
            occ = mf.mo_occ
            mo_energy = (mf.mo_energy[0], mf.mo_energy[1])
        return occ, mo_energy

    def _hdiag(self):
        occ, mo_energy = self._occ()
        if self.X:   # Fock-diagonal gaps (XTDA.py:594-597)
            fa, fb = self.mf.fock_mo()
            ea, eb = fa.diagonal(), fb.diagonal()
        else:        # orbital-energy gaps (XTDA.py:599-600)
            ea, eb = mo_energy
        e_ia_a = ea[occ[0] == 0] - ea[occ[0] > 0, None]
        e_ia_b = eb[occ[1] == 0] - eb[occ[1] > 0, None]
        return np.hstack((e_ia_a.ravel(), e_ia_b.ravel()))

    def gen_vind(self, mf=None):
        """(vind, hdiag); vind(zs) -> A zs, zs (nz, dim) host array or CUDA tensor."""
        assert mf is None or mf is self.mf
        op = self.operator()

        def vind(zs):
            if isinstance(zs, (list, tuple)):
                zs = np.asarray(zs)
            return op.apply_full(zs)
        return vind, self._hdiag()

    def get_init_guess(self, mf=None, nstates=None, wfnsym=None, return_symmetry=False):
        if nstates is None:
            nstates = self.nstates
        occ, mo_energy = self._occ()
        e_ia_a = mo_energy[0][occ[0] == 0] - mo_energy[0][occ[0] > 0, None]
        e_ia_b = mo_energy[1][occ[1] == 0] - mo_energy[1][occ[1] > 0, None]
        nov = e_ia_a.size + e_ia_b.size
        nstates = min(nstates, nov)
        e_ia = np.append(e_ia_a.ravel(), e_ia_b.ravel())
        e_threshold = np.partition(e_ia, nstates - 1)[nstates - 1] + 0.001   # deg_eia_thresh
        idx = np.where(e_ia <= e_threshold)[0]
        x0 = np.zeros((idx.size, nov))
        x0[np.arange(idx.size), idx] = 1
        return x0

    def get_precond(self, hdiag):
        return _dav.DiagPrecond(hdiag, level_shift=self.mf.level_shift, device=self.device)

    def Davidson(self, x0=None, nstates=None):
        nstates = self.nstates if nstates is None else nstates
        vind, hdiag = self.gen_vind()
        precond = self.get_precond(hdiag)

        def pickeig(w, v, nroots, envs):
            idx = np.where(w > 0.001)[0]   # positive_eig_threshold
            return w[idx], v[:, idx], idx
        if x0 is None:
            x0 = self.get_init_guess(self.mf, nstates)
        self.converged, self.e, x1, self.icyc = _dav.davidson1(
            vind, x0, precond, tol_residual=self.conv_tol, lindep=self.lindep, nroots=nstates,
            pick=pickeig, max_cycle=self.max_cycle, device=self.device, callback=self.callback,
            lockstep=self.shard[1] > 1)
        info = self.mf.shape_info()
        nc, no, nv = info['nc'], info['no'], info['nv']
        v = np.asarray(x1).T
        self.nc, self.no, self.nv = nc, no, nv
        # ROKS and UKS alike: "my order" and Delta<S^2> (XTDA.py:796-815)
        self.order = order_pyscf2my(nc, no, nv)
        self.v = v[self.order, :]
        self._split_blocks()
        self.dS2 = self.deltaS2()
        return self.e

    def full_diag(self):
        """Explicit A (XTDA.full_diag) through the device operator, host eigh."""
        op = self.operator()
        dim = op.dim
        A = np.empty((dim, dim))
        blk = 256
        for j0 in range(0, dim, blk):
            j1 = min(dim, j0 + blk)
            eye = np.zeros((j1 - j0, dim))
            eye[np.arange(j1 - j0), np.arange(j0, j1)] = 1.0
            A[:, j0:j1] = op.apply_full(eye).T
        info = self.mf.shape_info()
        nc, no, nv = info['nc'], info['no'], info['nv']
        self.nc, self.no, self.nv = nc, no, nv
        self.order = order_pyscf2my(nc, no, nv)
        A = A[self.order][:, self.order]
        self.A = A
        e, v = scipy.linalg.eigh(A)
        self.e = e[:self.nstates]
        self.e_eV = self.e * HA2EV
        self.v = v[:, :self.nstates]
        self._split_blocks()
        self.dS2 = self.deltaS2()
        return self.e

    # ---------------------------------------------------------- properties
    def _split_blocks(self):
        nc, no, nv = self.nc, self.no, self.nv
        vt = self.v.T
        self.xycv_a = vt[:, :nc * nv]
        self.xyov_a = vt[:, nc * nv:(nc + no) * nv]
        self.xyco_b = vt[:, (nc + no) * nv:(nc + no) * nv + nc * no]
        self.xycv_b = vt[:, (nc + no) * nv + nc * no:]

    def deltaS2(self):
        """XTDA.deltaS2 (XTDA.py:831-836)."""
        return (np.einsum('ij,ij->i', self.xycv_a, self.xycv_a)
                + np.einsum('ij,ij->i', self.xycv_b, self.xycv_b)
                - 2 * np.einsum('ij,ij->i', self.xycv_a, self.xycv_b))

    def osc_str(self, dipole_ao=None):
        """Length-form oscillator strengths (XTDA.py:838-858).  ``dipole_ao``
        (3, nao, nao) defaults to ``mol.intor_symmetric('int1e_r', comp=3)`` (the
        reference's call, origin 0) when ``mol`` provides integrals."""
        if dipole_ao is None:
            mol = self.mol if hasattr(self.mol, "intor_symmetric") else self.mf.extra.get("qc_mol")
            if mol is None or not hasattr(mol, "intor_symmetric"):
                raise ValueError("osc_str needs AO dipole integrals: pass dipole_ao or a Mole with intor")
            dipole_ao = mol.intor_symmetric("int1e_r", comp=3)
        tdip = self._transition(dipole_ao)
        return 2. / 3. * np.einsum('s,sx,sx->s', self.e[:self.nstates], tdip, tdip)

    def _spin_orbitals(self):
        """(C_occ_a, C_vir_a, C_occ_b, C_vir_b): ROKS occupations >= 1 / >= 2
        (XTDA.py:807-810); UKS per-spin coefficients."""
        mf = self.mf
        if self.X:
            c = mf.mo_coeff
            return (c[:, mf.mo_occ >= 1], c[:, mf.mo_occ == 0], c[:, mf.mo_occ >= 2], c[:, mf.mo_occ != 2])
        ca, cb = mf.mo_coeff[0], mf.mo_coeff[1]
        oa, ob = mf.mo_occ[0], mf.mo_occ[1]
        return ca[:, oa > 0], ca[:, oa == 0], cb[:, ob > 0], cb[:, ob == 0]

    def _transition(self, op_ao):
        """<0|op|n> (n, 3) of a 3-component AO operator for the roots in self.v."""
        coa, cva, cob, cvb = self._spin_orbitals()
        a = np.einsum('xpq,pi,qj->xij', op_ao, coa, cva).reshape(3, -1)
        b = np.einsum('xpq,pi,qj->xij', op_ao, cob, cvb).reshape(3, -1)
        na = (self.nc + self.no) * self.nv
        b = b[:, self.order[na:] - na]
        vt = self.v.T
        return np.einsum('xi,yi->yx', a, vt[:, :na]) + np.einsum('xi,yi->yx', b, vt[:, na:])

    def _qc_mol(self):
        mol = self.mol if hasattr(self.mol, "intor") else self.mf.extra.get("qc_mol")
        if mol is None or not hasattr(mol, "intor"):
            raise ValueError("AO property integrals need a Mole with intor (xtddft_amd.qc)")
        return mol

    def rot_str(self, dip_ele_ao=None, dip_meg_ao=None):
        """Rotatory strengths (XTDA.py:860-891): velocity-form electric
        (``int1e_ipovlp``) and magnetic (``int1e_cg_irxp``, gauge origin 0)
        transition dipoles, R = sum_x (1/w) mu_x m_x in cgs units (the
        reference's ``unit.cgs2au``, Gaussian/ORCA convention)."""
        if dip_ele_ao is None or dip_meg_ao is None:
            mol = self._qc_mol()
            dip_ele_ao = mol.intor('int1e_ipovlp', comp=3, hermi=2)
            dip_meg_ao = mol.intor('int1e_cg_irxp', comp=3, hermi=2)
        ele = -self._transition(dip_ele_ao)
        meg = 0.5 * self._transition(dip_meg_ao)
        omega = self.e[:self.nstates]
        return np.einsum('s,sx,sx->s', 1.0 / omega, ele, meg) / CGS2AU

    def properties(self):
        """What XTDA.Davidson reports after the solve (XTDA.py:815-829): Delta<S^2>,
        oscillator strengths and, for chiral molecules only, rotatory strengths."""
        from .qc.gto import chiral_mol
        mol = self._qc_mol()
        self.os = self.osc_str()
        self.rs = self.rot_str() if chiral_mol(mol) else np.zeros(self.nstates)
        return self.dS2, self.os, self.rs

    def analyze(self, threshold=0.1, verbose=True):
        nc, nv, no = self.nc, self.nv, self.no
        vv = _so2st(self.v, nc, no, nv) if self.so2st else self.v
        lines = []
        tags = ('CV(0)', 'OV(0)', 'CO(0)', 'CV(1)') if self.so2st else ('CV(aa)', 'OV(aa)', 'CO(bb)', 'CV(bb)')
        for n in range(min(self.nstates, vv.shape[1])):
            val = vv[:, n]
            blocks = [val[:nc * nv].reshape(nc, nv), val[nc * nv:(nc + no) * nv].reshape(no, nv),
                      val[(nc + no) * nv:(nc + no) * nv + nc * no].reshape(nc, no),
                      val[(nc + no) * nv + nc * no:].reshape(nc, nv)]
            offs = [(0, nc + no), (nc, nc + no), (0, nc), (0, nc + no)]
            lines.append(f'D{n + 1}    w:{self.e[n] * HA2EV:10.4f} eV    d<S^2>:{self.dS2[n]:8.4f}')
            for tag, b, (oo, vo) in zip(tags, blocks, offs):
                for o, v in zip(*np.where(abs(b) > threshold)):
                    lines.append(f'    {tag} {o + 1 + oo:3d} -> {v + 1 + vo:3d}    c_i: {b[o, v]:8.5f}'
                                 f'    Per: {100 * b[o, v] ** 2:5.2f}%')
        if verbose:
            print("\n".join(lines))
        return lines
