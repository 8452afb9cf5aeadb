"""SCF potentials on the GPU: the mean field's J/K and XC through the library's
FP64-MFMA GEMM (``xt_dgemm``, the contraction engine of the hot path) with the
DF factor and the grid resident in HBM ("ROKS/UKS SCF
driver reusing the HIP J/K + XC kernels").

* J[D] = sum_P B_P <B_P, D>: two GEMMs over the pair index;
* K[D] = sum_P B_P D B_P for a symmetric D = V diag(lam) V^T (host eigh of the
  small density, |lam| > 1e-14 kept -- the occupied factorisation gpu4pyscf's
  tagged densities give, XTDA_GPU.py:232): T = B V (one GEMM), then
  K = T' diag(lam) T'^T over (P, i) (one GEMM), 2 naux nao^2 rank x 2 flop instead
  of 4 naux nao^3; a non-symmetric D takes the plain B D B route;
* the factor is the DF factor, the device integral-direct Cholesky factor of the
  exact ERIs (``qc.dchol``, already in HBM), or the pivoted Cholesky of stored
  ERIs (small molecules);
* rho, grad rho from C = Phi_0 D (GEMM) and row dots; V_xc = Phi_0^T (sum_y wv_y
  Phi_y) (+ transpose for GGA) as GEMMs; the functional and its first / second
  derivatives (vxc, the cached fxc of ``cache_xc_kernel``, XTDA.py:504, and the
  ALDA0 kernel of ``cache_xc_kernel_sf``, SF_TDA.py:39-88) by autograd on the
  device (``xc.eval_xc_eff_torch``).

The host SCF (``scf.py``) delegates to this engine after ``mf.to_device()``;
results equal the host path to round-off (tests/test_gpu_qc.py).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _capi
from . import xc as _xc


class DeviceEngine:
    def __init__(self, mf, device: int = 0):
        import torch
        self.torch = torch
        self.dev = torch.device(f"cuda:{device}")
        self.L = _capi.lib()
        self.xc = mf.xc
        self.xctype = mf.xctype
        n = mf.mol.nao
        self.n = n
        if mf.with_df is not None:
            b = np.asarray(mf.with_df.cderi)
        elif getattr(mf, "cderi_exact", None) is not None:
            b = mf.cderi_exact                 # device tensor from qc.dchol
        else:   # stored exact ERIs: their pivoted Cholesky factor is an exact "DF" factor
            from .scf import pivoted_cholesky
            b = pivoted_cholesky(mf.eri.reshape(n * n, n * n), 1e-14).reshape(-1, n, n)
        self.naux = b.shape[0]
        self.B = b.to(self.dev).contiguous() if isinstance(b, torch.Tensor) else \
            torch.as_tensor(np.ascontiguousarray(b), device=self.dev)                    # (P, m, l)
        # range-separated hybrids: the long-range factor of the same route (K_LR only)
        self.B_lr = None
        if getattr(mf, "omega", 0.0) != 0:
            if mf.with_df is not None:
                bl = np.asarray(mf.with_df.cderi_lr(mf.omega))
            elif getattr(mf, "cderi_exact_lr", None) is not None:
                bl = mf.cderi_exact_lr
            else:
                from .scf import pivoted_cholesky
                bl = pivoted_cholesky(mf.eri_lr.reshape(n * n, n * n), 1e-14).reshape(-1, n, n)
            self.B_lr = bl.to(self.dev).contiguous() if isinstance(bl, torch.Tensor) else \
                torch.as_tensor(np.ascontiguousarray(bl), device=self.dev)
        if mf.xctype != "HF":
            ao = mf.ao
            self.ao = ao.to(self.dev) if isinstance(ao, torch.Tensor) else \
                torch.as_tensor(np.ascontiguousarray(ao), device=self.dev)               # (ncomp, G, n)
            self.w = torch.as_tensor(np.ascontiguousarray(mf.grids.weights), device=self.dev)

    # ------------------------------------------------------------ GEMM
    def _gemm(self, ta, tb, m, n, k, alpha, a, lda, b, ldb, beta, c, ldc):
        st = self.torch.cuda.current_stream(self.dev).cuda_stream
        with self.torch.cuda.device(self.dev):
            _capi.check(self.L.xt_dgemm(ta, tb, m, n, k, alpha, a.data_ptr(), lda, b.data_ptr(), ldb,
                                        beta, c.data_ptr(), ldc, ctypes.c_void_p(st)), "xt_dgemm")

    def _mm(self, a, b, ta=0, tb=0):
        """op(a) @ op(b) for 2-D contiguous device tensors."""
        m = a.shape[1] if ta else a.shape[0]
        k = a.shape[0] if ta else a.shape[1]
        n = b.shape[0] if tb else b.shape[1]
        c = self.torch.empty((m, n), dtype=self.torch.float64, device=self.dev)
        self._gemm(ta, tb, m, n, k, 1.0, a, a.shape[1], b, b.shape[1], 0.0, c, n)
        return c

    # ------------------------------------------------------------ J / K
    def get_jk(self, dms, with_j=True, with_k=True, factors=None):
        """J / K of densities dms; ``factors`` (C_s with dms[s] = C_s C_s^T, from the SCF's
        orbitals) lets K skip the eigendecomposition of each density."""
        torch = self.torch
        d = np.asarray(dms, dtype=np.float64)
        shape = d.shape
        n, P = self.n, self.naux
        dt = torch.as_tensor(np.ascontiguousarray(d.reshape(-1, n, n)), device=self.dev)
        vj = vk = None
        if with_j:
            b2 = self.B.reshape(P, n * n)
            gam = self._mm(b2, dt.reshape(-1, n * n), tb=1)                  # (P, nset)
            vj = self._mm(gam, b2, ta=1).reshape(shape).cpu().numpy()        # (nset, n^2)
        if with_k:
            if factors is not None and len(factors) == dt.shape[0]:
                vk = np.stack([self._k_factor(np.asarray(f, dtype=np.float64)) for f in factors]).reshape(shape)
            else:
                vk = np.stack([self._k(d.reshape(-1, n, n)[x], dt[x]) for x in range(dt.shape[0])]).reshape(shape)
        return vj, vk

    def _k_factor(self, c, B=None):
        """K[C C^T] = sum_P (B_P C)(B_P C)^T."""
        torch = self.torch
        B = self.B if B is None else B
        n, P = self.n, B.shape[0]
        r = c.shape[1]
        if r == 0:
            return np.zeros((n, n))
        vt = torch.as_tensor(np.ascontiguousarray(c), device=self.dev)
        t = self._mm(B.reshape(P * n, n), vt).reshape(P, n, r)             # T_P = B_P C
        return self._reduce_p(t, t, nt=True).cpu().numpy()                 # sum_P T_P T_P^T

    def get_k(self, dms, lr=False, factors=None):
        """K[D] (lr: the long-range K_LR[D]) for each density of dms (``factors`` as in
        get_jk)."""
        d = np.asarray(dms, dtype=np.float64)
        B = self.B_lr if lr else self.B
        if B is None:
            raise ValueError("no long-range factor: the functional is not range-separated")
        if factors is not None and len(factors) == d.reshape(-1, self.n, self.n).shape[0]:
            return np.stack([self._k_factor(np.asarray(f, dtype=np.float64), B) for f in factors]).reshape(d.shape)
        dt = self.torch.as_tensor(np.ascontiguousarray(d.reshape(-1, self.n, self.n)), device=self.dev)
        return np.stack([self._k(d.reshape(-1, self.n, self.n)[x], dt[x], B) for x in range(dt.shape[0])]
                        ).reshape(d.shape)

    def _reduce_p(self, t, b, nt):
        """sum_P op(t_P) b_P for slabs t (P, n, k) and b (P, k, n) or, with nt, b (P, n, k)
        transposed: one engine GEMM whose reduce index is P (``xt_dgemm_strided``) --
        no (n, P k) re-layout copy, and no row stride P k (which the engine's 32-bit
        tile addressing caps near 2M at large aux counts)."""
        torch = self.torch
        P, m, k = t.shape
        n = b.shape[1] if nt else b.shape[2]
        c = torch.empty((m, n), dtype=torch.float64, device=self.dev)
        sbk, sbn = (1, k) if nt else (n, 1)
        st = torch.cuda.current_stream(self.dev).cuda_stream
        with torch.cuda.device(self.dev):
            _capi.check(self.L.xt_dgemm_strided(m, n, k, P, 1, 1.0, t.data_ptr(), k, 1, m * k, 0,
                                                b.data_ptr(), sbk, sbn, b.shape[1] * b.shape[2], 0, 0.0,
                                                c.data_ptr(), n, 0, ctypes.c_void_p(st)), "xt_dgemm_strided")
        return c

    def _k(self, dh, dd, B=None):
        """K[D] (host array) for one density (dh host, dd the same on the device)."""
        torch = self.torch
        B = self.B if B is None else B
        n, P = self.n, B.shape[0]
        if np.abs(dh - dh.T).max() <= 1e-14 * max(1.0, np.abs(dh).max()):
            lam, v = np.linalg.eigh(0.5 * (dh + dh.T))
            keep = np.abs(lam) > 1e-14 * max(1.0, np.abs(lam).max())
            r = int(keep.sum())
            if r == 0:
                return np.zeros((n, n))
            vt = torch.as_tensor(np.ascontiguousarray(v[:, keep]), device=self.dev)
            t = self._mm(B.reshape(P * n, n), vt).reshape(P, n, r)       # T_P = B_P V
            ts = t * torch.as_tensor(lam[keep], device=self.dev)
            return self._reduce_p(t, ts, nt=True).cpu().numpy()          # sum_P T_P lam T_P^T
        t = self._mm(B.reshape(P * n, n), dd).reshape(P, n, n)           # B_P D
        return self._reduce_p(t, B, nt=False).cpu().numpy()              # sum_P B_P D B_P

    # ------------------------------------------------------------ XC
    def _rho(self, dm):
        """(ncomp, G) density and gradient (MGGA: + tau) of a symmetric density matrix."""
        ao = self.ao
        c0 = self._mm(ao[0], dm)
        rho = [(ao[0] * c0).sum(1)]
        for k in range(1, ao.shape[0]):
            rho.append(2.0 * (ao[k] * c0).sum(1))
        if self.xctype == "MGGA":
            rho.append(0.5 * sum((ao[k] * self._mm(ao[k], dm)).sum(1) for k in range(1, 4)))
        return self.torch.stack(rho)

    def rho(self, dms):
        torch = self.torch
        d = torch.as_tensor(np.ascontiguousarray(np.asarray(dms, dtype=np.float64)), device=self.dev)
        return torch.stack([self._rho(d[0]), self._rho(d[1])])

    def vxc(self, dms):
        """(E_xc[DFT], V_xc (2, nao, nao)) at spin densities dms (host SCF's _vxc)."""
        torch = self.torch
        rho = self.rho(dms)
        exc, vxc, _ = _xc.eval_xc_eff_torch(self.xc, rho, deriv=1)
        e = float((self.w * exc * (rho[0, 0] + rho[1, 0])).sum())
        ao = self.ao
        vm = []
        for s in range(2):
            wv = vxc[s] * self.w
            if self.xctype in ("GGA", "MGGA"):
                wv = wv.clone()
                wv[0] *= 0.5
                aow = (wv[:4, :, None] * ao[:4]).sum(0)
                v = self._mm(ao[0], aow, ta=1)
                v = v + v.T
                if self.xctype == "MGGA":     # tau part: 1/2 sum_c grad_c phi^T w_tau grad_c phi
                    for k in range(1, 4):
                        v = v + 0.5 * self._mm(ao[k], (wv[4][:, None] * ao[k]).contiguous(), ta=1)
                vm.append(v)
            else:
                vm.append(self._mm(ao[0], (wv[0][:, None] * ao[0]).contiguous(), ta=1))
        return e, torch.stack(vm).cpu().numpy()

    def kernels(self, dms):
        """(fxc (2, ncomp, 2, ncomp, G), ALDA0 fxc_ab (G)) at the SCF density:
        cache_xc_kernel (XTDA.py:504) and cache_xc_kernel_sf (SF_TDA.py:69-85)."""
        rho = self.rho(dms)
        fxc = _xc.eval_xc_eff_torch(self.xc, rho, deriv=2)[2]
        rho0 = self.torch.zeros_like(rho)
        rho0[:, 0] = rho[:, 0]
        vxc0 = _xc.eval_xc_eff_torch(self.xc, rho0, deriv=1)[1]
        fxc_sf = (vxc0[0, 0] * self.w - vxc0[1, 0] * self.w) / (rho[0, 0] - rho[1, 0] + 1e-9)
        return fxc.cpu().numpy(), fxc_sf.cpu().numpy()
