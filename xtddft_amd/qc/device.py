"""SCF potentials on the GPU: the mean field's J/K and XC through the library's
FP64-MFMA GEMM (``xt_dgemm``, the contraction engine of the hot path) with the
DF factor and the grid resident in HBM ("ROKS/UKS SCF
driver reusing the HIP J/K + XC kernels").

* J[D] = sum_P B_P <B_P, D>: two GEMMs over the pair index;
* K[D] = sum_P B_P D B_P: T = B^(mP) D then K = T B over (P, l) -- two GEMMs on
  the factor kept in both (P, m, l) and (m, P, l) layouts;
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
        else:   # exact ERIs: their pivoted Cholesky factor is an exact "DF" factor
            from .scf import pivoted_cholesky
            b = pivoted_cholesky(mf.eri.reshape(n * n, n * n), 1e-14).reshape(-1, n, n)
        self.naux = b.shape[0]
        self.B = torch.as_tensor(np.ascontiguousarray(b), device=self.dev)              # (P, m, l)
        self.Bt = self.B.permute(1, 0, 2).contiguous()                                  # (m, P, l)
        if mf.xctype != "HF":
            self.ao = torch.as_tensor(np.ascontiguousarray(mf.ao), device=self.dev)      # (ncomp, G, n)
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
    def get_jk(self, dms, with_j=True, with_k=True):
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
            out = []
            for x in range(dt.shape[0]):
                t = self._mm(self.Bt.reshape(n * P, n), dt[x])               # [(m, P), l] = (B_P D)[m, l]
                out.append(self._mm(t.reshape(n, P * n), self.B.reshape(P * n, n)))
            vk = torch.stack(out).reshape(shape).cpu().numpy()
        return vj, vk

    # ------------------------------------------------------------ XC
    def _rho(self, dm):
        """(ncomp, G) density and gradient of a symmetric density matrix."""
        ao = self.ao
        c0 = self._mm(ao[0], dm)
        rho = [(ao[0] * c0).sum(1)]
        for k in range(1, ao.shape[0]):
            rho.append(2.0 * (ao[k] * c0).sum(1))
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
            if self.xctype == "GGA":
                wv = wv.clone()
                wv[0] *= 0.5
                aow = (wv[:, :, None] * ao).sum(0)
                v = self._mm(ao[0], aow, ta=1)
                vm.append(v + v.T)
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
