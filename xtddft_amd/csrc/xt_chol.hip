// Pivoted Cholesky of the 8-fold packed ERI supermatrix (jk_mode ERI8).
//
//   V[(mu nu), (la si)] = (mu nu|la si),  V = sum_P L_P L_P^T  (P < rank)
//
// The reference consumes stored ERIs through PySCF get_jk (incore mf._eri,
// 's8' packing, XTDA.py:518-543).  Here the supermatrix is factorised once
// per solve so the stored-ERI mode reuses the MO-route DF engine: the
// Cholesky vectors L_P, unpacked to symmetric nao x nao matrices, are an
// exact (to the pivot tolerance) "DF factor".
//
// Packing (PySCF ao2mo 's8'): pair ij = i(i+1)/2 + j (i >= j); element
// (ij|kl) at ij(ij+1)/2 + kl (ij >= kl).  L is stored row-major by vector:
// Lt[t * ldL + ij], so the per-pivot update streams coalesced rows.
// Memory bound: step k reads k rows of npair doubles (HBM / L2 streaming).

#include <hip/hip_runtime.h>
#include "xt_kernels.h"

namespace xt {

__device__ __forceinline__ long s8_index(long ij, long kl) {
  const long a = ij > kl ? ij : kl, b = ij > kl ? kl : ij;
  return a * (a + 1) / 2 + b;
}

__global__ void k_eri_diag(long npair, const double* __restrict__ eri, double* __restrict__ d) {
  for (long ij = blockIdx.x * (long)blockDim.x + threadIdx.x; ij < npair; ij += (long)gridDim.x * blockDim.x)
    d[ij] = eri[s8_index(ij, ij)];
}

// out[0] = max_i d[i], out[1] = its smallest index (as a double): deterministic pivots.
__global__ void __launch_bounds__(1024) k_argmax(long n, const double* __restrict__ d, double* __restrict__ out) {
  __shared__ double sv[1024];
  __shared__ long si[1024];
  double bv = -1.0;
  long bi = 0;
  for (long i = threadIdx.x; i < n; i += blockDim.x) {
    const double v = d[i];
    if (v > bv) { bv = v; bi = i; }
  }
  sv[threadIdx.x] = bv; si[threadIdx.x] = bi;
  __syncthreads();
  for (int off = blockDim.x / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      const double v = sv[threadIdx.x + off];
      const long i = si[threadIdx.x + off];
      if (v > sv[threadIdx.x] || (v == sv[threadIdx.x] && i < si[threadIdx.x])) {
        sv[threadIdx.x] = v; si[threadIdx.x] = i;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = sv[0]; out[1] = (double)si[0]; }
}

// New vector k for pivot p (residual diagonal dp = d[p]):
//   L_k = (V[:, p] - sum_{t<k} L_t L_t[p]) / sqrt(dp);  d -= L_k^2;  d[p] = 0
__global__ void k_chol_step(long npair, int k, long p, double inv_sqrt_dp, const double* __restrict__ eri,
                            double* __restrict__ Lt, long ldL, double* __restrict__ d) {
  for (long ij = blockIdx.x * (long)blockDim.x + threadIdx.x; ij < npair; ij += (long)gridDim.x * blockDim.x) {
    double s0 = eri[s8_index(ij, p)], s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int t = 0;
    for (; t + 4 <= k; t += 4) {
      s0 -= Lt[(long)t * ldL + ij] * Lt[(long)t * ldL + p];
      s1 -= Lt[(long)(t + 1) * ldL + ij] * Lt[(long)(t + 1) * ldL + p];
      s2 -= Lt[(long)(t + 2) * ldL + ij] * Lt[(long)(t + 2) * ldL + p];
      s3 -= Lt[(long)(t + 3) * ldL + ij] * Lt[(long)(t + 3) * ldL + p];
    }
    for (; t < k; ++t) s0 -= Lt[(long)t * ldL + ij] * Lt[(long)t * ldL + p];
    const double l = ((s0 + s1) + (s2 + s3)) * inv_sqrt_dp;
    Lt[(long)k * ldL + ij] = l;
    d[ij] = (ij == p) ? 0.0 : d[ij] - l * l;
  }
}

// B[P][mu][nu] = L_{p0+P}[pair(mu, nu)]  (symmetric fill), P < np
__global__ void k_chol_unpack(int np, int p0, int nao, const double* __restrict__ Lt, long ldL,
                              double* __restrict__ B) {
  const long aa = (long)nao * nao;
  const long total = (long)np * aa;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int P = (int)(idx / aa);
    const long e = idx - P * aa;
    const int mu = (int)(e / nao), nu = (int)(e - (long)mu * nao);
    const long i = mu > nu ? mu : nu, j = mu > nu ? nu : mu;
    B[idx] = Lt[(long)(p0 + P) * ldL + i * (i + 1) / 2 + j];
  }
}

static int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

void eri_diag(hipStream_t st, long npair, const double* eri, double* d) {
  hipLaunchKernelGGL(k_eri_diag, dim3(grid_for(npair)), dim3(256), 0, st, npair, eri, d);
}
void argmax(hipStream_t st, long n, const double* d, double* out2) {
  hipLaunchKernelGGL(k_argmax, dim3(1), dim3(1024), 0, st, n, d, out2);
}
void chol_step(hipStream_t st, long npair, int k, long p, double dp, const double* eri, double* Lt, long ldL,
               double* d) {
  hipLaunchKernelGGL(k_chol_step, dim3(grid_for(npair)), dim3(256), 0, st, npair, k, p, 1.0 / sqrt(dp), eri,
                     Lt, ldL, d);
}
void chol_unpack(hipStream_t st, int np, int p0, int nao, const double* Lt, long ldL, double* B) {
  hipLaunchKernelGGL(k_chol_unpack, dim3(grid_for((long)np * nao * nao)), dim3(256), 0, st, np, p0, nao, Lt,
                     ldL, B);
}

}  // namespace xt
