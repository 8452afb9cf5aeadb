// 3-index Coulomb integrals (ab|c) over contracted Cartesian Gaussians on the GPU,
// by the McMurchie-Davidson scheme: the DF integrals behind the mean field's
// density-fitting factor (PySCF df.incore.aux_e2 'int3c2e', the factor whose
// get_jk XTDA.py:518-543 calls and whose MO transform replaces ao2mo.general,
// XTDA.py:120).  The host restatement is xtddft_amd/qc/ints.py:eri3c.
//
//   (ab|c) = sum_{q in pair prims} sum_{r in aux prims} 2 pi^2.5 / (p s sqrt(p + s))
//            sum_{t in tuv(la+lb)} E^{ab}_t(q) sum_{u in tuv(lc)} (-1)^{|u|} E^c_u(r) R_{t+u}(alpha, P_q - C_r)
//
// The Hermite expansion coefficients E (contraction coefficients folded in) are
// per shell pair / aux shell and cheap: the caller prepares them.  This kernel does
// the quartic part -- Boys functions, the Hermite integrals R_tuv by the downward
// recursion, and the two contractions -- one thread per (shell pair, aux shell),
// the R table in private memory.  Not a hot-path kernel (once per mean field).
// omega > 0 evaluates the long-range operator erf(omega r12)/r12 instead (the
// range-separated exchange factors; qc/ints.py _attenuate).
#include <hip/hip_runtime.h>
#include <math.h>
#include "xt_internal.h"

namespace xt {

constexpr int I3_MAXLAB = 4;                   // d shells on the orbital side
constexpr int I3_MAXLC = 6;                    // auxiliary shells up to i (ket pairs up to d d)
constexpr int I3_MAXL = I3_MAXLAB + I3_MAXLC;
constexpr int I3_NTUV = (I3_MAXL + 1) * (I3_MAXL + 2) * (I3_MAXL + 3) / 6;
constexpr int I3_NTAB = (I3_MAXLAB + 1) * (I3_MAXLAB + 2) * (I3_MAXLAB + 3) / 6;

__host__ __device__ inline int ntuv(int L) { return (L + 1) * (L + 2) * (L + 3) / 6; }
__host__ __device__ inline int ncart(int l) { return (l + 1) * (l + 2) / 2; }
// position of (t, u, v) in the order of qc/ints.py hermite_index: by n = t + u + v,
// then t descending, then u descending
__device__ inline int tuv_pos(int t, int u, int v) {
  const int n = t + u + v, d = n - t;
  return n * (n + 1) * (n + 2) / 6 + d * (d + 1) / 2 + (d - u);
}

// F_n(T), n = 0..m: the series for F_m and downward recursion below T = 30 (all
// terms positive, no cancellation), F_0 = sqrt(pi/T) erf(sqrt T) / 2 and upward
// recursion above (e^-T <= 1e-13 against (2n+1) F_n: stable)
__device__ void boys_all(int m, double T, double* F) {
  if (T < 30.0) {
    double term = 1.0 / (2 * m + 1), sum = term;
    for (int k = 1; k < 400; ++k) {
      term *= 2.0 * T / (2 * m + 2 * k + 1);
      sum += term;
      if (term < 1e-17 * sum) break;
    }
    const double et = exp(-T);
    F[m] = et * sum;
    for (int n = m - 1; n >= 0; --n) F[n] = (2.0 * T * F[n + 1] + et) / (2 * n + 1);
  } else {
    const double et = exp(-T);
    F[0] = 0.5 * sqrt(M_PI / T) * erf(sqrt(T));
    for (int n = 0; n < m; ++n) F[n + 1] = ((2 * n + 1) * F[n] - et) / (2.0 * T);
  }
}

// R^0_tuv(alpha, X, Y, Z) for all t + u + v <= L (qc/ints.py hermite_r)
__device__ void hermite_r(int L, double alpha, double X, double Y, double Z, double* R, double* S) {
  double F[I3_MAXL + 1];
  boys_all(L, alpha * (X * X + Y * Y + Z * Z), F);
  const double m2a = -2.0 * alpha;
  double pw = 1.0;
  for (int n = 0; n < L; ++n) pw *= m2a;
  double* prev = R;
  double* cur = S;
  if (L % 2) { prev = S; cur = R; }           // the last level (n = 0) lands in R
  prev[0] = pw * F[L];
  for (int n = L - 1; n >= 0; --n) {
    pw /= m2a;
    cur[0] = pw * F[n];
    for (int tot = 1; tot <= L - n; ++tot)
      for (int t = tot; t >= 0; --t)
        for (int u = tot - t; u >= 0; --u) {
          const int v = tot - t - u;
          double val;
          if (t > 0) {
            val = X * prev[tuv_pos(t - 1, u, v)];
            if (t > 1) val += (t - 1) * prev[tuv_pos(t - 2, u, v)];
          } else if (u > 0) {
            val = Y * prev[tuv_pos(0, u - 1, v)];
            if (u > 1) val += (u - 1) * prev[tuv_pos(0, u - 2, v)];
          } else {
            val = Z * prev[tuv_pos(0, 0, v - 1)];
            if (v > 1) val += (v - 1) * prev[tuv_pos(0, 0, v - 2)];
          }
          cur[tuv_pos(t, u, v)] = val;
        }
    double* tmp = prev; prev = cur; cur = tmp;
  }
}

// pair_info[8 k + .]: la, lb, npp, prim0, e0, row0;  pair_prim[4 q + .]: p, Px, Py, Pz
// aux_info[8 j + .]:  lc, nprim, prim0, e0, col0, nc; aux_prim[4 r + .]:  s, Cx, Cy, Cz
// eab (pair k): [a][b][t][q] over ncart(la) x ncart(lb) x ntuv(la+lb) x npp
// ek (aux j):   [c][u][r]    over nc x ntuv(lc) x nprim
// The ket may be a shell pair too (4-index (ab|cd)): lc = l_c + l_d, nc = ncart(l_c)
// ncart(l_d) components, its primitive pairs and Hermite coefficients as the bra's.
__global__ void __launch_bounds__(64)
k_int3c2e_cart(int npair, const int* __restrict__ pair_info, const double* __restrict__ pair_prim,
               const double* __restrict__ eab, int naux, const int* __restrict__ aux_info,
               const double* __restrict__ aux_prim, const double* __restrict__ ek,
               double* __restrict__ out, long ldo, double omega) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)npair * naux) return;
  const int k = (int)(id / naux), j = (int)(id % naux);
  const int* pi = pair_info + 8 * k;
  const int* ai = aux_info + 8 * j;
  const int la = pi[0], lb = pi[1], npp = pi[2], pq0 = pi[3], pe0 = pi[4], row0 = pi[5];
  const int lc = ai[0], nr = ai[1], ar0 = ai[2], ae0 = ai[3], col0 = ai[4];
  const int lab = la + lb, L = lab + lc;
  const int nab = ncart(la) * ncart(lb), ntab = ntuv(lab), nc = ai[5], ntc = ntuv(lc);
  double R[I3_NTUV], S[I3_NTUV], M[I3_NTAB];
  for (int q = 0; q < npp; ++q) {
    const double* pp = pair_prim + 4 * (long)(pq0 + q);
    const double p = pp[0];
    for (int r = 0; r < nr; ++r) {
      const double* cp = aux_prim + 4 * (long)(ar0 + r);
      const double s = cp[0];
      double alpha = p * s / (p + s), scale = 1.0;
      if (omega > 0.0) {   // erf(omega r)/r: 1/a' = 1/alpha + 1/omega^2, times sqrt(a'/alpha)
        const double w2 = omega * omega, a2 = alpha * w2 / (alpha + w2);
        scale = sqrt(a2 / alpha);
        alpha = a2;
      }
      hermite_r(L, alpha, pp[1] - cp[1], pp[2] - cp[2], pp[3] - cp[3], R, S);
      const double pref = 2.0 * pow(M_PI, 2.5) / (p * s * sqrt(p + s)) * scale;
      for (int c = 0; c < nc; ++c) {
        // M[t] = sum_u (-1)^{|u|} E^c_u(r) R[t + u]
        const double* e = ek + ae0 + ((long)c * ntc) * nr + r;
        for (int it = 0; it < ntab; ++it) M[it] = 0.0;
        int iu = 0;
        for (int nu = 0; nu <= lc; ++nu)
          for (int tu = nu; tu >= 0; --tu)
            for (int uu = nu - tu; uu >= 0; --uu, ++iu) {
              const int vu = nu - tu - uu;
              const double w = ((nu & 1) ? -1.0 : 1.0) * e[(long)iu * nr];
              if (w == 0.0) continue;
              int it = 0;
              for (int nt = 0; nt <= lab; ++nt)
                for (int tt = nt; tt >= 0; --tt)
                  for (int ut = nt - tt; ut >= 0; --ut, ++it)
                    M[it] += w * R[tuv_pos(tt + tu, ut + uu, nt - tt - ut + vu)];
            }
        for (int ab = 0; ab < nab; ++ab) {
          const double* ea = eab + pe0 + ((long)ab * ntab) * npp + q;
          double acc = 0.0;
          for (int it = 0; it < ntab; ++it) acc += ea[(long)it * npp] * M[it];
          out[(long)(row0 + ab) * ldo + col0 + c] += pref * acc;
        }
      }
    }
  }
}

int int3c2e_cart(int npair, const int* pair_info, const double* pair_prim, const double* eab, int naux_shells,
                 const int* aux_info, const double* aux_prim, const double* ek, double* out, long ldo,
                 double omega, hipStream_t st) {
  const long n = (long)npair * naux_shells;
  if (n == 0) return 0;
  const int blk = 64;
  hipLaunchKernelGGL(k_int3c2e_cart, dim3((unsigned)((n + blk - 1) / blk)), dim3(blk), 0, st, npair, pair_info,
                     pair_prim, eab, naux_shells, aux_info, aux_prim, ek, out, ldo, omega);
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
