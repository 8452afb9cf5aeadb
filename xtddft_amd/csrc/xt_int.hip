// Two-electron Coulomb integrals over contracted Cartesian Gaussians on the GPU, by
// the McMurchie-Davidson scheme, and the AO values / gradients on the DFT grid --
// the mean-field front end of SURVEY.md 8(f) row 1:
//
//  * (ab|c): the DF integrals behind the density-fitting factor (PySCF
//    df.incore.aux_e2 'int3c2e', the factor whose get_jk XTDA.py:518-543 calls and
//    whose MO transform replaces ao2mo.general, XTDA.py:120); host restatement
//    xtddft_amd/qc/ints.py:eri3c;
//  * (ab|cd): the ket given as shell pairs -- the exact ERIs of the direct-SCF mean
//    field (PySCF mol.intor('int2e')), as whole blocks, as the diagonal (ab|ab) or as
//    the pivot columns of the integral-direct Cholesky factorisation (qc/dchol.py);
//  * point charges as an s "auxiliary" of infinite exponent give the nuclear
//    attraction (int1e_nuc) through the same kernel;
//  * ao(g) and grad ao(g) (PySCF eval_ao / ni.block_loop, SF_TDA.py:63-68): one
//    thread per (grid point, shell).
//
//   (ab|c) = sum_{q in pair prims} sum_{r in ket prims} 2 pi^2.5 / (p s sqrt(p + s))
//            sum_{t in tuv(la+lb)} E^{ab}_t(q) sum_{u in tuv(lc)} (-1)^{|u|} E^c_u(r) R_{t+u}(alpha, P_q - C_r)
//
// The Hermite expansion coefficients E (contraction coefficients folded in) are
// per shell pair / ket shell and cheap: the caller prepares them.  The kernel does
// the quartic part -- Boys functions, the Hermite integrals R_tuv by the downward
// recursion, and the two contractions -- one thread per (bra pair, ket), the bra index
// fastest over pairs the caller orders by class (qc/dints.py PairTable), so a wave's
// quartets share their class.  Quartets with lab, lc <= 4 and L <= 6 (the contracted s /
// p shells, most primitive quartets) run compile-time (t, u, v) code with the R table in
// registers (quartet_cls); the rest keep it in private memory sized by the template
// bucket (total order L <= 8: d shells; L <= 13: f shells with auxiliary shells up to
// l = 7 or f f kets).
// Schwarz screening: with bounds q_bra / q_ket, a (bra, ket) block whose bound
// product is below q_thr is skipped (left as the caller's zeros).  Not a hot-path
// kernel (once per mean field).  omega > 0 evaluates the long-range operator
// erf(omega r12)/r12 instead (the range-separated exchange factors; qc/ints.py
// _attenuate).
#include <hip/hip_runtime.h>
#include <math.h>
#include <mutex>
#include "xt_internal.h"

namespace xt {

__host__ __device__ constexpr int ntuv(int L) { return (L + 1) * (L + 2) * (L + 3) / 6; }
__host__ __device__ constexpr int ncart(int l) { return (l + 1) * (l + 2) / 2; }
// position of (t, u, v) in the order of qc/ints.py hermite_index: by n = t + u + v,
// then t descending, then u descending
__host__ __device__ constexpr int tuv_pos(int t, int u, int v) {
  const int n = t + u + v, d = n - t;
  return n * (n + 1) * (n + 2) / 6 + d * (d + 1) / 2 + (d - u);
}

// F_n(T), n = 0..m: the series for F_m and downward recursion below T = 30 (all
// terms positive, no cancellation), F_0 = sqrt(pi/T) erf(sqrt T) / 2 and upward
// recursion above (the amplification (2n+1)/(2T) < 1 for n <= 13 < T: stable).
// The series runs only to fill the table below (its ~T + 30 divisions per call made
// the Boys function the bulk of an s-shell quartet's cost).
__device__ void boys_series(int m, double T, double* F) {
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

// Tabulated F_n(T_i), T_i = i h on [0, 30], n <= BOYS_NM - 1: below T = 30, F_m(T) is the
// 7-term Taylor series about the nearest T_i (dF_n/dT = -F_{n+1}; |T - T_i| <= h / 2 =
// 0.025: remainder <= F_m 0.025^7 / 7! ~ 1.2e-15 relative), the lower orders by the
// downward recursion from it.  Filled once per device by k_boys_init (the series above).
constexpr int BOYS_NM = kIntMaxL + 7;
constexpr int BOYS_NT = 601;
constexpr double BOYS_H = 0.05;
__device__ double g_boys_tab[BOYS_NT * BOYS_NM];

__global__ void k_boys_init() {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < BOYS_NT) {
    double F[BOYS_NM];
    boys_series(BOYS_NM - 1, i * BOYS_H, F);
    for (int n = 0; n < BOYS_NM; ++n) g_boys_tab[i * BOYS_NM + n] = F[n];
  }
}

__device__ __forceinline__ void boys_all(int m, double T, double* F) {
  if (T < 30.0) {
    const int i = (int)(T * (1.0 / BOYS_H) + 0.5);
    const double md = i * BOYS_H - T;            // -(T - T_i)
    const double* f = g_boys_tab + i * BOYS_NM + m;
    double v = f[6];
#pragma unroll
    for (int k = 5; k >= 0; --k) v = f[k] + md * (1.0 / (k + 1)) * v;
    F[m] = v;
    const double et = exp(-T);
    for (int n = m - 1; n >= 0; --n) F[n] = (2.0 * T * F[n + 1] + et) * (1.0 / (2 * n + 1));
  } else {
    boys_series(m, T, F);
  }
}

// R^0_tuv(alpha, X, Y, Z) for all t + u + v <= L (qc/ints.py hermite_r); R and S
// are two level buffers of ntuv(L) doubles, the result lands in R
template <int MAXL>
__device__ void hermite_r(int L, double alpha, double X, double Y, double Z, double* R, double* S) {
  double F[MAXL + 1];
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


// ---- quartets of total Hermite order L = LAB + LC <= 6 (the contracted s / p shells: many
// primitive quartets each) with compile-time (t, u, v) loops: the R table, the ket
// contraction M and the bra contraction stay in registers (the runtime-L path below keeps
// them in private memory and spends more scalar loop control than arithmetic).
template <int L>
__device__ __forceinline__ void hermite_rc(double alpha, double X, double Y, double Z, double (&R)[ntuv(L)]) {
  double F[L + 1];
  boys_all(L, alpha * (X * X + Y * Y + Z * Z), F);
  const double m2a = -2.0 * alpha;
  double pw[L + 1];
  pw[0] = 1.0;
#pragma unroll
  for (int n = 0; n < L; ++n) pw[n + 1] = pw[n] * m2a;
  // in place, one level at a time: level n at (t, u, v) reads level n + 1 at orders
  // tot - 1 and tot - 2 only, so walking tot downwards overwrites nothing still needed
  R[0] = pw[L] * F[L];
#pragma unroll
  for (int n = L - 1; n >= 0; --n) {
#pragma unroll
    for (int tot = L - n; tot >= 1; --tot)
#pragma unroll
      for (int t = tot; t >= 0; --t)
#pragma unroll
        for (int u = tot - t; u >= 0; --u) {
          const int v = tot - t - u;
          double val;
          if (t > 0) {
            val = X * R[tuv_pos(t - 1, u, v)];
            if (t > 1) val += (t - 1) * R[tuv_pos(t - 2, u, v)];
          } else if (u > 0) {
            val = Y * R[tuv_pos(0, u - 1, v)];
            if (u > 1) val += (u - 1) * R[tuv_pos(0, u - 2, v)];
          } else {
            val = Z * R[tuv_pos(0, 0, v - 1)];
            if (v > 1) val += (v - 1) * R[tuv_pos(0, 0, v - 2)];
          }
          R[tuv_pos(t, u, v)] = val;
        }
    R[0] = pw[n] * F[n];
  }
}

template <int LAB, int LC>
__device__ __forceinline__ void quartet_cls(int npp, const double* __restrict__ pp0, const double* __restrict__ ea0,
                                            int nab, int nr, const double* __restrict__ cp0,
                                            const double* __restrict__ e0, int nc, double omega,
                                            double* __restrict__ out, long ldo) {
  constexpr int L = LAB + LC, NT = ntuv(LAB), NU = ntuv(LC);
  for (int q = 0; q < npp; ++q) {
    const double* pp = pp0 + 4 * (long)q;
    const double p = pp[0];
    for (int r = 0; r < nr; ++r) {
      const double* cp = cp0 + 4 * (long)r;
      const double s = cp[0];
      double alpha = p * s / (p + s), scale = 1.0;
      if (omega > 0.0) {
        const double w2 = omega * omega, a2 = alpha * w2 / (alpha + w2);
        scale = sqrt(a2 / alpha);
        alpha = a2;
      }
      double R[ntuv(L)];
      hermite_rc<L>(alpha, pp[1] - cp[1], pp[2] - cp[2], pp[3] - cp[3], R);
      const double pref = 2.0 * pow(M_PI, 2.5) / (p * s * sqrt(p + s)) * scale;
      for (int c = 0; c < nc; ++c) {
        const double* e = e0 + ((long)c * NU) * nr + r;
        double M[NT];
#pragma unroll
        for (int it = 0; it < NT; ++it) M[it] = 0.0;
#pragma unroll
        for (int nu = 0; nu <= LC; ++nu)
#pragma unroll
          for (int tu = nu; tu >= 0; --tu)
#pragma unroll
            for (int uu = nu - tu; uu >= 0; --uu) {
              const int vu = nu - tu - uu, iu = tuv_pos(tu, uu, vu);
              const double w = ((nu & 1) ? -1.0 : 1.0) * e[(long)iu * nr];
#pragma unroll
              for (int nt = 0; nt <= LAB; ++nt)
#pragma unroll
                for (int tt = nt; tt >= 0; --tt)
#pragma unroll
                  for (int ut = nt - tt; ut >= 0; --ut)
                    M[tuv_pos(tt, ut, nt - tt - ut)] += w * R[tuv_pos(tt + tu, ut + uu, nt - tt - ut + vu)];
            }
        for (int ab = 0; ab < nab; ++ab) {
          const double* ea = ea0 + ((long)ab * NT) * npp + q;
          double acc = 0.0;
#pragma unroll
          for (int it = 0; it < NT; ++it) acc += ea[(long)it * npp] * M[it];
          out[(long)ab * ldo + c] += pref * acc;
        }
      }
    }
  }
}

// pair_info[8 k + .]: la, lb, npp, prim0, e0, row0;  pair_prim[4 q + .]: p, Px, Py, Pz
// ket_info[8 j + .]:  lc, nprim, prim0, e0, col0, nc; ket_prim[4 r + .]:  s, Cx, Cy, Cz
// eab (pair k): [a][b][t][q] over ncart(la) x ncart(lb) x ntuv(la+lb) x npp
// ek (ket j):   [c][u][r]    over nc x ntuv(lc) x nprim
// The ket may be a shell pair too (4-index (ab|cd)): lc = l_c + l_d, nc = ncart(l_c)
// ncart(l_d), its primitive pairs and Hermite coefficients as the bra's.
// diag != 0: one thread per bra pair k with the ket j = k (the ERI diagonal blocks).
template <int MAXL, int MAXLAB>
__global__ void __launch_bounds__(64)
k_int_cart(int npair, const int* __restrict__ pair_info, const double* __restrict__ pair_prim,
           const double* __restrict__ eab, int nket, const int* __restrict__ ket_info,
           const double* __restrict__ ket_prim, const double* __restrict__ ek, double* __restrict__ out,
           long ldo, double omega, const double* __restrict__ q_bra, const double* __restrict__ q_ket,
           double q_thr, int diag) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  int k, j;
  if (diag) {
    if (id >= npair) return;
    k = j = (int)id;
  } else {   // bra fastest: the table orders pairs by class (qc/dints.py PairTable)
    if (id >= (long)npair * nket) return;
    j = (int)(id / npair);
    k = (int)(id % npair);
  }
  if (q_bra != nullptr && q_bra[k] * q_ket[j] < q_thr) return;
  const int* pi = pair_info + 8 * k;
  const int* ai = ket_info + 8 * j;
  const int la = pi[0], lb = pi[1], npp = pi[2], pq0 = pi[3], pe0 = pi[4], row0 = pi[5];
  const int lc = ai[0], nr = ai[1], ar0 = ai[2], ae0 = ai[3], col0 = ai[4];
  const int lab = la + lb, L = lab + lc;
  const int nab = ncart(la) * ncart(lb), ntab = ntuv(lab), nc = ai[5], ntc = ntuv(lc);
  if (L <= 6 && lab <= 4 && lc <= 4) {
    const double* pp0 = pair_prim + 4 * (long)pq0;
    const double* cp0 = ket_prim + 4 * (long)ar0;
    double* o = out + (long)row0 * ldo + col0;
#define XT_QC(A, C) \
  case 5 * A + C: quartet_cls<A, C>(npp, pp0, eab + pe0, nab, nr, cp0, ek + ae0, nc, omega, o, ldo); return;
    switch (5 * lab + lc) {
      XT_QC(0, 0) XT_QC(0, 1) XT_QC(0, 2) XT_QC(0, 3) XT_QC(0, 4)
      XT_QC(1, 0) XT_QC(1, 1) XT_QC(1, 2) XT_QC(1, 3) XT_QC(1, 4)
      XT_QC(2, 0) XT_QC(2, 1) XT_QC(2, 2) XT_QC(2, 3) XT_QC(2, 4)
      XT_QC(3, 0) XT_QC(3, 1) XT_QC(3, 2) XT_QC(3, 3)
      XT_QC(4, 0) XT_QC(4, 1) XT_QC(4, 2)
      default: break;
    }
#undef XT_QC
  }
  double R[ntuv(MAXL)], S[ntuv(MAXL)], M[ntuv(MAXLAB)];
  for (int q = 0; q < npp; ++q) {
    const double* pp = pair_prim + 4 * (long)(pq0 + q);
    const double p = pp[0];
    for (int r = 0; r < nr; ++r) {
      const double* cp = ket_prim + 4 * (long)(ar0 + r);
      const double s = cp[0];
      double alpha = p * s / (p + s), scale = 1.0;
      if (omega > 0.0) {   // erf(omega r)/r: 1/a' = 1/alpha + 1/omega^2, times sqrt(a'/alpha)
        const double w2 = omega * omega, a2 = alpha * w2 / (alpha + w2);
        scale = sqrt(a2 / alpha);
        alpha = a2;
      }
      hermite_r<MAXL>(L, alpha, pp[1] - cp[1], pp[2] - cp[2], pp[3] - cp[3], R, S);
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

int int2e_cart(int npair, const int* pair_info, const double* pair_prim, const double* eab, int nket,
               const int* ket_info, const double* ket_prim, const double* ek, int lmax_orb, int lket,
               double omega, const double* q_bra, const double* q_ket, double q_thr, int diag, double* out,
               long ldo, hipStream_t st) {
  const long n = diag ? (long)npair : (long)npair * nket;
  if (n == 0) return 0;
  {   // the Boys table, once per device (stream-ordered before this launch)
    static std::mutex mu;
    static unsigned long long done = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    if (dev >= 64 || !(done >> dev & 1ull)) {
      hipLaunchKernelGGL(k_boys_init, dim3((BOYS_NT + 63) / 64), dim3(64), 0, st);
      if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return XT_ERR_HIP;
      if (dev < 64) done |= 1ull << dev;
    }
  }
  const int blk = 64;
  const dim3 grid((unsigned)((n + blk - 1) / blk));
  if (2 * lmax_orb <= 4 && 2 * lmax_orb + lket <= 8)
    hipLaunchKernelGGL((k_int_cart<8, 4>), grid, dim3(blk), 0, st, npair, pair_info, pair_prim, eab, nket,
                       ket_info, ket_prim, ek, out, ldo, omega, q_bra, q_ket, q_thr, diag);
  else if (2 * lmax_orb <= 6 && 2 * lmax_orb + lket <= kIntMaxL)
    hipLaunchKernelGGL((k_int_cart<kIntMaxL, 6>), grid, dim3(blk), 0, st, npair, pair_info, pair_prim, eab,
                       nket, ket_info, ket_prim, ek, out, ldo, omega, q_bra, q_ket, q_thr, diag);
  else
    return XT_ERR_ARG;
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

// ---------------------------------------------------------------- AO on the grid
// shell_info[8 s + .]: l, nprim, data offset (exponents, then coefficients x radial
// norms, then the centre), first AO; sph: real solid-harmonic tables of l = 0..4
// (libcint order, qc/gto.py _sph_transform) concatenated; norm: per-AO normalisation.
// out[c * comp_stride + g * ldo + ao] for c = value (, d/dx, d/dy, d/dz).
__global__ void __launch_bounds__(256)
k_eval_ao(int ngrid, const double* __restrict__ coords, int nshell, const int* __restrict__ shell_info,
          const double* __restrict__ dat, const double* __restrict__ sph, const double* __restrict__ norm,
          int deriv, double* __restrict__ out, long ldo, long comp_stride) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)ngrid * nshell) return;
  const int g = (int)(id / nshell), s = (int)(id % nshell);
  const int* si = shell_info + 8 * s;
  const int l = si[0], np = si[1], off = si[2], ao0 = si[3];
  const double* ex = dat + off;
  const double* cf = ex + np;
  const double* ctr = cf + np;
  const double dx = coords[3 * (long)g] - ctr[0], dy = coords[3 * (long)g + 1] - ctr[1],
               dz = coords[3 * (long)g + 2] - ctr[2];
  const double r2 = dx * dx + dy * dy + dz * dz;
  double g0 = 0.0, g1 = 0.0;
  for (int k = 0; k < np; ++k) {
    const double e = cf[k] * exp(-ex[k] * r2);
    g0 += e;
    g1 -= 2.0 * ex[k] * e;
  }
  // powers d^0..d^l per direction
  double px[kAoMaxL + 1], py[kAoMaxL + 1], pz[kAoMaxL + 1];
  px[0] = py[0] = pz[0] = 1.0;
  for (int i = 1; i <= l; ++i) {
    px[i] = px[i - 1] * dx;
    py[i] = py[i - 1] * dy;
    pz[i] = pz[i - 1] * dz;
  }
  constexpr int NC = ncart(kAoMaxL);
  double cv[NC], cgx[NC], cgy[NC], cgz[NC];
  int c = 0;
  for (int ix = l; ix >= 0; --ix)
    for (int iy = l - ix; iy >= 0; --iy, ++c) {
      const int iz = l - ix - iy;
      const double poly = px[ix] * py[iy] * pz[iz];
      cv[c] = poly * g0;
      if (deriv) {
        const double pg = poly * g1;
        cgx[c] = (ix ? ix * px[ix - 1] * py[iy] * pz[iz] * g0 : 0.0) + pg * dx;
        cgy[c] = (iy ? iy * px[ix] * py[iy - 1] * pz[iz] * g0 : 0.0) + pg * dy;
        cgz[c] = (iz ? iz * px[ix] * py[iy] * pz[iz - 1] * g0 : 0.0) + pg * dz;
      }
    }
  const int nc = ncart(l), ns = 2 * l + 1;
  int toff = 0;
  for (int k = 0; k < l; ++k) toff += (2 * k + 1) * ncart(k);
  const double* T = sph + toff;
  double* o = out + (long)g * ldo + ao0;
  for (int m = 0; m < ns; ++m) {
    double v = 0.0, vx = 0.0, vy = 0.0, vz = 0.0;
    for (int k = 0; k < nc; ++k) {
      const double t = T[m * nc + k];
      v += t * cv[k];
      if (deriv) {
        vx += t * cgx[k];
        vy += t * cgy[k];
        vz += t * cgz[k];
      }
    }
    const double nm = norm[ao0 + m];
    o[m] = nm * v;
    if (deriv) {
      o[comp_stride + m] = nm * vx;
      o[2 * comp_stride + m] = nm * vy;
      o[3 * comp_stride + m] = nm * vz;
    }
  }
}

int eval_ao(int ngrid, const double* coords, int nshell, const int* shell_info, const double* dat,
            const double* sph, const double* norm, int deriv, double* out, long ldo, long comp_stride,
            hipStream_t st) {
  const long n = (long)ngrid * nshell;
  if (n == 0) return 0;
  const int blk = 256;
  hipLaunchKernelGGL(k_eval_ao, dim3((unsigned)((n + blk - 1) / blk)), dim3(blk), 0, st, ngrid, coords, nshell,
                     shell_info, dat, sph, norm, deriv, out, ldo, comp_stride);
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
