// Element-wise / gather kernels of the TDA hot path (gfx950).
//
// Layout conventions (all FP64, row-major):
//   Ze   (nz, O, V)    one spin channel's trial vectors embedded in the
//                      superset occupied (O = nc+no) x virtual (V = no+nv)
//                      block; positions outside the channel's own block are 0.
//   Phi  (ncomp, ngrid, nmo) MO values/gradients on the grid.
//   U/S  (ncomp, G, nz*O)    per grid chunk: U_c = PhiV^c Ze^T, overwritten
//                            in place by the back-projection factors S_c.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include "xt_internal.h"
#include "xt_kernels.h"

namespace xt {

static inline int nblocks(long n, int bs = 256, int cap = 65536) {
  long b = (n + bs - 1) / bs;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

#define GRID_STRIDE(i, n) \
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

// ---- X-TDA / U-TDA: PySCF-order vectors <-> embedded channels -------------
// za (nocc_a = O, nvir_a = nv) sits at columns [no, V); zb (nocc_b = nc, nvir_b = V)
// sits at rows [0, nc)  (XTDA.py:619-620).
__global__ void k_embed_xtda(int nz, int nc, int no, int nv, const double* __restrict__ z,
                             double* __restrict__ ze) {
  const int O = nc + no, V = no + nv;
  const long dim = (long)O * nv + (long)nc * V;
  const long n = 2L * nz * O * V;
  GRID_STRIDE(t, n) {
    long r = t;
    const int a = (int)(r % V); r /= V;
    const int i = (int)(r % O); r /= O;
    const int x = (int)(r % nz);
    const int ch = (int)(r / nz);
    double v = 0.0;
    if (ch == 0) {
      if (a >= no) v = z[x * dim + (long)i * nv + (a - no)];
    } else {
      if (i < nc) v = z[x * dim + (long)O * nv + (long)i * V + a];
    }
    ze[t] = v;
  }
}

// sigma_out = acc - kx (kx in (O, nz, V) layout per channel)
__global__ void k_extract_xtda(int nz, int nc, int no, int nv, const double* __restrict__ acc,
                               const double* __restrict__ kx, double* __restrict__ out) {
  const int O = nc + no, V = no + nv;
  const long dim = (long)O * nv + (long)nc * V;
  const long chs = (long)nz * O * V;
  GRID_STRIDE(t, (long)nz * dim) {
    const int x = (int)(t / dim);
    const long e = t % dim;
    int ch, i, a;
    if (e < (long)O * nv) { ch = 0; i = (int)(e / nv); a = (int)(e % nv) + no; }
    else { const long f = e - (long)O * nv; ch = 1; i = (int)(f / V); a = (int)(f % V); }
    double v = acc[ch * chs + ((long)x * O + i) * V + a];
    if (kx) v -= kx[ch * chs + ((long)i * nz + x) * V + a];
    out[t] = v;
  }
}

// Single channel (SF / XSF): sigma = acc - kx
__global__ void k_extract_one(int nz, int O, int V, const double* __restrict__ acc,
                              const double* __restrict__ kx, double* __restrict__ out) {
  GRID_STRIDE(t, (long)nz * O * V) {
    const int a = (int)(t % V);
    const long r = t / V;
    const int i = (int)(r % O);
    const int x = (int)(r / O);
    double v = acc[t];
    if (kx) v -= kx[((long)i * nz + x) * V + a];
    out[t] = v;
  }
}

// (nz, O, V) -> (O, nz, V)
__global__ void k_permute_xi(int nz, int O, int V, const double* __restrict__ src,
                             double* __restrict__ dst) {
  GRID_STRIDE(t, (long)nz * O * V) {
    const int a = (int)(t % V);
    const long r = t / V;
    const int x = (int)(r % nz);
    const int i = (int)(r / nz);
    dst[t] = src[((long)x * O + i) * V + a];
  }
}

// dst(nz, O, V) += alpha * src(O, nz, V)
__global__ void k_permute_add(int nz, int O, int V, double alpha, const double* __restrict__ src,
                              double* __restrict__ dst) {
  GRID_STRIDE(t, (long)nz * O * V) {
    const int a = (int)(t % V);
    const long r = t / V;
    const int i = (int)(r % O);
    const int x = (int)(r / O);
    dst[t] += alpha * src[((long)i * nz + x) * V + a];
  }
}

// S[x*svS + j*ldS + b] += alpha * src[(j*nz + x)*ncy + b]
__global__ void k_permute_add_strided(int nz, int nry, int ncy, double alpha, const double* __restrict__ src,
                                      double* __restrict__ dst, long ldS, long svS) {
  GRID_STRIDE(t, (long)nz * nry * ncy) {
    const int b = (int)(t % ncy);
    const long r = t / ncy;
    const int x = (int)(r % nz);
    const int j = (int)(r / nz);
    dst[(long)x * svS + (long)j * ldS + b] += alpha * src[t];
  }
}

// XSF trace / rank-one Delta-A terms, one block per trial vector (XSF_TDA.py:1235-1269):
//   t_oo = tr(oo), t_cv = <fs_cv, cv>, t_co = <fB_co, co>, t_ov = sum fA_vo[a,u] ov[u,a]
//   cv += a2*fs_cv*t_oo ; co += a4*fB_co*t_oo ; ov -= a4*fA_vo^T*t_oo
//   oo_vv += a2*t_cv + a4*(t_co - t_ov)          (a2 = fg*foo*f2/si, a4 = fg*foo*f4)
__global__ void k_xsf_rank1(int nz, int nc, int no, int nv, int nmo, double a2, double a4,
                            const double* __restrict__ ze, const double* __restrict__ fs,
                            const double* __restrict__ fa, const double* __restrict__ fb,
                            double* __restrict__ acc) {
  __shared__ double red[4][256];
  const int x = blockIdx.x;
  const int O = nc + no, V = no + nv;
  const int mo = nc, mv = nc + no;
  const double* z = ze + (long)x * O * V;
  double* s = acc + (long)x * O * V;
  double t[4] = {0, 0, 0, 0};
  for (int k = threadIdx.x; k < no; k += blockDim.x) t[0] += z[(long)(nc + k) * V + k];
  for (long k = threadIdx.x; k < (long)nc * nv; k += blockDim.x) {
    const int i = (int)(k / nv), a = (int)(k % nv);
    t[1] += fs[(long)i * nmo + mv + a] * z[(long)i * V + no + a];
  }
  for (long k = threadIdx.x; k < (long)nc * no; k += blockDim.x) {
    const int i = (int)(k / no), u = (int)(k % no);
    t[2] += fb[(long)i * nmo + mo + u] * z[(long)i * V + u];
  }
  for (long k = threadIdx.x; k < (long)no * nv; k += blockDim.x) {
    const int u = (int)(k / nv), a = (int)(k % nv);
    t[3] += fa[(long)(mv + a) * nmo + mo + u] * z[(long)(nc + u) * V + no + a];
  }
  for (int q = 0; q < 4; ++q) red[q][threadIdx.x] = t[q];
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) for (int q = 0; q < 4; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + w];
    __syncthreads();
  }
  const double t_oo = red[0][0], t_cv = red[1][0], t_co = red[2][0], t_ov = red[3][0];
  for (long k = threadIdx.x; k < (long)nc * nv; k += blockDim.x) {
    const int i = (int)(k / nv), a = (int)(k % nv);
    s[(long)i * V + no + a] += a2 * fs[(long)i * nmo + mv + a] * t_oo;
  }
  for (long k = threadIdx.x; k < (long)nc * no; k += blockDim.x) {
    const int i = (int)(k / no), u = (int)(k % no);
    s[(long)i * V + u] += a4 * fb[(long)i * nmo + mo + u] * t_oo;
  }
  for (long k = threadIdx.x; k < (long)no * nv; k += blockDim.x) {
    const int u = (int)(k / nv), a = (int)(k % nv);
    s[(long)(nc + u) * V + no + a] -= a4 * fa[(long)(mv + a) * nmo + mo + u] * t_oo;
  }
  for (int v = threadIdx.x; v < no; v += blockDim.x)
    s[(long)(nc + v) * V + v] += a2 * t_cv + a4 * (t_co - t_ov);
}

// U-TDA orbital-energy term: acc[ch][x][i][a] += (eps_v[a] - eps_o[i]) * ze[ch][x][i][a]
// (XTDA.py:685-687).  eps_* of channel ch live at eps + ch*nmo.
__global__ void k_ediag(int nz, int O, int V, int nmo, int v0, const double* __restrict__ eps,
                        const double* __restrict__ ze, double* __restrict__ acc) {
  const long chs = (long)nz * O * V;
  GRID_STRIDE(t, 2 * chs) {
    const int ch = (int)(t / chs);
    const long e = t % chs;
    const int a = (int)(e % V);
    const int i = (int)((e / V) % O);
    const double* ep = eps + (long)ch * nmo;
    acc[t] += (ep[v0 + a] - ep[i]) * ze[t];
  }
}

// ---- XC response on the grid, UKS kernel (PySCF nr_uks_fxc semantics) ----
// For each grid point g and vector x (one 64-lane wave):
//   rho1[s][0]  = sum_i U0[s][g][x,i] * PhiO0[s][g][i]
//   rho1[s][c]  = sum_i (U0 PhiOc + Uc PhiO0)        c = 1..3 (GGA)
//   wv[s][y]    = sum_{t,y'} wfxc[t,y'][s,y][g] rho1[t][y']   (weight folded in)
//   S0[s][g][x,i] = wv0 PhiO0 + sum_c wvc PhiOc ;  Sc = wvc PhiO0
// U is overwritten by S.  U layout: (nch, ncomp, G, nz*O); PhiO of channel s
// is phi[s] + comp*ngrid*nmo + (g0+g)*nmo + i.
template <int NC>
__global__ void __launch_bounds__(256)
k_xc_uks(int G, int g0, int ngrid, int nz, int O, int nmo,
         const double* __restrict__ phi0, const double* __restrict__ phi1,
         const double* __restrict__ wfxc, double* __restrict__ U) {
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwork = (long)G * nz;
  if (wid >= nwork) return;
  const int g = (int)(wid / nz);
  const int x = (int)(wid % nz);
  const long ldU = (long)nz * O;
  const long compU = (long)G * ldU;
  const long chU = NC * compU;
  const long compP = (long)ngrid * nmo;
  const double* phis[2] = {phi0, phi1};

  double rho[2][NC];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const double* ph = phis[s] + (long)(g0 + g) * nmo;
    const double* u = U + s * chU + (long)g * ldU + (long)x * O;
    double acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0;
    for (int i = lane; i < O; i += 64) {
      const double u0 = u[i];
      const double p0 = ph[i];
      acc[0] += u0 * p0;
#pragma unroll
      for (int c = 1; c < NC; ++c)
        acc[c] += u0 * ph[c * compP + i] + u[c * compU + i] * p0;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      double v = acc[c];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      rho[s][c] = v;
    }
  }
  // wv[s][y] = sum_{t,y'} f[t,y',s,y] rho[t][y']  ; f layout (2,NC,2,NC,ngrid)
  double wv[2][NC];
  const long gg = g0 + g;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int y = 0; y < NC; ++y) {
      double v = 0.0;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int yy = 0; yy < NC; ++yy)
          v += wfxc[((((long)t * NC + yy) * 2 + s) * NC + y) * ngrid + gg] * rho[t][yy];
      wv[s][y] = v;
    }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const double* ph = phis[s] + (long)(g0 + g) * nmo;
    double* u = U + s * chU + (long)g * ldU + (long)x * O;
    for (int i = lane; i < O; i += 64) {
      const double p0 = ph[i];
      double s0 = wv[s][0] * p0;
#pragma unroll
      for (int c = 1; c < NC; ++c) {
        s0 += wv[s][c] * ph[c * compP + i];
        u[c * compU + i] = wv[s][c] * p0;
      }
      u[i] = s0;
    }
  }
}

// ---- XC response, "W route" (one 256-thread block per grid point g) ---------
// Spin channel s of trial vector x holds, at grid point g (g0 + g globally):
//   U_s[g][x*O + i] = sum_a PhiV0[g][a] Z[x][i][a]       (GEMM, xc forward)
//   R_s[g][3x + c-1] = sum_a W[g][x][a] PhiVc[g][a]      (fused GEMM, GGA only;
//                      W[g][x][a] = sum_i PhiO0[g][i] Z[x][i][a] is never stored)
// and this kernel forms (PySCF eval_rho for a non-hermitian dm + nr_uks_fxc):
//   rho1[s][0] = sum_i U PhiO0 ;  rho1[s][c] = sum_i U PhiOc + R_s[c-1]
//   wv[s][y]   = sum_{t,y'} (w fxc)[t,y'][s,y] rho1[t][y']
//   U <- L = wv0 PhiO0 + sum_c wvc PhiOc ;  R_s <- wv[s][1..3]
// so that sigma += L^T PhiV0 + PhiO0^T M with M = sum_c wvc PhiVc generated
// inside the back GEMM.  The grid point's occupied MO values / gradients and
// the 2NC x 2NC kernel block are staged once in LDS and reused by all 2*nz
// vectors; each wave handles one x for both spins (HBM-bound on U / L).
// NS = 2: the spin-conserving UKS response (nr_uks_fxc); NS = 1: one spin-flip channel
// with the multicollinear kernel (nr_uks_fxc_sf_tda_mc, SF_TDA.py:976-1047), kernel
// layout (NC, NC, ngrid) -- the same contraction with the spin index dropped.
template <int NC, int NS>
__global__ void __launch_bounds__(256, 4)
k_xc_uks_w(int g0, int ngrid, int nz, int O, int nmo, long compP,
           const double* __restrict__ pO0, const double* __restrict__ pO1,
           const double* __restrict__ wfxc,
           double* __restrict__ U0, long ldU0, double* __restrict__ U1, long ldU1,
           double* __restrict__ R0, long ldR0, double* __restrict__ R1, long ldR1) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ double sk[NS * NS * NC * NC];   // sk[((t*NC + y')*NS + s)*NC + y] = (w fxc) at this point
  const int g = blockIdx.x;
  const long gg = g0 + g;
  const bool same = (NS == 1 || pO0 == pO1);
  const double* so[2];
  so[0] = sm;
  so[1] = same ? so[0] : sm + NC * O;
  for (int s = 0; s < (same ? 1 : 2); ++s) {
    const double* po = s ? pO1 : pO0;
    double* dso = sm + s * NC * O;
    for (int k = threadIdx.x; k < NC * O; k += blockDim.x) {
      const int cc = k / O, i = k % O;
      dso[k] = po[cc * compP + gg * nmo + i];
    }
  }
  for (int k = threadIdx.x; k < NS * NS * NC * NC; k += blockDim.x) sk[k] = wfxc[(long)k * ngrid + gg];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwave = blockDim.x >> 6;
  double* Ub[2] = {U0 + g * ldU0, U1 + g * ldU1};
  double* Rb[2] = {R0 ? R0 + g * ldR0 : nullptr, R1 ? R1 + g * ldR1 : nullptr};
  for (int x = wave; x < nz; x += nwave) {
    double acc[NS][NC];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[s][c] = 0.0;
    for (int i = lane; i < O; i += 64) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const double a = Ub[s][(long)x * O + i];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[s][c] += a * so[s][c * O + i];
      }
    }
    double rho[NS][NC];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        double v = acc[s][c];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (NC > 1 && c > 0) v += Rb[s][3 * x + c - 1];
        rho[s][c] = v;
      }
    double wv[NS][NC];
    // keep the NS^2 NC^2 kernel values in LDS (re-read per x): hoisted out of the
    // x loop they would pin 2 NS^2 NC^2 VGPRs
    asm volatile("" ::: "memory");
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int y = 0; y < NC; ++y) {
        double v = 0.0;
#pragma unroll
        for (int t = 0; t < NS; ++t)
#pragma unroll
          for (int yy = 0; yy < NC; ++yy) v += sk[((t * NC + yy) * NS + s) * NC + y] * rho[t][yy];
        wv[s][y] = v;
      }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      double* u = Ub[s] + (long)x * O;
      for (int i = lane; i < O; i += 64) {
        double l = 0.0;
#pragma unroll
        for (int c = 0; c < NC; ++c) l += wv[s][c] * so[s][c * O + i];
        u[i] = l;
      }
    }
    if (NC > 1 && lane < 3 * NS) {   // all reads of R for this x are done (shuffle-synchronised wave)
      const int s = lane / 3, c = lane % 3 + 1;
      double v = 0.0;
#pragma unroll
      for (int ss = 0; ss < NS; ++ss)
#pragma unroll
        for (int y = 1; y < NC; ++y)
          if (ss == s && y == c) v = wv[ss][y];
      Rb[s][3 * x + c - 1] = v;
    }
  }
}

// Same contraction, one wave per grid point (4 per block), no LDS and no
// block barrier: the point's occupied MO values / gradients live in registers
// (IC chunks of 64 orbitals per lane), the 2NC partial sums of each x are reduced
// by a transposing butterfly (halving steps hand each lane half of the values:
// v_permlane32/16_swap for the cross-row steps, shuffles inside rows): 10
// exchanges for the 8 GGA sums instead of 8 x 6, and lane l < 2NC computes
// wv[l] from its own column of the kernel block.  HBM-bound on U / L.
__device__ __forceinline__ void swap_rows32(double& A, double& B) {
  const unsigned alo = (unsigned)__double2loint(A), ahi = (unsigned)__double2hiint(A);
  const unsigned blo = (unsigned)__double2loint(B), bhi = (unsigned)__double2hiint(B);
  const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
  A = __hiloint2double((int)hi[0], (int)lo[0]);
  B = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap_rows16(double& A, double& B) {
  const unsigned alo = (unsigned)__double2loint(A), ahi = (unsigned)__double2hiint(A);
  const unsigned blo = (unsigned)__double2loint(B), bhi = (unsigned)__double2hiint(B);
  const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
  A = __hiloint2double((int)hi[0], (int)lo[0]);
  B = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Sum each of NV (power of two, <= 8) per-lane values over the wave; value j
// ends in the lanes with lane >> (6 - log2 NV) == j.  Halving step at offset o:
// the lower half (lane & o == 0) keeps index k, the upper k + n/2, each adding
// its partner's copy (permlane swap of the pair (v[k], v[k + n/2]) leaves the
// two copies of one index split across the two results in every lane).
template <int NV>
__device__ __forceinline__ double wave_sum_transpose(double (&v)[NV], int lane) {
  static_assert(NV == 1 || NV == 2 || NV == 4 || NV == 8, "NV");
  int n = NV;
  if constexpr (NV >= 2) {
#pragma unroll
    for (int k = 0; k < NV / 2; ++k) { swap_rows32(v[k], v[k + NV / 2]); v[k] += v[k + NV / 2]; }
    n = NV / 2;
  }
  if constexpr (NV >= 4) {
#pragma unroll
    for (int k = 0; k < NV / 4; ++k) { swap_rows16(v[k], v[k + NV / 4]); v[k] += v[k + NV / 4]; }
    n = NV / 4;
  }
  if constexpr (NV >= 8) {   // offset 8 inside a row: explicit keep / send
    const bool up = lane & 8;
    const double send = up ? v[0] : v[1];
    const double keep = up ? v[1] : v[0];
    v[0] = keep + __shfl_xor(send, 8);
  }
  (void)n;
  double t = v[0];
#pragma unroll
  for (int o = 32 / NV; o > 0; o >>= 1) t += __shfl_xor(t, o);
  return t;
}

template <int NC, int IC, int NS>
__global__ void __launch_bounds__(256)
k_xc_point(int G, int g0, int ngrid, int nz, int O, int nmo, long compP,
           const double* __restrict__ pO0, const double* __restrict__ pO1,
           const double* __restrict__ wfxc,
           double* __restrict__ U0, long ldU0, double* __restrict__ U1, long ldU1,
           double* __restrict__ R0, long ldR0, double* __restrict__ R1, long ldR1) {
  constexpr int NV = NS * NC;
  constexpr int SH = NV == 8 ? 3 : (NV == 4 ? 4 : (NV == 2 ? 5 : 6));   // value j lives at lanes j << SH
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= G) return;   // whole waves only; no block-level synchronisation below
  const long gg = g0 + g;
  double ph[NS][NC][IC];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const double* po = s ? pO1 : pO0;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int m = 0; m < IC; ++m) {
        const int i = lane + 64 * m;
        ph[s][c][m] = i < O ? po[c * compP + gg * nmo + i] : 0.0;
      }
  }
  // lane l < NV: column (s, y) = (l / NC, l % NC) of the (w fxc) block at this point
  const int sl = lane / NC, yl = lane % NC;
  double fk[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int t = k / NC, yy = k % NC;
    fk[k] = lane < NV ? wfxc[(long)(((t * NC + yy) * NS + sl) * NC + yl) * ngrid + gg] : 0.0;
  }
  double* Ub[2] = {U0 + g * ldU0, U1 + g * ldU1};
  double* Rb[2] = {R0 ? R0 + g * ldR0 : nullptr, R1 ? R1 + g * ldR1 : nullptr};
  // the next x's U row and rhoW values are loaded before this x's reductions, so
  // two rows per wave are in flight (the loop is HBM-latency-bound otherwise)
  double un[NS][IC], rn[NS][NC > 1 ? NC - 1 : 1];
  auto load_x = [&](int x) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
      for (int m = 0; m < IC; ++m) {
        const int i = lane + 64 * m;
        un[s][m] = i < O ? Ub[s][(long)x * O + i] : 0.0;
      }
      if constexpr (NC > 1) {
#pragma unroll
        for (int c = 1; c < NC; ++c) rn[s][c - 1] = Rb[s][3 * x + c - 1];
      }
    }
  };
  load_x(0);
  for (int x = 0; x < nz; ++x) {
    double u[NS][IC], rw_[NS][NC > 1 ? NC - 1 : 1];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
      for (int m = 0; m < IC; ++m) u[s][m] = un[s][m];
#pragma unroll
      for (int c = 0; c < (NC > 1 ? NC - 1 : 1); ++c) rw_[s][c] = rn[s][c];
    }
    if (x + 1 < nz) load_x(x + 1);
    double v[NV];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        double a = 0.0;
#pragma unroll
        for (int m = 0; m < IC; ++m) a += u[s][m] * ph[s][c][m];
        v[s * NC + c] = a;
      }
    }
    const double tot = wave_sum_transpose<NV>(v, lane);
    double rho[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) rho[j] = readlane_d(tot, j << SH);
    if constexpr (NC > 1) {
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int c = 1; c < NC; ++c) rho[s * NC + c] += rw_[s][c - 1];
    }
    double wl = 0.0;
#pragma unroll
    for (int k = 0; k < NV; ++k) wl += fk[k] * rho[k];
    double wv[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) wv[j] = readlane_d(wl, j);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int m = 0; m < IC; ++m) {
        const int i = lane + 64 * m;
        double l = 0.0;
#pragma unroll
        for (int c = 0; c < NC; ++c) l += wv[s * NC + c] * ph[s][c][m];
        if (i < O) Ub[s][(long)x * O + i] = l;
      }
    if constexpr (NC > 1) {
      if (lane < NV && yl > 0) Rb[sl][3 * x + yl - 1] = wl;
    }
  }
}

// Sum each of 32 per-lane values over the wave; value j ends in lanes 2 j and 2 j + 1
// (the wave_sum_transpose halving steps carried down to offset 2, then one xor-1 add).
// The offset 8 / 2 / 1 exchanges are DPP moves inside a 16-lane row (row_ror 8, quad_perm),
// offset 4 a ds_bpermute.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int O>
__device__ __forceinline__ double xchg(double send) {
  if constexpr (O == 8) return dpp_d<0x128>(send);                                 // row_ror:8
  else if constexpr (O == 4) return __shfl_xor(send, 4);
  else if constexpr (O == 2) return dpp_d<0x4E>(send);                             // quad_perm 2,3,0,1
  else return dpp_d<0xB1>(send);                                                   // quad_perm 1,0,3,2
}
template <int N, int O>
__device__ __forceinline__ void halve_xor(double (&v)[32], int lane) {
  const bool up = lane & O;
#pragma unroll
  for (int k = 0; k < N / 2; ++k) {
    const double send = up ? v[k] : v[k + N / 2];
    const double keep = up ? v[k + N / 2] : v[k];
    v[k] = keep + xchg<O>(send);
  }
}
__device__ __forceinline__ double wave_sum_transpose32(double (&v)[32], int lane) {
#pragma unroll
  for (int k = 0; k < 16; ++k) { swap_rows32(v[k], v[k + 16]); v[k] += v[k + 16]; }
#pragma unroll
  for (int k = 0; k < 8; ++k) { swap_rows16(v[k], v[k + 8]); v[k] += v[k + 8]; }
  halve_xor<8, 8>(v, lane);
  halve_xor<4, 4>(v, lane);
  halve_xor<2, 2>(v, lane);
  return v[0] + xchg<1>(v[0]);
}

// The grid point kernel with XB = 32 / NV trial vectors per reduction (NV = 2 NC values per
// vector: spin x component): k_xc_point reduces the NV values of ONE vector per wave-wide
// transpose and broadcasts them back with 2 NV readlanes, a dependency chain that leaves the
// kernel issue- and latency-bound when O is small (C5: O = 37, 1030 SIMD cycles per vector
// and point).  Here one transpose reduces the 32 values of XB vectors (value j = (xb, s, c) in
// lanes 2 j, 2 j + 1), the w fxc contraction runs lane-parallel (lane j: column (s, c) of its
// vector, the NV rho of that vector gathered through 256 B of LDS), and the wv values go back
// to the occupied lanes through LDS broadcast reads.  Same arithmetic per (point, vector).
// The next batch's U rows are loaded while this one is reduced.
template <int NC, int IC, int NS>
__global__ void __launch_bounds__(256)
k_xc_point_b(int G, int g0, int ngrid, int nz, int O, int nmo, long compP,
             const double* __restrict__ pO0, const double* __restrict__ pO1,
             const double* __restrict__ wfxc,
             double* __restrict__ U0, long ldU0, double* __restrict__ U1, long ldU1,
             double* __restrict__ R0, long ldR0, double* __restrict__ R1, long ldR1) {
  constexpr int NV = NS * NC, XB = 32 / NV;
  __shared__ __attribute__((aligned(16))) double sh[4][2][32];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = blockIdx.x * 4 + wid;
  if (g >= G) return;   // whole waves only; the LDS slots are per wave
  const long gg = g0 + g;
  double* rs = sh[wid][0];
  double* ws = sh[wid][1];
  double ph[NS][NC][IC];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const double* po = s ? pO1 : pO0;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int m = 0; m < IC; ++m) {
        const int i = lane + 64 * m;
        ph[s][c][m] = i < O ? po[c * compP + gg * nmo + i] : 0.0;
      }
  }
  // this lane's value j = lane >> 1 = (xb, sl, yl) after the reduction
  const int j = lane >> 1, xbl = j / NV, kl = j % NV, sl = kl / NC, yl = kl % NC;
  double fk[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int t = k / NC, yy = k % NC;
    fk[k] = wfxc[(long)(((t * NC + yy) * NS + sl) * NC + yl) * ngrid + gg];
  }
  double* Ub[2] = {U0 + g * ldU0, U1 + g * ldU1};
  double* Rl = (NC > 1 && yl > 0) ? (sl ? R1 + g * ldR1 : R0 + g * ldR0) + yl - 1 : nullptr;
  // batch loads: U rows of XB vectors (lanes over occupied), this lane's rhoW value.
  // Branch-free: lanes past O and vectors past nz read a clamped (valid) element and
  // keep zero.
  const double* ul[NS][IC];
  bool iv[IC];
#pragma unroll
  for (int m = 0; m < IC; ++m) {
    const int i = lane + 64 * m;
    iv[m] = i < O;
#pragma unroll
    for (int s = 0; s < NS; ++s) ul[s][m] = Ub[s] + (i < O ? i : O - 1);
  }
  const double* rl = Rl ? Rl : (R0 ? R0 + g * ldR0 : Ub[0]);
  double un[XB][NS][IC], rn;
  auto load_b = [&](int x0, double (&ub)[XB][NS][IC], double& rb) __attribute__((always_inline)) {
#pragma unroll
    for (int xb = 0; xb < XB; ++xb) {
      const int x = x0 + xb < nz ? x0 + xb : nz - 1;
      const bool xv = x0 + xb < nz;
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int m = 0; m < IC; ++m) {
          const double t = ul[s][m][(long)x * O];
          ub[xb][s][m] = (iv[m] && xv) ? t : 0.0;
        }
    }
    rb = 0.0;
    if constexpr (NC > 1) {
      const int x = x0 + xbl < nz ? x0 + xbl : nz - 1;
      const double t = rl[3 * x];
      rb = (Rl && x0 + xbl < nz) ? t : 0.0;
    }
  };
  auto body = [&](int x0, const double (&u)[XB][NS][IC], double r) __attribute__((always_inline)) {
    double v[32];
#pragma unroll
    for (int xb = 0; xb < XB; ++xb)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          double a = 0.0;
#pragma unroll
          for (int m = 0; m < IC; ++m) a += u[xb][s][m] * ph[s][c][m];
          v[xb * NV + s * NC + c] = a;
        }
    const double rho = wave_sum_transpose32(v, lane) + r;
    if (!(lane & 1)) rs[j] = rho;
    __builtin_amdgcn_wave_barrier();   // LDS is in order within a wave; no memory fence (it
                                       // would wait for the next batch's loads)
    double wl = 0.0;
#pragma unroll
    for (int k = 0; k < NV; k += 2) {
      const double2 p = *(const double2*)(rs + xbl * NV + k);
      wl += fk[k] * p.x + fk[k + 1] * p.y;
    }
    if (!(lane & 1)) ws[j] = wl;
    if constexpr (NC > 1) {
      if (Rl && !(lane & 1) && x0 + xbl < nz) Rl[3 * (x0 + xbl)] = wl;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int xb = 0; xb < XB; ++xb) {
      double wv[NV];
#pragma unroll
      for (int k = 0; k < NV; k += 2) {
        const double2 p = *(const double2*)(ws + xb * NV + k);
        wv[k] = p.x; wv[k + 1] = p.y;
      }
      if (x0 + xb < nz) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int m = 0; m < IC; ++m) {
            const int i = lane + 64 * m;
            double l = 0.0;
#pragma unroll
            for (int c = 0; c < NC; ++c) l += wv[s * NC + c] * ph[s][c][m];
            if (i < O) Ub[s][(long)(x0 + xb) * O + i] = l;
          }
      }
    }
    // the next batch's LDS writes come after every lane's reads of this one
    __builtin_amdgcn_wave_barrier();
  };
  load_b(0, un, rn);
  for (int x0 = 0; x0 < nz; x0 += XB) {
    double u[XB][NS][IC];
#pragma unroll
    for (int xb = 0; xb < XB; ++xb)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int m = 0; m < IC; ++m) u[xb][s][m] = un[xb][s][m];
    const double r = rn;
    if (x0 + XB < nz) load_b(x0 + XB, un, rn);
    body(x0, u, r);
  }
}

// ALDA0 spin-flip kernel (SF_TDA.py:90-160): rho1 = sum_i U0 PhiO, wv = rho1*fsf, S0 = wv*PhiO
__global__ void __launch_bounds__(256)
k_xc_sf(int G, int g0, int nz, int O, int nmo, const double* __restrict__ phio,
        const double* __restrict__ fsf, double* __restrict__ U) {
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  if (wid >= (long)G * nz) return;
  const int g = (int)(wid / nz);
  const int x = (int)(wid % nz);
  const double* ph = phio + (long)(g0 + g) * nmo;
  double* u = U + (long)g * nz * O + (long)x * O;
  double acc = 0.0;
  for (int i = lane; i < O; i += 64) acc += u[i] * ph[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  const double wv = acc * fsf[g0 + g];
  for (int i = lane; i < O; i += 64) u[i] = wv * ph[i];
}

// Same ALDA0 contraction, one wave per grid point for all nz trial vectors: the
// point's occupied MO values stay in registers (IC chunks of 64 orbitals per lane),
// 8 vectors' rows are loaded together and their 8 partial sums reduced by one
// transposing butterfly (wave_sum_transpose<8>) instead of 8 x 6 shuffles; the
// next group's rows are loaded before this group's reduction.  HBM-bound on U.
template <int IC>
__global__ void __launch_bounds__(256)
k_xc_sf_pt(int G, int g0, int nz, int O, int nmo, const double* __restrict__ phio,
           const double* __restrict__ fsf, double* __restrict__ U) {
  constexpr int NV = 8;
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= G) return;   // whole waves only; no block-level synchronisation below
  const long gg = g0 + g;
  double ph[IC];
#pragma unroll
  for (int m = 0; m < IC; ++m) {
    const int i = lane + 64 * m;
    ph[m] = i < O ? phio[gg * nmo + i] : 0.0;
  }
  const double f = fsf[gg];
  double* ub = U + (long)g * nz * O;
  double un[NV][IC];
  auto load = [&](int x0) {
#pragma unroll
    for (int xx = 0; xx < NV; ++xx)
#pragma unroll
      for (int m = 0; m < IC; ++m) {
        const int i = lane + 64 * m, x = x0 + xx;
        un[xx][m] = (x < nz && i < O) ? ub[(long)x * O + i] : 0.0;
      }
  };
  load(0);
  for (int x0 = 0; x0 < nz; x0 += NV) {
    double v[NV];
#pragma unroll
    for (int xx = 0; xx < NV; ++xx) {
      double a = 0.0;
#pragma unroll
      for (int m = 0; m < IC; ++m) a += un[xx][m] * ph[m];
      v[xx] = a;
    }
    if (x0 + NV < nz) load(x0 + NV);
    const double tot = wave_sum_transpose<NV>(v, lane);
#pragma unroll
    for (int xx = 0; xx < NV; ++xx) {
      const int x = x0 + xx;
      const double wv = readlane_d(tot, xx << 3) * f;
#pragma unroll
      for (int m = 0; m < IC; ++m) {
        const int i = lane + 64 * m;
        if (x < nz && i < O) ub[(long)x * O + i] = wv * ph[m];
      }
    }
  }
}

// wfxc = scale * fxc * w  (fxc layout (2,nc,2,nc,ngrid), or (nc,nc,ngrid) with scale 2 for the
// multicollinear spin-flip kernel: wv = einsum('bg,abg->ag', rho1sf, 2 fxc) w, SF_TDA.py:1003)
__global__ void k_weight_fxc(long n4, int ngrid, double scale, const double* __restrict__ w, double* __restrict__ f) {
  GRID_STRIDE(t, n4 * ngrid) f[t] *= scale * w[t % ngrid];
}

// ---- XSF: cv|co|ov|oo blocks <-> full (nocc_a x nvir_b) spin-flip block ----
// full Z[i][a'] rows i: c then o; cols a': o then v.  OO optionally expanded
// by the compression basis vects (no^2 x (no^2-1)) (XSF_TDA.py:1011-1027).
__global__ void k_xsf_assemble(int nz, int nc, int no, int nv, int remove,
                               const double* __restrict__ vects, const double* __restrict__ z,
                               double* __restrict__ ze) {
  const int O = nc + no, V = no + nv;
  const long d1 = (long)nc * nv, d2 = d1 + (long)nc * no, d3 = d2 + (long)no * nv;
  const long dim = d3 + (long)no * no - (remove ? 1 : 0);
  GRID_STRIDE(t, (long)nz * O * V) {
    const int a = (int)(t % V);
    const long r = t / V;
    const int i = (int)(r % O);
    const int x = (int)(r / O);
    const double* zx = z + x * dim;
    double v;
    if (i < nc) {
      v = (a >= no) ? zx[(long)i * nv + (a - no)] : zx[d1 + (long)i * no + a];
    } else {
      const int u = i - nc;
      if (a >= no) v = zx[d2 + (long)u * nv + (a - no)];
      else {
        const int row = u * no + a;
        if (remove) {
          const int m = no * no - 1;
          double s = 0.0;
          for (int y = 0; y < m; ++y) s += vects[(long)row * m + y] * zx[d3 + y];
          v = s;
        } else {
          v = zx[d3 + row];
        }
      }
    }
    ze[t] = v;
  }
}

// full (nz, O, V) sigma -> cv|co|ov|oo (OO compressed with vects^T when remove)
__global__ void k_xsf_extract(int nz, int nc, int no, int nv, int remove,
                              const double* __restrict__ vects, const double* __restrict__ full,
                              double* __restrict__ out) {
  const int O = nc + no, V = no + nv;
  const long d1 = (long)nc * nv, d2 = d1 + (long)nc * no, d3 = d2 + (long)no * nv;
  const int noo = no * no - (remove ? 1 : 0);
  const long dim = d3 + noo;
  GRID_STRIDE(t, (long)nz * dim) {
    const int x = (int)(t / dim);
    const long e = t % dim;
    const double* f = full + (long)x * O * V;
    double v;
    if (e < d1) { const int i = (int)(e / nv), a = (int)(e % nv); v = f[(long)i * V + no + a]; }
    else if (e < d2) { const long k = e - d1; const int i = (int)(k / no), u = (int)(k % no); v = f[(long)i * V + u]; }
    else if (e < d3) { const long k = e - d2; const int u = (int)(k / nv), a = (int)(k % nv); v = f[(long)(nc + u) * V + no + a]; }
    else {
      const int y = (int)(e - d3);
      if (remove) {
        const int m = no * no - 1;
        double s = 0.0;
        for (int row = 0; row < no * no; ++row)
          s += vects[(long)row * m + y] * f[(long)(nc + row / no) * V + (row % no)];
        v = s;
      } else {
        v = f[(long)(nc + y / no) * V + (y % no)];
      }
    }
    out[t] = v;
  }
}

// XSF J diagonals: co_j[i][u] = sum_P B[P][i][nc+u]^2 ; ov_j[u][a] = sum_P B[P][nc+u][nc+no+a]^2
__global__ void k_xsf_jdiag(int naux, int nmo, int nc, int no, int nv, const double* __restrict__ bmo,
                            double* __restrict__ co_j, double* __restrict__ ov_j) {
  const long nco = (long)nc * no, nov = (long)no * nv;
  GRID_STRIDE(t, nco + nov) {
    long row, col;
    if (t < nco) { row = t / no; col = nc + t % no; }
    else { const long k = t - nco; row = nc + k / nv; col = nc + no + k % nv; }
    double s = 0.0;
    for (int P = 0; P < naux; ++P) {
      const double b = bmo[(long)P * nmo * nmo + row * nmo + col];
      s += b * b;
    }
    if (t < nco) co_j[t] = s; else ov_j[t - nco] = s;
  }
}

// ---- Davidson helpers -----------------------------------------------------
__global__ void k_precond(int nrow, int dim, const double* __restrict__ diag, const double* __restrict__ e,
                          double shift, const double* __restrict__ r, double* __restrict__ out) {
  GRID_STRIDE(t, (long)nrow * dim) {
    const int row = (int)(t / dim);
    double d = diag[t % dim] - (e[row] - shift);
    if (fabs(d) < 1e-8) d = 1e-8;
    out[t] = r[t] / d;
  }
}

__global__ void k_row_norms2(int nrow, int dim, const double* __restrict__ x, double* __restrict__ out) {
  __shared__ double red[256];
  const int row = blockIdx.x;
  double s = 0.0;
  for (long j = threadIdx.x; j < dim; j += blockDim.x) { const double v = x[(long)row * dim + j]; s += v * v; }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[row] = red[0];
}

__global__ void k_row_scale(int nrow, int dim, double* __restrict__ x, const double* __restrict__ s) {
  GRID_STRIDE(t, (long)nrow * dim) x[t] *= s[t / dim];
}

// ---- launch wrappers --------------------------------------------------------
void embed_xtda(hipStream_t st, int nz, int nc, int no, int nv, const double* z, double* ze) {
  const long n = 2L * nz * (nc + no) * (no + nv);
  hipLaunchKernelGGL(k_embed_xtda, dim3(nblocks(n)), dim3(256), 0, st, nz, nc, no, nv, z, ze);
}
void extract_xtda(hipStream_t st, int nz, int nc, int no, int nv, const double* acc, const double* kx, double* out) {
  const long n = (long)nz * ((long)(nc + no) * nv + (long)nc * (no + nv));
  hipLaunchKernelGGL(k_extract_xtda, dim3(nblocks(n)), dim3(256), 0, st, nz, nc, no, nv, acc, kx, out);
}
void extract_one(hipStream_t st, int nz, int O, int V, const double* acc, const double* kx, double* out) {
  hipLaunchKernelGGL(k_extract_one, dim3(nblocks((long)nz * O * V)), dim3(256), 0, st, nz, O, V, acc, kx, out);
}
// Kx[(i,a),(j,b)] = Kx[(j,b),(i,a)] for the blocks build_kx left out: one 64 x 64 tile of
// one block pair per 256-thread block, through LDS (reads along a of block (j, i), writes
// along b of block (i, j), both coalesced)
__global__ void __launch_bounds__(256) k_kx_mirror(int V, long ld, int i0, int fold, double* __restrict__ K) {
  const int i = i0 + blockIdx.y, j = i0 + blockIdx.z;
  const int ci = i0 + ((i - i0) / fold) * fold;
  if (j >= ci) return;                         // built directly (or its own mirror source)
  const int nt = (V + 63) / 64;
  const int ta = blockIdx.x % nt, tb = blockIdx.x / nt;
  __shared__ double s[64][65];
  const int tid = threadIdx.x, cx = tid & 63, ry = tid >> 6;
  const double* src = K + ((long)j * V) * ld + (long)i * V;   // block (j, i): row b, column a
  double* dst = K + ((long)i * V) * ld + (long)j * V;         // block (i, j): row a, column b
#pragma unroll 4
  for (int r = 0; r < 16; ++r) {
    const int b = tb * 64 + 4 * r + ry, a = ta * 64 + cx;
    if (a < V && b < V) s[4 * r + ry][cx] = src[(long)b * ld + a];
  }
  __syncthreads();
#pragma unroll 4
  for (int r = 0; r < 16; ++r) {
    const int a = ta * 64 + 4 * r + ry, b = tb * 64 + cx;
    if (a < V && b < V) dst[(long)a * ld + b] = s[cx][4 * r + ry];
  }
}

void kx_mirror(hipStream_t st, int O, int V, long ld, int i0, int i1, int fold, double* K) {
  (void)O;
  const int nt = (V + 63) / 64, n = i1 - i0;
  if (n <= fold) return;                       // one chunk: every block built directly
  hipLaunchKernelGGL(k_kx_mirror, dim3(nt * nt, n, n), dim3(256), 0, st, V, ld, i0, fold, K);
}

void permute_xi(hipStream_t st, int nz, int O, int V, const double* src, double* dst) {
  hipLaunchKernelGGL(k_permute_xi, dim3(nblocks((long)nz * O * V)), dim3(256), 0, st, nz, O, V, src, dst);
}
void permute_add(hipStream_t st, int nz, int O, int V, double alpha, const double* src, double* dst) {
  hipLaunchKernelGGL(k_permute_add, dim3(nblocks((long)nz * O * V)), dim3(256), 0, st, nz, O, V, alpha, src, dst);
}
void permute_add_strided(hipStream_t st, int nz, int nry, int ncy, double alpha, const double* src,
                         double* dst, long ldS, long svS) {
  hipLaunchKernelGGL(k_permute_add_strided, dim3(nblocks((long)nz * nry * ncy)), dim3(256), 0, st,
                     nz, nry, ncy, alpha, src, dst, ldS, svS);
}
// XSF superset blocks (rows [0,nc) core / [nc,O) open; cols [0,no) open / [no,V) virtual):
// 0 cv, 1 co, 2 ov, 3 oo
__device__ __forceinline__ int xsf_block(int i, int a, int nc, int no) {
  return (i < nc ? 0 : 2) + (a < no ? 1 : 0);
}

// zb[X nz + x][(i,a)] = ze[x][(i,a)] if (i,a) is in block X else 0   (4 nz rows)
__global__ void k_xsf_split4(int nz, int O, int V, int nc, int no, const double* __restrict__ ze,
                             double* __restrict__ zb) {
  const long ov = (long)O * V, total = 4L * nz * ov;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long e = t % ov;
    const int row = (int)(t / ov), X = row / nz, x = row % nz;
    const int i = (int)(e / V), a = (int)(e % V);
    zb[t] = xsf_block(i, a, nc, no) == X ? ze[(long)x * ov + e] : 0.0;
  }
}

// acc[x][(i,a)] += sum_X w[X][Y(i,a)] yb[X nz + x][(i,a)]
__global__ void k_xsf_combine4(int nz, int O, int V, int nc, int no, W16 w16,
                               const double* __restrict__ yb, double* __restrict__ acc) {
  const long ov = (long)O * V, total = (long)nz * ov;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long e = t % ov;
    const int x = (int)(t / ov);
    const int i = (int)(e / V), a = (int)(e % V);
    const int Y = xsf_block(i, a, nc, no);
    double s = 0.0;
#pragma unroll
    for (int X = 0; X < 4; ++X) s += w16.w[4 * X + Y] * yb[((long)X * nz + x) * ov + e];
    acc[t] += s;
  }
}

void xsf_rank1(hipStream_t st, int nz, int nc, int no, int nv, int nmo, double a2, double a4,
               const double* ze, const double* fs, const double* fa, const double* fb, double* acc) {
  hipLaunchKernelGGL(k_xsf_rank1, dim3(nz), dim3(256), 0, st, nz, nc, no, nv, nmo, a2, a4, ze, fs, fa, fb, acc);
}
void ediag(hipStream_t st, int nz, int O, int V, int nmo, int v0, const double* eps, const double* ze, double* acc) {
  hipLaunchKernelGGL(k_ediag, dim3(nblocks(2L * nz * O * V)), dim3(256), 0, st, nz, O, V, nmo, v0, eps, ze, acc);
}
void xc_uks(hipStream_t st, int ncomp, int G, int g0, int ngrid, int nz, int O, int nmo,
            const double* phi0, const double* phi1, const double* wfxc, double* U) {
  const long waves = (long)G * nz;
  const int blocks = (int)((waves * 64 + 255) / 256);
  if (ncomp == 4)
    hipLaunchKernelGGL(k_xc_uks<4>, dim3(blocks), dim3(256), 0, st, G, g0, ngrid, nz, O, nmo, phi0, phi1, wfxc, U);
  else
    hipLaunchKernelGGL(k_xc_uks<1>, dim3(blocks), dim3(256), 0, st, G, g0, ngrid, nz, O, nmo, phi0, phi1, wfxc, U);
}
// Meta-GGA point kernel (nr_uks_fxc's MGGA branch, XTDA.py:514; explicit form
// XTDA.py:239-276): the GGA contraction above plus the kinetic-energy density,
//   tau1[s] = 1/2 sum_c sum_i dPhiO_c[i] T_s[c][x][i],  T_s[c] = dPhiV_c Ze^T (GEMMs),
// the 5 x 5 (rho, grad rho, tau) kernel block, and the tau potential's back operands
//   T_s[c][x][i] <- 1/2 wv[s][4] dPhiO_c[i]       (sigma += T_c^T dPhiV_c, GEMMs).
// One block per grid point, one wave per trial vector x (both spins); correctness
// first (the MGGA classes are plain GEMMs around it).  NS = 1: one spin-flip channel
// with the multicollinear (rho, grad rho, tau) kernel (nr_uks_fxc_sf_tda_mc's MGGA branch,
// SF_TDA.py:1028-1041), kernel layout (NK, NK, ngrid).
template <int NS>
__global__ void __launch_bounds__(256)
k_xc_uks_mgga(int g0, int ngrid, int nz, int O, int nmo, long compP,
              const double* __restrict__ pO0, const double* __restrict__ pO1,
              const double* __restrict__ wfxc,
              double* __restrict__ U0, long ldU0, double* __restrict__ U1, long ldU1,
              double* __restrict__ T0, double* __restrict__ T1, long tcs,
              double* __restrict__ R0, long ldR0, double* __restrict__ R1, long ldR1) {
  constexpr int NC = 4, NK = 5;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ double sk[NS * NS * NK * NK];   // sk[((t*NK + y')*NS + s)*NK + y] = (w fxc) at this point
  const int g = blockIdx.x;
  const long gg = g0 + g;
  const bool same = (NS == 1 || pO0 == pO1);
  const double* so[2];
  so[0] = sm;
  so[1] = same ? so[0] : sm + NC * O;
  for (int s = 0; s < (same ? 1 : 2); ++s) {
    const double* po = s ? pO1 : pO0;
    double* dso = sm + s * NC * O;
    for (int k = threadIdx.x; k < NC * O; k += blockDim.x) {
      const int cc = k / O, i = k % O;
      dso[k] = po[cc * compP + gg * nmo + i];
    }
  }
  for (int k = threadIdx.x; k < NS * NS * NK * NK; k += blockDim.x) sk[k] = wfxc[(long)k * ngrid + gg];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwave = blockDim.x >> 6;
  double* Ub[2] = {U0 + g * ldU0, U1 + g * ldU1};
  double* Tb[2] = {T0 + g * ldU0, T1 + g * ldU1};
  double* Rb[2] = {R0 + g * ldR0, R1 + g * ldR1};
  for (int x = wave; x < nz; x += nwave) {
    double acc[NS][NK];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int c = 0; c < NK; ++c) acc[s][c] = 0.0;
    for (int i = lane; i < O; i += 64) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const double u = Ub[s][(long)x * O + i];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[s][c] += u * so[s][c * O + i];
#pragma unroll
        for (int c = 1; c < NC; ++c) acc[s][4] += Tb[s][(c - 1) * tcs + (long)x * O + i] * so[s][c * O + i];
      }
    }
    double rho[NS][NK];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int c = 0; c < NK; ++c) {
        double v = acc[s][c];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (c >= 1 && c <= 3) v += Rb[s][3 * x + c - 1];
        rho[s][c] = c == 4 ? 0.5 * v : v;
      }
    double wv[NS][NK];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int y = 0; y < NK; ++y) {
        double v = 0.0;
#pragma unroll
        for (int t = 0; t < NS; ++t)
#pragma unroll
          for (int yy = 0; yy < NK; ++yy) v += sk[((t * NK + yy) * NS + s) * NK + y] * rho[t][yy];
        wv[s][y] = v;
      }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      for (int i = lane; i < O; i += 64) {
        double l = 0.0;
#pragma unroll
        for (int c = 0; c < NC; ++c) l += wv[s][c] * so[s][c * O + i];
        Ub[s][(long)x * O + i] = l;
#pragma unroll
        for (int c = 1; c < NC; ++c) Tb[s][(c - 1) * tcs + (long)x * O + i] = 0.5 * wv[s][4] * so[s][c * O + i];
      }
    }
    if (lane < 3 * NS) {   // all reads of R for this x are done (shuffle-synchronised wave)
      const int s = lane / 3, c = lane % 3 + 1;
      double v = 0.0;
#pragma unroll
      for (int ss = 0; ss < NS; ++ss)
#pragma unroll
        for (int y = 1; y < NC; ++y)
          if (ss == s && y == c) v = wv[ss][y];
      Rb[s][3 * x + c - 1] = v;
    }
  }
}
void xc_uks_mgga(hipStream_t st, int ns, int G, int g0, int ngrid, int nz, int O, int nmo, long compP,
                 const double* pO0, const double* pO1, const double* wfxc, double* U0, long ldU0, double* U1,
                 long ldU1, double* T0, double* T1, long tcs, double* R0, long ldR0, double* R1, long ldR1) {
  if (G <= 0 || nz <= 0 || O <= 0) return;
  const bool same = (ns == 1 || pO0 == pO1);
  const size_t lds = (same ? 1 : 2) * (size_t)4 * O * sizeof(double);
  if (ns == 1)
    hipLaunchKernelGGL(k_xc_uks_mgga<1>, dim3(G), dim3(256), lds, st, g0, ngrid, nz, O, nmo, compP, pO0, pO0, wfxc,
                       U0, ldU0, U0, ldU0, T0, T0, tcs, R0, ldR0, R0, ldR0);
  else
    hipLaunchKernelGGL(k_xc_uks_mgga<2>, dim3(G), dim3(256), lds, st, g0, ngrid, nz, O, nmo, compP, pO0, pO1, wfxc,
                       U0, ldU0, U1, ldU1, T0, T1, tcs, R0, ldR0, R1, ldR1);
}
void xc_uks_w(hipStream_t st, int ns, int ncomp, int G, int g0, int ngrid, int nz, int O, int nmo, long compP,
              const double* pO0, const double* pO1, const double* wfxc, double* U0, long ldU0,
              double* U1, long ldU1, double* R0, long ldR0, double* R1, long ldR1) {
  if (G <= 0 || nz <= 0 || O <= 0) return;
  if (ns == 1) {   // one spin-flip channel: the second channel's pointers are never read
    pO1 = pO0; U1 = U0; ldU1 = ldU0; R1 = R0; ldR1 = ldR0;
  }
  if (O <= 256) {   // one wave per grid point, occupied values in registers
    const dim3 grid((G + 3) / 4), blk(256);
#define XT_POINT(NC, IC, NS) hipLaunchKernelGGL((k_xc_point<NC, IC, NS>), grid, blk, 0, st, G, g0, ngrid, nz, O, nmo, \
                                                compP, pO0, pO1, wfxc, U0, ldU0, U1, ldU1, R0, ldR0, R1, ldR1)
#define XT_POINT_B(IC, NS) hipLaunchKernelGGL((k_xc_point_b<4, IC, NS>), grid, blk, 0, st, G, g0, ngrid, nz, O, nmo, \
                                              compP, pO0, pO1, wfxc, U0, ldU0, U1, ldU1, R0, ldR0, R1, ldR1)
    // GGA, O <= 128: several vectors per reduction (k_xc_point_b; same box: C5 18.5-18.6 ->
    // 17.6-17.7 ms per A.x, C2 10.72-10.75 -> 10.17-10.26, headline neutral; two batches in
    // flight or ds_bpermute instead of DPP: within 1 %)
    if (ncomp == 4 && O <= 128) {
      if (ns == 1) { if (O <= 64) XT_POINT_B(1, 1); else XT_POINT_B(2, 1); }
      else         { if (O <= 64) XT_POINT_B(1, 2); else XT_POINT_B(2, 2); }
      return;
    }
    if (ncomp == 4) { if (ns == 1) XT_POINT(4, 4, 1); else XT_POINT(4, 4, 2); }
    else            { if (O <= 64) XT_POINT(1, 1, 2); else if (O <= 128) XT_POINT(1, 2, 2); else XT_POINT(1, 4, 2); }
#undef XT_POINT
#undef XT_POINT_B
    return;
  }
  const bool same = (ns == 1 || pO0 == pO1);
  const size_t lds = (same ? 1 : 2) * (size_t)ncomp * O * sizeof(double);
  if (ncomp == 4 && ns == 1)
    hipLaunchKernelGGL((k_xc_uks_w<4, 1>), dim3(G), dim3(256), lds, st, g0, ngrid, nz, O, nmo, compP,
                       pO0, pO1, wfxc, U0, ldU0, U1, ldU1, R0, ldR0, R1, ldR1);
  else if (ncomp == 4)
    hipLaunchKernelGGL((k_xc_uks_w<4, 2>), dim3(G), dim3(256), lds, st, g0, ngrid, nz, O, nmo, compP,
                       pO0, pO1, wfxc, U0, ldU0, U1, ldU1, R0, ldR0, R1, ldR1);
  else
    hipLaunchKernelGGL((k_xc_uks_w<1, 2>), dim3(G), dim3(256), lds, st, g0, ngrid, nz, O, nmo, compP,
                       pO0, pO1, wfxc, U0, ldU0, U1, ldU1, R0, ldR0, R1, ldR1);
}
void xc_sf(hipStream_t st, int G, int g0, int nz, int O, int nmo, const double* phio, const double* fsf, double* U) {
  if (O <= 256) {   // one wave per grid point; the wave-per-(point, vector) kernel beyond
    const dim3 grid((G + 3) / 4), blk(256);
    if (O <= 128)      hipLaunchKernelGGL((k_xc_sf_pt<2>), grid, blk, 0, st, G, g0, nz, O, nmo, phio, fsf, U);
    else if (O <= 192) hipLaunchKernelGGL((k_xc_sf_pt<3>), grid, blk, 0, st, G, g0, nz, O, nmo, phio, fsf, U);
    else               hipLaunchKernelGGL((k_xc_sf_pt<4>), grid, blk, 0, st, G, g0, nz, O, nmo, phio, fsf, U);
    return;
  }
  const long waves = (long)G * nz;
  const int blocks = (int)((waves * 64 + 255) / 256);
  hipLaunchKernelGGL(k_xc_sf, dim3(blocks), dim3(256), 0, st, G, g0, nz, O, nmo, phio, fsf, U);
}
void weight_fxc(hipStream_t st, long n4, int ngrid, double scale, const double* w, double* f) {
  hipLaunchKernelGGL(k_weight_fxc, dim3(nblocks(n4 * ngrid)), dim3(256), 0, st, n4, ngrid, scale, w, f);
}
void xsf_assemble(hipStream_t st, int nz, int nc, int no, int nv, int remove, const double* vects, const double* z, double* ze) {
  const long n = (long)nz * (nc + no) * (no + nv);
  hipLaunchKernelGGL(k_xsf_assemble, dim3(nblocks(n)), dim3(256), 0, st, nz, nc, no, nv, remove, vects, z, ze);
}
void xsf_extract(hipStream_t st, int nz, int nc, int no, int nv, int remove, const double* vects, const double* full, double* out) {
  const long dim = (long)nc * nv + (long)nc * no + (long)no * nv + (long)no * no - (remove ? 1 : 0);
  hipLaunchKernelGGL(k_xsf_extract, dim3(nblocks((long)nz * dim)), dim3(256), 0, st, nz, nc, no, nv, remove, vects, full, out);
}
void xsf_jdiag(hipStream_t st, int naux, int nmo, int nc, int no, int nv, const double* bmo, double* co_j, double* ov_j) {
  const long n = (long)nc * no + (long)no * nv;
  hipLaunchKernelGGL(k_xsf_jdiag, dim3(nblocks(n)), dim3(256), 0, st, naux, nmo, nc, no, nv, bmo, co_j, ov_j);
}
void precond(hipStream_t st, int nrow, int dim, const double* diag, const double* e, double shift, const double* r, double* out) {
  hipLaunchKernelGGL(k_precond, dim3(nblocks((long)nrow * dim)), dim3(256), 0, st, nrow, dim, diag, e, shift, r, out);
}
void row_norms2(hipStream_t st, int nrow, int dim, const double* x, double* out) {
  hipLaunchKernelGGL(k_row_norms2, dim3(nrow), dim3(256), 0, st, nrow, dim, x, out);
}
void row_scale(hipStream_t st, int nrow, int dim, double* x, const double* s) {
  hipLaunchKernelGGL(k_row_scale, dim3(nblocks((long)nrow * dim)), dim3(256), 0, st, nrow, dim, x, s);
}

}  // namespace xt

namespace xt {
void xsf_split4(hipStream_t st, int nz, int O, int V, int nc, int no, const double* ze, double* zb) {
  hipLaunchKernelGGL(k_xsf_split4, dim3(nblocks(4L * nz * O * V)), dim3(256), 0, st, nz, O, V, nc, no, ze, zb);
}
void xsf_combine4(hipStream_t st, int nz, int O, int V, int nc, int no, const W16& w16, const double* yb,
                  double* acc) {
  hipLaunchKernelGGL(k_xsf_combine4, dim3(nblocks((long)nz * O * V)), dim3(256), 0, st, nz, O, V, nc, no, w16, yb,
                     acc);
}
}  // namespace xt
