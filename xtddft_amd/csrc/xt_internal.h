// Internal declarations shared by the HIP translation units of libxtddft_amd.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#define XT_OK 0
#define XT_ERR_ARG -1
#define XT_ERR_OOM -2
#define XT_ERR_HIP -3
#define XT_ERR_STATE -4
#define XT_ERR_RCCL -5

namespace xt {

// Buffer descriptor over a wave-uniform base (readfirstlane'd so the compiler can prove it:
// cdna_hip_programming.md T20); loads through it take a 32-bit lane offset and a scalar one,
// so no 64-bit address arithmetic runs on the VALU.  The range is 2 GB from the base.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const double* p) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ double bld8(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}

// sum of v over the four 16-lane rows of a wave (lanes l, l^16, l^32, l^48), in every lane:
// two row-pair swaps of both halves of the double (v_permlane16_swap, v_permlane32_swap)
__device__ __forceinline__ double rows4(double v) {
  auto pair = [](double x, bool p32) __attribute__((always_inline)) {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto a = p32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                       : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = p32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                       : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
  };
  return pair(pair(v, false), true);
}

// Fused XC grid contractions (GEMM modes, xt_gemm.hip).  Spin-channel x trial
// vector pairs xg < nx, virtual index a < V, grid point g.
//  mode 1 "rho forward":  rows m = 16 xg + a_l, reduce index r = a-block (a = 16 r + a_l),
//    A(r, m, k) = A[k sAk + xg ablk + 16 r + a_l]  (W = PhiO Zp, never stored);
//    out: rho[g rg + 3 xg + c] = sum_a W[g, xg, a] w[c wc + g wg + a]   (c < 3)
//  mode 2 "M backward":   B(g, n) generated as sum_c rho[g rg + 3 xg + c] w[c wc + g wg + a]
//    with n -> (xg, a) in (XC_M_BN / 16) x 16 blocks (xg-block fastest); C column xg V + a;
//    N must be xc_m_cols(nx, V, mbn).
int xc_m_bn();                // mode 2 column-tile width (64)
inline int xc_m_cols(int nx, int V, int bn) {
  return ((nx + bn / 16 - 1) / (bn / 16)) * ((V + 15) / 16) * bn;
}
struct XcFuse {
  int mode = 0;
  const double* w = nullptr;   // weights (grid gradients of the virtual MOs)
  long wc = 0, wg = 0;
  double* rho = nullptr;       // mode 1 output / mode 2 input, (g, xg, 3)
  long rg = 0;
  long ablk = 0;               // mode 1: A offset between consecutive xg
  int V = 0, nx = 0;
  int mbn = 64;                // mode 2: column-tile width (xc_m_bn())
};

// Public-facing GEMM description (see xt_gemm.hip for the contraction).
struct GemmDesc {
  int M = 0, N = 0, K = 0, R = 1;
  int nb1 = 1, nb2 = 1;               // batch = nb1 x nb2
  const double* A = nullptr;
  long sAm = 0, sAk = 0, sAr = 0, sAb1 = 0, sAb2 = 0;
  const double* B = nullptr;
  long sBk = 0, sBn = 0, sBr = 0, sBb1 = 0, sBb2 = 0;
  double* C = nullptr;
  long ldc = 0, sCb1 = 0, sCb2 = 0;
  double alpha = 1.0, beta = 0.0;
  // two-level rows (rdiv > 0; plain mode, A m-contiguous): row m = (hi, lo) = (m / rdiv,
  // m % rdiv) sits at hi sAm_hi + lo in A and at hi sC_hi + lo ldc in C -- e.g. the stored
  // exchange build's rows (i, j) over a padded MO factor and a padded Kx
  int rdiv = 0;
  long sAm_hi = 0, sC_hi = 0;
  int max_split = 0;                  // 0 = heuristic
  int tag = 0;                        // kernel identity for profiling (see xt_gemm.hip)
  double flops = 0.0;                 // algorithmic flops for profiling (0: 2 M N K R batch)
  double bytes = 0.0;                 // compulsory HBM bytes for profiling (0: A, B, C once)
  XcFuse fz;                          // fused XC mode (fz.mode != 0)
};

struct GemmParams {
  int M, N, K, R;
  int nbatch, nb2, nsplit;
  const double* A; long sAm, sAk, sAr, sAb1, sAb2;
  const double* B; long sBk, sBn, sBr, sBb1, sBb2;
  double* C; long ldc, sCb1, sCb2;
  double alpha, beta;
  double* ws;
  XcFuse fz;
  int rdiv; long sAm_hi, sC_hi;       // two-level rows (GemmDesc)
};

void plan_gemm(const GemmDesc& d, GemmParams* p, int* cfg);
// skinny streaming GEMM (xt_exch.hip): C = alpha A B + beta C for M <= 48 rows,
// B (K x N, 16-B aligned rows of stride ldb: a multiple of 4 >= N, the padding
// readable) streamed once from HBM
constexpr int SKINNY_MAX_M = 160;   // 48-row tile up to 48 rows, 160-row tile beyond
// B must stay readable (finite, zero-filled) SKINNY_B_SLACK rows past row K - 1: the
// streaming loads run a whole chunk plus the prefetch ring past a split's end
constexpr int SKINNY_B_SLACK = 128;
int skinny_splits(int N, int K);
size_t skinny_workspace_bytes(int M, int N, int K);
int skinny_gemm(int M, int N, int K, double alpha, const double* A, long lda, const double* B, long ldb,
                double beta, double* C, long ldc, double* ws, size_t ws_bytes, hipStream_t st);
// dedicated XC M-backward (xt_xcm.hip): accT[i][xg V + a] += sum_g PhiO[g][i] *
// sum_c wv[g][xg][c] dPhiV_c[g][a], O <= 128; split over g through a workspace
// the grid arrays it reads (PhiO, dPhiV, wv) must stay readable XC_GRID_SLACK rows past
// the chunk's last point: PhiO / dPhiV finite there, wv ZERO there (the kernel does not
// mask grid points past n)
constexpr int XC_GRID_SLACK = 64;
// Trial-pair segments for the dedicated XC kernels (Davidson steps with nx not a multiple
// of 8): nx pairs covered by blocks of 8 / 4 / 2 / 1 pairs minimising the summed per-block
// cost (cost[k]: a block of 8 >> k pairs); returns the segment count, segment s covering the
// next cnt[s] pairs with blocks of pb[s] pairs, largest blocks first (one launch each)
inline int xc_pair_segments(int nx, const double cost[4], int pb[4], int cnt[4]) {
  if (nx <= 0) return 0;
  double best[1025];
  int pick[1025];
  const int m_max = nx < 1024 ? nx : 1024;
  best[0] = 0.0;
  for (int m = 1; m <= m_max; ++m) {
    best[m] = 1e300; pick[m] = 0;
    for (int k = 0; k < 4; ++k) {
      const int sz = 8 >> k, rest = m > sz ? m - sz : 0;
      const double c = cost[k] + best[rest];
      if (c < best[m] - 1e-12) { best[m] = c; pick[m] = k; }
    }
  }
  int pairs[4] = {nx - m_max, 0, 0, 0};   // beyond 1024 pairs: 8-pair blocks
  for (int m = m_max; m > 0;) {
    const int k = pick[m], sz = 8 >> k;
    pairs[k] += m < sz ? m : sz;
    m = m > sz ? m - sz : 0;
  }
  int ns = 0;
  for (int k = 0; k < 4; ++k)
    if (pairs[k] > 0) { pb[ns] = 8 >> k; cnt[ns] = pairs[k]; ++ns; }
  return ns;
}
size_t xc_back_m_workspace_bytes(int O, int nx, int V, int n);
int xc_back_m(int O, int nx, int V, int n, const double* PO, long ldp, const double* W, long wc, long wg,
              const double* R, long rg, double* C, long ldc, double* ws, size_t ws_bytes, hipStream_t st);
// dedicated XC rho-forward (xt_xcw.hip): rhoW[g][xg][c] = sum_a dPhiV_c[g][a] sum_i
// PhiO[g][i] Zp[i zi + xg zx + a]; reads Zp up to 7 rows past O and WA - 1 columns past
// V (zeroed slack), grid arrays XC_GRID_SLACK rows past n
size_t xc_rho_w_lds_bytes(int O);
// the same for O <= 48 (xt_xcws.hip): blocks of 64 points over every pair, gradient weights
// staged once per 64-virtual chunk; same operand slack; XT_ERR_ARG past O = 48
size_t xc_rho_ws_lds_bytes(int O);
int xc_rho_ws(int O, int nx, int V, int n, const double* PO, long ldp, const double* Z, long zi, long zx,
              const double* W, long wc, long wg, double* R, long rg, hipStream_t st);
// Coulomb integrals over Cartesian Gaussians and AO values on the grid (xt_int.hip):
// orbital l <= 3, total Hermite order 2 l_orb + l_ket <= kIntMaxL; AO values l <= kAoMaxL
constexpr int kIntMaxLOrb = 3, kIntMaxL = 13, kAoMaxL = 4;
int int2e_cart(int npair, const int* pair_info, const double* pair_prim, const double* eab, int nket,
               const int* ket_info, const double* ket_prim, const double* ek, int lmax_orb, int lket,
               double omega, const double* q_bra, const double* q_ket, double q_thr, int diag, double* out,
               long ldo, hipStream_t st);
int eval_ao(int ngrid, const double* coords, int nshell, const int* shell_info, const double* dat,
            const double* sph, const double* norm, int deriv, double* out, long ldo, long comp_stride,
            hipStream_t st);
int xc_rho_w(int O, int nx, int V, int n, const double* PO, long ldp, const double* Z, long zi, long zx,
             const double* W, long wc, long wg, double* R, long rg, hipStream_t st);
size_t dgemm_workspace_bytes(const GemmDesc& d);
int dgemm(const GemmDesc& d, hipStream_t st, double* ws, size_t ws_bytes);

}  // namespace xt
