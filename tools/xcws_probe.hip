// Where the small-O rho-forward kernel (xt_xcws.hip) spends its time: a copy of
// k_xc_rho_ws with diagnostic switches, timed standalone at a config's shape.
//   DIAG bit 0: no gradient contraction (racc update) -- the MFMA stream alone
//   DIAG bit 1: weights staged for chunk 0 only (no barrier / staging after it)
//   DIAG bit 2: Zp loaded once (the ring is never refilled)
//   DIAG bit 3: no per-pair output (rows4 reduction, partial-sum load, store)
//   DIAG bit 6: chunks past 0 keep their barriers but stage no global loads (LDS writes of a constant)
//   DIAG bits 4-5: waves 4..7 sleep 16 / 32 / 64 x 64 cycles after each chunk barrier (phase stagger)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xtddft_amd/csrc tools/xcws_probe.hip -o tools/bin/xcws_probe
// Run:   tools/bin/xcws_probe O nx V n [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../xtddft_amd/csrc/xt_xcws.hip"

namespace xp {
using namespace xt;
#define XT_INLINE __attribute__((always_inline))
typedef double d4s __attribute__((ext_vector_type(4)));
typedef double d2s __attribute__((ext_vector_type(2)));
constexpr int SW_WA = 32, SW_TMA = 2, SW_NW = 8, SW_TNG = 4, SW_GB = 64, SW_AC = 64, SW_WP = 66, SW_PP = 52;
constexpr int SW_W_IMG = 3 * SW_GB * SW_WP, SW_P1 = 5;
constexpr size_t SW_LDS = sizeof(double) * ((size_t)SW_GB * SW_PP + SW_W_IMG + (size_t)SW_GB * SW_P1);

template <int KS, int DIAG>
__global__ void __launch_bounds__(64 * SW_NW) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_probe(int O, int nx, int V, int n, const double* __restrict__ PO, long ldp, const double* __restrict__ Z, long zi,
        long zx, const double* __restrict__ Wg, long wc, long wg, double* __restrict__ Rout, long rg) {
  constexpr int NT = 64 * SW_NW, KP = KS / 2, KI = 4 * KS, ZD = KS;
  constexpr bool ODD = (KS & 1) != 0;
  constexpr int W_LD = 3 * SW_GB * SW_AC / NT;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* sP = sm;
  double* sW = sm + SW_GB * SW_PP;
  double* sP1 = sW + SW_W_IMG;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int g0 = blockIdx.x * SW_GB;
  const int nat = (V + SW_WA - 1) / SW_WA;
  const int nck = (nat + 1) / 2;
  const int npw = wave < nx ? (nx - wave + SW_NW - 1) / SW_NW : 0;
  for (int p = tid; p < KI * SW_GB; p += NT) {
    const int g = p / KI, i = p % KI;
    const double v = (i < O && g0 + g < n) ? PO[(long)(g0 + g) * ldp + i] : 0.0;
    sP[g * SW_PP + i] = v;
    if (ODD && i >= 8 * KP) sP1[g * SW_P1 + i - 8 * KP] = v;
  }
  const __amdgpu_buffer_rsrc_t zrs = rsrc_of(Z);
  const unsigned z_off = (unsigned)(((long)2 * q * zi + r16) * 8);
  const unsigned z_off1 = (unsigned)(((long)q * zi + r16) * 8);
  int wc_ = 0, wp_ = 0, wt_ = 0;
  auto unit_off = [&](int ch, int pi, int tc) XT_INLINE {
    return (int)((((long)(wave + SW_NW * pi)) * zx + (long)(2 * ch + tc) * SW_WA) * 8);
  };
  auto advance = [&]() XT_INLINE {
    const int ntc = 2 * wc_ + 1 < nat ? 2 : 1;
    if (wt_ + 1 < ntc) { ++wt_; return; }
    if (wp_ + 1 < npw) { ++wp_; wt_ = 0; return; }
    if (wc_ + 1 < nck) { ++wc_; wp_ = 0; wt_ = 0; }
  };
  double zq[ZD][SW_TMA];
  auto load_z = [&](int s, int uoff) XT_INLINE {
    const bool single = ODD && s == KS - 1;
    const int so = uoff + (single ? 8 * KP : 8 * (s / 2) + (s & 1)) * (int)zi * 8;
#pragma unroll
    for (int t = 0; t < SW_TMA; ++t) zq[s][t] = bld8(zrs, (single ? z_off1 : z_off) + 128 * t, so);
  };
  if (npw > 0) {
    const int u0 = unit_off(0, 0, 0);
#pragma unroll
    for (int s = 0; s < ZD; ++s) load_z(s, u0);
    advance();
  }
  d2s bq[2][SW_TNG];
  double bs[SW_TNG];
  const double* const b_lane = sP + r16 * SW_PP + 2 * q;
  auto bread = [&](int p, d2s* dst) XT_INLINE {
    const d2s* src = (const d2s*)(b_lane + 8 * p);
#pragma unroll
    for (int j = 0; j < SW_TNG; ++j) dst[j] = src[(16 * j * SW_PP) / 2];
  };
  auto bread1 = [&]() XT_INLINE {
    const double* src = sP1 + r16 * SW_P1 + q;
#pragma unroll
    for (int j = 0; j < SW_TNG; ++j) bs[j] = src[16 * j * SW_P1];
  };
  auto bfirst = [&]() XT_INLINE {
    if constexpr (KP > 0) bread(0, bq[0]);
    else bread1();
  };
  d4s acc[SW_TMA][SW_TNG];
  double racc[SW_TNG][3];
#pragma unroll
  for (int j = 0; j < SW_TNG; ++j)
#pragma unroll
    for (int c = 0; c < 3; ++c) racc[j][c] = 0.0;
  auto tile = [&](int tc, int unext) XT_INLINE {
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      if (p + 1 < KP) bread(p + 1, bq[(p + 1) & 1]);
      else if constexpr (ODD) bread1();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int s = 2 * p + h;
#pragma unroll
        for (int t = 0; t < SW_TMA; ++t)
#pragma unroll
          for (int j = 0; j < SW_TNG; ++j)
            acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(zq[s][t], bq[p & 1][j][h],
                                                             s == 0 ? (d4s){0.0, 0.0, 0.0, 0.0} : acc[t][j], 0, 0, 0);
        if (!(DIAG & 4)) load_z(s, unext);
      }
    }
    if constexpr (ODD) {
#pragma unroll
      for (int t = 0; t < SW_TMA; ++t)
#pragma unroll
        for (int j = 0; j < SW_TNG; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(zq[KS - 1][t], bs[j],
                                                           KS == 1 ? (d4s){0.0, 0.0, 0.0, 0.0} : acc[t][j], 0, 0, 0);
      if (!(DIAG & 4)) load_z(KS - 1, unext);
    }
    bfirst();
    if constexpr (DIAG & 1) {
#pragma unroll
      for (int t = 0; t < SW_TMA; ++t)
#pragma unroll
        for (int j = 0; j < SW_TNG; ++j) racc[j][t] += acc[t][j][0];
      return;
    }
    const double* w = sW + r16 * SW_WP + tc * SW_WA + q;
    constexpr int JH = SW_TNG / 2;
    double wb[2][JH * 3];
    auto wread = [&](int hh, double* dst) XT_INLINE {
      const int rw_ = hh / 2, j0 = (hh % 2) * JH;
      const int t = rw_ / 4, r = rw_ % 4;
#pragma unroll
      for (int jj = 0; jj < JH; ++jj)
#pragma unroll
        for (int c = 0; c < 3; ++c) dst[3 * jj + c] = w[(c * SW_GB + 16 * (j0 + jj)) * SW_WP + 16 * t + 4 * r];
    };
    wread(0, wb[0]);
#pragma unroll
    for (int hh = 0; hh < 8 * SW_TMA; ++hh) {
      if (hh + 1 < 8 * SW_TMA) wread(hh + 1, wb[(hh + 1) & 1]);
      const int rw_ = hh / 2, j0 = (hh % 2) * JH;
      const int t = rw_ / 4, r = rw_ % 4;
#pragma unroll
      for (int jj = 0; jj < JH; ++jj)
#pragma unroll
        for (int c = 0; c < 3; ++c) racc[j0 + jj][c] += acc[t][j0 + jj][r] * wb[hh & 1][3 * jj + c];
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const int wa = tid & (SW_AC - 1), wr = tid / SW_AC;
  auto stage = [&](int ch) XT_INLINE {
    const int a = ch * SW_AC + wa;
    double rw[W_LD];
#pragma unroll
    for (int k = 0; k < W_LD; ++k) {
      const int g = g0 + wr + 8 * (k % 8);
      if ((DIAG & 64) && ch > 0) rw[k] = 0.5;
      else rw[k] = (a < V && g < n) ? Wg[(long)(k / 8) * wc + (long)g * wg + a] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < W_LD; ++k) sW[((k / 8) * SW_GB + wr + 8 * (k % 8)) * SW_WP + wa] = rw[k];
  };
  for (int ch = 0; ch < nck; ++ch) {
    if (!(DIAG & 2) || ch == 0) {
      if (ch > 0) __syncthreads();
      stage(ch);
      __syncthreads();
    }
    if (npw == 0) continue;
    if constexpr ((DIAG & 48) != 0) {
      if (wave >= 4) {
        if constexpr ((DIAG & 48) == 16) __builtin_amdgcn_s_sleep(16);
        else if constexpr ((DIAG & 48) == 32) __builtin_amdgcn_s_sleep(32);
        else { __builtin_amdgcn_s_sleep(64); }
      }
    }
    if (ch == 0) bfirst();
    const int ntc = 2 * ch + 1 < nat ? 2 : 1;
    for (int pi = 0; pi < npw; ++pi) {
      const int xg = wave + SW_NW * pi;
      const int go = g0 + 16 * q + r16;
      double prev[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) prev[c] = (ch > 0 && go < n) ? Rout[(long)go * rg + 3 * xg + c] : 0.0;
      for (int tc = 0; tc < ntc; ++tc) {
        const int un = unit_off(wc_, wp_, wt_);
        advance();
        tile(tc, un);
      }
      if constexpr ((DIAG & 8) != 0) {   // keep the MFMA chain live without the output path
        if (racc[0][0] == -1.2345e300) Rout[go] = racc[1][1] + racc[2][2] + racc[3][0];
        continue;
      }
      double tot[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int j = 0; j < SW_TNG; ++j)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const double v = rows4(racc[j][c]);
          racc[j][c] = 0.0;
          tot[c] = q == j ? v : tot[c];
        }
      if (go < n) {
#pragma unroll
        for (int c = 0; c < 3; ++c) Rout[(long)go * rg + 3 * xg + c] = prev[c] + tot[c];
      }
    }
  }
}
}  // namespace xp

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int DIAG>
static float run_probe(int O, int nx, int V, int n, const double* PO, long ldp, const double* Z, long zi, long zx,
                       const double* W, long wc, long wg, double* R, long rg, int reps) {
  constexpr int KS = 9;
  CK(hipFuncSetAttribute((const void*)xp::k_probe<KS, DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)xp::SW_LDS));
  const int blocks = (n + 63) / 64;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL((xp::k_probe<KS, DIAG>), dim3(blocks), dim3(512), xp::SW_LDS, 0, O, nx, V, n, PO, ldp, Z, zi, zx,
                       W, wc, wg, R, rg);
  CK(hipEventRecord(a));
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL((xp::k_probe<KS, DIAG>), dim3(blocks), dim3(512), xp::SW_LDS, 0, O, nx, V, n, PO, ldp, Z, zi, zx,
                       W, wc, wg, R, rg);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int O = argc > 1 ? atoi(argv[1]) : 34, nx = argc > 2 ? atoi(argv[2]) : 20;
  const int V = argc > 3 ? atoi(argv[3]) : 146, n = argc > 4 ? atoi(argv[4]) : 216000;
  const int reps = argc > 5 ? atoi(argv[5]) : 20;
  if ((O + 3) / 4 != 9) { printf("probe is built for KS = 9 (O 33..36)\n"); return 1; }
  const long ldp = 180, zi = (long)nx * V, zx = V, wg = ldp, wc = (long)n * ldp, rg = 3L * nx;
  const size_t nP = (size_t)4 * n * ldp, nZ = (size_t)(O + 8) * zi + 64, nR = (size_t)(n + 64) * rg;
  std::vector<double> h(nP > nZ ? nP : nZ);
  srand(7);
  for (auto& v : h) v = (double)rand() / RAND_MAX - 0.5;
  double *P, *Z, *R0, *R1;
  CK(hipMalloc(&P, nP * 8)); CK(hipMalloc(&Z, nZ * 8)); CK(hipMalloc(&R0, nR * 8)); CK(hipMalloc(&R1, nR * 8));
  CK(hipMemcpy(P, h.data(), nP * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Z, h.data(), nZ * 8, hipMemcpyHostToDevice));
  CK(hipMemset(R0, 0, nR * 8)); CK(hipMemset(R1, 0, nR * 8));
  const double* W = P + (size_t)n * ldp;   // gradient planes 1..3
  // product kernel vs the probe copy (DIAG 0): same output
  if (xt::xc_rho_ws(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R0, rg, 0)) { printf("launch failed\n"); return 1; }
  hipLaunchKernelGGL((xp::k_probe<9, 0>), dim3((n + 63) / 64), dim3(512), xp::SW_LDS, 0, O, nx, V, n, P, ldp, Z, zi,
                     zx, W + 34, wc, wg, R1, rg);
  CK(hipDeviceSynchronize());
  std::vector<double> r0(nR), r1(nR);
  CK(hipMemcpy(r0.data(), R0, nR * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1.data(), R1, nR * 8, hipMemcpyDeviceToHost));
  double md = 0, mx = 0;
  for (size_t i = 0; i < nR; ++i) { md = fmax(md, fabs(r0[i] - r1[i])); mx = fmax(mx, fabs(r1[i])); }
  printf("product vs probe copy: max abs diff %.3e, rel %.3e\n", md, md / mx);
  const double fl = 2.0 * n * nx * (double)O * V;
  auto rep = [&](const char* name, float ms) { printf("%-34s %8.4f ms  %6.2f TF strict  frac %.3f\n", name, ms, fl / ms / 1e9, fl / ms / 1e9 / 78.6); };
  auto time_product = [&]() {
    for (int w = 0; w < 3; ++w) xt::xc_rho_ws(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R0, rg, 0);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int w = 0; w < reps; ++w) xt::xc_rho_ws(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R0, rg, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
  };
  for (int it = 0; it < 2; ++it) {
    rep("product kernel", time_product());
    rep("full (DIAG 0)", run_probe<0>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("no contraction (1)", run_probe<1>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("weights once (2)", run_probe<2>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("Zp once (4)", run_probe<4>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("MFMA only (7)", run_probe<7>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("MFMA only, no output (15)", run_probe<15>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("barriers, no staging loads (64)", run_probe<64>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("stagger 16 (16)", run_probe<16>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("stagger 32 (32)", run_probe<32>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("stagger 64 (48)", run_probe<48>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
    rep("weights once + no contraction (3)", run_probe<3>(O, nx, V, n, P, ldp, Z, zi, zx, W + 34, wc, wg, R1, rg, reps));
  }
  return 0;
}
