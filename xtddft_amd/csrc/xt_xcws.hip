// XC rho-forward (W route) for small occupied spaces (O <= 48: C2, C5 and the small
// molecules), the same contraction as xt_xcw.hip (XTDA.py:514, nr_uks_fxc):
//
//   rhoW[g][xg][c] = sum_a dPhiV_c[g][a] * sum_i PhiO[g][i] * Zp[i][xg][a]     (c < 3)
//
// At O = 37 an a-tile's K loop is 10 k-steps (80 MFMAs per wave), so the per-a-tile
// costs of the large-O kernel (xt_xcw.hip) -- its barrier, the weight image staged per 8-pair set
// and re-read from HBM by every one of the nx / 8 sets -- are 2.7x heavier relative to
// the MFMAs there (0.41 of the FP64 roof at C5).  This kernel turns the loops around:
//   * a block owns 64 grid points and ALL trial pairs: wave w walks pairs w, w + 8, ...;
//   * the gradient weights dPhiV_c[g][a] of the block's points are staged into LDS once
//     per 64-virtual chunk (one or two a-tiles), shared by every pair -- each weight is
//     read from HBM once, and there is no barrier inside the pair loop;
//   * PhiO (the MFMA B operand, K = i) is resident in LDS for the block's lifetime;
//   * Zp (the A operand, rows = virtuals) streams global -> registers through a ring of
//     2 KP slots: one whole a-tile of k-steps ahead, so every a-tile starts at slot 0
//     and the walk over (chunk, pair, a-tile) prefetches across pairs and chunks;
//   * the rows4 reduction of a pair's per-lane partials runs once per (pair, chunk); the
//     chunks of one pair are summed in the output (the same lane reads back what it wrote
//     a chunk earlier; the old value is prefetched when the pair starts).
//   * the next chunk's weight lines are pulled into L2 during the wave's last pair of a chunk;
//   * the blocks of the last, partial round over the CUs split their trial pairs S ways
//     (pair subsets p = s (mod S)): that round then takes a fraction of a block time
//     instead of a whole one (n = 200 000, 3125 = 12 x 256 + 53 blocks: 0.814 -> 0.800 ms
//     at S = 4, tools/xcws_probe.hip).
// Operand conventions are those of xc_rho_w (xt_internal.h): Zp readable 7 rows past O
// and 31 columns past V (zeroed slack), PhiO / dPhiV rows past n are not read.
#include <hip/hip_runtime.h>
#include <mutex>
#include <type_traits>
#include "xt_internal.h"

namespace xt {

#define XT_INLINE __attribute__((always_inline))
typedef double d4s __attribute__((ext_vector_type(4)));
typedef double d2s __attribute__((ext_vector_type(2)));

namespace {
constexpr int SW_WA = 32;                  // virtuals per a-tile (2 MFMA row sub-tiles)
constexpr int SW_TMA = SW_WA / 16;
constexpr int SW_NW = 8;                   // waves per block
constexpr int SW_TNG = 4;                  // 16-point column sub-tiles (64 grid points)
constexpr int SW_GB = 16 * SW_TNG;
constexpr int SW_AC = 2 * SW_WA;           // virtuals per staged chunk
constexpr int SW_WP = SW_AC + 2;           // weight pitch, 2 mod 32: conflict-free ds_read_b64
constexpr int SW_PP = 52;                  // PhiO pitch, 4 mod 8: conflict-free ds_read_b128
constexpr int SW_W_IMG = 3 * SW_GB * SW_WP;
// The single k-step of an odd KS reads one double per lane (rows 8 KP + q): from the PhiO
// image (pitch 52, 8 mod 16 in bank pairs) the 16 lanes of a ds_read2 group would hit 4
// bank pairs 4 times each (measured: 0.41 SQ_LDS_BANK_CONFLICT cycles per LDS instruction
// at C2, O = 34); those four rows get their own image of odd pitch 5 (16 distinct pairs).
constexpr int SW_P1 = 5;
constexpr size_t SW_LDS = sizeof(double) * ((size_t)SW_GB * SW_PP + SW_W_IMG + (size_t)SW_GB * SW_P1);
constexpr int SW_KS_MAX = 12;              // k-steps: KI = 4 KS <= 48 <= SW_PP
}  // namespace

// KS = ceil(O / 4) k-steps per a-tile: KS / 2 k-step pairs (one ds_read_b128 of PhiO per
// pair) and, for odd KS, one single k-step (O = 34: 9 k-steps instead of 10)
template <int KS>
__global__ void __launch_bounds__(64 * SW_NW) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_xc_rho_ws(int O, int nx, int V, int n,
            const double* __restrict__ PO, long ldp,
            const double* __restrict__ Z, long zi, long zx,
            const double* __restrict__ Wg, long wc, long wg,
            double* __restrict__ Rout, long rg, int nb_main, int split) {
  constexpr int NT = 64 * SW_NW, KP = KS / 2, KI = 4 * KS, ZD = KS;
  constexpr bool ODD = (KS & 1) != 0;
  constexpr int W_LD = 3 * SW_GB * SW_AC / NT;       // weight elements staged per thread and chunk (24)
  static_assert(W_LD * NT == 3 * SW_GB * SW_AC && NT == 8 * SW_AC, "weight staging map");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* sP = sm;                                   // [GB][PP]
  double* sW = sm + SW_GB * SW_PP;                   // [3][GB][WP]
  double* sP1 = sW + SW_W_IMG;                       // [GB][P1]: PhiO rows 8 KP .. 8 KP + 3 (odd KS)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  // block -> 64-point block pb and pair subset {pbase + pstride j}: blocks past nb_main are
  // the last round's point blocks, each split over `split` blocks
  const int tb = (int)blockIdx.x - nb_main;
  const int pb = tb < 0 ? (int)blockIdx.x : nb_main + tb / split;
  const int pbase = tb < 0 ? 0 : tb % split, pstride = tb < 0 ? 1 : split;
  const int g0 = pb * SW_GB;
  const int nat = (V + SW_WA - 1) / SW_WA;           // a-tiles
  const int nck = (nat + 1) / 2;                     // chunks of two a-tiles
  const int nxs = (nx - pbase + pstride - 1) / pstride;   // pairs of the block
  const int npw = wave < nxs ? (nxs - wave + SW_NW - 1) / SW_NW : 0;   // pairs of this wave
  auto pair_of = [&](int pi) XT_INLINE { return pbase + pstride * (wave + SW_NW * pi); };

  // ---- PhiO tile -> LDS, once (rows past O and points past n as zero) ---------------
  for (int p = tid; p < KI * SW_GB; p += NT) {
    const int g = p / KI, i = p % KI;
    const double v = (i < O && g0 + g < n) ? PO[(long)(g0 + g) * ldp + i] : 0.0;
    sP[g * SW_PP + i] = v;
    if (ODD && i >= 8 * KP) sP1[g * SW_P1 + i - 8 * KP] = v;
  }

  // ---- Zp walk: units (chunk, pair, a-tile of the chunk) in order; lane (q, r16) of
  // k-step s supplies row i = 8 (s / 2) + 2 q + (s & 1) (the single step: 8 KP + q) of
  // virtual 16 t + r16 of the unit's a-tile.  zq[s] holds the current unit's k-step s until its MFMAs issue, then the next
  // unit's (the last unit reloads itself: never consumed).
  const __amdgpu_buffer_rsrc_t zrs = rsrc_of(Z);
  const unsigned z_off = (unsigned)(((long)2 * q * zi + r16) * 8);
  const unsigned z_off1 = (unsigned)(((long)q * zi + r16) * 8);
  int wc_ = 0, wp_ = 0, wt_ = 0;                     // walker: chunk, pair index, tile in chunk
  auto unit_off = [&](int ch, int pi, int tc) XT_INLINE {
    return (int)((((long)pair_of(pi)) * zx + (long)(2 * ch + tc) * SW_WA) * 8);
  };
  auto advance = [&]() XT_INLINE {                   // walker -> next unit (stays on the last)
    const int ntc = 2 * wc_ + 1 < nat ? 2 : 1;
    if (wt_ + 1 < ntc) { ++wt_; return; }
    if (wp_ + 1 < npw) { ++wp_; wt_ = 0; return; }
    if (wc_ + 1 < nck) { ++wc_; wp_ = 0; wt_ = 0; }
  };
  double zq[ZD][SW_TMA];
  auto load_z = [&](int s, int uoff) XT_INLINE {     // s compile-time after unrolling
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

  // B fragments of k-step pair p: columns 16 j + r16, rows 8 p + 2 q + {0, 1}; of the
  // single k-step: rows 8 KP + q
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
  auto bfirst = [&]() XT_INLINE {                   // the B operand of a tile's first k-step
    if constexpr (KP > 0) bread(0, bq[0]);
    else bread1();
  };

  d4s acc[SW_TMA][SW_TNG];
  double racc[SW_TNG][3];
#pragma unroll
  for (int j = 0; j < SW_TNG; ++j)
#pragma unroll
    for (int c = 0; c < 3; ++c) racc[j][c] = 0.0;

  // one a-tile (chunk-local tile tc) of the current unit: K loop, then the contraction
  // racc[j][c] += sum_{t, r} T[a = 16 t + q + 4 r][g = 16 j + r16] * w_c[g][a]
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
        load_z(s, unext);
      }
    }
    if constexpr (ODD) {
#pragma unroll
      for (int t = 0; t < SW_TMA; ++t)
#pragma unroll
        for (int j = 0; j < SW_TNG; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(zq[KS - 1][t], bs[j],
                                                           KS == 1 ? (d4s){0.0, 0.0, 0.0, 0.0} : acc[t][j], 0, 0, 0);
      load_z(KS - 1, unext);
    }
    bfirst();                                        // the next tile's first k-step (PhiO never changes)
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

  // weight staging of chunk ch: thread element k -> plane k / 8, grid row wr + 8 (k % 8),
  // column wa of the chunk (virtuals past V and points past n as zero)
  const int wa = tid & (SW_AC - 1), wr = tid / SW_AC;
  auto stage = [&](int ch) XT_INLINE {
    const int a = ch * SW_AC + wa;
    double rw[W_LD];
#pragma unroll
    for (int k = 0; k < W_LD; ++k) {
      const int g = g0 + wr + 8 * (k % 8);
      rw[k] = (a < V && g < n) ? Wg[(long)(k / 8) * wc + (long)g * wg + a] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < W_LD; ++k) sW[((k / 8) * SW_GB + wr + 8 * (k % 8)) * SW_WP + wa] = rw[k];
  };

  double sink = 0.0;
  for (int ch = 0; ch < nck; ++ch) {
    if (ch > 0) __syncthreads();                     // every wave is done with chunk ch - 1
    stage(ch);
    __syncthreads();
    if (npw == 0) continue;
    if (ch == 0) bfirst();
    const int ntc = 2 * ch + 1 < nat ? 2 : 1;
    for (int pi = 0; pi < npw; ++pi) {
      const int xg = pair_of(pi);
      // the chunks before this one left partial sums in the output: prefetch them, lane
      // row q holding (and later storing) column sub-tile j = q
      const int go = g0 + 16 * q + r16;
      double prev[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) prev[c] = (ch > 0 && go < n) ? Rout[(long)go * rg + 3 * xg + c] : 0.0;
      // the wave's last pair of the chunk pulls the next chunk's weight lines into L2 (one
      // 8-byte load per 128-B line: thread lines tid, tid + 512 of 3 x 64 rows x 4 lines), so
      // the staging after the barrier hits L2; the values only feed a sink
      double pf0 = 0.0, pf1 = 0.0;
      if (pi == npw - 1 && ch + 1 < nck) {
        auto line = [&](int L) XT_INLINE {
          const int gl = min(g0 + ((L >> 2) & 63), n - 1);
          const int a = min((ch + 1) * SW_AC + 16 * (L & 3), V - 1);
          return Wg[(long)(L >> 8) * wc + (long)gl * wg + a];
        };
        pf0 = line(tid);
        if (tid < 256) pf1 = line(tid + 512);
      }
      for (int tc = 0; tc < ntc; ++tc) {
        const int un = unit_off(wc_, wp_, wt_);
        advance();
        tile(tc, un);
      }
      sink += pf0 + pf1;
      double tot[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int j = 0; j < SW_TNG; ++j)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const double v = rows4(racc[j][c]);      // the same total in every lane row
          racc[j][c] = 0.0;
          tot[c] = q == j ? v : tot[c];
        }
      if (go < n) {
#pragma unroll
        for (int c = 0; c < 3; ++c) Rout[(long)go * rg + 3 * xg + c] = prev[c] + tot[c];
      }
    }
  }
  if (sink == -1.0e300) Rout[0] = sink;              // never (finite weights): keeps the prefetch
}

size_t xc_rho_ws_lds_bytes(int O) { return (O + 3) / 4 <= SW_KS_MAX ? SW_LDS : (size_t)1 << 40; }

int xc_rho_ws(int O, int nx, int V, int n, const double* PO, long ldp, const double* Z, long zi, long zx,
              const double* W, long wc, long wg, double* R, long rg, hipStream_t st) {
  if (O <= 0 || nx <= 0 || V <= 0 || n <= 0) return 0;
  const int KS = (O + 3) / 4;
  if (KS > SW_KS_MAX) return XT_ERR_ARG;
  // 32-bit buffer offsets over Zp: KI rows (+ the a-tile overhang) of zi doubles
  if ((double)(4 * KS + 1) * (double)zi * 8.0 >= 2147483647.0) return XT_ERR_ARG;
  static std::mutex mu;
  static unsigned long long done[SW_KS_MAX + 1] = {};
  static int ncu[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  int cus = 256;
  if (dev < 64) {
    std::lock_guard<std::mutex> lk(mu);
    if (!ncu[dev] && hipDeviceGetAttribute(&ncu[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu[dev] = 256;
    cus = ncu[dev] > 0 ? ncu[dev] : 256;
  }
  // one block per CU (LDS): the last round's point blocks split their pairs S ways when
  // each part keeps >= 4 pairs and the parts still fit in one round
  const int pblocks = (n + SW_GB - 1) / SW_GB;
  const int tail = pblocks > cus ? pblocks % cus : 0;
  int split = 1;
  for (int sp = 4; sp >= 2 && split == 1; sp /= 2)
    if (tail > 0 && tail * sp <= cus && nx >= 4 * sp) split = sp;
  const int nb_main = pblocks - (split > 1 ? tail : 0);
  const int blocks = nb_main + (split > 1 ? tail * split : 0);
#define XT_WS(K)                                                                                           \
  case K: {                                                                                                \
    {                                                                                                      \
      std::lock_guard<std::mutex> lk(mu);                                                                  \
      if (dev >= 64 || !(done[K] >> dev & 1ull)) {                                                         \
        (void)hipFuncSetAttribute((const void*)k_xc_rho_ws<K>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)SW_LDS);                                                            \
        if (dev < 64) done[K] |= 1ull << dev;                                                              \
      }                                                                                                    \
    }                                                                                                      \
    hipLaunchKernelGGL((k_xc_rho_ws<K>), dim3(blocks), dim3(64 * SW_NW), SW_LDS, st, O, nx, V, n, PO, ldp, Z, \
                       zi, zx, W, wc, wg, R, rg, nb_main, split);                                          \
    break;                                                                                                 \
  }
  switch (KS) {
    XT_WS(1) XT_WS(2) XT_WS(3) XT_WS(4) XT_WS(5) XT_WS(6) XT_WS(7) XT_WS(8) XT_WS(9) XT_WS(10) XT_WS(11) XT_WS(12)
    default: return XT_ERR_ARG;
  }
#undef XT_WS
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
