// XC rho-forward (W route) as a dedicated kernel: the gradient-of-virtual half of
// the transition-density gradient that nr_uks_fxc contracts (XTDA.py:514):
//
//   rhoW[g][xg][c] = sum_a dPhiV_c[g][a] * sum_i PhiO[g][i] * Zp[i][xg][a]     (c < 3)
//
// The intermediate T[g][xg][a] = sum_i PhiO Zp (nx V values per grid point) never
// leaves registers.  MFMA orientation: rows = virtuals a, columns = grid points g,
// K = occupied i.  A block covers 8 trial pairs and 64 grid points; each of its 8
// waves owns one pair (one block per CU):
//   * A = Zp[i][xg][a] (16 contiguous a per fragment row): loaded straight from
//     global memory into registers through a 4-k-step ring (each wave's own pairs);
//   * B = PhiO[g][i]: the block's 16 TNG x O tile, loaded ONCE per block into LDS
//     and resident for the whole a loop;
//   * after each 32-wide a-tile's K loop the accumulators T[a][g] are contracted
//     with dPhiV_c[g][a] (staged per a-tile in LDS, shared by the block's waves)
//     into per-lane partial sums racc[j][c] -- the
//     sum over a stays in-lane (rows a of a lane are q + 4 reg + 16 t) and only the
//     final 4-row reduction crosses lanes, once per block.
// One barrier per a-tile (26 k-steps x 8 MFMAs per wave at O = 101).
// LDS images are [row][g] with g XOR-swizzled by h(row) = (row & 15) | (row & 1) << 4:
// the global loads run along the row index (coalesced), so 16 lanes of a
// ds_write_b64 group write 16 consecutive rows at one g -> 16 distinct bank pairs;
// the fragment / weight reads (16 consecutive g, two rows of opposite parity per
// 32-lane group) land in opposite bank halves.
#include <hip/hip_runtime.h>
#include <mutex>
#include <type_traits>
#include "xt_internal.h"

namespace xt {

#define XT_INLINE __attribute__((always_inline))
typedef double d4w __attribute__((ext_vector_type(4)));

constexpr int WA = 32;           // virtuals per a-tile (2 MFMA row sub-tiles)
constexpr int TMA = WA / 16;
constexpr int WXB = 8;           // trial pairs per block (one per wave)
constexpr int ZD = 4;            // Zp prefetch ring depth (k-steps; 2 measured +6.5 %, 6 +2.8 %, 8 spills)
constexpr int TNG = 4;           // 16-point column sub-tiles per block (64 grid points)

__device__ __forceinline__ int swz(int row) { return (row & 15) | ((row & 1) << 4); }

// transposing 4-row sum (lanes l, l^16, l^32, l^48): every lane ends with the total
__device__ __forceinline__ double rows4(double v) {
  auto pair = [](double x, bool p32) XT_INLINE {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto a = p32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                       : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = p32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                       : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
  };
  return pair(pair(v, false), true);
}

// PB trial pairs per block (8, 4, 2, 1; Davidson steps with few new vectors): the
// H = 8 / PB waves of a pair split each a-tile's k-steps into H even ranges, contract
// their partial T with the same staged weights (the contraction is linear in T) and
// their partial sums are added through LDS once at the end -- every wave of the block
// works when nx < 8, and the weight staging stays one image per a-tile.
template <int PB>
__global__ void __launch_bounds__(64 * WXB) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_xc_rho_w(int O, int nx, int V, int n,
           const double* __restrict__ PO, long ldp,
           const double* __restrict__ Z, long zi, long zx,
           const double* __restrict__ Wg, long wc, long wg,
           double* __restrict__ Rout, long rg) {
  constexpr int GB = 16 * TNG;                 // grid points per block
  constexpr int W_IMG = 3 * WA * GB;           // one weight buffer (doubles)
  constexpr int NT = 64 * WXB;                 // threads per block
  // each a-tile's weights are staged in two halves (loaded before / stored after each half
  // of the K loop), 6 staging registers instead of 12
  constexpr int W_LD = W_IMG / NT / 2;         // weight elements staged per thread and half
  static_assert(W_IMG % (2 * NT) == 0, "weight staging map");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int KI = (O + 7) & ~7;                 // occupied rows in the image (k-steps even)
  double* sP = sm;                             // [KI][GB]
  double* sW = sm + KI * GB;                   // [2][3][WA][GB]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;

  // block -> (xg-set, g-tile), g-tile fastest within an XCD's contiguous range: the
  // blocks resident on one XCD share the xg-set's Zp slice in its L2
  const int ntg = (n + GB - 1) / GB;
  const int nblk = gridDim.x;
  int lid = blockIdx.x;
  {
    const int xcd = lid & 7, idx = lid >> 3, qn = nblk >> 3, rem = nblk & 7;
    lid = xcd * qn + (xcd < rem ? xcd : rem) + idx;
  }
  // (trial-pair sets of one g-tile side by side instead, sharing its gradient weights
  // in L2: neutral, 168.1-168.3 vs 168.2-168.6 ms/step)
  constexpr int H = WXB / PB;                  // waves per pair
  const int gt = lid % ntg, xs = lid / ntg;
  const int g0 = gt * GB, x0 = xs * PB;
  const int pl = wave % PB, h = wave / PB;
  const int xg = x0 + pl;                      // this wave's trial pair
  const int nat = (V + WA - 1) / WA;
  const int KS = KI / 4;
  // this wave's k-steps of every a-tile: [s_lo, s_hi), even bounds (the ring phase stays even)
  const int s_lo = H == 1 ? 0 : 2 * ((h * (KS / 2)) / H), s_hi = H == 1 ? KS : 2 * (((h + 1) * (KS / 2)) / H);
  const bool wave_on = H == 1 ? xg < nx : (xg < nx && s_hi > s_lo);

  // ---- PhiO tile -> LDS (once) ----------------------------------------------
  for (int p = tid; p < KI * GB; p += NT) {
    const int g = p / KI, i = p % KI;
    const double v = i < O ? PO[(long)(g0 + g) * ldp + i] : 0.0;   // rows past n: zeroed slack
    sP[i * GB + (g ^ swz(i))] = v;
  }
  // ---- weights of a-tile `at` (global -> registers -> LDS) -------------------
  double rw[W_LD];
  auto load_w = [&](int at, int ph) XT_INLINE {
#pragma unroll
    for (int e = 0; e < W_LD; ++e) {
      const int p = tid + NT * (e + ph * W_LD), c = p / (WA * GB), g = (p / WA) % GB, a = p % WA;
      rw[e] = Wg[c * wc + (long)(g0 + g) * wg + min(at * WA + a, V - 1)];
    }
  };
  auto store_w = [&](int buf, int at, int ph) XT_INLINE {
#pragma unroll
    for (int e = 0; e < W_LD; ++e) {
      const int p = tid + NT * (e + ph * W_LD), c = p / (WA * GB), g = (p / WA) % GB, a = p % WA;
      sW[buf * W_IMG + (c * WA + a) * GB + (g ^ swz(a))] = at * WA + a < V ? rw[e] : 0.0;
    }
  };
  load_w(0, 0);
  store_w(0, 0, 0);
  load_w(0, 1);
  store_w(0, 0, 1);

  // ---- Zp ring: k-step u of the whole a loop (a-tile u / KS, k-step u % KS) ----
  // lane (q, r16) loads rows i = 4 s + q (past O: zeroed slack rows of Zp) of
  // columns at WA + 16 t + r16 (past V: the next pair's values, weighted by zero)
  const double* zb = Z + (long)(wave_on ? xg : 0) * zx + r16 + (long)q * zi;
  double zq[ZD][TMA];
  const long zstep = 4 * zi;
  const double* zn = H == 1 ? zb : zb + s_lo * zstep;   // next k-step to load: a-tile za, k-step zs
  int zs = s_lo, za = 0;
  // advance to the next k-step; past the wave's last k-step of an a-tile the pointer jumps
  // to its first k-step of the next tile (the last tile repeats itself: those loads are
  // never consumed).  An if/else, which splits the unrolled K loop into one basic block
  // per k-step (a select-based form with one block per 4 k-steps measured 4 % slower).
  auto load_z = [&](int slot) XT_INLINE {
#pragma unroll
    for (int t = 0; t < TMA; ++t) zq[slot][t] = zn[16 * t];
    if constexpr (H == 1) {
      if (++zs == KS) { zs = 0; za = za + 1 < nat ? za + 1 : za; zn = zb + za * WA; }
      else zn += zstep;
    } else {
      if (++zs == s_hi) { zs = s_lo; za = za + 1 < nat ? za + 1 : za; zn = zb + za * WA + s_lo * zstep; }
      else zn += zstep;
    }
  };
  if (H == 1 || wave_on) {   // (a wave with no k-steps must not walk the ring)
#pragma unroll
    for (int d = 0; d < ZD; ++d) load_z(d);
  }

  d4w acc[TMA][TNG];
  double racc[TNG][3];
#pragma unroll
  for (int j = 0; j < TNG; ++j)
#pragma unroll
    for (int c = 0; c < 3; ++c) racc[j][c] = 0.0;

  const int p_lane = q * GB;                   // B image: row 4 s + q, column (16 j + r16) ^ swz
  // B fragments one k-step ahead: step s reads bq[s & 1] and loads step s + 1's into
  // bq[(s + 1) & 1] before its MFMAs, so their LDS latency hides under this step's
  // matrix work (a read past the last k-step lands in the weight image: unused)
  double bq[2][TNG];
  auto bload = [&](int s, double* dst) XT_INLINE {
    const int sw = swz(4 * s + q);
#pragma unroll
    for (int j = 0; j < TNG; ++j) dst[j] = sP[p_lane + 4 * s * GB + ((16 * j + r16) ^ sw)];
  };
  // one k-step from ring slot `slot` and B buffer `bb` (compile-time after unrolling)
  auto step = [&](int s, int slot, int bb) XT_INLINE {
    bload(s + 1, bq[bb ^ 1]);
    double af[TMA];
#pragma unroll
    for (int t = 0; t < TMA; ++t) af[t] = zq[slot][t];
    load_z(slot);
#pragma unroll
    for (int t = 0; t < TMA; ++t)
#pragma unroll
      for (int j = 0; j < TNG; ++j)
        acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t], bq[bb][j], acc[t][j], 0, 0, 0);
  };
  // the K loop of one a-tile whose first k-step sits in ring slot PH (KS is even, so
  // PH is even); the slots stay compile-time constants inside each unrolled group
  auto kloop = [&](auto PH, int s0, int s1) XT_INLINE {
    constexpr int P = decltype(PH)::value;
    bload(s0, bq[0]);
    int s = s0;
    for (; s + ZD <= s1; s += ZD) {
#pragma unroll
      for (int d = 0; d < ZD; ++d) step(s + d, (P + d) % ZD, d & 1);
    }
#pragma unroll
    for (int d = 0; d < ZD; ++d)
      if (s + d < s1) step(s + d, (P + d) % ZD, d & 1);
  };
  // k-steps [s0, s1) of a-tile at (s0 even: the ring phase stays even)
  auto krange = [&](int at, int s0, int s1) XT_INLINE {
    static_assert(ZD == 4, "ring phases");
    const int ph = H == 1 ? (int)(((long)at * KS + s0) % ZD) : (int)(((long)at * (s_hi - s_lo) + s0 - s_lo) % ZD);
    if (ph == 0) kloop(std::integral_constant<int, 0>{}, s0, s1);
    else         kloop(std::integral_constant<int, 2>{}, s0, s1);
  };
  __syncthreads();
  const int s_mid = s_lo + (((s_hi - s_lo) / 2) & ~1);
  for (int at = 0; at < nat; ++at) {
    const int buf = at & 1;
    if (at + 1 < nat) load_w(at + 1, 0);
#pragma unroll
    for (int t = 0; t < TMA; ++t)
#pragma unroll
      for (int j = 0; j < TNG; ++j) acc[t][j] = (d4w){0.0, 0.0, 0.0, 0.0};
    if (at + 1 < nat) {
      store_w(buf ^ 1, at + 1, 0);
      load_w(at + 1, 1);
    }
    if (wave_on) {
      krange(at, s_lo, s_hi);
      // contraction with the a-tile's weights: acc[t][j][r] = T[a = 16 t + q + 4 r][g = 16 j + r16].
      // Half a row (t, r) of weights at a time, the next half's reads issued before this
      // half's FMAs (two 6-value buffers; unfenced, the compiler hoists all 96 reads and
      // spills; fenced without the lookahead, every row waits out the LDS latency)
      const double* w = sW + buf * W_IMG;
      constexpr int JH = TNG / 2;                // half a row: JH column sub-tiles x 3 weights
      double wb[2][JH * 3];
      auto wread = [&](int h, double* dst) XT_INLINE {
        const int rw = h / 2, j0 = (h % 2) * JH;
        const int t = rw / 4, r = rw % 4;
        const int a = 16 * t + q + 4 * r;
        const int sa = swz(a);
#pragma unroll
        for (int jj = 0; jj < JH; ++jj) {
          const int col = (16 * (j0 + jj) + r16) ^ sa;
#pragma unroll
          for (int c = 0; c < 3; ++c) dst[3 * jj + c] = w[(c * WA + a) * GB + col];
        }
      };
      wread(0, wb[0]);
#pragma unroll
      for (int h = 0; h < 8 * TMA; ++h) {
        if (h + 1 < 8 * TMA) wread(h + 1, wb[(h + 1) & 1]);
        const int rw = h / 2, j0 = (h % 2) * JH;
        const int t = rw / 4, r = rw % 4;
#pragma unroll
        for (int jj = 0; jj < JH; ++jj)
#pragma unroll
          for (int c = 0; c < 3; ++c)
            racc[j0 + jj][c] += acc[t][j0 + jj][r] * wb[h & 1][3 * jj + c];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (at + 1 < nat) store_w(buf ^ 1, at + 1, 1);
    __syncthreads();
  }
  if constexpr (H > 1) {
    // the H waves of a pair hold partial sums over disjoint k-ranges: add them through
    // LDS (the weight buffers are free after the last barrier)
    double* red = sW;                            // [wave][j c][lane]
    if (h > 0) {
#pragma unroll
      for (int j = 0; j < TNG; ++j)
#pragma unroll
        for (int c = 0; c < 3; ++c) red[(wave * 3 * TNG + j * 3 + c) * 64 + lane] = racc[j][c];
    }
    __syncthreads();
    if (h == 0) {
      for (int hh = 1; hh < H; ++hh) {
        const int w2 = pl + hh * PB;
#pragma unroll
        for (int j = 0; j < TNG; ++j)
#pragma unroll
          for (int c = 0; c < 3; ++c) racc[j][c] += red[(w2 * 3 * TNG + j * 3 + c) * 64 + lane];
      }
    }
  }
  if (h != 0 || xg >= nx) return;
#pragma unroll
  for (int j = 0; j < TNG; ++j) {
    const int g = g0 + 16 * j + r16;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double v = rows4(racc[j][c]);
      if (q == 0 && g < n) Rout[(long)g * rg + 3 * xg + c] = v;
    }
  }
}

// Measured and removed: 32-point blocks, two per CU (178 vs 168 ms/step);
// two trial pairs per wave on 32-point blocks (163.3 vs 168.5 on one box, 170.0 vs 168.9
// on another: not reproducible); two pairs per wave on 64-point blocks (spills, 345).
static size_t rho_w_lds(int O) {
  constexpr int GB = 16 * TNG;
  return sizeof(double) * ((size_t)((O + 7) & ~7) * GB + 2 * 3 * WA * GB);
}

size_t xc_rho_w_lds_bytes(int O) { return rho_w_lds(O); }

// the 160 KB dynamic-LDS attribute, set once per device and kernel (thread-safe)
template <typename K>
static void lds_attribute(K kern, int slot) {
  static std::mutex mu;
  static unsigned long long done[4] = {0, 0, 0, 0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  if (dev < 64 && (done[slot] >> dev & 1ull)) return;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (dev < 64) done[slot] |= 1ull << dev;
}

// pairs per block: relative block time ~ PB / 8 (the k-steps each wave runs) + 0.13 (the
// per-a-tile contraction, staging and barrier, ~21 of 168 ms at PB 8), times the blocks
// per grid tile; the cheapest wins
static int rho_w_pb(int nx) {
  int best = 8;
  double best_cost = 1e30;
  for (int pb = 8; pb >= 1; pb /= 2) {
    const double cost = (double)((nx + pb - 1) / pb) * (pb / 8.0 + 0.13);
    if (cost < best_cost - 1e-9) { best_cost = cost; best = pb; }
  }
  return best;
}

int xc_rho_w(int O, int nx, int V, int n, const double* PO, long ldp, const double* Z, long zi, long zx,
             const double* W, long wc, long wg, double* R, long rg, hipStream_t st) {
  if (O <= 0 || nx <= 0 || V <= 0 || n <= 0) return 0;
  const size_t lds = rho_w_lds(O);
  if (lds > 160 * 1024) return XT_ERR_ARG;
  constexpr int GB = 16 * TNG;
  const int ntg = (n + GB - 1) / GB;
  const int pb = rho_w_pb(nx);
  const int blocks = ntg * ((nx + pb - 1) / pb);
#define XT_W(PBV, S)                                                                                       \
  case PBV:                                                                                                \
    lds_attribute(k_xc_rho_w<PBV>, S);                                                                     \
    hipLaunchKernelGGL((k_xc_rho_w<PBV>), dim3(blocks), dim3(64 * WXB), lds, st, O, nx, V, n, PO, ldp, Z, \
                       zi, zx, W, wc, wg, R, rg);                                                          \
    break;
  switch (pb) { XT_W(8, 0) XT_W(4, 1) XT_W(2, 2) default: XT_W(1, 3) }
#undef XT_W
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
