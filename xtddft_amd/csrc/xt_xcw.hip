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
//     global memory into registers through a 4-slot ring, 3 k-steps ahead;
//   * B = PhiO[g][i]: the block's 64 x O tile, loaded ONCE per block into LDS and
//     resident for the whole a loop;
//   * after each 32-wide a-tile's K loop the accumulators T[a][g] are contracted
//     with dPhiV_c[g][a] (staged per a-tile in LDS, shared by the block's waves)
//     into per-lane partial sums racc[j][c] -- the sum over a stays in-lane (rows a
//     of a lane are q + 4 reg + 16 t) and only the final 4-row reduction crosses
//     lanes, once per block.
//
// Built for the FP64 issue model measured on gfx950 (tools/mfma_probe2.hip): every VALU
// instruction in the MFMA stream costs its issue cycles to the matrix pipe (4 integer adds
// per 8 MFMAs: -2.6 %; 4 v_mov_b64: -8 %), while LDS reads at immediate offsets are free
// (-1 %).  So the hot loop carries no per-step VALU at all:
//   * k index permutation: lane q of k-step pair p supplies i = 8 p + 2 q + (step & 1),
//     so one ds_read_b128 per 16-column sub-tile feeds two k-steps;
//   * LDS images are padded, not XOR-swizzled, so every address is a lane base plus a
//     compile-time offset: PhiO [g][i] with pitch KI + 4 (= 4 mod 8 doubles: the four
//     16-lane ds_read_b128 groups cover all 64 banks), weights [c][g][a] with pitch 34
//     (32-lane ds_read_b64 groups conflict-free, 16-lane write runs contiguous);
//   * global addresses are a wave-uniform base (SGPRs, scalar arithmetic) plus a fixed
//     32-bit lane offset;
//   * the first k-step of an a-tile multiplies into a zero accumulator (no 32-move reset);
//   * ring slots and weight buffers are compile-time in every unrolled a-tile (a-tiles
//     run in pairs when the ring phase alternates), so no register rotation.
// One barrier per a-tile.
#include <hip/hip_runtime.h>
#include <mutex>
#include <type_traits>
#include "xt_internal.h"

namespace xt {

#define XT_INLINE __attribute__((always_inline))
typedef double d4w __attribute__((ext_vector_type(4)));
typedef double d2w __attribute__((ext_vector_type(2)));

constexpr int WA = 32;           // virtuals per a-tile (2 MFMA row sub-tiles)
constexpr int TMA = WA / 16;
constexpr int WXB = 8;           // waves per block
constexpr int ZD = 4;            // Zp ring slots (loads ZD - 1 k-steps ahead; 2 slots measured +6.5 %, 8 spills)
constexpr int TNG = 4;           // 16-point column sub-tiles per block (64 grid points)
constexpr int GB = 16 * TNG;     // grid points per block
constexpr int WP = WA + 2;       // weight image pitch (doubles)
constexpr int W_IMG = 3 * GB * WP;   // one weight buffer (doubles)

// PhiO image pitch (doubles): 4 mod 8 for conflict-free ds_read_b128 groups, compile-time so
// the 16-column sub-tile offsets are immediates; the image holds KI = O rounded up to 8 <= 112
// rows (O <= 112), and with two weight buffers fills the 160 KB exactly
constexpr int PP = 116;
constexpr int RHO_W_MAX_O = 112;
__host__ __device__ constexpr int rho_w_ki(int O) { return (O + 7) & ~7; }   // occupied rows (k-step pairs whole)

// PB trial pairs per block (8, 4, 2, 1; Davidson steps with few new vectors): the
// H = 8 / PB waves of a pair split each a-tile's k-step pairs into H even ranges,
// contract their partial T with the same staged weights (the contraction is linear in T)
// and add their partial sums through LDS once at the end -- every wave of the block
// works when nx < 8, and the weight staging stays one image per a-tile.
template <int PB>
__global__ void __launch_bounds__(64 * WXB) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_xc_rho_w(int O, int nx, int V, int n,
           const double* __restrict__ PO, long ldp,
           const double* __restrict__ Z, long zi, long zx,
           const double* __restrict__ Wg, long wc, long wg,
           double* __restrict__ Rout, long rg) {
  constexpr int NT = 64 * WXB;                 // threads per block
  constexpr int W_LD = 3 * GB * WA / NT;       // weight elements staged per thread and a-tile (12)
  static_assert(3 * GB * WA == W_LD * NT && GB * WA / NT == 4, "weight staging map");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int KI = rho_w_ki(O);
  double* sP = sm;                             // [GB][PP]
  double* sW = sm + GB * PP;                   // [2][3][GB][WP]

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
  constexpr int H = WXB / PB;                  // waves per pair
  const int gt = lid % ntg, xs = lid / ntg;
  const int g0 = gt * GB, x0 = xs * PB;
  const int pl = wave % PB, h = wave / PB;
  const int xg = x0 + pl;                      // this wave's trial pair
  const int nat = (V + WA - 1) / WA;
  const int KP = KI / 8;                       // k-step pairs per a-tile
  // this wave's k-step pairs of every a-tile: [p_lo, p_hi)
  const int p_lo = H == 1 ? 0 : (h * KP) / H, p_hi = H == 1 ? KP : ((h + 1) * KP) / H;
  const int np = p_hi - p_lo;
  const bool wave_on = xg < nx && np > 0;

  // ---- PhiO tile -> LDS (once; rows past n read the zeroed grid slack) ----------
  for (int p = tid; p < KI * GB; p += NT) {
    const int g = p / KI, i = p % KI;
    sP[g * PP + i] = i < O ? PO[(long)(g0 + g) * ldp + i] : 0.0;
  }
  // ---- weights of a-tile `at` (global -> registers -> LDS) -------------------
  // thread element k (0..11): plane c = k / 4, grid row wr + 16 (k % 4), column wa.
  // Columns past V read the next grid row (the arrays are row-padded and followed by
  // XC_GRID_SLACK rows) and are stored as zero.
  const int wa = tid & (WA - 1), wr = tid / WA;
  const unsigned w_off = (unsigned)(((long)wr * wg + wa) * 8);
  const __amdgpu_buffer_rsrc_t wrs[3] = {rsrc_of(Wg + (long)g0 * wg), rsrc_of(Wg + wc + (long)g0 * wg),
                                         rsrc_of(Wg + 2 * wc + (long)g0 * wg)};
  double rw[W_LD];
  auto load_w1 = [&](int k, int at) XT_INLINE {   // k compile-time after unrolling
    rw[k] = bld8(wrs[k / 4], w_off, (int)((16 * (k % 4) * wg + (long)at * WA) * 8));
  };
  auto load_w = [&](int k0, int at) XT_INLINE {
#pragma unroll
    for (int k = 0; k < W_LD; ++k)
      if (k >= k0) load_w1(k, at);
  };
  double* const w_st = sW + wr * WP + wa;
  auto store_w = [&](auto BUF, int at) XT_INLINE {
    constexpr int B = decltype(BUF)::value;
    if ((at + 1) * WA <= V) {
#pragma unroll
      for (int k = 0; k < W_LD; ++k) w_st[B * W_IMG + ((k / 4) * GB + 16 * (k % 4)) * WP] = rw[k];
    } else {
      const bool live = at * WA + wa < V;
#pragma unroll
      for (int k = 0; k < W_LD; ++k) w_st[B * W_IMG + ((k / 4) * GB + 16 * (k % 4)) * WP] = live ? rw[k] : 0.0;
    }
  };
  load_w(0, 0);
  store_w(std::integral_constant<int, 0>{}, 0);

  // ---- Zp ring: lane (q, r16) of k-step s supplies row i = 8 (s / 2) + 2 q + (s & 1)
  // (past O: zeroed slack rows of Zp) of columns at WA + 16 t + r16 (past V: the next
  // pair's values, weighted by zero).  The walker (zs, za) is the next k-step to load:
  // past the wave's last k-step of an a-tile it moves to its first k-step of the next
  // tile (the last tile repeats itself: those loads are never consumed).
  const __amdgpu_buffer_rsrc_t zrs = rsrc_of(Z + (long)(wave_on ? xg : 0) * zx);
  const unsigned z_off = (unsigned)(((long)2 * q * zi + r16) * 8);
  double zq[ZD][TMA];
  const int s_lo = 2 * p_lo, s_hi = 2 * p_hi;
  const int z_lo = 8 * p_lo * (int)zi * 8;     // byte offset of row 8 p_lo (scalar)
  int zs = s_lo, za = 0, zso = z_lo;           // zso: byte offset of k-step zs's rows in a-tile za
  auto load_z = [&](int slot) XT_INLINE {
#pragma unroll
    for (int t = 0; t < TMA; ++t) zq[slot][t] = bld8(zrs, z_off + 128 * t, zso);
    if (++zs == s_hi) {
      zs = s_lo;
      za = za + 1 < nat ? za + 1 : za;
      zso = za * WA * 8 + z_lo;
    } else {
      zso += (zs & 1 ? 1 : 7) * (int)zi * 8;   // rows 8 p + {0, 1} of a pair, then the next pair
    }
  };

  d4w acc[TMA][TNG];
  double racc[TNG][3];
#pragma unroll
  for (int j = 0; j < TNG; ++j)
#pragma unroll
    for (int c = 0; c < 3; ++c) racc[j][c] = 0.0;

  // B fragments of k-step pair p: columns 16 j + r16, rows 8 p + 2 q + {0, 1}
  d2w bq[2][TNG];
  const double* const b_lane = sP + r16 * PP + 2 * q;
  auto bread = [&](int p, d2w* dst) XT_INLINE {
    const d2w* src = (const d2w*)(b_lane + 8 * p);
#pragma unroll
    for (int j = 0; j < TNG; ++j) dst[j] = src[(16 * j * PP) / 2];
  };
  // one k-step from ring slot SL and B buffer BB, half SUB of the pair; ZERO: the first
  // k-step of the a-tile, into a zero accumulator; NT_: the a-tile's live row sub-tiles
  // (1 for a last a-tile with V % 32 <= 16: its second sub-tile is all padding)
  auto step = [&](auto SL, auto BB, auto SUB, auto ZERO, auto NT_) XT_INLINE {
    constexpr int sl = decltype(SL)::value, bb = decltype(BB)::value, sub = decltype(SUB)::value;
    load_z((sl + ZD - 1) % ZD);   // into the slot the previous k-step consumed (whole ring rows)
#pragma unroll
    for (int t = 0; t < decltype(NT_)::value; ++t)
#pragma unroll
      for (int j = 0; j < TNG; ++j)
        acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(
            zq[sl][t], bq[bb][j][sub], decltype(ZERO)::value ? (d4w){0.0, 0.0, 0.0, 0.0} : acc[t][j], 0, 0, 0);
  };
  // one k-step pair in ring slots SL, SL + 1 from B buffer BB; prefetches pair pn's B
  auto kpair = [&](auto SL, auto BB, auto ZERO, auto NT_, int pn) XT_INLINE {
    constexpr int sl = decltype(SL)::value, bb = decltype(BB)::value;
    bread(pn, bq[bb ^ 1]);
    step(std::integral_constant<int, sl>{}, BB, std::integral_constant<int, 0>{}, ZERO, NT_);
    step(std::integral_constant<int, (sl + 1) % ZD>{}, BB, std::integral_constant<int, 1>{},
         std::integral_constant<bool, false>{}, NT_);
  };
  using F = std::integral_constant<bool, false>;
  using T1 = std::integral_constant<bool, true>;
  // kpair that also issues the next a-tile's weight loads K0 and K0 + 1, one before each
  // k-step.  The 12 weight loads of an a-tile are spread over its first 12 k-steps: issued
  // together at the tile start they queue ahead of the Zp ring's loads, and the ring's
  // in-order vmcnt waits then stall on them (same box: 147.2 -> 142.8 ms per step; 4 / 2
  // loads per k-step pair 144.8 / 143.3)
  auto kpair_w = [&](auto SL, auto BB, auto ZERO, auto NT_, int pn, auto K0, bool wn, int at) XT_INLINE {
    constexpr int sl = decltype(SL)::value, bb = decltype(BB)::value, k0 = decltype(K0)::value;
    bread(pn, bq[bb ^ 1]);
    if (wn) load_w1(k0, at);
    step(std::integral_constant<int, sl>{}, BB, std::integral_constant<int, 0>{}, ZERO, NT_);
    if (wn) load_w1(k0 + 1, at);
    step(std::integral_constant<int, (sl + 1) % ZD>{}, BB, std::integral_constant<int, 1>{},
         std::integral_constant<bool, false>{}, NT_);
  };
  using W0 = std::integral_constant<int, 0>;
  using W2 = std::integral_constant<int, 2>;
  using W4 = std::integral_constant<int, 4>;
  using W6 = std::integral_constant<int, 6>;
  using W8 = std::integral_constant<int, 8>;
  using W10 = std::integral_constant<int, 10>;

  // one a-tile: ring phase P (slot of its first k-step), weight buffer BUF and live row
  // sub-tiles NT_ compile-time
  auto tile = [&](auto PH, auto BUF, auto NT_, int at) XT_INLINE {
    constexpr int P = decltype(PH)::value, B = decltype(BUF)::value, NTL = decltype(NT_)::value;
    using SA = std::integral_constant<int, P>;               // ring slots of even / odd pairs
    using SB = std::integral_constant<int, (P + 2) % ZD>;
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    const bool wn = at + 1 < nat;
    if (!wave_on && wn) load_w(0, at + 1);
    if (wave_on) {
      kpair_w(SA{}, B0{}, T1{}, NT_, p_lo + 1, W0{}, wn, at + 1);
      int k = 1;
      if (np >= 7) {          // the first three pairs of k-step pairs peeled: weights 2 .. 11
        kpair_w(SB{}, B1{}, F{}, NT_, p_lo + 2, W2{}, wn, at + 1);
        kpair_w(SA{}, B0{}, F{}, NT_, p_lo + 3, W4{}, wn, at + 1);
        kpair_w(SB{}, B1{}, F{}, NT_, p_lo + 4, W6{}, wn, at + 1);
        kpair_w(SA{}, B0{}, F{}, NT_, p_lo + 5, W8{}, wn, at + 1);
        kpair_w(SB{}, B1{}, F{}, NT_, p_lo + 6, W10{}, wn, at + 1);
        kpair(SA{}, B0{}, F{}, NT_, p_lo + 7);
        k = 7;
      } else if (wn) {
        load_w(2, at + 1);
      }
      for (; k + 2 <= np; k += 2) {
        kpair(std::integral_constant<int, (P + 2) % ZD>{}, std::integral_constant<int, 1>{}, F{}, NT_, p_lo + k + 1);
        kpair(std::integral_constant<int, P>{}, std::integral_constant<int, 0>{}, F{}, NT_, p_lo + k + 2);
      }
      if (k < np)
        kpair(std::integral_constant<int, (P + 2) % ZD>{}, std::integral_constant<int, 1>{}, F{}, NT_, p_lo + k + 1);
      bread(p_lo, bq[0]);        // the next a-tile's first pair (the PhiO image never changes)
      // contraction with the a-tile's weights: acc[t][j][r] = T[a = 16 t + q + 4 r][g = 16 j + r16].
      // Half a row (t, r) of weights at a time, the next half's reads issued before this
      // half's FMAs (two 6-value buffers; unfenced, the compiler hoists all 96 reads)
      const double* w = sW + B * W_IMG + r16 * WP + q;
      constexpr int JH = TNG / 2;
      double wb[2][JH * 3];
      auto wread = [&](int hh, double* dst) XT_INLINE {
        const int rw_ = hh / 2, j0 = (hh % 2) * JH;
        const int t = rw_ / 4, r = rw_ % 4;
#pragma unroll
        for (int jj = 0; jj < JH; ++jj)
#pragma unroll
          for (int c = 0; c < 3; ++c) dst[3 * jj + c] = w[(c * GB + 16 * (j0 + jj)) * WP + 16 * t + 4 * r];
      };
      wread(0, wb[0]);
#pragma unroll
      for (int hh = 0; hh < 8 * NTL; ++hh) {
        if (hh + 1 < 8 * NTL) wread(hh + 1, wb[(hh + 1) & 1]);
        const int rw_ = hh / 2, j0 = (hh % 2) * JH;
        const int t = rw_ / 4, r = rw_ % 4;
#pragma unroll
        for (int jj = 0; jj < JH; ++jj)
#pragma unroll
          for (int c = 0; c < 3; ++c)
            racc[j0 + jj][c] += acc[t][j0 + jj][r] * wb[hh & 1][3 * jj + c];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (at + 1 < nat) store_w(std::integral_constant<int, B ^ 1>{}, at + 1);
    __syncthreads();
  };

  __syncthreads();
  if (wave_on) {
#pragma unroll
    for (int d = 0; d < ZD - 1; ++d) load_z(d);
    bread(p_lo, bq[0]);
  }
  // a-tiles in pairs: with an odd pair count per a-tile the ring phase alternates 0, 2.
  // A last a-tile holding <= 16 live virtuals (V = 901: 5) runs one row sub-tile.
  using NF = std::integral_constant<int, TMA>;
  using NH = std::integral_constant<int, 1>;
  const bool half_last = (V % WA) != 0 && (V % WA) <= 16;
  const int nfull = half_last ? nat - 1 : nat;
  auto run = [&](auto ALT) XT_INLINE {
    constexpr int P1 = decltype(ALT)::value ? 2 : 0;
    using Q0 = std::integral_constant<int, 0>;
    using Q1 = std::integral_constant<int, P1>;
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    int at = 0;
    for (; at + 2 <= nfull; at += 2) {
      tile(Q0{}, B0{}, NF{}, at);
      tile(Q1{}, B1{}, NF{}, at + 1);
    }
    if (at < nfull) tile(Q0{}, B0{}, NF{}, at++);
    if (half_last) {     // a-tile `at`: phase and buffer by its parity
      if (at & 1) tile(Q1{}, B1{}, NH{}, at);
      else tile(Q0{}, B0{}, NH{}, at);
    }
  };
  if (np & 1) run(T1{});
  else run(F{});

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
  return O > RHO_W_MAX_O ? (size_t)1 << 40 : sizeof(double) * ((size_t)GB * PP + 2 * W_IMG);
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

// Block shapes by the trial pairs: relative block time ~ PB / 8 (the k-steps each wave
// runs) + 0.27 (the per-a-tile contraction, staging and barrier; fitted to the nvec sweep of
// the VALU-free kernel: a 4-pair block costs 0.60, a 2-pair block 0.415 of an 8-pair block).
// A step's nx pairs are split into segments of one shape each (xc_pair_segments, e.g.
// 10 = 8 + 2 instead of three 4-pair blocks), one launch per segment.
static const double kRhoWCost[4] = {1.0 + 0.27, 0.5 + 0.27, 0.25 + 0.27, 0.125 + 0.27};

int xc_rho_w(int O, int nx, int V, int n, const double* PO, long ldp, const double* Z, long zi, long zx,
             const double* W, long wc, long wg, double* R, long rg, hipStream_t st) {
  if (O <= 0 || nx <= 0 || V <= 0 || n <= 0) return 0;
  const size_t lds = rho_w_lds(O);
  if (lds > 160 * 1024) return XT_ERR_ARG;
  const int ntg = (n + GB - 1) / GB;
  int pbs[4], cnt[4];
  const int ns = xc_pair_segments(nx, kRhoWCost, pbs, cnt);
  for (int s = 0, x0 = 0; s < ns; x0 += cnt[s], ++s) {
    const int nxs = cnt[s], pb = pbs[s];
    const int blocks = ntg * ((nxs + pb - 1) / pb);
    const double* Zs = Z + (long)x0 * zx;
    double* Rs = R + 3L * x0;
#define XT_W(PBV, S)                                                                                         \
  case PBV:                                                                                                  \
    lds_attribute(k_xc_rho_w<PBV>, S);                                                                       \
    hipLaunchKernelGGL((k_xc_rho_w<PBV>), dim3(blocks), dim3(64 * WXB), lds, st, O, nxs, V, n, PO, ldp, Zs, \
                       zi, zx, W, wc, wg, Rs, rg);                                                           \
    break;
    switch (pb) { XT_W(8, 0) XT_W(4, 1) XT_W(2, 2) default: XT_W(1, 3) }
#undef XT_W
  }
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
