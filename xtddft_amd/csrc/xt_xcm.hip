// XC M-backward as a dedicated kernel (the GGA half of nr_uks_fxc's projection,
// XTDA.py:514 through PySCF numint):
//
//   accT[i][xg V + a] += sum_g PhiO[g][i] * sum_c wv[g][xg][c] * dPhiV_c[g][a]
//
// i < O occupied MO, xg < nx (spin channel, trial vector) pairs, a < V virtual MO,
// g a grid point of the chunk.  The generated operand M[g][xg][a] = sum_c wv dPhiV
// (nx V values per grid point) never exists in HBM.
//
// Why a kernel of its own (the generic engine's mode 2 runs a 128 x 64 tile, BK 16,
// two blocks per CU): there each wave does 16 MFMAs between barriers and builds its
// share of the generated tile into LDS before the barrier, so barrier, staging and
// generation are a large fraction of the loop.  Here:
//   * one 8-wave block per CU, wave w owns trial pair xg0 + w and 32 virtuals: a
//     (16 TM) x 32 accumulator tile, TM = ceil(O / 16) <= 8 row sub-tiles;
//   * per K-tile of 32 grid points every wave issues 8 k-steps x 2 TM MFMAs
//     (TM 7: 112, ~7k cycles of matrix pipe) per barrier;
//   * only RAW inputs are staged through LDS (PhiO tile, the block's 32 columns of
//     the three gradient planes, the block's 8 x 3 wv values per point); each wave
//     generates its own B fragments in registers from them (3 FMAs per fragment
//     element, LDS reads broadcast where 16 lanes share a value);
//   * LDS images are XOR-swizzled at 16-double granularity on the grid row parity so
//     the two 16-lane row halves of a 32-lane ds_read_b64 group hit disjoint bank
//     halves (64 banks x 4 B, MI355X_MICROARCH.md LDS table) and stores of 16
//     contiguous lanes stay contiguous.
// Split over the grid (K) for occupancy: each split writes its own slab, reduced in a
// fixed order (deterministic) and added to accT.
#include <hip/hip_runtime.h>
#include <type_traits>
#include "xt_internal.h"

namespace xt {

#define XT_INLINE __attribute__((always_inline))
typedef double d4m __attribute__((ext_vector_type(4)));

constexpr int BM_AB = 32;        // virtuals per block (2 MFMA column sub-tiles per wave)
// Block shapes: NW waves (one trial pair each), K-tiles of 4 NW grid points, LDS ~15 NW KB
// (TM 7); 8 waves per CU in all shapes (256 VGPRs):
//   NW 8: 512 threads, 32-point K-tiles, one block per CU (the shape for nx >= 8)
//   NW 4 / 2 / 1: two / four / eight blocks per CU, for Davidson steps with few trial
//   pairs (nx = 2 nz < 8 would leave most waves of an 8-wave block idle)

// LDS images (doubles), one buffer:
//   A  [g 32][i 16 TM]        swizzle i ^ 16 (g & 1) for even TM (odd TM: the row pitch
//                             16 TM = 16 mod 32 doubles already separates the halves)
//   W  [c 3][g 32][a 32]      swizzle a ^ 16 (g & 1)
//   R  [g 32][xg 8][c 3]      (broadcast reads)
template <int TM, int NW>
struct BmLds {
  static constexpr int BK = 4 * NW, XB = NW;
  static constexpr int A = BK * 16 * TM;
  static constexpr int W = 3 * BK * BM_AB;
  static constexpr int R = BK * XB * 3;
  static constexpr int BUF = A + W + R;
};

// rows4: sum of v over the four 16-lane rows (lanes l, l^16, l^32, l^48), in every lane
__device__ __forceinline__ double rows4_m(double v) {
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

// RV > 0: the last 16-row block of the occupied rows holds only RV <= 8 rows (O = 16
// (TM - 1) + RV); those rows are accumulated on the VALU (RV x 2 FMAs per k-step
// against the same B fragments, ~55 cycles at RV = 5) instead of a 16-row MFMA
// sub-tile (2 MFMAs, ~145 cycles), and reduced over the four k-rows once per block.
template <int TM, int RV, int NW>
__global__ void __launch_bounds__(64 * NW)
k_xc_back_m(int O, int nx, int V, int n, int ktiles_per_split,
            const double* __restrict__ PO, long ldp,
            const double* __restrict__ Wg, long wc, long wg,
            const double* __restrict__ R, long rg,
            double* __restrict__ out, long ldo, long slab) {
  using L = BmLds<TM, NW>;
  constexpr int BM_BK = L::BK, BM_XB = L::XB, NT = 64 * NW;
  constexpr int R_LD = (L::R + NT - 1) / NT;
  constexpr int PA = 16 * TM;                  // A row length (i)
  constexpr int A_LD = BM_BK * PA / NT;        // = TM doubles per thread
  constexpr int W_LD = 3 * BM_BK * BM_AB / NT;   // = 6
  constexpr int SWA = TM % 2 == 0 ? 16 : 0;    // A-image swizzle (see BmLds)
  __shared__ __attribute__((aligned(16))) double sm[2 * L::BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;

  // ---- block -> (split, a-tile, xg-tile) -----------------------------------
  // blocks are dealt round-robin over the 8 XCDs: renumber so each XCD runs a
  // contiguous range, ordered split-major, then a-tile, xg-tile fastest -- the
  // xg-tiles sharing one a-tile's gradient columns run side by side on one XCD
  // (its L2 serves the re-reads) and every block of a split reads the same PhiO rows.
  const int ntx = (nx + BM_XB - 1) / BM_XB, nta = (V + BM_AB - 1) / BM_AB;
  const int nblk = gridDim.x;
  int lid = blockIdx.x;
  {
    const int xcd = lid & 7, idx = lid >> 3, qn = nblk >> 3, rem = nblk & 7;
    lid = xcd * qn + (xcd < rem ? xcd : rem) + idx;
  }
  const int xt = lid % ntx;
  const int at = (lid / ntx) % nta;
  const int split = lid / (ntx * nta);
  const int x0 = xt * BM_XB, a0 = at * BM_AB;
  const int nkt = (n + BM_BK - 1) / BM_BK;
  const int kt0 = split * ktiles_per_split;
  const int kt1 = min(kt0 + ktiles_per_split, nkt);
  const int xg = x0 + wave;                    // this wave's trial pair
  const bool wave_on = xg < nx;

  // ---- staging maps (per thread, fixed) -------------------------------------
  // A: element e -> (g = (tid + 512 e) / PA, i = (tid + 512 e) % PA): 16-lane runs of
  //    consecutive i (one 128-B global segment, one conflict-free ds_write_b64 group)
  // W: element e -> (c, g, a) with a fastest over 32
  // R: element e -> (g, xg_l, c), 768 values, threads 0..255 load a second one
  double ra[A_LD], rw[W_LD], rr[R_LD];
  // per-thread byte offsets from the K-tile's (wave-uniform) row bases, columns
  // clamped once here.  Rows past n of the last K-tile are read unclamped: the
  // callers keep BM_BK rows of zeroed slack after the grid arrays (XC_GRID_SLACK),
  // and those rows' wv are stored as zero, so they add nothing.
  unsigned oa[A_LD], ow[W_LD], orr[R_LD];
#pragma unroll
  for (int e = 0; e < A_LD; ++e) {
    const int p = tid + NT * e, gl = p / PA, i = p % PA;
    oa[e] = (unsigned)(((long)gl * ldp + min(i, O - 1)) * 8);
  }
#pragma unroll
  for (int e = 0; e < W_LD; ++e) {
    const int p = tid + NT * e, gl = (p / BM_AB) % BM_BK, al = p % BM_AB;
    ow[e] = (unsigned)(((long)gl * wg + min(a0 + al, V - 1)) * 8);
  }
#pragma unroll
  for (int e = 0; e < R_LD; ++e) {
    const int p = min(tid + NT * e, L::R - 1), gl = p / (3 * BM_XB), xc = p % (3 * BM_XB);
    orr[e] = (unsigned)(((long)gl * rg + 3 * min(x0 + xc / 3, nx - 1) + xc % 3) * 8);
  }
  // Loads through buffer descriptors rebased per K-tile on wave-uniform (scalar) row
  // pointers: the per-element offsets above are the only lane-varying part, so the
  // staging runs no 64-bit address arithmetic on the VALU (whose issue cycles the FP64
  // matrix pipe pays, tools/mfma_probe2.hip)
  auto load = [&](int kt) XT_INLINE {
    const long g0 = (long)kt * BM_BK;
    const __amdgpu_buffer_rsrc_t pa = rsrc_of(PO + g0 * ldp), pr = rsrc_of(R + g0 * rg);
    const __amdgpu_buffer_rsrc_t pw[3] = {rsrc_of(Wg + g0 * wg), rsrc_of(Wg + wc + g0 * wg),
                                          rsrc_of(Wg + 2 * wc + g0 * wg)};
#pragma unroll
    for (int e = 0; e < A_LD; ++e) ra[e] = bld8(pa, oa[e], 0);
#pragma unroll
    for (int e = 0; e < W_LD; ++e) rw[e] = bld8(pw[e / 2], ow[e], 0);
#pragma unroll
    for (int e = 0; e < R_LD; ++e) rr[e] = bld8(pr, orr[e], 0);
  };
  // Padding: virtuals past V and pairs past nx read clamped (finite) columns and feed only
  // accumulator columns / waves that are never stored.  Grid points past n read R's zeroed
  // slack rows (xc_back_m's contract), so their B rows are zero.  LDS addresses are a
  // per-thread base plus a compile-time offset (BUF is a template constant: the K loop is
  // unrolled over the two buffers).
  auto store = [&](auto BUF, int kt) XT_INLINE {
    constexpr int B = decltype(BUF)::value;
    double* s = sm + B * L::BUF;
#pragma unroll
    for (int e = 0; e < A_LD; ++e) {
      const int p = tid + NT * e, gl = p / PA, i = p % PA;
      s[gl * PA + (i ^ ((gl & 1) * SWA))] = ra[e];
    }
#pragma unroll
    for (int e = 0; e < W_LD; ++e) {
      const int p = tid + NT * e, c = p / (BM_BK * BM_AB), gl = (p / BM_AB) % BM_BK, al = p % BM_AB;
      s[L::A + (c * BM_BK + gl) * BM_AB + (al ^ ((gl & 1) << 4))] = rw[e];
    }
    (void)kt;
#pragma unroll
    for (int e = 0; e < R_LD; ++e)
      if (tid + NT * e < L::R) s[L::A + L::W + tid + NT * e] = rr[e];
  };

  constexpr int TMM = RV ? TM - 1 : TM;        // MFMA row sub-tiles
  constexpr int RVA = RV ? RV : 1;
  d4m acc[TMM > 0 ? TMM : 1][2];
#pragma unroll
  for (int t = 0; t < TMM; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[t][j] = (d4m){0.0, 0.0, 0.0, 0.0};
  double part[RVA][2];
#pragma unroll
  for (int r = 0; r < RVA; ++r) part[r][0] = part[r][1] = 0.0;

  // one K-tile: 8 k-steps; lane (q, r16) feeds k = g_l = 4 s + q.  Row parity of g_l
  // is the parity of q, so the swizzles are per-lane constants and every LDS address
  // below is a lane base plus a compile-time offset.
  // The B fragments of k-step s + 1 are generated before the MFMAs of step s in
  // program order (their LDS reads and the 3-deep FP64 chain then overlap step s's
  // matrix work instead of stalling step s + 1's first MFMA; building all 8 steps'
  // fragments up front measured +4 %).
  const int swl = (q & 1) << 4;
  const int a_lane = q * PA + ((r16) ^ ((q & 1) * SWA));        // A: row q, column r16 (+16 t via XOR-free add)
  const int w_lane = L::A + q * BM_AB;                           // W: row q
  const int r_lane = L::A + L::W + q * (3 * BM_XB) + 3 * wave;   // R: row q, this wave's pair
  auto compute = [&](auto BUF) XT_INLINE {
    const double* s = sm + decltype(BUF)::value * L::BUF;
    auto gen = [&](int ks, double* b) XT_INLINE {
      const double* rrow = s + r_lane + 4 * ks * (3 * BM_XB);
      const double w0 = rrow[0], w1 = rrow[1], w2 = rrow[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const double* wr = s + w_lane + 4 * ks * BM_AB + ((16 * j + r16) ^ swl);
        b[j] = w0 * wr[0] + w1 * wr[BM_BK * BM_AB] + w2 * wr[2 * BM_BK * BM_AB];
      }
    };
    auto mma = [&](int ks, const double* b) XT_INLINE {
      double af[TMM > 0 ? TMM : 1];
#pragma unroll
      for (int t = 0; t < TMM; ++t) {
        // (16 t + r16) ^ sw = 16 (t ^ (sw / 16)) + r16: the swizzle permutes whole sub-tiles
        const int tt = SWA ? (t ^ (q & 1)) : t;
        af[t] = s[q * PA + 4 * ks * PA + 16 * tt + r16];
      }
      if constexpr (RV > 0) {
        // the remainder rows: phi_i(g) for i = 16 (TM - 1) + r, broadcast over the 16 lanes of a k-row
        const int tl = SWA ? ((TM - 1) ^ (q & 1)) : TM - 1;
        const double* rrw = s + q * PA + 4 * ks * PA + 16 * tl;
#pragma unroll
        for (int r = 0; r < RV; ++r) {
          const double v = rrw[r];
          part[r][0] += v * b[0];
          part[r][1] += v * b[1];
        }
      }
#pragma unroll
      for (int t = 0; t < TMM; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t], b[j], acc[t][j], 0, 0, 0);
    };
    double b[2][2];
    gen(0, b[0]);
#pragma unroll
    for (int ks = 0; ks < BM_BK / 4; ++ks) {
      if (ks + 1 < BM_BK / 4) gen(ks + 1, b[(ks + 1) & 1]);
      mma(ks, b[ks & 1]);
    }
  };
  (void)a_lane;

  if (kt0 < kt1) {
    // K-tile kt + 1 is written to LDS right after the barrier that opens K-tile kt (its
    // buffer was last read by K-tile kt - 1) and kt + 2 is loaded right after: the
    // stores overlap the other waves' MFMAs instead of delaying the barrier (writing
    // them before the closing barrier instead: +1 %)
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    load(kt0);
    store(B0{}, kt0);
    if (kt0 + 1 < kt1) load(kt0 + 1);
    __syncthreads();
    // one K-tile from buffer BUF (kt + 1 is staged into the other one)
    auto tile = [&](auto BUF, int kt) XT_INLINE {
      constexpr int B = decltype(BUF)::value;
      if (kt + 1 < kt1) store(std::integral_constant<int, B ^ 1>{}, kt + 1);
      if (kt + 2 < kt1) load(kt + 2);
      if (wave_on) compute(BUF);
      __syncthreads();
    };
    int kt = kt0;
    for (; kt + 2 <= kt1; kt += 2) {
      tile(B0{}, kt);
      tile(B1{}, kt + 1);
    }
    if (kt < kt1) tile(B0{}, kt);
  }
  if (!wave_on) return;
  // C/D layout: col = lane & 15, row = q + 4 reg
  double* o = out + (long)split * slab;
#pragma unroll
  for (int t = 0; t < TMM; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * t + q + 4 * r;
      if (i >= O) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int a = a0 + 16 * j + r16;
        if (a < V) o[(long)i * ldo + (long)xg * V + a] = acc[t][j][r];
      }
    }
  if constexpr (RV > 0) {
#pragma unroll
    for (int r = 0; r < RV; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const double v = rows4_m(part[r][j]);
        const int i = 16 * (TM - 1) + r, a = a0 + 16 * j + r16;
        if (q == 0 && i < O && a < V) o[(long)i * ldo + (long)xg * V + a] = v;
      }
  }
}

// accT[i][col] += sum_s ws[s][i][col]   (fixed order)
__global__ void k_xc_back_m_reduce(int O, long cols, int nsplit, const double* __restrict__ ws, long slab,
                                   double* __restrict__ C, long ldc) {
  const long total = (long)O * cols;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long i = t / cols, col = t % cols;
    double s = 0.0;
    for (int sp = 0; sp < nsplit; ++sp) s += ws[sp * slab + i * cols + col];
    C[i * ldc + col] += s;
  }
}

// Split count: the fewest splits whose blocks fill the chip's block slots (256 CUs x
// blocks per CU) in whole rounds (within 3 %) while keeping >= 16 K-tiles per split.
static int back_m_splits(int tiles, int nkt, int slots) {
  int best = 1;
  double best_eff = 0.0;
  for (int s = 1; s <= 64; ++s) {
    if (s > 1 && nkt / s < 16) break;
    const long blocks = (long)tiles * s;
    const double rounds = (double)blocks / slots;
    const double eff = rounds / ((blocks + slots - 1) / slots);
    if (eff > best_eff + 0.03 || (best_eff < 0.97 && eff > best_eff)) { best_eff = eff; best = s; }
    if (eff >= 0.97 && blocks >= 2 * slots) break;
  }
  return best;
}

// Block shape by the trial pairs: relative cost = blocks per a-tile x NW (the MFMA work)
// x (1 + the shape's overhead): smaller K-tiles mean more barriers and more PhiO staging
// per MFMA (per pair, relative to NW 8 at nx = 8: NW 4 +12 %, NW 2 +75 %)
static int back_m_nw(int nx) {
  const int nws[4] = {8, 4, 2, 1};
  const double pen[4] = {0.0, 0.12, 0.75, 2.0};   // measured at the headline shape
  int best = 8;
  double best_cost = 1e30;
  for (int k = 0; k < 4; ++k) {
    const int nw = nws[k];
    const double cost = (double)((nx + nw - 1) / nw) * nw * (1.0 + pen[k]);
    if (cost < best_cost - 1e-9) { best_cost = cost; best = nw; }
  }
  return best;
}

struct BackMPlan { int nw, tiles, nkt, splits, kps, used, blocks; };
static BackMPlan back_m_plan(int nx, int V, int n) {
  BackMPlan p;
  p.nw = back_m_nw(nx);
  const int bk = 4 * p.nw, xb = p.nw;
  p.tiles = ((nx + xb - 1) / xb) * ((V + BM_AB - 1) / BM_AB);
  p.nkt = (n + bk - 1) / bk;
  p.splits = back_m_splits(p.tiles, p.nkt, 256 * (8 / p.nw));
  p.kps = (p.nkt + p.splits - 1) / p.splits;
  p.used = (p.nkt + p.kps - 1) / p.kps;
  p.blocks = p.tiles * p.used;
  return p;
}

size_t xc_back_m_workspace_bytes(int O, int nx, int V, int n) {
  const BackMPlan p = back_m_plan(nx, V, n);
  return sizeof(double) * (size_t)p.splits * O * (size_t)nx * V;
}

// remainder rows on the VALU for the occupied counts of the BASELINE shapes (O = 33..40:
// C2, C5; O = 97..104: the headline): RV = O - 16 (TM - 1) <= 8 (<= 6 at TM 7: more
// spills at 256 VGPRs); otherwise 16-row MFMA tiles throughout
template <int TM, int NW>
static void launch_back_m(int O, int nx, int V, int n, int kps, int blocks, const double* PO, long ldp,
                          const double* W, long wc, long wg, const double* R, long rg, double* ws, long slab,
                          hipStream_t st) {
  const int rv = O - 16 * (TM - 1);
  const dim3 grid(blocks), blk(64 * NW);
  const long ldo = (long)nx * V;
  if constexpr (TM == 3 || TM == 7) {
    if (!(TM == 7 && rv > 6)) {
#define XT_RV(N) case N: hipLaunchKernelGGL((k_xc_back_m<TM, N, NW>), grid, blk, 0, st, O, nx, V, n, kps, PO, ldp, W, \
                                            wc, wg, R, rg, ws, ldo, slab); return;
      switch (rv) { XT_RV(1) XT_RV(2) XT_RV(3) XT_RV(4) XT_RV(5) XT_RV(6) XT_RV(7) XT_RV(8) default: break; }
#undef XT_RV
    }
  }
  hipLaunchKernelGGL((k_xc_back_m<TM, 0, NW>), grid, blk, 0, st, O, nx, V, n, kps, PO, ldp, W, wc, wg, R, rg, ws, ldo,
                     slab);
}

template <int NW>
static void launch_back_m_tm(int TM, int O, int nx, int V, int n, int kps, int blocks, const double* PO, long ldp,
                             const double* W, long wc, long wg, const double* R, long rg, double* ws, long slab,
                             hipStream_t st) {
#define XT_TM(N) case N: launch_back_m<N, NW>(O, nx, V, n, kps, blocks, PO, ldp, W, wc, wg, R, rg, ws, slab, st); break;
  switch (TM) { XT_TM(1) XT_TM(2) XT_TM(3) XT_TM(4) XT_TM(5) XT_TM(6) XT_TM(7) default: XT_TM(8) }
#undef XT_TM
}

int xc_back_m(int O, int nx, int V, int n, const double* PO, long ldp, const double* W, long wc, long wg,
              const double* R, long rg, double* C, long ldc, double* ws, size_t ws_bytes, hipStream_t st) {
  if (O <= 0 || nx <= 0 || V <= 0 || n <= 0) return 0;
  if (O > 128) return XT_ERR_ARG;                      // one row tile (the engine's mode 2 covers more)
  const BackMPlan p = back_m_plan(nx, V, n);
  const long slab = (long)O * nx * V;
  if (ws_bytes < sizeof(double) * (size_t)p.splits * slab) return XT_ERR_ARG;
  const int TM = (O + 15) / 16;
  switch (p.nw) {
    case 8: launch_back_m_tm<8>(TM, O, nx, V, n, p.kps, p.blocks, PO, ldp, W, wc, wg, R, rg, ws, slab, st); break;
    case 4: launch_back_m_tm<4>(TM, O, nx, V, n, p.kps, p.blocks, PO, ldp, W, wc, wg, R, rg, ws, slab, st); break;
    case 2: launch_back_m_tm<2>(TM, O, nx, V, n, p.kps, p.blocks, PO, ldp, W, wc, wg, R, rg, ws, slab, st); break;
    default: launch_back_m_tm<1>(TM, O, nx, V, n, p.kps, p.blocks, PO, ldp, W, wc, wg, R, rg, ws, slab, st); break;
  }
  const long total = slab;
  int rb = (int)((total + 255) / 256);
  if (rb > 8192) rb = 8192;
  hipLaunchKernelGGL(k_xc_back_m_reduce, dim3(rb), dim3(256), 0, st, O, (long)nx * V, p.used, ws, slab, C, ldc);
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
