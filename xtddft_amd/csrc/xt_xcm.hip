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
typedef double d2m __attribute__((ext_vector_type(2)));

constexpr int BM_AB = 32;        // virtuals per block (2 MFMA column sub-tiles per wave)
// Block shapes: NW waves (one trial pair each), K-tiles of 4 NW grid points, LDS ~15 NW KB
// (TM 7); 8 waves per CU in all shapes (256 VGPRs):
//   NW 8: 512 threads, 32-point K-tiles, one block per CU (the shape for nx >= 8)
//   NW 4 / 2 / 1: two / four / eight blocks per CU, for Davidson steps with few trial
//   pairs (nx = 2 nz < 8 would leave most waves of an 8-wave block idle)

// K-tile grid points of an NW-wave block: whole k-step pairs (8 points per pair)
__host__ __device__ constexpr int bm_bk(int nw) { return nw >= 2 ? 4 * nw : 8; }

// LDS images in 16-B slots, each holding one value at a POINT PAIR (g, g + 1): lane q of
// k-step pair p supplies grid points 2 (4 p + q) + {0, 1} to k-steps 2 p and 2 p + 1 (the
// same permutation of the sum over g in both operands), so one ds_read_b128 feeds two
// k-steps and every read is a per-lane base plus a compile-time offset.  The two buffers
// of an image sit side by side (offsets stay inside the 16-bit ds offset field).
//   A  [pair][i < 16 TMM]         PhiO, the MFMA rows
//   W  [c 3][pair][a 32]          gradient planes of the block's virtuals
//   R  [pair][xg NW][c 3]         wv (broadcast reads)
//   RM [pair][r 8]                PhiO remainder rows 16 TMM + r (broadcast; RV > 0)
// Conflicts: ds_read_b128 serves 16-lane groups mixing two q rows, so each image's row
// length is 0 mod 16 slots (A, W) or the two rows' broadcast slots differ mod 16 (R: 3 NW,
// RM: 8); ds_write_b128 groups of 8 lanes write 8 consecutive slots.
template <int TM, int RV, int NW>
struct BmLds {
  static constexpr int TMM = RV ? TM - 1 : TM;
  static constexpr int BK = bm_bk(NW), NPR = BK / 2, KP = BK / 8;
  static constexpr int PI = 16 * TMM, PR = 3 * NW;
  static constexpr int A = NPR * PI, W = 3 * NPR * BM_AB, R = NPR * PR, RM = RV ? NPR * 8 : 0;
  static constexpr int OA = 0, OW = 2 * A, OR = OW + 2 * W, ORM = OR + 2 * R, TOTAL = ORM + 2 * RM;
};

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
  using L = BmLds<TM, RV, NW>;
  constexpr int TMM = L::TMM, BK = L::BK, KP = L::KP, PI = L::PI, PR = L::PR, NT = 64 * NW;
  constexpr int A_PT = (L::A + NT - 1) / NT, W_PT = (L::W + NT - 1) / NT;
  constexpr int R_PT = (L::R + NT - 1) / NT, M_PT = RV ? (L::RM + NT - 1) / NT : 0;
  static_assert((L::NPR * BM_AB) % NT == 0, "a thread's W slots stay in one gradient plane");
  __shared__ d2m smv[L::TOTAL];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;

  // ---- block -> (split, a-tile, xg-tile) -----------------------------------
  // blocks are dealt round-robin over the 8 XCDs: renumber so each XCD runs a
  // contiguous range, ordered split-major, then a-tile, xg-tile fastest -- the
  // xg-tiles sharing one a-tile's gradient columns run side by side on one XCD
  // (its L2 serves the re-reads) and every block of a split reads the same PhiO rows.
  const int ntx = (nx + NW - 1) / NW, nta = (V + BM_AB - 1) / BM_AB;
  const int nblk = gridDim.x;
  int lid = blockIdx.x;
  {
    const int xcd = lid & 7, idx = lid >> 3, qn = nblk >> 3, rem = nblk & 7;
    lid = xcd * qn + (xcd < rem ? xcd : rem) + idx;
  }
  const int xt = lid % ntx;
  const int at = (lid / ntx) % nta;
  const int split = lid / (ntx * nta);
  const int x0 = xt * NW, a0 = at * BM_AB;
  const int nkt = (n + BK - 1) / BK;
  const int kt0 = split * ktiles_per_split;
  const int kt1 = min(kt0 + ktiles_per_split, nkt);
  const int xg = x0 + wave;                    // this wave's trial pair
  const bool wave_on = xg < nx;

  // ---- staging: slot e of an image -> (point pair, column); a slot's two values come
  // from grid rows 2 pair and 2 pair + 1 (the second through a scalar offset of one row).
  // Columns past V / pairs past nx / occupied rows past O are clamped (finite values
  // feeding accumulator columns, waves or rows that are never stored); grid points past
  // n read the zeroed wv slack (xc_back_m's contract), so their B rows are zero.
  unsigned oa[A_PT], ow[W_PT], orr[R_PT], om[M_PT > 0 ? M_PT : 1];
#pragma unroll
  for (int e = 0; e < A_PT; ++e) {
    const int sl = min(tid + NT * e, L::A - 1), pr = sl / PI, i = sl % PI;
    oa[e] = (unsigned)(((long)2 * pr * ldp + min(i, O - 1)) * 8);
  }
#pragma unroll
  for (int e = 0; e < W_PT; ++e) {
    const int sl = min(tid + NT * e, L::W - 1), pr = (sl / BM_AB) % L::NPR, al = sl % BM_AB;
    ow[e] = (unsigned)(((long)2 * pr * wg + min(a0 + al, V - 1)) * 8);
  }
#pragma unroll
  for (int e = 0; e < R_PT; ++e) {
    const int sl = min(tid + NT * e, L::R - 1), pr = sl / PR, xc = sl % PR;
    orr[e] = (unsigned)(((long)2 * pr * rg + 3 * min(x0 + xc / 3, nx - 1) + xc % 3) * 8);
  }
#pragma unroll
  for (int e = 0; e < M_PT; ++e) {
    const int sl = min(tid + NT * e, L::RM - 1), pr = sl / 8, r = sl % 8;
    om[e] = (unsigned)(((long)2 * pr * ldp + 16 * TMM + min(r, RV - 1)) * 8);
  }
  d2m ra[A_PT], rw[W_PT], rr[R_PT], rm_[M_PT > 0 ? M_PT : 1];
  // loads through buffer descriptors rebased per K-tile on wave-uniform row pointers
  // (no 64-bit address arithmetic on the VALU, whose issue cycles the FP64 matrix pipe pays)
  auto load = [&](int kt) XT_INLINE {
    const long g0 = (long)kt * BK;
    const __amdgpu_buffer_rsrc_t pa = rsrc_of(PO + g0 * ldp), pr = rsrc_of(R + g0 * rg);
    const __amdgpu_buffer_rsrc_t pw[3] = {rsrc_of(Wg + g0 * wg), rsrc_of(Wg + wc + g0 * wg),
                                          rsrc_of(Wg + 2 * wc + g0 * wg)};
    const int sp = (int)(ldp * 8), sw = (int)(wg * 8), sr = (int)(rg * 8);
#pragma unroll
    for (int e = 0; e < A_PT; ++e) ra[e] = (d2m){bld8(pa, oa[e], 0), bld8(pa, oa[e], sp)};
#pragma unroll
    for (int e = 0; e < W_PT; ++e) {
      constexpr int WPC = L::NPR * BM_AB / NT;   // slots per thread and plane
      rw[e] = (d2m){bld8(pw[e / WPC], ow[e], 0), bld8(pw[e / WPC], ow[e], sw)};
    }
#pragma unroll
    for (int e = 0; e < R_PT; ++e) rr[e] = (d2m){bld8(pr, orr[e], 0), bld8(pr, orr[e], sr)};
#pragma unroll
    for (int e = 0; e < M_PT; ++e) rm_[e] = (d2m){bld8(pa, om[e], 0), bld8(pa, om[e], sp)};
  };
  auto store = [&](auto BUF) XT_INLINE {
    constexpr int B = decltype(BUF)::value;
#pragma unroll
    for (int e = 0; e < A_PT; ++e)
      if (L::A % NT == 0 || tid + NT * e < L::A) smv[L::OA + B * L::A + tid + NT * e] = ra[e];
#pragma unroll
    for (int e = 0; e < W_PT; ++e)
      if (L::W % NT == 0 || tid + NT * e < L::W) smv[L::OW + B * L::W + tid + NT * e] = rw[e];
#pragma unroll
    for (int e = 0; e < R_PT; ++e)
      if (L::R % NT == 0 || tid + NT * e < L::R) smv[L::OR + B * L::R + tid + NT * e] = rr[e];
#pragma unroll
    for (int e = 0; e < M_PT; ++e)
      if (L::RM % NT == 0 || tid + NT * e < L::RM) smv[L::ORM + B * L::RM + tid + NT * e] = rm_[e];
  };

  constexpr int RVA = RV ? RV : 1;
  d4m acc[TMM > 0 ? TMM : 1][2];
#pragma unroll
  for (int t = 0; t < TMM; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[t][j] = (d4m){0.0, 0.0, 0.0, 0.0};
  double part[RVA][2];
#pragma unroll
  for (int r = 0; r < RVA; ++r) part[r][0] = part[r][1] = 0.0;

  // one K-tile: KP k-step pairs.  The B fragments of pair p + 1 are generated before the
  // MFMAs of pair p in program order (their LDS reads and the 3-deep FP64 chain overlap
  // pair p's matrix work).
  const int la = q * PI + r16, lw = q * BM_AB + r16, lr = q * PR + 3 * wave, lm = q * 8;
  auto compute = [&](auto BUF) XT_INLINE {
    constexpr int B = decltype(BUF)::value;
    const d2m* sA = smv + L::OA + B * L::A + la;
    const d2m* sW = smv + L::OW + B * L::W + lw;
    const d2m* sR = smv + L::OR + B * L::R + lr;
    const d2m* sM = smv + L::ORM + B * L::RM + lm;
    auto gen = [&](int p, double (*b)[2]) XT_INLINE {   // b[step][j]
      const d2m w0 = sR[4 * p * PR], w1 = sR[4 * p * PR + 1], w2 = sR[4 * p * PR + 2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const d2m g0 = sW[(4 * p) * BM_AB + 16 * j];
        const d2m g1 = sW[(L::NPR + 4 * p) * BM_AB + 16 * j];
        const d2m g2 = sW[(2 * L::NPR + 4 * p) * BM_AB + 16 * j];
        b[0][j] = w0[0] * g0[0] + w1[0] * g1[0] + w2[0] * g2[0];
        b[1][j] = w0[1] * g0[1] + w1[1] * g1[1] + w2[1] * g2[1];
      }
    };
    // small O (TM <= 3: 8 MFMAs per k-step pair) reads pair p + 1's fragments during pair p:
    // read in the pair that uses them, their LDS latency opened every pair with a stall
    constexpr bool FA = TM <= 3;
    d2m af[FA ? 2 : 1][TMM > 0 ? TMM : 1], mr[FA ? 2 : 1][RVA];
    auto frag = [&](int p, int sl) XT_INLINE {  // pair p's A fragments and remainder values
#pragma unroll
      for (int t = 0; t < TMM; ++t) af[sl][t] = sA[4 * p * PI + 16 * t];
      if constexpr (RV > 0) {
#pragma unroll
        for (int r = 0; r < RV; ++r) mr[sl][r] = sM[4 * p * 8 + r];
      }
    };
    auto mma = [&](double (*b)[2], int sl) XT_INLINE {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        if constexpr (RV > 0) {
#pragma unroll
          for (int r = 0; r < RV; ++r) {
            part[r][0] += mr[sl][r][st] * b[st][0];
            part[r][1] += mr[sl][r][st] * b[st][1];
          }
        }
#pragma unroll
        for (int t = 0; t < TMM; ++t)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[sl][t][st], b[st][j], acc[t][j], 0, 0, 0);
      }
    };
    // Per k-step pair, one scheduling region: all its LDS reads first (pair p's fragments,
    // then pair p + 1's generator inputs), then the 2 TMM x 2 MFMAs of pair p with the
    // FP64 VALU (pair p + 1's generation, pair p's remainder rows) interleaved between them
    // -- left alone, the scheduler emitted read burst / wait / VALU burst / MFMA burst, so
    // the LDS latency and the VALU were serialised with the matrix work.
    constexpr int NMF = 2 * 2 * (TMM > 0 ? TMM : 1);
    double b[2][2][2];
    gen(0, b[0]);
    if constexpr (FA) frag(0, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      if constexpr (FA) {
        if (p + 1 < KP) frag(p + 1, (p + 1) & 1);
      } else {
        frag(p, 0);
      }
      if (p + 1 < KP) gen(p + 1, b[(p + 1) & 1]);
      mma(b[p & 1], FA ? (p & 1) : 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);   // the first fragments
#pragma unroll
      for (int k = 0; k < NMF / 4; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // four MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);   // four DS reads
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);   // up to eight VALU
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if (kt0 < kt1) {
    // K-tile kt + 1 is written to LDS right after the barrier that opens K-tile kt (its
    // buffer was last read by K-tile kt - 1) and kt + 2 is loaded right after: the
    // stores overlap the other waves' MFMAs instead of delaying the barrier (writing
    // them before the closing barrier instead: +1 %)
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    load(kt0);
    store(B0{});
    if (kt0 + 1 < kt1) load(kt0 + 1);
    __syncthreads();
    // one K-tile from buffer BUF (kt + 1 is staged into the other one)
    auto tile = [&](auto BUF, int kt) XT_INLINE {
      constexpr int B = decltype(BUF)::value;
      if (kt + 1 < kt1) store(std::integral_constant<int, B ^ 1>{});
      if (kt + 2 < kt1) load(kt + 2);
      if (wave_on) compute(BUF);
      __syncthreads();
    };
    // the younger half of the 8 waves (two per SIMD) no longer loses VALU arbitration at each
    // segment start (one static s_setprio, no flips): same box 141.30-141.49 -> 140.76-141.04
    // ms per step (rho-forward: neutral, not applied there)
    if constexpr (NW == 8)
      if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
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
        const double v = rows4(part[r][j]);
        const int i = 16 * TMM + r, a = a0 + 16 * j + r16;
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

// Block shapes by the trial pairs: relative cost of a block of NW = 8 / 4 / 2 / 1 pairs per
// a-tile = NW (its MFMA work) x (1 + the shape's overhead) / 8: smaller K-tiles mean more
// barriers and more PhiO / weight staging per MFMA (per pair, relative to NW 8 at nx = 8:
// NW 4 +12 %, NW 2 +75 %, measured at the headline shape).  A step's nx pairs
// are split into segments of one shape each (xc_pair_segments), e.g. 10 = 8 + 2.
static const double kBackMCost[4] = {1.0, 4.0 * 1.12 / 8.0, 2.0 * 1.75 / 8.0, 1.0 * 3.0 / 8.0};

struct BackMPlan { int nw, tiles, nkt, splits, kps, used, blocks; };
static BackMPlan back_m_plan(int nw, int nx, int V, int n) {
  BackMPlan p;
  p.nw = nw;
  const int bk = bm_bk(p.nw), xb = p.nw;
  p.tiles = ((nx + xb - 1) / xb) * ((V + BM_AB - 1) / BM_AB);
  p.nkt = (n + bk - 1) / bk;
  p.splits = back_m_splits(p.tiles, p.nkt, 256 * (8 / p.nw));
  p.kps = (p.nkt + p.splits - 1) / p.splits;
  p.used = (p.nkt + p.kps - 1) / p.kps;
  p.blocks = p.tiles * p.used;
  return p;
}

size_t xc_back_m_workspace_bytes(int O, int nx, int V, int n) {
  int pb[4], cnt[4];
  const int ns = xc_pair_segments(nx, kBackMCost, pb, cnt);
  size_t need = 0;
  for (int s = 0; s < ns; ++s) {
    const BackMPlan p = back_m_plan(pb[s], cnt[s], V, n);
    const size_t b = sizeof(double) * (size_t)p.splits * O * (size_t)cnt[s] * V;
    need = b > need ? b : need;
  }
  return need;
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
  if (ws_bytes < xc_back_m_workspace_bytes(O, nx, V, n)) return XT_ERR_ARG;
  const int TM = (O + 15) / 16;
  int pb[4], cnt[4];
  const int ns = xc_pair_segments(nx, kBackMCost, pb, cnt);
  // segment s: pairs [x0, x0 + cnt) -- its wv columns and accT columns, a workspace laid
  // out for its own pairs, reduced into C's column window
  for (int s = 0, x0 = 0; s < ns; x0 += cnt[s], ++s) {
    const int nxs = cnt[s];
    const BackMPlan p = back_m_plan(pb[s], nxs, V, n);
    const long slab = (long)O * nxs * V;
    const double* Rs = R + 3L * x0;
    switch (p.nw) {
      case 8: launch_back_m_tm<8>(TM, O, nxs, V, n, p.kps, p.blocks, PO, ldp, W, wc, wg, Rs, rg, ws, slab, st); break;
      case 4: launch_back_m_tm<4>(TM, O, nxs, V, n, p.kps, p.blocks, PO, ldp, W, wc, wg, Rs, rg, ws, slab, st); break;
      case 2: launch_back_m_tm<2>(TM, O, nxs, V, n, p.kps, p.blocks, PO, ldp, W, wc, wg, Rs, rg, ws, slab, st); break;
      default: launch_back_m_tm<1>(TM, O, nxs, V, n, p.kps, p.blocks, PO, ldp, W, wc, wg, Rs, rg, ws, slab, st); break;
    }
    int rb = (int)((slab + 255) / 256);
    if (rb > 8192) rb = 8192;
    hipLaunchKernelGGL(k_xc_back_m_reduce, dim3(rb), dim3(256), 0, st, O, (long)nxs * V, p.used, ws, slab,
                       C + (long)x0 * V, ldc);
  }
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
