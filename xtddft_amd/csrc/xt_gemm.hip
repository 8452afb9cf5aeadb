// FP64 MFMA GEMM for gfx950 (CDNA4), the contraction engine of the TDA hot path.
//
//   C[b](m,n) = alpha * sum_{r<R} sum_{k<K} A(b,r,m,k) * B(b,r,k,n) + beta * C[b](m,n)
//
// A(b,r,m,k) = A[b1*sAb1 + b2*sAb2 + r*sAr + m*sAm + k*sAk]   (b = b1*nb2 + b2)
// B(b,r,k,n) = B[b1*sBb1 + b2*sBb2 + r*sBr + k*sBk + n*sBn]
// Exactly one of (sAm, sAk) is 1 and one of (sBk, sBn) is 1; the contiguous
// axis is a template parameter so global loads are always coalesced.
//
// Every contraction of the MO-route A.x (DF-J/K sandwiches over the aux
// index P, the XC grid projections, the Fock/Delta-A MO products, the
// Davidson subspace products) is an instance: the "reduce" index r carries the
// second level of a two-level contraction (e.g. P in sum_P sum_b), so no
// operand is ever re-laid-out in HBM to fit a plain GEMM.
//
// Tiling: BM x BN block tile, BK-deep K tiles, WGM x WGN waves, each wave
// (BM/WGM)x(BN/WGN) made of 16x16 v_mfma_f64_16x16x4_f64 tiles (configs: kCfg).
// LDS holds As[m][k] / Bs[n][k] (k contiguous, odd row pitch BK + 1 doubles),
// double buffered with register staging.  Lane l (q = l>>4) feeds MFMA step s
// of a K-tile with k = q + 4s (k = koff(q) + s on the 64 x 64 BK 32 tile: bank-conflict-
// free fragment reads, see compute) -- the k permutation is applied identically to
// A and B, so the sum over k is unchanged.  Staging addresses are per-thread
// 32-bit offsets computed once; the K loop body is branch-free.
// C/D layout of the f64 MFMA: col = lane & 15, row = (lane >> 4) + 4*reg
// (checked on hardware, tools/mfma_probe.hip).
//
// Split-K: the reduction domain (R x ceil(K/BK) tile units) is cut into
// nsplit contiguous ranges (grid.z = nbatch * nsplit).  With nsplit > 1 every
// split writes its own slab of the workspace and xt_splitk_reduce sums the
// slabs in a fixed order (deterministic), then applies alpha/beta.

#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>
#include <type_traits>
#include <stdlib.h>
#include <map>
#include <mutex>
#include <queue>
#include <tuple>
#include <vector>
#include "xt_internal.h"

namespace xt {

typedef double d4 __attribute__((ext_vector_type(4)));

// LDS row pitch in doubles (LDP = BK + 1).  The compiler pairs the per-step fragment reads into
// ds_read2_b64, whose lane groups are 16 lanes over 32 banks: lane (q, r) of a
// group reads row r at k = q + 4s, i.e. dword 2*(LDP*r + q) mod 32, which is
// conflict-free for any odd pitch.  Odd pitch also keeps both staging stores
// (16 consecutive k of one row, or one k of 16 consecutive rows) conflict-free.
// Kernel-local lambdas capture register arrays (accumulators, staging) by
// reference: they must inline, or the arrays are demoted to scratch memory.
#define XT_INLINE __attribute__((always_inline))
constexpr int GROUP_M = 8;       // m-tiles per grouped sweep over n (L2 panel reuse)

// Sum of v over the four 16-lane rows of the wave (lanes l, l^16, l^32, l^48),
// identical in every lane, on the VALU: v_permlane16/32_swap of a register with
// itself leaves row pairs split across the two results, whose sum is the pair
// sum in every lane (ds_bpermute-based __shfl_xor goes through the LDS pipe).
__device__ __forceinline__ double rows_sum4(double v) {
  auto pair16 = [](double x) XT_INLINE {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
  };
  auto pair32 = [](double x) XT_INLINE {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
  };
  return pair32(pair16(v));
}

// Row-pair swaps (v_permlane32_swap / v_permlane16_swap on both halves of a double):
// swap32(A, B) exchanges A's lanes 32-63 with B's lanes 0-31; swap16(A, B) A's lanes
// 16-31 / 48-63 with B's 0-15 / 32-47.  After swap32(A, B); A += B the lower half
// holds A summed over the two halves and the upper half B's; swap16 then does the
// same inside each half: a transposing 4-row reduction (each row of lanes ends
// with the full sum of one of four values).
__device__ __forceinline__ void swap32_d(double& A, double& B) {
  const unsigned alo = (unsigned)__double2loint(A), ahi = (unsigned)__double2hiint(A);
  const unsigned blo = (unsigned)__double2loint(B), bhi = (unsigned)__double2hiint(B);
  const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
  A = __hiloint2double((int)hi[0], (int)lo[0]);
  B = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap16_d(double& A, double& B) {
  const unsigned alo = (unsigned)__double2loint(A), ahi = (unsigned)__double2hiint(A);
  const unsigned blo = (unsigned)__double2loint(B), bhi = (unsigned)__double2hiint(B);
  const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
  A = __hiloint2double((int)hi[0], (int)lo[0]);
  B = __hiloint2double((int)hi[1], (int)lo[1]);
}

// TAG only gives hot call sites their own kernel symbol (rocprofv3 identity).
// MINW = waves per SIMD the register budget must allow (occupancy target).
// MODE: 0 plain GEMM, 1 / 2 fused XC contractions (XcFuse, xt_internal.h).
// ROWSIMD: waves w and w + 4 share a SIMD; by default wn = w % WGN, so with WGN = 4
// the column index picks the SIMD and a ragged last column tile (N % BN small) lands
// on one SIMD.  ROWSIMD (WGM = 4) takes wm = w % 4 instead: a ragged column edge then
// spreads over all four SIMDs (a ragged row edge concentrates).
template <int BM, int BN, int WGM, int WGN, int BK, int MINW, bool A_KC, bool B_KC, int TAG, int MODE = 0,
          int MAP = 0, bool ROWSIMD = false, bool KMASK = true>
__global__ void __launch_bounds__(64 * WGM * WGN, MINW)
dgemm_kernel(GemmParams p) {
  static_assert(MODE == 0 || ((BM == 128 || (MODE == 2 && BM == 64)) && WGM * WGN == 8 && !A_KC && B_KC),
                "fused XC modes run on 128-row (mode 2 also 64-row) 8-wave tiles, A MN-contiguous, "
                "B staged K-contiguous");
  static_assert(MODE != 2 || (WGM == 2 && WGN == 4), "mode 2 staging map assumes 2x4 waves");
  // (Pitch 18 for the k-contiguous BK 16 tiles makes their ds_read_b64 fragment reads
  // conflict-free but measured slower: C2 forward U 1.71-1.74 -> 1.76 ms, same box.)
  constexpr int LDP = BK + 1;
  constexpr int NTHREADS = 64 * WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;    // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;      // MFMA tiles per wave
  constexpr int A_ELEMS = BM * BK / NTHREADS;    // doubles staged per thread
  constexpr int B_ELEMS = BN * BK / NTHREADS;
  constexpr int STAGE = (BM + BN) * LDP;         // one LDS buffer (A then B)
  // staging geometry: a K-contiguous operand is staged as k = tid % BK of rows
  // tid / BK + e * STEP; an MN-contiguous one as m = tid % BM of k-rows tid / BM + e * STEP
  constexpr int A_STEP = A_KC ? NTHREADS / BK : NTHREADS / BM;
  constexpr int B_STEP = B_KC ? NTHREADS / BK : NTHREADS / BN;
  static_assert(NTHREADS % BK == 0 && NTHREADS % BM == 0 && NTHREADS % BN == 0, "staging map");

  // mode 1 also stages the gradient weights of the current a-block (3 BN rows of 16, pitch 17)
  constexpr int WSZ = MODE == 1 ? 3 * BN * 17 : 0;
  __shared__ __attribute__((aligned(16))) double smem[2 * STAGE + WSZ];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);   // wave-uniform (SGPR) copy
  const int wm = ROWSIMD ? wave_u % WGM : wave_u / WGN;
  const int wn = ROWSIMD ? wave_u / WGM : wave_u % WGN;
  const int q = lane >> 4, r16 = lane & 15;

  // ---- block -> (tile, batch, split) ---------------------------------------
  // Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
  // "Workgroup dispatch"); renumber so each XCD runs a contiguous range of
  // tiles, and walk tiles in GROUP_M-tall column sweeps so the blocks resident
  // on one XCD share A and B panels in its L2.
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int ntile = tiles_m * tiles_n;
  int lid = blockIdx.x + ntile * blockIdx.z;
  {
    const int nblk = ntile * gridDim.z;
    const int xcd = lid & 7, idx = lid >> 3, qn = nblk >> 3, rem = nblk & 7;
    lid = xcd * qn + (xcd < rem ? xcd : rem) + idx;
  }
  const int z = lid / ntile;
  const int tile = lid - z * ntile;
  const int per_group = GROUP_M * tiles_n;
  const int first_m = (tile / per_group) * GROUP_M;
  const int gsz = (tiles_m - first_m < GROUP_M) ? tiles_m - first_m : GROUP_M;
  const int tm = first_m + (tile % per_group) % gsz;
  const int tn = (tile % per_group) / gsz;
  const int split = z % p.nsplit;
  const int b = z / p.nsplit;
  const int b1 = b / p.nb2, b2 = b % p.nb2;

  const int m0 = tm * BM, n0 = tn * BN;
  const int nkt = (p.K + BK - 1) / BK;
  // mode 2: n-tile tn covers xg-block tn % nxb (XGB = BN / 16 xg) x a-block tn / nxb (16 a)
  constexpr int XGB = BN / 16;
  const int nxb = (p.fz.nx + XGB - 1) / XGB;
  const int xg_blk = MODE == 2 ? tn % nxb : 0, a_blk = MODE == 2 ? tn / nxb : 0;
  const long units = (long)p.R * nkt;
  const long u_per = (units + p.nsplit - 1) / p.nsplit;
  const long u0 = split * u_per;
  const long u1 = (u0 + u_per < units) ? (u0 + u_per) : units;

  const double* __restrict__ Ab = p.A + b1 * p.sAb1 + b2 * p.sAb2 +
                                  (MODE == 1 || p.rdiv ? 0L : (A_KC ? (long)m0 * p.sAm : (long)m0));
  const double* __restrict__ Bb = p.B + b1 * p.sBb1 + b2 * p.sBb2 +
                                  (B_KC ? (long)n0 * p.sBn : (long)n0);

  d4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};

  // Per-thread byte offsets from the tile origin, fixed for the whole K loop.
  // Rows (cols) past M (N) are clamped to the last valid one: they only feed
  // accumulator rows (cols) that are never stored.  32-bit offsets: dgemm()
  // rejects strides that would overflow them.
  const int a_fix = A_KC ? tid % BK : tid % BM, a_var = A_KC ? tid / BK : tid / BM;
  const int b_fix = B_KC ? tid % BK : tid % BN, b_var = B_KC ? tid / BK : tid / BN;
  unsigned aoff[A_ELEMS], boff[B_ELEMS];
  // mode 1 rows m = 16 xg + a_l sit at xg * ablk + a_l (the a-block via r * sAr)
  auto rowoff = [&](int mg) XT_INLINE -> long {
    if (MODE == 0 && !A_KC && p.rdiv) return (long)(mg / p.rdiv) * p.sAm_hi + mg % p.rdiv;
    return MODE == 1 ? (long)(mg >> 4) * p.fz.ablk + (mg & 15) : (long)(mg - m0);
  };
#pragma unroll
  for (int e = 0; e < A_ELEMS; ++e) {
    if (A_KC) {
      int mm = min(m0 + a_var + e * A_STEP, p.M - 1) - m0;
      aoff[e] = (unsigned)(((long)mm * p.sAm + a_fix) * 8);
    } else {
      const long mo = rowoff(min(m0 + a_fix, p.M - 1));
      aoff[e] = (unsigned)(((long)(a_var + e * A_STEP) * p.sAk + mo) * 8);
    }
  }
#pragma unroll
  for (int e = 0; e < B_ELEMS; ++e) {
    if (B_KC) {
      int nn = min(n0 + b_var + e * B_STEP, p.N - 1) - n0;
      boff[e] = (unsigned)(((long)nn * p.sBn + b_fix) * 8);
    } else {
      int nn = min(n0 + b_fix, p.N - 1) - n0;
      boff[e] = (unsigned)(((long)(b_var + e * B_STEP) * p.sBk + nn) * 8);
    }
  }
  // mode 2 staging maps: thread -> k row g2, NX xg (local xg_l) x NU a (local a_l)
  //  BK 32 x BN 128 (8 xg x 16 a): g2 = 4 wave + (tid >> 2 & 3), xg_l = 2 (tid >> 4 & 3) + x,
  //    a_l = 4 (tid & 3) + u: 6 rho + 12 gradient loads for 8 elements, each wave-load
  //    touching 4 grid rows; the LDS stores of a 16-lane group land on 16 distinct
  //    bank pairs (4 rows x 4 quads, pitch 33).
  //  BK 16 x BN 64 (4 xg x 16 a): g2 = tid >> 5, xg_l = tid >> 3 & 3, a_l = 2 (tid & 7) + u:
  //    3 rho + 6 gradient loads for 2 elements; stores of a 16-lane group hit
  //    columns 2 ap + u + {0, 16} (pitch 17: distinct bank pairs).
  //  MAP 1, BK 16 x BN 64: g2 = tid >> 5, xg_l = 2 (tid >> 4 & 1) + x, a_l = tid & 15: a
  //    16-lane group covers the 16 a of one xg -- coalesced 128-B gradient loads, one
  //    broadcast rho load per (xg, c), and LDS stores on 16 distinct bank pairs
  //    (MAP 0 puts two xg 16 columns apart in one group: 2-way ds_write_b64 conflicts).
  static_assert(MODE != 2 || (BK == 32 && BN == 128 && NTHREADS == 512) ||
                (BK == 16 && BN == 64 && NTHREADS == 512), "mode 2 staging map");
  static_assert(MAP == 0 || (BK == 16 && BN == 64), "MAP 1 is the BK 16 x BN 64 map");
  constexpr int NX = BN == 128 ? 2 : (MAP == 1 ? 2 : 1), NU = BN == 128 ? 4 : (MAP == 1 ? 1 : 2);
  const int g2 = BN == 128 ? (tid >> 6) * 4 + ((tid >> 2) & 3) : tid >> 5;
  auto xg_loc = [&](int x) XT_INLINE {
    return BN == 128 ? 2 * ((tid >> 4) & 3) + x : (MAP == 1 ? 2 * ((tid >> 4) & 1) + x : (tid >> 3) & 3);
  };
  auto a_loc = [&](int u) XT_INLINE {
    return BN == 128 ? 4 * (tid & 3) + u : (MAP == 1 ? (tid & 15) : 2 * (tid & 7) + u);
  };
  int xg2[NX], a2[NU];
  bool ok2[NX][NU];
#pragma unroll
  for (int x = 0; x < NX; ++x) xg2[x] = xg_blk * XGB + xg_loc(x);
#pragma unroll
  for (int u = 0; u < NU; ++u) a2[u] = a_blk * 16 + a_loc(u);
#pragma unroll
  for (int x = 0; x < NX; ++x)
#pragma unroll
    for (int u = 0; u < NU; ++u) ok2[x][u] = xg2[x] < p.fz.nx && a2[u] < p.fz.V;
#pragma unroll
  for (int x = 0; x < NX; ++x) xg2[x] = xg2[x] < p.fz.nx ? xg2[x] : p.fz.nx - 1;
#pragma unroll
  for (int u = 0; u < NU; ++u) a2[u] = a2[u] < p.fz.V ? a2[u] : p.fz.V - 1;
  double bw[MODE == 2 ? NU : 1][3];                // mode 2: w_c[g][a_u]
  double br[MODE == 2 ? NX : 1][3];                // mode 2: rho[g][xg_x][c]

  double ra[A_ELEMS], rb[B_ELEMS];

  // Stage K-tile (r, kt) into registers.  Branch-free: k past K (last tile of
  // each r) reads k = 0 of the same row instead; the B copy of those k is
  // zeroed in store_tile, so they add nothing.  Returns the valid k count.
  // EDGE: the tile may reach past K (masked staging); !EDGE: a whole K-tile, staged with
  // no per-element selects (the VALU issue cycles they cost come out of the FP64 matrix
  // pipe, tools/mfma_probe2.hip)
  auto load_tile = [&](auto EDGE, int r, int kt) XT_INLINE -> int {
    constexpr bool edge = decltype(EDGE)::value;
    const int k0 = kt * BK;
    const int kv = p.K - k0;
    const char* At = (const char*)(Ab + (long)r * p.sAr + (A_KC ? (long)k0 : (long)k0 * p.sAk));
    const char* Bt = (const char*)(Bb + (long)r * p.sBr + (B_KC ? (long)k0 : (long)k0 * p.sBk));
    // buffer loads off the tile's (block-uniform) origin: 32-bit lane offsets, no 64-bit
    // address arithmetic on the VALU
    const __amdgpu_buffer_rsrc_t ars = rsrc_of((const double*)At), brs = rsrc_of((const double*)Bt);
#pragma unroll
    for (int e = 0; e < A_ELEMS; ++e) {
      unsigned o = aoff[e];
      if (!edge) {}
      else if (A_KC) o = (a_fix < kv) ? aoff[e] : aoff[e] - (unsigned)(a_fix * 8);
      else      o = (a_var + e * A_STEP < kv) ? aoff[e] : aoff[e] - (unsigned)((a_var + e * A_STEP) * p.sAk * 8);
      ra[e] = bld8(ars, o, 0);
    }
    if constexpr (MODE == 2) {
      // generated operand: raw inputs of k row g (clamped to the tile's first row past K)
      const long g = k0 + (g2 < kv ? g2 : 0);
#pragma unroll
      for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int c = 0; c < 3; ++c) br[x][c] = p.fz.rho[g * p.fz.rg + 3 * xg2[x] + c];
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int u = 0; u < NU; ++u) bw[u][c] = p.fz.w[c * p.fz.wc + g * p.fz.wg + a2[u]];
    } else {
#pragma unroll
      for (int e = 0; e < B_ELEMS; ++e) {
        unsigned o = boff[e];
        if (!edge) {}
        else if (B_KC) o = (b_fix < kv) ? boff[e] : boff[e] - (unsigned)(b_fix * 8);
        else      o = (b_var + e * B_STEP < kv) ? boff[e] : boff[e] - (unsigned)((b_var + e * B_STEP) * p.sBk * 8);
        rb[e] = bld8(brs, o, 0);
      }
    }
    return kv;
  };
  auto store_tile = [&](auto EDGE, int buf, int kv) XT_INLINE {
    constexpr bool edge = decltype(EDGE)::value;
#pragma unroll
    for (int e = 0; e < A_ELEMS; ++e) {
      int mm, kk;
      if (A_KC) { mm = a_var + e * A_STEP; kk = a_fix; } else { kk = a_var + e * A_STEP; mm = a_fix; }
      smem[buf * STAGE + mm * LDP + kk] = ra[e];
    }
    if constexpr (MODE == 2) {
#pragma unroll
      for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int nn = xg_loc(x) * 16 + a_loc(u);
          const double v = br[x][0] * bw[u][0] + br[x][1] * bw[u][1] + br[x][2] * bw[u][2];
          smem[buf * STAGE + BM * LDP + nn * LDP + g2] = (ok2[x][u] && g2 < kv) ? v : 0.0;
        }
    } else {
#pragma unroll
      for (int e = 0; e < B_ELEMS; ++e) {
        int nn, kk;
        if (B_KC) { nn = b_var + e * B_STEP; kk = b_fix; } else { kk = b_var + e * B_STEP; nn = b_fix; }
        smem[buf * STAGE + BM * LDP + nn * LDP + kk] = (!edge || kk < kv) ? rb[e] : 0.0;
      }
    }
  };
  // MFMA sub-tiles of this wave that hold any row < M / col < N; a wave whose
  // sub-tiles are all in range on a K-full tile takes the pipelined path
  int mi = (p.M - m0 - wm * WM + 15) / 16;
  int nj = (p.N - n0 - wn * WN + 15) / 16;
  mi = mi < 0 ? 0 : (mi > TM ? TM : mi);
  nj = nj < 0 ? 0 : (nj > TN ? TN : nj);
  const bool wave_full = (mi == TM) && (nj == TN);
  constexpr int SK = BK / 4;   // MFMA k-steps per tile
  // One K-tile of MFMAs, fragments software-pipelined one k-step ahead.
  // MN_EDGE: skip MFMAs of sub-tiles wholly past M / N (their accumulators are
  // never stored); K_EDGE: skip k-steps wholly past K (their B rows are zero).
  // Fragment reads stay unconditional (LDS holds clamped rows), so the read
  // pipelining is identical in every variant.
  // Lane row q's k offset inside a K-tile and the k stride between MFMA steps: k = q + 4 s,
  // except on the 64 x 64 BK 32 tile, k = koff(q) + s with koff = 0, 16, 8, 24.  The fragment
  // reads the compiler emits as ds_read_b64 serve lanes 0-31 (q = 0, 1) and 32-63 (q = 2, 3)
  // in one LDS cycle each over 64 banks: with k = q + 4 s and the odd pitch, lane (r + 1,
  // q = 0) and lane (r, q = 1) hit the same bank pair (a 2-way conflict on every read: one
  // SQ_LDS_BANK_CONFLICT cycle per LDS instruction on C2's back L, which runs this tile);
  // 16 doubles apart the two lane rows use disjoint halves of the banks (C2 back L: 0
  // conflicts, 2.15-2.19 -> 2.11-2.15 ms same box).  On the 128 x 128 BK 32 tile the same
  // permutation removes the conflicts but measured slower (headline back L 141.0-141.3 ->
  // 143.9-144.1 ms per step, same box): not applied there.
  constexpr bool KPERM = BK == 32 && BM == 64 && BN == 64;
  constexpr int KSTEP = KPERM ? 1 : 4;
  const int koff = KPERM ? 16 * (q & 1) + 8 * (q >> 1) : q;
  auto compute = [&](int buf, auto MN_EDGE, auto K_EDGE, int kv) XT_INLINE {
    constexpr bool mn_edge = decltype(MN_EDGE)::value;
    constexpr bool k_edge = decltype(K_EDGE)::value;
    const int abase = buf * STAGE + (wm * WM + r16) * LDP + koff;
    const int bbase = buf * STAGE + BM * LDP + (wn * WN + r16) * LDP + koff;
    if constexpr (MINW >= 4) {
      // >= 4 waves per SIMD hide the LDS latency across waves: single-buffered
      // fragments keep the wave inside a 128-register budget
#pragma unroll
      for (int s = 0; s < SK; ++s) {
        double af1[TM], bf1[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af1[i] = smem[abase + i * 16 * LDP + KSTEP * s];
#pragma unroll
        for (int j = 0; j < TN; ++j) bf1[j] = smem[bbase + j * 16 * LDP + KSTEP * s];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if ((!k_edge || KSTEP * s < kv) && (!mn_edge || (i < mi && j < nj)))
              acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af1[i], bf1[j], acc[i][j], 0, 0, 0);
          }
      }
      return;
    }
    double af[2][TM], bf[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[0][i] = smem[abase + i * 16 * LDP];
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[0][j] = smem[bbase + j * 16 * LDP];
#pragma unroll
    for (int s = 0; s < SK; ++s) {
      const int cur = s & 1, nxt = cur ^ 1;
      if (s + 1 < SK) {   // prefetch the next step's fragments behind this step's MFMAs
#pragma unroll
        for (int i = 0; i < TM; ++i) af[nxt][i] = smem[abase + i * 16 * LDP + KSTEP * (s + 1)];
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[nxt][j] = smem[bbase + j * 16 * LDP + KSTEP * (s + 1)];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if ((!k_edge || KSTEP * s < kv) && (!mn_edge || (i < mi && j < nj)))
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[cur][i], bf[cur][j], acc[i][j], 0, 0, 0);
    }
  };

  // The K loop.  All tiles but the last run the branch-free pipelined body
  // (loads of tile u+1 interleave with the MFMAs of tile u); the last tile,
  // which is the K-edge tile whenever K % BK != 0 and R == 1, is peeled and
  // skips the k-steps past K.  Waves whose sub-tiles reach past M / N run the
  // MN_EDGE variant of the same loop (wave-uniform choice; both variants pass
  // the same barriers).
  // KMASK: ragged K inside every reduce index (R > 1, BK does not divide K): every K-tile
  // takes the masked staging.  Otherwise at most one K-tile is ragged (the last one, R == 1)
  // and it runs FIRST, staged by the prologue: the pipelined loop then stages whole tiles
  // only, with no per-element selects (the VALU issue cycles they cost come out of the
  // FP64 matrix pipe, tools/mfma_probe2.hip) and no second loop body competing for the
  // 128-register budget.  The order of the k sum changes, not its terms.
  auto run = [&](auto MN_EDGE) XT_INLINE {
    if constexpr (KMASK) {
      int r = (int)(u0 / nkt), kt = (int)(u0 % nkt);
      int kv = load_tile(std::true_type{}, r, kt);
      store_tile(std::true_type{}, 0, kv);
      __syncthreads();
      int buf = 0;
      for (long u = u0; u + 1 < u1; ++u) {
        int ktn = kt + 1, rn = r;
        if (ktn == nkt) { ktn = 0; rn = r + 1; }
        kv = load_tile(std::true_type{}, rn, ktn);
        compute(buf, MN_EDGE, std::false_type{}, BK);
        // keep the LDS stores (and their vmcnt waits) behind every MFMA of this
        // tile: hoisted into the MFMA stream they stall it on global latency
        // (measured: stores pinned mid-tile are 3-5 % slower)
        __builtin_amdgcn_sched_barrier(0);
        store_tile(std::true_type{}, buf ^ 1, kv);
        __syncthreads();
        r = rn; kt = ktn;
        buf ^= 1;
      }
      compute(buf, MN_EDGE, std::true_type{}, p.K - kt * BK);
    } else {
      const bool ragged = (p.K % BK != 0) && u1 == units;   // this split holds the ragged tile
      const long first = ragged ? units - 1 : u0;
      long u = ragged ? u0 : u0 + 1;                         // the rest: [u, rest_end)
      const long rest_end = ragged ? units - 1 : u1;
      const int kv0 = load_tile(std::true_type{}, (int)(first / nkt), (int)(first % nkt));
      store_tile(std::true_type{}, 0, kv0);
      __syncthreads();
      if (u >= rest_end) {
        compute(0, MN_EDGE, std::true_type{}, kv0);
        return;
      }
      int r = (int)(u / nkt), kt = (int)(u % nkt);
      int buf = 0;
      // the first tile (ragged or whole) under the next one's staging
      load_tile(std::false_type{}, r, kt);
      compute(0, MN_EDGE, std::true_type{}, kv0);
      __builtin_amdgcn_sched_barrier(0);
      store_tile(std::false_type{}, 1, BK);
      __syncthreads();
      buf = 1;
      for (++u; u < rest_end; ++u) {
        if (++kt == nkt) { kt = 0; ++r; }
        load_tile(std::false_type{}, r, kt);
        compute(buf, MN_EDGE, std::false_type{}, BK);
        __builtin_amdgcn_sched_barrier(0);
        store_tile(std::false_type{}, buf ^ 1, BK);
        __syncthreads();
        buf ^= 1;
      }
      compute(buf, MN_EDGE, std::false_type{}, BK);
    }
  };
  if constexpr (MODE == 1) {
    // rho forward: one a-block (16 a of the block's xg) per r; after its last
    // K-tile the accumulators (W for the block's grid points) are contracted with
    // the gradient weights and reduced over a.  Row sub-tile i holds
    // xg_l = wm TM + i (16 a each); lane q keeps the sub-tiles i = q (mod 4).
    // Runs at two blocks per CU (128-register budget): one block's reduction
    // overlaps the other's MFMAs.
    static_assert(TM % 4 == 0, "lane-q ownership of the row sub-tiles");
    constexpr int TQ = TM / 4;
    double racc[TQ][TN][3];
#pragma unroll
    for (int u = 0; u < TQ; ++u)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int c = 0; c < 3; ++c) racc[u][j][c] = 0.0;
    // Gradient weights w_c[g][a] of the block's columns and a-block r, staged
    // through LDS after the a-block's last K-tile: sw[(c BN + n) 17 + a_l] (odd
    // pitch: the reads in reduce(), 16 lanes = 16 n at one a_l, hit 16 distinct
    // bank pairs).  a >= V is stored as 0.
    constexpr int WP = 17;
    static_assert((3 * BN * 16) % NTHREADS == 0, "w staging map");
    constexpr int W_ELEMS = 3 * BN * 16 / NTHREADS;
    double wl[W_ELEMS];
    auto load_w = [&](int r) XT_INLINE {
      const int a = 16 * r + (tid & 15);
      const int acl = a < p.fz.V ? a : p.fz.V - 1;
#pragma unroll
      for (int e = 0; e < W_ELEMS; ++e) {
        const int cn = (tid >> 4) + e * (NTHREADS / 16), c = cn / BN, n = cn % BN;
        const int g = min(n0 + n, p.N - 1);
        wl[e] = p.fz.w[c * p.fz.wc + (long)g * p.fz.wg + acl];
      }
    };
    auto store_w = [&](int r) XT_INLINE {
      const bool ok = 16 * r + (tid & 15) < p.fz.V;
#pragma unroll
      for (int e = 0; e < W_ELEMS; ++e) {
        const int cn = (tid >> 4) + e * (NTHREADS / 16);
        smem[2 * STAGE + cn * WP + (tid & 15)] = ok ? wl[e] : 0.0;
      }
    };
    // contract the accumulators with the weights, reduce over the 16 a of each
    // row sub-tile (4 in-lane FMAs, then the 4 rows of lanes), clear them.  Lane row
    // q owns sub-tiles i = q (mod 4): a transposing reduction (swap32 + swap16 over
    // the four sub-tiles of a group) leaves row q with the full sum of sub-tile q --
    // 3 row swaps per (j, c, group of 4) instead of 4 all-row sums.
    static_assert(TM % 4 == 0, "transposing reduction over groups of 4 sub-tiles");
    auto reduce = [&]() XT_INLINE {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wn * WN + j * 16 + r16;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          double wz[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) wz[t] = smem[2 * STAGE + (c * BN + n) * WP + q + 4 * t];
#pragma unroll
          for (int g4 = 0; g4 < TM / 4; ++g4) {
            double v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const d4 a = acc[4 * g4 + i][j];
              v[i] = a[0] * wz[0] + a[1] * wz[1] + a[2] * wz[2] + a[3] * wz[3];
            }
            swap32_d(v[0], v[2]); v[0] += v[2];
            swap32_d(v[1], v[3]); v[1] += v[3];
            swap16_d(v[0], v[1]); v[0] += v[1];
            racc[g4][j][c] += v[0];
          }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
      }
    };
    auto run1 = [&](auto MN_EDGE) XT_INLINE {
      int kv = load_tile(std::true_type{}, 0, 0);
      store_tile(std::true_type{}, 0, kv);
      __syncthreads();
      int buf = 0;
      for (int r = 0; r < p.R; ++r) {
        for (int kt = 0; kt + 1 < nkt; ++kt) {
          kv = load_tile(std::true_type{}, r, kt + 1);
          compute(buf, MN_EDGE, std::false_type{}, BK);
          __builtin_amdgcn_sched_barrier(0);
          store_tile(std::true_type{}, buf ^ 1, kv);
          __syncthreads();
          buf ^= 1;
        }
        kv = load_tile(std::true_type{}, r + 1 < p.R ? r + 1 : r, 0);   // first tile of the next a-block
        compute(buf, MN_EDGE, std::true_type{}, p.K - (nkt - 1) * BK);
        __builtin_amdgcn_sched_barrier(0);
        store_tile(std::true_type{}, buf ^ 1, kv);
        __syncthreads();
        buf ^= 1;
        // (prefetching the weights under the K loop costs registers past the
        // two-blocks-per-CU budget; an LDS-DMA prefetch and a reduction
        // interleaved into the next a-block's MFMAs both measured slower)
        load_w(r);
        store_w(r);
        __syncthreads();
        reduce();
      }
    };
    if (nkt > 0) {
      if (wave_full) run1(std::false_type{});
      else           run1(std::true_type{});
    }
#pragma unroll
    for (int u = 0; u < TQ; ++u) {
      const int xg = (m0 >> 4) + wm * TM + 4 * u + q;
      if (xg < p.fz.nx) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int g = n0 + wn * WN + j * 16 + r16;
          if (g < p.N)
#pragma unroll
            for (int c = 0; c < 3; ++c) p.fz.rho[(long)g * p.fz.rg + 3 * xg + c] = racc[u][j][c];
        }
      }
    }
    return;
  } else {
    if (u0 < u1) {
      if (wave_full) run(std::false_type{});
      else           run(std::true_type{});
    }
  }

  // ---- epilogue ------------------------------------------------------------
  // mode 2: logical column n -> C column xg V + a (-1: padding, not stored)
  auto ccol = [&](int nl) XT_INLINE -> long {
    if (MODE != 2) return nl;
    const int c = nl - n0;
    const int xg = xg_blk * XGB + c / 16, a = a_blk * 16 + (c & 15);
    return (xg < p.fz.nx && a < p.fz.V) ? (long)xg * p.fz.V + a : -1L;
  };
  if (p.nsplit > 1) {
    double* W = p.ws + ((long)split * p.nbatch + b) * (long)p.M * p.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          int gm = m0 + wm * WM + i * 16 + q + 4 * t;
          int gn = n0 + wn * WN + j * 16 + r16;
          if (gm < p.M && gn < p.N) W[(long)gm * p.N + gn] = acc[i][j][t];
        }
  } else {
    double* Cb = p.C + b1 * p.sCb1 + b2 * p.sCb2;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          int gm = m0 + wm * WM + i * 16 + q + 4 * t;
          int gn = n0 + wn * WN + j * 16 + r16;
          const long cn = ccol(gn);
          if (gm < p.M && gn < p.N && cn >= 0) {
            const long crow = p.rdiv ? (long)(gm / p.rdiv) * p.sC_hi + (long)(gm % p.rdiv) * p.ldc : (long)gm * p.ldc;
            double* c = Cb + crow + cn;
            double v = p.alpha * acc[i][j][t];
            if (p.beta != 0.0) v += p.beta * (*c);
            *c = v;
          }
        }
  }
}

__global__ void splitk_reduce(GemmParams p) {
  const long mn = (long)p.M * p.N;
  const long total = mn * p.nbatch;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int b = (int)(idx / mn);
    const long e = idx % mn;
    const int m = (int)(e / p.N), n = (int)(e % p.N);
    long cn = n;
    if (p.fz.mode == 2) {   // logical column -> xg V + a (see dgemm_kernel mode 2)
      const int bn = p.fz.mbn, xgb = bn / 16;
      const int nxb = (p.fz.nx + xgb - 1) / xgb, tn = n / bn, cc = n % bn;
      const int xg = (tn % nxb) * xgb + cc / 16, a = (tn / nxb) * 16 + (cc & 15);
      if (xg >= p.fz.nx || a >= p.fz.V) continue;
      cn = (long)xg * p.fz.V + a;
    }
    double s = 0.0;
    for (int sp = 0; sp < p.nsplit; ++sp) s += p.ws[((long)sp * p.nbatch + b) * mn + e];
    const int b1 = b / p.nb2, b2 = b % p.nb2;
    const long crow = p.rdiv ? (long)(m / p.rdiv) * p.sC_hi + (long)(m % p.rdiv) * p.ldc : (long)m * p.ldc;
    double* c = p.C + b1 * p.sCb1 + b2 * p.sCb2 + crow + cn;
    double v = p.alpha * s;
    if (p.beta != 0.0) v += p.beta * (*c);
    *c = v;
  }
}

// Tile configurations.  C8: 128x128, 8 waves (64x32 each), BK 32, one block
// per CU (135 KB LDS); with BK 16 (70 KB) two such blocks share a CU, so one
// block's barrier / prologue / epilogue hides under the other's MFMAs.
// C4: 4 waves of 64x64.  Narrow tiles for small M or N.
struct Cfg { int bm, bn, bk, slots, wgm, wgn; };
static const Cfg kCfg[] = {   // (bm, bn, bk, concurrent block slots, wgm, wgn)
  {128, 128, 32, 256, 2, 4},   // 0: C8
  {128, 128, 16, 512, 2, 2},   // 1: C4
  {128, 64, 32, 256, 2, 2},    // 2
  {64, 128, 32, 256, 2, 2},    // 3
  {64, 64, 32, 512, 2, 2},     // 4
  {128, 128, 16, 512, 2, 4},   // 5: C8 with BK 16, two blocks per CU
  {256, 128, 16, 256, 4, 2},   // 6: 256x128, 8 waves of 64x64, BK 16 (tuning only)
  {128, 64, 16, 512, 2, 4},    // 7: 128x64, 8 waves of 64x16, BK 16, two blocks per CU
  {128, 128, 16, 512, 4, 2},   // 8: cfg 5 as 8 waves of 32x64 with rows on the SIMDs (ROWSIMD)
  {128, 128, 32, 256, 4, 2},   // 9: cfg 8 with BK 32, one block per CU (both operands k-strided)
};

template <int BM, int BN, int WGM, int WGN, int BKT, int MINW, bool AK, bool BKc, int TAG, int MODE = 0,
          int MAP = 0, bool ROWSIMD = false>
static void launch_one(const GemmParams& p, hipStream_t st) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const dim3 grid(tiles, 1, p.nbatch * p.nsplit), blk(64 * WGM * WGN);
  // the fused modes and ragged K under several reduce indices stage every tile masked (the
  // latter under the untagged symbol: one masked instantiation per layout, not per call site)
  if (MODE != 0)
    hipLaunchKernelGGL((dgemm_kernel<BM, BN, WGM, WGN, BKT, MINW, AK, BKc, TAG, MODE, MAP, ROWSIMD, true>), grid, blk,
                       0, st, p);
  else if (p.R > 1 && p.K % BKT != 0)
    hipLaunchKernelGGL((dgemm_kernel<BM, BN, WGM, WGN, BKT, MINW, AK, BKc, 0, 0, MAP, ROWSIMD, true>), grid, blk, 0,
                       st, p);
  else
    hipLaunchKernelGGL((dgemm_kernel<BM, BN, WGM, WGN, BKT, MINW, AK, BKc, TAG, MODE, MAP, ROWSIMD, false>), grid,
                       blk, 0, st, p);
}

// Engine shapes measured and removed: mode 1 on 128-point grid tiles
// (one block per CU), mode 2 on a 128-wide column tile (BK 32) and with the old
// staging map (2-way ds_write_b64 conflicts).
int xc_m_bn() { return 64; }

// Tagged call sites get their own kernel symbol for their one operand layout:
// 1 exchange contraction (A k-contig, B n-contig), 2 XC forward U (k, k),
// 3 XC back L (m, n), 4 XC forward W (k, n), 5 XC back M (m, n).
template <int BM, int BN, int WGM, int WGN, int BKT, int MINW, bool RS = false>
static void launch_cfg(const GemmParams& p, hipStream_t st, bool akc, bool bkc, int tag) {
  if (tag == 1 && akc && !bkc) launch_one<BM, BN, WGM, WGN, BKT, MINW, true, false, 1, 0, 0, RS>(p, st);
  else if (tag == 2 && akc && bkc) launch_one<BM, BN, WGM, WGN, BKT, MINW, true, true, 2, 0, 0, RS>(p, st);
  else if (tag == 3 && !akc && !bkc) launch_one<BM, BN, WGM, WGN, BKT, MINW, false, false, 3, 0, 0, RS>(p, st);
  else if (tag == 4 && akc && !bkc) launch_one<BM, BN, WGM, WGN, BKT, MINW, true, false, 4, 0, 0, RS>(p, st);
  else if (tag == 5 && !akc && !bkc) launch_one<BM, BN, WGM, WGN, BKT, MINW, false, false, 5, 0, 0, RS>(p, st);
  else if (akc && bkc) launch_one<BM, BN, WGM, WGN, BKT, MINW, true, true, 0, 0, 0, RS>(p, st);
  else if (akc)        launch_one<BM, BN, WGM, WGN, BKT, MINW, true, false, 0, 0, 0, RS>(p, st);
  else if (bkc)        launch_one<BM, BN, WGM, WGN, BKT, MINW, false, true, 0, 0, 0, RS>(p, st);
  else                 launch_one<BM, BN, WGM, WGN, BKT, MINW, false, false, 0, 0, 0, RS>(p, st);
}

size_t dgemm_workspace_bytes(const GemmDesc& d) {
  // mirrors the split choice in dgemm(); callers size their workspace with it
  GemmParams p; int cfg;
  plan_gemm(d, &p, &cfg);
  if (p.nsplit <= 1) return 0;
  return sizeof(double) * (size_t)p.nsplit * p.nbatch * (size_t)p.M * p.N;
}

// Relative MFMA time of a tile with vm valid rows / vn valid cols: the busiest
// SIMD's share (waves w and w + 4 share a SIMD; MN-edge waves skip their
// out-of-range 16x16 sub-tiles), 1 for an interior tile.
static bool cfg_rowsimd(const Cfg& c) { return &c == &kCfg[8] || &c == &kCfg[9]; }

static double tile_cost(const Cfg& c, int vm, int vn) {
  const int WM = c.bm / c.wgm, WN = c.bn / c.wgn, TM = WM / 16, TN = WN / 16;
  const int nw = c.wgm * c.wgn;
  const bool rs = cfg_rowsimd(c);
  double simd[4] = {0, 0, 0, 0};
  for (int w = 0; w < nw; ++w) {
    const int wm = rs ? w % c.wgm : w / c.wgn, wn = rs ? w / c.wgm : w % c.wgn;
    int mi = (vm - wm * WM + 15) / 16, nj = (vn - wn * WN + 15) / 16;
    mi = mi < 0 ? 0 : (mi > TM ? TM : mi);
    nj = nj < 0 ? 0 : (nj > TN ? TN : nj);
    simd[w % 4] += mi * nj;
  }
  const double full = (double)((nw + 3) / 4) * TM * TN;
  double mx = 0;
  for (double v : simd) mx = v > mx ? v : mx;
  return mx / full;
}

// Split-K count: list-schedule the blocks of each candidate split over the
// chip's concurrent block slots (tile categories interior / M-edge / N-edge /
// corner, each block = cost x K-tiles + a fixed prologue/epilogue) and add the
// split-K reduction's HBM time; keep >= 8 K-tiles per split.  Cached per shape.
static int choose_split(const Cfg& c, int M, int N, long nbatch, long units) {
  const int tm = (M + c.bm - 1) / c.bm, tn = (N + c.bn - 1) / c.bn;
  const long tiles = (long)tm * tn * nbatch;
  if (tiles >= 4L * c.slots || units < 16) return 1;
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, long, long>, int> cache;
  const auto key = std::make_tuple((int)(&c - kCfg), M, N, nbatch, units);
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  const int vm = M - (tm - 1) * c.bm, vn = N - (tn - 1) * c.bn;
  const double cost[4] = {tile_cost(c, c.bm, c.bn), tile_cost(c, vm, c.bn),
                          tile_cost(c, c.bm, vn), tile_cost(c, vm, vn)};
  const long cnt[4] = {(long)(tm - 1) * (tn - 1) * nbatch, (long)(tn - 1) * nbatch,
                       (long)(tm - 1) * nbatch, nbatch};
  const double t_kt = 2.0 * c.bm * c.bn * c.bk * c.slots / 70e12;   // s per K-tile per block
  const double t_blk = 2e-6;                                        // prologue + epilogue
  int best = 1;
  double best_t = 1e30;
  for (int s = 1; s <= 64; ++s) {
    if (s > 1 && units / s < 8) break;
    if (tiles * s > 32768) break;
    const long ku = (units + s - 1) / s;
    std::priority_queue<double, std::vector<double>, std::greater<double>> slots;
    for (int i = 0; i < c.slots; ++i) slots.push(0.0);
    double span = 0.0;
    for (int k = 0; k < 4; ++k)
      for (long b = 0; b < cnt[k] * s; ++b) {
        const double t = slots.top() + cost[k] * ku * t_kt + t_blk;
        slots.pop();
        slots.push(t);
        span = t > span ? t : span;
      }
    if (s > 1) span += (s + 1.0) * M * N * nbatch * 8.0 / 4e12 + 4e-6;
    if (span < best_t * 0.995) { best_t = span; best = s; }
  }
  std::lock_guard<std::mutex> g(mu);
  cache[key] = best;
  return best;
}

void plan_gemm(const GemmDesc& d, GemmParams* pp, int* cfg_out) {
  GemmParams& p = *pp;
  p.M = d.M; p.N = d.N; p.K = d.K; p.R = d.R > 0 ? d.R : 1;
  p.A = d.A; p.sAm = d.sAm; p.sAk = d.sAk; p.sAr = d.sAr; p.sAb1 = d.sAb1; p.sAb2 = d.sAb2;
  p.B = d.B; p.sBk = d.sBk; p.sBn = d.sBn; p.sBr = d.sBr; p.sBb1 = d.sBb1; p.sBb2 = d.sBb2;
  p.C = d.C; p.ldc = d.ldc; p.sCb1 = d.sCb1; p.sCb2 = d.sCb2;
  p.rdiv = d.rdiv; p.sAm_hi = d.sAm_hi; p.sC_hi = d.sC_hi;
  p.alpha = d.alpha; p.beta = d.beta;
  p.nb2 = d.nb2 > 0 ? d.nb2 : 1;
  p.nbatch = (d.nb1 > 0 ? d.nb1 : 1) * p.nb2;
  p.ws = nullptr;
  p.fz = d.fz;
  if (d.fz.mode != 0) {   // fused XC modes: fixed tiles (mode 1 128x64, mode 2 64 / 128 wide)
    const Cfg& c = (d.fz.mode == 2 && d.fz.mbn == 128) ? kCfg[0] : kCfg[7];
    const long units = (long)p.R * ((d.K + c.bk - 1) / c.bk);
    p.nsplit = d.fz.mode == 1 ? 1 : choose_split(c, d.M, d.N, p.nbatch, units);
    if (d.max_split > 0 && p.nsplit > d.max_split) p.nsplit = d.max_split;
    *cfg_out = 0;
    return;
  }
  int cfg;
  // 128x128: two 8-wave blocks per CU (BK 16, 128-register budget) for every
  // layout (the k-edge fallback offsets are recomputed per load so the
  // (m-contiguous A, n-contiguous B) layout fits too: XC back L 151 -> 150 ms)
  const bool ff = (d.sAk != 1) && (d.sBk != 1);
  if (d.M >= 96 && d.N >= 96) cfg = 5;
  else if (d.M >= 96) cfg = 2;
  else if (d.N >= 96) cfg = 3;
  else cfg = 4;
  // the stored-exchange stream (skinny M, K = N = O V, HBM-bound): the 8-wave
  // two-blocks-per-CU tile keeps more loads in flight than 64x128 (21.4 -> 20.0 ms)
  if (d.tag == 1 && !ff && d.N >= 96) cfg = 5;
  if (cfg == 5 && !(d.tag == 1 && !ff)) {
    // ragged column edge: rows on the SIMDs when that makes the edge tiles cheaper
    const int vm = d.M - ((d.M + 127) / 128 - 1) * 128, vn = d.N - ((d.N + 127) / 128 - 1) * 128;
    const long tm = (d.M + 127) / 128, tn = (d.N + 127) / 128;
    auto total = [&](const Cfg& cc) {
      return (double)(tm - 1) * (tn - 1) * tile_cost(cc, 128, 128) + (double)(tn - 1) * tile_cost(cc, vm, 128) +
             (double)(tm - 1) * tile_cost(cc, 128, vn) + tile_cost(cc, vm, vn);
    };
    if (total(kCfg[8]) < 0.97 * total(kCfg[5])) cfg = 8;   // (model gains under 3 % measured neutral or worse)
  }
  // both operands k-strided (rows of A and columns of B contiguous, e.g. XC back L): BK 32 with
  // one block per CU halves the barriers per k and stages whole 256-B rows per k; rows on the
  // SIMDs (back L 150.5 -> 143.7 ms same-box; BK 32 without ROWSIMD 145.2, and BK 32 for the
  // k-contiguous forward U 132.9 -> 140.0, so it stays on this layout)
  // The stored-exchange build's two-level rows (rdiv > 0) keep their measured tile (0.80 s
  // at the headline; 0.84 s on this one).
  if (ff && d.M >= 96 && d.N >= 96 && d.rdiv == 0) cfg = 9;
  // XC back L with few virtual columns: a 128-wide tile whose ragged column edge wastes much
  // of the MFMA work (and stages whole panels for it) loses to the 64 x 64 tile (C2, N = V
  // = 147: 2.45 -> 2.10 ms per step; 128 x 64: 2.15; C5, N = 117 in one 128-wide tile: 128 x
  // 128 BK 32 stays, 2.88 against 3.22 / 3.31; C4 N = 661 and the headline N = 901 keep it
  // too)
  if (cfg == 9 && d.tag == 3) {
    const double e128 = (double)d.N / (128.0 * ((d.N + 127) / 128)), e64 = (double)d.N / (64.0 * ((d.N + 63) / 64));
    if (e128 < 0.75 && e64 - e128 > 0.12) cfg = 4;
  }
  if (d.tag == 2 || d.tag == 3) {   // tuning hooks (A/B runs, read once per process):
                                    // XT_GEMM_U_CFG / XT_GEMM_L_CFG = 2, 3, 4, 5, 8 or 9
    static const int forced[2] = {[] { const char* e = getenv("XT_GEMM_U_CFG"); return e ? atoi(e) : -1; }(),
                                  [] { const char* e = getenv("XT_GEMM_L_CFG"); return e ? atoi(e) : -1; }()};
    const int f = forced[d.tag - 2];
    if (f == 2 || f == 3 || f == 4 || f == 5 || f == 8 || f == 9) cfg = f;
  }
  const Cfg& c = kCfg[cfg];
  const long units = (long)p.R * ((d.K + c.bk - 1) / c.bk);
  int nsplit = choose_split(c, d.M, d.N, p.nbatch, units);
  if (d.max_split > 0 && nsplit > d.max_split) nsplit = d.max_split;
  p.nsplit = nsplit;
  *cfg_out = cfg;
}

int dgemm(const GemmDesc& d, hipStream_t st, double* ws, size_t ws_bytes) {
  if (d.M <= 0 || d.N <= 0) return 0;
  const int mode = d.fz.mode;
  if (mode != 0 && (d.sAm != 1 || d.fz.w == nullptr || d.fz.rho == nullptr || d.fz.nx <= 0 || d.fz.V <= 0))
    return XT_ERR_ARG;
  if (mode == 1 && (d.sBk != 1 || d.nb1 > 1 || d.nb2 > 1 || d.M != 16 * d.fz.nx)) return XT_ERR_ARG;
  if (mode == 2 && (d.R > 1 || d.nb1 > 1 || d.nb2 > 1 || d.fz.mbn != xc_m_bn() ||
                    d.N != xc_m_cols(d.fz.nx, d.fz.V, d.fz.mbn))) return XT_ERR_ARG;
  const bool akc = mode == 0 && (d.sAk == 1);
  const bool bkc = mode != 0 || (d.sBk == 1);
  if (d.rdiv < 0 || (d.rdiv > 0 && (mode != 0 || d.sAm != 1 || d.sAk == 1))) return XT_ERR_ARG;
  if (!akc && d.sAm != 1) return XT_ERR_ARG;
  if (!bkc && d.sBn != 1) return XT_ERR_ARG;
  // the kernel addresses a tile with 32-bit byte offsets from its origin
  const long lim = 1L << 32;
  if ((akc ? (256L * d.sAm + 32) : (32L * d.sAk + 256L)) * 8 >= lim) return XT_ERR_ARG;
  // two-level rows: the whole row range sits in one 2 GB buffer window off the batch origin
  if (d.rdiv > 0 && (((long)(d.M / d.rdiv) * d.sAm_hi + d.rdiv + 32L * d.sAk) * 8 >= (1L << 31))) return XT_ERR_ARG;
  if ((bkc ? (256L * d.sBn + 32) : (32L * d.sBk + 256L)) * 8 >= lim) return XT_ERR_ARG;
  GemmParams p; int cfg;
  plan_gemm(d, &p, &cfg);
  if (d.K <= 0) {   // C = beta*C
    p.nsplit = 1;
    p.R = 1; p.K = 0;
  }
  if (p.nsplit > 1) {
    size_t need = sizeof(double) * (size_t)p.nsplit * p.nbatch * (size_t)p.M * p.N;
    if (ws == nullptr || ws_bytes < need) {
      // fall back to fewer splits that fit the workspace
      long per = sizeof(double) * (long)p.nbatch * p.M * p.N;
      long s = ws ? (long)(ws_bytes / per) : 0;
      p.nsplit = s >= 2 ? (int)s : 1;
      if (p.nsplit > 64) p.nsplit = 64;
    }
    p.ws = ws;
  }
  if (mode == 1) {
    launch_one<128, 64, 2, 4, 16, 4, false, true, 4, 1>(p, st);
  } else if (mode == 2) {
    // rows = occupied orbitals: a 64-row tile when they fit (small molecules)
    if (d.M <= 64) launch_one<64, 64, 2, 4, 16, 4, false, true, 5, 2, 1>(p, st);
    else           launch_one<128, 64, 2, 4, 16, 4, false, true, 5, 2, 1>(p, st);
  } else switch (cfg) {
    case 2: launch_cfg<128, 64, 2, 2, 32, 1>(p, st, akc, bkc, d.tag); break;
    case 3: launch_cfg<64, 128, 2, 2, 32, 1>(p, st, akc, bkc, d.tag); break;
    case 5: launch_cfg<128, 128, 2, 4, 16, 4>(p, st, akc, bkc, d.tag); break;
    case 8: launch_cfg<128, 128, 4, 2, 16, 4, true>(p, st, akc, bkc, d.tag); break;
    case 9: launch_cfg<128, 128, 4, 2, 32, 2, true>(p, st, akc, bkc, d.tag); break;
    default: launch_cfg<64, 64, 2, 2, 32, 2>(p, st, akc, bkc, d.tag); break;
  }
  if (p.nsplit > 1) {
    long total = (long)p.nbatch * p.M * p.N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_reduce, dim3(blocks), dim3(256), 0, st, p);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
