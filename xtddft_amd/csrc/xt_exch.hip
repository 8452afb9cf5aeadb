// Skinny streaming GEMM for the stored exchange (XT_K_STORED):
//
//   C[m][n] = alpha * sum_k A[m][k] B[k][n] + beta * C[m][n],   m < M <= 48
//
// with B = the stored MO exchange matrix Kx (K x N, row-major, tens of GB,
// streamed from HBM exactly once) and A = the trial vectors of one channel
// group (M = 2 nz or nz rows), given transposed (AT[k][m], 48 columns,
// zero-padded) so its rows are contiguous.  Every Kx element feeds M MACs
// (~10 flop per byte): the kernel has to stream HBM near its peak while
// keeping the FP64 matrix cores busy, which the generic 128 x 128 GEMM tile
// (rows 40..127 of it idle, an LDS round trip and a barrier per 16-deep
// k-tile for B) cannot do.
//
// Layout: one 512-thread block per 512-column strip of C and K-split s
// (grid = strips x splits).  Each wave owns 64 columns (4 MFMA column
// sub-tiles) x all 48 rows (3 sub-tiles): 12 v_mfma_f64_16x16x4_f64 per k-step
// of 4.  B goes global -> registers straight into the MFMA B operand (no LDS,
// no barrier): lane (q, r) loads Kx[k + q][n_w + 4 r .. 4 r + 3] (2 x 16 B),
// and column sub-tile j takes element j -- sub-tile j's column r is the
// physical column 4 r + j, undone at the store.  A loads are staged through
// LDS once per 64-deep chunk for the 8 waves (As[k][m], pitch 48: the
// ds_read_b64 lane groups of one fragment hit 32 distinct double slots).  A
// ring of D = 4 k-steps of B loads is kept in flight per wave.
// K splits write partial sums to a workspace; skinny_reduce adds them in a
// fixed order (deterministic) and applies alpha / beta.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include "xt_internal.h"

namespace xt {

#define XT_INLINE __attribute__((always_inline))
typedef double d4x __attribute__((ext_vector_type(4)));
typedef double d2x __attribute__((ext_vector_type(2)));

// Two families: <1..3, 4, 64> (M <= 48: the X-TDA / SF exchange, 2 nz or nz rows; two
// blocks per CU) and <6 | 8 | 10, 2, 32> (M <= 96 / 128 / 160: larger batches and the XSF
// exchange with its four spin-adaptation source blocks, 4 nz rows; one block per CU, up to
// 160 accumulator VGPRs).
constexpr int SK_WAVES = 8;
constexpr int SK_MAXM = 160;

// SK_D: B prefetch ring depth in k-steps (Kx streams from HBM: the ring has to
// cover an HBM miss under full load, ~2-4 us, with 8 waves per CU)
// SK_RV > 0: rows 16 SK_TM .. 16 SK_TM + SK_RV - 1 (the A image keeps a third 16-row
// block) are accumulated on the VALU against the same B values (SK_RV x SK_TN FMAs
// per k-step instead of SK_TN MFMAs on a mostly empty 16-row sub-tile) and reduced
// over the four k-rows at the end: M = 40 (the headline's 2 nz) as 32 + 8.
template <int SK_TM, int SK_TN, int SK_BK, int SK_D, int SK_RV = 0>
__global__ void __launch_bounds__(512, SK_TM <= 3 ? 2 : 1)
k_skinny(int N, int K, int kchunk, const double* __restrict__ AT,
         const double* __restrict__ B, long ldb, double* __restrict__ out, long ldo) {
  constexpr int SK_MP = 16 * SK_TM + (SK_RV ? 16 : 0);   // rows of the A image
  constexpr int SK_BN = 16 * SK_TN * SK_WAVES;     // columns per block
  constexpr int A_PIECES = SK_BK * SK_MP / 2;      // 16-B pieces per chunk
  static_assert(A_PIECES % 512 == 0, "A staging map");
  constexpr int A_E = A_PIECES / 512;
  static_assert((SK_BK / 4) % SK_D == 0, "ring slots");
  __shared__ __attribute__((aligned(16))) double As[2][SK_BK * SK_MP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r = lane & 15;
  const int strip = blockIdx.x, split = blockIdx.y;
  const int k0 = split * kchunk;
  const int k1 = (k0 + kchunk < K) ? k0 + kchunk : K;
  const int nw = strip * SK_BN + wave * (16 * SK_TN);
  // this lane's SK_TN physical columns c0 .. c0 + SK_TN - 1.  Rows are readable up
  // to ldb (a multiple of 4 >= N, zero padding), so a lane with c0 < N loads its
  // columns whole; lanes past N load the last ones and store nothing.
  const int c0 = nw + SK_TN * r;
  const int cl = c0 + SK_TN <= (int)ldb ? c0 : (int)ldb - SK_TN;
  const int nchunks = (k1 - k0 + SK_BK - 1) / SK_BK;

  d4x acc[SK_TM][SK_TN];
#pragma unroll
  for (int i = 0; i < SK_TM; ++i)
#pragma unroll
    for (int j = 0; j < SK_TN; ++j) acc[i][j] = (d4x){0.0, 0.0, 0.0, 0.0};
  constexpr int RVA = SK_RV ? SK_RV : 1;
  double part[RVA][SK_TN];
#pragma unroll
  for (int i = 0; i < RVA; ++i)
#pragma unroll
    for (int j = 0; j < SK_TN; ++j) part[i][j] = 0.0;

  // A chunk staging: SK_BK k x SK_MP m doubles in 16-B pieces, A_E per thread; rows
  // past this split's k1 are zero, which makes whole chunks safe at the end
  d2x ra[A_E];
  auto load_a = [&](int ch) XT_INLINE {
#pragma unroll
    for (int e = 0; e < A_E; ++e) {
      const int piece = tid + 512 * e;
      const int kk = piece / (SK_MP / 2), mm = 2 * (piece % (SK_MP / 2));
      const int k = k0 + ch * SK_BK + kk;   // <= K + SK_BK - 1: AT's zeroed slack rows
      const d2x v = *(const d2x*)(AT + (long)k * SK_MP + mm);
      ra[e] = k < k1 ? v : (d2x){0.0, 0.0};
    }
  };
  auto store_a = [&](int buf) XT_INLINE {
#pragma unroll
    for (int e = 0; e < A_E; ++e) {
      const int piece = tid + 512 * e;
      *(d2x*)(&As[buf][(piece / (SK_MP / 2)) * SK_MP + 2 * (piece % (SK_MP / 2))]) = ra[e];
    }
  };
  // B: k-step s of this split -> row k0 + 4 s + q, clamped to K - 1 (those rows
  // meet zero A rows); branch-free so the loads pipeline across k-steps
  typedef double bvec __attribute__((ext_vector_type(SK_TN)));
  // running row pointer (no per-load clamp / 64-bit multiply): rows past K are the
  // caller's zeroed slack (SKINNY_B_SLACK rows), met by zero A rows
  const double* bp = B + (long)(k0 + q) * ldb + cl;
  const long bstep = 4 * ldb;
  auto load_b = [&](int s, bvec& v) XT_INLINE {
    (void)s;
    const double* p = bp;
    bp += bstep;
    if constexpr (SK_TN == 4) {
      const d2x lo = *(const d2x*)p, hi = *(const d2x*)(p + 2);
      v = (bvec){lo[0], lo[1], hi[0], hi[1]};
    } else {
      v = *(const d2x*)p;
    }
  };

  bvec bq[SK_D];
#pragma unroll
  for (int t = 0; t < SK_D; ++t) load_b(t, bq[t]);
  load_a(0);
  store_a(0);
  __syncthreads();
  int s = 0;   // k-step index of this split
  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = ch & 1;
    load_a(ch + 1);                                  // (past the last chunk: zeros, unused)
    // 16 k-steps per chunk, unrolled by the ring depth so the ring slots are static
#pragma unroll
    for (int t0 = 0; t0 < SK_BK / 4; t0 += SK_D) {
#pragma unroll
      for (int u = 0; u < SK_D; ++u) {
        const int kk = 4 * (t0 + u) + q;             // k within the chunk
        double af[SK_TM];
#pragma unroll
        for (int i = 0; i < SK_TM; ++i) af[i] = As[buf][kk * SK_MP + 16 * i + r];
        const bvec bv = bq[u];
        load_b(s + SK_D, bq[u]);                     // refill this ring slot
        if constexpr (SK_RV > 0) {
          const double* ar = &As[buf][kk * SK_MP + 16 * SK_TM];   // broadcast over the 16 lanes of a k-row
#pragma unroll
          for (int i = 0; i < SK_RV; ++i) {
            const double av = ar[i];
#pragma unroll
            for (int j = 0; j < SK_TN; ++j) part[i][j] += av * bv[j];
          }
        }
#pragma unroll
        for (int i = 0; i < SK_TM; ++i)
#pragma unroll
          for (int j = 0; j < SK_TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bv[j], acc[i][j], 0, 0, 0);
        ++s;
      }
    }
    // As[buf ^ 1] held chunk ch - 1, read by every wave before the previous
    // barrier; one barrier publishes chunk ch + 1
    store_a(buf ^ 1);
    __syncthreads();
  }
  // the VALU rows: sum the four k-rows (lanes r, r+16, r+32, r+48), every lane
  if constexpr (SK_RV > 0) {
#pragma unroll
    for (int i = 0; i < SK_RV; ++i)
#pragma unroll
      for (int j = 0; j < SK_TN; ++j) {
        double v = part[i][j];
        auto pair = [](double x, bool p32) XT_INLINE {
          const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
          const auto a = p32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                             : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
          const auto b = p32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                             : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
          return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
        };
        part[i][j] = pair(pair(v, false), true);
      }
  }
  // C/D layout: col = lane & 15 (= r), row = 4 reg + q; sub-tile j col r -> TN r + j
  if (c0 >= N) return;
  double* o = out + (long)split * SK_MP * ldo;
  if constexpr (SK_RV > 0) {
    if (q == 0) {
#pragma unroll
      for (int i = 0; i < SK_RV; ++i) {
        const int m = 16 * SK_TM + i;
        if (c0 + SK_TN - 1 < N) {
#pragma unroll
          for (int j = 0; j < SK_TN; j += 2)
            *(d2x*)(o + (long)m * ldo + c0 + j) = (d2x){part[i][j], part[i][j + 1]};
        } else {
#pragma unroll
          for (int j = 0; j < SK_TN; ++j) if (c0 + j < N) o[(long)m * ldo + c0 + j] = part[i][j];
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < SK_TM; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int m = 16 * i + q + 4 * t;
      bvec v;
#pragma unroll
      for (int j = 0; j < SK_TN; ++j) v[j] = acc[i][j][t];
      if (c0 + SK_TN - 1 < N) {
#pragma unroll
        for (int j = 0; j < SK_TN; j += 2) *(d2x*)(o + (long)m * ldo + c0 + j) = (d2x){v[j], v[j + 1]};
      } else {
#pragma unroll
        for (int j = 0; j < SK_TN; ++j) if (c0 + j < N) o[(long)m * ldo + c0 + j] = v[j];
      }
    }
}

// C[m][n] = alpha * sum_s part[s][m][n] + beta * C[m][n]  (fixed summation order)
__global__ void k_skinny_reduce(int M, int N, int nsplit, int MP, const double* __restrict__ part, long ldp,
                                double alpha, double beta, double* __restrict__ C, long ldc) {
  const long total = (long)M * N;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int m = (int)(t / N), n = (int)(t % N);
    double acc = 0.0;
    for (int s = 0; s < nsplit; ++s) acc += part[((long)s * MP + m) * ldp + n];
    double* c = C + (long)m * ldc + n;
    *c = alpha * acc + (beta != 0.0 ? beta * (*c) : 0.0);
  }
}

// A (M x K, row stride lda) -> AT (K x MP), zero-padded rows m >= M, and kslack
// zero rows past K
__global__ void k_skinny_transpose(int M, int K, int kslack, int MP, const double* __restrict__ A, long lda,
                                   double* __restrict__ AT) {
  const long total = (long)(K + kslack) * MP;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int k = (int)(t / MP), m = (int)(t % MP);
    AT[t] = (m < M && k < K) ? A[(long)m * lda + k] : 0.0;
  }
}

namespace {
struct SkShape { int mp, bn, bk, slots; };
// (padded rows, columns per block, k per chunk, concurrent blocks per CU)
// The A image is as tall as the smallest MFMA row count that covers M (16 / 32 / 48):
// a Davidson step with few new vectors streams Kx without the padded rows' MFMAs
// (M = 2 nz <= 16 through 48 rows made the stream matrix-pipe bound).  M = 33..40
// takes 32 MFMA rows + the VALU remainder rows (48-row image).
// Past 48 rows the one-block-per-CU shape of 2 MFMA column sub-tiles per wave, in the
// smallest of 96 / 128 / 160 rows that covers M (X-TDA Davidson steps of 25-80 vectors,
// XSF steps of 13-40: M = 2 nz or 4 nz; headline operator, same box: 30 vectors 37.8 ->
// 22.6 ms, 40 vectors 37.8 -> 23.9 ms per A.x; C4's 20-root solve 10.17-10.20 -> 10.01 s).
SkShape sk_shape(int M) {
  if (M <= 16) return {16, 16 * 4 * SK_WAVES, 64, 2};
  if (M <= 32) return {32, 16 * 4 * SK_WAVES, 64, 2};
  if (M <= 48) return {48, 16 * 4 * SK_WAVES, 64, 2};
  if (M <= 96) return {96, 16 * 2 * SK_WAVES, 32, 1};
  if (M <= 128) return {128, 16 * 2 * SK_WAVES, 32, 1};
  return {160, 16 * 2 * SK_WAVES, 32, 1};
}
}  // namespace

// K splits: the grid (strips x splits blocks) runs in rounds of the chip's block slots,
// so the split count is chosen for the fill of the last round (every block streams the
// same bytes): the fewest splits whose fill is within 2 % of the best seen, up to 8 rounds
// and >= 4 k-chunks per split.  (Slots + 1 blocks would leave one round to 22 blocks.)
static int skinny_splits_m(int M, int N, int K) {
  const SkShape sh = sk_shape(M);
  const long strips = (N + sh.bn - 1) / sh.bn, slots = (long)sh.slots * 256;
  const int max_s = (K + 4 * sh.bk - 1) / (4 * sh.bk);
  int best = 1;
  double fill = -1.0;
  for (int s = 1; s <= max_s; ++s) {
    const long blocks = strips * s, rounds = (blocks + slots - 1) / slots;
    if (rounds > 8) break;
    const double f = (double)blocks / (double)(rounds * slots);
    if (f > fill + 0.02) { fill = f; best = s; }
  }
  return best;
}

int skinny_splits(int N, int K) { return skinny_splits_m(48, N, K); }

size_t skinny_workspace_bytes(int M, int N, int K) {
  const SkShape sh = sk_shape(M);
  const int nsplit = skinny_splits_m(M, N, K);
  return sizeof(double) * ((size_t)(K + sh.bk) * sh.mp + (size_t)nsplit * sh.mp * N);
}

int skinny_gemm(int M, int N, int K, double alpha, const double* A, long lda, const double* B, long ldb,
                double beta, double* C, long ldc, double* ws, size_t ws_bytes, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (M > SK_MAXM || N < 4 || K <= 0) return XT_ERR_ARG;
  if (ws_bytes < skinny_workspace_bytes(M, N, K)) return XT_ERR_ARG;
  // 16-B aligned rows, readable (zero-padded) up to column ldb >= N rounded up to 4
  if ((ldb & 3) || ldb < ((N + 3) & ~3) || (reinterpret_cast<size_t>(B) & 15)) return XT_ERR_ARG;
  const SkShape sh = sk_shape(M);
  if (K > (1 << 30) / sh.mp) return XT_ERR_ARG;
  const int nsplit = skinny_splits_m(M, N, K);
  int kchunk = (K + nsplit - 1) / nsplit;
  kchunk = ((kchunk + sh.bk - 1) / sh.bk) * sh.bk;
  double* AT = ws;
  double* part = ws + (size_t)(K + sh.bk) * sh.mp;
  const long tot = (long)(K + sh.bk) * sh.mp;
  hipLaunchKernelGGL(k_skinny_transpose, dim3((unsigned)((tot + 255) / 256 < 65536 ? (tot + 255) / 256 : 65536)),
                     dim3(256), 0, st, M, K, sh.bk, sh.mp, A, lda, AT);
  const int strips = (N + sh.bn - 1) / sh.bn;
  const int used = (K + kchunk - 1) / kchunk;
  // M = 33..40: 32 MFMA rows + the remainder rows on the VALU (48 MFMA rows measured
  // 18.65 vs 18.1 ms per headline step)
  const bool rv = M > 32 && M <= 40;
  if (sh.mp == 16)
    hipLaunchKernelGGL((k_skinny<1, 4, 64, 4>), dim3(strips, used), dim3(512), 0, st, N, K, kchunk, AT, B, ldb, part,
                       (long)N);
  else if (sh.mp == 32)
    hipLaunchKernelGGL((k_skinny<2, 4, 64, 4>), dim3(strips, used), dim3(512), 0, st, N, K, kchunk, AT, B, ldb, part,
                       (long)N);
  else if (sh.mp == 48 && rv)
    hipLaunchKernelGGL((k_skinny<2, 4, 64, 4, 8>), dim3(strips, used), dim3(512), 0, st, N, K, kchunk, AT, B, ldb,
                       part, (long)N);
  else if (sh.mp == 48)
    hipLaunchKernelGGL((k_skinny<3, 4, 64, 4>), dim3(strips, used), dim3(512), 0, st, N, K, kchunk, AT, B, ldb, part,
                       (long)N);
  else if (sh.mp == 96)
    hipLaunchKernelGGL((k_skinny<6, 2, 32, 4>), dim3(strips, used), dim3(512), 0, st, N, K, kchunk, AT, B, ldb,
                       part, (long)N);
  else if (sh.mp == 128)
    hipLaunchKernelGGL((k_skinny<8, 2, 32, 4>), dim3(strips, used), dim3(512), 0, st, N, K, kchunk, AT, B, ldb,
                       part, (long)N);
  else
    hipLaunchKernelGGL((k_skinny<10, 2, 32, 4>), dim3(strips, used), dim3(512), 0, st, N, K, kchunk, AT, B, ldb,
                       part, (long)N);
  const long mn = (long)M * N;
  hipLaunchKernelGGL(k_skinny_reduce, dim3((unsigned)((mn + 255) / 256 < 8192 ? (mn + 255) / 256 : 8192)),
                     dim3(256), 0, st, M, N, used, sh.mp, part, (long)N, alpha, beta, C, ldc);
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
