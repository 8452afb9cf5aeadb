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
#include "xt_internal.h"

namespace xt {

#define XT_INLINE __attribute__((always_inline))
typedef double d4x __attribute__((ext_vector_type(4)));
typedef double d2x __attribute__((ext_vector_type(2)));

constexpr int SK_MP = 48;        // padded rows (3 MFMA sub-tiles)
constexpr int SK_TM = 3;
constexpr int SK_TN = 4;         // 16-column sub-tiles per wave
constexpr int SK_WAVES = 8;
constexpr int SK_BN = 16 * SK_TN * SK_WAVES;   // 512 columns per block
constexpr int SK_BK = 64;        // k per LDS chunk (16 k-steps)
constexpr int SK_D = 4;          // B prefetch depth (k-steps)

__global__ void __launch_bounds__(512, 2)
k_skinny(int N, int K, int kchunk, const double* __restrict__ AT,
         const double* __restrict__ B, long ldb, double* __restrict__ out, long ldo) {
  __shared__ __attribute__((aligned(16))) double As[2][SK_BK * SK_MP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r = lane & 15;
  const int strip = blockIdx.x, split = blockIdx.y;
  const int k0 = split * kchunk;
  const int k1 = (k0 + kchunk < K) ? k0 + kchunk : K;
  const int nw = strip * SK_BN + wave * (16 * SK_TN);
  // this lane's 4 physical columns c0 .. c0 + 3.  Rows are readable up to ldb
  // (a multiple of 4 >= N, zero padding), so a lane with c0 < N loads its 4
  // columns whole; lanes past N load the last 4 columns and store nothing.
  const int c0 = nw + 4 * r;
  const int cl = c0 + 4 <= (int)ldb ? c0 : (int)ldb - 4;
  const int nchunks = (k1 - k0 + SK_BK - 1) / SK_BK;

  d4x acc[SK_TM][SK_TN];
#pragma unroll
  for (int i = 0; i < SK_TM; ++i)
#pragma unroll
    for (int j = 0; j < SK_TN; ++j) acc[i][j] = (d4x){0.0, 0.0, 0.0, 0.0};

  // A chunk staging: 64 k x 48 m doubles = 1536 16-B pieces, 3 per thread; rows
  // past this split's k1 are zero, which makes whole 16-step chunks safe at the end
  d2x ra[3];
  auto load_a = [&](int ch) XT_INLINE {
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const int piece = tid + 512 * e;             // 0..1535
      const int kk = piece / 24, mm = 2 * (piece % 24);
      const int k = k0 + ch * SK_BK + kk;
      const d2x v = *(const d2x*)(AT + (long)(k < K ? k : K - 1) * SK_MP + mm);
      ra[e] = k < k1 ? v : (d2x){0.0, 0.0};
    }
  };
  auto store_a = [&](int buf) XT_INLINE {
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const int piece = tid + 512 * e;
      *(d2x*)(&As[buf][(piece / 24) * SK_MP + 2 * (piece % 24)]) = ra[e];
    }
  };
  // B: k-step s of this split -> row k0 + 4 s + q, clamped to K - 1 (those rows
  // meet zero A rows); branch-free so the loads pipeline across k-steps
  auto load_b = [&](int s, d4x& v) XT_INLINE {
    const int k = k0 + 4 * s + q;
    const double* p = B + (long)(k < K ? k : K - 1) * ldb + cl;
    const d2x lo = *(const d2x*)p, hi = *(const d2x*)(p + 2);
    v = (d4x){lo[0], lo[1], hi[0], hi[1]};
  };

  d4x bq[SK_D];
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
        const d4x bv = bq[u];
        load_b(s + SK_D, bq[u]);                     // refill this ring slot
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
  // C/D layout: col = lane & 15 (= r), row = 4 reg + q; sub-tile j col r -> 4 r + j
  if (c0 >= N) return;
  double* o = out + (long)split * SK_MP * ldo;
#pragma unroll
  for (int i = 0; i < SK_TM; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int m = 16 * i + q + 4 * t;
      d4x v;
#pragma unroll
      for (int j = 0; j < SK_TN; ++j) v[j] = acc[i][j][t];
      if (c0 + 3 < N) {
        *(d2x*)(o + (long)m * ldo + c0) = (d2x){v[0], v[1]};
        *(d2x*)(o + (long)m * ldo + c0 + 2) = (d2x){v[2], v[3]};
      } else {
#pragma unroll
        for (int j = 0; j < SK_TN; ++j) if (c0 + j < N) o[(long)m * ldo + c0 + j] = v[j];
      }
    }
}

// C[m][n] = alpha * sum_s part[s][m][n] + beta * C[m][n]  (fixed summation order)
__global__ void k_skinny_reduce(int M, int N, int nsplit, const double* __restrict__ part, long ldp,
                                double alpha, double beta, double* __restrict__ C, long ldc) {
  const long total = (long)M * N;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int m = (int)(t / N), n = (int)(t % N);
    double acc = 0.0;
    for (int s = 0; s < nsplit; ++s) acc += part[((long)s * SK_MP + m) * ldp + n];
    double* c = C + (long)m * ldc + n;
    *c = alpha * acc + (beta != 0.0 ? beta * (*c) : 0.0);
  }
}

// A (M x K, row stride lda) -> AT (K x 48), zero-padded rows m >= M
__global__ void k_skinny_transpose(int M, int K, const double* __restrict__ A, long lda, double* __restrict__ AT) {
  const long total = (long)K * SK_MP;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int k = (int)(t / SK_MP), m = (int)(t % SK_MP);
    AT[t] = m < M ? A[(long)m * lda + k] : 0.0;
  }
}

int skinny_splits(int N, int K);

size_t skinny_workspace_bytes(int M, int N, int K) {
  (void)M;
  const int nsplit = skinny_splits(N, K);
  return sizeof(double) * ((size_t)K * SK_MP + (size_t)nsplit * SK_MP * N);
}

int skinny_splits(int N, int K) {
  const int strips = (N + SK_BN - 1) / SK_BN;
  int s = (2 * 256 + strips - 1) / strips;        // >= two blocks per CU over the chip
  const int max_s = (K + 4 * SK_BK - 1) / (4 * SK_BK);   // keep >= 4 chunks per split
  if (s > max_s) s = max_s;
  return s < 1 ? 1 : s;
}

int skinny_gemm(int M, int N, int K, double alpha, const double* A, long lda, const double* B, long ldb,
                double beta, double* C, long ldc, double* ws, size_t ws_bytes, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (M > SK_MP || N < 4 || K <= 0) return XT_ERR_ARG;
  if (ws_bytes < skinny_workspace_bytes(M, N, K)) return XT_ERR_ARG;
  // 16-B aligned rows, readable (zero-padded) up to column ldb >= N rounded up to 4
  if ((ldb & 3) || ldb < ((N + 3) & ~3) || (reinterpret_cast<size_t>(B) & 15)) return XT_ERR_ARG;
  if (K > (1 << 30) / SK_MP) return XT_ERR_ARG;
  const int nsplit = skinny_splits(N, K);
  int kchunk = (K + nsplit - 1) / nsplit;
  kchunk = ((kchunk + SK_BK - 1) / SK_BK) * SK_BK;
  double* AT = ws;
  double* part = ws + (size_t)K * SK_MP;
  const long tot = (long)K * SK_MP;
  hipLaunchKernelGGL(k_skinny_transpose, dim3((unsigned)((tot + 255) / 256 < 65536 ? (tot + 255) / 256 : 65536)),
                     dim3(256), 0, st, M, K, A, lda, AT);
  const int strips = (N + SK_BN - 1) / SK_BN;
  const int used = (K + kchunk - 1) / kchunk;
  hipLaunchKernelGGL(k_skinny, dim3(strips, used), dim3(512), 0, st, N, K, kchunk, AT, B, ldb, part, (long)N);
  const long mn = (long)M * N;
  hipLaunchKernelGGL(k_skinny_reduce, dim3((unsigned)((mn + 255) / 256 < 8192 ? (mn + 255) / 256 : 8192)),
                     dim3(256), 0, st, M, N, used, part, (long)N, alpha, beta, C, ldc);
  return hipGetLastError() == hipSuccess ? 0 : XT_ERR_HIP;
}

}  // namespace xt
