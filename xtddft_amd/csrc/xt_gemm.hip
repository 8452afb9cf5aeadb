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
// Tiling: BM x BN block tile, BK = 16, WGM x WGN waves (128x128: 2x4 waves,
// 512 threads; smaller tiles 2x2), each wave (BM/WGM)x(BN/WGN) made of 16x16
// v_mfma_f64_16x16x4_f64 tiles.
// LDS holds As[m][k] / Bs[n][k] (k contiguous, row pitch 18 doubles), double
// buffered with register staging.  Lane l (q = l>>4) feeds MFMA step s of a
// K-tile with k = 4q + s, so each lane reads 4 consecutive k per operand
// (one 8-byte LDS read per MFMA step) -- the k permutation is applied
// identically to A and B, so the sum over k is unchanged.
// C/D layout of the f64 MFMA: col = lane & 15, row = (lane >> 4) + 4*reg
// (checked on hardware, tools/mfma_probe.hip).
//
// Split-K: the reduction domain (R x ceil(K/BK) tile units) is cut into
// nsplit contiguous ranges (grid.z = nbatch * nsplit).  With nsplit > 1 every
// split writes its own slab of the workspace and xt_splitk_reduce sums the
// slabs in a fixed order (deterministic), then applies alpha/beta.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "xt_internal.h"

namespace xt {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int BK = 16;
constexpr int LDP = 18;          // LDS row pitch in doubles (16 + 2 pad, keeps 16-B alignment)

// TAG only gives hot call sites their own kernel symbol (rocprofv3 identity):
// 1 = DF-exchange contraction, 2 = XC grid forward, 3 = XC grid back-projection.
template <int BM, int BN, int WGM, int WGN, bool A_KC, bool B_KC, int TAG>
__global__ void __launch_bounds__(64 * WGM * WGN, 2)
dgemm_kernel(GemmParams p) {
  constexpr int NTHREADS = 64 * WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;    // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;      // MFMA tiles per wave
  constexpr int A_ELEMS = BM * BK / NTHREADS;    // doubles staged per thread
  constexpr int B_ELEMS = BN * BK / NTHREADS;
  constexpr int STAGE = (BM + BN) * LDP;         // one LDS buffer (A then B)

  __shared__ __attribute__((aligned(16))) double smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int q = lane >> 4, r16 = lane & 15;

  // ---- block -> (tile, batch, split) ---------------------------------------
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.N + BN - 1) / BN;
  int tile = blockIdx.x;
  // group consecutive blocks along m so blocks sharing a B panel run together
  const int tm = tile % tiles_m;
  const int tn = tile / tiles_m;
  if (tn >= tiles_n) return;
  const int z = blockIdx.z;
  const int split = z % p.nsplit;
  const int b = z / p.nsplit;
  const int b1 = b / p.nb2, b2 = b % p.nb2;

  const int m0 = tm * BM, n0 = tn * BN;
  const int nkt = (p.K + BK - 1) / BK;
  const long units = (long)p.R * nkt;
  const long u_per = (units + p.nsplit - 1) / p.nsplit;
  const long u0 = split * u_per;
  const long u1 = (u0 + u_per < units) ? (u0 + u_per) : units;

  const double* __restrict__ Ab = p.A + b1 * p.sAb1 + b2 * p.sAb2;
  const double* __restrict__ Bb = p.B + b1 * p.sBb1 + b2 * p.sBb2;

  d4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};

  double ra[A_ELEMS], rb[B_ELEMS];

  // staging index maps.  K-contiguous: 16 threads cover one row's 16 k.
  // MN-contiguous: consecutive threads cover consecutive m (or n) of one k.
  auto load_tile = [&](long u) {
    const int r = (int)(u / nkt);
    const int k0 = (int)(u % nkt) * BK;
    const double* Ar = Ab + (long)r * p.sAr;
    const double* Br = Bb + (long)r * p.sBr;
#pragma unroll
    for (int e = 0; e < A_ELEMS; ++e) {
      int idx = tid + e * NTHREADS;
      int mm, kk;
      if (A_KC) { mm = idx / BK; kk = idx % BK; } else { kk = idx / BM; mm = idx % BM; }
      int gm = m0 + mm, gk = k0 + kk;
      double v = 0.0;
      if (gm < p.M && gk < p.K)
        v = A_KC ? Ar[(long)gm * p.sAm + gk] : Ar[(long)gk * p.sAk + gm];
      ra[e] = v;
    }
#pragma unroll
    for (int e = 0; e < B_ELEMS; ++e) {
      int idx = tid + e * NTHREADS;
      int nn, kk;
      if (B_KC) { nn = idx / BK; kk = idx % BK; } else { kk = idx / BN; nn = idx % BN; }
      int gn = n0 + nn, gk = k0 + kk;
      double v = 0.0;
      if (gn < p.N && gk < p.K)
        v = B_KC ? Br[(long)gn * p.sBn + gk] : Br[(long)gk * p.sBk + gn];
      rb[e] = v;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int e = 0; e < A_ELEMS; ++e) {
      int idx = tid + e * NTHREADS;
      int mm, kk;
      if (A_KC) { mm = idx / BK; kk = idx % BK; } else { kk = idx / BM; mm = idx % BM; }
      smem[buf * STAGE + mm * LDP + kk] = ra[e];
    }
#pragma unroll
    for (int e = 0; e < B_ELEMS; ++e) {
      int idx = tid + e * NTHREADS;
      int nn, kk;
      if (B_KC) { nn = idx / BK; kk = idx % BK; } else { kk = idx / BN; nn = idx % BN; }
      smem[buf * STAGE + BM * LDP + nn * LDP + kk] = rb[e];
    }
  };
  auto compute = [&](int buf) {
    const int abase = buf * STAGE + (wm * WM + r16) * LDP + 4 * q;
    const int bbase = buf * STAGE + BM * LDP + (wn * WN + r16) * LDP + 4 * q;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      double af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = smem[abase + i * 16 * LDP + s];
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = smem[bbase + j * 16 * LDP + s];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };

  if (u0 < u1) {
    load_tile(u0);
    store_tile(0);
    __syncthreads();
    int buf = 0;
    for (long u = u0; u < u1; ++u) {
      const bool more = (u + 1 < u1);
      if (more) load_tile(u + 1);
      compute(buf);
      if (more) store_tile(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // ---- epilogue ------------------------------------------------------------
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
          if (gm < p.M && gn < p.N) {
            double* c = Cb + (long)gm * p.ldc + gn;
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
    double s = 0.0;
    for (int sp = 0; sp < p.nsplit; ++sp) s += p.ws[((long)sp * p.nbatch + b) * mn + e];
    const int b1 = b / p.nb2, b2 = b % p.nb2;
    double* c = p.C + b1 * p.sCb1 + b2 * p.sCb2 + (long)m * p.ldc + n;
    double v = p.alpha * s;
    if (p.beta != 0.0) v += p.beta * (*c);
    *c = v;
  }
}

template <int BM, int BN, int WGM, int WGN, int TAG>
static void launch_tag(const GemmParams& p, hipStream_t st, bool akc, bool bkc) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles, 1, p.nbatch * p.nsplit);
  dim3 block(64 * WGM * WGN);
  if (akc && bkc)  hipLaunchKernelGGL((dgemm_kernel<BM, BN, WGM, WGN, true, true, TAG>), grid, block, 0, st, p);
  else if (akc)    hipLaunchKernelGGL((dgemm_kernel<BM, BN, WGM, WGN, true, false, TAG>), grid, block, 0, st, p);
  else if (bkc)    hipLaunchKernelGGL((dgemm_kernel<BM, BN, WGM, WGN, false, true, TAG>), grid, block, 0, st, p);
  else             hipLaunchKernelGGL((dgemm_kernel<BM, BN, WGM, WGN, false, false, TAG>), grid, block, 0, st, p);
}

template <int BM, int BN, int WGM, int WGN, bool AK, bool BKc, int TAG>
static void launch_one(const GemmParams& p, hipStream_t st) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((dgemm_kernel<BM, BN, WGM, WGN, AK, BKc, TAG>), dim3(tiles, 1, p.nbatch * p.nsplit),
                     dim3(64 * WGM * WGN), 0, st, p);
}

// Tagged call sites get their own kernel symbol for their one operand layout:
// 1 exchange contraction (A k-contig, B n-contig), 2 XC forward U (k, k),
// 3 XC back L (m, n), 4 XC forward W (k, n), 5 XC back M (m, n).
template <int BM, int BN, int WGM, int WGN>
static void launch_cfg(const GemmParams& p, hipStream_t st, bool akc, bool bkc, int tag) {
  if (tag == 1 && akc && !bkc) launch_one<BM, BN, WGM, WGN, true, false, 1>(p, st);
  else if (tag == 2 && akc && bkc) launch_one<BM, BN, WGM, WGN, true, true, 2>(p, st);
  else if (tag == 3 && !akc && !bkc) launch_one<BM, BN, WGM, WGN, false, false, 3>(p, st);
  else if (tag == 4 && akc && !bkc) launch_one<BM, BN, WGM, WGN, true, false, 4>(p, st);
  else if (tag == 5 && !akc && !bkc) launch_one<BM, BN, WGM, WGN, false, false, 5>(p, st);
  else launch_tag<BM, BN, WGM, WGN, 0>(p, st, akc, bkc);
}

size_t dgemm_workspace_bytes(const GemmDesc& d) {
  // mirrors the split choice in dgemm(); callers size their workspace with it
  GemmParams p; int bm, bn;
  plan_gemm(d, &p, &bm, &bn);
  if (p.nsplit <= 1) return 0;
  return sizeof(double) * (size_t)p.nsplit * p.nbatch * (size_t)p.M * p.N;
}

void plan_gemm(const GemmDesc& d, GemmParams* pp, int* bm_out, int* bn_out) {
  GemmParams& p = *pp;
  p.M = d.M; p.N = d.N; p.K = d.K; p.R = d.R > 0 ? d.R : 1;
  p.A = d.A; p.sAm = d.sAm; p.sAk = d.sAk; p.sAr = d.sAr; p.sAb1 = d.sAb1; p.sAb2 = d.sAb2;
  p.B = d.B; p.sBk = d.sBk; p.sBn = d.sBn; p.sBr = d.sBr; p.sBb1 = d.sBb1; p.sBb2 = d.sBb2;
  p.C = d.C; p.ldc = d.ldc; p.sCb1 = d.sCb1; p.sCb2 = d.sCb2;
  p.alpha = d.alpha; p.beta = d.beta;
  p.nb2 = d.nb2 > 0 ? d.nb2 : 1;
  p.nbatch = (d.nb1 > 0 ? d.nb1 : 1) * p.nb2;
  p.ws = nullptr;
  int bm = (d.M >= 96) ? 128 : 64;
  int bn = (d.N >= 96) ? 128 : 64;
  // small-M/N problems with few tiles prefer 64-wide tiles for parallelism
  long tiles = (long)((d.M + bm - 1) / bm) * ((d.N + bn - 1) / bn) * p.nbatch;
  if (tiles < 256 && bm == 128 && bn == 128) { bn = 64; tiles *= 2; }
  const long units = (long)p.R * ((d.K + BK - 1) / BK);
  int nsplit = 1;
  const long target = 2 * 256;   // 2 blocks per CU
  if (tiles < target && units >= 16) {
    long s = (target + tiles - 1) / tiles;
    long smax = units / 8;      // keep >= 8 K-tiles per split
    if (s > smax) s = smax;
    if (s > 64) s = 64;
    if (s > 1) nsplit = (int)s;
  }
  if (d.max_split > 0 && nsplit > d.max_split) nsplit = d.max_split;
  p.nsplit = nsplit;
  *bm_out = bm; *bn_out = bn;
}

int dgemm(const GemmDesc& d, hipStream_t st, double* ws, size_t ws_bytes) {
  if (d.M <= 0 || d.N <= 0) return 0;
  const bool akc = (d.sAk == 1);
  const bool bkc = (d.sBk == 1);
  if (!akc && d.sAm != 1) return XT_ERR_ARG;
  if (!bkc && d.sBn != 1) return XT_ERR_ARG;
  GemmParams p; int bm, bn;
  plan_gemm(d, &p, &bm, &bn);
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
  if (bm == 128 && bn == 128)      launch_cfg<128, 128, 2, 4>(p, st, akc, bkc, d.tag);
  else if (bm == 128)              launch_cfg<128, 64, 2, 2>(p, st, akc, bkc, d.tag);
  else if (bn == 128)              launch_cfg<64, 128, 2, 2>(p, st, akc, bkc, d.tag);
  else                             launch_cfg<64, 64, 2, 2>(p, st, akc, bkc, d.tag);
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
