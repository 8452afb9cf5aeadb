// FP64 MFMA rate at the rho-forward kernel's occupancy: one 8-wave block per CU (two
// waves per SIMD), 8 independent 16x16x4 accumulators per wave, with and without the
// K loop's per-k-step LDS B-fragment reads (4 ds_read_b64) and global A loads (2).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe2.hip -o /tmp/mp2 && /tmp/mp2
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"
typedef double d4 __attribute__((ext_vector_type(4)));

// MODE 0: MFMA only; 1: + 4 ds_read_b64 per step used in the same step; 2: 1 + 2 global
// loads per step; 3: the 4 reads one step ahead; 4: 2 ds_read_b128 per step (same bytes);
// 5: 1 + 12 VALU integer ops per step; 6: 1 + a uniform scalar branch per step;
// 7: 3 + 2 global loads per step three steps ahead (a 4-slot ring, L2-resident array);
// 8: 7 over a 1 GiB array (L2 misses, the rho-forward kernel's Zp stream);
// 9: 3 with each LDS address computed by a v_add_u32 (4 independent integer VALU per step);
// 10: 3 + 2 independent v_fma_f64 per step; 11: 3 + 4 independent v_mov_b64 per step;
// 12: 4 LDS reads one step ahead at immediate offsets (no VALU: one lane base per 8 steps);
// 13: 12 + 4 independent v_add_u32 per step; 14: 12 + 2 v_fma_f64 per step
template <int MODE>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
probe(const double* __restrict__ g, double* out, int iters) {
  __shared__ __attribute__((aligned(16))) double sb[8192];
  const int tid = threadIdx.x;
  for (int i = tid; i < 8192; i += 512) sb[i] = 1e-3 * i;
  __syncthreads();
  d4 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[t][j] = (d4){0, 0, 0, 0};
  double a0 = 1e-3 * tid, a1 = 2e-3 * tid;
  double b[4] = {1.0, 1.1, 1.2, 1.3}, bn[4];
  const double* gp = g + (blockIdx.x * 512 + tid) % 65536;
  int ctr = tid;
  // MODE 7 / 8 ring: slot u % 4 holds k-step u's two A values, loaded 3 steps ahead
  const long span = MODE == 8 ? (1l << 27) : 65536;
  const double* gr = g + ((long)blockIdx.x * 4096 + tid) % span;
  double ring[4][2];
  if (MODE == 7 || MODE == 8) {
#pragma unroll
    for (int u = 0; u < 3; ++u) { ring[u][0] = gr[(u * 128) % span]; ring[u][1] = gr[(u * 128 + 64) % span]; }
  }
  if (MODE == 3 || MODE >= 9) {
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = sb[((tid + 16 * j) & 8191)];
  }
  if (MODE >= 12) {
    const double* lb = sb + (tid & 63);
    unsigned x0 = tid, x1 = tid * 3, x2 = tid * 5, x3 = tid * 7;
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = lb[16 * j];
    for (int it = 0; it < iters; it += 8) {
      const double* lp = lb + ((it * 64) & 4095);
#pragma unroll
      for (int d = 0; d < 8; ++d) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bn[j] = lp[(d + 1) * 64 + 16 * j];
        if (MODE == 13) { x0 += 3; x1 += 5; x2 += 7; x3 += 9; asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)); }
        if (MODE == 14) { a0 = __builtin_fma(a0, 1.0000001, 1e-9); a1 = __builtin_fma(a1, 1.0000001, 1e-9); }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            acc[t][jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(t ? a1 : a0, b[jj], acc[t][jj], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = bn[j];
      }
    }
    ctr = x0 ^ x1 ^ x2 ^ x3;
  } else
  if (MODE == 7 || MODE == 8) {
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = sb[((tid + 16 * j) & 8191)];
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const long u = it + d + 3;
        ring[(d + 3) % 4][0] = gr[(u * 128) % span];
        ring[(d + 3) % 4][1] = gr[(u * 128 + 64) % span];
#pragma unroll
        for (int j = 0; j < 4; ++j) bn[j] = sb[(((it + d + 1) * 64 + tid + 16 * j) & 8191)];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ring[d][t], b[j], acc[t][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = bn[j];
      }
    }
  } else
  for (int it = 0; it < iters; ++it) {
    if (MODE == 1 || MODE == 2 || MODE == 5 || MODE == 6) {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = sb[((it * 64 + tid + 16 * j) & 8191)];
    }
    if (MODE == 3 || MODE >= 10) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bn[j] = sb[(((it + 1) * 64 + tid + 16 * j) & 8191)];
    }
    if (MODE == 9) {
      // per-lane offsets that change every step (opaque to the compiler): one add each
#pragma unroll
      for (int j = 0; j < 4; ++j) bn[j] = sb[(ctr + __builtin_amdgcn_readfirstlane(it) * 64 + 16 * j * (1 + (it & 1))) & 8191];
    }
    if (MODE == 10) { a0 = __builtin_fma(a0, 1.0000001, 1e-9); a1 = __builtin_fma(a1, 1.0000001, 1e-9); }
    if (MODE == 11) {
      asm volatile("v_mov_b64 v[240:241], v[242:243]\n v_mov_b64 v[244:245], v[246:247]\n"
                   "v_mov_b64 v[248:249], v[250:251]\n v_mov_b64 v[252:253], v[254:255]" ::: "v240", "v241", "v244", "v245", "v248", "v249", "v252", "v253");
    }
    if (MODE == 4) {
      typedef double d2 __attribute__((ext_vector_type(2)));
      const d2* p2 = (const d2*)sb;
      const d2 u = p2[((it * 64 + tid) & 4095)], v = p2[((it * 64 + tid + 32) & 4095)];
      b[0] = u[0]; b[1] = u[1]; b[2] = v[0]; b[3] = v[1];
    }
    if (MODE == 2) {
      a0 = gp[(it * 128) & 65535];
      a1 = gp[(it * 128 + 64) & 65535];
    }
    if (MODE == 5) {
#pragma unroll
      for (int k = 0; k < 12; ++k) ctr = (ctr * 3 + k) ^ (ctr >> 2);
    }
    if (MODE == 6) {
      if (__builtin_amdgcn_readfirstlane(it) % 7 == 3) a0 += 1e-9;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(t ? a1 : a0, b[j], acc[t][j], 0, 0, 0);
    if (MODE == 3 || MODE >= 9) {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = bn[j];
    }
  }
  double s = ctr * 1e-30;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[t][j][0];
  if (s == 12345.0) out[0] = s;
}

int main() {
  double *g, *out;
  hipMalloc(&g, 8l << 27);
  hipMalloc(&out, 8);
  hipMemset(g, 0, 8l << 27);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int blocks : {256}) {
    for (int mode = 0; mode < 15; ++mode) {
      auto run = [&]() {
        if (mode == 0) probe<0><<<blocks, 512>>>(g, out, iters);
        if (mode == 1) probe<1><<<blocks, 512>>>(g, out, iters);
        if (mode == 2) probe<2><<<blocks, 512>>>(g, out, iters);
        if (mode == 3) probe<3><<<blocks, 512>>>(g, out, iters);
        if (mode == 4) probe<4><<<blocks, 512>>>(g, out, iters);
        if (mode == 5) probe<5><<<blocks, 512>>>(g, out, iters);
        if (mode == 6) probe<6><<<blocks, 512>>>(g, out, iters);
        if (mode == 7) probe<7><<<blocks, 512>>>(g, out, iters);
        if (mode == 8) probe<8><<<blocks, 512>>>(g, out, iters);
        if (mode == 9) probe<9><<<blocks, 512>>>(g, out, iters);
        if (mode == 10) probe<10><<<blocks, 512>>>(g, out, iters);
        if (mode == 11) probe<11><<<blocks, 512>>>(g, out, iters);
        if (mode == 12) probe<12><<<blocks, 512>>>(g, out, iters);
        if (mode == 13) probe<13><<<blocks, 512>>>(g, out, iters);
        if (mode == 14) probe<14><<<blocks, 512>>>(g, out, iters);
      };
      run();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      run();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double flops = 2.0 * 16 * 16 * 4 * 8.0 * iters * (blocks * 512 / 64);
      const char* what[15] = {"MFMA only", "+4 ds_read_b64/step", "+4 LDS +2 global loads/step",
                             "+4 LDS reads one step ahead", "+2 ds_read_b128/step", "+4 LDS +12 VALU int/step",
                             "+4 LDS + scalar branch/step", "+4 LDS ahead +2 global 3 ahead (L2)",
                             "+4 LDS ahead +2 global 3 ahead (1 GiB stream)",
                             "+4 LDS ahead, 4 int adds for the addresses", "+4 LDS ahead +2 v_fma_f64/step",
                             "+4 LDS ahead +4 v_mov_b64/step", "+4 LDS ahead, immediate offsets (no VALU)",
                             "+4 LDS imm +4 indep. v_add_u32/step", "+4 LDS imm +2 v_fma_f64/step"};
      printf("blocks %d mode %d (%s): %.1f TFLOP/s\n", blocks, mode, what[mode], flops / ms / 1e9);
    }
  }
  return 0;
}
