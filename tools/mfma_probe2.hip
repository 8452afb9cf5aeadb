// FP64 MFMA rate at the rho-forward kernel's occupancy: one 8-wave block per CU (two
// waves per SIMD), 8 independent 16x16x4 accumulators per wave, with and without the
// K loop's per-k-step LDS B-fragment reads (4 ds_read_b64) and global A loads (2).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe2.hip -o /tmp/mp2 && /tmp/mp2
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
probe(const double* __restrict__ g, double* out, int iters) {
  __shared__ double sb[8192];
  const int tid = threadIdx.x;
  for (int i = tid; i < 8192; i += 512) sb[i] = 1e-3 * i;
  __syncthreads();
  d4 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[t][j] = (d4){0, 0, 0, 0};
  double a0 = 1e-3 * tid, a1 = 2e-3 * tid;
  double b[4] = {1.0, 1.1, 1.2, 1.3};
  const double* gp = g + (blockIdx.x * 512 + tid) % 65536;
  for (int it = 0; it < iters; ++it) {
    if (MODE >= 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = sb[((it * 64 + tid + 16 * j) & 8191)];
    }
    if (MODE >= 2) {
      a0 = gp[(it * 128) & 65535];
      a1 = gp[(it * 128 + 64) & 65535];
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[t][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(t ? a1 : a0, b[j], acc[t][j], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[t][j][0];
  if (s == 12345.0) out[0] = s;
}

int main() {
  double *g, *out;
  hipMalloc(&g, 8 * 65536 * 2);
  hipMalloc(&out, 8);
  hipMemset(g, 0, 8 * 65536 * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int blocks : {256, 512}) {
    for (int mode = 0; mode < 3; ++mode) {
      auto run = [&]() {
        if (mode == 0) probe<0><<<blocks, 512>>>(g, out, iters);
        if (mode == 1) probe<1><<<blocks, 512>>>(g, out, iters);
        if (mode == 2) probe<2><<<blocks, 512>>>(g, out, iters);
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
      printf("blocks %d mode %d (%s): %.1f TFLOP/s\n", blocks, mode,
             mode == 0 ? "MFMA only" : mode == 1 ? "+4 LDS reads/step" : "+2 global loads/step", flops / ms / 1e9);
    }
  }
  return 0;
}
