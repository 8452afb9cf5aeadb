// Can FP64 MFMA and FP64 VALU FMAs execute concurrently on one gfx950 SIMD?
// Each 512-thread block holds 8 waves (2 per SIMD).  Variants:
//   mfma : every wave runs v_mfma_f64_16x16x4_f64 chains
//   valu : every wave runs v_fma_f64 chains
//   mixed: waves 0-3 MFMA, waves 4-7 VALU (one of each per SIMD)
// If the pipes are independent for f64, "mixed" takes about max(t_mfma/2, t_valu/2)
// worth of the pure runs' per-wave work, i.e. its FLOP rate approaches the sum.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int KIND>   // 0 mfma, 1 valu, 2 mixed
__global__ void __launch_bounds__(512) probe(double* out, int iters_m, int iters_v) {
  const int wave = threadIdx.x >> 6;
  const bool do_m = KIND == 0 || (KIND == 2 && wave < 4);
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double s = 0.0;
  if (do_m) {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
    for (int i = 0; i < iters_m; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
      c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c4, 0, 0, 0);
      c5 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c5, 0, 0, 0);
      c6 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c6, 0, 0, 0);
      c7 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c7, 0, 0, 0);
    }
    s = c0[0] + c1[1] + c2[2] + c3[3] + c4[0] + c5[1] + c6[2] + c7[3];
  } else {
    double c[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) c[j] = j;
    for (int i = 0; i < iters_v; ++i) {
#pragma unroll
      for (int j = 0; j < 16; ++j) c[j] = fma(a, b, c[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) s += c[j];
  }
  if (s == 12345.0) out[0] = s;
}

template <int KIND>
static float run(double* d, int nblk, int im, int iv) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  probe<KIND><<<nblk, 512>>>(d, 10, 10);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  probe<KIND><<<nblk, 512>>>(d, im, iv);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  double* d;
  hipMalloc(&d, 8);
  const int nblk = 256 * 2;          // two 8-wave blocks per CU
  const int im = 4000, iv = 16000;   // per wave: 8*4000 MFMA (65.5 MFLOP) vs 16*16000 FMA lanes
  const double waves = nblk * 8.0;
  const double fm = 2.0 * 16 * 16 * 4 * 8.0 * im;     // flops per MFMA wave
  const double fv = 2.0 * 16 * iv * 64.0;             // flops per VALU wave
  float tm = run<0>(d, nblk, im, iv), tv = run<1>(d, nblk, im, iv), tx = run<2>(d, nblk, im, iv);
  printf("mfma only : %8.3f ms  %6.1f TF/s\n", tm, waves * fm / tm / 1e9);
  printf("valu only : %8.3f ms  %6.1f TF/s\n", tv, waves * fv / tv / 1e9);
  printf("mixed     : %8.3f ms  %6.1f TF/s (half the waves each; independent pipes -> ~ %.3f ms)\n", tx,
         (waves / 2 * fm + waves / 2 * fv) / tx / 1e9, (tm > tv ? tm : tv) / 2);
  return 0;
}
