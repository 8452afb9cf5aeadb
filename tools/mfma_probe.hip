#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
typedef double double4_t __attribute__((ext_vector_type(4)));

// layout probe: A (16x4), B (4x16) -> D (16x16)
__global__ void layout_probe(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];   // A[i=l&15][k=l>>4]
  double b = B[(l >> 4) * 16 + (l & 15)];  // B[k=l>>4][j=l&15]
  double4_t c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];  // raw dump: lane, reg
}

__global__ void rate_probe(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double4_t c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  double s = c0[0] + c1[1] + c2[2] + c3[3];
  if (s == 12345.0) out[0] = s;
}

__global__ void fma_probe(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double c[8] = {0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(a, b, c[j]);
  }
  double s = 0; for (int j = 0; j < 8; ++j) s += c[j];
  if (s == 12345.0) out[0] = s;
}

int main() {
  std::vector<double> A(64), B(64), D(256);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i*4+k] = (i+1) + 100.0*(k+1);
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k*16+j] = (k==0) ? 1.0 : 0.0; // picks A[:,0]... use asym
  // Asymmetric: B[k][j] = (k==0)*(j+1)*1e-3... use exact ints
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k*16+j] = (k==1) ? (double)(j+1) : 0.0;
  double *dA, *dB, *dD; hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 2048);
  hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice); hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice);
  layout_probe<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost);
  // expected C[i][j] = A[i][1]*B[1][j] = (i+1+200)*(j+1)
  int ok_guide = 0, ok_f32 = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int col = l & 15;
    int row_g = (l >> 4) + 4 * r;   // guide's f64 claim
    int row_f = (l >> 4) * 4 + r;   // f32-style
    double v = D[l*4+r];
    if (v == (row_g + 1 + 200.0) * (col + 1)) ok_guide++;
    if (v == (row_f + 1 + 200.0) * (col + 1)) ok_f32++;
  }
  printf("layout: guide-map matches %d/256, f32-map matches %d/256\n", ok_guide, ok_f32);
  double* dout; hipMalloc(&dout, 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int iters = 20000; int nblk = 256 * 8; int nthr = 256;
  rate_probe<<<nblk, nthr>>>(dout, 100);
  hipDeviceSynchronize();
  hipEventRecord(e0); rate_probe<<<nblk, nthr>>>(dout, iters); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double flops = 2.0 * 16 * 16 * 4 * 4.0 * iters * (nblk * nthr / 64);
  printf("mfma_f64_16x16x4: %.1f TFLOP/s (%.3f ms)\n", flops / ms / 1e9, ms);
  fma_probe<<<nblk, nthr>>>(dout, 100); hipDeviceSynchronize();
  hipEventRecord(e0); fma_probe<<<nblk, nthr>>>(dout, iters); hipEventRecord(e1); hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  flops = 2.0 * 8 * iters * (double)(nblk * nthr);
  printf("v_fma_f64: %.1f TFLOP/s (%.3f ms)\n", flops / ms / 1e9, ms);
  return 0;
}
