// Measured dense FP64 MFMA peak of the card (the MFMA-side roofline of hbm::k_gemm):
// every wave issues independent chains of v_mfma_f64_16x16x4f64 (2048 flop each).
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_f64_peak tools/mfma_f64_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_peak(double* out, int iters, double a, double b) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  const double x = a + threadIdx.x * 1e-9, y = b - threadIdx.x * 1e-9;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, c3, 0, 0, 0);
  }
  const d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];  // vector store
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8, threads = 256, iters = 20000;
  double* out;
  if (hipMalloc(&out, sizeof(double) * blocks * threads) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_peak<<<blocks, threads>>>(out, 100, 1.0, 0.5);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    k_peak<<<blocks, threads>>>(out, iters, 1.0, 0.5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2048.0 * 4 * iters * (double(blocks) * threads / 64);
    std::printf("mfma_f64_16x16x4f64: %d CUs, %.3f ms, %.1f TFLOP/s\n", cus, ms, flops / (ms * 1e-3) / 1e12);
  }
  hipFree(out);
  return 0;
}
