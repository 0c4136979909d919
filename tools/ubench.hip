// Diagnostic micro-benchmarks (not part of the product): shader-clock cycles
// per dependent operation on gfx950, to calibrate the chain engine's latency
// model (LDS round trip, v_readlane search, FP64 div/sqrt, barriers).
// Build/run: hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench tools/ubench.hip && /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>

#define REPS 2048

__global__ void __launch_bounds__(256) k_lds(unsigned long long* out, int stride) {
  __shared__ int buf[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[i] = (i + stride) & 4095;
  __syncthreads();
  int idx = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; ++r) idx = buf[idx];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = idx; }
}

__global__ void __launch_bounds__(256) k_lds_d(unsigned long long* out) {
  __shared__ double buf[2048];
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) buf[i] = (double)((i + 1) & 2047);
  __syncthreads();
  int idx = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; ++r) idx = (int)buf[idx];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = idx; }
}

__global__ void __launch_bounds__(256) k_div(unsigned long long* out, double s) {
  double x = s + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; ++r) x = 1.0 / (x + 1.0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = (unsigned long long)(x * 1e9); }
}

__global__ void __launch_bounds__(256) k_sqrt(unsigned long long* out, double s) {
  double x = s + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; ++r) x = sqrt(x + 1.0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = (unsigned long long)(x * 1e9); }
}

__global__ void __launch_bounds__(256) k_hypot(unsigned long long* out, double s) {
  double x = s + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; ++r) x = hypot(x, 0.5) * 0.5;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = (unsigned long long)(x * 1e9); }
}

__global__ void __launch_bounds__(256) k_fma(unsigned long long* out, double s) {
  double x = s + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; ++r) x = fma(x, 0.999, 1e-3);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = (unsigned long long)(x * 1e9); }
}

__global__ void __launch_bounds__(256) k_sync(unsigned long long* out) {
  __shared__ int buf[256];
  buf[threadIdx.x] = threadIdx.x;
  int acc = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; ++r) {
    __syncthreads();
    acc += buf[(threadIdx.x + r) & (blockDim.x - 1)];
    __syncthreads();
    buf[threadIdx.x] = acc;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = acc; }
}

__global__ void __launch_bounds__(256) k_readlane(unsigned long long* out, int nq) {
  int reg = threadIdx.x * 7;
  int e = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; ++r) {
    int q = -1;
    for (int b = 0; b < nq; ++b) q += (__builtin_amdgcn_readlane(reg, b) <= e) ? 1 : 0;
    e = (e + q) & 255;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = e; }
}

__global__ void __launch_bounds__(256) k_gload(unsigned long long* out, const int* g) {
  int idx = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < 256; ++r) idx = g[idx];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = idx; }
}

int main() {
  unsigned long long* d;
  unsigned long long h[2];
  int* g;
  hipMalloc(&d, 16);
  hipMalloc(&g, 4096 * 4);
  int hg[4096];
  for (int i = 0; i < 4096; ++i) hg[i] = (i + 67) & 4095;
  hipMemcpy(g, hg, sizeof(hg), hipMemcpyHostToDevice);
  auto rep = [&](const char* name, double n) {
    hipDeviceSynchronize();
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("%-28s %8.1f cycles/op\n", name, double(h[0]) / n);
  };
  for (int nt : {64, 256}) {
    printf("-- block %d threads\n", nt);
    for (int w = 0; w < 2; ++w) {  // second pass = warm
      k_lds<<<1, nt>>>(d, 1); if (w) rep("lds int dependent load", REPS);
      k_lds<<<1, nt>>>(d, 64); if (w) rep("lds int dep load stride64", REPS);
      k_lds_d<<<1, nt>>>(d); if (w) rep("lds f64 dep load+cvt", REPS);
      k_div<<<1, nt>>>(d, 1.0); if (w) rep("f64 div (dep)", REPS);
      k_sqrt<<<1, nt>>>(d, 1.0); if (w) rep("f64 sqrt (dep)", REPS);
      k_hypot<<<1, nt>>>(d, 1.0); if (w) rep("f64 hypot (dep)", REPS);
      k_fma<<<1, nt>>>(d, 1.0); if (w) rep("f64 fma (dep)", REPS);
      k_sync<<<1, nt>>>(d); if (w) rep("2x syncthreads + lds rw", REPS);
      k_readlane<<<1, nt>>>(d, 6); if (w) rep("readlane search Q1=6", REPS);
      k_readlane<<<1, nt>>>(d, 21); if (w) rep("readlane search Q1=21", REPS);
      k_gload<<<1, nt>>>(d, g); if (w) rep("global dep load (L2)", 256);
    }
  }
  return 0;
}
