// Diagnostic (not part of the product): cycles per engine phase of one chain
// on a realistic entangled state, timed in tight loops inside one workgroup.
// State: Mott product |1..1> (L=5, p=5, Q=5) evolved 60 steps at U 2 -> 6.
// Build/run: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I optimalcontrolmps_amd/csrc \
//              -o /tmp/ubench_engine tools/ubench_engine.hip && /tmp/ubench_engine
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#ifndef OCG_NT
#define OCG_NT 64
#endif
#include "kernels.hpp"
#include "params.hpp"

using ocg::Chain;
using ocg::Pool;
using ocg::zc;
static constexpr int NT = OCG_NT;

__global__ __launch_bounds__(NT) void k_prep(OcgParams P, const zc* gf, const zc* gb, const int* md, Pool pool,
                                             const double* u, int nsteps) {
  extern __shared__ __align__(16) char smem[];
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  c.load(pool.dims, pool.data);
  for (int s = 0; s < nsteps; ++s) c.step(u[s], u[s + 1], 1);
  c.store(pool.dims, pool.data);
}

// out[k] = cycles per call of phase k
__global__ __launch_bounds__(NT) void k_phases(OcgParams P, const zc* gf, const zc* gb, const int* md, Pool pool,
                                               int reps, unsigned long long* out, int which) {
  extern __shared__ __align__(16) char smem[];
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  c.load(pool.dims, pool.data);
  unsigned long long t0, t1;
  auto stamp = [&]() {
    __syncthreads();
    return (unsigned long long)__builtin_amdgcn_s_memtime();
  };
  const int i1 = 2;
  c.store(pool.dims + P.nsq, pool.data + P.cap);
  c.build_theta(i1);
  if (which >= 0) {  // single-phase mode (one phase per dispatch, for PMC counters)
    t0 = stamp();
    for (int r = 0; r < reps; ++r) {
      if (which == 0) c.build_theta(i1);
      else if (which == 1) c.apply_gate(i1, 1, 0, 0);
      else if (which == 2) c.decompose(ocg::kFromleft, P.cutoff, P.maxm, true, c.MD + i1 * P.Q1);
      else if (which == 5) { c.gauge_right(3, OCG_GAUGE_CUTOFF, 1 << 30); c.gauge_left(4, OCG_GAUGE_CUTOFF, 1 << 30); }
      else if (which == 6) c.overlap(pool.dims + P.nsq, pool.data + P.cap, 0);
      else if (which == 7) { c.step(4.0, 5.0, 1); c.step(5.0, 4.0, 0); }
    }
    t1 = stamp();
    if (threadIdx.x == 0) out[which] = (t1 - t0) / reps;
    return;
  }
  // 0: build_theta
  t0 = stamp();
  for (int r = 0; r < reps; ++r) c.build_theta(i1);
  t1 = stamp();
  if (threadIdx.x == 0) out[0] = (t1 - t0) / reps;
  // 1: apply_gate (TH/X swap each call)
  t0 = stamp();
  for (int r = 0; r < reps; ++r) c.apply_gate(i1, 1, 0, 0);
  t1 = stamp();
  if (threadIdx.x == 0) out[1] = (t1 - t0) / reps;
  c.build_theta(i1);
  // 2: decompose Fromleft with truncation (two-site, includes Jacobi)
#ifdef OCG_PROFILE
  if (threadIdx.x == 0)
    for (int k = 0; k < 32; ++k) c.PROF[k] = 0;
  c.pf(12);
#endif
  t0 = stamp();
  for (int r = 0; r < reps; ++r) c.decompose(ocg::kFromleft, P.cutoff, P.maxm, true, c.MD + i1 * P.Q1);
  t1 = stamp();
  if (threadIdx.x == 0) out[2] = (t1 - t0) / reps;
#ifdef OCG_PROFILE
  // per-phase breakdown of the Fromleft decompositions above (PROF slots)
  if (threadIdx.x == 0)
    for (int k = 0; k < 32; ++k) out[16 + k] = (unsigned long long)(c.PROF[k] * 1000.0 / reps);
#endif
  // 3: decompose Fromright
  t0 = stamp();
  for (int r = 0; r < reps; ++r) c.decompose(ocg::kFromright, P.cutoff, P.maxm, true, c.MD + i1 * P.Q1);
  t1 = stamp();
  if (threadIdx.x == 0) out[3] = (t1 - t0) / reps;
  // 4: site_to_theta (left grouping of site 3)
  t0 = stamp();
  for (int r = 0; r < reps; ++r) c.site_to_theta(3, true);
  t1 = stamp();
  if (threadIdx.x == 0) out[4] = (t1 - t0) / reps;
  // 5: gauge move pair 3 -> 4 -> 3 (two gauge moves)
  t0 = stamp();
  for (int r = 0; r < reps; ++r) {
    c.gauge_right(3, OCG_GAUGE_CUTOFF, 1 << 30);
    c.gauge_left(4, OCG_GAUGE_CUTOFF, 1 << 30);
  }
  t1 = stamp();
  if (threadIdx.x == 0) out[5] = (t1 - t0) / (2 * reps);
  // 6: overlap <psi|psi> with the stored state (global X)
  c.store(pool.dims + P.nsq, pool.data + P.cap);
  t0 = stamp();
  zc acc = ocg::c2(0, 0);
  for (int r = 0; r < reps; ++r) acc = ocg::cadd(acc, c.overlap(pool.dims + P.nsq, pool.data + P.cap, 0));
  t1 = stamp();
  if (threadIdx.x == 0) out[6] = (t1 - t0) / reps;
  // 7: full Trotter step (forward then backward to stay near the state)
#ifdef OCG_PROFILE
  if (threadIdx.x == 0)
    for (int k = 0; k < 32; ++k) c.PROF[k] = 0;
  c.pf(12);
#endif
  t0 = stamp();
  for (int r = 0; r < reps; ++r) {
    c.step(4.0, 5.0, 1);
    c.step(5.0, 4.0, 0);
  }
  t1 = stamp();
  if (threadIdx.x == 0) out[7] = (t1 - t0) / (2 * reps);
#ifdef OCG_PROFILE
  if (threadIdx.x == 0)
    for (int k = 0; k < 32; ++k) out[64 + k] = (unsigned long long)(c.PROF[k] * 1000.0 / (2 * reps));
#endif
  // 8: apply_dH (on a copy: reload the state each rep)
  t0 = stamp();
  for (int r = 0; r < reps; ++r) {
    c.load(pool.dims + P.nsq, pool.data + P.cap);
    c.apply_dH();
  }
  t1 = stamp();
  if (threadIdx.x == 0) out[8] = (t1 - t0) / reps;
  // 9: load alone
  t0 = stamp();
  for (int r = 0; r < reps; ++r) c.load(pool.dims + P.nsq, pool.data + P.cap);
  t1 = stamp();
  if (threadIdx.x == 0) {
    out[9] = (t1 - t0) / reps;
    out[10] = (unsigned long long)(acc.x * 1e6);
  }
}

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));           \
      return 1;                                                      \
    }                                                                \
  } while (0)

int main() {
  const int L = 5, p = 5, Q = 5;
  OcgParams P;
  std::vector<int> md;
  std::string e = ocg_host::build_params(P, md, L, p, Q, 0.01, 1e-8, 80);
  if (!e.empty()) { printf("%s\n", e.c_str()); return 1; }
  std::vector<double> gf, gb;
  ocg_host::gate_tables(P, 1.0, gf, gb);
  P.lds_bytes = ocg::lds_layout(P, NT).bytes;
  printf("NT %d  LDS %d B  cap %d thcap %d\n", NT, P.lds_bytes, P.cap, P.thcap);
  // Mott product state: bond b holds q = b; site k block (q=k-1, n=1) = 1
  std::vector<int> dims(P.nsq, 0);
  for (int b = 0; b <= L; ++b) dims[b * P.Q1 + b] = 1;
  std::vector<zc> data(2 * P.cap, ocg::c2(0, 0));
  for (int k = 1; k <= L; ++k) data[P.site_base[k]] = ocg::c2(1, 0);
  zc *dgf, *dgb;
  int *dmd, *dd;
  zc* dx;
  double* du;
  unsigned long long* dout;
  CK(hipMalloc(&dgf, gf.size() * 8));
  CK(hipMalloc(&dgb, gb.size() * 8));
  CK(hipMalloc(&dmd, md.size() * 4));
  CK(hipMalloc(&dd, 2 * P.nsq * 4));
  CK(hipMalloc(&dx, 2 * P.cap * sizeof(zc)));
  CK(hipMalloc(&du, 128 * 8));
  CK(hipMalloc(&dout, 128 * 8));
  CK(hipMemcpy(dgf, gf.data(), gf.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dgb, gb.data(), gb.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dmd, md.data(), md.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dd, dims.data(), P.nsq * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, data.data(), P.cap * sizeof(zc), hipMemcpyHostToDevice));
  std::vector<double> u(128);
  for (int i = 0; i < 128; ++i) u[i] = 2.0 + 4.0 * i / 127.0;
  CK(hipMemcpy(du, u.data(), 128 * 8, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)k_prep, hipFuncAttributeMaxDynamicSharedMemorySize, P.lds_bytes));
  CK(hipFuncSetAttribute((const void*)k_phases, hipFuncAttributeMaxDynamicSharedMemorySize, P.lds_bytes));
  Pool pool{dd, dx};
  hipLaunchKernelGGL(k_prep, dim3(1), dim3(NT), P.lds_bytes, 0, P, dgf, dgb, dmd, pool, du, 60);
  CK(hipDeviceSynchronize());
  std::vector<int> hd(P.nsq);
  CK(hipMemcpy(hd.data(), dd, P.nsq * 4, hipMemcpyDeviceToHost));
  printf("bond dims:");
  for (int b = 0; b <= L; ++b) {
    int s = 0;
    for (int q = 0; q < P.Q1; ++q) s += hd[b * P.Q1 + q];
    printf(" %d", s);
  }
  printf("\n");
  const char* names[] = {"build_theta", "apply_gate", "decompose Fromleft", "decompose Fromright", "site_to_theta",
                         "gauge move", "overlap", "full step", "apply_dH", "load"};
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(k_phases, dim3(1), dim3(NT), P.lds_bytes, 0, P, dgf, dgb, dmd, pool, 20, dout, -1);
    CK(hipDeviceSynchronize());
  }
  // one dispatch per phase (PMC attribution): 0 build_theta, 1 gate, 2 decompose, 5 gauge pair, 6 overlap, 7 step pair
  for (int w : {0, 1, 2, 5, 6, 7}) {
    hipLaunchKernelGGL(k_phases, dim3(1), dim3(NT), P.lds_bytes, 0, P, dgf, dgb, dmd, pool, 20, dout + 100, w);
    CK(hipDeviceSynchronize());
  }
  unsigned long long out[128];
  CK(hipMemcpy(out, dout, 128 * 8, hipMemcpyDeviceToHost));
  for (int k = 0; k < 10; ++k) printf("%-22s %10llu cycles\n", names[k], out[k]);
#ifdef OCG_PROFILE
  const char* pn[] = {"build_theta", "apply_gate", "gram", "jacobi(rest)", "rank/trunc", "factors", "scatter",
                      "gauge wb", "overlap", "phase/norm", "load/store", "dH zip", "other", "jacobi A", "jacobi B",
                      "theta tabs", "decomp setup"};
  printf("decompose Fromleft breakdown (cycles per call, incl. ~s_memtime overhead):\n");
  for (int k = 0; k < 17; ++k)
    if (out[16 + k]) printf("   %-14s %10.0f\n", pn[k], out[16 + k] / 1000.0);
  printf("   sweeps/call %.2f  rounds/sweep %.2f\n", out[16 + 20] / 1000.0, out[16 + 22] / 1000.0);
  printf("full step breakdown (cycles per step):\n");
  for (int k = 0; k < 17; ++k)
    if (out[64 + k]) printf("   %-14s %10.0f\n", pn[k], out[64 + k] / 1000.0);
#endif
  return 0;
}
