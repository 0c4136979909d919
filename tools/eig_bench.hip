// Stand-alone benchmark + residual check of the HBM engine's Hermitian
// eigensolver kernels on random Gram blocks rho = M M^H (decaying spectrum).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../optimalcontrolmps_amd/csrc tools/eig_bench.hip
// usage: eig_bench n batch k [regmin] [thr_rel] [rank]   (EIG_OLD=1: orders above RNMAX on the eager L2 kernel)
#include <hip/hip_runtime.h>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <algorithm>
#include <vector>
#include "hbm_device.hpp"
#define COOP_GRID(G, B) (8 * (G) * (((B) + 7) / 8))
using namespace hbm;
using cd = std::complex<double>;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 128, B = argc > 2 ? atoi(argv[2]) : 1;
  const int kk = std::min(argc > 3 ? atoi(argv[3]) : 32, argc > 1 ? atoi(argv[1]) : 128);
  const int regmin = argc > 4 ? atoi(argv[4]) : kRegMin;
  const double thr_rel = argc > 5 ? atof(argv[5]) : 0.0;
  const int rank = argc > 6 ? atoi(argv[6]) : n;  // rank of M (rank-deficient Gram blocks: reduced columns, tau = 0)
  const int reps = 5;
  std::mt19937_64 g(7);
  std::normal_distribution<double> N01;
  std::vector<std::vector<cd>> As(B);
  for (int b = 0; b < B; ++b) {
    if (b > 0 && getenv("EIG_SAME")) { As[b] = As[0]; continue; }  // every problem the same block
    std::vector<cd> M(size_t(n) * n), A(size_t(n) * n);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) M[i * n + j] = j < rank ? cd(N01(g), N01(g)) * std::exp(-0.08 * j) : cd(0, 0);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        cd s = 0;
        for (int l = 0; l < n; ++l) s += M[i * n + l] * std::conj(M[j * n + l]);
        A[i * n + j] = s;
      }
    As[b] = A;
  }
  // device problems
  std::vector<EProb> P(B);
  z *dA, *dU, *dph;
  double *dd, *de, *dtau, *dw, *dZ, *dDv;
  int* dkept;
  const size_t nn = size_t(n) * n;
  CK(hipMalloc(&dA, sizeof(z) * nn * B));
  CK(hipMalloc(&dU, sizeof(z) * nn * B));
  CK(hipMalloc(&dph, sizeof(z) * n * B));
  CK(hipMalloc(&dd, 8 * n * B)); CK(hipMalloc(&de, 8 * n * B)); CK(hipMalloc(&dtau, 8 * (n + 64) * B));
  CK(hipMalloc(&dw, 8 * n * B)); CK(hipMalloc(&dZ, 8 * nn * B)); CK(hipMalloc(&dDv, 8 * nn * B));
  CK(hipMalloc(&dkept, 4 * B));
  std::vector<int> kept(B, kk);
  CK(hipMemcpy(dkept, kept.data(), 4 * B, hipMemcpyHostToDevice));
  for (int b = 0; b < B; ++b) {
    EProb& p = P[b];
    p.A = dA + nn * b; p.U = dU + nn * b; p.ph = dph + n * b;
    p.d = dd + n * b; p.e = de + n * b; p.tau = dtau + (n + 64) * b; p.w = dw + n * b;
    p.Z = dZ + nn * b; p.Dv = dDv + nn * b; p.n = n; p.q = 0; p.kept = dkept + b; p.thr_rel = thr_rel;
    p.ks = getenv("EIG_KS") ? atoi(getenv("EIG_KS")) : 1;  // shifts per multisection thread
  }
  EProb* dP;
  CK(hipMalloc(&dP, sizeof(EProb) * B));
  CK(hipMemcpy(dP, P.data(), sizeof(EProb) * B, hipMemcpyHostToDevice));
  std::vector<int> idx(B);
  for (int b = 0; b < B; ++b) idx[b] = b;
  int* didx;
  CK(hipMalloc(&didx, 4 * B));
  CK(hipMemcpy(didx, idx.data(), 4 * B, hipMemcpyHostToDevice));
  std::vector<int2> bt;
  for (int b = 0; b < B; ++b)
    if (n > 64 && n <= kBtRows)
      for (int cb = 0; 16 * cb < n; ++cb) bt.push_back(make_int2(b, cb));
  int2* dbt = nullptr;
  if (!bt.empty()) {
    CK(hipMalloc(&dbt, sizeof(int2) * bt.size()));
    CK(hipMemcpy(dbt, bt.data(), sizeof(int2) * bt.size(), hipMemcpyHostToDevice));
  }
  // EIG_COOP=G: the multi-CU kernel with G workgroups per block (EIG_TMO: its
  // wait bound in s_memrealtime ticks; 0 forces every group onto the fallback)
  const int coopG = getenv("EIG_COOP") ? atoi(getenv("EIG_COOP")) : 0;
  const long long coop_tmo = getenv("EIG_TMO") ? atoll(getenv("EIG_TMO")) : 5000000LL;
  int* dctl = nullptr;
  CK(hipMalloc(&dctl, sizeof(int) * kCoopCtl * B));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
  double tv = 0, tvec = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int b = 0; b < B; ++b) CK(hipMemcpy(dA + nn * b, As[b].data(), sizeof(z) * nn, hipMemcpyHostToDevice));
    CK(hipEventRecord(e0));
    if (coopG > 0) {
      CK(hipMemsetAsync(dctl, 0, sizeof(int) * kCoopCtl * B, 0));
      hipLaunchKernelGGL(k_heev_vals_coop, dim3(COOP_GRID(coopG, B)), dim3(CPT), 0, 0, dP, didx, B, coopG, dctl,
                         coop_tmo);
      hipLaunchKernelGGL(k_heev_vals_coop_fix, dim3(B), dim3(VBG), 0, 0, dP, didx, dctl, nullptr);
    } else if (n > RNMAX && n <= kBigMax && !getenv("EIG_OLD")) {
      hipLaunchKernelGGL(k_heev_vals_big, dim3(B), dim3(VBG), 0, 0, dP, didx);
    } else {
      const int lds = (n >= regmin && n <= RNMAX) ? reg_lds_bytes(reg_grid(n)) : 64 * n + (n <= kLdsOrder ? 16 * n * n : 0) + 64;
      hipLaunchKernelGGL(k_heev_vals_any, dim3(B), dim3(RNT), lds, 0, dP, didx, regmin);
    }
    CK(hipEventRecord(e1));
    hipLaunchKernelGGL(k_heev_vecs_reg, dim3(B), dim3(VNT), 0, 0, dP, B);
    if (dbt) hipLaunchKernelGGL(k_heev_bt, dim3(int(bt.size())), dim3(BNT), 0, 0, dP, dbt);
    CK(hipEventRecord(e2));
    CK(hipEventSynchronize(e2));
    float a, b2;
    CK(hipEventElapsedTime(&a, e0, e1)); CK(hipEventElapsedTime(&b2, e1, e2));
    if (rep > 0) { tv += a; tvec += b2; }
  }
  // check problem 0: eigenvalues vs residuals
  std::vector<double> w(n);
  std::vector<z> U(size_t(n) * kk);
  CK(hipMemcpy(w.data(), dw, 8 * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(U.data(), dU, sizeof(z) * n * kk, hipMemcpyDeviceToHost));
  const auto& A = As[0];
  double res = 0, orth = 0, tr = 0, sw = 0;
  for (int i = 0; i < n; ++i) { tr += A[i * n + i].real(); sw += w[i]; }
  for (int c = 0; c < kk; ++c) {
    for (int i = 0; i < n; ++i) {
      cd s = 0;
      for (int l = 0; l < n; ++l) s += A[i * n + l] * cd(U[l * kk + c].x, U[l * kk + c].y);
      res = std::max(res, std::abs(s - w[c] * cd(U[i * kk + c].x, U[i * kk + c].y)));
    }
    for (int c2 = 0; c2 < kk; ++c2) {
      cd s = 0;
      for (int l = 0; l < n; ++l) s += std::conj(cd(U[l * kk + c].x, U[l * kk + c].y)) * cd(U[l * kk + c2].x, U[l * kk + c2].y);
      orth = std::max(orth, std::abs(s - (c == c2 ? 1.0 : 0.0)));
    }
  }
#ifdef HBM_STAMP
  {
    // the vals kernel alone once more (the vecs kernel reuses P.Z), then its stamps
    CK(hipMemcpy(dA, As[0].data(), sizeof(z) * nn, hipMemcpyHostToDevice));
    {
      const int lds = (n >= regmin && n <= RNMAX) ? reg_lds_bytes(reg_grid(n)) : 64 * n + (n <= kLdsOrder ? 16 * n * n : 0) + 64;
      if (n <= RNMAX) hipLaunchKernelGGL(k_heev_vals_any, dim3(1), dim3(RNT), lds, 0, dP, didx, regmin);
      CK(hipDeviceSynchronize());
    }
    std::vector<double> st(8);
    CK(hipMemcpy(st.data(), dZ, 64, hipMemcpyDeviceToHost));
    const char* nm[8] = {"colprep", "barA", "reflector", "barA'", "matvec", "barB/C", "combine+K", "update"};
    double tot = 0;
    for (double v : st) tot += v;
    printf("stamps (wave 0, s_memtime ticks, last rep):");
    for (int q = 0; q < 8; ++q) printf(" %s %.0f (%.0f%%)", nm[q], st[q], 100 * st[q] / tot);
    printf(" | per column %.0f\n", tot / (n - 1));
    // vecs kernel stamps (written after the vals ones were read: rerun vecs once)
    hipLaunchKernelGGL(k_heev_vecs_reg, dim3(B), dim3(VNT), 0, 0, dP, B);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), dZ, 64, hipMemcpyDeviceToHost));
    const char* nv[5] = {"invit", "orth", "U init", "BT loads", "BT apply"};
    printf("vecs stamps:");
    for (int q = 0; q < 5; ++q) printf(" %s %.0f", nv[q], st[q]);
    printf("\n");
  }
#endif
  if (coopG > 0) {
    std::vector<int> ctl(kCoopCtl * B);
    CK(hipMemcpy(ctl.data(), dctl, sizeof(int) * ctl.size(), hipMemcpyDeviceToHost));
    int ab = 0;
    for (int b = 0; b < B; ++b) ab += ctl[kCoopCtl * b + 32] != 0;
    printf("coop G=%d: %d of %d groups fell back | ", coopG, ab, B);
  }
  // eigenvalues of every problem vs problem 0's (the same matrix in every slot)
  {
    std::vector<double> wa(size_t(n) * B);
    CK(hipMemcpy(wa.data(), dw, 8 * n * B, hipMemcpyDeviceToHost));
    double dmax = 0;
    for (int b = 1; b < B; ++b)
      for (int i = 0; i < n; ++i) dmax = std::max(dmax, std::abs(wa[size_t(b) * n + i] - wa[i]));
    if (getenv("EIG_DUMPW")) {
      FILE* f = fopen(getenv("EIG_DUMPW"), "wb");
      fwrite(wa.data(), 8, n, f);
      fclose(f);
    }
    printf("max|w_b - w_0| %.2e | ", dmax);
  }
  printf("n=%d B=%d k=%d: vals %.1f us  vecs %.1f us per launch | max|A u - w u|/w0 = %.2e  orth %.2e  "
         "trace err %.2e  w0 %.3e w[k-1] %.3e\n", n, B, kk, 1e3 * tv / (reps - 1), 1e3 * tvec / (reps - 1),
         res / w[0], orth, std::abs(tr - sw) / tr, w[0], w[kk - 1]);
  return 0;
}
