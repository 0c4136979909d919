// Kernel bodies of liboptimalcontrolmps_amd (device code, gfx950).  The
// __global__ entry points in ocmps.hip only declare the dynamic LDS and call
// these; one workgroup = one MPS chain (engine_device.hpp).
#pragma once

#include "engine_device.hpp"

namespace ocg {

// --------------------------------------------------------------------------
// device statistics: [kind][0] = alg bytes, [1] = alg flops, [2] = steps
struct StatAcc {
  double bytes = 0, flops = 0, steps = 0;
};

template <int T>
__device__ inline double site_nelem(const Chain<T>& c, int k) {
  double s = 0;
  for (int q = 0; q < c.P.Q1; ++q)
    for (int n = 0; n < c.P.p; ++n)
      if (q + n <= c.P.Q) s += double(c.d(k - 1, q)) * c.d(k, q + n);
  return s;
}
template <int T>
__device__ inline double mps_nelem(const Chain<T>& c) {
  double s = 0;
  for (int k = 1; k <= c.P.L; ++k) s += site_nelem(c, k);
  return s;
}

// algorithmic traffic of one Trotter sweep, evaluated on the post-step dims:
// every two-site update reads both site tensors + the Δ-gate table and writes
// both back; flops = 8 x complex MACs of Θ, gate, Gram
// and factor formation at those dims.
template <int T>
__device__ inline void sweep_model(const Chain<T>& c, double& bytes, double& flops) {
  const int p = c.P.p;
  double b = 0, f = 0;
  for (int g = 0; g < c.P.ngates; ++g) {
    int i1 = c.P.gate_i1[g];
    double s1 = site_nelem(c, i1), s2 = site_nelem(c, i1 + 1);
    b += 16.0 * (2.0 * (s1 + s2) + c.P.gtotal);
    for (int q = 0; q < c.P.Q1; ++q) {
      double R = 0, C = 0;
      for (int n = 0; n < p; ++n) { R += c.d(i1 - 1, q - n); if (q + n <= c.P.Q) C += c.d(i1 + 1, q + n); }
      double m = c.d(i1, q);
      double n = R < C ? R : C;
      f += 8.0 * (R * C * m + R * C * p + n * n * (R > C ? R : C) + 2.0 * R * C * m);
    }
  }
  bytes = b;
  flops = f;
}

template <int T>
__device__ inline void flush_stats(const Chain<T>& c, double* stats, double bytes, double flops, double steps) {
  if (threadIdx.x == 0 && stats) {
    atomicAdd(stats + 0, bytes);
    atomicAdd(stats + 1, flops);
    atomicAdd(stats + 2, steps);
  }
}

struct Pool {
  int* dims;       // [nslots][nsq]
  double2* data;   // [nslots][cap]
};

#define SLOT_D(pool, P, s) ((pool).dims + (size_t)(s) * (P).nsq)
#define SLOT_X(pool, P, s) ((pool).data + (size_t)(s) * (P).cap)

// --------------------------------------------------------------------------
template <int NT>
__device__ void body_trajectory(char* smem, OcgParams P, const double2* gf, const double2* gb, const int* md,
                                                   Pool pool, int slot_init, int slot_target, int psi_base,
                                                   int xi_base, const double* u, int N, int which, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int chain = (which == 3) ? blockIdx.x : (which == 1 ? 0 : 1);
  double bytes = 0, flops = 0;
  if (chain == 0) {
    c.load(SLOT_D(pool, P, slot_init), SLOT_X(pool, P, slot_init));
    c.store(SLOT_D(pool, P, psi_base), SLOT_X(pool, P, psi_base));
    for (int i = 0; i + 1 < N; ++i) {
      c.step(u[i], u[i + 1], 1);
      c.store(SLOT_D(pool, P, psi_base + i + 1), SLOT_X(pool, P, psi_base + i + 1));
      if (threadIdx.x == 0) { double b, f; sweep_model(c, b, f); bytes += b; flops += f; }
    }
  } else {
    c.load(SLOT_D(pool, P, slot_target), SLOT_X(pool, P, slot_target));
    c.store(SLOT_D(pool, P, xi_base + N - 1), SLOT_X(pool, P, xi_base + N - 1));
    for (int i = N - 1; i > 0; --i) {
      c.step(u[i], u[i - 1], 0);
      c.store(SLOT_D(pool, P, xi_base + i - 1), SLOT_X(pool, P, xi_base + i - 1));
      if (threadIdx.x == 0) { double b, f; sweep_model(c, b, f); bytes += b; flops += f; }
    }
  }
  flush_stats(c, stats, bytes, flops, double(N - 1));
}

// out[i] = <x_i|y_i> or <x_i|dH|y_i>
template <int NT>
__device__ void body_overlaps(char* smem, OcgParams P, const double2* gf, const double2* gb, const int* md,
                                                 Pool pool, const int* xs, const int* ys, int npairs, int with_dH,
                                                 double2* out, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= npairs) return;
  c.load(SLOT_D(pool, P, ys[i]), SLOT_X(pool, P, ys[i]));
  double2 r = c.overlap(SLOT_D(pool, P, xs[i]), SLOT_X(pool, P, xs[i]), with_dH);
  if (threadIdx.x == 0) out[i] = r;
  if (threadIdx.x == 0) {
    double b = 32.0 * mps_nelem(c);
    flush_stats(c, stats, b, 8.0 * b / 16.0 * 4.0, 0.0);
  }
}

template <int NT>
__device__ void body_apply_dH(char* smem, OcgParams P, const double2* gf, const double2* gb, const int* md,
                                                 Pool pool, const int* in, const int* outs, int n, double* norms,
                                                 double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= n) return;
  c.load(SLOT_D(pool, P, in[i]), SLOT_X(pool, P, in[i]));
  double b0 = (threadIdx.x == 0) ? 16.0 * mps_nelem(c) : 0.0;
  c.apply_dH();
  double n2 = c.site_norm2(1);
  c.store(SLOT_D(pool, P, outs[i]), SLOT_X(pool, P, outs[i]));
  if (threadIdx.x == 0) {
    if (norms) norms[i] = sqrt(n2);
    double b = b0 + 16.0 * mps_nelem(c);
    flush_stats(c, stats, b, 8.0 * b, 0.0);
  }
}

// calcHessianRow (src/OptimalControl.cpp:251-279)
template <int NT>
__device__ void body_hessian_rows(char* smem, OcgParams P, const double2* gf, const double2* gb,
                                                     const int* md, Pool pool, int psi_base, int xih_base,
                                                     const int* rows, int nrows, const double* u, int N,
                                                     const double2* divT, double2 F, double* H, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int r = blockIdx.x;
  if (r >= nrows) return;
  const int i = rows[r];
  const double dt2 = P.dt * P.dt;
  c.load(SLOT_D(pool, P, psi_base + i), SLOT_X(pool, P, psi_base + i));
  c.apply_dH();  // psiH = exactApplyMPO(propDeriv, psi_t[i], args)
  const double normiH = sqrt(c.site_norm2(1));
  double bytes = 0, flops = 0;
  {
    double2 ov = c.overlap(SLOT_D(pool, P, xih_base + i), SLOT_X(pool, P, xih_base + i), 0);
    if (threadIdx.x == 0) {
      double2 dv = divT[i];
      double v1 = F.x * ov.x - F.y * ov.y;          // Re(F <xiH_i|psiH>)
      double v2 = -(dv.x * dv.x + dv.y * dv.y);     // -|divT_i|^2
      H[(size_t)i * N + i] = dt2 * (v1 + v2);
    }
  }
  for (int j = i + 1; j + 1 < N; ++j) {
    c.step(u[j - 1], u[j], 1);
    double2 ov = c.overlap(SLOT_D(pool, P, xih_base + j), SLOT_X(pool, P, xih_base + j), 0);
    if (threadIdx.x == 0) {
      double2 di = divT[i], dj = divT[j];
      double v1 = (F.x * ov.x - F.y * ov.y) * normiH;   // Re(F <xiH_j|psiH> n_i)
      double v2 = -(di.x * dj.x + di.y * dj.y);          // -Re(divT_i conj(divT_j))
      double res = dt2 * (v1 + v2);
      H[(size_t)i * N + j] = res;
      H[(size_t)j * N + i] = res;
      double b, f;
      sweep_model(c, b, f);
      bytes += b + 32.0 * mps_nelem(c);
      flops += f;
    }
  }
  flush_stats(c, stats, bytes, flops, double(N - 2 - i > 0 ? N - 2 - i : 0));
}

// nsteps steps per state; u holds nsteps+1 controls per state (u_stride apart)
template <int NT>
__device__ void body_steps(char* smem, OcgParams P, const double2* gf, const double2* gb, const int* md,
                                              Pool pool, const int* slots, int n, const double* u, int u_stride,
                                              int nsteps, int forward, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= n) return;
  c.load(SLOT_D(pool, P, slots[i]), SLOT_X(pool, P, slots[i]));
  double bytes = 0, flops = 0;
  const double* ui = u + (size_t)i * u_stride;
  for (int s = 0; s < nsteps; ++s) {
    c.step(ui[s], ui[s + 1], forward);
    if (threadIdx.x == 0) { double b, f; sweep_model(c, b, f); bytes += b; flops += f; }
  }
  c.store(SLOT_D(pool, P, slots[i]), SLOT_X(pool, P, slots[i]));
  flush_stats(c, stats, bytes, flops, double(nsteps));
}


}  // namespace ocg
