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

#ifdef OCG_PROFILE
__device__ double g_ocg_prof[32];
#endif

template <int T>
__device__ inline void flush_stats(const Chain<T>& c, double* stats, double bytes, double flops, double steps) {
#ifdef OCG_PROFILE
  const_cast<Chain<T>&>(c).pf(12);
  if (threadIdx.x == 0)
    for (int i = 0; i < 32; ++i) atomicAdd(&g_ocg_prof[i], c.PROF[i]);
#endif
  if (threadIdx.x == 0 && stats) {
    atomicAdd(stats + 0, bytes);
    atomicAdd(stats + 1, flops);
    atomicAdd(stats + 2, steps);
  }
}

struct Pool {
  int* dims;       // [nslots][nsq]
  zc* data;   // [nslots][cap]
};

#define SLOT_D(pool, P, s) ((pool).dims + (size_t)(s) * (P).nsq)
#define SLOT_X(pool, P, s) ((pool).data + (size_t)(s) * (P).cap)

// --------------------------------------------------------------------------
template <int NT>
__device__ void body_trajectory(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                   Pool pool, int slot_init, int slot_target, int psi_base,
                                                   int xi_base, const double* u, int N, int which, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int chain = (which == 3) ? blockIdx.x : (which == 1 ? 0 : 1);
  // chain 0: psi_t forward from psi_init (calcPsi, src/OptimalControl.cpp:375-390)
  // chain 1: xi_t backward from psi_target (calcXi, :392-407)
  const int fwd = (chain == 0) ? 1 : 0;
  const int base = fwd ? psi_base : xi_base;
  const int src = fwd ? slot_init : slot_target;
  double bytes = 0, flops = 0;
  c.load(SLOT_D(pool, P, src), SLOT_X(pool, P, src));
  int t = fwd ? 0 : N - 1;
  c.store(SLOT_D(pool, P, base + t), SLOT_X(pool, P, base + t));
  for (int s = 0; s + 1 < N; ++s) {
    const int tn = fwd ? t + 1 : t - 1;
    c.step(u[t], u[tn], fwd);
    c.store(SLOT_D(pool, P, base + tn), SLOT_X(pool, P, base + tn));
    if (threadIdx.x == 0) { double b, f; sweep_model(c, b, f); bytes += b; flops += f; }
    t = tn;
  }
  flush_stats(c, stats, bytes, flops, double(N - 1));
}

// out[i] = <x_i|y_i> or <x_i|dH|y_i>
template <int NT>
__device__ void body_overlaps(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                 Pool pool, const int* xs, const int* ys, int npairs, int with_dH,
                                                 zc* out, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= npairs) return;
  c.load(SLOT_D(pool, P, ys[i]), SLOT_X(pool, P, ys[i]));
  zc r = c.overlap(SLOT_D(pool, P, xs[i]), SLOT_X(pool, P, xs[i]), with_dH);
  if (threadIdx.x == 0) out[i] = r;
  if (threadIdx.x == 0) {
    double b = 32.0 * mps_nelem(c);
    flush_stats(c, stats, b, 8.0 * b / 16.0 * 4.0, 0.0);
  }
}

template <int NT>
__device__ void body_apply_dH(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
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

// calcHessianRow (src/OptimalControl.cpp:251-279).  psiH_i =
// exactApplyMPO(propDeriv, psi_t[i]) and its norm normiH come from a preceding
// batched body_apply_dH launch (slots psih_base + i, norms[i]).
template <int NT>
__device__ void body_hessian_rows(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md, Pool pool,
                                  int psih_base, int xih_base, const int* rows, int nrows, const double* norms,
                                  const double* u, int N, const zc* divT, zc F, double* H, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int r = blockIdx.x;
  if (r >= nrows) return;
  const int i = rows[r];
  const double dt2 = P.dt * P.dt;
  const double normiH = norms[i];
  c.load(SLOT_D(pool, P, psih_base + i), SLOT_X(pool, P, psih_base + i));
  double bytes = 0, flops = 0;
  // j = i: diagonal entry (:259-264); j > i: step psiH once, then overlap (:266-278)
  for (int j = i; j + 1 < N; ++j) {
    if (j > i) c.step(u[j - 1], u[j], 1);
    zc ov = c.overlap(SLOT_D(pool, P, xih_base + j), SLOT_X(pool, P, xih_base + j), 0);
    if (threadIdx.x == 0) {
      zc di = divT[i], dj = divT[j];
      double v1 = (F.x * ov.x - F.y * ov.y) * (j > i ? normiH : 1.0);  // Re(F <xiH_j|psiH> n_i)
      double v2 = -(di.x * dj.x + di.y * dj.y);                        // -Re(divT_i conj(divT_j))
      double res = dt2 * (v1 + v2);
      H[(size_t)i * N + j] = res;
      if (j > i) H[(size_t)j * N + i] = res;
      if (j > i) {
        double b, f;
        sweep_model(c, b, f);
        bytes += b;
        flops += f;
      }
      bytes += 32.0 * mps_nelem(c);
    }
  }
  flush_stats(c, stats, bytes, flops, double(N - 2 - i > 0 ? N - 2 - i : 0));
}

// nsteps steps per state; u holds nsteps+1 controls per state (u_stride apart)
template <int NT>
__device__ void body_steps(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
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
