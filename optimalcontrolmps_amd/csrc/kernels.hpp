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

#ifdef OCG_PROFILE
__device__ double g_ocg_prof[32];
#endif

template <int T>
__device__ inline void flush_stats(Chain<T>& c, double* stats, double bytes, double flops, double steps) {
#ifdef OCG_PROFILE
  c.pf(12);
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
__device__ OCG_INLINE void body_trajectory(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
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
    t = tn;
  }
  c.model_totals(bytes, flops);
  flush_stats(c, stats, bytes, flops, double(N - 1));
}

// out[i] = <x_i|y_i> or <x_i|dH|y_i>
template <int NT>
__device__ OCG_INLINE void body_overlaps(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                 Pool pool, const int* xs, const int* ys, int npairs, int with_dH,
                                                 zc* out, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= npairs) return;
  c.load(SLOT_D(pool, P, ys[i]), SLOT_X(pool, P, ys[i]));
  zc r = c.overlap(SLOT_D(pool, P, xs[i]), SLOT_X(pool, P, xs[i]), with_dH);
  const double b = 32.0 * c.mps_used();
  if (threadIdx.x == 0) out[i] = r;
  flush_stats(c, stats, b, 8.0 * b / 16.0 * 4.0, 0.0);
}

template <int NT>
__device__ OCG_INLINE void body_apply_dH(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                 Pool pool, const int* in, const int* outs, int n, double* norms,
                                                 double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= n) return;
  c.load(SLOT_D(pool, P, in[i]), SLOT_X(pool, P, in[i]));
  const double b0 = 16.0 * c.mps_used();
  c.apply_dH();
  double n2 = c.site_norm2(1);
  c.store(SLOT_D(pool, P, outs[i]), SLOT_X(pool, P, outs[i]));
  const double b = b0 + 16.0 * c.mps_used();
  if (threadIdx.x == 0 && norms) norms[i] = sqrt(n2);
  flush_stats(c, stats, b, 8.0 * b, 0.0);
}

// calcHessianRow (src/OptimalControl.cpp:251-279).  psiH_i =
// exactApplyMPO(propDeriv, psi_t[i]) and its norm normiH come from a preceding
// batched body_apply_dH launch (slots psih_base + i, norms[i]).
template <int NT>
__device__ OCG_INLINE void body_hessian_rows(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md, Pool pool,
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
    const double used = c.mps_used();
    if (threadIdx.x == 0) {
      zc di = divT[i], dj = divT[j];
      double v1 = (F.x * ov.x - F.y * ov.y) * (j > i ? normiH : 1.0);  // Re(F <xiH_j|psiH> n_i)
      double v2 = -(di.x * dj.x + di.y * dj.y);                        // -Re(divT_i conj(divT_j))
      double res = dt2 * (v1 + v2);
      H[(size_t)i * N + j] = res;
      if (j > i) H[(size_t)j * N + i] = res;
      bytes += 32.0 * used;
    }
  }
  double mb, mf;
  c.model_totals(mb, mf);
  bytes += mb;
  flops += mf;
  flush_stats(c, stats, bytes, flops, double(N - 2 - i > 0 ? N - 2 - i : 0));
}

// nsteps steps per state; u holds nsteps+1 controls per state (u_stride apart)
template <int NT>
__device__ OCG_INLINE void body_steps(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
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
  }
  c.store(SLOT_D(pool, P, slots[i]), SLOT_X(pool, P, slots[i]));
  c.model_totals(bytes, flops);
  flush_stats(c, stats, bytes, flops, double(nsteps));
}


}  // namespace ocg
