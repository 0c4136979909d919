// liboptimalcontrolmps_amd: HIP kernels (gfx950) + the C-ABI of include/ocmps.h.
//
// Kernels (one workgroup = one MPS chain resident in LDS, engine_device.hpp):
//   k_trajectory  : psi_t forward chain and xi_t backward chain (calcPsi / calcXi)
//   k_overlaps    : batched <x|y> / <x|dH|y> (calcDivT, fidelities, overlapFactor)
//   k_apply_dH    : batched exactApplyMPO(propDeriv, .) (xiHlist)
//   k_hessian_rows: calcHessianRow — dH psi_i, then re-propagate + overlap per j
//   k_steps       : TimeStepper::step on host-provided states
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ocmps.h"
#include "engine.hpp"
#include "hbm.hpp"
#include "engine_device.hpp"
#include "params.hpp"
#include "fast_plan.hpp"

using ocg::Chain;
using ocg::zc;
static inline zc mkz(double x, double y) { zc r; r.x = x; r.y = y; return r; }

#ifndef OCG_NT
#define OCG_NT 128
#endif
static constexpr int NT = OCG_NT;
static constexpr int kXiHWorkers = 12;  // A/B (config 1, one-wave chain): 8 -> 7.62 ms, 12 -> 7.53, 16 -> 7.53, 24 -> 7.49 per pipeline

#include "kernels.hpp"
using ocg::Pool;

// --------------------------------------------------------------------------
// __global__ entry points
__global__ __launch_bounds__(NT) void k_trajectory(OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                   Pool pool, int slot_init, int slot_target, int psi_base,
                                                   int xi_base, const double* u, int N, int which, double* stats,
                                                   int cs) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_trajectory<NT>(smem, P, gf, gb, md, pool, slot_init, slot_target, psi_base, xi_base, u, N, which, stats,
                           cs);
}

__global__ __launch_bounds__(NT) void k_overlaps(OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                 Pool pool, const int* xs, const int* ys, int npairs, int with_dH,
                                                 zc* out, double* stats) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_overlaps<NT>(smem, P, gf, gb, md, pool, xs, ys, npairs, with_dH, out, stats);
}

__global__ __launch_bounds__(NT) void k_apply_dH(OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                 Pool pool, const int* in, const int* outs, int n, double* norms,
                                                 double* stats) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_apply_dH<NT>(smem, P, gf, gb, md, pool, in, outs, n, norms, stats);
}

__global__ __launch_bounds__(NT) void k_hessian_rows(OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                     Pool pool, int psih_base, int xih_base, const int* rows,
                                                     int nrows, const double* norms, const double* u, int N,
                                                     const zc* divT, zc F, double* H, double* stats) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_hessian_rows<NT>(smem, P, gf, gb, md, pool, psih_base, xih_base, rows, nrows, norms, u, N, divT, F, H,
                             stats);
}

__global__ __launch_bounds__(NT) void k_pipeline(OcgParams P, const zc* gf, const zc* gb, const int* md, Pool pool,
                                                 int slot_init, int slot_target, int psi_base, int xi_base,
                                                 int xih_base, const double* u, int N, const int* rows, int nrows,
                                                 const int* rbase, Pool rs, double* rnorm, int* flags, int epoch,
                                                 int* err, int nxw, double* stats, int K, int cs) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_pipeline<NT>(smem, P, gf, gb, md, pool, slot_init, slot_target, psi_base, xi_base, xih_base, u, N, rows,
                         nrows, rbase, rs, rnorm, flags, epoch, err, nxw, stats, K, cs);
}

__global__ __launch_bounds__(NT) void k_row_overlaps(OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                     Pool pool, int xih_base, const int* rows, int nrows,
                                                     const int* rbase, Pool rs, const double* rnorm,
                                                     const zc* divT, const zc* F, int N, double* H, double* stats,
                                                     int K, int cs) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_row_overlaps<NT>(smem, P, gf, gb, md, pool, xih_base, rows, nrows, rbase, rs, rnorm, divT, F, N, H,
                             stats, K, cs);
}

// the same body on one wave per overlap: the contraction's barriers become
// wave barriers and twice as many overlaps fit a CU (the pairs are small)
__global__ __launch_bounds__(64) void k_row_overlaps_w(OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                       Pool pool, int xih_base, const int* rows, int nrows,
                                                       const int* rbase, Pool rs, const double* rnorm,
                                                       const zc* divT, const zc* F, int N, double* H, double* stats,
                                                       int K, int cs) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_row_overlaps<64>(smem, P, gf, gb, md, pool, xih_base, rows, nrows, rbase, rs, rnorm, divT, F, N, H,
                             stats, K, cs);
}

// the row overlaps on the padded layout (fast_overlap.hpp): one wave, ~12 KB
__global__ __launch_bounds__(64) void k_row_overlaps_pad(OcgParams P, Pool pool, int xih_base, const int* rows,
                                                         int nrows, const int* rbase, Pool rs, const double* rnorm,
                                                         const zc* divT, const zc* F, int N, double* H,
                                                         double* stats, int K, int cs) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_row_overlaps_pad(smem, P, pool, xih_base, rows, nrows, rbase, rs, rnorm, divT, F, N, H, stats, K, cs);
}

// <x|y> / <x|dH|y> pairs on the padded layout (fast_overlap.hpp): one wave per pair
__global__ __launch_bounds__(64) void k_overlaps_pad(OcgParams P, Pool pool, const int* xs, const int* ys, int n,
                                                     int with_dH, zc* out, double* stats) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_overlaps_pad(smem, P, pool, xs, ys, n, with_dH, out, stats);
}

__global__ __launch_bounds__(NT) void k_steps(OcgParams P, const zc* gf, const zc* gb, const int* md,
                                              Pool pool, const int* slots, int n, const double* u, int u_stride,
                                              int nsteps, int forward, double* stats) {
  extern __shared__ __align__(16) char smem[];
  ocg::body_steps<NT>(smem, P, gf, gb, md, pool, slots, n, u, u_stride, nsteps, forward, stats);
}

// ControlBasis::convertHessian (src/ControlBasis.cpp:91-116): H_c = V H_u V^T,
// V_{n i} = S_i f_{i n}.  Every entry is one sequential inner product in the
// reference's order (std::inner_product: acc = acc + a * b, no fused
// multiply-add), so the device result is bit-identical to the host facade's.
// Stage 1, one workgroup per row k of H_u (row staged in LDS), one thread per
// basis vector j: HV[j][k] = sum_l H_u[k][l] V[j][l] (V read transposed,
// coalesced over j).  Stage 2, one thread per (i, j >= i):
// H_c[i][j] = H_c[j][i] = sum_k V[i][k] HV[j][k].
__global__ __launch_bounds__(256) void k_project_hv(const double* Hu, const double* Vt, int N, int M, double* HV) {
#pragma clang fp contract(off)
  extern __shared__ __align__(16) char smem[];
  double* row = (double*)smem;
  const int k = blockIdx.x;
  for (int l = threadIdx.x; l < N; l += blockDim.x) row[l] = Hu[(size_t)k * N + l];
  __syncthreads();
  for (int j = threadIdx.x; j < M; j += blockDim.x) {
    double acc = 0.0;
    for (int l = 0; l < N; ++l) acc = acc + row[l] * Vt[(size_t)l * M + j];
    HV[(size_t)j * N + k] = acc;
  }
}
__global__ __launch_bounds__(256) void k_project_c(const double* V, const double* HV, int N, int M, double* Hc) {
#pragma clang fp contract(off)
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * M) return;
  const int i = t / M, j = t % M;
  if (j < i) return;
  double acc = 0.0;
  for (int k = 0; k < N; ++k) acc = acc + V[(size_t)i * N + k] * HV[(size_t)j * N + k];
  Hc[(size_t)i * M + j] = acc;
  Hc[(size_t)j * M + i] = acc;
}

// ==========================================================================
// host side
// ==========================================================================
namespace {

thread_local std::string g_create_error;

struct KStat {
  double ms = 0;
  long launches = 0;
};

}  // namespace

struct ocg_ctx {
  int device = 0;
  hbm_engine* hbm = nullptr;  // set: this context runs on the HBM-resident engine (hbm.hip)
  OcgParams P{};
  int lds_np = 0;   // LDS of the kernels that never step (no plan slots)
  int lds_ovl = 0;  // LDS of the overlap-only kernels (compact layout)
  // parameter block of the overlap-only kernels
  OcgParams Po() const {
    OcgParams q = P;
    q.fplan = nullptr;
    q.nplan = 0;
    q.plan_pe = 0;
    q.lds_bytes = lds_ovl;
    return q;
  }
  // chain parameter block sized for two chain workgroups per CU (plan slots
  // shrunk to half the LDS, or none): many concurrent chains (ocg_hessian_multi)
  int plan_pe2 = 0, lds2 = 0;
  // the one-wave chain's region aliasing the general chain's LDS (fast_off 0, the
  // larger of the two sizes): for kernels whose workgroups use the general chain
  // only before the one-wave chain starts (k_trajectory, k_steps, k_pipeline);
  // k_hessian_rows hands states back and forth and keeps the two regions apart
  int lds_alias = 0;
  OcgParams Pa() const {
    OcgParams q = P;
    if (P.fplan && lds_alias > 0) {
      q.fast_off = 0;
      q.lds_bytes = lds_alias;
    }
    return q;
  }
  OcgParams P2() const {
    OcgParams q = P;
    if (P.fplan) return Pa();  // the one-wave chain: aliased regions (two or more chains per CU)
    if (plan_pe2 >= 32) {
      q.plan_pe = plan_pe2;
      q.lds_bytes = lds2;
    } else {
      q.nplan = 0;
      q.plan_pe = 0;
      q.lds_bytes = lds_np;
    }
    return q;
  }
  // parameter block of those kernels: plans off, smaller LDS
  OcgParams Pn() const {
    OcgParams q = P;
    q.fplan = nullptr;
    q.nplan = 0;
    q.plan_pe = 0;
    q.lds_bytes = lds_np;
    return q;
  }
  double J = 1.0;
  std::vector<int> md;  // (L+1)*Q1 rank bounds
  std::string err;
  // HBM engine getHessian path counters (ocg_kernel_stats kind 8): pipelined
  // calls completed, and two-phase retries after a pipeline that ran out of memory
  long pipe_runs = 0, pipe_fallbacks = 0, ckpt_runs = 0, ckpt_k = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t evh[4] = {nullptr, nullptr, nullptr, nullptr};  // ocg_hessian phase marks
  // device buffers
  zc *d_gf = nullptr, *d_gb = nullptr;
  int* d_md = nullptr;
  Pool pool{nullptr, nullptr};
  int nslots = 0;
  double* d_stats = nullptr;  // [8][3]
  int* d_idx = nullptr;       // index scratch
  int idx_cap = 0;
  double* d_u = nullptr;
  int u_cap = 0;
  zc* d_c = nullptr;     // complex scratch (overlaps / divT)
  int c_cap = 0;
  double* d_H = nullptr;
  size_t H_cap = 0;
  double* d_norms = nullptr;
  int norms_cap = 0;
  double* d_rnorm = nullptr;  // psiH norms (by row index)
  int rnorm_cap = 0;
  int* d_idx2 = nullptr;      // index scratch of the psiH launch
  int idx2_cap = 0;
  // fused pipeline (ocg_hessian)
  Pool rs{nullptr, nullptr};  // stored psiH_i(j) states
  size_t rs_cap = 0;
  char* h_pin = nullptr;      // pinned host staging of the fused getHessian's uploads / results
  size_t pin_cap = 0;
  int* d_flags = nullptr;     // [2N] psi / xi publication epochs
  int flags_cap = 0;
  int flags_N = -1, flags_K = -1;  // (N, K) layout of the flag buffer's current epoch run
  int epoch = 0;
  int* d_err = nullptr;
  int* d_rows = nullptr;      // rows, then rbase (nrows + 1)
  int rows_cap = 0;
  double* d_proj = nullptr;   // convertHessian operands (H_u, V, V^T, HV, H_c)
  size_t proj_cap = 0;
  zc* d_pc = nullptr;         // divT (N) and F (1) on the device
  int pc_cap = 0;
  double* d_prn = nullptr;    // psiH norms by row slot
  int prn_cap = 0;
  int* d_fplan = nullptr;     // plan image of the one-wave padded chain (null: off)
  int* d_oplan = nullptr;     // overlap plan of the padded layout (null: off)
  std::string fast_why;       // why it is off
  // trajectory state
  int N = 0;
  std::vector<double> u_psi, u_xi;  // controls of the device psi_t / xi_t (empty: none)
  bool have_states = false, have_psi = false, have_xi = false, have_xih = false;
  KStat kst[8];
  // slot map
  int slot_init() const { return 0; }
  int slot_target() const { return 1; }
  int slot_tmp(int i) const { return 2 + i; }          // 4 scratch slots
  int psi_base() const { return 6; }
  int xi_base() const { return 6 + N; }
  int xih_base() const { return 6 + 2 * N; }
  int psih_base() const { return 6 + 3 * N; }
};

#define HIPCHK(ctx, expr)                                                               \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                   \
      return OCG_EHIP;                                                                  \
    }                                                                                   \
  } while (0)

static int fail(ocg_ctx* c, int code, const std::string& m) {
  c->err = m;
  return code;
}

static int upload_gates(ocg_ctx* c) {
  std::vector<double> gf, gb;
  ocg_host::gate_tables(c->P, c->J, gf, gb);
  const int off = c->P.gtotal;
  if (!c->d_gf) {
    HIPCHK(c, hipMalloc(&c->d_gf, sizeof(zc) * off));
    HIPCHK(c, hipMalloc(&c->d_gb, sizeof(zc) * off));
  }
  HIPCHK(c, hipMemcpyAsync(c->d_gf, gf.data(), sizeof(zc) * off, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_gb, gb.data(), sizeof(zc) * off, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

static int build_params(ocg_ctx* c, int L, int p, int npart, double tstep, double cutoff, int maxm) {
  std::string e = ocg_host::build_params(c->P, c->md, L, p, npart, tstep, cutoff, maxm);
  if (!e.empty()) return fail(c, e.find("too large") != std::string::npos ? OCG_ECAP : OCG_EINVAL, e);
  return 0;
}

static int ensure_slots(ocg_ctx* c, int nslots) {
  if (nslots <= c->nslots) return 0;
  int n = std::max(nslots, 2 * c->nslots);
  int* nd = nullptr;
  zc* nx = nullptr;
  HIPCHK(c, hipMalloc(&nd, sizeof(int) * size_t(n) * c->P.nsq));
  HIPCHK(c, hipMalloc(&nx, sizeof(zc) * size_t(n) * c->P.cap));
  // every copy / fill is ordered on the context's (non-blocking) stream: a
  // null-stream hipMemset / device-to-device hipMemcpy is asynchronous to the
  // host and unordered with it, so a later upload or kernel could overtake it
  HIPCHK(c, hipMemsetAsync(nd, 0, sizeof(int) * size_t(n) * c->P.nsq, c->stream));
  if (c->nslots) {
    HIPCHK(c, hipMemcpyAsync(nd, c->pool.dims, sizeof(int) * size_t(c->nslots) * c->P.nsq, hipMemcpyDeviceToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(nx, c->pool.data, sizeof(zc) * size_t(c->nslots) * c->P.cap, hipMemcpyDeviceToDevice,
                             c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->nslots) {
    (void)hipFree(c->pool.dims);
    (void)hipFree(c->pool.data);
  }
  c->pool.dims = nd;
  c->pool.data = nx;
  c->nslots = n;
  return 0;
}

template <class T>
static int ensure_buf(ocg_ctx* c, T*& ptr, int& cap, int n) {
  if (n <= cap) return 0;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // queued work may still read the old buffer
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  int m = std::max(n, 2 * cap);
  HIPCHK(c, hipMalloc(&ptr, sizeof(T) * size_t(m)));
  cap = m;
  return 0;
}

// pinned host staging of at least `bytes` (the stream is drained before a
// reallocation: queued copies may still use the old buffer)
static int ensure_pin(ocg_ctx* c, size_t bytes) {
  if (bytes <= c->pin_cap) return 0;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t m = std::max(bytes, 2 * c->pin_cap);
  if (c->h_pin) (void)hipHostFree(c->h_pin);
  c->h_pin = nullptr;
  c->pin_cap = 0;
  HIPCHK(c, hipHostMalloc((void**)&c->h_pin, m, hipHostMallocDefault));
  c->pin_cap = m;
  return 0;
}

// host compact <-> slot layout
static size_t nelem_of(const OcgParams& P, const int* dims, int k) {
  size_t s = 0;
  for (int q = 0; q < P.Q1; ++q)
    for (int n = 0; n < P.p && q + n <= P.Q; ++n) s += size_t(dims[(k - 1) * P.Q1 + q]) * dims[k * P.Q1 + q + n];
  return s;
}

static int validate_dims(ocg_ctx* c, const int* dims) {
  const OcgParams& P = c->P;
  if (dims[0] != 1) return fail(c, OCG_EINVAL, "bond 0 must be one state with q = 0");
  for (int q = 1; q < P.Q1; ++q)
    if (dims[q] != 0) return fail(c, OCG_EINVAL, "bond 0 must be one state with q = 0");
  for (int q = 0; q < P.Q1; ++q)
    if (dims[P.L * P.Q1 + q] != (q == P.Q ? 1 : 0))
      return fail(c, OCG_EINVAL, "bond L must be one state with q = Q (particle number mismatch?)");
  for (int b = 0; b <= P.L; ++b)
    for (int q = 0; q < P.Q1; ++q) {
      int v = dims[b * P.Q1 + q];
      if (v < 0) return fail(c, OCG_EINVAL, "negative bond dimension");
      if (v > c->md[b * P.Q1 + q])
        return fail(c, OCG_ECAP, "bond " + std::to_string(b) + " sector " + std::to_string(q) +
                                      " exceeds its Schmidt-rank bound");
    }
  return 0;
}

static int upload_mps(ocg_ctx* c, int slot, const int* dims, const double* data) {
  const OcgParams& P = c->P;
  if (int rc = validate_dims(c, dims)) return rc;
  std::vector<zc> buf(P.cap, mkz(0, 0));
  size_t off = 0;
  for (int k = 1; k <= P.L; ++k) {
    size_t n = nelem_of(P, dims, k);
    if (n > size_t(P.site_cap[k])) return fail(c, OCG_ECAP, "site tensor exceeds capacity");
    for (size_t i = 0; i < n; ++i) buf[P.site_base[k] + i] = mkz(data[2 * (off + i)], data[2 * (off + i) + 1]);
    off += n;
  }
  HIPCHK(c, hipMemcpyAsync(SLOT_D(c->pool, P, slot), dims, sizeof(int) * P.nsq, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(SLOT_X(c->pool, P, slot), buf.data(), sizeof(zc) * P.cap, hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

static int download_mps(ocg_ctx* c, int slot, int* dims, double* data, size_t cap, size_t* nelem) {
  const OcgParams& P = c->P;
  std::vector<int> d(P.nsq);
  std::vector<zc> buf(P.cap);
  HIPCHK(c, hipMemcpyAsync(d.data(), SLOT_D(c->pool, P, slot), sizeof(int) * P.nsq, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(buf.data(), SLOT_X(c->pool, P, slot), sizeof(zc) * P.cap, hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  size_t tot = 0;
  for (int k = 1; k <= P.L; ++k) tot += nelem_of(P, d.data(), k);
  if (nelem) *nelem = tot;
  if (tot > cap) return fail(c, OCG_ECAP, "output buffer too small");
  std::memcpy(dims, d.data(), sizeof(int) * P.nsq);
  size_t off = 0;
  for (int k = 1; k <= P.L; ++k) {
    size_t n = nelem_of(P, d.data(), k);
    for (size_t i = 0; i < n; ++i) {
      data[2 * (off + i)] = buf[P.site_base[k] + i].x;
      data[2 * (off + i) + 1] = buf[P.site_base[k] + i].y;
    }
    off += n;
  }
  return 0;
}

static int begin_kernel(ocg_ctx* c) {
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  return 0;
}
// After a synchronised launch: a nonzero device error word (a Jacobi that hit
// its sweep cap, a pipeline watchdog) fails the call with OCG_ENUM and
// invalidates every device-resident trajectory (a partly rewritten slot must
// not be read as a valid psi_t / xi_t / xiH_t).
static int check_err(ocg_ctx* c) {
  int err = 0;
  HIPCHK(c, hipMemcpyAsync(&err, c->d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (!err) return 0;
  HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->have_psi = c->have_xi = c->have_xih = false;
  std::string m;
  if (err & OCG_ERR_JACOBI) m += "eigensolver did not converge within its sweep cap; ";
  if (err & OCG_ERR_WATCHDOG) m += "pipeline watchdog: a consumer saw no producer progress for ~15 s; ";
  return fail(c, OCG_ENUM, m.empty() ? std::string("kernel error flag set") : m);
}

static int end_kernel(ocg_ctx* c, int kind) {
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  HIPCHK(c, hipEventSynchronize(c->ev1));
  float ms = 0;
  HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->kst[kind].ms += ms;
  c->kst[kind].launches += 1;
  return check_err(c);
}

static int set_lds(ocg_ctx* c) {
  const int bytes = c->P.lds_bytes;
  HIPCHK(c, hipFuncSetAttribute((const void*)k_trajectory, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIPCHK(c, hipFuncSetAttribute((const void*)k_overlaps, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIPCHK(c, hipFuncSetAttribute((const void*)k_apply_dH, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIPCHK(c, hipFuncSetAttribute((const void*)k_hessian_rows, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIPCHK(c, hipFuncSetAttribute((const void*)k_steps, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIPCHK(c, hipFuncSetAttribute((const void*)k_pipeline, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIPCHK(c, hipFuncSetAttribute((const void*)k_row_overlaps, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIPCHK(c, hipFuncSetAttribute((const void*)k_row_overlaps_w, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  return 0;
}

static int finish_params(ocg_ctx* c) {
  if (c->P.gtotal <= 0) return fail(c, OCG_ESTATE, "internal: gate tables must be built before the LDS layout");
  c->P.nplan = 0;
  c->P.plan_pe = 0;
  c->lds_ovl = ocg::lds_layout_ovl(c->P, NT).bytes;
  ocg::LdsLayout l = ocg::lds_layout(c->P, NT);
  c->P.lds_bytes = l.bytes;
  c->lds_np = l.bytes;
  hipDeviceProp_t prop;
  HIPCHK(c, hipGetDeviceProperties(&prop, c->device));
  size_t limit = prop.sharedMemPerBlock;
  if (prop.maxSharedMemoryPerMultiProcessor > limit) limit = prop.maxSharedMemoryPerMultiProcessor;
  // decomposition plans (one slot per decomposition of a step: the gates and
  // the gauge moves between them) when their 16-bit offsets suffice; the
  // per-slot element capacity is the two-site / site bound, shrunk to the LDS
  // left over (a decomposition larger than its slot just runs unplanned)
  const char* np = std::getenv("OCG_NO_PLANS");  // diagnostic / test switch: general path only
  const bool plans_off = np && np[0] && np[0] != '0';
  // plan slot capacity (elements) that fits `lim` bytes of LDS, 0 if none
  auto plan_fit = [&](size_t lim, int& bytes) {
    if (plans_off || !(c->P.cap < 65536 && c->P.thcap < 65536 && c->P.evcap < 4096)) return 0;
    OcgParams q = c->P;
    q.nplan = q.ngates + ocg_host::step_gauge_moves(q);
    q.plan_pe = 0;
    const int b0 = ocg::lds_layout(q, NT).bytes;
    q.plan_pe = 64;
    const int per = (ocg::lds_layout(q, NT).bytes - b0 + 63) / 64;  // bytes per element, all slots
    const int want = std::max(q.th2cap, q.max_site_cap);
    q.plan_pe = std::min(want, per > 0 ? int((long(lim) - b0) / per) - 8 : 0);
    while (q.plan_pe >= 32 && size_t(ocg::lds_layout(q, NT).bytes) > lim) q.plan_pe -= 8;
    if (q.plan_pe < 32) return 0;
    bytes = ocg::lds_layout(q, NT).bytes;
    return q.plan_pe;
  };
  const int nplan = c->P.ngates + ocg_host::step_gauge_moves(c->P);  // slots: one per decomposition of a step
  int b1 = 0, b2 = 0;
  const int pe1 = plan_fit(limit, b1);                                            // one chain per CU
  c->plan_pe2 = plan_fit(std::max<size_t>(size_t(l.bytes), limit / 2), b2);      // two chains per CU
  c->lds2 = b2;
  if (pe1 >= 32) {
    c->P.nplan = nplan;
    c->P.plan_pe = pe1;
    c->P.lds_bytes = b1;
  }
  if (size_t(l.bytes) > limit)
    return fail(c, OCG_ECAP,
                "chain workgroup needs " + std::to_string(l.bytes) + " B of LDS (> " + std::to_string(limit) +
                    "): configuration exceeds the single-workgroup engine (see DESIGN.md §Scope)");
  // the one-wave padded chain (fast_chain.hpp) for every step when the
  // configuration fits it (OCG_NO_FAST=1: the general chain steps, A/B and tests);
  // its region follows the plan-less layout, whose decompositions (exactApplyMPO,
  // the ground state) need no plans
  c->P.fplan = nullptr;
  c->P.fast_off = 0;
  c->P.oplan = nullptr;
  c->P.ovl_bytes = 0;
  c->P.ovl_dh_bytes = 0;
  const char* nf = std::getenv("OCG_NO_FAST");
  if (nf && nf[0] && nf[0] != '0') {
    c->fast_why = "OCG_NO_FAST";
    return 0;
  }
  ocg_host::FastPlanBuild fb = ocg_host::build_fast_plan(c->P, c->md);
  if (!fb.why_not.empty()) {
    c->fast_why = fb.why_not;
    return 0;
  }
  const int off = (l.bytes + 255) & ~255;
  const int fbytes = ocg_host::fast_lds_bytes(fb.plan, c->P);
  if (size_t(off + fbytes) > limit) {
    c->fast_why = "LDS";
    return 0;
  }
  HIPCHK(c, hipMalloc(&c->d_fplan, sizeof(int) * fb.plan.size()));
  HIPCHK(c, hipMemcpyAsync(c->d_fplan, fb.plan.data(), sizeof(int) * fb.plan.size(), hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->P.fplan = c->d_fplan;
  c->P.fast_off = off;
  c->P.nplan = 0;
  c->P.plan_pe = 0;
  c->P.lds_bytes = off + fbytes;
  c->plan_pe2 = 0;
  c->lds2 = 0;
  // the padded overlap (fast_overlap.hpp) for getHessian's row overlaps; in
  // k_hessian_rows it lives in the general chain's region, so it must fit there
  // (OCG_NO_FAST_OVL=1: the general contraction, A/B and tests)
#ifndef OCG_PROFILE  // (the diagnostic build's phase counters live in that region)
  {
    const char* no = std::getenv("OCG_NO_FAST_OVL");
    const std::vector<int> ov = ocg_host::build_overlap_plan(c->P, c->md);
    const int ob = ov.empty() ? 0 : ocg_host::overlap_lds_bytes(ov, c->P);
    const int obd = ov.empty() ? 0 : ocg_host::overlap_lds_bytes(ov, c->P, true);
    if (!ov.empty() && ob <= off && obd <= 65536 && !(no && no[0] && no[0] != '0')) {
      HIPCHK(c, hipMalloc(&c->d_oplan, sizeof(int) * ov.size()));
      HIPCHK(c, hipMemcpyAsync(c->d_oplan, ov.data(), sizeof(int) * ov.size(), hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      c->P.oplan = c->d_oplan;
      c->P.ovl_bytes = ob;
      c->P.ovl_dh_bytes = obd;
      if (std::getenv("OCG_FAST_DUMP"))
        std::fprintf(stderr, "[fast ovl] np %d nblk %d ints %d bytes %d\n", ov[ocg::fastp::kOvNp],
                     ov[ocg::fastp::kOvNblk], ov[ocg::fastp::kOvNint], ob);
    }
  }
#endif
#ifdef OCG_PROFILE
  c->lds_alias = 0;  // the diagnostic build's phase counters live in the general chain's LDS
#else
  c->lds_alias = std::max(l.bytes, fbytes);
  if (const char* e = std::getenv("OCG_FAST_ALIAS"))
    if (e[0] == '0') c->lds_alias = 0;
#endif
  return 0;
}


// the context's stream and timing events (every copy, fill and launch of a
// context is ordered on this one non-blocking stream)
static bool make_stream(ocg_ctx* c) {
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreate(&c->evh[0]) != hipSuccess || hipEventCreate(&c->evh[1]) != hipSuccess ||
      hipEventCreate(&c->evh[2]) != hipSuccess || hipEventCreate(&c->evh[3]) != hipSuccess) {
    c->err = "stream/event creation failed";
    return false;
  }
  return true;
}

// controls of the device trajectories, so a Hessian at the control of the
// last gradient reuses psi_t / xi_t / xiHlist (BH_nlp::eval_h after
// eval_grad_f, src/BH_nlp.cpp:189)
static void note_u(ocg_ctx* c, const double* u, int N, int which) {
  if (which & 1) c->u_psi.assign(u, u + N);
  if (which & 2) c->u_xi.assign(u, u + N);
}
static bool same_u(const std::vector<double>& a, const double* u, int N) {
  return a.size() == size_t(N) && std::memcmp(a.data(), u, sizeof(double) * N) == 0;
}

// forward an HBM-engine status (its message becomes the context's)
static int hb(ocg_ctx* c, int rc) {
  if (rc) c->err = hbm_last_error(c->hbm);
  return rc;
}
extern "C" {

const char* ocg_last_error(const ocg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

size_t ocg_mps_nelem(int L, int p, int Q, const int* dims) {
  size_t s = 0;
  int Q1 = Q + 1;
  for (int k = 1; k <= L; ++k)
    for (int q = 0; q < Q1; ++q)
      for (int n = 0; n < p && q + n <= Q; ++n) s += size_t(dims[(k - 1) * Q1 + q]) * dims[k * Q1 + q + n];
  return s;
}

int ocg_device_count(int* n) {
  if (!n) return OCG_EINVAL;
  *n = 0;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess || *n <= 0) {
    g_create_error = std::string("no HIP device available: ") + hipGetErrorString(e);
    *n = 0;
    return OCG_EHIP;
  }
  return OCG_OK;
}

// the HBM-resident engine for configurations beyond the LDS chain engine
static int create_hbm(ocg_ctx* c, int L, int p, int npart, double tstep, double cutoff, int maxm) {
  std::vector<int> md, mdz;
  ocg_host::rank_bounds(L, p, npart, md, mdz);
  OcgParams G{};
  G.p = p;
  G.dt = tstep;
  std::vector<double> gf, gb;
  ocg_host::gate_tables(G, c->J, gf, gb);
  std::string err;
  const int rc = hbm_create(c->device, L, p, npart, c->J, tstep, cutoff, maxm, md, mdz, gf, gb, G.glo, G.gsz,
                            G.goff, G.gtotal, ocg_host::gate_order(L), &c->hbm, err);
  if (rc) return fail(c, rc, "HBM engine: " + err);
  c->P.L = L; c->P.p = p; c->P.Q = npart; c->P.Q1 = npart + 1; c->P.nsq = (L + 1) * (npart + 1);
  c->P.dt = tstep; c->P.cutoff = cutoff; c->P.maxm = maxm > 0 ? maxm : 5000;
  return 0;
}

int ocg_create_ex(int device, int L, int p, int npart, double J, double tstep, double cutoff, int maxm, int engine,
                  ocg_ctx** out) {
  if (!out) { g_create_error = "out is NULL"; return OCG_EINVAL; }
  *out = nullptr;
  if (engine < 0 || engine > 2) { g_create_error = "engine must be 0 (auto), 1 (LDS) or 2 (HBM)"; return OCG_EINVAL; }
  auto* c = new ocg_ctx;
  c->device = device;
  c->J = J;
  auto bail = [&](int code) {
    g_create_error = c->err;
    ocg_destroy(c);
    return code;
  };
  // the LDS chain engine's parameter block holds up to OCG_MAXL sites and
  // OCG_MAXQ1 sectors; the HBM engine takes up to 63 sites (config 5: L = 50)
  const bool lds_fits = L <= OCG_MAXL && npart + 1 <= OCG_MAXQ1;
  if (L < 2 || L > 63 || p < 2 || p > OCG_MAXP || npart < 0 || npart + 1 > 1024 || npart > L * (p - 1) ||
      !(tstep == tstep) || !(cutoff >= 0) || (engine == 1 && !lds_fits)) {
    int rc = build_params(c, L, p, npart, tstep, cutoff, maxm);  // same messages as before
    if (!rc) { c->err = "bad argument"; rc = OCG_EINVAL; }
    return bail(rc);
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) {
    c->err = std::string("no HIP device available: ") + hipGetErrorString(e);
    return bail(OCG_EHIP);
  }
  if (device < 0 || device >= ndev) { c->err = "device index out of range"; return bail(OCG_EINVAL); }
  if (hipSetDevice(device) != hipSuccess) { c->err = "hipSetDevice failed"; return bail(OCG_EHIP); }
  if (!make_stream(c)) return bail(OCG_EHIP);
  int rc = 0;
  if (engine != 2 && lds_fits) {
    rc = build_params(c, L, p, npart, tstep, cutoff, maxm);
    // gate tables first: their size (gtotal) is part of the LDS layout
    if (!rc) rc = upload_gates(c);
    if (!rc) rc = finish_params(c);
    if (rc == OCG_ECAP && engine == 0) {
      // beyond the single-workgroup LDS engine: the HBM-resident engine
      const std::string why = c->err;
      ocg_ctx* h = new ocg_ctx;
      h->device = device;
      h->J = J;
      if (!make_stream(h)) {
        ocg_destroy(h);
        return bail(OCG_EHIP);
      }
      std::swap(c, h);
      ocg_destroy(h);
      if ((rc = create_hbm(c, L, p, npart, tstep, cutoff, maxm))) return bail(rc);
    } else if (rc) {
      return bail(rc);
    }
  } else if ((rc = create_hbm(c, L, p, npart, tstep, cutoff, maxm))) {
    return bail(rc);
  }
  if (c->hbm) {
    *out = c;
    return 0;
  }
  if (hipMalloc(&c->d_md, sizeof(int) * c->md.size()) != hipSuccess ||
      hipMemcpyAsync(c->d_md, c->md.data(), sizeof(int) * c->md.size(), hipMemcpyHostToDevice, c->stream) !=
          hipSuccess ||
      hipMalloc(&c->d_stats, sizeof(double) * 24) != hipSuccess ||
      hipMemsetAsync(c->d_stats, 0, sizeof(double) * 24, c->stream) != hipSuccess ||
      hipMalloc(&c->d_err, sizeof(int)) != hipSuccess || hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    c->err = "device allocation failed";
    return bail(OCG_EHIP);
  }
  c->P.err = c->d_err;
  if ((rc = set_lds(c))) return bail(rc);
  if ((rc = ensure_slots(c, 8))) return bail(rc);
  *out = c;
  return 0;
}

int ocg_create(int device, int L, int p, int npart, double J, double tstep, double cutoff, int maxm, ocg_ctx** out) {
  return ocg_create_ex(device, L, p, npart, J, tstep, cutoff, maxm, 0, out);
}

int ocg_destroy(ocg_ctx* c) {
  if (!c) return 0;
  if (c->device >= 0) (void)hipSetDevice(c->device);
  if (c->hbm) hbm_destroy(c->hbm);
  if (c->d_gf) (void)hipFree(c->d_gf);
  if (c->d_gb) (void)hipFree(c->d_gb);
  if (c->d_md) (void)hipFree(c->d_md);
  if (c->pool.dims) (void)hipFree(c->pool.dims);
  if (c->pool.data) (void)hipFree(c->pool.data);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->rs.dims) (void)hipFree(c->rs.dims);
  if (c->rs.data) (void)hipFree(c->rs.data);
  if (c->d_flags) (void)hipFree(c->d_flags);
  if (c->d_err) (void)hipFree(c->d_err);
  if (c->d_rows) (void)hipFree(c->d_rows);
  if (c->d_pc) (void)hipFree(c->d_pc);
  if (c->d_prn) (void)hipFree(c->d_prn);
  if (c->d_proj) (void)hipFree(c->d_proj);
  if (c->d_idx) (void)hipFree(c->d_idx);
  if (c->d_u) (void)hipFree(c->d_u);
  if (c->d_c) (void)hipFree(c->d_c);
  if (c->d_H) (void)hipFree(c->d_H);
  if (c->h_pin) (void)hipHostFree(c->h_pin);
  if (c->d_norms) (void)hipFree(c->d_norms);
  if (c->d_rnorm) (void)hipFree(c->d_rnorm);
  if (c->d_idx2) (void)hipFree(c->d_idx2);
  if (c->d_fplan) (void)hipFree(c->d_fplan);
  if (c->d_oplan) (void)hipFree(c->d_oplan);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  for (auto& e : c->evh)
    if (e) (void)hipEventDestroy(e);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int ocg_abi_version(void) { return OCG_ABI_VERSION; }

int ocg_get_info_sz(const ocg_ctx* c, ocg_info* info, size_t info_size) {
  if (!c || !info) return OCG_EINVAL;
  ocg_info full{};
  const int rc = ocg_get_info(c, &full);
  if (rc) return rc;
  std::memcpy(info, &full, std::min(info_size, sizeof(full)));
  return 0;
}

int ocg_get_path_stats(ocg_ctx* c, ocg_path_stats* out) {
  if (!c || !out || out->size < sizeof(size_t)) return OCG_EINVAL;
  ocg_path_stats v{};
  v.size = sizeof(v);
  v.pipe_runs = c->pipe_runs;
  v.pipe_fallbacks = c->pipe_fallbacks;
  v.ckpt_runs = c->ckpt_runs;
  v.ckpt_k = c->ckpt_k;
  if (c->hbm) {
    const int rc = hbm_coop_stats(c->hbm, &v.coop_launches, &v.coop_groups, &v.coop_fallbacks);
    if (rc) return hb(c, rc);
  }
  const size_t sz = std::min(out->size, sizeof(v));
  std::memcpy(out, &v, sz);
  out->size = sz;
  return 0;
}

int ocg_get_info(const ocg_ctx* c, ocg_info* info) {
  if (!c || !info) return OCG_EINVAL;
  if (c->hbm) {
    info->L = c->P.L; info->p = c->P.p; info->Q = c->P.Q;
    info->mps_max_nelem = hbm_mps_max_nelem(c->hbm);
    info->lds_bytes = 0;
    info->block_threads = 256;
    info->device = c->device;
    info->fast_chain = 0;
    return 0;
  }
  info->L = c->P.L; info->p = c->P.p; info->Q = c->P.Q;
  info->mps_max_nelem = size_t(c->P.cap);
  info->lds_bytes = c->P.lds_bytes;
  info->block_threads = NT;
  info->device = c->device;
  info->fast_chain = c->P.fplan != nullptr;
  return 0;
}

int ocg_set_tstep(ocg_ctx* c, double tstep) {
  if (!c) return OCG_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  c->P.dt = tstep;
  c->have_psi = c->have_xi = c->have_xih = false;
  c->u_psi.clear();  // trajectories of the old dt are never reused
  c->u_xi.clear();
  if (c->hbm) {
    OcgParams G{};
    G.p = c->P.p;
    G.dt = tstep;
    std::vector<double> gf, gb;
    ocg_host::gate_tables(G, c->J, gf, gb);
    return hb(c, hbm_set_tstep(c->hbm, tstep, gf, gb, G.glo, G.gsz, G.goff, G.gtotal));
  }
  return upload_gates(c);
}

static int launch_steps(ocg_ctx* c, int slot, const double* u, int nsteps, int forward) {
  const OcgParams& P = c->P;
  if (int rc = ensure_buf(c, c->d_u, c->u_cap, nsteps + 1)) return rc;
  if (int rc = ensure_buf(c, c->d_idx, c->idx_cap, 1)) return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_u, u, sizeof(double) * (nsteps + 1), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_idx, &slot, sizeof(int), hipMemcpyHostToDevice, c->stream));
  if (int rc = begin_kernel(c)) return rc;
  const OcgParams Pa = c->Pa();  // the one-wave chain aliases the general LDS
  hipLaunchKernelGGL(k_steps, dim3(1), dim3(NT), Pa.lds_bytes, c->stream, Pa, c->d_gf, c->d_gb, c->d_md, c->pool,
                     c->d_idx, 1, c->d_u, nsteps + 1, nsteps, forward, c->d_stats + 4 * 3);
  return end_kernel(c, 4);
}

int ocg_steps(ocg_ctx* c, const int* dims, const double* data, const double* u, int nsteps, int forward,
              int* out_dims, double* out_data, size_t out_cap, size_t* out_nelem) {
  if (!c || !dims || !data || !u || nsteps < 0) return c ? fail(c, OCG_EINVAL, "null argument") : OCG_EINVAL;
  if (c->hbm) {
    const int fw = forward;
    double* od[1] = {out_data};
    return hb(c, hbm_steps(c->hbm, 1, dims, &data, u, nsteps + 1, nsteps, &fw, out_dims, od, &out_cap, out_nelem));
  }
  HIPCHK(c, hipSetDevice(c->device));
  int slot = c->slot_tmp(0);
  if (int rc = upload_mps(c, slot, dims, data)) return rc;
  if (nsteps > 0)
    if (int rc = launch_steps(c, slot, u, nsteps, forward)) return rc;
  return download_mps(c, slot, out_dims, out_data, out_cap, out_nelem);
}

int ocg_step(ocg_ctx* c, const int* dims, const double* data, double from, double to, int forward, int* out_dims,
             double* out_data, size_t out_cap, size_t* out_nelem) {
  double u[2] = {from, to};
  return ocg_steps(c, dims, data, u, 1, forward, out_dims, out_data, out_cap, out_nelem);
}

// Ground-state preparation (InitializeState, include/InitializeState.hpp:18-117):
// nsteps imaginary-time Trotter steps exp(-tau H) at constant U, the same
// sweep as BH_tDMRG::step with the gates and phases of imaginary time
// (doStep normalises after every gate and at the end).  The context's real-
// time gates are swapped back afterwards; device trajectories stay valid.
int ocg_imag_steps(ocg_ctx* c, const int* dims, const double* data, double U, double tau, int nsteps,
                   int* out_dims, double* out_data, size_t out_cap, size_t* out_nelem) {
  if (!c || !dims || !data || !out_dims || !out_data || nsteps < 0 || !(tau > 0))
    return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const double dt0 = c->P.dt;
  std::vector<double> u(size_t(nsteps) + 1, U);
  int rc = 0;
  if (c->hbm) {
    OcgParams G{};
    G.p = c->P.p;
    G.dt = tau;
    G.imag = 1;
    std::vector<double> gf, gb;
    ocg_host::gate_tables(G, c->J, gf, gb);
    rc = hb(c, hbm_swap_gates(c->hbm, 1, tau, gf, gb, G.glo, G.gsz, G.goff, G.gtotal));
    if (!rc) rc = ocg_steps(c, dims, data, u.data(), nsteps, 1, out_dims, out_data, out_cap, out_nelem);
    G.dt = dt0;
    G.imag = 0;
    ocg_host::gate_tables(G, c->J, gf, gb);
    const int rc2 = hbm_swap_gates(c->hbm, 0, dt0, gf, gb, G.glo, G.gsz, G.goff, G.gtotal);
    if (!rc && rc2) rc = hb(c, rc2);
    return rc;
  }
  c->P.dt = tau;
  c->P.imag = 1;
  rc = upload_gates(c);
  if (!rc) rc = ocg_steps(c, dims, data, u.data(), nsteps, 1, out_dims, out_data, out_cap, out_nelem);
  c->P.dt = dt0;
  c->P.imag = 0;
  const int rc2 = upload_gates(c);
  return rc ? rc : rc2;
}

static int launch_overlaps(ocg_ctx* c, const std::vector<int>& xs, const std::vector<int>& ys, int with_dH,
                           std::vector<zc>& out);

// InitializeState's whole tau schedule with the state resident on the device:
// per stage blocks of `block` imaginary-time steps until 1 - |<prev|new>| < tol
// (or max_steps), one device overlap per block, no host round trip.
int ocg_ground_state(ocg_ctx* c, const int* dims, const double* data, double U, int ntau, const double* taus,
                     int block, double tol, int max_steps, int* out_dims, double* out_data, size_t out_cap,
                     size_t* out_nelem, int* steps_done) {
  if (!c || !dims || !data || !out_dims || !out_data || ntau < 0 || (ntau > 0 && !taus) || block < 1 ||
      max_steps < 0)
    return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  for (int s = 0; s < ntau; ++s)
    if (!(taus[s] > 0)) return fail(c, OCG_EINVAL, "tau must be > 0");
  HIPCHK(c, hipSetDevice(c->device));
  const double dt0 = c->P.dt;
  if (c->hbm) {
    OcgParams G{};
    G.p = c->P.p;
    G.imag = 1;
    std::vector<std::vector<double>> gf(ntau), gb(ntau);
    for (int s = 0; s < ntau; ++s) {
      G.dt = taus[s];
      ocg_host::gate_tables(G, c->J, gf[s], gb[s]);
    }
    G.dt = dt0;
    G.imag = 0;
    std::vector<double> gf0, gb0;
    ocg_host::gate_tables(G, c->J, gf0, gb0);
    return hb(c, hbm_ground_state(c->hbm, dims, data, U, ntau, taus, gf, gb, G.glo, G.gsz, G.goff, G.gtotal, dt0,
                                  gf0, gb0, block, tol, max_steps, out_dims, out_data, out_cap, out_nelem, steps_done));
  }
  // LDS engine: the state in scratch slot 0, the block's starting state copied to slot 1
  const OcgParams& P = c->P;
  const int a = c->slot_tmp(0), b = c->slot_tmp(1);
  if (int rc = upload_mps(c, a, dims, data)) return rc;
  const std::vector<double> u(size_t(block) + 1, U);
  int done = 0, rc = 0;
  for (int s = 0; s < ntau && !rc; ++s) {
    c->P.dt = taus[s];
    c->P.imag = 1;
    if ((rc = upload_gates(c))) break;
    for (int d = 0; d < max_steps; d += block) {
      hipError_t e = hipMemcpyAsync(SLOT_D(c->pool, P, b), SLOT_D(c->pool, P, a), sizeof(int) * P.nsq,
                                    hipMemcpyDeviceToDevice, c->stream);
      if (e == hipSuccess)
        e = hipMemcpyAsync(SLOT_X(c->pool, P, b), SLOT_X(c->pool, P, a), sizeof(zc) * P.cap, hipMemcpyDeviceToDevice,
                           c->stream);
      if (e != hipSuccess) {
        rc = fail(c, OCG_EHIP, std::string("slot copy: ") + hipGetErrorString(e));
        break;
      }
      if ((rc = launch_steps(c, a, u.data(), block, 1))) break;
      done += block;
      std::vector<zc> ov;
      if ((rc = launch_overlaps(c, {b}, {a}, 0, ov))) break;
      if (1.0 - std::hypot(ov[0].x, ov[0].y) < tol) break;
    }
  }
  c->P.dt = dt0;
  c->P.imag = 0;
  const int rc2 = upload_gates(c);
  if (steps_done) *steps_done = done;
  if (rc || rc2) return rc ? rc : rc2;
  return download_mps(c, a, out_dims, out_data, out_cap, out_nelem);
}

int ocg_step_batch(ocg_ctx* c, int n, const int* dims, const double* const* data, const double* u_from,
                   const double* u_to, int forward, int* out_dims, double* const* out_data, const size_t* out_cap,
                   size_t* out_nelem) {
  if (!c || n < 0 || (n > 0 && (!dims || !data || !u_from || !u_to || !out_dims || !out_data || !out_cap)))
    return c ? fail(c, OCG_EINVAL, "null argument") : OCG_EINVAL;
  if (n == 0) return 0;
  if (c->hbm) {
    std::vector<double> uu(2 * size_t(n));
    std::vector<int> fw(n, forward);
    for (int i = 0; i < n; ++i) { uu[2 * i] = u_from[i]; uu[2 * i + 1] = u_to[i]; }
    return hb(c, hbm_steps(c->hbm, n, dims, data, uu.data(), 2, 1, fw.data(), out_dims, out_data, out_cap, out_nelem));
  }
  HIPCHK(c, hipSetDevice(c->device));
  const OcgParams& P = c->P;
  // scratch slots after the trajectory slots (their contents are left alone)
  const int base = 6 + 4 * c->N;
  if (int rc = ensure_slots(c, base + n)) return rc;
  std::vector<int> slots(n);
  std::vector<double> uu(2 * size_t(n));
  for (int i = 0; i < n; ++i) {
    slots[i] = base + i;
    if (int rc = upload_mps(c, slots[i], dims + size_t(i) * P.nsq, data[i])) return rc;
    uu[2 * i] = u_from[i];
    uu[2 * i + 1] = u_to[i];
  }
  if (int rc = ensure_buf(c, c->d_u, c->u_cap, 2 * n)) return rc;
  if (int rc = ensure_buf(c, c->d_idx, c->idx_cap, n)) return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_u, uu.data(), sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_idx, slots.data(), sizeof(int) * n, hipMemcpyHostToDevice, c->stream));
  if (int rc = begin_kernel(c)) return rc;
  const OcgParams Pa = c->Pa();  // the one-wave chain aliases the general LDS
  hipLaunchKernelGGL(k_steps, dim3(n), dim3(NT), Pa.lds_bytes, c->stream, Pa, c->d_gf, c->d_gb, c->d_md, c->pool,
                     c->d_idx, n, c->d_u, 2, 1, forward, c->d_stats + 4 * 3);
  if (int rc = end_kernel(c, 4)) return rc;
  for (int i = 0; i < n; ++i)
    if (int rc = download_mps(c, slots[i], out_dims + size_t(i) * P.nsq, out_data[i], out_cap[i],
                              out_nelem ? out_nelem + i : nullptr))
      return rc;
  return 0;
}

// n pairs <x|y> (with_dH: <x|dH|y>) of slot lists xs, ys (device) into out (device), on the
// context's stream: the padded contraction when the context has its plan, else Chain::overlap
static void ovl_pairs(ocg_ctx* c, const int* xs, const int* ys, int n, int with_dH, zc* out) {
  if (n <= 0) return;
  if (c->P.oplan) {
    hipLaunchKernelGGL(k_overlaps_pad, dim3(unsigned(n)), dim3(64), c->P.ovl_dh_bytes, c->stream, c->P, c->pool, xs,
                       ys, n, with_dH, out, c->d_stats + 1 * 3);
    return;
  }
  const OcgParams Po = c->Po();
  hipLaunchKernelGGL(k_overlaps, dim3(unsigned(n)), dim3(NT), Po.lds_bytes, c->stream, Po, c->d_gf, c->d_gb, c->d_md,
                     c->pool, xs, ys, n, with_dH, out, c->d_stats + 1 * 3);
}

static int launch_overlaps(ocg_ctx* c, const std::vector<int>& xs, const std::vector<int>& ys, int with_dH,
                           std::vector<zc>& out) {
  const OcgParams& P = c->P;
  int n = int(xs.size());
  if (n == 0) return 0;
  if (int rc = ensure_buf(c, c->d_idx, c->idx_cap, 2 * n)) return rc;
  if (int rc = ensure_buf(c, c->d_c, c->c_cap, n)) return rc;
  std::vector<int> idx(xs);
  idx.insert(idx.end(), ys.begin(), ys.end());
  HIPCHK(c, hipMemcpyAsync(c->d_idx, idx.data(), sizeof(int) * 2 * n, hipMemcpyHostToDevice, c->stream));
  if (int rc = begin_kernel(c)) return rc;
  ovl_pairs(c, c->d_idx, c->d_idx + n, n, with_dH, c->d_c);
  if (int rc = end_kernel(c, 1)) return rc;
  out.resize(n);
  HIPCHK(c, hipMemcpyAsync(out.data(), c->d_c, sizeof(zc) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

int ocg_overlap(ocg_ctx* c, const int* dims_x, const double* x, const int* dims_y, const double* y, int with_dH,
                double* out) {
  if (!c || !dims_x || !x || !dims_y || !y || !out) return c ? fail(c, OCG_EINVAL, "null argument") : OCG_EINVAL;
  if (c->hbm) return hb(c, hbm_overlap(c->hbm, dims_x, x, dims_y, y, with_dH, out));
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = upload_mps(c, c->slot_tmp(0), dims_x, x)) return rc;
  if (int rc = upload_mps(c, c->slot_tmp(1), dims_y, y)) return rc;
  std::vector<zc> r;
  if (int rc = launch_overlaps(c, {c->slot_tmp(0)}, {c->slot_tmp(1)}, with_dH, r)) return rc;
  out[0] = r[0].x;
  out[1] = r[0].y;
  return 0;
}

static int launch_apply_dH(ocg_ctx* c, const std::vector<int>& in, const std::vector<int>& outs, double* norms) {
  const OcgParams& P = c->P;
  int n = int(in.size());
  if (int rc = ensure_buf(c, c->d_idx, c->idx_cap, 2 * n)) return rc;
  if (norms)
    if (int rc = ensure_buf(c, c->d_norms, c->norms_cap, n)) return rc;
  std::vector<int> idx(in);
  idx.insert(idx.end(), outs.begin(), outs.end());
  HIPCHK(c, hipMemcpyAsync(c->d_idx, idx.data(), sizeof(int) * 2 * n, hipMemcpyHostToDevice, c->stream));
  if (int rc = begin_kernel(c)) return rc;
  const OcgParams Pn = c->Pn();
  hipLaunchKernelGGL(k_apply_dH, dim3(n), dim3(NT), Pn.lds_bytes, c->stream, Pn, c->d_gf, c->d_gb, c->d_md, c->pool,
                     c->d_idx, c->d_idx + n, n, norms ? c->d_norms : nullptr, c->d_stats + 2 * 3);
  if (int rc = end_kernel(c, 2)) return rc;
  if (norms) {
    HIPCHK(c, hipMemcpyAsync(norms, c->d_norms, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return 0;
}

int ocg_apply_dH(ocg_ctx* c, const int* dims, const double* data, int* out_dims, double* out_data, size_t out_cap,
                 size_t* out_nelem, double* norm) {
  if (!c || !dims || !data) return c ? fail(c, OCG_EINVAL, "null argument") : OCG_EINVAL;
  if (c->hbm) return hb(c, hbm_apply_dH(c->hbm, dims, data, out_dims, out_data, out_cap, out_nelem, norm));
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = upload_mps(c, c->slot_tmp(0), dims, data)) return rc;
  double nrm = 0;
  if (int rc = launch_apply_dH(c, {c->slot_tmp(0)}, {c->slot_tmp(1)}, &nrm)) return rc;
  if (norm) *norm = nrm;
  return download_mps(c, c->slot_tmp(1), out_dims, out_data, out_cap, out_nelem);
}

int ocg_set_states(ocg_ctx* c, const int* dims_target, const double* target, const int* dims_init,
                   const double* init) {
  if (!c || !dims_target || !target || !dims_init || !init) return c ? fail(c, OCG_EINVAL, "null argument") : OCG_EINVAL;
  c->u_psi.clear();
  c->u_xi.clear();
  if (c->hbm) return hb(c, hbm_set_states(c->hbm, dims_target, target, dims_init, init));
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = upload_mps(c, c->slot_target(), dims_target, target)) return rc;
  if (int rc = upload_mps(c, c->slot_init(), dims_init, init)) return rc;
  c->have_states = true;
  c->have_psi = c->have_xi = c->have_xih = false;
  return 0;
}

int ocg_propagate(ocg_ctx* c, const double* u, int N, int which) {
  if (!c || !u || N < 2 || which < 1 || which > 3) return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  if (which & 1) c->u_psi.clear();
  if (which & 2) c->u_xi.clear();
  if (c->hbm) {
    const int rc = hb(c, hbm_propagate(c->hbm, u, N, which));
    if (!rc) note_u(c, u, N, which);
    return rc;
  }
  if (!c->have_states) return fail(c, OCG_ESTATE, "ocg_set_states first");
  HIPCHK(c, hipSetDevice(c->device));
  const OcgParams& P = c->P;
  if (N != c->N) {
    c->N = N;
    c->have_psi = c->have_xi = c->have_xih = false;
  }
  if (int rc = ensure_slots(c, 6 + 4 * N)) return rc;
  if (int rc = ensure_buf(c, c->d_u, c->u_cap, N)) return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_u, u, sizeof(double) * N, hipMemcpyHostToDevice, c->stream));
  int grid = (which == 3) ? 2 : 1;
  if (int rc = begin_kernel(c)) return rc;
  const OcgParams Pa = c->Pa();  // the one-wave chain aliases the general LDS
  hipLaunchKernelGGL(k_trajectory, dim3(grid), dim3(NT), Pa.lds_bytes, c->stream, Pa, c->d_gf, c->d_gb, c->d_md,
                     c->pool, c->slot_init(), c->slot_target(), c->psi_base(), c->xi_base(), c->d_u, N, which,
                     c->d_stats + 0 * 3, 0);
  if (int rc = end_kernel(c, 0)) return rc;
  if (which & 1) { c->have_psi = true; c->have_xih = c->have_xih && (which & 2); }
  if (which & 2) { c->have_xi = true; c->have_xih = false; }
  note_u(c, u, N, which);
  return 0;
}

int ocg_gradient(ocg_ctx* c, const double* u, int N, double* divT, double* F) {
  if (!c || !u || !divT || !F || N < 2) return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  if (c->hbm) {
    // the stored trajectories when psi_t + xi_t + xiH_t fit half the free HBM (they
    // stay for eval_h's reuse), else psi || xi meeting in the middle (N states);
    // OCG_HBM_MID=1 / 0 forces either
    const char* e = std::getenv("OCG_HBM_MID");
    int mid = e ? std::atoi(e) : -1;
    if (mid < 0) {
      size_t fr = 0, tot = 0;
      HIPCHK(c, hipSetDevice(c->device));
      HIPCHK(c, hipMemGetInfo(&fr, &tot));
      mid = hbm_traj_bytes(c->hbm, N) > 0.5 * double(fr) ? 1 : 0;
    }
    if (mid == 1) {
      c->u_psi.clear();
      c->u_xi.clear();
      return hb(c, hbm_gradient_mid(c->hbm, u, N, divT, F));
    }
  }
  if (int rc = ocg_propagate(c, u, N, 3)) return rc;
  if (int rc = ocg_div_t(c, divT)) return rc;
  return ocg_overlap_factor(c, F);
}

int ocg_gradient_multi(ocg_ctx* c, int K, const double* u, int N, double* divT, double* F) {
  if (!c || !u || !divT || !F || N < 2 || K < 1) return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  if (size_t(K) * 4 * size_t(N) + 6 > size_t(INT32_MAX)) return fail(c, OCG_EINVAL, "K * N too large");
  if (c->hbm && K > 1) {
    // One batch of 2K chains when what it newly allocates fits half the free HBM,
    // else in turn.  The heap grows by copying into a new allocation while the
    // old one is live, so the whole new heap (the context's own 3N + 6 slots +
    // 2N per extra control) counts, plus the 2K chains; the extra slots are
    // given back after the call, also when it fails (hbm_gradient_multi).  A
    // batched call that still fails (allocation) falls back to the in-turn loop.
    size_t fr = 0, tot = 0;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemGetInfo(&fr, &tot));
    if (hbm_gradient_multi_bytes(c->hbm, K, N) <= 0.5 * double(fr)) {
      c->u_psi.clear();
      c->u_xi.clear();
      if (hb(c, hbm_gradient_multi(c->hbm, K, u, N, divT, F)) == 0) {
        note_u(c, u, N, 3);
        return 0;
      }
    }
  }
  // LDS engine: control k's psi / xi at slot stride 2N (psi_t, xi_t only; control
  // 1's psi_t takes control 0's xiH_t slots, which this call invalidates anyway).
  // The slot pool must fit half the free HBM, else the controls run in turn.
  bool lds_batch = !c->hbm && K > 1;
  if (lds_batch) {
    size_t fr = 0, tot = 0;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemGetInfo(&fr, &tot));
    const double need = (6.0 + 2.0 * N * K) * (sizeof(zc) * double(c->P.cap) + sizeof(int) * double(c->P.nsq));
    lds_batch = 6 + 2 * N * K <= c->nslots || need <= 0.5 * double(fr);  // growth copies: old + new live
  }
  if (!lds_batch) {  // controls in turn (last first: control 0's trajectories stay)
    for (int k = K - 1; k >= 0; --k) {
      if (int rc = ocg_propagate(c, u + size_t(k) * N, N, 3)) return rc;
      if (int rc = ocg_div_t(c, divT + size_t(k) * 2 * N)) return rc;
      if (int rc = ocg_overlap_factor(c, F + 2 * k)) return rc;
    }
    return 0;
  }
  if (!c->have_states) return fail(c, OCG_ESTATE, "ocg_set_states first");
  HIPCHK(c, hipSetDevice(c->device));
  const OcgParams& P = c->P;
  if (N != c->N) {
    c->N = N;
    c->have_psi = c->have_xi = c->have_xih = false;
  }
  c->u_psi.clear();
  c->u_xi.clear();
  const int cs = 2 * N;  // slot stride between controls: psi_t, xi_t
  if (int rc = ensure_slots(c, 6 + cs * K)) return rc;
  if (int rc = ensure_buf(c, c->d_u, c->u_cap, K * N)) return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_u, u, sizeof(double) * K * N, hipMemcpyHostToDevice, c->stream));
  if (int rc = begin_kernel(c)) return rc;
  const OcgParams Pa = c->Pa();  // the one-wave chain aliases the general LDS
  hipLaunchKernelGGL(k_trajectory, dim3(2 * K), dim3(NT), Pa.lds_bytes, c->stream, Pa, c->d_gf, c->d_gb, c->d_md,
                     c->pool, c->slot_init(), c->slot_target(), c->psi_base(), c->xi_base(), c->d_u, N, 3,
                     c->d_stats + 0 * 3, cs);
  if (int rc = end_kernel(c, 0)) return rc;
  c->have_psi = c->have_xi = true;
  c->have_xih = false;
  note_u(c, u, N, 3);  // control 0's trajectories stay in the context
  // divT of every control (<xi_i|dH|psi_i>, ocg_div_t's pairs), then every F (<psi_{N-1}|target>)
  std::vector<int> xs(size_t(K) * N), ys(size_t(K) * N);
  for (int k = 0; k < K; ++k)
    for (int i = 0; i < N; ++i) {
      xs[size_t(k) * N + i] = c->xi_base() + k * cs + i;
      ys[size_t(k) * N + i] = c->psi_base() + k * cs + i;
    }
  std::vector<zc> r;
  if (int rc = launch_overlaps(c, xs, ys, 1, r)) return rc;
  for (size_t e = 0; e < size_t(K) * N; ++e) { divT[2 * e] = r[e].x; divT[2 * e + 1] = r[e].y; }
  std::vector<int> fx(K), fy(K, c->slot_target());
  for (int k = 0; k < K; ++k) fx[k] = c->psi_base() + k * cs + N - 1;
  if (int rc = launch_overlaps(c, fx, fy, 0, r)) return rc;
  for (int k = 0; k < K; ++k) { F[2 * k] = r[k].x; F[2 * k + 1] = r[k].y; }
  return 0;
}

int ocg_overlap_factor(ocg_ctx* c, double* F) {
  if (!c || !F) return OCG_EINVAL;
  if (c->hbm) return hb(c, hbm_overlap_factor(c->hbm, F));
  if (!c->have_psi) return fail(c, OCG_ESTATE, "psi_t not propagated");
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<zc> r;
  // overlapC(psi_t.back(), psi_target) = <psi_T|target>
  if (int rc = launch_overlaps(c, {c->psi_base() + c->N - 1}, {c->slot_target()}, 0, r)) return rc;
  F[0] = r[0].x;
  F[1] = r[0].y;
  return 0;
}

int ocg_fidelities(ocg_ctx* c, double* fid) {
  if (!c || !fid) return OCG_EINVAL;
  if (c->hbm) return hb(c, hbm_fidelities(c->hbm, fid));
  if (!c->have_psi) return fail(c, OCG_ESTATE, "psi_t not propagated");
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<int> xs(c->N, c->slot_target()), ys(c->N);
  for (int i = 0; i < c->N; ++i) ys[i] = c->psi_base() + i;
  std::vector<zc> r;
  if (int rc = launch_overlaps(c, xs, ys, 0, r)) return rc;
  for (int i = 0; i < c->N; ++i) fid[i] = r[i].x * r[i].x + r[i].y * r[i].y;
  return 0;
}

int ocg_div_t(ocg_ctx* c, double* divT) {
  if (!c || !divT) return OCG_EINVAL;
  if (c->hbm) return hb(c, hbm_div_t(c->hbm, divT));
  if (!c->have_psi || !c->have_xi) return fail(c, OCG_ESTATE, "psi_t and xi_t must be propagated");
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<int> xs(c->N), ys(c->N);
  for (int i = 0; i < c->N; ++i) { xs[i] = c->xi_base() + i; ys[i] = c->psi_base() + i; }
  std::vector<zc> r;
  if (int rc = launch_overlaps(c, xs, ys, 1, r)) return rc;
  for (int i = 0; i < c->N; ++i) { divT[2 * i] = r[i].x; divT[2 * i + 1] = r[i].y; }
  return 0;
}

int ocg_xi_dH(ocg_ctx* c) {
  if (!c) return OCG_EINVAL;
  if (c->hbm) return hb(c, hbm_xi_dH(c->hbm));
  if (!c->have_xi) return fail(c, OCG_ESTATE, "xi_t not propagated");
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<int> in(c->N), outs(c->N);
  for (int i = 0; i < c->N; ++i) { in[i] = c->xi_base() + i; outs[i] = c->xih_base() + i; }
  if (int rc = launch_apply_dH(c, in, outs, nullptr)) return rc;
  c->have_xih = true;
  return 0;
}

int ocg_hessian_rows(ocg_ctx* c, const double* u, int N, const int* rows, int nrows, const double* F,
                     const double* divT, double* H) {
  if (!c || !u || !rows || !F || !divT || !H || nrows < 0) return c ? fail(c, OCG_EINVAL, "null argument") : OCG_EINVAL;
  if (c->hbm) {
    for (int r = 0; r < nrows; ++r)
      if (rows[r] < 1 || rows[r] > N - 2) return fail(c, OCG_EINVAL, "row index out of [1, N-2]");
    return hb(c, hbm_hessian_rows(c->hbm, u, N, rows, nrows, F, divT, H));
  }
  if (N != c->N || !c->have_psi || !c->have_xih) return fail(c, OCG_ESTATE, "propagate(3) + xi_dH first");
  for (int r = 0; r < nrows; ++r)
    if (rows[r] < 1 || rows[r] > N - 2) return fail(c, OCG_EINVAL, "row index out of [1, N-2]");
  if (nrows == 0) return 0;
  HIPCHK(c, hipSetDevice(c->device));
  const OcgParams& P = c->P;
  if (int rc = ensure_buf(c, c->d_idx, c->idx_cap, nrows)) return rc;
  if (int rc = ensure_buf(c, c->d_u, c->u_cap, N)) return rc;
  if (int rc = ensure_buf(c, c->d_c, c->c_cap, N)) return rc;
  size_t hn = size_t(N) * N;
  if (hn > c->H_cap) {
    if (c->d_H) (void)hipFree(c->d_H);
    HIPCHK(c, hipMalloc(&c->d_H, sizeof(double) * hn));
    c->H_cap = hn;
  }
  HIPCHK(c, hipMemcpyAsync(c->d_idx, rows, sizeof(int) * nrows, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_u, u, sizeof(double) * N, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_c, divT, sizeof(zc) * N, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_H, 0, sizeof(double) * hn, c->stream));
  // psiH_i = exactApplyMPO(propDeriv, psi_t[i]) and normiH for the requested rows
  {
    std::vector<int> in(nrows), outs(nrows);
    for (int r = 0; r < nrows; ++r) { in[r] = c->psi_base() + rows[r]; outs[r] = c->psih_base() + rows[r]; }
    if (int rc = ensure_buf(c, c->d_rnorm, c->rnorm_cap, N)) return rc;
    if (int rc = ensure_buf(c, c->d_idx2, c->idx2_cap, 2 * nrows)) return rc;
    in.insert(in.end(), outs.begin(), outs.end());
    HIPCHK(c, hipMemcpyAsync(c->d_idx2, in.data(), sizeof(int) * 2 * nrows, hipMemcpyHostToDevice, c->stream));
    if (int rc = begin_kernel(c)) return rc;
    const OcgParams Pn = c->Pn();
    hipLaunchKernelGGL(k_apply_dH, dim3(nrows), dim3(NT), Pn.lds_bytes, c->stream, Pn, c->d_gf, c->d_gb, c->d_md,
                       c->pool, c->d_idx2, c->d_idx2 + nrows, nrows, c->d_rnorm, c->d_stats + 2 * 3);
    if (int rc = end_kernel(c, 2)) return rc;
    // k_apply_dH writes norms[r] (row order); scatter to index i on the host side of the rows kernel
    std::vector<double> nr(nrows), ni(N, 0.0);
    HIPCHK(c, hipMemcpyAsync(nr.data(), c->d_rnorm, sizeof(double) * nrows, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int r = 0; r < nrows; ++r) ni[rows[r]] = nr[r];
    HIPCHK(c, hipMemcpyAsync(c->d_rnorm, ni.data(), sizeof(double) * N, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  zc f2 = mkz(F[0], F[1]);
  if (int rc = begin_kernel(c)) return rc;
  hipLaunchKernelGGL(k_hessian_rows, dim3(nrows), dim3(NT), P.lds_bytes, c->stream, P, c->d_gf, c->d_gb, c->d_md,
                     c->pool, c->psih_base(), c->xih_base(), c->d_idx, nrows, c->d_rnorm, c->d_u, N, c->d_c, f2,
                     c->d_H, c->d_stats + 3 * 3);
  if (int rc = end_kernel(c, 3)) return rc;
  std::vector<double> h(hn);
  HIPCHK(c, hipMemcpyAsync(h.data(), c->d_H, sizeof(double) * hn, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // entries of the requested rows and their mirrors (disjoint per row)
  for (int r = 0; r < nrows; ++r) {
    int i = rows[r];
    for (int j = i; j + 1 < N; ++j) {
      H[size_t(i) * N + j] = h[size_t(i) * N + j];
      H[size_t(j) * N + i] = h[size_t(j) * N + i];
    }
  }
  return 0;
}

// getHessian's fidelity part from the separate entry points (calcPsiXiDivT,
// xiHlist, calcHessianRow over all rows: src/OptimalControl.cpp:281-338)
// When the device psi_t / xi_t already belong to u (a Hessian at the control
// of the last gradient: BH_nlp::eval_h after eval_grad_f, src/BH_nlp.cpp:189,
// whose getHessian always passes new_control = true) they, and xiHlist if
// present, are reused: the same states, so the same Hessian bit for bit.
static int hessian_unfused(ocg_ctx* c, const double* u, int N, const int* rows, int nrows, double* H, double* divT,
                           double* F) {
  const bool have_psi = c->hbm ? hbm_have(c->hbm, 1) : c->have_psi;
  const bool have_xi = c->hbm ? hbm_have(c->hbm, 2) : c->have_xi;
  const bool reuse = have_psi && have_xi && same_u(c->u_psi, u, N) && same_u(c->u_xi, u, N);
  if (!reuse)
    if (int rc = ocg_propagate(c, u, N, 3)) return rc;
  if (int rc = ocg_div_t(c, divT)) return rc;
  if (int rc = ocg_overlap_factor(c, F)) return rc;
  const bool have_xih = c->hbm ? hbm_have(c->hbm, 3) : c->have_xih;
  if (!(reuse && have_xih))
    if (int rc = ocg_xi_dH(c)) return rc;
  return ocg_hessian_rows(c, u, N, rows, nrows, F, divT, H);
}

static int hessian_fused(ocg_ctx* c, int K, const double* u, int N, const int* rows, int nrows, double* H,
                         double* divT, double* F);

int ocg_hessian(ocg_ctx* c, const double* u, int N, const int* rows, int nrows, double* H, double* divT,
                double* F) {
  if (!c || !u || !H || !divT || !F || (nrows > 0 && !rows) || nrows < 0 || N < 4)
    return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  if (c->hbm) {
    for (int r = 0; r < nrows; ++r)
      if (rows[r] < 1 || rows[r] > N - 2) return fail(c, OCG_EINVAL, "row index out of [1, N-2]");
    // trajectory checkpointing when psi_t + xi_t + xiH_t would not fit half of
    // the free HBM (config 5: ~600 GB at N_t = 1001), or when OCG_HBM_CKPT=K asks
    // for it (segment length K; tests, A/B)
    int K = 0;
    if (const char* e = std::getenv("OCG_HBM_CKPT")) K = std::atoi(e);
    if (K <= 0) {
      size_t fr = 0, tot = 0;
      HIPCHK(c, hipSetDevice(c->device));
      HIPCHK(c, hipMemGetInfo(&fr, &tot));
      if (hbm_traj_bytes(c->hbm, N) > 0.5 * double(fr)) K = std::max(1, int(std::ceil(std::sqrt(double(N)))));
    }
    if (K > 0) {
      c->u_psi.clear();
      c->u_xi.clear();
      const int rc = hb(c, hbm_hessian_ckpt(c->hbm, u, N, rows, nrows, H, divT, F, K));
      if (rc == 0) {
        ++c->ckpt_runs;
        c->ckpt_k = K;
      }
      return rc;
    }
    // pipelined (psi + rows || dH || xi on three streams) when the row states fit
    // half the free HBM and the trajectories of u are not already on the device
    // (BH_nlp::eval_h after eval_grad_f reuses them); OCG_HBM_PIPE=0 turns it off
    const char* pe = std::getenv("OCG_HBM_PIPE");
    const int pipe_env = pe ? std::atoi(pe) : -1;
    const bool reuse = hbm_have(c->hbm, 1) && hbm_have(c->hbm, 2) && same_u(c->u_psi, u, N) && same_u(c->u_xi, u, N);
    if (pipe_env != 0 && !reuse && nrows > 0) {
      size_t fr = 0, tot = 0;
      HIPCHK(c, hipMemGetInfo(&fr, &tot));
      if (pipe_env == 1 || hbm_pipe_bytes(c->hbm, N, rows, nrows) <= 0.5 * double(fr)) {
        c->u_psi.clear();
        c->u_xi.clear();
        const int rc = hb(c, hbm_hessian_pipe(c->hbm, u, N, rows, nrows, H, divT, F));
        if (rc == 0) {
          ++c->pipe_runs;
          note_u(c, u, N, 3);
          return 0;
        }
        // Only a pipeline that ran out of memory (a worker's pools or arenas
        // beyond the estimate) is retried, and only when the pipeline was not
        // asked for explicitly: it has given back everything it grew, and the
        // two-phase path writes the same entries of H.  Any other failure is the
        // call's status.
        if (rc != OCG_ENOMEM || pipe_env == 1) return rc;
        ++c->pipe_fallbacks;
        const int rc2 = hessian_unfused(c, u, N, rows, nrows, H, divT, F);
        if (rc2 == 0) c->err.clear();
        return rc2;
      }
    }
    return hessian_unfused(c, u, N, rows, nrows, H, divT, F);
  }
  return hessian_fused(c, 1, u, N, rows, nrows, H, divT, F);
}

// The fused LDS-engine getHessian for K control vectors in one k_pipeline launch
// (K = 1: ocg_hessian).  Control k's trajectories use the slots k * cs after
// control 0's (cs = 4N), its flags the k-th block of 2N + 2, its row states
// the k-th block of total; the context keeps control 0's trajectories.
static int hessian_fused(ocg_ctx* c, int K, const double* u, int N, const int* rows, int nrows, double* H,
                         double* divT, double* F) {
  if (!c->have_states) return fail(c, OCG_ESTATE, "ocg_set_states first");
  for (int r = 0; r < nrows; ++r)
    if (rows[r] < 1 || rows[r] > N - 2) return fail(c, OCG_EINVAL, "row index out of [1, N-2]");
  HIPCHK(c, hipSetDevice(c->device));
  const OcgParams& P = c->P;
  if (N != c->N) {
    c->N = N;
    c->have_psi = c->have_xi = c->have_xih = false;
  }
  const int cs = 4 * N;  // slot stride between controls
  if (int rc = ensure_slots(c, 6 + cs * K)) return rc;
  if (int rc = ensure_buf(c, c->d_u, c->u_cap, K * N)) return rc;
  if (int rc = ensure_buf(c, c->d_pc, c->pc_cap, K * (N + 1))) return rc;
  if (int rc = ensure_buf(c, c->d_rows, c->rows_cap, 2 * nrows + 2)) return rc;
  if (int rc = ensure_buf(c, c->d_prn, c->prn_cap, K * nrows + 1)) return rc;
  const int nflags = K * (2 * N + 2) + 1;  // K blocks (psi / xi flags, progress, spare) + the ticket counter
  if (nflags > c->flags_cap) {
    if (c->d_flags) (void)hipFree(c->d_flags);
    c->d_flags = nullptr;
    c->flags_cap = 0;
    if (int rc = ensure_buf(c, c->d_flags, c->flags_cap, nflags)) return rc;
    c->flags_N = -1;
  }
  // Publication flags hold epochs; each control's progress counter and the
  // ticket counter share the buffer at positions that depend on (N, K).  When
  // the layout changes, a stale counter could sit where a flag now lives and
  // read as already published, so the whole prefix restarts at 0 (< any epoch).
  if (c->flags_N != N || c->flags_K != K) {
    HIPCHK(c, hipMemsetAsync(c->d_flags, 0, sizeof(int) * c->flags_cap, c->stream));
    c->epoch = 0;
    c->flags_N = N;
    c->flags_K = K;
  }
  // stored row states: row i keeps psiH_i(j), j = i..N-2 (O(N^2) states).
  // Past the memory budget (or int offsets) the unfused path runs instead:
  // same arithmetic per row (test_fused_equals_unfused_bitwise), O(N) states.
  size_t total = 0;
  for (int r = 0; r < nrows; ++r) total += size_t(N - 1 - rows[r]);
  {
    static const double budget_mb = [] {
      const char* e = std::getenv("OCG_RS_BUDGET_MB");
      return e ? std::atof(e) : 16384.0;
    }();
    const double need = double(K) * double(total) * (sizeof(zc) * double(P.cap) + sizeof(int) * double(P.nsq));
    if (size_t(K) * total > size_t(INT32_MAX / 2) || need > budget_mb * 1048576.0) {
      for (int k = 0; k < K; ++k) {  // controls one after another (last first: control 0's trajectories stay)
        const int kk = K - 1 - k;
        if (int rc = hessian_unfused(c, u + size_t(kk) * N, N, rows, nrows, H + size_t(kk) * N * N,
                                     divT + size_t(kk) * 2 * N, F + 2 * kk))
          return rc;
      }
      return 0;
    }
  }
  std::vector<int> rb(2 * nrows + 1);  // rows[0..nrows) then rbase[0..nrows]
  total = 0;
  for (int r = 0; r < nrows; ++r) rb[r] = rows[r];
  for (int r = 0; r < nrows; ++r) {
    rb[nrows + r] = int(total);
    total += size_t(N - 1 - rows[r]);
  }
  rb[2 * nrows] = int(total);
  if (size_t(K) * total > c->rs_cap) {
    if (c->rs.dims) (void)hipFree(c->rs.dims);
    if (c->rs.data) (void)hipFree(c->rs.data);
    c->rs = Pool{nullptr, nullptr};
    c->rs_cap = 0;
    HIPCHK(c, hipMalloc(&c->rs.dims, sizeof(int) * K * total * P.nsq));
    HIPCHK(c, hipMalloc(&c->rs.data, sizeof(zc) * K * total * P.cap));
    c->rs_cap = size_t(K) * total;
  }
  size_t hn = size_t(K) * N * N;
  if (hn > c->H_cap) {
    if (c->d_H) (void)hipFree(c->d_H);
    HIPCHK(c, hipMalloc(&c->d_H, sizeof(double) * hn));
    c->H_cap = hn;
  }
  const int epoch = ++c->epoch;
  // pinned staging: [u | row table | pair lists] uploaded, [err | divT, F | H]
  // downloaded, all as DMA copies (pageable copies are staged and block)
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t nidx = 2 * size_t(K) * N + 2 * K;
  const size_t o_rb = al(sizeof(double) * K * N), o_idx = o_rb + al(sizeof(int) * rb.size());
  const size_t o_err = o_idx + al(sizeof(int) * nidx), o_pc = o_err + 256;
  const size_t o_h = o_pc + al(sizeof(zc) * K * (N + 1)), pin_bytes = o_h + sizeof(double) * hn;
  if (int rc = ensure_pin(c, pin_bytes)) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // no copy of an earlier (failed) call still reads the staging
  std::memcpy(c->h_pin, u, sizeof(double) * K * N);
  std::memcpy(c->h_pin + o_rb, rb.data(), sizeof(int) * rb.size());
  HIPCHK(c, hipMemcpyAsync(c->d_u, c->h_pin, sizeof(double) * K * N, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_rows, c->h_pin + o_rb, sizeof(int) * rb.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_H, 0, sizeof(double) * hn, c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_flags + K * (2 * N + 2), 0, sizeof(int), c->stream));  // role tickets
  const int* d_rows = c->d_rows;
  const int* d_rbase = c->d_rows + nrows;
  // divT_i = <xi_i|dH|psi_i> and F = <psi_{N-1}|target> pair lists
  // K N dH pairs (xs then ys), then K F pairs (xs then ys)
  int* idx = (int*)(c->h_pin + o_idx);
  for (int k = 0; k < K; ++k) {
    for (int i = 0; i < N; ++i) {
      idx[k * N + i] = c->xi_base() + k * cs + i;
      idx[K * N + k * N + i] = c->psi_base() + k * cs + i;
    }
    idx[2 * K * N + k] = c->psi_base() + k * cs + N - 1;
    idx[2 * K * N + K + k] = c->slot_target();
  }
  if (int rc = ensure_buf(c, c->d_idx, c->idx_cap, int(nidx))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_idx, idx, sizeof(int) * nidx, hipMemcpyHostToDevice, c->stream));
  // the three launches back to back, one host synchronisation at the end;
  // the phase marks give the per-kernel times (ocg_kernel_stats kinds 5, 1, 6)
  HIPCHK(c, hipEventRecord(c->evh[0], c->stream));
  // xiH workers: the xi chain publishes one state per step and one dH
  // application costs about one step, so a few workers keep up
  static const int xiw = [] {  // A/B: OCG_XIH_WORKERS
    const char* e = std::getenv("OCG_XIH_WORKERS");
    const int v = e ? std::atoi(e) : kXiHWorkers;
    return v > 0 ? v : kXiHWorkers;
  }();
  const int nxw = std::min(N, xiw);
  // many controls: chain workgroups sized for two per CU (smaller plan slots; plans are
  // bitwise-neutral) — measured 37.3k vs 33.0k rows/s at K = 8, slower below (OCG_MULTI_SHARE_K)
  static const int share_k = [] {
    const char* e = std::getenv("OCG_MULTI_SHARE_K");
    return e ? std::atoi(e) : 8;
  }();
  const OcgParams Pl = (share_k > 0 && K >= share_k) ? c->P2() : c->Pa();
  hipLaunchKernelGGL(k_pipeline, dim3(K * (2 + nxw + nrows)), dim3(NT), Pl.lds_bytes, c->stream, Pl, c->d_gf,
                     c->d_gb, c->d_md, c->pool, c->slot_init(), c->slot_target(), c->psi_base(), c->xi_base(),
                     c->xih_base(), c->d_u, N, d_rows, nrows, d_rbase, c->rs, c->d_prn, c->d_flags, epoch, c->d_err,
                     nxw, c->d_stats + 5 * 3, K, cs);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->evh[1], c->stream));
  const OcgParams Po = c->Po();
  // divT of every control at d_pc[k N + i], F of control k at d_pc[K N + k]
  ovl_pairs(c, c->d_idx, c->d_idx + K * N, K * N, 1, c->d_pc);
  ovl_pairs(c, c->d_idx + 2 * K * N, c->d_idx + 2 * K * N + K, K, 0, c->d_pc + K * N);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->evh[2], c->stream));
  static const int rov_w = [] {  // A/B switch: OCG_ROWOV_WAVE=0 -> two-wave row overlaps
    const char* e = std::getenv("OCG_ROWOV_WAVE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  // Row overlaps: exactly one resident wave of workgroups, every CU full (CUs x
  // workgroups the LDS admits per CU), each taking pairs grid-stride, so the
  // pairs are dealt evenly and none waits for a second dispatch round
  // (config 1: 1536 = 256 x 6 -> 0.428 ms, against 0.496 at 4096, 0.584 at
  // 1024, 0.640 at 1792, 0.818 one per pair); OCG_ROWOV_GRID overrides
  static const int rov_env = [] {
    const char* e = std::getenv("OCG_ROWOV_GRID");
    return e ? std::atoi(e) : -1;
  }();
  int rov_grid = rov_env;
  if (rov_grid < 0) {
    int ncu = 0, lds_cu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
    (void)hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, c->device);
    const int per = (Po.lds_bytes > 0 && lds_cu > 0) ? std::max(1, lds_cu / Po.lds_bytes) : 6;
    rov_grid = std::max(1, ncu) * std::min(per, 16);
  }
  const size_t ktotal = size_t(K) * total;
  const int rgrid = (rov_grid > 0 && size_t(rov_grid) < ktotal) ? rov_grid : int(ktotal);
  if (total > 0 && c->P.oplan) {
    // the padded overlap: one wave and ~12 KB per workgroup, so up to 16 per CU
    int ncu = 0, lds_cu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
    (void)hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, c->device);
    const int pb = c->P.ovl_bytes + 4 * (2 * nrows + 1);  // + the row table (kernels.hpp)
    const int per = lds_cu > 0 ? std::max(1, lds_cu / pb) : 8;
    const size_t pg = rov_env > 0 ? size_t(rov_env) : size_t(std::max(1, ncu)) * std::min(per, 16);
    const int pgrid = int(std::min(pg, ktotal));
    if (pb > 65536) HIPCHK(c, hipFuncSetAttribute((const void*)k_row_overlaps_pad,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, pb));
    hipLaunchKernelGGL(k_row_overlaps_pad, dim3(unsigned(pgrid)), dim3(64), pb, c->stream, c->P,
                       c->pool, c->xih_base(), d_rows, nrows, d_rbase, c->rs, c->d_prn, c->d_pc, c->d_pc + K * N, N,
                       c->d_H, c->d_stats + 6 * 3, K, cs);
  } else if (total > 0 && rov_w)
    hipLaunchKernelGGL(k_row_overlaps_w, dim3(unsigned(rgrid)), dim3(64), Po.lds_bytes, c->stream, Po, c->d_gf,
                       c->d_gb, c->d_md, c->pool, c->xih_base(), d_rows, nrows, d_rbase, c->rs, c->d_prn, c->d_pc,
                       c->d_pc + K * N, N, c->d_H, c->d_stats + 6 * 3, K, cs);
  else if (total > 0)
    hipLaunchKernelGGL(k_row_overlaps, dim3(unsigned(rgrid)), dim3(NT), Po.lds_bytes, c->stream, Po, c->d_gf,
                       c->d_gb, c->d_md, c->pool, c->xih_base(), d_rows, nrows, d_rbase, c->rs, c->d_prn, c->d_pc,
                       c->d_pc + K * N, N, c->d_H, c->d_stats + 6 * 3, K, cs);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->evh[3], c->stream));
  const zc* pc = (const zc*)(c->h_pin + o_pc);
  const double* h = (const double*)(c->h_pin + o_h);
  HIPCHK(c, hipMemcpyAsync(c->h_pin + o_err, c->d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->h_pin + o_pc, c->d_pc, sizeof(zc) * K * (N + 1), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->h_pin + o_h, c->d_H, sizeof(double) * hn, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int err = *(const int*)(c->h_pin + o_err);
  const int kinds[3] = {5, 1, 6};
  for (int k = 0; k < 3; ++k) {
    if (k == 2 && total == 0) break;
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, c->evh[k], c->evh[k + 1]));
    c->kst[kinds[k]].ms += ms;
    c->kst[kinds[k]].launches += 1;
  }
  if (err) {
    c->have_psi = c->have_xi = c->have_xih = false;
    HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return fail(c, OCG_ENUM, std::string((err & OCG_ERR_WATCHDOG) ? "pipeline watchdog: a consumer saw no producer "
                                                                    "progress for ~15 s; " : "") +
                                 ((err & OCG_ERR_JACOBI) ? "eigensolver did not converge within its sweep cap" : ""));
  }
  c->have_psi = c->have_xi = c->have_xih = true;
  note_u(c, u, N, 3);  // control 0's trajectories stay in the context
  for (int k = 0; k < K; ++k) {
    double* Hk = H + size_t(k) * N * N;
    const double* hk = h + size_t(k) * N * N;
    for (int i = 0; i < N; ++i) {
      divT[2 * (size_t(k) * N + i)] = pc[size_t(k) * N + i].x;
      divT[2 * (size_t(k) * N + i) + 1] = pc[size_t(k) * N + i].y;
    }
    F[2 * k] = pc[size_t(K) * N + k].x;
    F[2 * k + 1] = pc[size_t(K) * N + k].y;
    for (int r = 0; r < nrows; ++r) {
      const int i = rows[r];
      for (int j = i; j + 1 < N; ++j) {
        Hk[size_t(i) * N + j] = hk[size_t(i) * N + j];
        Hk[size_t(j) * N + i] = hk[size_t(j) * N + i];
      }
    }
  }
  return 0;
}

int ocg_hessian_multi(ocg_ctx* c, int K, const double* u, int N, const int* rows, int nrows, double* H,
                      double* divT, double* F) {
  if (!c || !u || !H || !divT || !F || (nrows > 0 && !rows) || nrows < 0 || N < 4 || K < 1)
    return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  if (size_t(K) * 4 * size_t(N) + 6 > size_t(INT32_MAX) || size_t(K) * N * N > (size_t(1) << 40))
    return fail(c, OCG_EINVAL, "K * N too large");
  if (c->hbm || K == 1) {  // HBM engine: its row batches already fill the device; controls in turn
    for (int k = K - 1; k >= 0; --k)
      if (int rc = ocg_hessian(c, u + size_t(k) * N, N, rows, nrows, H + size_t(k) * N * N, divT + size_t(k) * 2 * N,
                               F + 2 * k))
        return rc;
    return 0;
  }
  for (int r = 0; r < nrows; ++r)
    if (rows[r] < 1 || rows[r] > N - 2) return fail(c, OCG_EINVAL, "row index out of [1, N-2]");
  return hessian_fused(c, K, u, N, rows, nrows, H, divT, F);
}

int ocg_convert_hessian(ocg_ctx* c, const double* Hu, int N, const double* V, int M, double* Hc) {
  if (!c || !Hu || !V || !Hc || N < 1 || M < 1) return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t nn = size_t(N) * N, mn = size_t(M) * N, need = nn + 3 * mn + size_t(M) * M;
  if (need > c->proj_cap) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->d_proj) (void)hipFree(c->d_proj);
    c->d_proj = nullptr;
    c->proj_cap = 0;
    HIPCHK(c, hipMalloc(&c->d_proj, sizeof(double) * need));
    c->proj_cap = need;
  }
  double *dH = c->d_proj, *dV = dH + nn, *dVt = dV + mn, *dHV = dVt + mn, *dHc = dHV + mn;
  std::vector<double> vt(mn);
  for (int j = 0; j < M; ++j)
    for (int l = 0; l < N; ++l) vt[size_t(l) * M + j] = V[size_t(j) * N + l];
  HIPCHK(c, hipMemcpyAsync(dH, Hu, sizeof(double) * nn, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dV, V, sizeof(double) * mn, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dVt, vt.data(), sizeof(double) * mn, hipMemcpyHostToDevice, c->stream));
  const int bt = std::min(256, ((M + 63) / 64) * 64);
  hipLaunchKernelGGL(k_project_hv, dim3(N), dim3(bt), sizeof(double) * N, c->stream, dH, dVt, N, M, dHV);
  hipLaunchKernelGGL(k_project_c, dim3((M * M + 255) / 256), dim3(256), 0, c->stream, dV, dHV, N, M, dHc);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(Hc, dHc, sizeof(double) * M * M, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

int ocg_denmat_decomp(ocg_ctx* c, int nm, const int* rows, const int* cols, const double* const* M, double cutoff,
                      int maxm, int* kept, double* const* w, double* const* A, double* const* B) {
  if (!c || nm < 0 || (nm > 0 && (!rows || !cols || !M || !kept)))
    return c ? fail(c, OCG_EINVAL, "bad argument") : OCG_EINVAL;
  if (!c->hbm) return fail(c, OCG_EINVAL, "ocg_denmat_decomp: HBM engine contexts only (ocg_create_ex engine 2)");
  if (nm == 0) return 0;
  return hb(c, hbm_denmat_decomp(c->hbm, nm, rows, cols, M, cutoff, maxm, kept, w, A, B));
}

int ocg_get_state(ocg_ctx* c, int which, int t, int* dims, double* data, size_t cap, size_t* nelem) {
  if (!c || !dims || !data) return OCG_EINVAL;
  if (c->hbm) return hb(c, hbm_get_state(c->hbm, which, t, dims, data, cap, nelem));
  if (t < 0 || t >= c->N) return fail(c, OCG_EINVAL, "t out of range");
  bool ok = (which == 0 && c->have_psi) || (which == 1 && c->have_xi) || (which == 2 && c->have_xih);
  if (!ok) return fail(c, OCG_ESTATE, "requested trajectory not available");
  HIPCHK(c, hipSetDevice(c->device));
  int base = which == 0 ? c->psi_base() : (which == 1 ? c->xi_base() : c->xih_base());
  return download_mps(c, base + t, dims, data, cap, nelem);
}

int ocg_kernel_stats(ocg_ctx* c, int kind, double* total_ms, long* launches, double* alg_bytes, double* alg_flops,
                     long* sweep_steps) {
  if (!c || kind < 0 || kind > 8) return OCG_EINVAL;
  if (kind == 8) {  // getHessian path counters (HBM engine; zeros on the LDS engine)
    if (total_ms) *total_ms = 0;
    if (launches) *launches = c->pipe_runs;
    if (alg_bytes) *alg_bytes = double(c->ckpt_k);
    if (alg_flops) *alg_flops = double(c->ckpt_runs);
    if (sweep_steps) *sweep_steps = c->pipe_fallbacks;
    return 0;
  }
  if (c->hbm) return hb(c, hbm_stats(c->hbm, kind, total_ms, launches, alg_bytes, alg_flops, sweep_steps));
  if (kind == 7) {  // the MFMA contraction kernel exists only in the HBM engine
    if (total_ms) *total_ms = 0;
    if (launches) *launches = 0;
    if (alg_bytes) *alg_bytes = 0;
    if (alg_flops) *alg_flops = 0;
    if (sweep_steps) *sweep_steps = 0;
    return 0;
  }
  HIPCHK(c, hipSetDevice(c->device));
  double s[3];
  HIPCHK(c, hipMemcpyAsync(s, c->d_stats + 3 * kind, sizeof(s), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (total_ms) *total_ms = c->kst[kind].ms;
  if (launches) *launches = c->kst[kind].launches;
  if (alg_bytes) *alg_bytes = s[0];
  if (alg_flops) *alg_flops = s[1];
  if (sweep_steps) *sweep_steps = long(s[2] + 0.5);
  return 0;
}

// diagnostic: per-phase shader-clock cycles summed over workgroups (only in
// a -DOCG_PROFILE build; zeros otherwise).  reset != 0 clears afterwards.
int ocg_profile(ocg_ctx* c, double* out32, int reset) {
  if (!c || !out32) return OCG_EINVAL;
#ifdef OCG_PROFILE
  HIPCHK(c, hipMemcpyFromSymbol(out32, HIP_SYMBOL(ocg::g_ocg_prof), sizeof(double) * 32));
  if (reset) {
    std::vector<double> z(32, 0.0);
    HIPCHK(c, hipMemcpyToSymbol(HIP_SYMBOL(ocg::g_ocg_prof), z.data(), sizeof(double) * 32));
  }
#else
  (void)reset;
  for (int i = 0; i < 32; ++i) out32[i] = 0.0;
#endif
  return 0;
}

int ocg_reset_stats(ocg_ctx* c) {
  if (!c) return OCG_EINVAL;
  c->pipe_runs = c->pipe_fallbacks = c->ckpt_runs = c->ckpt_k = 0;
  if (c->hbm) {
    hbm_reset_stats(c->hbm);
    return 0;
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemsetAsync(c->d_stats, 0, sizeof(double) * 24, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (auto& k : c->kst) k = KStat{};
  return 0;
}

}  // extern "C"
