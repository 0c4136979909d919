// ORACLE — TEST INFRASTRUCTURE ONLY (see tdmrg_oracle.hpp header).
// C-ABI over the CPU restatement so pytest (ctypes) and bench.py's
// cpu_baseline leg can drive it.  Never linked by the product.
#include <chrono>
#include <cstring>
#include <memory>

#include "tdmrg_oracle.hpp"

using namespace oracle;

struct OrcCtx {
  Stepper st;
};
struct OrcOC {
  std::unique_ptr<OC> oc;
};

static int copy_out(const MPS& m, int* fd, double* data, size_t cap, size_t* nelem) {
  std::vector<int> f;
  std::vector<double> d;
  m.to_flat(f, d);
  if (nelem) *nelem = d.size() / 2;
  if (d.size() / 2 > cap) return 2;
  std::memcpy(fd, f.data(), f.size() * sizeof(int));
  std::memcpy(data, d.data(), d.size() * sizeof(double));
  return 0;
}

extern "C" {

void* orc_new(int L, int p, int Q, double J, double dt, double cutoff, int maxm) {
  return new OrcCtx{Stepper(L, p, Q, J, dt, cutoff, maxm)};
}
void orc_free(void* h) { delete static_cast<OrcCtx*>(h); }

int orc_gate(void* h, int forward, double* out /* 2*p^4 */) {
  auto* c = static_cast<OrcCtx*>(h);
  const auto& G = forward ? c->st.Gf : c->st.Gb;
  for (size_t i = 0; i < G.size(); ++i) { out[2 * i] = G[i].real(); out[2 * i + 1] = G[i].imag(); }
  return 0;
}

int orc_step(void* h, const int* fd, const double* data, double from, double to, int forward,
             int* out_fd, double* out_data, size_t cap, size_t* nelem) {
  auto* c = static_cast<OrcCtx*>(h);
  MPS m = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fd, data);
  c->st.step(m, from, to, forward != 0);
  return copy_out(m, out_fd, out_data, cap, nelem);
}

int orc_steps(void* h, const int* fd, const double* data, const double* u, int nsteps, int forward,
              int* out_fd, double* out_data, size_t cap, size_t* nelem) {
  auto* c = static_cast<OrcCtx*>(h);
  MPS m = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fd, data);
  for (int i = 0; i < nsteps; ++i) c->st.step(m, u[i], u[i + 1], forward != 0);
  return copy_out(m, out_fd, out_data, cap, nelem);
}

int orc_overlap(void* h, const int* fdx, const double* dx, const int* fdy, const double* dy, double* out) {
  auto* c = static_cast<OrcCtx*>(h);
  MPS X = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fdx, dx);
  MPS Y = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fdy, dy);
  cplx z = overlapC(X, Y);
  out[0] = z.real(); out[1] = z.imag();
  return 0;
}

int orc_overlap_dH(void* h, const int* fdx, const double* dx, const int* fdy, const double* dy, double* out) {
  auto* c = static_cast<OrcCtx*>(h);
  MPS X = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fdx, dx);
  MPS Y = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fdy, dy);
  cplx z = overlapC_diag(X, c->st.dH, Y);
  out[0] = z.real(); out[1] = z.imag();
  return 0;
}

int orc_apply_dH(void* h, const int* fd, const double* data, int* out_fd, double* out_data, size_t cap,
                 size_t* nelem) {
  auto* c = static_cast<OrcCtx*>(h);
  MPS m = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fd, data);
  MPS r = c->st.apply_dH(m);
  return copy_out(r, out_fd, out_data, cap, nelem);
}

int orc_heev(int n, const double* a /* 2 n^2 */, double* w, double* v /* 2 n^2 */) {
  std::vector<cplx> A(size_t(n) * n);
  for (size_t i = 0; i < A.size(); ++i) A[i] = cplx(a[2 * i], a[2 * i + 1]);
  std::vector<double> ww;
  std::vector<cplx> V;
  heev_jacobi(n, A, ww, V);
  for (int i = 0; i < n; ++i) w[i] = ww[i];
  for (size_t i = 0; i < V.size(); ++i) { v[2 * i] = V[i].real(); v[2 * i + 1] = V[i].imag(); }
  return 0;
}
// the Householder + QL solver (ORC_HEEV=ql) on its own, for its tests
int orc_heev_ql(int n, const double* a /* 2 n^2 */, double* w, double* v /* 2 n^2 */) {
  std::vector<cplx> A(size_t(n) * n);
  for (size_t i = 0; i < A.size(); ++i) A[i] = cplx(a[2 * i], a[2 * i + 1]);
  std::vector<double> ww;
  std::vector<cplx> V;
  heev_ql(n, A, ww, V);
  for (int i = 0; i < n; ++i) w[i] = ww[i];
  for (size_t i = 0; i < V.size(); ++i) { v[2 * i] = V[i].real(); v[2 * i + 1] = V[i].imag(); }
  return 0;
}

int orc_truncate(const double* P, int n, double cutoff, int maxm) {
  return truncate_count(std::vector<double>(P, P + n), cutoff, maxm, 1);
}

// ---------------------------------------------------------------- OC level
void* orc_oc_new(void* h, const int* fdt, const double* dt_, const int* fdi, const double* di, int N,
                 double gamma) {
  auto* c = static_cast<OrcCtx*>(h);
  MPS T = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fdt, dt_);
  MPS I = MPS::from_flat(c->st.L, c->st.p, c->st.Q, fdi, di);
  auto* o = new OrcOC;
  o->oc.reset(new OC(c->st, T, I, size_t(N), gamma));
  return o;
}
void orc_oc_free(void* o) { delete static_cast<OrcOC*>(o); }
// nested != 0: getHessian's threads also split the U(1) sectors inside each step
void orc_oc_set_nested(void* o, int nested) { static_cast<OrcOC*>(o)->oc->nested = nested; }
// sector threads of the calling thread's steps / applications (1: serial)
void orc_set_sector_threads(int n) { sector_threads() = n < 1 ? 1 : n; }
void orc_oc_set_gamma(void* o, double g) { static_cast<OrcOC*>(o)->oc->gamma = g; }

double orc_oc_cost(void* o, const double* u) {
  auto& oc = *static_cast<OrcOC*>(o)->oc;
  return oc.cost(std::vector<double>(u, u + oc.N));
}
int orc_oc_fidelities(void* o, const double* u, double* out) {
  auto& oc = *static_cast<OrcOC*>(o)->oc;
  oc.calcPsi(std::vector<double>(u, u + oc.N));
  auto f = oc.fidelities();
  for (size_t i = 0; i < f.size(); ++i) out[i] = f[i];
  return 0;
}
int orc_oc_gradient(void* o, const double* u, int bfgs, double* out) {
  auto& oc = *static_cast<OrcOC*>(o)->oc;
  auto g = oc.gradient(std::vector<double>(u, u + oc.N), bfgs != 0);
  for (size_t i = 0; i < g.size(); ++i) out[i] = g[i];
  return 0;
}
// divT (2N) and F (2) from the last gradient/hessian call
int orc_oc_divT(void* o, double* divT, double* F) {
  auto& oc = *static_cast<OrcOC*>(o)->oc;
  for (size_t i = 0; i < oc.divT.size(); ++i) { divT[2 * i] = oc.divT[i].real(); divT[2 * i + 1] = oc.divT[i].imag(); }
  cplx f = oc.overlapFactor();
  F[0] = f.real(); F[1] = f.imag();
  return 0;
}
int orc_oc_hessian(void* o, const double* u, int threads, double* out) {
  auto& oc = *static_cast<OrcOC*>(o)->oc;
  auto H = oc.hessian(std::vector<double>(u, u + oc.N), threads);
  std::memcpy(out, H.data(), H.size() * sizeof(double));
  return 0;
}
// Fidelity-Hessian entries of the given rows only (psi, xi, divT and xiH are
// recomputed for u; no regularisation): the per-rank shard of a row-sharded
// getHessian, written into a zeroed N x N `out`.
int orc_oc_rows(void* o, const double* u, const int* rows, int nrows, double* out) {
  auto& oc = *static_cast<OrcOC*>(o)->oc;
  std::vector<double> uu(u, u + oc.N);
  oc.calcPsi(uu);
  oc.calcXi(uu);
  oc.calcDivT();
  oc.xiH.assign(oc.N, MPS());
  for (size_t i = 0; i < oc.N; ++i) oc.xiH[i] = oc.st.apply_dH(oc.xi_t[i]);
  std::vector<double> H(oc.N * oc.N, 0.0);
  const cplx F = oc.overlapFactor();
  for (int r = 0; r < nrows; ++r) {
    if (rows[r] < 1 || size_t(rows[r]) + 1 >= oc.N) return 1;
    oc.hessianRow(size_t(rows[r]), uu, F, H);
  }
  std::memcpy(out, H.data(), H.size() * sizeof(double));
  return 0;
}
// which: 0 = psi_t, 1 = xi_t, 2 = xiH
int orc_oc_state(void* o, int which, int t, int* fd, double* data, size_t cap, size_t* nelem) {
  auto& oc = *static_cast<OrcOC*>(o)->oc;
  const auto& v = which == 0 ? oc.psi_t : (which == 1 ? oc.xi_t : oc.xiH);
  if (t < 0 || size_t(t) >= v.size()) return 3;
  return copy_out(v[t], fd, data, cap, nelem);
}

// Wall time of one full getHessian (psi, xi, divT, xiH, rows) with `threads`
// row workers — the CPU baseline leg (mirrors main/TestRuntimes.cpp:65-71).
double orc_oc_time_hessian(void* o, const double* u, int threads, double* out) {
  auto& oc = *static_cast<OrcOC*>(o)->oc;
  auto t0 = std::chrono::steady_clock::now();
  auto H = oc.hessian(std::vector<double>(u, u + oc.N), threads);
  auto t1 = std::chrono::steady_clock::now();
  if (out) std::memcpy(out, H.data(), H.size() * sizeof(double));
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
