// TEST INFRASTRUCTURE ONLY — runs the device bodies of kernels.hpp on the CPU
// (one std::thread per lane of a 64-lane workgroup, std::barrier for
// __syncthreads) so the engine's logic can be debugged against the oracle
// without a GPU.  Not a fallback: the product library never contains or
// loads this code; GPU parity is established by the -m gpu tests.
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "hip/hip_runtime.h"
#include "../../optimalcontrolmps_amd/csrc/kernels.hpp"
#include "../../optimalcontrolmps_amd/csrc/params.hpp"
#include "../../optimalcontrolmps_amd/csrc/fast_plan.hpp"

thread_local emu_dim3 threadIdx, blockIdx, gridDim;
thread_local std::barrier<>* emu_bar;
thread_local std::barrier<>* emu_wbar;
thread_local uint64_t* emu_xbuf;

#ifndef EMU_NT
#define EMU_NT 64
#endif
constexpr int NT = EMU_NT;

struct Emu {
  OcgParams P;
  std::vector<int> md;
  std::vector<int> fplan;  // one-wave padded chain plan (empty: off)
  std::vector<int> oplan;  // padded overlap plan (empty: off)
  std::vector<double> gf, gb;
  int lds = 0;
  std::vector<int> dims;       // pool
  std::vector<ocg::zc> data;
  int nslots = 0;
  double stats[15] = {0};
  void slots(int n) {
    if (n <= nslots) return;
    dims.resize(size_t(n) * P.nsq, 0);
    data.resize(size_t(n) * P.cap, ocg::c2(0, 0));
    nslots = n;
  }
  ocg::Pool pool() { return ocg::Pool{dims.data(), data.data()}; }
  const ocg::zc* GF() { return reinterpret_cast<const ocg::zc*>(gf.data()); }
  const ocg::zc* GB() { return reinterpret_cast<const ocg::zc*>(gb.data()); }
};

static void launch(Emu& e, int grid, const std::function<void(char*)>& body) {
  for (int b = 0; b < grid; ++b) {
    std::vector<ocg::zc> smem((e.lds + 15) / 16 + 1);
    std::barrier<> bar(NT);
    std::vector<std::unique_ptr<std::barrier<>>> wb;
    for (int w = 0; w < NT / 64; ++w) wb.emplace_back(new std::barrier<>(64));
    std::vector<uint64_t> xb(NT, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < NT; ++t)
      th.emplace_back([&, t, b]() {
        threadIdx.x = t;
        blockIdx.x = b;
        gridDim.x = grid;
        emu_bar = &bar;
        emu_wbar = wb[t / 64].get();
        emu_xbuf = xb.data();
        body(reinterpret_cast<char*>(smem.data()));
      });
    for (auto& x : th) x.join();
  }
}

static size_t nelem_site(const OcgParams& P, const int* d, int k) {
  size_t s = 0;
  for (int q = 0; q < P.Q1; ++q)
    for (int n = 0; n < P.p && q + n <= P.Q; ++n) s += size_t(d[(k - 1) * P.Q1 + q]) * d[k * P.Q1 + q + n];
  return s;
}
static void put(Emu& e, int slot, const int* dims, const double* x) {
  const OcgParams& P = e.P;
  std::memcpy(&e.dims[size_t(slot) * P.nsq], dims, sizeof(int) * P.nsq);
  size_t off = 0;
  for (int k = 1; k <= P.L; ++k) {
    size_t n = nelem_site(P, dims, k);
    for (size_t i = 0; i < n; ++i)
      e.data[size_t(slot) * P.cap + P.site_base[k] + i] = ocg::c2(x[2 * (off + i)], x[2 * (off + i) + 1]);
    off += n;
  }
}
static size_t get(Emu& e, int slot, int* dims, double* x) {
  const OcgParams& P = e.P;
  const int* d = &e.dims[size_t(slot) * P.nsq];
  std::memcpy(dims, d, sizeof(int) * P.nsq);
  size_t off = 0;
  for (int k = 1; k <= P.L; ++k) {
    size_t n = nelem_site(P, d, k);
    for (size_t i = 0; i < n; ++i) {
      ocg::zc z = e.data[size_t(slot) * P.cap + P.site_base[k] + i];
      x[2 * (off + i)] = z.x;
      x[2 * (off + i) + 1] = z.y;
    }
    off += n;
  }
  return off;
}

extern "C" {

void* emu_new(int L, int p, int Q, double J, double dt, double cutoff, int maxm) {
  auto* e = new Emu;
  std::string err = ocg_host::build_params(e->P, e->md, L, p, Q, dt, cutoff, maxm);
  if (!err.empty()) { delete e; return nullptr; }
  ocg_host::gate_tables(e->P, J, e->gf, e->gb);
  e->lds = ocg::lds_layout(e->P, NT).bytes;
  e->P.lds_bytes = e->lds;
  e->slots(8);
  return e;
}
// fast != 0: every step runs on the one-wave padded chain (fast_chain.hpp) when
// its plan builds; returns null if requested and unavailable
void* emu_new_ex(int L, int p, int Q, double J, double dt, double cutoff, int maxm, int fast) {
  auto* e = static_cast<Emu*>(emu_new(L, p, Q, J, dt, cutoff, maxm));
  if (!e || !fast) return e;
  ocg_host::FastPlanBuild fb = ocg_host::build_fast_plan(e->P, e->md);
  if (!fb.why_not.empty()) {
    std::fprintf(stderr, "fast plan: %s\n", fb.why_not.c_str());
    delete e;
    return nullptr;
  }
  e->fplan = fb.plan;
  const int off = (e->lds + 255) & ~255;
  e->P.fplan = e->fplan.data();
  e->P.fast_off = off;
  e->lds = off + ocg_host::fast_lds_bytes(e->fplan, e->P);
  e->P.lds_bytes = e->lds;
  // the padded overlap, as ocmps.hip's finish_params (OCG_NO_FAST_OVL=1: off)
  const char* no = std::getenv("OCG_NO_FAST_OVL");
  e->oplan = ocg_host::build_overlap_plan(e->P, e->md);
  if (!e->oplan.empty() && ocg_host::overlap_lds_bytes(e->oplan, e->P) <= off && !(no && no[0] && no[0] != '0')) {
    e->P.oplan = e->oplan.data();
    e->P.ovl_bytes = ocg_host::overlap_lds_bytes(e->oplan, e->P);
    e->P.ovl_dh_bytes = ocg_host::overlap_lds_bytes(e->oplan, e->P, true);
  }
  return e;
}
void emu_free(void* h) { delete static_cast<Emu*>(h); }
int emu_lds_bytes(void* h) { return static_cast<Emu*>(h)->lds; }

size_t emu_steps(void* h, const int* dims, const double* x, const double* u, int nsteps, int fwd, int* od,
                 double* ox) {
  Emu& e = *static_cast<Emu*>(h);
  put(e, 2, dims, x);
  int slot = 2;
  OcgParams P = e.P;
  P.fast_off = 0;  // as ocg_steps: the one-wave chain's region aliases the general chain's LDS
  launch(e, 1, [&](char* smem) {
    ocg::body_steps<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), &slot, 1, u, nsteps + 1, nsteps, fwd,
                        e.stats + 12);
  });
  return get(e, 2, od, ox);
}

size_t emu_apply_dH(void* h, const int* dims, const double* x, int* od, double* ox, double* norm) {
  Emu& e = *static_cast<Emu*>(h);
  put(e, 2, dims, x);
  int in = 2, out = 3;
  OcgParams P = e.P;
  launch(e, 1, [&](char* smem) {
    ocg::body_apply_dH<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), &in, &out, 1, norm, e.stats + 6);
  });
  return get(e, 3, od, ox);
}

#ifndef EMU_STEPS_ONLY  // the sanitizer build (tests/test_sanitizers.py) runs steps only
void emu_overlap(void* h, const int* dx, const double* x, const int* dy, const double* y, int with_dH,
                 double* out) {
  Emu& e = *static_cast<Emu*>(h);
  put(e, 2, dx, x);
  put(e, 3, dy, y);
  int xs = 2, ys = 3;
  ocg::zc r = ocg::c2(0, 0);
  OcgParams P = e.P;
  launch(e, 1, [&](char* smem) {
    ocg::body_overlaps<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), &xs, &ys, 1, with_dH, &r, e.stats + 3);
  });
  out[0] = r.x;
  out[1] = r.y;
}

// the same pair on the padded contraction (fast_overlap.hpp; fast contexts only): 0, or -1 without the plan
int emu_overlap_pad(void* h, const int* dx, const double* x, const int* dy, const double* y, int with_dH,
                    double* out) {
  Emu& e = *static_cast<Emu*>(h);
  if (!e.P.oplan) return -1;
  put(e, 2, dx, x);
  put(e, 3, dy, y);
  int xs = 2, ys = 3;
  ocg::zc r = ocg::c2(0, 0);
  OcgParams P = e.P;
  const int lds = e.lds;
  e.lds = std::max(e.lds, P.ovl_dh_bytes);
  launch(e, 1, [&](char* smem) { ocg::body_overlaps_pad(smem, P, e.pool(), &xs, &ys, 1, with_dH, &r, e.stats + 3); });
  e.lds = lds;
  out[0] = r.x;
  out[1] = r.y;
  return 0;
}

// full getHessian pipeline (GRAPE, no regularisation): H (N*N), divT (2N), F (2), fid (N)
void emu_hessian(void* h, const int* dt_, const double* tgt, const int* di, const double* ini, const double* u, int N,
                 double* H, double* divT, double* F, double* fid, int nrows_max) {
  Emu& e = *static_cast<Emu*>(h);
  e.slots(6 + 3 * N);
  put(e, 1, dt_, tgt);
  put(e, 0, di, ini);
  OcgParams P = e.P;
  const int psi = 6, xi = 6 + N, xih = 6 + 2 * N;
  launch(e, 2, [&](char* smem) {
    ocg::body_trajectory<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), 0, 1, psi, xi, u, N, 3, e.stats, 0);
  });
  std::vector<int> xs(N), ys(N);
  std::vector<ocg::zc> r(N);
  for (int i = 0; i < N; ++i) { xs[i] = xi + i; ys[i] = psi + i; }
  launch(e, N, [&](char* smem) {
    ocg::body_overlaps<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), xs.data(), ys.data(), N, 1, r.data(),
                           e.stats + 3);
  });
  for (int i = 0; i < N; ++i) { divT[2 * i] = r[i].x; divT[2 * i + 1] = r[i].y; }
  for (int i = 0; i < N; ++i) { xs[i] = 1; ys[i] = psi + i; }
  launch(e, N, [&](char* smem) {
    ocg::body_overlaps<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), xs.data(), ys.data(), N, 0, r.data(),
                           e.stats + 3);
  });
  for (int i = 0; i < N; ++i) fid[i] = r[i].x * r[i].x + r[i].y * r[i].y;
  int a = psi + N - 1, b = 1;
  ocg::zc f = ocg::c2(0, 0);
  launch(e, 1, [&](char* smem) {
    ocg::body_overlaps<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), &a, &b, 1, 0, &f, e.stats + 3);
  });
  F[0] = f.x;
  F[1] = f.y;
  std::vector<int> in(N), outs(N);
  for (int i = 0; i < N; ++i) { in[i] = xi + i; outs[i] = xih + i; }
  launch(e, N, [&](char* smem) {
    ocg::body_apply_dH<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), in.data(), outs.data(), N, nullptr,
                           e.stats + 6);
  });
  std::vector<int> rows;
  for (int i = 1; i + 1 < N && int(rows.size()) < nrows_max; ++i) rows.push_back(i);
  std::vector<ocg::zc> dv(N);
  for (int i = 0; i < N; ++i) dv[i] = ocg::c2(divT[2 * i], divT[2 * i + 1]);
  std::memset(H, 0, sizeof(double) * N * N);
  e.slots(6 + 4 * N);
  const int psih = 6 + 3 * N;
  std::vector<int> pin(rows.size()), pout(rows.size());
  std::vector<double> nr(rows.size()), ni(N, 0.0);
  for (size_t r = 0; r < rows.size(); ++r) { pin[r] = psi + rows[r]; pout[r] = psih + rows[r]; }
  launch(e, int(rows.size()), [&](char* smem) {
    ocg::body_apply_dH<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), pin.data(), pout.data(),
                           int(rows.size()), nr.data(), e.stats + 6);
  });
  for (size_t r = 0; r < rows.size(); ++r) ni[rows[r]] = nr[r];
  launch(e, int(rows.size()), [&](char* smem) {
    ocg::body_hessian_rows<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), psih, xih, rows.data(),
                               int(rows.size()), ni.data(), u, N, dv.data(), f, H, e.stats + 9);
  });
}

// fused pipeline (ocg_hessian): k_pipeline then divT/F overlaps then k_row_overlaps
void emu_hessian_fused(void* h, const int* dt_, const double* tgt, const int* di, const double* ini, const double* u,
                       int N, double* H, double* divT, double* F) {
  Emu& e = *static_cast<Emu*>(h);
  e.slots(6 + 4 * N);
  put(e, 1, dt_, tgt);
  put(e, 0, di, ini);
  OcgParams P = e.P;
  const int psi = 6, xi = 6 + N, xih = 6 + 2 * N;
  std::vector<int> rows, rb;
  for (int i = 1; i + 1 < N; ++i) rows.push_back(i);
  const int nrows = int(rows.size());
  int total = 0;
  for (int r = 0; r < nrows; ++r) { rb.push_back(total); total += N - 1 - rows[r]; }
  rb.push_back(total);
  std::vector<int> rsd(size_t(total) * P.nsq, 0);
  std::vector<ocg::zc> rsx(size_t(total) * P.cap, ocg::c2(0, 0));
  ocg::Pool rs{rsd.data(), rsx.data()};
  std::vector<double> rn(nrows, 0.0);
  std::vector<int> flags(2 * N + 3, 0);
  int err = 0;
  const int nxw = N < 8 ? N : 8;
  OcgParams PA = P;
  PA.fast_off = 0;  // as ocg_hessian: aliased regions in k_pipeline
  launch(e, 2 + nxw + nrows, [&](char* smem) {
    ocg::body_pipeline<NT>(smem, PA, e.GF(), e.GB(), e.md.data(), e.pool(), 0, 1, psi, xi, xih, u, N, rows.data(),
                           nrows, rb.data(), rs, rn.data(), flags.data(), 1, &err, nxw, e.stats, 1, 0);
  });
  std::vector<int> xs(N), ys(N);
  std::vector<ocg::zc> pc(N + 1);
  for (int i = 0; i < N; ++i) { xs[i] = xi + i; ys[i] = psi + i; }
  launch(e, N, [&](char* smem) {
    ocg::body_overlaps<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), xs.data(), ys.data(), N, 1, pc.data(),
                           e.stats + 3);
  });
  int a = psi + N - 1, b = 1;
  launch(e, 1, [&](char* smem) {
    ocg::body_overlaps<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), &a, &b, 1, 0, pc.data() + N, e.stats + 3);
  });
  std::memset(H, 0, sizeof(double) * N * N);
  if (P.oplan) e.lds = std::max(e.lds, P.ovl_bytes + 4 * (2 * nrows + 1));  // + the row table
  launch(e, total, [&](char* smem) {
    if (P.oplan)
      ocg::body_row_overlaps_pad(smem, P, e.pool(), xih, rows.data(), nrows, rb.data(), rs, rn.data(), pc.data(),
                                 pc.data() + N, N, H, e.stats + 9, 1, 0);
    else
      ocg::body_row_overlaps<NT>(smem, P, e.GF(), e.GB(), e.md.data(), e.pool(), xih, rows.data(), nrows, rb.data(),
                                 rs, rn.data(), pc.data(), pc.data() + N, N, H, e.stats + 9, 1, 0);
  });
  for (int i = 0; i < N; ++i) { divT[2 * i] = pc[i].x; divT[2 * i + 1] = pc[i].y; }
  F[0] = pc[N].x;
  F[1] = pc[N].y;
  if (err) std::fprintf(stderr, "pipeline err %d\n", err);
}

}  // extern "C"

extern "C" size_t emu_position(void* h, const int* dims, const double* x, int target, int back, int* od, double* ox) {
  Emu& e = *static_cast<Emu*>(h);
  put(e, 2, dims, x);
  OcgParams P = e.P;
  launch(e, 1, [&](char* smem) {
    ocg::Chain<NT> c(P, smem);
    c.load_tables(e.GF(), e.GB(), e.md.data());
    c.load(&e.dims[2 * P.nsq], &e.data[2 * P.cap]);
    int centre = 1;
    c.position(centre, target);
    if (back) c.position(centre, 1);
    c.store(&e.dims[2 * P.nsq], &e.data[2 * P.cap]);
  });
  return get(e, 2, od, ox);
}

extern "C" size_t emu_zip(void* h, const int* dims, const double* x, int sweep, int* od, double* ox) {
  Emu& e = *static_cast<Emu*>(h);
  put(e, 2, dims, x);
  OcgParams P = e.P;
  launch(e, 1, [&](char* smem) {
    ocg::Chain<NT> c(P, smem);
    c.load_tables(e.GF(), e.GB(), e.md.data());
    c.load(&e.dims[2 * P.nsq], &e.data[2 * P.cap]);
    c.apply_dH(sweep != 0);
    c.store(&e.dims[2 * P.nsq], &e.data[2 * P.cap]);
  });
  return get(e, 2, od, ox);
}

// one Θ block (R x C, complex) -> decompose(dir) ; returns kept, fills X (R*k), Y (k*C), lam
extern "C" int emu_decompose(void* h, int R, int C, const double* M, int dir, double cutoff, double* X, double* Y) {
  Emu& e = *static_cast<Emu*>(h);
  OcgParams P = e.P;
  int kept = 0;
  std::vector<int> bound(P.Q1, 1 << 30);
  launch(e, 1, [&](char* smem) {
    ocg::Chain<NT> c(P, smem);
    c.load_tables(e.GF(), e.GB(), e.md.data());
    if (c.tid == 0) {
      for (int q = 0; q < P.Q1; ++q) { c.THR[q] = 0; c.THC[q] = 0; c.THO[q] = 0; }
      c.THR[0] = R; c.THC[0] = C;
      for (int q = 1; q <= P.Q1; ++q) c.THO[q] = R * C;
    }
    c.sync();
    for (int i = c.tid; i < R * C; i += NT) c.TH[i] = ocg::c2(M[2 * i], M[2 * i + 1]);
    c.sync();
    c.decompose(dir, cutoff, 1 << 30, false, (LDS const int*)bound.data());
    if (c.tid == 0) {
      kept = c.KEPT[0];
      for (int i = 0; i < R * kept; ++i) { ocg::zc z = c.X[i]; X[2 * i] = z.x; X[2 * i + 1] = z.y; }
      for (int i = 0; i < kept * C; ++i) { ocg::zc z = c.Y[i]; Y[2 * i] = z.x; Y[2 * i + 1] = z.y; }
    }
    c.sync();
  });
  return kept;
}

// multi-block: nb blocks (nb <= Q1), Rs/Cs sizes, M concatenated row-major blocks
extern "C" void emu_decompose_multi(void* h, int nb, const int* Rs, const int* Cs, const double* M, int dir,
                                    double cutoff, int* kept, double* X, double* Y) {
  Emu& e = *static_cast<Emu*>(h);
  OcgParams P = e.P;
  std::vector<int> bound(P.Q1, 1 << 30);
  launch(e, 1, [&](char* smem) {
    ocg::Chain<NT> c(P, smem);
    c.load_tables(e.GF(), e.GB(), e.md.data());
    int tot = 0;
    if (c.tid == 0) {
      int off = 0;
      for (int q = 0; q < P.Q1; ++q) {
        int R = q < nb ? Rs[q] : 0, C = q < nb ? Cs[q] : 0;
        c.THR[q] = R; c.THC[q] = C; c.THO[q] = off; off += R * C;
      }
      c.THO[P.Q1] = off;
    }
    c.sync();
    tot = c.THO[P.Q1];
    for (int i = c.tid; i < tot; i += NT) c.TH[i] = ocg::c2(M[2 * i], M[2 * i + 1]);
    c.sync();
    c.decompose(dir, cutoff, 1 << 30, false, (LDS const int*)bound.data());
    if (c.tid == 0) {
      for (int q = 0; q < nb; ++q) kept[q] = c.KEPT[q];
      for (int i = 0; i < c.XOFF[P.Q1]; ++i) { ocg::zc z = c.X[i]; X[2 * i] = z.x; X[2 * i + 1] = z.y; }
      for (int i = 0; i < c.YOFF[P.Q1]; ++i) { ocg::zc z = c.Y[i]; Y[2 * i] = z.x; Y[2 * i + 1] = z.y; }
    }
    c.sync();
  });
}
#else
}  // extern "C" (closed inside the excluded part otherwise)
#endif  // EMU_STEPS_ONLY
