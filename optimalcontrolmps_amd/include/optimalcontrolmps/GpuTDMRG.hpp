// GpuTDMRG: the MI355X TimeStepper behind the reference's stepper concept
// (reference include/BH_tDMRG.hpp:17-40, src/BH_tDMRG.cpp), implemented over
// the C-ABI of liboptimalcontrolmps_amd.so (include/ocmps.h).
//
// Stepper members kept with the reference's names and meaning:
//   GpuTDMRG(sites, J, tstep, args)          BH_tDMRG(sites, J, tstep, args)  (:34)
//   setTstep / getTstep / getArgs            (:35, :38, :39)
//   step(psi, from, to, propagateForward)    (:36; src/BH_tDMRG.cpp:111-230)
//   propagatorDeriv(u)                       (:37; src/BH_tDMRG.cpp:238-241)
// The particle number is taken from the states (ITensor infers it from the
// IQMPS quantum numbers), so device contexts are created on first use.
//
// OptimalControl<GpuTDMRG> drives the batched device paths through
// GpuTDMRG::Engine: psi_t / xi_t / xiHlist stay resident in HBM, and the
// Hessian rows are sharded zig-zag over the devices selected by
// setThreadCount (one context, stream and host thread per device).
#pragma once

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/ocmps.h"
#include "ControlBasis.hpp"
#include "MPS.hpp"

namespace ocmps {

namespace detail {
inline void check(int rc, const ocg_ctx* ctx, const char* what) {
  if (rc != OCG_OK) {
    const char* msg = ocg_last_error(ctx);
    throw std::runtime_error(std::string(what) + ": " + (msg ? msg : "error"));
  }
}
struct CtxDeleter {
  void operator()(ocg_ctx* c) const {
    if (c) ocg_destroy(c);
  }
};
using CtxPtr = std::unique_ptr<ocg_ctx, CtxDeleter>;

inline CtxPtr make_ctx(int dev, int L, int p, int Q, double J, double dt, const Args& a) {
  ocg_ctx* c = nullptr;
  check(ocg_create(dev, L, p, Q, J, dt, a.cutoff, a.maxm, &c), nullptr, "ocg_create");
  return CtxPtr(c);
}
inline MPS fetch_state(ocg_ctx* c, int L, int p, int Q, int which, int t) {
  ocg_info info;
  check(ocg_get_info(c, &info), c, "ocg_get_info");
  std::vector<int> dims(size_t(L + 1) * (Q + 1));
  std::vector<Cplx> data(info.mps_max_nelem);
  size_t n = 0;
  check(ocg_get_state(c, which, t, dims.data(), reinterpret_cast<double*>(data.data()), data.size(), &n), c,
        "ocg_get_state");
  data.resize(n);
  return MPS(L, p, Q, std::move(dims), std::move(data));
}
}  // namespace detail

// propagatorDeriv: the constant on-site MPO dH = sum_k 0.5 n_k (n_k - 1)
// (src/BH_tDMRG.cpp:10-14, :238-241); the control argument is ignored.
struct DerivMPO {
  int L = 0, p = 0;
  std::vector<double> onsite;  // 0.5 n (n-1), n = 0..p-1
};

class GpuTDMRG {
 public:
  class Engine;

  GpuTDMRG() = default;
  GpuTDMRG(const BoseHubbard& sites, double J_, double tstep_, const Args& args_ = Args())
      : L(sites.L), p(sites.localDim()), J(J_), tstep(tstep_), args(args_), scratch(std::make_shared<Scratch>()) {}

  void setTstep(double t) {
    tstep = t;
    scratch = std::make_shared<Scratch>();  // contexts carry dt-dependent gates
  }
  double getTstep() const { return tstep; }
  Args getArgs() const { return args; }
  DerivMPO propagatorDeriv(const double& /*control_n*/) const {
    DerivMPO m{L, p, std::vector<double>(p)};
    for (int n = 0; n < p; ++n) m.onsite[n] = 0.5 * n * (n - 1);
    return m;
  }
  // one Trotter step of psi in place (src/BH_tDMRG.cpp:111-125)
  void step(MPS& psi, double from, double to, bool propagateForward = true) const {
    ocg_ctx* c = scratch_ctx(psi.Q);
    std::vector<int> od(psi.dims.size());
    ocg_info info;
    detail::check(ocg_get_info(c, &info), c, "ocg_get_info");
    std::vector<Cplx> out(info.mps_max_nelem);
    size_t n = 0;
    detail::check(ocg_step(c, psi.dims.data(), psi.raw(), from, to, propagateForward ? 1 : 0, od.data(),
                           reinterpret_cast<double*>(out.data()), out.size(), &n),
                  c, "ocg_step");
    out.resize(n);
    psi = MPS(L, p, psi.Q, std::move(od), std::move(out));
  }
  // device used for single steps / the first shard (default 0)
  void setDevice(int dev) {
    device = dev;
    scratch = std::make_shared<Scratch>();
  }
  int getDevice() const { return device; }

  // trajectory engine owned by one OptimalControl (see OptimalControl.hpp)
  std::unique_ptr<Engine> makeEngine(const MPS& target, const MPS& init, size_t N) const;

  int sitesL() const { return L; }
  int localDim() const { return p; }
  double hopping() const { return J; }

 private:
  struct Scratch {
    std::mutex mu;
    std::map<int, detail::CtxPtr> byQ;
  };
  ocg_ctx* scratch_ctx(int Q) const {
    std::lock_guard<std::mutex> lk(scratch->mu);
    auto& c = scratch->byQ[Q];
    if (!c) c = detail::make_ctx(device, L, p, Q, J, tstep, args);
    return c.get();
  }
  int L = 0, p = 0, device = 0;
  double J = 1.0, tstep = 0.01;
  Args args;
  std::shared_ptr<Scratch> scratch;  // step() is const in the reference; the context cache is shared by copies
};

// Device-resident trajectories of one OptimalControl instance.  Shard s owns
// a context on device (first + s); every shard recomputes psi_t / xi_t /
// xiHlist itself (2(N-1) steps, small next to the (N-2)(N-3)/2 row steps).
class GpuTDMRG::Engine {
 public:
  Engine(const GpuTDMRG& st, const MPS& target, const MPS& init, size_t N_)
      : stepper(st), tgt(target), ini(init), N(N_) {
    if (target.Q != init.Q || target.L != st.L || init.L != st.L || target.p != st.p || init.p != st.p)
      throw std::invalid_argument("OptimalControl: target/init states do not match the stepper's sites");
    setShards(1);
  }
  // setThreadCount: number of GPUs (shards) the Hessian rows are spread over.
  // Existing shards keep their trajectories; new shards replay the controls
  // of the current psi_t / xi_t before their first use.
  void setShards(size_t n) {
    if (n < 1) throw std::invalid_argument("Mininum threadCount is 1.");
    while (shards.size() > n) shards.pop_back();
    const size_t kept = shards.size();
    int ndev = 0;
    detail::check(ocg_device_count(&ndev), nullptr, "ocg_device_count");
    while (shards.size() < n) {
      // shard s on device (first + s) mod #devices: more shards than GPUs run
      // concurrently on separate streams of the same device
      const int dev = (stepper.device + int(shards.size())) % ndev;
      detail::CtxPtr c = detail::make_ctx(dev, stepper.L, stepper.p, tgt.Q, stepper.J, stepper.tstep, stepper.args);
      detail::check(ocg_set_states(c.get(), tgt.dims.data(), tgt.raw(), ini.dims.data(), ini.raw()), c.get(),
                    "ocg_set_states");
      shards.push_back(std::move(c));
    }
    // shards created by this call replay shard 0's controls before first use;
    // existing shards keep their trajectories (and their flags)
    fresh.resize(shards.size(), 1);
    xih_done.resize(shards.size(), 0);
    if (kept == 0) fresh[0] = 0;  // shard 0 is the reference copy
    for (size_t s = kept; s < shards.size(); ++s) xih_done[s] = 0;
  }
  size_t nShards() const { return shards.size(); }
  // which: 1 psi_t (calcPsi), 2 xi_t (calcXi), 3 both concurrently
  void propagate(const stdvec& u, int which) {
    check_len(u);
    on_all([&](ocg_ctx* c) { detail::check(ocg_propagate(c, u.data(), int(N), which), c, "ocg_propagate"); });
    if (which & 1) u_psi = u;
    if (which & 2) u_xi = u;
    for (size_t s = 0; s < shards.size(); ++s) xih_done[s] = 0;
  }
  std::vector<Cplx> divT() {
    std::vector<Cplx> d(N);
    ocg_ctx* c = shards[0].get();
    detail::check(ocg_div_t(c, reinterpret_cast<double*>(d.data())), c, "ocg_div_t");
    return d;
  }
  Cplx overlapFactor() {
    double F[2];
    ocg_ctx* c = shards[0].get();
    detail::check(ocg_overlap_factor(c, F), c, "ocg_overlap_factor");
    return Cplx(F[0], F[1]);
  }
  stdvec fidelities() {
    stdvec f(N);
    ocg_ctx* c = shards[0].get();
    detail::check(ocg_fidelities(c, f.data()), c, "ocg_fidelities");
    return f;
  }
  void precomputeXiH() {
    replay_fresh();
    on_all([&](ocg_ctx* c) { detail::check(ocg_xi_dH(c), c, "ocg_xi_dH"); });
  }
  // calcHessianRow for rows 1..N-2 (zig-zag over shards), added into H
  void hessianRows(const stdvec& u, Cplx F, const std::vector<Cplx>& dT, rowmat& H) {
    check_len(u);
    const size_t G = shards.size();
    std::vector<std::vector<int>> rows(G);
    replay_fresh();
    for (size_t i = 1, k = 0; i + 1 < N; ++i, ++k) {
      const size_t r = k % (2 * G);
      rows[r < G ? r : 2 * G - 1 - r].push_back(int(i));
    }
    std::vector<std::vector<double>> part(G, std::vector<double>(N * N, 0.0));
    const double Fv[2] = {F.real(), F.imag()};
    on_all_indexed([&](size_t s, ocg_ctx* c) {
      if (rows[s].empty()) return;
      detail::check(ocg_hessian_rows(c, u.data(), int(N), rows[s].data(), int(rows[s].size()), Fv,
                                     reinterpret_cast<const double*>(dT.data()), part[s].data()),
                    c, "ocg_hessian_rows");
    });
    gather_rows(rows, part, H);
  }
  // getHessian(u, new_control = true) fidelity part in one pipelined call per
  // shard (ocg_hessian): trajectories, xiHlist and the shard's rows overlap
  void hessianFresh(const stdvec& u, Cplx& F, std::vector<Cplx>& dT, rowmat& H) {
    check_len(u);
    const size_t G = shards.size();
    std::vector<std::vector<int>> rows(G);
    for (size_t i = 1, k = 0; i + 1 < N; ++i, ++k) {
      const size_t r = k % (2 * G);
      rows[r < G ? r : 2 * G - 1 - r].push_back(int(i));
    }
    std::vector<std::vector<double>> part(G, std::vector<double>(N * N, 0.0));
    std::vector<double> dv(2 * N);
    double Fv[2] = {0, 0};
    on_all_indexed([&](size_t s, ocg_ctx* c) {
      std::vector<double> dvs(2 * N);
      double Fs[2];
      detail::check(ocg_hessian(c, u.data(), int(N), rows[s].data(), int(rows[s].size()), part[s].data(), dvs.data(),
                                Fs),
                    c, "ocg_hessian");
      if (s == 0) {
        dv = dvs;
        Fv[0] = Fs[0];
        Fv[1] = Fs[1];
      }
    });
    for (size_t s = 0; s < G; ++s) fresh[s] = 0;
    u_psi = u;
    u_xi = u;
    F = Cplx(Fv[0], Fv[1]);
    dT.resize(N);
    for (size_t i = 0; i < N; ++i) dT[i] = Cplx(dv[2 * i], dv[2 * i + 1]);
    gather_rows(rows, part, H);
  }
  // ControlBasis::convertHessian (src/ControlBasis.cpp:91-116) on shard 0's
  // device: bit-identical to the host restatement (ocg_convert_hessian)
  rowmat convertHessian(const ControlBasis& basis, const rowmat& Hu) {
    const rowmat& V = basis.basisMatrix();
    const size_t M = V.size(), n = Hu.size();
    if (M == 0 || n != N) return basis.convertHessian(Hu);
    std::vector<double> h(n * n), v(M * n), hc(M * M);
    for (size_t i = 0; i < n; ++i) std::copy(Hu[i].begin(), Hu[i].end(), h.begin() + i * n);
    for (size_t j = 0; j < M; ++j) std::copy(V[j].begin(), V[j].end(), v.begin() + j * n);
    ocg_ctx* c = shards[0].get();
    detail::check(ocg_convert_hessian(c, h.data(), int(n), v.data(), int(M), hc.data()), c, "ocg_convert_hessian");
    rowmat Hc(M, stdvec(M));
    for (size_t i = 0; i < M; ++i) std::copy(hc.begin() + i * M, hc.begin() + (i + 1) * M, Hc[i].begin());
    return Hc;
  }
  std::vector<MPS> psiTrajectory() {
    std::vector<MPS> out;
    for (size_t t = 0; t < N; ++t)
      out.push_back(detail::fetch_state(shards[0].get(), stepper.L, stepper.p, tgt.Q, 0, int(t)));
    return out;
  }

 private:
  // Shard s wrote the entries (i, j >= i) of its rows and their mirrors; the
  // entry sets of different shards are disjoint, so adding only those is the
  // exact sum of the partial matrices (O(N^2) in total instead of G N^2).
  void gather_rows(const std::vector<std::vector<int>>& rows, const std::vector<std::vector<double>>& part,
                   rowmat& H) const {
    for (size_t s = 0; s < rows.size(); ++s)
      for (int i : rows[s])
        for (size_t j = size_t(i); j + 1 < N; ++j) {
          H[i][j] += part[s][size_t(i) * N + j];
          if (j > size_t(i)) H[j][i] += part[s][j * N + size_t(i)];
        }
  }
  // bring shards created after the last propagation up to shard 0's state
  void replay_fresh() {
    for (size_t s = 0; s < shards.size(); ++s) {
      if (!fresh[s]) continue;
      ocg_ctx* c = shards[s].get();
      if (!u_psi.empty()) detail::check(ocg_propagate(c, u_psi.data(), int(N), 1), c, "ocg_propagate");
      if (!u_xi.empty()) detail::check(ocg_propagate(c, u_xi.data(), int(N), 2), c, "ocg_propagate");
      fresh[s] = 0;
    }
  }
  void check_len(const stdvec& u) const {
    if (u.size() != N) throw std::invalid_argument("control has length " + std::to_string(u.size()) +
                                                   ", expected N = " + std::to_string(N));
  }
  template <class F>
  void on_all(F f) {
    on_all_indexed([&](size_t, ocg_ctx* c) { f(c); });
  }
  template <class F>
  void on_all_indexed(F f) {
    if (shards.size() == 1) { f(0, shards[0].get()); return; }
    std::vector<std::thread> th;
    std::vector<std::string> err(shards.size());
    for (size_t s = 0; s < shards.size(); ++s)
      th.emplace_back([&, s]() {
        try { f(s, shards[s].get()); } catch (const std::exception& e) { err[s] = e.what(); }
      });
    for (auto& t : th) t.join();
    for (auto& e : err)
      if (!e.empty()) throw std::runtime_error(e);
  }
  GpuTDMRG stepper;
  MPS tgt, ini;
  size_t N;
  std::vector<detail::CtxPtr> shards;
  std::vector<char> fresh, xih_done;
  stdvec u_psi, u_xi;  // controls of the current device trajectories
};

inline std::unique_ptr<GpuTDMRG::Engine> GpuTDMRG::makeEngine(const MPS& target, const MPS& init, size_t N) const {
  return std::unique_ptr<Engine>(new Engine(*this, target, init, N));
}

}  // namespace ocmps
