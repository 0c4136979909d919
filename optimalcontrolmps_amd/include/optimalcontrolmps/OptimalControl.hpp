// OptimalControl<TimeStepper>: the IPOPT-facing surface of the reference
// (include/OptimalControl.hpp:17-75, src/OptimalControl.cpp:1-592) with the
// same names, signatures and new_control caching semantics, over a
// TimeStepper whose Engine keeps the trajectories (psi_t, xi_t, xiHlist) and
// runs the hot path: GpuTDMRG::Engine (HBM-resident, HIP) in the product;
// the CPU restatement in tests/ (tests/cpp/oracle_stepper.hpp).
//
// TimeStepper concept (reference include/BH_tDMRG.hpp:34-39 plus the engine):
//   double getTstep() const;  Args getArgs() const;
//   void step(MPS&, double from, double to, bool forward = true) const;
//   std::unique_ptr<Engine> makeEngine(const MPS& target, const MPS& init, size_t N) const;
//   Engine: setShards(n), propagate(u, which), divT(), overlapFactor(),
//           fidelities(), precomputeXiH(), hessianRows(u, F, divT, H),
//           hessianFresh(u, F&, divT&, H) (all of the above for a new control), psiTrajectory(),
//           convertHessian(basis, Hu) (ControlBasis::convertHessian, src/ControlBasis.cpp:91-116).
//
// Host-side arithmetic kept verbatim from the reference: the regularisation
// terms (:88-143), the gradient assembly g_i = dt Re(divT_i F i) (:240-246),
// the GROUP conversions (ControlBasis.hpp) and the caching flags.
// Threading: setThreadCount(n) selects the number of row shards (GPUs for
// GpuTDMRG); psi_t and xi_t always propagate concurrently on the device.
#pragma once

#include <cmath>
#include <complex>
#include <memory>
#include <stdexcept>
#include <vector>

#include "ControlBasis.hpp"
#include "MPS.hpp"

template <class TimeStepper>
class OptimalControl {
 public:
  using MPS = ocmps::MPS;
  using Cplx = ocmps::Cplx;
  using stdvec = ocmps::stdvec;
  using rowmat = ocmps::rowmat;
  using Engine = typename TimeStepper::Engine;

  // GRAPE constructor (src/OptimalControl.cpp:7-27)
  OptimalControl(MPS& psi_target_, MPS& psi_init_, TimeStepper& stepper_, size_t N_, double gamma_,
                 bool BFGS_ = false)
      : timeStepper(stepper_), gamma(gamma_), tstep(stepper_.getTstep()), N(N_), M(0),
        psi_target(psi_target_), psi_init(psi_init_), GRAPE(true), BFGS(BFGS_) {
    init();
  }
  // GROUP constructor (:30-50)
  OptimalControl(MPS& psi_target_, MPS& psi_init_, TimeStepper& stepper_, ControlBasis& basis_, double gamma_,
                 bool BFGS_ = false)
      : timeStepper(stepper_), basis(basis_), gamma(gamma_), tstep(stepper_.getTstep()), N(basis_.getN()),
        M(basis_.getM()), psi_target(psi_target_), psi_init(psi_init_), GRAPE(false), BFGS(BFGS_) {
    init();
  }

  std::vector<MPS> getPsit() const { return engine->psiTrajectory(); }
  size_t getM() const { return M; }
  size_t getN() const { return N; }
  stdvec getControl(const stdvec& control) { return GRAPE ? control : basis.convertControl(control); }
  // t = 0, dt, ... accumulated like the reference (:183-197)
  stdvec getTimeAxis() const {
    stdvec t;
    const double h = timeStepper.getTstep();
    for (double x = 0; std::fabs(x - N * h) > 1e-2 * h; x += h) t.push_back(x);
    return t;
  }
  void setGamma(double g) { gamma = g; }
  void setThreadCount(const size_t n) {
    if (n < 1) throw std::invalid_argument("Mininum threadCount is 1.");
    threadCount = n;
    engine->setShards(n);
  }
  void setGRAPE(const bool useGRAPE) {
    GRAPE = useGRAPE;
    calculatedXi = false;
  }
  void setBFGS(const bool useBFGS) {
    BFGS = useBFGS;
    calculatedXi = false;
  }
  bool useBFGS() const { return BFGS; }

  void propagatePsi(const stdvec& control) { calcPsi(GRAPE ? control : basis.convertControl(control)); }
  double getCost(const stdvec& control, const bool new_control = true) {
    return GRAPE ? calcCost(control, new_control) : calcCost(basis.convertControl(control, new_control), new_control);
  }
  stdvec getAnalyticGradient(const stdvec& control, const bool new_control = true) {
    if (GRAPE) return calcAnalyticGradient(control, new_control);
    return basis.convertGradient(calcAnalyticGradient(basis.convertControl(control, new_control), new_control));
  }
  // one code path for any threadCount: the rows are sharded by the engine
  rowmat getHessian(const stdvec& control, const bool new_control = true) {
    if (GRAPE) return calcHessian(control, new_control);
    // ControlBasis::convertHessian by the engine (the GPU engine projects on the device)
    return engine->convertHessian(basis, calcHessian(basis.convertControl(control, new_control), new_control));
  }
  stdvec getFidelityForAllT(const stdvec& control, const bool new_control = true) {
    return GRAPE ? calcFidelityForAllT(control, new_control)
                 : calcFidelityForAllT(basis.convertControl(control, new_control), new_control);
  }
  rowmat getControlJacobian() const {
    if (!GRAPE) return basis.getControlJacobian();
    rowmat I(N, stdvec(N, 0.0));
    for (size_t i = 0; i < N; ++i) I[i][i] = 1;
    return I;
  }

  // engine access (benchmarks, diagnostics)
  Engine& getEngine() { return *engine; }

 private:
  void init() {
    if (N < 4) throw std::invalid_argument("OptimalControl: N must be >= 4 (regularisation stencils)");
    threadCount = 1;
    calculatedXi = false;
    engine = timeStepper.makeEngine(psi_target, psi_init, N);
    divT.assign(N, Cplx(0, 0));
  }
  // ---- trajectories (:374-438)
  void calcPsi(const stdvec& u) {
    engine->propagate(u, 1);
    calculatedXi = false;
  }
  void calcXi(const stdvec& u) {
    engine->propagate(u, 2);
    calculatedXi = true;
  }
  void calcDivT() { divT = engine->divT(); }
  void calcPsiXiDivT(const stdvec& u) {
    engine->propagate(u, 3);
    calculatedXi = true;
    calcDivT();
  }
  // ---- regularisation (:88-143)
  double calcRegularization(const stdvec& u) const {
    double s = 0;
    for (size_t i = 0; i + 1 < N; ++i) {
      const double d = u[i + 1] - u[i];
      s += d * d / tstep;
    }
    return gamma / 2.0 * s;
  }
  stdvec calcRegularizationGrad(const stdvec& u) const {
    stdvec g(N);
    g[0] = -gamma * (-5.0 * u[1] + 4.0 * u[2] - u[3] + 2.0 * u[0]) / tstep;
    for (size_t i = 1; i + 1 < N; ++i) g[i] = -gamma * (u[i + 1] + u[i - 1] - 2.0 * u[i]) / tstep;
    g[N - 1] = -gamma * (-5.0 * u[N - 2] + 4.0 * u[N - 3] - u[N - 4] + 2.0 * u[N - 1]) / tstep;
    return g;
  }
  rowmat calcRegularizationHessian() const {
    rowmat H(N, stdvec(N, 0.0));
    const double g = gamma / tstep;
    for (size_t i = 1; i + 1 < N; ++i) {
      H[i][i - 1] = -g;
      H[i][i + 1] = -g;
      H[i][i] = 2.0 * g;
    }
    H[1][0] = 0;  // control endpoints are fixed
    H[N - 2][N - 1] = 0;
    return H;
  }
  // ---- cost / gradient / Hessian (:204-249, :281-372, :440-490)
  double calcCost(const stdvec& u, const bool new_control) {
    if (new_control) calcPsi(u);
    const double f = std::norm(engine->overlapFactor());  // |<target|psi_T>|^2
    return 0.5 * (1.0 - f) + calcRegularization(u);
  }
  stdvec calcFidelityGrad(const stdvec& u, const bool new_control) {
    if (new_control) {
      calculatedXi = false;
      if (BFGS) {
        // calcPsi + the inline xi propagation of the BFGS path (:210-229): xi
        // never reads psi, so both chains run concurrently in one launch
        engine->propagate(u, 3);
        calcDivT();
      } else {
        calcPsiXiDivT(u);
      }
    } else if (BFGS) {
      // the reference re-propagates xi inline on every BFGS gradient (:217-229)
      engine->propagate(u, 2);
      calcDivT();
    }
    if (!BFGS && !calculatedXi) {
      calcXi(u);
      calcDivT();
    }
    const Cplx F = engine->overlapFactor();
    stdvec g(N);
    for (size_t i = 0; i < N; ++i) g[i] = tstep * (divT[i] * F * Cplx(0, 1)).real();
    return g;
  }
  stdvec calcAnalyticGradient(const stdvec& u, const bool new_control) {
    stdvec g = calcFidelityGrad(u, new_control);
    const stdvec r = calcRegularizationGrad(u);
    for (size_t i = 0; i < N; ++i) g[i] += r[i];
    return g;
  }
  rowmat calcHessian(const stdvec& u, const bool new_control) {
    if (new_control) {
      // psi, xi, divT, xiHlist and the rows in one pipelined engine call
      rowmat H = calcRegularizationHessian();
      Cplx F;
      engine->hessianFresh(u, F, divT, H);
      calculatedXi = true;
      return H;
    }
    if (!calculatedXi) {
      calcXi(u);
      calcDivT();
    }
    rowmat H = calcRegularizationHessian();
    const Cplx F = engine->overlapFactor();
    engine->precomputeXiH();  // xiHlist (:300-303), recomputed on every call like the reference
    engine->hessianRows(u, F, divT, H);
    return H;
  }
  stdvec calcFidelityForAllT(const stdvec& u, const bool new_control) {
    if (new_control) calcPsi(u);
    return engine->fidelities();
  }

  TimeStepper timeStepper;
  ControlBasis basis;
  double gamma, tstep;
  size_t N, M, threadCount = 1;
  MPS psi_target, psi_init;
  std::vector<Cplx> divT;
  bool GRAPE, BFGS, calculatedXi = false;
  std::unique_ptr<Engine> engine;
};
