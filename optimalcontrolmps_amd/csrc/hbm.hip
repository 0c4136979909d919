// Host side of the HBM-resident tDMRG engine (see hbm_device.hpp for the
// kernels and DESIGN.md §9 for the data layout).  Restates, batched over many
// MPS chains at once and with every tensor in HBM:
//   BH_tDMRG::step / doStep                  (reference src/BH_tDMRG.cpp:111-230)
//   ITensor denmatDecomp + truncate per QN   (called at src/BH_tDMRG.cpp:178,191,209)
//   MPS::position / normalize                (src/BH_tDMRG.cpp:187,198,217,228)
//   exactApplyMPO(propDeriv, psi)            (src/OptimalControl.cpp:256,302)
//   overlapC(psi, phi) / overlapC(psi,H,phi) (src/OptimalControl.cpp:242,261,272,412)
// with the same arithmetic choices as the LDS chain engine and the oracle
// (Gram on the smaller side, ITensor truncation rule, gauge cutoff 1e-14).
//
// Site storage ("left-grouped"): site k holds, for every right sector q' of
// bond k (ascending), the left matricisation Lmat_q' = rows (n, a in bond
// k-1 sector q'-n) n-ascending, cols = bond-k states of sector q', row-major.
// Block (q, n) of the site is therefore one contiguous row-major
// dims[k-1][q] x dims[k][q+n] matrix (the interchange format's block, in a
// different block order), Lmat_q' is contiguous, and the right
// matricisation's column segments are those blocks.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "hbm.hpp"
#include "hbm_device.hpp"

namespace hbm {

// ---------------------------------------------------------------- errors
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
#define HCK(expr)                                                                                 \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) throw ::hbm::Error(3, std::string(#expr) + ": " + hipGetErrorString(e_));     \
  } while (0)
// allocations: out of device / pinned memory is its own status (OCG_ENOMEM), the
// only failure after which ocg_hessian may retry a getHessian on another path
#define HCKA(expr)                                                                                \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      throw ::hbm::Error(e_ == hipErrorOutOfMemory ? 6 : 3, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr double kGaugeCutoff = 1e-14;  // = OCG_GAUGE_CUTOFF of the LDS engine and the oracle
constexpr int kNoMaxm = 1 << 30;

// ---------------------------------------------------------------- dims / layouts
struct Dims {
  int L = 0, Q1 = 0;
  std::vector<int> v;  // (L+1) * Q1
  int operator()(int b, int q) const { return (q < 0 || q >= Q1) ? 0 : v[size_t(b) * Q1 + q]; }
  int& at(int b, int q) { return v[size_t(b) * Q1 + q]; }
  int bond(int b) const {
    int s = 0;
    for (int q = 0; q < Q1; ++q) s += v[size_t(b) * Q1 + q];
    return s;
  }
};

// offsets (in z) of site k's pieces for the given bond dims
struct SiteLayout {
  std::vector<long> lmat;   // [q'] offset of Lmat_q' (-1 if empty)
  std::vector<int> lrows;   // [q'] rows of Lmat_q'
  std::vector<int> rowoff;  // [q' * p + n] row of segment n inside Lmat_q' (-1 absent)
  long size = 0;
  // block (q, n): offset and leading dimension (= cols)
  long blk(int q, int n, int p, const Dims& d, int k, int* ld = nullptr) const {
    const int qq = q + n;
    if (qq >= int(lmat.size()) || lmat[qq] < 0 || rowoff[qq * p + n] < 0 || d(k - 1, q) == 0) return -1;
    const int c = d(k, qq);
    if (ld) *ld = c;
    return lmat[qq] + long(rowoff[qq * p + n]) * c;
  }
};
static SiteLayout site_layout(const Dims& d, int k, int p) {
  SiteLayout s;
  const int Q1 = d.Q1;
  s.lmat.assign(Q1, -1);
  s.lrows.assign(Q1, 0);
  s.rowoff.assign(size_t(Q1) * p, -1);
  long off = 0;
  for (int qq = 0; qq < Q1; ++qq) {
    const int c = d(k, qq);
    int r = 0;
    for (int n = 0; n < p; ++n) {
      const int dl = d(k - 1, qq - n);
      if (dl > 0) { s.rowoff[qq * p + n] = r; r += dl; }
    }
    s.lrows[qq] = r;
    if (c > 0 && r > 0) { s.lmat[qq] = off; off += long(r) * c; }
  }
  s.size = off;
  return s;
}

// ---------------------------------------------------------------- device buffers
template <class T>
struct DBuf {
  T* p = nullptr;
  size_t cap = 0;
  void reserve(size_t n) {
    if (n <= cap) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    HCKA(hipMalloc(&p, sizeof(T) * n));
    cap = n;
  }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
};

// ---------------------------------------------------------------- MPS objects
// A view of an MPS: bond dims + the device address of every site.
struct View {
  const Dims* d = nullptr;
  std::array<z*, 64> site{};
};

// Chain: an MPS being propagated, two buffers per site (the new layout of a
// site is written to its other buffer, then the two are swapped).
struct Chain {
  Dims dims;
  std::vector<z*> buf[2];
  std::vector<int> cur;
  bool wide = false;
  z* site(int k) const { return buf[cur[k]][k]; }
  z* other(int k) const { return buf[1 - cur[k]][k]; }
  void flip(int k) { cur[k] ^= 1; }
  View view() const {
    View v;
    v.d = &dims;
    for (size_t k = 1; k < cur.size(); ++k) v.site[k] = site(int(k));
    return v;
  }
};

// Stored state (trajectory slot): contiguous sites in site order.
struct State {
  Dims dims;
  z* data = nullptr;
  std::vector<long> off;  // [k] site offset
  View view() const {
    View v;
    v.d = &dims;
    for (size_t k = 1; k < off.size(); ++k) v.site[k] = data + off[k];
    return v;
  }
};

// ---------------------------------------------------------------- engine
struct Engine {
  // model
  int L, p, Q, Q1;
  double J, dt, cutoff;
  int maxm;
  int device;
  std::vector<int> gate_i1;
  std::vector<double> dH;
  std::vector<int> md;   // (L+1)*Q1 Schmidt-rank bound per sector
  std::vector<int> mdz;  // inside the dH zip-up: min(HS_left, 2 min(HS_left, HS_right))
  std::vector<long long> hs_bond;  // total Hilbert-space bound per bond
  // capacities (complex elements per site) of normal and wide (dH zip-up) chains
  std::vector<int> bcap, bcapw;  // per bond
  std::vector<long> scap, scapw;
  long state_cap = 0;
  // device
  hipStream_t st = nullptr;
  GateConst gcst{};
  DBuf<z> d_gf, d_gb;
  DBuf<z> chain_pool, chain_pool_w;
  int nchain_cap = 0, nchain_cap_w = 0;
  std::vector<int> free_chain, free_chain_w;
  std::vector<std::unique_ptr<Chain>> chains;  // index = pool slot (normal), wide ones separate
  std::vector<std::unique_ptr<Chain>> chains_w;
  DBuf<z> heap;             // stored states
  size_t heap_slots = 0;
  std::vector<State> states;  // [slot]
  // stats
  double gemm_flops = 0, gemm_bytes = 0, gemm_ms = 0;
  long gemm_launches = 0;
  // OCG_GEMM_STATS=1: shape statistics of the GEMM launches, printed at destruction (diagnostic)
  bool gstat = std::getenv("OCG_GEMM_STATS") != nullptr;
  long eig_hist[34] = {0};  // Gram block orders in bins of 16 (OCG_GEMM_STATS)
  double gs_pad = 0, gs_iss = 0, gs_flop = 0, gs_tiles_hist[6] = {0}, gs_flop_m[6] = {0}, gs_flop_k[6] = {0};
  long gs_launch_hist[6] = {0};
  double gs_ms[6] = {0}, gs_bflop[6] = {0}, gs_ntask[6] = {0}, gs_nseg[6] = {0}, gs_m[6] = {0}, gs_n[6] = {0}, gs_k[6] = {0};
  std::vector<int> gs_evb;  // bucket of each pending gemm_ev pair
  // OCG_GEMM_STATS: eigensolver stream time (Gram done -> eigenvectors queued) of gauge moves
  // (cutoff <= 1e-13, no Maxm) and of the other decompositions
  struct EigEv { hipEvent_t a, b; int gauge; };
  std::vector<EigEv> eig_ev;
  double eig_ms[2] = {0, 0};
  long eig_calls[2] = {0, 0};
  static int gs_bucket(double x) { return x < 32 ? 0 : x < 64 ? 1 : x < 128 ? 2 : x < 256 ? 3 : x < 512 ? 4 : 5; }
  std::vector<std::pair<hipEvent_t, hipEvent_t>> gemm_ev;
  std::vector<hipEvent_t> ev_pool;
  hipEvent_t ev_kept = nullptr;
  // certified gauge moves (fast_certify / fast_factors); OCG_HBM_FASTGAUGE=0: eigen path only
  bool fast_gauge = !(std::getenv("OCG_HBM_FASTGAUGE") && std::getenv("OCG_HBM_FASTGAUGE")[0] == '0');
  DBuf<z> eye;  // kCholMax x kCholMax identity (ld kCholMax)
  long fast_moves[2] = {0, 0};  // certified / fell back to the eigen path (OCG_GEMM_STATS)
  // side stream: the blocked large-order eigenvalue kernel runs beside the other blocks' kernel
  hipStream_t st2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // smallest Gram order on the register eigensolver (OCG_HBM_REGMIN overrides: A/B and tests)
  int reg_min = kRegMin;
  // smallest Gram order on the blocked kernel k_heev_vals_big (default: the orders the register
  // kernels cannot hold); OCG_HBM_BIGMIN overrides (tests; > kBigMax: the eager L2 kernel, A/B)
  int big_min = std::getenv("OCG_HBM_BIGMIN") ? std::atoi(std::getenv("OCG_HBM_BIGMIN")) : RNMAX + 1;
  // Gram orders coop_min..CPT on the multi-CU reduction k_heev_vals_coop (hbm_coop.hpp), G
  // workgroups per block, G picked per launch from the CUs the launch's blocks leave (results do
  // not depend on G).  OCG_HBM_COOP=0: off (the one-CU kernels above); OCG_HBM_COOPMIN=n: the
  // smallest order; OCG_HBM_COOPG=g: fixed G (A/B, tests); OCG_HBM_COOP_TMO: the bound on every
  // wait in s_memrealtime ticks (100 MHz; a group that gives up is re-run on one CU)
  bool coop_on = !(std::getenv("OCG_HBM_COOP") && std::getenv("OCG_HBM_COOP")[0] == '0');
  int coop_min = std::getenv("OCG_HBM_COOPMIN") ? std::atoi(std::getenv("OCG_HBM_COOPMIN")) : RNMAX + 1;
  int coop_g = std::getenv("OCG_HBM_COOPG") ? std::atoi(std::getenv("OCG_HBM_COOPG")) : 0;
  long long coop_tmo = std::getenv("OCG_HBM_COOP_TMO") ? std::atoll(std::getenv("OCG_HBM_COOP_TMO")) : 20000000LL;
  int n_cu = 256;
  DBuf<int> coop_fb;  // [0]: groups re-run on one CU (k_heev_vals_coop_fix), read by path_stats
  long coop_launches = 0, coop_groups = 0;
  // workgroups per block for a launch of nb blocks whose largest order is nmax
  int coop_members(int nb, int nmax) const {
    if (coop_g > 0) return std::min(coop_g, kCoopMaxG);
    const int gmax = std::max(1, std::min(8, nmax / 64));
    return std::max(1, std::min(gmax, n_cu / std::max(nb, 1)));
  }
  // Maxm-boundary eigenvalue resolution (k_heev_thresh + k_heev_bisect) for
  // register-path Gram blocks of order >= thresh_min; OCG_HBM_THRESH=1: on,
  // OCG_HBM_THRESH=n > 1: on from order n.  Off by default: at config 4 the two
  // extra launches per decomposition cost more than the shorter multisection
  // saves (c4rows N_t = 33: 2138 vs 2055 ms per getHessian)
  bool thresh_on = std::getenv("OCG_HBM_THRESH") && std::atoi(std::getenv("OCG_HBM_THRESH")) != 0;
  int thresh_min = (std::getenv("OCG_HBM_THRESH") && std::atoi(std::getenv("OCG_HBM_THRESH")) > 1)
                       ? std::atoi(std::getenv("OCG_HBM_THRESH"))
                       : 48;
  // register-path Gram blocks of order >= split_min leave their multisection to
  // k_heev_bisect_split (split_spe eigenvalues per workgroup on many CUs);
  // OCG_HBM_SPLITMIN=n moves the threshold, 0 turns it off
  int split_min = std::getenv("OCG_HBM_SPLITMIN") ? std::atoi(std::getenv("OCG_HBM_SPLITMIN")) : 96;
  // eigenvalues per k_heev_bisect_split workgroup (RNT / split_spe threads each): 8, 16 or 32
  int split_spe = [] {
    const int v = std::getenv("OCG_HBM_SPLIT_SPE") ? std::atoi(std::getenv("OCG_HBM_SPLIT_SPE")) : 16;
    return (v == 8 || v == 16 || v == 32) ? v : 16;
  }();
  // shifts per thread and multisection round (EProb::ks): 1 = bisection (default), 4 = round 5's
  int bisect_ks = std::getenv("OCG_HBM_BISECT_KS") && std::atoi(std::getenv("OCG_HBM_BISECT_KS")) == 4 ? 4 : 1;
  long split_launches = 0, split_blocks = 0;
  // the split runs while its workgroups number at most split_max_wg per CU (OCG_HBM_SPLIT_WG)
  int split_max_wg = std::getenv("OCG_HBM_SPLIT_WG") ? std::atoi(std::getenv("OCG_HBM_SPLIT_WG")) : 2;
  double phase_ms[8] = {0};
  long phase_n[8] = {0};
  double steps_done[8] = {0};

  Engine(int device_, int L_, int p_, int npart, double J_, double dt_, double cutoff_, int maxm_)
      : L(L_), p(p_), Q(npart), Q1(npart + 1), J(J_), dt(dt_), cutoff(cutoff_),
        maxm(maxm_ > 0 ? maxm_ : 5000), device(device_) {}
  ~Engine() {
    if (gstat && gemm_launches) {
      if (st) (void)hipStreamSynchronize(st);
      resolve_timers();
      std::fprintf(stderr, "[gemm] launches %ld  alg/padded flops %.3f  alg/issued (live 16x16 units) %.3f\n", gemm_launches,
                   gs_flop / std::max(gs_pad, 1.0), gs_flop / std::max(gs_iss, 1.0));
      const char* lb[6] = {"<32", "<64", "<128", "<256", "<512", ">=512"};
      for (int b = 0; b < 6; ++b)
        std::fprintf(stderr, "[gemm] %-6s launches(tiles/8) %ld  tiles %.0f  ms %.1f  TF %.2f  flop share by max(m,n) %.3f  by k %.3f\n", lb[b],
                     gs_launch_hist[b], gs_tiles_hist[b], gs_ms[b], gs_bflop[b] / std::max(gs_ms[b], 1e-9) * 1e-9, gs_flop_m[b] / std::max(gs_flop, 1.0),
                     gs_flop_k[b] / std::max(gs_flop, 1.0));
      for (int b = 0; b < 6; ++b)
        if (gs_ntask[b] > 0)
          std::fprintf(stderr, "[gemm] %-6s tasks/launch %.1f  segs/task %.2f  avg m %.1f n %.1f k/seg %.1f\n", lb[b],
                       gs_ntask[b] / std::max<long>(gs_launch_hist[b], 1), gs_nseg[b] / gs_ntask[b], gs_m[b] / gs_ntask[b],
                       gs_n[b] / gs_ntask[b], gs_k[b] / std::max(gs_nseg[b], 1.0));
    }
    if (gstat) {
      std::fprintf(stderr, "[step] host ms over %ld gates: theta+gate queued %.1f, two-site decomposition %.1f, gauge moves %.1f, "
                   "gate sync %.1f; waits: certificate %.1f (%ld), eigen kept counts %.1f (%ld)\n", phase_n[0], phase_ms[0],
                   phase_ms[1], phase_ms[2], phase_ms[3], phase_ms[4], phase_n[1], phase_ms[5], phase_n[2]);
      std::fprintf(stderr, "[eig] stream ms: gauge moves %.1f (%ld calls), other decompositions %.1f (%ld calls); "
                   "certified gauge moves %ld, fell back %ld\n",
                   eig_ms[1], eig_calls[1], eig_ms[0], eig_calls[0], fast_moves[0], fast_moves[1]);
      long tot = 0;
      for (long v : eig_hist) tot += v;
      std::fprintf(stderr, "[eig] Gram blocks %ld by order:", tot);
      for (int b = 0; b < 34; ++b)
        if (eig_hist[b]) std::fprintf(stderr, " %d-%d:%ld", 16 * b, 16 * b + 15, eig_hist[b]);
      std::fprintf(stderr, "\n");
    }
    for (auto& e : ev_pool) (void)hipEventDestroy(e);
    for (auto& e : gemm_ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    if (ev_kept) (void)hipEventDestroy(ev_kept);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (st2) (void)hipStreamDestroy(st2);
    if (st) (void)hipStreamDestroy(st);
  }

  // stream priority: 1 high (the context engine, the dH worker: the rows'
  // critical path), -1 low (the pipelined getHessian's xi worker, whose
  // states are needed only by the closing overlap pass), 0 default.  The
  // three engines of the pipelined getHessian share the CUs; with the xi
  // worker's launches behind the critical path's the getHessian is faster
  // (same results bit for bit: the engines hand states over through counters).
  int prio_level = 0;
  hipError_t create_stream(hipStream_t* s, bool side = false) const {
    // OCG_HBM_PRIO: 3 (default) the main streams of the context engine and the dH
    // worker high, their side streams default, both xi-worker streams low; 1 the
    // side streams high as well; 2 only the xi worker low; 0 every stream default.
    // Measured (round 4, one box per row, results bitwise the same in every mode):
    // c4rows 3 -> 1670-1706 ms, 2 -> 1694-1758 ms, 0 -> 1856-2200 ms;
    // c5rows 3 / 1 -> 11.60-12.28 s, 2 -> 13.19-15.98 s, 0 -> 15.12-20.79 s.
    static const int mode = std::getenv("OCG_HBM_PRIO") ? std::atoi(std::getenv("OCG_HBM_PRIO")) : 3;
    if (mode != 0 && prio_level != 0 && !(mode == 2 && prio_level > 0) && !(mode == 3 && side && prio_level > 0)) {
      int least = 0, greatest = 0;
      if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
        return hipStreamCreateWithPriority(s, hipStreamNonBlocking, prio_level > 0 ? greatest : least);
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  }
  // ------------------------------------------------------------ setup
  void init(const std::vector<int>& md_in, const std::vector<int>& mdz_in, const std::vector<double>& gf,
            const std::vector<double>& gb, const int* glo, const int* gsz, const int* goff, int gtotal,
            const std::vector<int>& gates) {
    HCK(hipSetDevice(device));
    if (const char* e = std::getenv("OCG_HBM_REGMIN")) reg_min = std::max(2, std::atoi(e));
    thost.pinned = true;
    // both streams here, one after the other: which streams share a hardware queue
    // (GPU_MAX_HW_QUEUES) follows the creation order, and a side stream created on
    // first use landed on the pipeline's queues differently depending on whether the
    // engine had stepped before (c4rows 2.08 s vs 1.68-1.70 s, same results)
    HCK(create_stream(&st));
    HCK(create_stream(&st2, true));
    HCK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&ev_kept, hipEventDisableTiming));
    {
      int ncu = 0;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0) n_cu = ncu;
      coop_fb.reserve(1);
      HCK(hipMemsetAsync(coop_fb.p, 0, sizeof(int), st));  // ordered before every side-stream launch (ev_fork)
    }
    {
      std::vector<z> I(size_t(kCholMax) * kCholMax, mk(0, 0));
      for (int i = 0; i < kCholMax; ++i) I[size_t(i) * kCholMax + i] = mk(1, 0);
      eye.reserve(I.size());
      HCK(hipMemcpy(eye.p, I.data(), sizeof(z) * I.size(), hipMemcpyHostToDevice));
    }
    md = md_in;
    mdz = mdz_in;
    gate_i1 = gates;
    dH.resize(p);
    for (int n = 0; n < p; ++n) dH[n] = 0.5 * n * (n - 1);
    set_gates(gf, gb, glo, gsz, goff, gtotal);
    // bond capacities: Maxm (or the Hilbert-space bound) total per bond
    hs_bond.assign(L + 1, 0);
    for (int b = 0; b <= L; ++b) {
      long long s = 0;
      for (int q = 0; q < Q1; ++q) s += md[size_t(b) * Q1 + q];
      hs_bond[b] = s;
    }
    set_caps(0);
  }
  void set_gates(const std::vector<double>& gf, const std::vector<double>& gb, const int* glo, const int* gsz,
                 const int* goff, int gtotal) {
    gcst.p = p;
    gcst.Q1 = Q1;
    for (int D = 0; D < 24; ++D) { gcst.glo[D] = glo[D]; gcst.gsz[D] = gsz[D]; gcst.goff[D] = goff[D]; }
    d_gf.reserve(gtotal);
    d_gb.reserve(gtotal);
    sync();  // set_tstep: queued steps may still read the old gates
    HCK(hipMemcpyAsync(d_gf.p, gf.data(), sizeof(z) * gtotal, hipMemcpyHostToDevice, st));
    HCK(hipMemcpyAsync(d_gb.p, gb.data(), sizeof(z) * gtotal, hipMemcpyHostToDevice, st));
    sync();
  }
  // per-bond capacities from max(Maxm, widest state seen), capped by the
  // Hilbert-space bound; chains and the state heap are sized from them
  int widest = 0;
  void set_caps(int wider) {
    widest = std::max(widest, wider);
    const long long want = std::max<long long>(maxm, widest);
    std::vector<int> bc(L + 1), bw(L + 1);
    for (int b = 0; b <= L; ++b) {
      bc[b] = int(std::min<long long>(hs_bond[b], want));
      bw[b] = (b == 0 || b == L) ? bc[b] : 2 * bc[b];  // the zip-up doubles every inner bond
    }
    if (bc == bcap && bw == bcapw) return;
    // existing chains / states keep their buffers only if nothing grew
    if (!chains.empty() || !chains_w.empty() || !states.empty()) {
      bool grew = false;
      for (int b = 0; b <= L; ++b)
        if (bcap.size() && (bc[b] > bcap[b] || bw[b] > bcapw[b])) grew = true;
      if (grew) throw Error(2, "state wider than the engine capacity fixed at ocg_set_states");
      return;
    }
    bcap = bc;
    bcapw = bw;
    scap.assign(L + 1, 0);
    scapw.assign(L + 1, 0);
    state_cap = 0;
    for (int k = 1; k <= L; ++k) {
      scap[k] = std::max<long>(1, long(bcap[k - 1]) * bcap[k]);
      scapw[k] = std::max<long>(1, long(bcapw[k - 1]) * bcapw[k]);
      state_cap += scap[k];
    }
  }
  long chain_elems(bool wide) const {
    long s = 0;
    for (int k = 1; k <= L; ++k) s += 2 * (wide ? scapw[k] : scap[k]);
    return s;
  }
  size_t mps_max_nelem() const { return size_t(state_cap); }

  // ------------------------------------------------------------ chains
  void reserve_chains(int n, bool wide) {
    auto& pool = wide ? chain_pool_w : chain_pool;
    auto& capn = wide ? nchain_cap_w : nchain_cap;
    auto& vec = wide ? chains_w : chains;
    auto& fr = wide ? free_chain_w : free_chain;
    if (n <= capn) return;
    if (capn > 0) {
      // grow: keep it simple, every chain must be free (batches allocate at their start)
      if (int(fr.size()) != capn) throw Error(4, "internal: chain pool grown while chains are in use");
      sync();
    }
    const long per = chain_elems(wide);
    pool.reserve(size_t(per) * n);
    vec.clear();
    fr.clear();
    for (int i = 0; i < n; ++i) {
      auto c = std::make_unique<Chain>();
      c->wide = wide;
      c->buf[0].assign(L + 1, nullptr);
      c->buf[1].assign(L + 1, nullptr);
      c->cur.assign(L + 1, 0);
      z* b = pool.p + size_t(per) * i;
      for (int k = 1; k <= L; ++k) {
        const long sc = wide ? scapw[k] : scap[k];
        c->buf[0][k] = b; b += sc;
        c->buf[1][k] = b; b += sc;
      }
      vec.push_back(std::move(c));
      fr.push_back(n - 1 - i);
    }
    capn = n;
  }
  Chain* acquire(bool wide) {
    auto& fr = wide ? free_chain_w : free_chain;
    if (fr.empty()) throw Error(4, "internal: chain pool exhausted");
    const int i = fr.back();
    fr.pop_back();
    Chain* c = (wide ? chains_w : chains)[i].get();
    std::fill(c->cur.begin(), c->cur.end(), 0);
    return c;
  }
  void release(Chain* c) {
    auto& vec = c->wide ? chains_w : chains;
    for (size_t i = 0; i < vec.size(); ++i)
      if (vec[i].get() == c) { (c->wide ? free_chain_w : free_chain).push_back(int(i)); return; }
  }
  // Give the pool back down to n chains (every chain must be free): after a failed
  // call that grew it, so that the path the caller retries sees that memory free.
  void shrink_chains(int n) {
    if (n >= nchain_cap) return;
    if (int(free_chain.size()) != nchain_cap) throw Error(4, "internal: chain pool shrunk while chains are in use");
    sync();
    if (chain_pool.p) (void)hipFree(chain_pool.p);
    chain_pool.p = nullptr;
    chain_pool.cap = 0;
    chains.clear();
    free_chain.clear();
    nchain_cap = 0;
    if (n > 0) reserve_chains(n, false);
  }
  // Chains are held only inside one entry point: after a failed call every
  // chain is free again (the error path of guard()).
  void release_all() {
    free_chain.clear();
    free_chain_w.clear();
    for (int i = nchain_cap - 1; i >= 0; --i) free_chain.push_back(i);
    for (int i = nchain_cap_w - 1; i >= 0; --i) free_chain_w.push_back(i);
  }

  // ------------------------------------------------------------ states
  void reserve_states(size_t nslots) {
    if (nslots <= heap_slots) return;
    // keep the contents: copy into the new heap
    DBuf<z> nh;
    nh.reserve(size_t(state_cap) * nslots);
    if (heap_slots) HCK(hipMemcpyAsync(nh.p, heap.p, sizeof(z) * state_cap * heap_slots, hipMemcpyDeviceToDevice, st));
    sync();
    std::swap(heap.p, nh.p);
    std::swap(heap.cap, nh.cap);
    for (size_t s = 0; s < states.size(); ++s) states[s].data = heap.p + size_t(state_cap) * s;
    states.resize(nslots);
    for (size_t s = heap_slots; s < nslots; ++s) {
      states[s].data = heap.p + size_t(state_cap) * s;
      states[s].dims.L = L;
      states[s].dims.Q1 = Q1;
      states[s].dims.v.assign(size_t(L + 1) * Q1, 0);
      states[s].off.assign(L + 1, 0);
    }
    heap_slots = nslots;
  }
  // Give back the slots past nslots (after a call that needed many extra
  // trajectories): the first nslots keep their contents.
  void shrink_states(size_t nslots) {
    if (nslots >= heap_slots) return;
    sync();
    DBuf<z> nh;
    nh.reserve(size_t(state_cap) * std::max<size_t>(nslots, 1));
    if (nslots) HCK(hipMemcpyAsync(nh.p, heap.p, sizeof(z) * state_cap * nslots, hipMemcpyDeviceToDevice, st));
    sync();
    std::swap(heap.p, nh.p);
    std::swap(heap.cap, nh.cap);
    states.resize(nslots);
    for (size_t s = 0; s < nslots; ++s) states[s].data = heap.p + size_t(state_cap) * s;
    heap_slots = nslots;
  }
  double heap_bytes() const { return 16.0 * double(state_cap) * double(heap_slots); }
  void set_state_layout(State& s) {
    long o = 0;
    for (int k = 1; k <= L; ++k) {
      s.off[k] = o;
      o += site_layout(s.dims, k, p).size;
    }
    if (o > state_cap) throw Error(2, "state exceeds the slot capacity");
  }

  // ------------------------------------------------------------ arenas
  // Workspace and task uploads are bump-allocated from chunked arenas (device
  // blocks, pinned host staging) and recycled at every stream
  // synchronisation: nothing queued can still read them then.  Chunks are
  // kept across phases, so steady-state allocation is free.
  struct Arena {
    std::vector<std::pair<char*, size_t>> blk;
    size_t bi = 0, top = 0;
    bool pinned = false;
    bool same_va = true;  // pinned chunks: the device reads them at the host address
    char* get(size_t bytes) {
      bytes = (bytes + 255) & ~size_t(255);
      while (bi < blk.size() && top + bytes > blk[bi].second) { ++bi; top = 0; }
      if (bi == blk.size()) {
        const size_t sz = std::max<size_t>(bytes, blk.empty() ? (size_t(8) << 20) : 2 * blk.back().second);
        char* ptr = nullptr;
        if (pinned) {
          // coherent (not cached by the device): small task lists are read in place
          HCKA(hipHostMalloc((void**)&ptr, sz, hipHostMallocCoherent));
          void* dp = nullptr;
          if (hipHostGetDevicePointer(&dp, ptr, 0) != hipSuccess || dp != ptr) same_va = false;
        }
        else HCKA(hipMalloc((void**)&ptr, sz));
        blk.push_back({ptr, sz});
        top = 0;
      }
      char* r = blk[bi].first + top;
      top += bytes;
      return r;
    }
    void reset() { bi = 0; top = 0; }
    ~Arena() {
      for (auto& b : blk) {
        if (pinned) (void)hipHostFree(b.first);
        else (void)hipFree(b.first);
      }
    }
  };
  Arena work, tdev, thost;
  // error paths: wait for everything queued on this engine's streams (the side
  // stream's eigenvalue kernels read task lists and workspace the next call reuses)
  void drain() {
    (void)hipStreamSynchronize(st);
    if (st2) (void)hipStreamSynchronize(st2);
  }
  void sync() {
    HCK(hipStreamSynchronize(st));
    resolve_timers();
    work.reset();
    tdev.reset();
    thost.reset();
  }
  template <class T>
  T* walloc(size_t n) {
    return (T*)work.get(sizeof(T) * std::max<size_t>(n, 1));
  }
  // Task lists up to zc_max bytes are read by the kernels straight from
  // coherent pinned host memory (a few PCIe reads per workgroup) instead of
  // a host-to-device copy, which the stream serialises as one more blit
  // kernel before the launch; larger lists are copied.  The staging arena is
  // recycled only after a stream synchronisation, so nothing queued can still
  // read it.  OCG_HBM_ZC=bytes (0: always copy).
  // Gram orders <= kSmallMax on k_heev_vals_small beside the large-order kernel (OCG_HBM_SMALL=0: one launch)
  bool small_split = !(std::getenv("OCG_HBM_SMALL") && std::getenv("OCG_HBM_SMALL")[0] == '0');
  // k_gemm's XCD-grouped tile order (OCG_HBM_XCDMAP=0: dispatch order)
  bool xcd_map = !(std::getenv("OCG_HBM_XCDMAP") && std::getenv("OCG_HBM_XCDMAP")[0] == '0');
  size_t zc_max = std::getenv("OCG_HBM_ZC") ? size_t(std::atol(std::getenv("OCG_HBM_ZC"))) : size_t(16384);
  template <class T>
  const T* upload(const std::vector<T>& v) {
    if (v.empty()) return nullptr;
    const size_t bytes = sizeof(T) * v.size();
    char* h = thost.get(bytes);
    std::memcpy(h, v.data(), bytes);
    if (bytes <= zc_max && thost.same_va) return (const T*)h;
    char* d = tdev.get(bytes);
    HCK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
    return (const T*)d;
  }

  // three task arrays in one host-to-device copy (each 256-byte aligned)
  template <class A, class B, class C>
  void upload3(const std::vector<A>& a, const std::vector<B>& b, const std::vector<C>& c, const A*& da,
               const B*& db, const C*& dc) {
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t ba = sizeof(A) * a.size(), bb = sizeof(B) * b.size(), bc = sizeof(C) * c.size();
    const size_t oa = 0, ob = al(ba), oc = ob + al(bb), bytes = std::max<size_t>(oc + bc, 1);
    char* h = thost.get(bytes);
    if (ba) std::memcpy(h + oa, a.data(), ba);
    if (bb) std::memcpy(h + ob, b.data(), bb);
    if (bc) std::memcpy(h + oc, c.data(), bc);
    char* d = h;
    if (!(bytes <= zc_max && thost.same_va)) {
      d = tdev.get(bytes);
      HCK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
    }
    da = ba ? (const A*)(d + oa) : nullptr;
    db = bb ? (const B*)(d + ob) : nullptr;
    dc = bc ? (const C*)(d + oc) : nullptr;
  }

  // ------------------------------------------------------------ launches
  hipEvent_t get_event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    HCK(hipEventCreate(&e));
    return e;
  }
  void resolve_timers() {
    for (auto& e : eig_ev) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) eig_ms[e.gauge] += ms;
      ++eig_calls[e.gauge];
      ev_pool.push_back(e.a);
      ev_pool.push_back(e.b);
    }
    eig_ev.clear();
    for (size_t i = 0; i < gemm_ev.size(); ++i) {
      auto& pr = gemm_ev[i];
      float ms = 0;
      if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) gemm_ms += ms;
      if (gstat && i < gs_evb.size()) gs_ms[gs_evb[i]] += ms;
      ev_pool.push_back(pr.first);
      ev_pool.push_back(pr.second);
    }
    gemm_ev.clear();
    gs_evb.clear();
  }
  // GEMM tasks: drop empty outputs, prefix the tiles, account flops/bytes
  void gemm(std::vector<GTask>& tasks, const std::vector<GSeg>& segs) {
    const double f0 = gemm_flops;
    std::vector<GTask> t;
    t.reserve(tasks.size());
    int tiles = 0;
    for (auto& x : tasks) {
      if (x.m <= 0 || x.n <= 0) continue;
      x.tile0 = tiles;
      tiles += ((x.m + GT - 1) / GT) * ((x.n + GT - 1) / GT);
      for (int s = 0; s < x.nseg; ++s) {
        const GSeg& g = segs[x.seg0 + s];
        gemm_flops += 8.0 * x.m * x.n * g.k;
        if (gstat) {
          const double f = 8.0 * x.m * x.n * g.k;
          gs_flop += f;
          gs_pad += 8.0 * ((x.m + 31) / 32 * 32) * ((x.n + 31) / 32 * 32) * ((g.k + 3) / 4 * 4);
          gs_iss += 8.0 * ((x.m + 15) / 16 * 16) * ((x.n + 15) / 16 * 16) * ((g.k + 3) / 4 * 4);
          gs_flop_m[gs_bucket(std::max(x.m, x.n))] += f;
          gs_flop_k[gs_bucket(g.k)] += f;
        }
        gemm_bytes += 16.0 * (double(x.m) * g.k + double(g.k) * x.n);
      }
      gemm_bytes += 16.0 * x.m * x.n;
      t.push_back(x);
    }
    tasks.clear();
    if (t.empty()) return;
    if (gstat) {
      const int b = gs_bucket(tiles / 8.0);
      ++gs_launch_hist[b];
      gs_evb.push_back(b);
      gs_bflop[b] += gemm_flops - f0;
      gs_ntask[b] += t.size();
      for (auto& x : t) {
        gs_nseg[b] += x.nseg;
        gs_m[b] += x.m;
        gs_n[b] += x.n;
        for (int q = 0; q < x.nseg; ++q) gs_k[b] += segs[x.seg0 + q].k;
      }
      gs_tiles_hist[b] += tiles;
    }
    // per tile: its task and the task's first segment (-1: none)
    std::vector<int2> tmap(static_cast<size_t>(tiles));
    for (size_t i = 0; i < t.size(); ++i) {
      const int e = i + 1 < t.size() ? t[i + 1].tile0 : tiles;
      std::fill(tmap.begin() + t[i].tile0, tmap.begin() + e, make_int2(int(i), t[i].nseg > 0 ? t[i].seg0 : -1));
    }
    const GTask* dt_;
    const int2* dmap;
    const GSeg* ds;
    upload3(t, tmap, segs, dt_, dmap, ds);
    hipEvent_t a = get_event(), b = get_event();
    // start / stop events of the dispatch itself (not stream markers around it: with the
    // host building the next launch's tasks the stream idles between a marker and the kernel)
    hipExtLaunchKernelGGL(k_gemm, dim3(tiles), dim3(NT), 0, st, a, b, 0, dt_, dmap, ds, xcd_map ? 1 : 0);
    HCK(hipGetLastError());
    gemm_ev.push_back({a, b});
    ++gemm_launches;
  }
  void copy(std::vector<CTask>& tasks) {
    std::vector<CTask> t;
    long long tot = 0;
    for (auto& x : tasks) {
      if (x.rows <= 0 || x.cols <= 0) continue;
      x.e0 = tot;
      tot += (long long)x.rows * x.cols;
      t.push_back(x);
    }
    tasks.clear();
    if (t.empty()) return;
    const CTask* d = upload(t);
    const long long blocks = std::min<long long>((tot + NT - 1) / NT, 8192);
    hipLaunchKernelGGL(k_copy, dim3(unsigned(blocks)), dim3(NT), 0, st, d, int(t.size()), tot);
    HCK(hipGetLastError());
  }
  static CTask ctask(const z* src, z* dst, int rows, int cols, int lds, int ldd, int mode = 0) {
    CTask c{};
    c.src = src; c.dst = dst; c.rows = rows; c.cols = cols; c.lds = lds; c.ldd = ldd; c.mode = mode;
    c.f = mk(1, 0);
    return c;
  }
  static GTask gtask(z* C, int ldc, int m, int n, int seg0, int nseg) {
    GTask t{};
    t.C = C; t.ldc = ldc; t.m = m; t.n = n; t.seg0 = seg0; t.nseg = nseg;
    return t;
  }
  static GSeg gseg(const z* A, int lda, const z* B, int ldb, int k, int ops, double alpha = 1.0) {
    GSeg s{};
    s.A = A; s.B = B; s.lda = lda; s.ldb = ldb; s.k = k; s.ops = ops; s.alpha = alpha;
    return s;
  }

  // ------------------------------------------------------------ decomposition
  // One QN-blocked matrix per chain: sector q is R_q x C_q given as column
  // segments (each: pointer, leading dimension, width); rows contiguous.
  struct Seg {
    const z* ptr;
    int ld, c0, nc;
  };
  struct QMat {
    std::vector<int> R, C;
    std::vector<std::vector<Seg>> segs;  // [q]
  };
  // Result of one decomposition of one chain: per sector kept k_q and the
  // factors X (R x k, ld k) and Y (k x C, ld C), written where the caller
  // asked (dest pointers per sector; Y as column segments).
  struct Dest {
    std::vector<z*> X;                       // [q] (ld k_q); null: scratch
    std::vector<std::vector<z*>> Y;          // [q][seg] destination of Y's column segment (ld = segment width)
  };
  enum { kFromleft = 0, kFromright = 1 };

  struct DecompJob {
    QMat M;
    int dir;
    double cutoff;
    int maxm;
    int normalize;
    const int* bound;  // host array of per-sector bounds (Q1)
    // outputs (filled by decompose)
    std::vector<int> kept;
    std::vector<z*> X;  // scratch factors when no destination
    std::vector<z*> Y;
  };

  // Stage 1: Gram + eigenvalues + truncation; returns after the host knows
  // every kept count.  Stage 2 (factors) runs from decompose_factors.
  struct EigRun {
    std::vector<EProb> probs;
    std::vector<int> prob_job, prob_q;
    std::vector<int> side;  // per problem: 0 rows (M M^H), 1 cols (M^H M)
    int* d_kept = nullptr;
    double* d_keptw = nullptr;  // [job][2]
    std::vector<int> h_kept;
    std::vector<double> h_keptw;
    std::vector<int> job_p0;
    const EProb* d_probs = nullptr;
  };

  void decompose_eig(std::vector<DecompJob>& jobs, EigRun& R) {
    // problems and workspace
    size_t need = 0;
    for (auto& J : jobs)
      for (int q = 0; q < Q1; ++q) {
        const int Rq = J.M.R[q], Cq = J.M.C[q];
        if (Rq <= 0 || Cq <= 0) continue;
        const size_t n = size_t(std::min(Rq, Cq));
        need += (sizeof(z) * (2 * n * n + 2 * n) + sizeof(double) * (2 * n * n + 5 * n) + 4096);
      }
    need += sizeof(int) * 64 * (jobs.size() + 1) * Q1 + sizeof(double) * 2 * jobs.size() + 4096;
    R.probs.clear();
    R.prob_job.clear();
    R.prob_q.clear();
    R.side.clear();
    R.job_p0.assign(jobs.size() + 1, 0);
    int np = 0;
    for (size_t j = 0; j < jobs.size(); ++j) {
      R.job_p0[j] = np;
      for (int q = 0; q < Q1; ++q)
        if (jobs[j].M.R[q] > 0 && jobs[j].M.C[q] > 0) ++np;
    }
    R.job_p0[jobs.size()] = np;
    R.d_kept = walloc<int>(std::max(np, 1));
    R.d_keptw = walloc<double>(2 * std::max<size_t>(jobs.size(), 1));
    std::vector<GTask> gt;
    std::vector<GSeg> gs;
    std::vector<TItem> items;
    std::vector<int> bounds;
    bounds.reserve(np);
    int pi = 0;
    int maxn = 1, maxT = 0;
    for (size_t j = 0; j < jobs.size(); ++j) {
      DecompJob& J = jobs[j];
      int T = 0;
      for (int q = 0; q < Q1; ++q) {
        const int Rq = J.M.R[q], Cq = J.M.C[q];
        if (Rq <= 0 || Cq <= 0) continue;
        const int n = std::min(Rq, Cq);
        const int sd = Rq <= Cq ? 0 : 1;
        EProb P{};
        P.n = n;
        P.q = q;
        P.A = walloc<z>(size_t(n) * n);
        P.U = walloc<z>(size_t(n) * n);
        P.ph = walloc<z>(n);
        P.d = walloc<double>(n);
        P.e = walloc<double>(n);
        P.tau = walloc<double>(n);
        P.w = walloc<double>(n);
        P.Z = walloc<double>(size_t(n) * n);
        P.Dv = walloc<double>(size_t(n) * n);
        P.kept = R.d_kept + pi;
        P.ks = bisect_ks;
        R.probs.push_back(P);
        R.prob_job.push_back(int(j));
        R.prob_q.push_back(q);
        R.side.push_back(sd);
        bounds.push_back(J.bound[q]);
        maxn = std::max(maxn, n);
        T += n;
        // Gram: rows side G = M M^H = sum_seg S S^H; cols side G[seg a][seg b] = S_a^H S_b
        const auto& SG = J.M.segs[q];
        if (sd == 0) {
          const int s0 = int(gs.size());
          for (auto& s : SG) gs.push_back(gseg(s.ptr, s.ld, s.ptr, s.ld, s.nc, 2));
          gt.push_back(gtask(P.A, n, n, n, s0, int(SG.size())));
        } else {
          for (auto& a : SG)
            for (auto& b : SG) {
              const int s0 = int(gs.size());
              gs.push_back(gseg(a.ptr, a.ld, b.ptr, b.ld, Rq, 1));
              gt.push_back(gtask(P.A + size_t(a.c0) * n + b.c0, n, a.nc, b.nc, s0, 1));
            }
        }
        ++pi;
      }
      if (T > kMaxEig) throw Error(2, "decomposition with more eigenvalues than k_truncate holds");
      // unresolved eigenvalues of every sector stay below 1e-3 cutoff total / T in sum
      for (int i = R.job_p0[j]; i < pi; ++i) R.probs[i].thr_rel = J.cutoff > 1e-12 ? 1e-3 * J.cutoff / T : 0.0;
      maxT = std::max(maxT, T);
      TItem I{};
      I.p0 = R.job_p0[j];
      I.np = R.job_p0[j + 1] - R.job_p0[j];
      I.cutoff = J.cutoff;
      I.maxm = J.maxm;
      I.normalize = J.normalize;
      I.kept = R.d_kept + I.p0;
      I.keptw = R.d_keptw + 2 * j;
      items.push_back(I);
    }
    if (np == 0) {
      for (auto& J : jobs) J.kept.assign(Q1, 0);
      return;
    }
    gemm(gt, gs);
    hipEvent_t eva = nullptr;
    if (gstat) {
      eva = get_event();
      HCK(hipEventRecord(eva, st));
    }
    // OCG_HBM_THRESH: Maxm boundary first (k_heev_thresh), then only the
    // eigenvalues above it (k_heev_bisect) for the register-path sectors of
    // decompositions in which Maxm can bind
    std::vector<int> thr_items, deferred;
    int max_def = 0;
    if (thresh_on) {
      for (size_t j = 0; j < jobs.size(); ++j) {
        int T = 0;
        for (int i = R.job_p0[j]; i < R.job_p0[j + 1]; ++i) T += R.probs[i].n;
        if (T <= jobs[j].maxm + 1) continue;
        bool any = false;
        for (int i = R.job_p0[j]; i < R.job_p0[j + 1]; ++i) {
          const int n = R.probs[i].n;
          if (n >= std::max(reg_min, thresh_min) && n <= RNMAX && n < big_min) {
            R.probs[i].defer = 1;
            deferred.push_back(i);
            max_def = std::max(max_def, n);
            any = true;
          }
        }
        if (any) thr_items.push_back(int(j));
      }
    }
    // large register-path blocks: the tridiagonal in k_heev_vals_any, the
    // eigenvalues split over workgroups (k_heev_bisect_split) right after it
    // Only while the split's workgroups fit about two per CU: a launch with many
    // large blocks (the full-horizon row batches) already fills the GPU, and the
    // split's g threads per eigenvalue would only add Sturm work there.
    std::vector<int> split;
    int max_split = 0;
    if (!thresh_on && split_min > 0) {
      long ntask = 0;
      for (int i = 0; i < np; ++i) {
        const int n = R.probs[i].n;
        const bool other = (coop_on && n >= std::max(coop_min, 65) && n <= CPT) ||
                           (n >= std::max(big_min, 2) && n <= kBigMax) || (small_split && n <= kSmallMax);
        if (!other && n >= std::max(split_min, reg_min) && n <= RNMAX) {
          split.push_back(i);
          max_split = std::max(max_split, n);
          ntask += (n + split_spe - 1) / split_spe;
        }
      }
      if (ntask > long(split_max_wg) * n_cu) split.clear();
      for (int i : split) R.probs[i].defer = 1;
    }
    R.d_probs = upload(R.probs);
    // bounds: device copy, then point the items at it
    const int* d_bounds = upload(bounds);
    for (auto& I : items) I.bound = d_bounds + I.p0;
    const TItem* d_items = upload(items);
    // eigenvalues: blocks of order kRegMin..RNMAX on the register kernel,
    // the rest on the LDS / L2 kernel (LDS: 3 complex + 2 real vectors, plus
    // the Gram block if small)
    {
      // one launch: per block the register variant for its order (or the LDS / L2
      // kernel), largest blocks first; dynamic LDS = max over the variants present
      // orders big_min <= n <= kBigMax: the blocked reduction (k_heev_vals_big)
      // orders <= kSmallMax: k_heev_vals_small on the side stream (several workgroups per CU)
      std::vector<int> order, big, small, coop;
      for (int i = 0; i < np; ++i) {
        const int n = R.probs[i].n;
        if (coop_on && n >= std::max(coop_min, 65) && n <= CPT) coop.push_back(i);
        else if (n >= std::max(big_min, 2) && n <= kBigMax) big.push_back(i);
        else if (small_split && n <= kSmallMax) small.push_back(i);
        else order.push_back(i);
      }
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return R.probs[a].n > R.probs[b].n; });
      std::stable_sort(small.begin(), small.end(), [&](int a, int b) { return R.probs[a].n > R.probs[b].n; });
      if (gstat)
        for (int i = 0; i < np; ++i) ++eig_hist[std::min(R.probs[i].n / 16, 33)];
      std::stable_sort(big.begin(), big.end(), [&](int a, int b) { return R.probs[a].n > R.probs[b].n; });
      std::stable_sort(coop.begin(), coop.end(), [&](int a, int b) { return R.probs[a].n > R.probs[b].n; });
      const bool side = !big.empty() || !small.empty() || !coop.empty();
      if (side) {  // on the side stream, after everything st has queued (incl. this upload)
        const int* dbig = upload(big);
        const int* dsmall = upload(small);
        const int* dcoop = upload(coop);
        int* dctl = coop.empty() ? nullptr : walloc<int>(size_t(kCoopCtl) * coop.size());
        HCK(hipEventRecord(ev_fork, st));
        HCK(hipStreamWaitEvent(st2, ev_fork, 0));
        if (!coop.empty()) {
          // largest blocks first in dispatch order; every group's control words zeroed
          const int nc = int(coop.size()), G = coop_members(nc, R.probs[coop[0]].n);
          HCK(hipMemsetAsync(dctl, 0, sizeof(int) * kCoopCtl * nc, st2));
          hipLaunchKernelGGL(k_heev_vals_coop, dim3(8 * G * ((nc + 7) / 8)), dim3(CPT), 0, st2, R.d_probs, dcoop, nc,
                             G, dctl, coop_tmo);
          hipLaunchKernelGGL(k_heev_vals_coop_fix, dim3(nc), dim3(VBG), 0, st2, R.d_probs, dcoop,
                             (const int*)dctl, coop_fb.p);
          ++coop_launches;
          coop_groups += nc;
        }
        if (!big.empty())
          hipLaunchKernelGGL(k_heev_vals_big, dim3(int(big.size())), dim3(VBG), 0, st2, R.d_probs, dbig);
        if (!small.empty()) {
          int lds_s = 64;
          for (int i : small) {
            const int n = R.probs[i].n;
            lds_s = std::max(lds_s, n >= reg_min ? reg_lds_bytes(reg_grid(n)) : 64 * n + 16 * n * n + 64);
          }
          hipLaunchKernelGGL(k_heev_vals_small, dim3(int(small.size())), dim3(RNT), lds_s, st2, R.d_probs, dsmall,
                             reg_min);
        }
        HCK(hipGetLastError());
        HCK(hipEventRecord(ev_join, st2));
      }
      int lds_v = 64;
      for (int i : order) {
        const int n = R.probs[i].n;
        lds_v = std::max(lds_v, (n >= reg_min && n <= RNMAX) ? reg_lds_bytes(reg_grid(n))
                                                              : 64 * n + (n <= kLdsOrder ? 16 * n * n : 0) + 64);
      }
      if (!order.empty()) {
        hipLaunchKernelGGL(k_heev_vals_any, dim3(int(order.size())), dim3(RNT), lds_v, st, R.d_probs, upload(order),
                           reg_min);
        HCK(hipGetLastError());
      }
      if (!split.empty()) {
        std::vector<int2> tasks;
        for (int i : split)
          for (int c = 0; split_spe * c < R.probs[i].n; ++c) tasks.push_back(make_int2(i, c));
        // one completion counter per problem of the decomposition (k_heev_bisect_split's last-workgroup fill)
        int* dctr = walloc<int>(size_t(np));
        HCK(hipMemsetAsync(dctr, 0, sizeof(int) * size_t(np), st));
        hipLaunchKernelGGL(k_heev_bisect_split, dim3(int(tasks.size())), dim3(RNT), bisect_split_lds_bytes(max_split),
                           st, R.d_probs, upload(tasks), split_spe, dctr);
        HCK(hipGetLastError());
        ++split_launches;
        split_blocks += long(split.size());
      }
      if (!thr_items.empty()) {
        // the boundary counts read every sector's tridiagonal, the blocked kernel's too
        if (side) HCK(hipStreamWaitEvent(st, ev_join, 0));
        hipLaunchKernelGGL(k_heev_thresh, dim3(int(thr_items.size())), dim3(THN), thresh_lds_bytes(), st, d_items,
                           upload(thr_items), const_cast<EProb*>(R.d_probs));
        hipLaunchKernelGGL(k_heev_bisect, dim3(int(deferred.size())), dim3(BSN), bisect_lds_bytes(max_def), st,
                           R.d_probs, upload(deferred));
        HCK(hipGetLastError());
      }
      if (side) HCK(hipStreamWaitEvent(st, ev_join, 0));  // join before the truncation
    }
    int maxnp = 0;
    for (auto& I : items) maxnp = std::max(maxnp, I.np);
    hipLaunchKernelGGL(k_truncate, dim3(int(items.size())), dim3(TNT), truncate_lds(maxnp), st, d_items, R.d_probs);
    HCK(hipGetLastError());
    R.h_kept.assign(np, 0);
    R.h_keptw.assign(2 * jobs.size(), 0.0);
    // into pinned staging (asynchronous copies; pageable memory would block here)
    int* hk = (int*)thost.get(sizeof(int) * np);
    double* hw = (double*)thost.get(sizeof(double) * 2 * jobs.size());
    HCK(hipMemcpyAsync(hk, R.d_kept, sizeof(int) * np, hipMemcpyDeviceToHost, st));
    HCK(hipMemcpyAsync(hw, R.d_keptw, sizeof(double) * 2 * jobs.size(), hipMemcpyDeviceToHost, st));
    HCK(hipEventRecord(ev_kept, st));
    // eigenvectors of the kept eigenvalues (reads the kept counts on the device)
    hipLaunchKernelGGL(k_heev_vecs_reg, dim3(np), dim3(VNT), 0, st, R.d_probs, np);
    HCK(hipGetLastError());
    {
      // back-transformation of the larger problems (kept counts known on the device only:
      // every 16-column block a problem of this order could keep; the others exit at once)
      std::vector<int2> bt;
      for (int i = 0; i < np; ++i) {
        const int n = R.probs[i].n;
        if (n > 64 && n <= kBtRows)
          for (int cb = 0; 16 * cb < n; ++cb) bt.push_back(make_int2(i, cb));
      }
      if (!bt.empty()) {
        hipLaunchKernelGGL(k_heev_bt, dim3(int(bt.size())), dim3(BNT), 0, st, R.d_probs, upload(bt));
        HCK(hipGetLastError());
      }
    }
    if (gstat) {
      hipEvent_t evb = get_event();
      HCK(hipEventRecord(evb, st));
      const int gauge = jobs[0].cutoff <= 1e-13 && jobs[0].maxm >= kNoMaxm ? 1 : 0;
      eig_ev.push_back({eva, evb, gauge});
    }
    {
      const auto t0 = std::chrono::steady_clock::now();
      HCK(hipEventSynchronize(ev_kept));
      if (gstat) phase_ms[5] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      ++phase_n[2];
      std::memcpy(R.h_kept.data(), hk, sizeof(int) * np);
      std::memcpy(R.h_keptw.data(), hw, sizeof(double) * 2 * jobs.size());
    }
    for (size_t j = 0; j < jobs.size(); ++j) {
      jobs[j].kept.assign(Q1, 0);
      for (int i = R.job_p0[j]; i < R.job_p0[j + 1]; ++i) jobs[j].kept[R.prob_q[i]] = R.h_kept[i];
    }
    (void)maxT;
  }

  // Factors of every job: X (R x k) and Y (k x C) per sector.  xdst[j][q]:
  // destination of X (ld k) or null (scratch allocated here, returned in
  // job.X); ydst[j][q][seg]: destination of Y's column segment (ld = its
  // width) or empty (scratch, job.Y with ld C).
  void decompose_factors(std::vector<DecompJob>& jobs, EigRun& R, const std::vector<std::vector<z*>>& xdst,
                         const std::vector<std::vector<std::vector<z*>>>& ydst) {
    std::vector<GTask> gt;
    std::vector<GSeg> gs;
    std::vector<CTask> ct;
    for (size_t j = 0; j < jobs.size(); ++j) {
      DecompJob& J = jobs[j];
      J.X.assign(Q1, nullptr);
      J.Y.assign(Q1, nullptr);
      const double* inv = R.d_keptw + 2 * j + 1;
      for (int i = R.job_p0[j]; i < R.job_p0[j + 1]; ++i) {
        const int q = R.prob_q[i], k = J.kept[q];
        if (k <= 0) continue;
        const EProb& P = R.probs[i];
        const int Rq = J.M.R[q], Cq = J.M.C[q];
        const auto& SG = J.M.segs[q];
        z* X = (xdst.size() > j && xdst[j][q]) ? xdst[j][q] : walloc<z>(size_t(Rq) * k);
        J.X[q] = X;
        const bool ysplit = ydst.size() > j && !ydst[j][q].empty();
        z* Ys = ysplit ? nullptr : walloc<z>(size_t(k) * Cq);
        J.Y[q] = Ys;
        auto ydest = [&](size_t s, int& ld) -> z* {
          if (ysplit) { ld = SG[s].nc; return ydst[j][q][s]; }
          ld = Cq;
          return Ys + SG[s].c0;
        };
        if (R.side[i] == 0) {
          // U: eigenvectors of M M^H (R x k).  X = U [Fromright: * sigma inv]
          CTask c = ctask(P.U, X, Rq, k, k, k);
          if (J.dir == kFromright) { c.cs = P.w; c.smode = 1 << 2; c.sc = inv; }
          ct.push_back(c);
          // Y = U^H M [Fromleft: * inv; Fromright: / sigma per row], per column segment
          for (size_t s = 0; s < SG.size(); ++s) {
            int ld;
            z* Yd = ydest(s, ld);
            const int s0 = int(gs.size());
            gs.push_back(gseg(P.U, k, SG[s].ptr, SG[s].ld, Rq, 1));
            GTask t = gtask(Yd, ld, k, SG[s].nc, s0, 1);
            if (J.dir == kFromleft) t.sc = inv;
            else { t.rs = P.w; t.smode = 2; }
            gt.push_back(t);
          }
        } else {
          // W: eigenvectors of M^H M (C x k).  Y = W^H [Fromleft: * sigma inv]
          for (size_t s = 0; s < SG.size(); ++s) {
            int ld;
            z* Yd = ydest(s, ld);
            CTask c = ctask(P.U + size_t(SG[s].c0) * k, Yd, k, SG[s].nc, k, ld, 1);
            if (J.dir == kFromleft) { c.rs = P.w; c.smode = 1; c.sc = inv; }
            ct.push_back(c);
          }
          // X = M W [Fromleft: / sigma per column; Fromright: * inv]
          const int s0 = int(gs.size());
          for (auto& s : SG) gs.push_back(gseg(s.ptr, s.ld, P.U + size_t(s.c0) * k, k, s.nc, 0));
          GTask t = gtask(X, k, Rq, k, s0, int(SG.size()));
          if (J.dir == kFromleft) { t.cs = P.w; t.smode = 2 << 2; }
          else t.sc = inv;
          gt.push_back(t);
        }
      }
    }
    copy(ct);
    gemm(gt, gs);
  }

  // ------------------------------------------------------------ certified gauge moves
  // A gauge move keeps every Gram eigenvalue when the smallest exceeds
  // 10 x cutoff x total (hbm_eig.hpp, k_chol_cert); then it is factored by
  // CholeskyQR2 of the tall orientation T of each sector block M (R x C):
  //   Fromleft  (orthonormal X): R <= C: X = I, Y = M;  else T = M:
  //             X1 = M R1^-1, X = X1 R2^-1, Y = R2 R1
  //   Fromright (orthonormal rows Y): C <= R: Y = I, X = M;  else T = M^H:
  //             Q1 = M^H R1^-1, Q = Q1 R2^-1, Y = Q^H, X = (R2 R1)^H
  // with R1 from the Gram block on the small side (G1 = T^H T) and R2 from
  // G2 = T1^H T1 of the first pass.  Same state and bond dims as the eigen
  // path, a different (unobservable) gauge.
  struct FastRun {
    std::vector<int> job_p0, prob_q;
    std::vector<CholProb> probs;
    double* d_res = nullptr;
    std::vector<double> h_res;
  };
  // Gram block of sector q of M into G (n x n): rows side M M^H if R <= C, else M^H M
  void gram_tasks(const QMat& M, int q, z* G, std::vector<GTask>& gt, std::vector<GSeg>& gs) {
    const int Rq = M.R[q], Cq = M.C[q], n = std::min(Rq, Cq);
    const auto& SG = M.segs[q];
    if (Rq <= Cq) {
      const int s0 = int(gs.size());
      for (auto& sg : SG) gs.push_back(gseg(sg.ptr, sg.ld, sg.ptr, sg.ld, sg.nc, 2));
      gt.push_back(gtask(G, n, n, n, s0, int(SG.size())));
    } else {
      for (auto& a : SG)
        for (auto& b : SG) {
          const int s0 = int(gs.size());
          gs.push_back(gseg(a.ptr, a.ld, b.ptr, b.ld, Rq, 1));
          gt.push_back(gtask(G + size_t(a.c0) * n + b.c0, n, a.nc, b.nc, s0, 1));
        }
    }
  }
  // Cholesky factors of the problems' blocks, results read back to the host
  void chol_run(std::vector<CholProb>& probs, std::vector<double>& h_res, double* d_res) {
    hipLaunchKernelGGL(k_chol_cert, dim3(int(probs.size())), dim3(NT), 0, st, upload(probs));
    HCK(hipGetLastError());
    h_res.assign(2 * probs.size(), 0.0);
    // into pinned staging (an asynchronous copy; pageable memory would block here)
    double* hp = (double*)thost.get(sizeof(double) * h_res.size());
    HCK(hipMemcpyAsync(hp, d_res, sizeof(double) * h_res.size(), hipMemcpyDeviceToHost, st));
    HCK(hipEventRecord(ev_kept, st));
    const auto t0 = std::chrono::steady_clock::now();
    HCK(hipEventSynchronize(ev_kept));
    if (gstat) phase_ms[4] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ++phase_n[1];
    std::memcpy(h_res.data(), hp, sizeof(double) * h_res.size());
  }
  // per job: certified (kept = full rank per sector, F holds R1 / R1^-1) or
  // not (nothing of it changed: the eigen path).  Decided per chain from its
  // own blocks, so every batching takes the same path for it.
  std::vector<char> fast_certify(std::vector<DecompJob>& jobs, FastRun& F) {
    std::vector<char> ok(jobs.size(), 0);
    F.job_p0.assign(jobs.size() + 1, 0);
    F.prob_q.clear();
    F.probs.clear();
    int np = 0;
    for (size_t j = 0; j < jobs.size(); ++j) {
      F.job_p0[j] = np;
      bool fits = true;
      int nj = 0;
      for (int q = 0; q < Q1; ++q) {
        const int Rq = jobs[j].M.R[q], Cq = jobs[j].M.C[q];
        if (Rq <= 0 || Cq <= 0) continue;
        if (std::min(Rq, Cq) > kCholMax || std::min(Rq, Cq) > jobs[j].bound[q]) fits = false;
        ++nj;
      }
      ok[j] = fits && nj > 0;
      if (ok[j]) np += nj;
    }
    F.job_p0[jobs.size()] = np;
    if (np == 0) return ok;
    F.d_res = walloc<double>(2 * size_t(np));
    std::vector<GTask> gt;
    std::vector<GSeg> gs;
    for (size_t j = 0; j < jobs.size(); ++j) {
      if (!ok[j]) continue;
      for (int q = 0; q < Q1; ++q) {
        const int Rq = jobs[j].M.R[q], Cq = jobs[j].M.C[q];
        if (Rq <= 0 || Cq <= 0) continue;
        const int n = std::min(Rq, Cq);
        CholProb P{};
        P.n = n;
        P.G = walloc<z>(size_t(n) * n);
        P.R = walloc<z>(size_t(n) * n);
        P.Ri = walloc<z>(size_t(n) * n);
        P.res = F.d_res + 2 * F.probs.size();
        gram_tasks(jobs[j].M, q, const_cast<z*>(P.G), gt, gs);
        F.probs.push_back(P);
        F.prob_q.push_back(q);
      }
    }
    gemm(gt, gs);
    chol_run(F.probs, F.h_res, F.d_res);
    for (size_t j = 0; j < jobs.size(); ++j) {
      if (!ok[j]) continue;
      double total = 0;
      for (int i = F.job_p0[j]; i < F.job_p0[j + 1]; ++i) total += F.h_res[2 * i];
      bool c = total > 0;
      for (int i = F.job_p0[j]; i < F.job_p0[j + 1]; ++i) {
        const double inv2 = F.h_res[2 * i + 1];
        if (!(inv2 > 0) || !(1.0 > 10.0 * jobs[j].cutoff * total * inv2)) c = false;
      }
      ok[j] = c;
      if (!c) continue;
      jobs[j].kept.assign(Q1, 0);
      for (int i = F.job_p0[j]; i < F.job_p0[j + 1]; ++i) {
        const int q = F.prob_q[i];
        jobs[j].kept[q] = std::min(jobs[j].M.R[q], jobs[j].M.C[q]);
      }
    }
    return ok;
  }
  // the certified jobs' factors, into the destinations decompose_factors
  // would use.  The second pass cannot lose definiteness: the certificate
  // bounds cond(G1) by 1e13, so T1^H T1 = I + O(1e-3).
  void fast_factors(std::vector<DecompJob>& jobs, FastRun& F, const std::vector<char>& ok,
                    const std::vector<std::vector<z*>>& xdst,
                    const std::vector<std::vector<std::vector<z*>>>& ydst) {
    std::vector<GTask> gt;
    std::vector<GSeg> gs;
    std::vector<CTask> ct;
    std::vector<CholProb> p2;
    std::vector<int> p2_of(F.probs.size(), -1);
    std::vector<z*> T1(F.probs.size(), nullptr);
    // pass 1: T1 = T R1^-1 (Fromleft R x n, Fromright C x n), identity sectors done
    for (size_t j = 0; j < jobs.size(); ++j) {
      if (!ok[j]) continue;
      DecompJob& J = jobs[j];
      J.X.assign(Q1, nullptr);
      J.Y.assign(Q1, nullptr);
      for (int i = F.job_p0[j]; i < F.job_p0[j + 1]; ++i) {
        const int q = F.prob_q[i], Rq = J.M.R[q], Cq = J.M.C[q], n = F.probs[i].n;
        const auto& SG = J.M.segs[q];
        const bool left = J.dir == kFromleft, qr = left ? Rq > Cq : Cq > Rq;
        const bool ysplit = ydst.size() > j && !ydst[j][q].empty();
        z* X = (xdst.size() > j && xdst[j][q]) ? xdst[j][q] : nullptr;
        if (!qr) {
          if (left) {  // X = I (R x R), Y = M (the site itself: ld C, intact until the flip)
            if (!X) X = walloc<z>(size_t(Rq) * n);
            ct.push_back(ctask(eye.p, X, Rq, Rq, kCholMax, n));
            J.X[q] = X;
            J.Y[q] = const_cast<z*>(SG[0].ptr);
          } else {  // Y = I (C x C) by column segments, X = M (R x C, ld C)
            if (!X) X = walloc<z>(size_t(Rq) * n);
            z* Ys = ysplit ? nullptr : walloc<z>(size_t(n) * Cq);
            for (size_t sI = 0; sI < SG.size(); ++sI) {
              const int ld = ysplit ? SG[sI].nc : Cq;
              z* Yd = ysplit ? ydst[j][q][sI] : Ys + SG[sI].c0;
              ct.push_back(ctask(eye.p + SG[sI].c0, Yd, n, SG[sI].nc, kCholMax, ld));
              ct.push_back(ctask(SG[sI].ptr, X + SG[sI].c0, Rq, SG[sI].nc, SG[sI].ld, n));
            }
            J.X[q] = X;
            J.Y[q] = Ys;
          }
          continue;
        }
        const int m = left ? Rq : Cq;
        z* t1 = walloc<z>(size_t(m) * n);
        T1[i] = t1;
        if (left) {
          const int s0 = int(gs.size());
          gs.push_back(gseg(SG[0].ptr, SG[0].ld, F.probs[i].Ri, n, Cq, 0));
          gt.push_back(gtask(t1, n, Rq, n, s0, 1));
        } else {
          for (auto& sg : SG) {
            const int s0 = int(gs.size());
            gs.push_back(gseg(sg.ptr, sg.ld, F.probs[i].Ri, n, Rq, 1));
            gt.push_back(gtask(t1 + size_t(sg.c0) * n, n, sg.nc, n, s0, 1));
          }
        }
        CholProb P2{};
        P2.n = n;
        P2.G = walloc<z>(size_t(n) * n);
        P2.R = walloc<z>(size_t(n) * n);
        P2.Ri = walloc<z>(size_t(n) * n);
        p2_of[i] = int(p2.size());
        p2.push_back(P2);
      }
    }
    copy(ct);
    gemm(gt, gs);
    gs.clear();
    // pass 2: G2 = T1^H T1, R2, R2^-1
    if (!p2.empty()) {
      double* d_res2 = walloc<double>(2 * p2.size());
      for (size_t t = 0; t < p2.size(); ++t) p2[t].res = d_res2 + 2 * t;
      for (size_t i = 0; i < F.probs.size(); ++i) {
        if (p2_of[i] < 0) continue;  // (problems of uncertified jobs have none)
        const CholProb& P2 = p2[p2_of[i]];
        int jj = 0;
        while (F.job_p0[jj + 1] <= int(i)) ++jj;
        const int q = F.prob_q[i];
        const int m = jobs[jj].dir == kFromleft ? jobs[jj].M.R[q] : jobs[jj].M.C[q];
        const int s0 = int(gs.size());
        gs.push_back(gseg(T1[i], P2.n, T1[i], P2.n, m, 1));
        gt.push_back(gtask(const_cast<z*>(P2.G), P2.n, P2.n, P2.n, s0, 1));
      }
      gemm(gt, gs);
      gs.clear();
      // (no readback: the second pass cannot fail, see above)
      hipLaunchKernelGGL(k_chol_cert, dim3(int(p2.size())), dim3(NT), 0, st, upload(p2));
      HCK(hipGetLastError());
      // factors
      for (size_t j = 0; j < jobs.size(); ++j) {
        if (!ok[j]) continue;
        DecompJob& J = jobs[j];
        for (int i = F.job_p0[j]; i < F.job_p0[j + 1]; ++i) {
          if (p2_of[i] < 0) continue;
          const CholProb& P1 = F.probs[i];
          const CholProb& P2 = p2[p2_of[i]];
          const int q = F.prob_q[i], Rq = J.M.R[q], Cq = J.M.C[q], n = P1.n;
          const auto& SG = J.M.segs[q];
          z* X = (xdst.size() > j && xdst[j][q]) ? xdst[j][q] : walloc<z>(size_t(Rq) * n);
          J.X[q] = X;
          if (J.dir == kFromleft) {  // X = T1 R2^-1 (R x n), Y = R2 R1 (n x n = C)
            int s0 = int(gs.size());
            gs.push_back(gseg(T1[i], n, P2.Ri, n, n, 0));
            gt.push_back(gtask(X, n, Rq, n, s0, 1));
            z* Ys = walloc<z>(size_t(n) * Cq);
            s0 = int(gs.size());
            gs.push_back(gseg(P2.R, n, P1.R, n, n, 0));
            gt.push_back(gtask(Ys, Cq, n, n, s0, 1));
            J.Y[q] = Ys;
          } else {  // Q = T1 R2^-1 (C x n), Y = Q^H by column segments, X = R1^H R2^H (n x n = R)
            z* Q = walloc<z>(size_t(Cq) * n);
            int s0 = int(gs.size());
            gs.push_back(gseg(T1[i], n, P2.Ri, n, n, 0));
            gt.push_back(gtask(Q, n, Cq, n, s0, 1));
            s0 = int(gs.size());
            gs.push_back(gseg(P1.R, n, P2.R, n, n, 3));
            gt.push_back(gtask(X, n, n, n, s0, 1));
            const bool ysplit = ydst.size() > j && !ydst[j][q].empty();
            z* Ys = ysplit ? nullptr : walloc<z>(size_t(n) * Cq);
            for (size_t sI = 0; sI < SG.size(); ++sI) {
              const int ld = ysplit ? SG[sI].nc : Cq;
              z* Yd = ysplit ? ydst[j][q][sI] : Ys + SG[sI].c0;
              ct.push_back(ctask(Q + size_t(SG[sI].c0) * n, Yd, n, SG[sI].nc, n, ld, 1));
            }
            J.Y[q] = Ys;
          }
        }
      }
      gemm(gt, gs);
      copy(ct);
    }
  }

  // denmatDecomp(M, A, B, Fromleft, {Cutoff, Maxm}) of nm independent dense
  // blocks (one U(1) sector each): the decomposition path every two-site
  // update takes (Gram, eigenvalues, truncation, eigenvectors, factors), on
  // caller-supplied matrices.  A = U (R x k, orthonormal columns), B = U^H M
  // (k x C), w = the n = min(R, C) Gram eigenvalues as the eigensolver left
  // them (those below thr_rel * trace may be unresolved; see EProb).
  std::vector<int> decompose_dense(int nm, const int* rows, const int* cols, const double* const* M, double cutoff,
                                   int maxm, double* const* w, double* const* X, double* const* Y) {
    std::vector<DecompJob> jobs(static_cast<size_t>(nm));
    const std::vector<int> bnd(Q1, 1 << 30);
    for (int i = 0; i < nm; ++i) {
      const int r = rows[i], c = cols[i];
      z* d = walloc<z>(size_t(r) * c);
      HCK(hipMemcpyAsync(d, M[i], sizeof(z) * size_t(r) * c, hipMemcpyHostToDevice, st));
      QMat& Q = jobs[i].M;
      Q.R.assign(Q1, 0);
      Q.C.assign(Q1, 0);
      Q.segs.assign(Q1, {});
      Q.R[0] = r;
      Q.C[0] = c;
      Q.segs[0].push_back(Seg{d, c, 0, c});
      jobs[i].dir = kFromleft;
      jobs[i].cutoff = cutoff;
      jobs[i].maxm = maxm;
      jobs[i].normalize = 0;
      jobs[i].bound = bnd.data();
    }
    EigRun R;
    decompose_eig(jobs, R);
    decompose_factors(jobs, R, {}, {});
    std::vector<int> kept(static_cast<size_t>(nm), 0);
    for (int i = 0; i < nm; ++i) {
      const int k = jobs[i].kept[0], r = rows[i], c = cols[i];
      kept[i] = k;
      const EProb& P = R.probs[R.job_p0[i]];
      if (w && w[i]) HCK(hipMemcpyAsync(w[i], P.w, sizeof(double) * P.n, hipMemcpyDeviceToHost, st));
      if (k <= 0) continue;
      if (X && X[i]) HCK(hipMemcpyAsync(X[i], jobs[i].X[0], sizeof(z) * size_t(r) * k, hipMemcpyDeviceToHost, st));
      if (Y && Y[i]) HCK(hipMemcpyAsync(Y[i], jobs[i].Y[0], sizeof(z) * size_t(k) * c, hipMemcpyDeviceToHost, st));
    }
    sync();
    return kept;
  }

  // ------------------------------------------------------------ matricisations
  // Lmat of site k (rows (n, a), cols bond-k sector q): contiguous
  QMat lmat_of(const View& v, int k) const {
    const Dims& d = *v.d;
    SiteLayout sl = site_layout(d, k, p);
    QMat M;
    M.R.assign(Q1, 0);
    M.C.assign(Q1, 0);
    M.segs.assign(Q1, {});
    for (int q = 0; q < Q1; ++q) {
      if (sl.lmat[q] < 0) continue;
      M.R[q] = sl.lrows[q];
      M.C[q] = d(k, q);
      M.segs[q].push_back(Seg{v.site[k] + sl.lmat[q], d(k, q), 0, d(k, q)});
    }
    return M;
  }
  // Rmat of site k (rows bond k-1 sector q, cols (n, c)): blocks as segments
  QMat rmat_of(const View& v, int k) const {
    const Dims& d = *v.d;
    SiteLayout sl = site_layout(d, k, p);
    QMat M;
    M.R.assign(Q1, 0);
    M.C.assign(Q1, 0);
    M.segs.assign(Q1, {});
    for (int q = 0; q < Q1; ++q) {
      const int r = d(k - 1, q);
      if (r == 0) continue;
      int c = 0;
      for (int n = 0; n < p && q + n < Q1; ++n) {
        int ld;
        const long o = sl.blk(q, n, p, d, k, &ld);
        if (o < 0) continue;
        M.segs[q].push_back(Seg{v.site[k] + o, ld, c, ld});
        c += ld;
      }
      if (c == 0) { M.segs[q].clear(); continue; }
      M.R[q] = r;
      M.C[q] = c;
    }
    return M;
  }
  const int* bound_row(int b, bool zip) const { return (zip ? mdz.data() : md.data()) + size_t(b) * Q1; }

  // ------------------------------------------------------------ gauge moves
  // Decomposition of a batch of gauge-move jobs: the certified ones (fast_*,
  // when the move qualifies) and the eigen path for the others, each chain's
  // path decided from its own blocks.  layout(): the caller's destinations
  // from jobs[].kept, called once every kept count is known.
  template <class Layout>
  void decompose_gauge(std::vector<DecompJob>& jobs, double cut, int mm, const std::vector<std::vector<z*>>& xdst,
                       const std::vector<std::vector<std::vector<z*>>>& ydst, Layout layout) {
    std::vector<char> ok(jobs.size(), 0);
    FastRun F;
    if (fast_gauge && cut <= 1e-13 && mm >= kNoMaxm) ok = fast_certify(jobs, F);
    std::vector<int> eidx;
    for (size_t j = 0; j < jobs.size(); ++j)
      if (!ok[j]) eidx.push_back(int(j));
    if (gstat && fast_gauge && cut <= 1e-13 && mm >= kNoMaxm) {
      fast_moves[0] += long(jobs.size() - eidx.size());
      fast_moves[1] += long(eidx.size());
    }
    std::vector<DecompJob> sub;
    EigRun R;
    if (!eidx.empty()) {
      sub.reserve(eidx.size());
      for (int j : eidx) sub.push_back(jobs[j]);
      decompose_eig(sub, R);
      for (size_t t = 0; t < eidx.size(); ++t) jobs[eidx[t]].kept = sub[t].kept;
    }
    layout();
    if (eidx.size() < jobs.size()) fast_factors(jobs, F, ok, xdst, ydst);
    if (!eidx.empty()) {
      std::vector<std::vector<z*>> xs;
      std::vector<std::vector<std::vector<z*>>> ys;
      for (int j : eidx) {
        if (!xdst.empty()) xs.push_back(xdst[j]);
        if (!ydst.empty()) ys.push_back(ydst[j]);
      }
      decompose_factors(sub, R, xs, ys);
      for (size_t t = 0; t < eidx.size(); ++t) {
        jobs[eidx[t]].X = sub[t].X;
        jobs[eidx[t]].Y = sub[t].Y;
      }
    }
  }
  // MPS::position one site right / left for a batch (cutoff/maxm/normalize
  // as given; the gauge moves of doStep and exactApplyMPO use 1e-14, no Maxm).
  void move_right(std::vector<Chain*>& cs, int k, double cut, int mm, bool zip) {
    std::vector<DecompJob> jobs(cs.size());
    for (size_t i = 0; i < cs.size(); ++i) {
      jobs[i].M = lmat_of(cs[i]->view(), k);
      jobs[i].dir = kFromleft;
      jobs[i].cutoff = cut;
      jobs[i].maxm = mm;
      jobs[i].normalize = 0;
      jobs[i].bound = bound_row(k, zip);
    }
    // new bond k dims -> new layouts of sites k and k+1
    std::vector<std::vector<z*>> xdst(cs.size(), std::vector<z*>(Q1, nullptr));
    std::vector<Dims> nd(cs.size());
    auto layout = [&]() {
      for (size_t i = 0; i < cs.size(); ++i) {
        nd[i] = cs[i]->dims;
        for (int q = 0; q < Q1; ++q) nd[i].at(k, q) = jobs[i].kept[q];
        SiteLayout sl = site_layout(nd[i], k, p);
        for (int q = 0; q < Q1; ++q)
          xdst[i][q] = (jobs[i].kept[q] > 0 && sl.lmat[q] >= 0) ? cs[i]->other(k) + sl.lmat[q] : nullptr;
      }
    };
    decompose_gauge(jobs, cut, mm, xdst, {}, layout);
    // site k+1 <- Y * site k+1, block by block
    std::vector<GTask> gt;
    std::vector<GSeg> gs;
    for (size_t i = 0; i < cs.size(); ++i) {
      const Dims& od = cs[i]->dims;
      SiteLayout so = site_layout(od, k + 1, p), sn = site_layout(nd[i], k + 1, p);
      for (int q = 0; q < Q1; ++q) {
        const int kq = jobs[i].kept[q];
        if (kq <= 0) continue;
        for (int n = 0; n < p && q + n < Q1; ++n) {
          int ldo, ldn;
          const long oo = so.blk(q, n, p, od, k + 1, &ldo), on = sn.blk(q, n, p, nd[i], k + 1, &ldn);
          if (oo < 0 || on < 0) continue;
          const int s0 = int(gs.size());
          gs.push_back(gseg(jobs[i].Y[q], od(k, q), cs[i]->site(k + 1) + oo, ldo, od(k, q), 0));
          gt.push_back(gtask(cs[i]->other(k + 1) + on, ldn, kq, ldn, s0, 1));
        }
      }
    }
    gemm(gt, gs);
    for (size_t i = 0; i < cs.size(); ++i) {
      cs[i]->dims = nd[i];
      cs[i]->flip(k);
      cs[i]->flip(k + 1);
    }
  }
  void move_left(std::vector<Chain*>& cs, int k, double cut, int mm, bool zip) {
    std::vector<DecompJob> jobs(cs.size());
    for (size_t i = 0; i < cs.size(); ++i) {
      jobs[i].M = rmat_of(cs[i]->view(), k);
      jobs[i].dir = kFromright;
      jobs[i].cutoff = cut;
      jobs[i].maxm = mm;
      jobs[i].normalize = 0;
      jobs[i].bound = bound_row(k - 1, zip);
    }
    std::vector<std::vector<std::vector<z*>>> ydst(cs.size(), std::vector<std::vector<z*>>(Q1));
    std::vector<Dims> nd(cs.size());
    auto layout = [&]() {
      for (size_t i = 0; i < cs.size(); ++i) {
        nd[i] = cs[i]->dims;
        for (int q = 0; q < Q1; ++q) nd[i].at(k - 1, q) = jobs[i].kept[q];
        SiteLayout sl = site_layout(nd[i], k, p);
        for (int q = 0; q < Q1; ++q) {
          ydst[i][q].clear();
          if (jobs[i].kept[q] <= 0) continue;
          auto& segs = jobs[i].M.segs[q];
          // the segments are the blocks (q, n) with both dims nonzero, in n order
          for (int n = 0; n < p && q + n < Q1; ++n) {
            int ld;
            const long o = sl.blk(q, n, p, nd[i], k, &ld);
            if (o < 0) continue;
            ydst[i][q].push_back(cs[i]->other(k) + o);
          }
          if (ydst[i][q].size() != segs.size()) throw Error(4, "internal: right-matricisation segment mismatch");
        }
      }
    };
    decompose_gauge(jobs, cut, mm, {}, ydst, layout);
    // site k-1 <- site k-1 * X, block by block
    std::vector<GTask> gt;
    std::vector<GSeg> gs;
    for (size_t i = 0; i < cs.size(); ++i) {
      const Dims& od = cs[i]->dims;
      SiteLayout so = site_layout(od, k - 1, p), sn = site_layout(nd[i], k - 1, p);
      for (int ql = 0; ql < Q1; ++ql)
        for (int n = 0; n < p && ql + n < Q1; ++n) {
          const int q = ql + n, kq = jobs[i].kept[q];
          if (kq <= 0) continue;
          int ldo, ldn;
          const long oo = so.blk(ql, n, p, od, k - 1, &ldo), on = sn.blk(ql, n, p, nd[i], k - 1, &ldn);
          if (oo < 0 || on < 0) continue;
          const int s0 = int(gs.size());
          gs.push_back(gseg(cs[i]->site(k - 1) + oo, ldo, jobs[i].X[q], kq, ldo, 0));
          gt.push_back(gtask(cs[i]->other(k - 1) + on, ldn, od(k - 2, ql), kq, s0, 1));
        }
    }
    gemm(gt, gs);
    for (size_t i = 0; i < cs.size(); ++i) {
      cs[i]->dims = nd[i];
      cs[i]->flip(k);
      cs[i]->flip(k - 1);
    }
  }
  void position(std::vector<Chain*>& cs, int& centre, int target) {
    while (centre < target) { move_right(cs, centre, kGaugeCutoff, kNoMaxm, false); ++centre; }
    while (centre > target) { move_left(cs, centre, kGaugeCutoff, kNoMaxm, false); --centre; }
  }

  // ------------------------------------------------------------ site phases / norms
  // site k of every chain times ph(chain, n) (U gates; doStep :133-136, :222-223)
  void site_phase(std::vector<Chain*>& cs, int k, const std::vector<double>& u, const std::vector<double>& tau,
                  const std::vector<double>* inv_norm) {
    std::vector<CTask> ct;
    for (size_t i = 0; i < cs.size(); ++i) {
      const Dims& d = cs[i]->dims;
      SiteLayout sl = site_layout(d, k, p);
      for (int q = 0; q < Q1; ++q)
        for (int n = 0; n < p && q + n < Q1; ++n) {
          int ld;
          const long o = sl.blk(q, n, p, d, k, &ld);
          if (o < 0) continue;
          z* b = cs[i]->site(k) + o;
          CTask c = ctask(b, b, d(k - 1, q), ld, ld, ld);
          const double a = -0.25 * u[i] * tau[i] * n * (n - 1);
          c.f = gcst.imag ? mk(std::exp(a), 0.0) : mk(std::cos(a), std::sin(a));
          if (inv_norm) c.f = mk(c.f.x * (*inv_norm)[i], c.f.y * (*inv_norm)[i]);
          ct.push_back(c);
        }
    }
    copy(ct);
  }
  // |site k|^2 of every view (one reduction launch, host readback)
  // (k_sumsq: one workgroup per view, fixed summation order: deterministic)
  std::vector<double> site_norm2(const std::vector<View>& vs, int k) {
    if (vs.empty()) return {};
    double* acc = walloc<double>(vs.size());
    std::vector<CTask> ct;
    std::vector<int> t0(vs.size() + 1, 0);
    for (size_t i = 0; i < vs.size(); ++i) {
      const Dims& d = *vs[i].d;
      SiteLayout sl = site_layout(d, k, p);
      for (int q = 0; q < Q1; ++q) {
        if (sl.lmat[q] < 0 || sl.lrows[q] <= 0 || d(k, q) <= 0) continue;
        ct.push_back(ctask(vs[i].site[k] + sl.lmat[q], nullptr, sl.lrows[q], d(k, q), d(k, q), 0, 4));
      }
      t0[i + 1] = int(ct.size());
    }
    if (ct.empty()) ct.push_back(ctask(nullptr, nullptr, 0, 0, 0, 0, 4));  // every view empty: sums of nothing
    hipLaunchKernelGGL(k_sumsq, dim3(unsigned(vs.size())), dim3(NT), 0, st, upload(ct), upload(t0), acc);
    HCK(hipGetLastError());
    std::vector<double> h(vs.size());
    HCK(hipMemcpyAsync(h.data(), acc, sizeof(double) * vs.size(), hipMemcpyDeviceToHost, st));
    sync();
    return h;
  }

  // ------------------------------------------------------------ step
  // BH_tDMRG::step for a batch: chain i takes u_from[i] -> u_to[i] in
  // direction fwd[i] (src/BH_tDMRG.cpp:111-230, as the oracle restates it)
  void step(std::vector<Chain*>& cs, const std::vector<double>& uf, const std::vector<double>& ut,
            const std::vector<int>& fwd) {
    if (cs.empty()) return;
    const size_t B = cs.size();
    std::vector<double> tau(B);
    for (size_t i = 0; i < B; ++i) tau[i] = fwd[i] ? dt : -dt;
    if (L % 2 != 0) site_phase(cs, L, uf, tau, nullptr);  // lonely U_from on site L (:133-136)
    int centre = 1;
    bool fromLeft = true;
    const int ng = int(gate_i1.size());
    for (int g = 0; g < ng; ++g) {
      const int i1 = gate_i1[g], i2 = i1 + 1;
      const int mode = fromLeft ? 0 : 1;
      const bool lonely = fromLeft && i2 == L && L % 2 == 0;  // (:153-155)
      std::vector<ThetaJob> th(B);
      auto t0 = std::chrono::steady_clock::now();
      build_theta(cs, i1, th);
      apply_gate(cs, th, i1, uf, ut, tau, fwd, mode, lonely);
      auto t1 = std::chrono::steady_clock::now(), t2 = t1;
      if (g + 1 < ng) {
        const int ni1 = gate_i1[g + 1], ni2 = ni1 + 1;
        if (ni1 >= i2) {
          two_site(cs, th, i1, kFromleft);
          t2 = std::chrono::steady_clock::now();
          centre = i1 + 1;
          position(cs, centre, ni1);
        } else {
          two_site(cs, th, i1, kFromright);
          t2 = std::chrono::steady_clock::now();
          centre = i1;
          position(cs, centre, ni2);
        }
        if (i2 == ni1 || i1 == ni2) fromLeft = false;
      } else {
        two_site(cs, th, i1, kFromright);
        t2 = std::chrono::steady_clock::now();
        centre = i1;
        position(cs, centre, 1);
      }
      auto t3 = std::chrono::steady_clock::now();
      sync();
      if (gstat) {  // host wall per phase of the step (each ends at a stream synchronisation)
        auto t4 = std::chrono::steady_clock::now();
        phase_ms[0] += std::chrono::duration<double, std::milli>(t1 - t0).count();
        phase_ms[1] += std::chrono::duration<double, std::milli>(t2 - t1).count();
        phase_ms[2] += std::chrono::duration<double, std::milli>(t3 - t2).count();
        phase_ms[3] += std::chrono::duration<double, std::milli>(t4 - t3).count();
        ++phase_n[0];
      }
    }
    // U_to on site 1 (:222-223) and psi.normalize() (:228)
    std::vector<View> vs;
    for (auto* c : cs) vs.push_back(c->view());
    std::vector<double> n2 = site_norm2(vs, 1);
    std::vector<double> inv(B);
    for (size_t i = 0; i < B; ++i) inv[i] = n2[i] > 0 ? 1.0 / std::sqrt(n2[i]) : 1.0;
    site_phase(cs, 1, ut, tau, &inv);
    sync();
  }

  struct ThetaJob {
    z* th = nullptr;
    std::vector<long> thoff;
    std::vector<int> R, C, ro, co;  // ro/co: [q * p + n]
  };
  // Θ_q = Lmat(A_i1)_q * Rmat(A_i2)_q for every middle sector q (zero where
  // the middle sector is empty)
  void build_theta(std::vector<Chain*>& cs, int i1, std::vector<ThetaJob>& th) {
    size_t need = 0;
    for (size_t i = 0; i < cs.size(); ++i) {
      const Dims& d = cs[i]->dims;
      for (int q = 0; q < Q1; ++q) {
        long R = 0, C = 0;
        for (int n = 0; n < p; ++n) { R += d(i1 - 1, q - n); if (q + n < Q1) C += d(i1 + 1, q + n); }
        need += sizeof(z) * R * C + 256;
      }
    }
    std::vector<GTask> gt;
    std::vector<GSeg> gs;
    for (size_t i = 0; i < cs.size(); ++i) {
      const Dims& d = cs[i]->dims;
      ThetaJob& T = th[i];
      T.thoff.assign(Q1, 0);
      T.R.assign(Q1, 0);
      T.C.assign(Q1, 0);
      T.ro.assign(size_t(Q1) * p, -1);
      T.co.assign(size_t(Q1) * p, -1);
      long tot = 0;
      for (int q = 0; q < Q1; ++q) {
        int R = 0, C = 0;
        for (int n = 0; n < p; ++n) {
          if (d(i1 - 1, q - n) > 0) { T.ro[q * p + n] = R; R += d(i1 - 1, q - n); }
          if (q + n < Q1 && d(i1 + 1, q + n) > 0) { T.co[q * p + n] = C; C += d(i1 + 1, q + n); }
        }
        T.R[q] = R;
        T.C[q] = C;
        T.thoff[q] = tot;
        if (R > 0 && C > 0) tot += long(R) * C;
      }
      T.th = walloc<z>(std::max<long>(tot, 1));
      SiteLayout s1 = site_layout(d, i1, p), s2 = site_layout(d, i1 + 1, p);
      for (int q = 0; q < Q1; ++q) {
        if (T.R[q] == 0 || T.C[q] == 0) continue;
        const int m = d(i1, q);
        for (int n2 = 0; n2 < p && q + n2 < Q1; ++n2) {
          if (T.co[q * p + n2] < 0) continue;
          const int cw = d(i1 + 1, q + n2);
          z* out = T.th + T.thoff[q] + T.co[q * p + n2];
          int ld2;
          const long o2 = s2.blk(q, n2, p, d, i1 + 1, &ld2);
          if (m == 0 || s1.lmat[q] < 0 || o2 < 0) {
            gt.push_back(gtask(out, T.C[q], T.R[q], cw, 0, 0));  // zero block
            continue;
          }
          const int s0 = int(gs.size());
          gs.push_back(gseg(cs[i]->site(i1) + s1.lmat[q], m, cs[i]->site(i1 + 1) + o2, ld2, m, 0));
          gt.push_back(gtask(out, T.C[q], T.R[q], cw, s0, 1));
        }
      }
    }
    gemm(gt, gs);
  }
  void apply_gate(std::vector<Chain*>& cs, std::vector<ThetaJob>& th, int i1, const std::vector<double>& uf,
                  const std::vector<double>& ut, const std::vector<double>& tau, const std::vector<int>& fwd,
                  int mode, bool lonely) {
    std::vector<GateChain> gc(cs.size());
    std::vector<GateTask> tasks;
    std::vector<int> flat;
    std::vector<size_t> base(cs.size());
    long long tot = 0;
    for (size_t i = 0; i < cs.size(); ++i) {
      const ThetaJob& T = th[i];
      base[i] = flat.size();
      flat.resize(flat.size() + size_t(Q1) * (2 + 2 * p), -1);
      int* tb = flat.data() + base[i];
      for (int q = 0; q < Q1; ++q) {
        if (T.thoff[q] > (1L << 30)) throw Error(2, "Θ too large for 32-bit offsets");
        tb[q] = int(T.thoff[q]);
        tb[Q1 + q] = T.C[q];
      }
      for (int x = 0; x < Q1 * p; ++x) { tb[2 * Q1 + x] = T.ro[x]; tb[2 * Q1 + Q1 * p + x] = T.co[x]; }
      const Dims& d = cs[i]->dims;
      for (int ql = 0; ql < Q1; ++ql) {
        const int nl = d(i1 - 1, ql);
        if (nl == 0) continue;
        for (int D = 0; D <= 2 * (p - 1) && ql + D < Q1; ++D) {
          const int nr = d(i1 + 1, ql + D);
          if (nr == 0) continue;
          GateTask t{};
          t.chain = int(i);
          t.ql = ql;
          t.qr = ql + D;
          t.nl = nl;
          t.nr = nr;
          t.e0 = tot;
          tot += (long long)nl * nr;
          tasks.push_back(t);
        }
      }
    }
    if (tasks.empty()) return;
    const int* dflat = upload(flat);
    for (size_t i = 0; i < cs.size(); ++i) {
      GateChain& G = gc[i];
      G.th = th[i].th;
      G.tab = dflat + base[i];
      G.uf = uf[i];
      G.ut = ut[i];
      G.tau = tau[i];
      G.fwd = fwd[i];
      G.mode = mode;
      G.lonely = lonely ? 1 : 0;
    }
    const GateChain* dgc = upload(gc);
    const GateTask* dt_ = upload(tasks);
    const long long blocks = std::min<long long>((tot + NT - 1) / NT, 8192);
    hipLaunchKernelGGL(k_gate, dim3(unsigned(blocks)), dim3(NT), 0, st, dt_, int(tasks.size()), tot, dgc, gcst,
                       d_gf.p, d_gb.p);
    HCK(hipGetLastError());
  }

  // two-site decomposition of Θ into sites i1, i1+1 (denmatDecomp +
  // write-back + normalisation of the centre, :173-199 / :206-213)
  void two_site(std::vector<Chain*>& cs, std::vector<ThetaJob>& th, int i1, int dir) {
    std::vector<DecompJob> jobs(cs.size());
    for (size_t i = 0; i < cs.size(); ++i) {
      const ThetaJob& T = th[i];
      QMat& M = jobs[i].M;
      M.R = T.R;
      M.C = T.C;
      M.segs.assign(Q1, {});
      const Dims& d = cs[i]->dims;
      for (int q = 0; q < Q1; ++q) {
        if (T.R[q] == 0 || T.C[q] == 0) continue;
        // column segments n2 (for Y's write-back into site i1+1 blocks)
        for (int n2 = 0; n2 < p && q + n2 < Q1; ++n2) {
          if (T.co[q * p + n2] < 0) continue;
          const int w = d(i1 + 1, q + n2);
          M.segs[q].push_back(Seg{T.th + T.thoff[q] + T.co[q * p + n2], T.C[q], T.co[q * p + n2], w});
        }
      }
      jobs[i].dir = dir;
      jobs[i].cutoff = cutoff;
      jobs[i].maxm = maxm;
      jobs[i].normalize = 1;
      jobs[i].bound = bound_row(i1, false);
    }
    EigRun R;
    decompose_eig(jobs, R);
    std::vector<std::vector<z*>> xdst(cs.size(), std::vector<z*>(Q1, nullptr));
    std::vector<std::vector<std::vector<z*>>> ydst(cs.size(), std::vector<std::vector<z*>>(Q1));
    std::vector<Dims> nd(cs.size());
    for (size_t i = 0; i < cs.size(); ++i) {
      nd[i] = cs[i]->dims;
      for (int q = 0; q < Q1; ++q) nd[i].at(i1, q) = jobs[i].kept[q];
      SiteLayout s1 = site_layout(nd[i], i1, p), s2 = site_layout(nd[i], i1 + 1, p);
      for (int q = 0; q < Q1; ++q) {
        if (jobs[i].kept[q] <= 0) continue;
        if (s1.lmat[q] >= 0) xdst[i][q] = cs[i]->other(i1) + s1.lmat[q];
        for (int n2 = 0; n2 < p && q + n2 < Q1; ++n2) {
          if (th[i].co[q * p + n2] < 0) continue;
          int ld;
          const long o = s2.blk(q, n2, p, nd[i], i1 + 1, &ld);
          if (o < 0) throw Error(4, "internal: two-site write-back block missing");
          ydst[i][q].push_back(cs[i]->other(i1 + 1) + o);
        }
      }
    }
    decompose_factors(jobs, R, xdst, ydst);
    for (size_t i = 0; i < cs.size(); ++i) {
      cs[i]->dims = nd[i];
      cs[i]->flip(i1);
      cs[i]->flip(i1 + 1);
    }
  }

  // ------------------------------------------------------------ load / store
  void copy_sites(const View& src, const std::vector<z*>& dst, std::vector<CTask>& ct) {
    for (int k = 1; k <= L; ++k) {
      const long n = site_layout(*src.d, k, p).size;
      if (n <= 0) continue;
      // one row of n elements (k_copy tasks are 2-D; split long rows)
      const int W = 1 << 20;
      for (long o = 0; o < n; o += W) {
        const int w = int(std::min<long>(W, n - o));
        ct.push_back(ctask(src.site[k] + o, dst[k] + o, 1, w, w, w));
      }
    }
  }
  void load(Chain* c, const View& s) {
    c->dims = *s.d;
    std::fill(c->cur.begin(), c->cur.end(), 0);
    std::vector<CTask> ct;
    copy_sites(s, c->buf[0], ct);
    copy(ct);
  }
  void store(State& s, const Chain* c) {
    s.dims = c->dims;
    set_state_layout(s);
    std::vector<z*> dst(L + 1, nullptr);
    for (int k = 1; k <= L; ++k) dst[k] = s.data + s.off[k];
    std::vector<CTask> ct;
    copy_sites(c->view(), dst, ct);
    copy(ct);
  }
  void load_many(std::vector<Chain*>& cs, const std::vector<View>& vs) {
    std::vector<CTask> ct;
    for (size_t i = 0; i < cs.size(); ++i) {
      cs[i]->dims = *vs[i].d;
      std::fill(cs[i]->cur.begin(), cs[i]->cur.end(), 0);
      copy_sites(vs[i], cs[i]->buf[0], ct);
    }
    copy(ct);
  }
  void store_many(const std::vector<State*>& ss, const std::vector<Chain*>& cs) {
    std::vector<CTask> ct;
    for (size_t i = 0; i < cs.size(); ++i) {
      ss[i]->dims = cs[i]->dims;
      set_state_layout(*ss[i]);
      std::vector<z*> dst(L + 1, nullptr);
      for (int k = 1; k <= L; ++k) dst[k] = ss[i]->data + ss[i]->off[k];
      copy_sites(cs[i]->view(), dst, ct);
    }
    copy(ct);
  }

  // host interchange format (blocks (q, n) in (q, n) order) <-> device layout
  void upload_state(State& s, const int* dims, const double* data) {
    s.dims.L = L;
    s.dims.Q1 = Q1;
    s.dims.v.assign(dims, dims + size_t(L + 1) * Q1);
    int wid = 0;
    for (int b = 0; b <= L; ++b) wid = std::max(wid, s.dims.bond(b));
    set_caps(wid);
    set_state_layout(s);
    std::vector<z> buf(static_cast<size_t>(state_cap));
    size_t off = 0;
    for (int k = 1; k <= L; ++k) {
      SiteLayout sl = site_layout(s.dims, k, p);
      for (int q = 0; q < Q1; ++q)
        for (int n = 0; n < p && q + n < Q1; ++n) {
          const size_t cnt = size_t(s.dims(k - 1, q)) * s.dims(k, q + n);
          if (cnt == 0) continue;
          int ld;
          const long o = sl.blk(q, n, p, s.dims, k, &ld);
          for (size_t e = 0; e < cnt; ++e) buf[s.off[k] + o + e] = mk(data[2 * (off + e)], data[2 * (off + e) + 1]);
          off += cnt;
        }
    }
    HCK(hipMemcpyAsync(s.data, buf.data(), sizeof(z) * state_cap, hipMemcpyHostToDevice, st));
    sync();
  }
  size_t download_view(const View& v, int* dims, double* data, size_t cap) {
    const Dims& d = *v.d;
    size_t tot = 0;
    for (int k = 1; k <= L; ++k)
      for (int q = 0; q < Q1; ++q)
        for (int n = 0; n < p && q + n < Q1; ++n) tot += size_t(d(k - 1, q)) * d(k, q + n);
    if (tot > cap) return tot;
    std::memcpy(dims, d.v.data(), sizeof(int) * d.v.size());
    size_t off = 0;
    for (int k = 1; k <= L; ++k) {
      SiteLayout sl = site_layout(d, k, p);
      std::vector<z> h(std::max<long>(sl.size, 1));
      if (sl.size > 0) HCK(hipMemcpyAsync(h.data(), v.site[k], sizeof(z) * sl.size, hipMemcpyDeviceToHost, st));
      sync();
      for (int q = 0; q < Q1; ++q)
        for (int n = 0; n < p && q + n < Q1; ++n) {
          const size_t cnt = size_t(d(k - 1, q)) * d(k, q + n);
          if (cnt == 0) continue;
          int ld;
          const long o = sl.blk(q, n, p, d, k, &ld);
          for (size_t e = 0; e < cnt; ++e) {
            data[2 * (off + e)] = h[o + e].x;
            data[2 * (off + e) + 1] = h[o + e].y;
          }
          off += cnt;
        }
    }
    return tot;
  }

  // ------------------------------------------------------------ dH application
  // exactApplyMPO(propDeriv, psi) (src/OptimalControl.cpp:256, :302), as the
  // oracle restates it: bond-doubled exact MPO x MPS, gauge moves right with
  // the 1e-14 cutoff, then a right-to-left sweep truncating with the
  // stepper's Cutoff/Maxm.  Result right-orthonormal, centre site 1,
  // unnormalised; written into the normal chains `out`.
  void apply_dH(const std::vector<View>& in, std::vector<Chain*>& out) {
    const size_t B = in.size();
    reserve_chains(std::max<int>(nchain_cap_w, int(B)), true);
    std::vector<Chain*> w(B);
    for (size_t i = 0; i < B; ++i) w[i] = acquire(true);
    std::vector<CTask> ct;
    for (size_t i = 0; i < B; ++i) {
      const Dims& d = *in[i].d;
      Dims& f = w[i]->dims;
      f = d;
      for (int b = 1; b < L; ++b)
        for (int q = 0; q < Q1; ++q) f.at(b, q) = 2 * d(b, q);
      std::fill(w[i]->cur.begin(), w[i]->cur.end(), 0);
      for (int k = 1; k <= L; ++k) {
        SiteLayout sf = site_layout(f, k, p), sd = site_layout(d, k, p);
        if (sf.size > 0) {
          // zero fill, then the three placements of every block
          const int W = 1 << 20;
          for (long o = 0; o < sf.size; o += W) {
            const int wd = int(std::min<long>(W, sf.size - o));
            ct.push_back(ctask(nullptr, w[i]->site(k) + o, 1, wd, 0, wd, 2));
          }
        }
      }
    }
    copy(ct);
    for (size_t i = 0; i < B; ++i) {
      const Dims& d = *in[i].d;
      const Dims& f = w[i]->dims;
      for (int k = 1; k <= L; ++k) {
        SiteLayout sf = site_layout(f, k, p), sd = site_layout(d, k, p);
        for (int q = 0; q < Q1; ++q)
          for (int n = 0; n < p && q + n < Q1; ++n) {
            int lds, ldf;
            const long os = sd.blk(q, n, p, d, k, &lds), of = sf.blk(q, n, p, f, k, &ldf);
            if (os < 0 || of < 0) continue;
            const int dl = d(k - 1, q), dr = d(k, q + n);
            const bool lb = k == 1, rb = k == L;
            auto put = [&](int s, int t, double fac) {
              if (lb && s == 1) return;
              if (rb && t == 0) return;
              const int ro = lb ? 0 : s * dl, co = rb ? 0 : t * dr;
              CTask c = ctask(in[i].site[k] + os, w[i]->site(k) + of + long(ro) * ldf + co, dl, dr, lds, ldf);
              c.f = mk(fac, 0);
              ct.push_back(c);
            };
            put(0, 0, 1.0);
            if (dH[n] != 0.0) put(0, 1, dH[n]);
            put(1, 1, 1.0);
          }
      }
    }
    copy(ct);
    for (int k = 1; k < L; ++k) { move_right(w, k, kGaugeCutoff, kNoMaxm, true); sync(); }
    for (int k = L; k > 1; --k) { move_left(w, k, cutoff, maxm, false); sync(); }
    for (size_t i = 0; i < B; ++i) load(out[i], w[i]->view());
    sync();
    for (auto* c : w) release(c);
  }

  // ------------------------------------------------------------ overlaps
  // <x|y> (conj on x; overlapC) or <x| sum_k dH_k |y> per pair, batched:
  // transfer matrices E_k[q'] = sum_n X(q,n)^H (E_{k-1}[q] Y(q,n)), q' = q+n
  std::vector<std::complex<double>> overlaps(const std::vector<View>& xs, const std::vector<View>& ys, bool with_dH) {
    const size_t B = xs.size();
    std::vector<std::complex<double>> res(B, 0.0);
    if (B == 0) return res;
    // environments: E0 (nothing applied), E1 (dH applied once) per pair and sector
    struct Env {
      std::vector<z*> e0, e1;
    };
    std::vector<Env> cur(B), nxt(B);
    // workspace: environments of two consecutive bonds + T products
    size_t need = 0;
    for (size_t i = 0; i < B; ++i)
      for (int b = 0; b <= L; ++b) {
        size_t s = 0;
        for (int q = 0; q < Q1; ++q) s += size_t((*xs[i].d)(b, q)) * (*ys[i].d)(b, q);
        need = std::max(need, s);
      }
    // bond 0: E0 = [[1]] in sector 0, E1 = 0
    std::vector<CTask> ct;
    for (size_t i = 0; i < B; ++i) {
      cur[i].e0.assign(Q1, nullptr);
      cur[i].e1.assign(Q1, nullptr);
      z* one = walloc<z>(2);
      CTask c = ctask(nullptr, one, 1, 1, 0, 1, 8);  // fill with f = 1
      ct.push_back(c);
      cur[i].e0[0] = one;
      if (with_dH) {
        ct.push_back(ctask(nullptr, one + 1, 1, 1, 0, 1, 2));
        cur[i].e1[0] = one + 1;
      }
    }
    copy(ct);
    for (int k = 1; k <= L; ++k) {
      std::vector<GTask> gt;
      std::vector<GSeg> gs;
      // T0/T1[q][n] = E[q] Y(q, n)
      struct TT {
        std::vector<z*> t0, t1;
      };
      std::vector<TT> tt(B);
      for (size_t i = 0; i < B; ++i) {
        const Dims& dx = *xs[i].d;
        const Dims& dy = *ys[i].d;
        SiteLayout sy = site_layout(dy, k, p);
        tt[i].t0.assign(size_t(Q1) * p, nullptr);
        tt[i].t1.assign(size_t(Q1) * p, nullptr);
        for (int q = 0; q < Q1; ++q) {
          const int rx = dx(k - 1, q), ry = dy(k - 1, q);
          if (rx == 0 || ry == 0 || !cur[i].e0[q]) continue;
          for (int n = 0; n < p && q + n < Q1; ++n) {
            int ldy;
            const long oy = sy.blk(q, n, p, dy, k, &ldy);
            if (oy < 0 || dx(k, q + n) == 0) continue;
            z* t0 = walloc<z>(size_t(rx) * ldy);
            int s0 = int(gs.size());
            gs.push_back(gseg(cur[i].e0[q], ry, ys[i].site[k] + oy, ldy, ry, 0));
            gt.push_back(gtask(t0, ldy, rx, ldy, s0, 1));
            tt[i].t0[q * p + n] = t0;
            if (with_dH) {
              z* t1 = walloc<z>(size_t(rx) * ldy);
              s0 = int(gs.size());
              gs.push_back(gseg(cur[i].e1[q], ry, ys[i].site[k] + oy, ldy, ry, 0));
              gt.push_back(gtask(t1, ldy, rx, ldy, s0, 1));
              tt[i].t1[q * p + n] = t1;
            }
          }
        }
      }
      gemm(gt, gs);
      // E'[q'] = sum_n X(q'-n, n)^H T[q'-n][n]  (E1' also + dH[n] X^H T0)
      for (size_t i = 0; i < B; ++i) {
        const Dims& dx = *xs[i].d;
        const Dims& dy = *ys[i].d;
        SiteLayout sx = site_layout(dx, k, p);
        nxt[i].e0.assign(Q1, nullptr);
        nxt[i].e1.assign(Q1, nullptr);
        for (int qq = 0; qq < Q1; ++qq) {
          const int cx = dx(k, qq), cy = dy(k, qq);
          if (cx == 0 || cy == 0) continue;
          const int s0 = int(gs.size());
          int ns = 0;
          std::vector<GSeg> s1;
          for (int n = 0; n < p && qq - n >= 0; ++n) {
            const int q = qq - n;
            const z* t0 = tt[i].t0[q * p + n];
            if (!t0) continue;
            int ldx;
            const long ox = sx.blk(q, n, p, dx, k, &ldx);
            if (ox < 0) continue;
            const int rx = dx(k - 1, q);
            gs.push_back(gseg(xs[i].site[k] + ox, ldx, t0, cy, rx, 1));
            ++ns;
            if (with_dH) {
              s1.push_back(gseg(xs[i].site[k] + ox, ldx, tt[i].t1[q * p + n], cy, rx, 1));
              if (dH[n] != 0.0) s1.push_back(gseg(xs[i].site[k] + ox, ldx, t0, cy, rx, 1, dH[n]));
            }
          }
          if (ns == 0) continue;
          z* e0 = walloc<z>(size_t(cx) * cy);
          gt.push_back(gtask(e0, cy, cx, cy, s0, ns));
          nxt[i].e0[qq] = e0;
          if (with_dH) {
            z* e1 = walloc<z>(size_t(cx) * cy);
            const int s1b = int(gs.size());
            gs.insert(gs.end(), s1.begin(), s1.end());
            gt.push_back(gtask(e1, cy, cx, cy, s1b, int(s1.size())));
            nxt[i].e1[qq] = e1;
          }
        }
      }
      gemm(gt, gs);
      std::swap(cur, nxt);
    }
    std::vector<z> h(B, mk(0, 0));
    for (size_t i = 0; i < B; ++i) {
      const z* e = with_dH ? cur[i].e1[Q] : cur[i].e0[Q];
      if (e) HCK(hipMemcpyAsync(&h[i], e, sizeof(z), hipMemcpyDeviceToHost, st));
    }
    sync();
    for (size_t i = 0; i < B; ++i) res[i] = std::complex<double>(h[i].x, h[i].y);
    return res;
  }
};

}  // namespace hbm

// =====================================================================
// Entry points used by ocmps.hip (the C-ABI) — see hbm.hpp
// =====================================================================
using hbm::Chain;
using hbm::State;
using hbm::View;

struct hbm_engine {
  std::unique_ptr<hbm::Engine> E;
  // worker engines of the pipelined getHessian (own stream, arenas, chains; they
  // read and write E's state heap) and what they are built from
  std::unique_ptr<hbm::Engine> W[2];
  std::vector<int> md, mdz, gates;
  std::vector<double> gf, gb;
  int glo[24] = {0}, gsz[24] = {0}, goff[24] = {0}, gtotal = 0;
  long gates_version = 0, w_version[2] = {-1, -1};
  std::string err;
  int N = 0;
  bool have_states = false, have_psi = false, have_xi = false, have_xih = false;
  // state slots: 0 init, 1 target, 2.. scratch, then psi_t, xi_t, xiH_t
  int psi_base() const { return 4; }
  int xi_base() const { return 4 + N; }
  int xih_base() const { return 4 + 2 * N; }
  double ms[8] = {0};
  long launches[8] = {0};
  long steps[8] = {0};
  hipEvent_t e0 = nullptr, e1 = nullptr;
};

namespace {
int widest_of(const hbm::Engine& E, const int* dims) {
  int w = 0;
  for (int b = 0; b <= E.L; ++b) {
    int a = 0;
    for (int q = 0; q < E.Q1; ++q) a += dims[b * E.Q1 + q];
    w = std::max(w, a);
  }
  return w;
}
// Every entry point runs inside guard(): exceptions become status codes, and a
// failed call leaves no chain acquired (work already queued on the stream is
// drained first, so a later call cannot reuse a buffer a kernel still writes).
// Entry points that overwrite trajectory slots clear the matching have_* flags
// before they start and set them only on success.
template <class F>
int guard(hbm_engine* h, F f) {
  int rc = 0;
  try {
    HCK(hipSetDevice(h->E->device));
    f();
    return 0;
  } catch (const hbm::Error& e) {
    h->err = e.what();
    rc = e.code;
  } catch (const std::bad_alloc& e) {
    h->err = std::string("host allocation failed: ") + e.what();
    rc = 6;
  } catch (const std::exception& e) {
    h->err = e.what();
    rc = 3;
  }
  h->E->drain();
  h->E->release_all();
  for (auto& W : h->W)
    if (W) {
      W->drain();
      W->release_all();
    }
  return rc;
}
struct Timer {
  hbm_engine* h;
  int kind;
  Timer(hbm_engine* h_, int k) : h(h_), kind(k) { HCK(hipEventRecord(h->e0, h->E->st)); }
  void stop(long nsteps = 0) {
    HCK(hipEventRecord(h->e1, h->E->st));
    HCK(hipEventSynchronize(h->e1));
    float ms = 0;
    HCK(hipEventElapsedTime(&ms, h->e0, h->e1));
    h->ms[kind] += ms;
    h->launches[kind] += 1;
    h->steps[kind] += nsteps;
  }
};
}  // namespace

int hbm_create(int device, int L, int p, int npart, double J, double tstep, double cutoff, int maxm,
               const std::vector<int>& md, const std::vector<int>& mdz, const std::vector<double>& gf,
               const std::vector<double>& gb, const int* glo, const int* gsz, const int* goff, int gtotal,
               const std::vector<int>& gates, hbm_engine** out, std::string& err) {
  auto* h = new hbm_engine;
  h->E.reset(new hbm::Engine(device, L, p, npart, J, tstep, cutoff, maxm));
  h->E->prio_level = 1;
  h->md = md;
  h->mdz = mdz;
  h->gates = gates;
  h->gf = gf;
  h->gb = gb;
  for (int D = 0; D < 24; ++D) { h->glo[D] = glo[D]; h->gsz[D] = gsz[D]; h->goff[D] = goff[D]; }
  h->gtotal = gtotal;
  try {
    HCK(hipSetDevice(device));
    h->E->init(md, mdz, gf, gb, glo, gsz, goff, gtotal, gates);
    HCK(hipEventCreate(&h->e0));
    HCK(hipEventCreate(&h->e1));
  } catch (const hbm::Error& e) {
    err = e.what();
    delete h;
    return e.code;
  }
  *out = h;
  return 0;
}
void hbm_destroy(hbm_engine* h) {
  if (!h) return;
  (void)hipSetDevice(h->E->device);
  if (h->e0) (void)hipEventDestroy(h->e0);
  if (h->e1) (void)hipEventDestroy(h->e1);
  delete h;
}
const char* hbm_last_error(const hbm_engine* h) { return h->err.c_str(); }
size_t hbm_mps_max_nelem(const hbm_engine* h) { return h->E->mps_max_nelem(); }

int hbm_set_tstep(hbm_engine* h, double tstep, const std::vector<double>& gf, const std::vector<double>& gb,
                  const int* glo, const int* gsz, const int* goff, int gtotal) {
  return guard(h, [&] {
    h->E->dt = tstep;
    h->E->set_gates(gf, gb, glo, gsz, goff, gtotal);
    h->have_psi = h->have_xi = h->have_xih = false;
    h->gf = gf;
    h->gb = gb;
    ++h->gates_version;
  });
}

int hbm_swap_gates(hbm_engine* h, int imag, double tstep, const std::vector<double>& gf,
                   const std::vector<double>& gb, const int* glo, const int* gsz, const int* goff, int gtotal) {
  return guard(h, [&] {
    h->E->dt = tstep;
    h->E->set_gates(gf, gb, glo, gsz, goff, gtotal);
    h->E->gcst.imag = imag;
  });
}

int hbm_steps(hbm_engine* h, int n, const int* dims, const double* const* data, const double* u, int u_stride,
              int nsteps, const int* fwd, int* out_dims, double* const* out_data, const size_t* out_cap,
              size_t* out_nelem) {
  return guard(h, [&] {
    hbm::Engine& E = *h->E;
    const int nsq = (E.L + 1) * E.Q1;
    for (int i = 0; i < n; ++i) E.set_caps(widest_of(E, dims + size_t(i) * nsq));
    E.reserve_states(size_t(h->xih_base() + h->N + n));
    const int sb = h->xih_base() + h->N;
    for (int i = 0; i < n; ++i) E.upload_state(E.states[sb + i], dims + size_t(i) * nsq, data[i]);
    E.reserve_chains(std::max(E.nchain_cap, n), false);
    std::vector<Chain*> cs(n);
    std::vector<View> vs(n);
    for (int i = 0; i < n; ++i) { cs[i] = E.acquire(false); vs[i] = E.states[sb + i].view(); }
    E.load_many(cs, vs);
    Timer t(h, 4);
    std::vector<double> uf(n), ut(n);
    std::vector<int> fw(fwd, fwd + n);
    for (int s = 0; s < nsteps; ++s) {
      for (int i = 0; i < n; ++i) { uf[i] = u[size_t(i) * u_stride + s]; ut[i] = u[size_t(i) * u_stride + s + 1]; }
      E.step(cs, uf, ut, fw);
    }
    t.stop(long(n) * nsteps);
    for (int i = 0; i < n; ++i) {
      const size_t tot = E.download_view(cs[i]->view(), out_dims + size_t(i) * nsq, out_data[i], out_cap[i]);
      if (out_nelem) out_nelem[i] = tot;
      if (tot > out_cap[i]) { for (auto* c : cs) E.release(c); throw hbm::Error(2, "output buffer too small"); }
    }
    for (auto* c : cs) E.release(c);
  });
}

int hbm_overlap(hbm_engine* h, const int* dx, const double* x, const int* dy, const double* y, int with_dH,
                double* out) {
  return guard(h, [&] {
    hbm::Engine& E = *h->E;
    E.set_caps(std::max(widest_of(E, dx), widest_of(E, dy)));
    E.reserve_states(size_t(h->xih_base() + h->N + 2));
    const int sb = h->xih_base() + h->N;
    E.upload_state(E.states[sb], dx, x);
    E.upload_state(E.states[sb + 1], dy, y);
    Timer t(h, 1);
    auto r = E.overlaps({E.states[sb].view()}, {E.states[sb + 1].view()}, with_dH != 0);
    t.stop();
    out[0] = r[0].real();
    out[1] = r[0].imag();
  });
}

int hbm_apply_dH(hbm_engine* h, const int* dims, const double* data, int* out_dims, double* out_data, size_t cap,
                 size_t* nelem, double* norm) {
  return guard(h, [&] {
    hbm::Engine& E = *h->E;
    E.set_caps(widest_of(E, dims));
    E.reserve_states(size_t(h->xih_base() + h->N + 1));
    const int sb = h->xih_base() + h->N;
    E.upload_state(E.states[sb], dims, data);
    E.reserve_chains(std::max(E.nchain_cap, 1), false);
    std::vector<Chain*> cs{E.acquire(false)};
    Timer t(h, 2);
    E.apply_dH({E.states[sb].view()}, cs);
    t.stop();
    const double n2 = E.site_norm2({cs[0]->view()}, 1)[0];
    if (norm) *norm = std::sqrt(std::max(0.0, n2));
    const size_t tot = E.download_view(cs[0]->view(), out_dims, out_data, cap);
    if (nelem) *nelem = tot;
    E.release(cs[0]);
    if (tot > cap) throw hbm::Error(2, "output buffer too small");
  });
}

int hbm_set_states(hbm_engine* h, const int* dt_, const double* t, const int* di, const double* in) {
  return guard(h, [&] {
    hbm::Engine& E = *h->E;
    int wid = 0;
    for (int b = 0; b <= E.L; ++b) {
      int a = 0, c = 0;
      for (int q = 0; q < E.Q1; ++q) { a += dt_[b * E.Q1 + q]; c += di[b * E.Q1 + q]; }
      wid = std::max(wid, std::max(a, c));
    }
    E.set_caps(wid);  // before any slot exists: inputs may be wider than Maxm
    E.reserve_states(size_t(h->xih_base() + h->N + 1));
    E.upload_state(E.states[1], dt_, t);
    E.upload_state(E.states[0], di, in);
    h->have_states = true;
    h->have_psi = h->have_xi = h->have_xih = false;
  });
}

static void hbm_prepare_N(hbm_engine* h, int N) {
  if (N != h->N) {
    h->N = N;
    h->have_psi = h->have_xi = h->have_xih = false;
  }
  h->E->reserve_states(size_t(h->xih_base() + N + 2));
}

int hbm_propagate(hbm_engine* h, const double* u, int N, int which) {
  return guard(h, [&] {
    if (!h->have_states) throw hbm::Error(4, "ocg_set_states first");
    hbm_prepare_N(h, N);
    if (which & 1) h->have_psi = false;
    if (which & 2) h->have_xi = h->have_xih = false;
    hbm::Engine& E = *h->E;
    E.reserve_chains(std::max(E.nchain_cap, 2), false);
    std::vector<Chain*> cs;
    std::vector<int> kind;  // 0 psi, 1 xi
    if (which & 1) { cs.push_back(E.acquire(false)); kind.push_back(0); }
    if (which & 2) { cs.push_back(E.acquire(false)); kind.push_back(1); }
    std::vector<View> vs;
    for (int k : kind) vs.push_back(E.states[k == 0 ? 0 : 1].view());
    E.load_many(cs, vs);
    std::vector<State*> ss;
    for (int k : kind) ss.push_back(&E.states[k == 0 ? h->psi_base() : h->xi_base() + N - 1]);
    E.store_many(ss, cs);
    Timer t(h, 0);
    std::vector<double> uf(cs.size()), ut(cs.size());
    std::vector<int> fw(cs.size());
    for (int s = 0; s + 1 < N; ++s) {
      for (size_t i = 0; i < cs.size(); ++i) {
        if (kind[i] == 0) { uf[i] = u[s]; ut[i] = u[s + 1]; fw[i] = 1; }
        else { uf[i] = u[N - 1 - s]; ut[i] = u[N - 2 - s]; fw[i] = 0; }
      }
      E.step(cs, uf, ut, fw);
      ss.clear();
      for (size_t i = 0; i < cs.size(); ++i)
        ss.push_back(&E.states[kind[i] == 0 ? h->psi_base() + s + 1 : h->xi_base() + N - 2 - s]);
      E.store_many(ss, cs);
    }
    E.sync();
    t.stop(long(cs.size()) * (N - 1));
    for (auto* c : cs) E.release(c);
    if (which & 1) { h->have_psi = true; }
    if (which & 2) { h->have_xi = true; h->have_xih = false; }
  });
}

static std::vector<std::complex<double>> hbm_pairs(hbm_engine* h, const std::vector<int>& xs,
                                                   const std::vector<int>& ys, bool dH) {
  hbm::Engine& E = *h->E;
  std::vector<View> vx, vy;
  for (int s : xs) vx.push_back(E.states[s].view());
  for (int s : ys) vy.push_back(E.states[s].view());
  Timer t(h, 1);
  auto r = E.overlaps(vx, vy, dH);
  t.stop();
  return r;
}

int hbm_overlap_factor(hbm_engine* h, double* F) {
  return guard(h, [&] {
    if (!h->have_psi) throw hbm::Error(4, "psi_t not propagated");
    auto r = hbm_pairs(h, {h->psi_base() + h->N - 1}, {1}, false);
    F[0] = r[0].real();
    F[1] = r[0].imag();
  });
}
int hbm_fidelities(hbm_engine* h, double* fid) {
  return guard(h, [&] {
    if (!h->have_psi) throw hbm::Error(4, "psi_t not propagated");
    std::vector<int> xs(h->N, 1), ys(h->N);
    for (int i = 0; i < h->N; ++i) ys[i] = h->psi_base() + i;
    auto r = hbm_pairs(h, xs, ys, false);
    for (int i = 0; i < h->N; ++i) fid[i] = std::norm(r[i]);
  });
}
int hbm_div_t(hbm_engine* h, double* divT) {
  return guard(h, [&] {
    if (!h->have_psi || !h->have_xi) throw hbm::Error(4, "psi_t and xi_t must be propagated");
    std::vector<int> xs(h->N), ys(h->N);
    for (int i = 0; i < h->N; ++i) { xs[i] = h->xi_base() + i; ys[i] = h->psi_base() + i; }
    auto r = hbm_pairs(h, xs, ys, true);
    for (int i = 0; i < h->N; ++i) { divT[2 * i] = r[i].real(); divT[2 * i + 1] = r[i].imag(); }
  });
}

// getAnalyticGradient's device part (divT_t, F) without keeping the
// trajectories: psi forward and xi backward run as one lockstep batch and meet
// in the middle.  Phase 1 stores psi_0..psi_tm and xi_{N-1}..xi_{tm+1}
// (tm = (N-1)/2); phase 2 carries psi on to N-1, each new psi_t paired with the
// stored xi_t, and xi down to 0, each new xi_t paired with the stored psi_t.
// N states instead of the stored path's 2N (config 5 at N_t = 1001: 205 GB
// instead of 410 GB), the same N-1 dependent steps per chain, and the same
// states, overlaps and numbers bit for bit (every HBM-engine kernel is
// batch-independent and deterministic).  Leaves no device trajectories.
// A call that grows the state heap for slots it does not keep gives them back,
// down to the heap it began with, on success (done(): a device failure there is
// the call's status) and on failure (the destructor, errors swallowed while the
// guard unwinds), so later memory decisions (hipMemGetInfo) see the HBM free.
struct HeapRestore {
  hbm::Engine& E;
  size_t keep;
  bool ok = false;
  explicit HeapRestore(hbm::Engine& e) : E(e), keep(e.heap_slots) {}
  void done() {
    ok = true;
    E.shrink_states(keep);
  }
  ~HeapRestore() {
    if (ok) return;
    try {
      E.drain();
      E.shrink_states(keep);
    } catch (...) {
    }
  }
};

int hbm_gradient_mid(hbm_engine* h, const double* u, int N, double* divT, double* F) {
  return guard(h, [&] {
    if (!h->have_states) throw hbm::Error(4, "ocg_set_states first");
    if (N < 2) throw hbm::Error(1, "N < 2");
    hbm::Engine& E = *h->E;
    h->have_psi = h->have_xi = h->have_xih = false;  // the trajectory slots are overwritten
    h->N = 0;
    HeapRestore heap(E);  // the half trajectories are not kept (the footprint stayed at N + 2 slots)
    E.reserve_states(size_t(N) + 2);
    const int tm = (N - 1) / 2;
    auto slot = [](int t) { return 2 + t; };  // psi_t for t <= tm, xi_t above
    E.reserve_chains(std::max(E.nchain_cap, 2), false);
    Timer tt(h, 0);
    Chain* cp = E.acquire(false);
    Chain* cx = E.acquire(false);
    std::vector<Chain*> both{cp, cx};
    E.load_many(both, {E.states[0].view(), E.states[1].view()});
    E.store_many({&E.states[slot(0)], &E.states[slot(N - 1)]}, both);
    std::vector<std::complex<double>> dv(N);
    long nsteps = 0;
    // one lockstep step of the chains still moving: psi t -> t+1 while t < pe,
    // xi t -> t-1 while t > xe
    auto advance = [&](int& tp, int pe, int& tx, int xe) {
      std::vector<Chain*> c;
      std::vector<double> uf, ut;
      std::vector<int> fw;
      if (tp < pe) { c.push_back(cp); uf.push_back(u[tp]); ut.push_back(u[tp + 1]); fw.push_back(1); }
      if (tx > xe) { c.push_back(cx); uf.push_back(u[tx]); ut.push_back(u[tx - 1]); fw.push_back(0); }
      E.step(c, uf, ut, fw);
      nsteps += long(c.size());
      if (tp < pe) ++tp;
      if (tx > xe) --tx;
    };
    // phase 1: psi 0 -> tm, xi N-1 -> tm+1, both stored
    int tp = 0, tx = N - 1;
    while (tp < tm || tx > tm + 1) {
      const bool mp = tp < tm, mx = tx > tm + 1;
      advance(tp, tm, tx, tm + 1);
      std::vector<State*> ss;
      std::vector<Chain*> cc;
      if (mp) { ss.push_back(&E.states[slot(tp)]); cc.push_back(cp); }
      if (mx) { ss.push_back(&E.states[slot(tx)]); cc.push_back(cx); }
      E.store_many(ss, cc);
    }
    // phase 2: psi tm -> N-1 against the stored xi_t, xi tm+1 -> 0 against the stored psi_t
    while (tp < N - 1 || tx > 0) {
      const bool mp = tp < N - 1, mx = tx > 0;
      advance(tp, N - 1, tx, 0);
      std::vector<View> xs, ys;  // divT_t = overlapC(xi_t, dH, psi_t) (src/OptimalControl.cpp:409-419)
      if (mp) { xs.push_back(E.states[slot(tp)].view()); ys.push_back(cp->view()); }
      if (mx) { xs.push_back(cx->view()); ys.push_back(E.states[slot(tx)].view()); }
      const auto r = E.overlaps(xs, ys, true);
      int k = 0;
      if (mp) dv[tp] = r[k++];
      if (mx) dv[tx] = r[k++];
    }
    // F = overlapC(psi_{N-1}, target) (:242); the two end points of the trajectories
    // (divT_{N-1} with xi_{N-1} = target, divT_0 with psi_0 = init) came from phase 2
    const std::complex<double> Fc = E.overlaps({cp->view()}, {E.states[1].view()}, false)[0];
    E.sync();
    E.release(cp);
    E.release(cx);
    tt.stop(nsteps);
    F[0] = Fc.real();
    F[1] = Fc.imag();
    for (int t = 0; t < N; ++t) { divT[2 * t] = dv[t].real(); divT[2 * t + 1] = dv[t].imag(); }
    heap.done();
  });
}

// K controls' psi || xi in one lockstep batch of 2K chains, then their divT and F
// in two batched overlap launches (ocg_gradient_multi).  Control 0 uses the
// context's trajectory slots, control k >= 1 the 2N slots after xiH's block.
// Every kernel is batch-independent: per control the numbers of
// hbm_propagate(.., 3) + hbm_div_t + hbm_overlap_factor, bit for bit.
int hbm_gradient_multi(hbm_engine* h, int K, const double* U, int N, double* divT, double* F) {
  return guard(h, [&] {
    if (!h->have_states) throw hbm::Error(4, "ocg_set_states first");
    hbm_prepare_N(h, N);
    h->have_psi = h->have_xi = h->have_xih = false;
    hbm::Engine& E = *h->E;
    const int extra0 = h->xih_base() + N + 2;
    auto pb = [&](int k) { return k == 0 ? h->psi_base() : extra0 + 2 * N * (k - 1); };
    auto xb = [&](int k) { return k == 0 ? h->xi_base() : extra0 + 2 * N * (k - 1) + N; };
    // the other controls' trajectories are not kept: their slots are given back
    // afterwards, on success and on failure, down to the heap the call began with
    // (a previous pipelined getHessian's row-state slots stay for its next call)
    const size_t keep = std::max(size_t(extra0), E.heap_slots);
    struct ShrinkOnError {  // unwinding only: the success path shrinks inside the guard
      hbm::Engine& E;
      size_t keep;
      bool ok = false;
      ~ShrinkOnError() {
        if (ok) return;
        try {
          E.drain();
          E.shrink_states(keep);
        } catch (...) {
        }
      }
    } shrink{E, keep};
    E.reserve_states(size_t(extra0) + size_t(2) * N * (K - 1));
    E.reserve_chains(std::max(E.nchain_cap, 2 * K), false);
    std::vector<Chain*> cs(2 * K);
    std::vector<View> vs(2 * K);
    std::vector<State*> ss(2 * K);
    for (int k = 0; k < K; ++k) {
      cs[2 * k] = E.acquire(false);
      cs[2 * k + 1] = E.acquire(false);
      vs[2 * k] = E.states[0].view();      // psi_init
      vs[2 * k + 1] = E.states[1].view();  // psi_target
      ss[2 * k] = &E.states[pb(k)];
      ss[2 * k + 1] = &E.states[xb(k) + N - 1];
    }
    E.load_many(cs, vs);
    E.store_many(ss, cs);
    Timer t(h, 0);
    std::vector<double> uf(2 * K), ut(2 * K);
    std::vector<int> fw(2 * K);
    for (int s = 0; s + 1 < N; ++s) {
      for (int k = 0; k < K; ++k) {
        const double* u = U + size_t(k) * N;
        uf[2 * k] = u[s]; ut[2 * k] = u[s + 1]; fw[2 * k] = 1;
        uf[2 * k + 1] = u[N - 1 - s]; ut[2 * k + 1] = u[N - 2 - s]; fw[2 * k + 1] = 0;
        ss[2 * k] = &E.states[pb(k) + s + 1];
        ss[2 * k + 1] = &E.states[xb(k) + N - 2 - s];
      }
      E.step(cs, uf, ut, fw);
      E.store_many(ss, cs);
    }
    E.sync();
    t.stop(long(2 * K) * (N - 1));
    for (auto* c : cs) E.release(c);
    h->have_psi = h->have_xi = true;
    h->have_xih = false;
    std::vector<int> xs(size_t(K) * N), ys(size_t(K) * N);
    for (int k = 0; k < K; ++k)
      for (int i = 0; i < N; ++i) { xs[size_t(k) * N + i] = xb(k) + i; ys[size_t(k) * N + i] = pb(k) + i; }
    auto r = hbm_pairs(h, xs, ys, true);
    for (size_t e = 0; e < size_t(K) * N; ++e) { divT[2 * e] = r[e].real(); divT[2 * e + 1] = r[e].imag(); }
    std::vector<int> fx(K), fy(K, 1);
    for (int k = 0; k < K; ++k) fx[k] = pb(k) + N - 1;
    auto rf = hbm_pairs(h, fx, fy, false);
    for (int k = 0; k < K; ++k) { F[2 * k] = rf[k].real(); F[2 * k + 1] = rf[k].imag(); }
    shrink.ok = true;
    E.shrink_states(keep);  // a device failure here is this call's status
  });
}

// rows per batch of the Hessian / chunk of dH applications: bounded by memory
static int hbm_batch(hbm_engine* h, int want) {
  hbm::Engine& E = *h->E;
  const double per = 16.0 * E.chain_elems(false) * 4.0;  // chain + its share of workspace
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  const double budget = 0.5 * double(fr);
  int b = int(std::max(1.0, std::min(double(want), budget / std::max(per, 1.0))));
  return std::min(b, 1024);
}

int hbm_xi_dH(hbm_engine* h) {
  return guard(h, [&] {
    if (!h->have_xi) throw hbm::Error(4, "xi_t not propagated");
    h->have_xih = false;
    hbm::Engine& E = *h->E;
    const int N = h->N;
    const int B = hbm_batch(h, N);
    E.reserve_chains(std::max(E.nchain_cap, B), false);
    Timer t(h, 2);
    for (int t0 = 0; t0 < N; t0 += B) {
      const int nb = std::min(B, N - t0);
      std::vector<View> in;
      std::vector<Chain*> out;
      std::vector<State*> ss;
      for (int i = 0; i < nb; ++i) {
        in.push_back(E.states[h->xi_base() + t0 + i].view());
        out.push_back(E.acquire(false));
        ss.push_back(&E.states[h->xih_base() + t0 + i]);
      }
      E.apply_dH(in, out);
      E.store_many(ss, out);
      E.sync();
      for (auto* c : out) E.release(c);
    }
    t.stop();
    h->have_xih = true;
  });
}

// calcHessianRow (src/OptimalControl.cpp:251-279) for a set of rows, in
// batches: psiH_i = dH psi_i, then all rows of a batch step in lockstep
// (row i's s-th step uses u[i+s-1] -> u[i+s]) and overlap with xiH_{i+s}
int hbm_hessian_rows(hbm_engine* h, const double* u, int N, const int* rows, int nrows, const double* F,
                     const double* divT, double* H) {
  return guard(h, [&] {
    if (N != h->N || !h->have_psi || !h->have_xih) throw hbm::Error(4, "propagate(3) + xi_dH first");
    hbm::Engine& E = *h->E;
    const std::complex<double> Fc(F[0], F[1]);
    auto dv = [&](int i) { return std::complex<double>(divT[2 * i], divT[2 * i + 1]); };
    const double dt2 = E.dt * E.dt;
    std::vector<int> rs(rows, rows + nrows);
    std::sort(rs.begin(), rs.end());
    const int B = hbm_batch(h, nrows);
    E.reserve_chains(std::max(E.nchain_cap, B), false);
    Timer t(h, 3);
    long nsteps = 0;
    for (int r0 = 0; r0 < nrows; r0 += B) {
      const int nb = std::min(B, nrows - r0);
      std::vector<int> ri(rs.begin() + r0, rs.begin() + r0 + nb);
      std::vector<Chain*> cs(nb);
      std::vector<View> in(nb);
      for (int k = 0; k < nb; ++k) { cs[k] = E.acquire(false); in[k] = E.states[h->psi_base() + ri[k]].view(); }
      E.apply_dH(in, cs);
      std::vector<View> vs;
      for (auto* c : cs) vs.push_back(c->view());
      const std::vector<double> n2 = E.site_norm2(vs, 1);
      std::vector<double> nrm(nb);
      for (int k = 0; k < nb; ++k) nrm[k] = std::sqrt(std::max(0.0, n2[k]));
      // diagonal (:259-264)
      {
        std::vector<View> xs;
        for (int k = 0; k < nb; ++k) xs.push_back(E.states[h->xih_base() + ri[k]].view());
        auto ov = E.overlaps(xs, vs, false);
        for (int k = 0; k < nb; ++k) {
          const int i = ri[k];
          const double v1 = (Fc * ov[k]).real(), v2 = -std::norm(dv(i));
          H[size_t(i) * N + i] = dt2 * (v1 + v2);
        }
      }
      // off-diagonal (:266-278): lockstep over s
      std::vector<int> act(nb);
      for (int k = 0; k < nb; ++k) act[k] = k;
      for (int s = 1;; ++s) {
        std::vector<Chain*> a;
        std::vector<int> ak;
        for (int k : act)
          if (ri[k] + s <= N - 2) { a.push_back(cs[k]); ak.push_back(k); }
        if (a.empty()) break;
        std::vector<double> uf(a.size()), ut(a.size());
        std::vector<int> fw(a.size(), 1);
        for (size_t m = 0; m < a.size(); ++m) { const int j = ri[ak[m]] + s; uf[m] = u[j - 1]; ut[m] = u[j]; }
        E.step(a, uf, ut, fw);
        nsteps += long(a.size());
        std::vector<View> xs, ys;
        for (size_t m = 0; m < a.size(); ++m) {
          xs.push_back(E.states[h->xih_base() + ri[ak[m]] + s].view());
          ys.push_back(a[m]->view());
        }
        auto ov = E.overlaps(xs, ys, false);
        for (size_t m = 0; m < a.size(); ++m) {
          const int k = ak[m], i = ri[k], j = i + s;
          const double v1 = (Fc * ov[m] * nrm[k]).real();
          const double v2 = -(dv(i) * std::conj(dv(j))).real();
          const double r = dt2 * (v1 + v2);
          H[size_t(i) * N + j] = r;
          H[size_t(j) * N + i] = r;
        }
        act = ak;
      }
      for (auto* c : cs) E.release(c);
    }
    t.stop(nsteps);
  });
}

// bytes a call holding `slots` state slots must newly allocate: 0 when the heap
// already has them (a previous call grew it), else the whole grown heap
// (reserve_states copies into a new allocation beside the old one)
static double heap_growth_bytes(const hbm_engine* h, double slots) {
  return slots <= double(h->E->heap_slots) ? 0.0 : 16.0 * double(h->E->state_cap) * slots;
}
double hbm_traj_bytes(const hbm_engine* h, int N) { return heap_growth_bytes(h, 3.0 * N + 6.0); }
// bytes a pool of n chains would newly allocate on an engine holding `have`
// chains (the pool itself, 16 B per element, and half as much again for the
// workspace arenas the chains' launches draw on); a call that still runs out
// of memory fails cleanly and its caller takes the lighter path
static double chain_growth_bytes(const hbm::Engine& E, int n, int have, bool wide) {
  return n <= have ? 0.0 : 16.0 * 1.5 * double(E.chain_elems(wide)) * n;
}
double hbm_gradient_multi_bytes(const hbm_engine* h, int K, int N) {
  const hbm::Engine& E = *h->E;
  return heap_growth_bytes(h, 3.0 * N + 6.0 + 2.0 * N * (K - 1)) + chain_growth_bytes(E, 2 * K, E.nchain_cap, false);
}

// Checkpointed getHessian (see hbm.hpp).  Time-major row sweep: all rows of a
// batch advance together in absolute time j (row i joins at j = i with
// psiH_i = dH psi_i), so every active row needs the same xiH_j at step j and
// psi_i only when it joins; both are produced segment by segment from the
// checkpoints (psi forward from psi_{T_s}, xi backward from xi_{T_{s+1}}).
// Same steps, decompositions, dH applications and overlaps as the stored
// path, so the same numbers bit for bit (every kernel is batch-independent
// and deterministic).
int hbm_hessian_ckpt(hbm_engine* h, const double* u, int N, const int* rows, int nrows, double* H, double* divT,
                     double* F, int K) {
  return guard(h, [&] {
    if (!h->have_states) throw hbm::Error(4, "ocg_set_states first");
    if (N < 2) throw hbm::Error(1, "N < 2");
    hbm::Engine& E = *h->E;
    K = std::max(1, std::min(K, N - 1));
    const int S = (N - 1 + K - 1) / K;  // segments s = 0..S-1 cover [T_s, T_{s+1}], T_S = N - 1
    auto Tc = [&](int s) { return std::min(s * K, N - 1); };
    // slots: 0 init, 1 target, then ckpsi[S+1], ckxi[S+1], and a region that holds
    // first the meet-in-the-middle half trajectories (N slots, when they fit) and
    // then segpsi[K+1], segxi[K+1], segxiH[K+1]
    const int ckp = 2, ckx = ckp + S + 1, R = ckx + S + 1, sgp = R, sgx = sgp + K + 1, sgh = sgx + K + 1;
    h->have_psi = h->have_xi = h->have_xih = false;  // the trajectory slots are overwritten
    h->N = 0;
    // divT everywhere and F: psi || xi meeting in the middle (hbm_gradient_mid,
    // every checkpoint stored on the way) when N half-trajectory slots fit, so the
    // row passes recompute only the segments their rows need; else the
    // checkpoint-only pass and divT in the first row pass
    HeapRestore heap(E);  // checkpoints, half trajectories and segments are not kept
    bool mid = false;
    if (const char* e = std::getenv("OCG_HBM_CKPT_MID")) mid = std::atoi(e) != 0;
    else {
      // the middle path's N half-trajectory slots only when they leave room for what
      // follows: the row batches' chains (B + K + 2, priced as hbm_batch prices them)
      // and their workspace arenas, i.e. the new slots within half the free HBM
      // (an unbudgeted reservation starved the later chain pools)
      size_t fr = 0, tot = 0;
      (void)hipMemGetInfo(&fr, &tot);
      const double slots = double(R) + std::max(double(N), 3.0 * (K + 1));
      mid = heap_growth_bytes(h, slots) <= 0.5 * double(fr);
    }
    if (mid) {
      try {
        E.reserve_states(size_t(R) + std::max<size_t>(size_t(N), size_t(3) * (K + 1)));
      } catch (const hbm::Error& e) {
        if (e.code != 6) throw;
        (void)hipGetLastError();
        mid = false;
      }
    }
    E.reserve_states(size_t(sgh + K + 1));
    const double dt2 = E.dt * E.dt;
    Timer tall(h, 5);
    std::vector<std::complex<double>> dv(N, 0.0);
    std::complex<double> Fc;
    E.reserve_chains(std::max(E.nchain_cap, 2), false);
    auto ckpt_psi = [&](int t) { return (t == N - 1 || t % K == 0) ? ckp + (t == N - 1 ? S : t / K) : -1; };
    auto ckpt_xi = [&](int t) { return (t == N - 1 || t % K == 0) ? ckx + (t == N - 1 ? S : t / K) : -1; };
    if (mid) {
      const int tm = (N - 1) / 2;
      auto half = [&](int t) { return R + t; };  // psi_t for t <= tm, xi_t above
      Chain* cp = E.acquire(false);
      Chain* cx = E.acquire(false);
      std::vector<Chain*> both{cp, cx};
      E.load_many(both, {E.states[0].view(), E.states[1].view()});
      E.store_many({&E.states[half(0)], &E.states[ckp], &E.states[half(N - 1)], &E.states[ckx + S]}, {cp, cp, cx, cx});
      auto advance = [&](int& tp, int pe, int& tx, int xe) {
        std::vector<Chain*> c;
        std::vector<double> uf, ut;
        std::vector<int> fw;
        if (tp < pe) { c.push_back(cp); uf.push_back(u[tp]); ut.push_back(u[tp + 1]); fw.push_back(1); }
        if (tx > xe) { c.push_back(cx); uf.push_back(u[tx]); ut.push_back(u[tx - 1]); fw.push_back(0); }
        E.step(c, uf, ut, fw);
        if (tp < pe) ++tp;
        if (tx > xe) --tx;
      };
      int tp = 0, tx = N - 1;
      while (tp < tm || tx > tm + 1) {  // phase 1: both halves stored, checkpoints on the way
        const bool mp = tp < tm, mx = tx > tm + 1;
        advance(tp, tm, tx, tm + 1);
        std::vector<State*> ss;
        std::vector<Chain*> cc;
        if (mp) {
          ss.push_back(&E.states[half(tp)]); cc.push_back(cp);
          if (ckpt_psi(tp) >= 0) { ss.push_back(&E.states[ckpt_psi(tp)]); cc.push_back(cp); }
        }
        if (mx) {
          ss.push_back(&E.states[half(tx)]); cc.push_back(cx);
          if (ckpt_xi(tx) >= 0) { ss.push_back(&E.states[ckpt_xi(tx)]); cc.push_back(cx); }
        }
        E.store_many(ss, cc);
      }
      while (tp < N - 1 || tx > 0) {  // phase 2: each new state paired with the stored other half
        const bool mp = tp < N - 1, mx = tx > 0;
        advance(tp, N - 1, tx, 0);
        std::vector<State*> ss;
        std::vector<Chain*> cc;
        if (mp && ckpt_psi(tp) >= 0) { ss.push_back(&E.states[ckpt_psi(tp)]); cc.push_back(cp); }
        if (mx && ckpt_xi(tx) >= 0) { ss.push_back(&E.states[ckpt_xi(tx)]); cc.push_back(cx); }
        if (!ss.empty()) E.store_many(ss, cc);
        std::vector<View> xs, ys;  // divT_t = overlapC(xi_t, dH, psi_t) (:409-419)
        if (mp) { xs.push_back(E.states[half(tp)].view()); ys.push_back(cp->view()); }
        if (mx) { xs.push_back(cx->view()); ys.push_back(E.states[half(tx)].view()); }
        const auto r = E.overlaps(xs, ys, true);
        int k = 0;
        if (mp) dv[tp] = r[k++];
        if (mx) dv[tx] = r[k++];
      }
      Fc = E.overlaps({cp->view()}, {E.states[1].view()}, false)[0];  // F = overlapC(psi_{N-1}, target) (:242)
      E.sync();
      E.release(cp);
      E.release(cx);
    } else {
      // 1. psi forward / xi backward in one batch, checkpoints only
      std::vector<Chain*> cs{E.acquire(false), E.acquire(false)};
      E.load_many(cs, {E.states[0].view(), E.states[1].view()});
      E.store_many({&E.states[ckp], &E.states[ckx + S]}, cs);
      std::vector<double> uf(2), ut(2);
      std::vector<int> fw{1, 0};
      for (int s = 0; s + 1 < N; ++s) {
        uf[0] = u[s]; ut[0] = u[s + 1];
        uf[1] = u[N - 1 - s]; ut[1] = u[N - 2 - s];
        E.step(cs, uf, ut, fw);
        const int tp = s + 1, tx = N - 2 - s;
        std::vector<State*> ss;
        std::vector<Chain*> cc;
        if (ckpt_psi(tp) >= 0) { ss.push_back(&E.states[ckpt_psi(tp)]); cc.push_back(cs[0]); }
        if (tx % K == 0) { ss.push_back(&E.states[ckx + tx / K]); cc.push_back(cs[1]); }
        if (!ss.empty()) E.store_many(ss, cc);
      }
      E.sync();
      for (auto* c : cs) E.release(c);
      // F = overlapC(psi_{N-1}, target) (:242)
      Fc = E.overlaps({E.states[ckp + S].view()}, {E.states[1].view()}, false)[0];
    }
    F[0] = Fc.real();
    F[1] = Fc.imag();
    // 2. row batches (ascending rows; the first pass also forms divT everywhere)
    std::vector<int> rs(rows, rows + nrows);
    std::sort(rs.begin(), rs.end());
    const int B = std::max(1, hbm_batch(h, std::max(nrows, 1)));
    // in flight at once: the batch's row chains, a segment's xiH outputs (<= K)
    // and the two recomputation chains
    E.reserve_chains(std::max(E.nchain_cap, B + K + 2), false);
    bool first = !mid;  // without the middle pass the first row pass also forms divT
    for (int r0 = 0; first || r0 < nrows; r0 += B) {
      const int nb = std::min(B, nrows - r0);
      const int imin = nb > 0 ? rs[r0] : N;
      std::vector<Chain*> act;  // active rows, in joining order
      std::vector<int> ai;      // their i
      std::vector<double> nrm;
      int next = r0;            // next row of the batch to join
      const int s_begin = first ? 0 : std::min(S - 1, imin / K);
      for (int s = s_begin; s < S; ++s) {
        const int a = Tc(s), b = Tc(s + 1);  // segment [a, b]
        const bool need_rows = nb > 0 && b - 1 >= imin && a <= N - 2;
        if (!first && !need_rows) continue;
        // psi_a..psi_b forward and xi_b..xi_a backward from their checkpoints, one
        // batch of two chains (every HBM-engine kernel is batch-independent: the
        // same states as two single-chain passes, in half the dependent steps)
        {
          std::vector<Chain*> c2{E.acquire(false), E.acquire(false)};
          E.load_many(c2, {E.states[ckp + s].view(), E.states[ckx + s + 1].view()});
          E.store_many({&E.states[sgp], &E.states[sgx + b - a]}, c2);
          std::vector<double> uf(2), ut(2);
          const std::vector<int> fw{1, 0};
          for (int m = 0; m < b - a; ++m) {
            uf[0] = u[a + m]; ut[0] = u[a + m + 1];
            uf[1] = u[b - m]; ut[1] = u[b - m - 1];
            E.step(c2, uf, ut, fw);
            E.store_many({&E.states[sgp + m + 1], &E.states[sgx + b - m - 1 - a]}, c2);
          }
          E.sync();
          for (auto* c : c2) E.release(c);
        }
        // divT_t = overlapC(xi_t, dH, psi_t) (:409-419), t in [a, b) (and N-1 at the end)
        if (first) {
          std::vector<View> xs, ys;
          const int tend = (s == S - 1) ? b : b - 1;
          for (int t = a; t <= tend; ++t) { xs.push_back(E.states[sgx + t - a].view()); ys.push_back(E.states[sgp + t - a].view()); }
          const auto r = E.overlaps(xs, ys, true);
          for (int t = a; t <= tend; ++t) dv[t] = r[t - a];
        }
        if (!need_rows) continue;
        // xiH_j = exactApplyMPO(dH, xi_j) for the rows' times in this segment (:300-303)
        const int j0 = std::max(a, imin), j1 = std::min(b - 1, N - 2);
        {
          std::vector<View> in;
          std::vector<Chain*> out;
          std::vector<State*> ss;
          for (int j = j0; j <= j1; ++j) {
            in.push_back(E.states[sgx + j - a].view());
            out.push_back(E.acquire(false));
            ss.push_back(&E.states[sgh + j - a]);
          }
          E.apply_dH(in, out);
          E.store_many(ss, out);
          E.sync();
          for (auto* c : out) E.release(c);
        }
        for (int j = j0; j <= j1; ++j) {
          // active rows: step u[j-1] -> u[j] (timeStepper.step(psiH, ..), :269), overlap with xiH_j
          if (!act.empty()) {
            E.step(act, std::vector<double>(act.size(), u[j - 1]), std::vector<double>(act.size(), u[j]),
                   std::vector<int>(act.size(), 1));
            std::vector<View> xs(act.size(), E.states[sgh + j - a].view()), ys;
            for (auto* c : act) ys.push_back(c->view());
            const auto ov = E.overlaps(xs, ys, false);
            for (size_t m = 0; m < act.size(); ++m) {
              const int i = ai[m];
              const double v1 = (Fc * ov[m] * nrm[m]).real();
              const double v2 = -(dv[i] * std::conj(dv[j])).real();
              const double r = dt2 * (v1 + v2);
              H[size_t(i) * N + j] = r;
              H[size_t(j) * N + i] = r;
            }
          }
          // rows joining at j: psiH_i = dH psi_i, normiH, diagonal (:256-264)
          std::vector<int> join;
          while (next < r0 + nb && rs[next] == j) join.push_back(rs[next++]);
          if (!join.empty()) {
            std::vector<View> in(join.size(), E.states[sgp + j - a].view());
            std::vector<Chain*> cs;
            for (size_t m = 0; m < join.size(); ++m) cs.push_back(E.acquire(false));
            E.apply_dH(in, cs);
            std::vector<View> vs;
            for (auto* c : cs) vs.push_back(c->view());
            const std::vector<double> n2 = E.site_norm2(vs, 1);
            std::vector<View> xs(join.size(), E.states[sgh + j - a].view());
            const auto ov = E.overlaps(xs, vs, false);
            for (size_t m = 0; m < join.size(); ++m) {
              const int i = join[m];
              H[size_t(i) * N + i] = dt2 * ((Fc * ov[m]).real() - std::norm(dv[i]));
              act.push_back(cs[m]);
              ai.push_back(i);
              nrm.push_back(std::sqrt(std::max(0.0, n2[m])));
            }
          }
        }
      }
      for (auto* c : act) E.release(c);
      first = false;
      if (nb <= 0) break;
    }
    for (int t = 0; t < N; ++t) { divT[2 * t] = dv[t].real(); divT[2 * t + 1] = dv[t].imag(); }
    tall.stop();
    heap.done();
  });
}

int hbm_get_state(hbm_engine* h, int which, int t, int* dims, double* data, size_t cap, size_t* nelem) {
  return guard(h, [&] {
    if (t < 0 || t >= h->N) throw hbm::Error(1, "t out of range");
    const bool ok = (which == 0 && h->have_psi) || (which == 1 && h->have_xi) || (which == 2 && h->have_xih);
    if (!ok) throw hbm::Error(4, "requested trajectory not available");
    const int base = which == 0 ? h->psi_base() : (which == 1 ? h->xi_base() : h->xih_base());
    const size_t tot = h->E->download_view(h->E->states[base + t].view(), dims, data, cap);
    if (nelem) *nelem = tot;
    if (tot > cap) throw hbm::Error(2, "output buffer too small");
  });
}

int hbm_stats(hbm_engine* h, int kind, double* ms, long* launches, double* bytes, double* flops, long* steps) {
  if (kind == 7) {  // the GEMM (MFMA contraction) kernel: HIP-event time, algorithmic flops / bytes
    (void)guard(h, [&] { h->E->sync(); });
    if (ms) *ms = h->E->gemm_ms;
    if (launches) *launches = h->E->gemm_launches;
    if (bytes) *bytes = h->E->gemm_bytes;
    if (flops) *flops = h->E->gemm_flops;
    if (steps) *steps = 0;
    return 0;
  }
  if (ms) *ms = h->ms[kind];
  if (launches) *launches = h->launches[kind];
  if (bytes) *bytes = 0;
  if (flops) *flops = 0;
  if (steps) *steps = h->steps[kind];
  return 0;
}
int hbm_coop_stats(hbm_engine* h, long* launches, long* groups, long* fallbacks) {
  long l = 0, g = 0, f = 0;
  const int rc = guard(h, [&] {
    for (hbm::Engine* X : {h->E.get(), h->W[0].get(), h->W[1].get()}) {
      if (!X) continue;
      l += X->coop_launches;
      g += X->coop_groups;
      if (X->coop_fb.p) {
        int v = 0;
        HCK(hipStreamSynchronize(X->st2));
        HCK(hipMemcpy(&v, X->coop_fb.p, sizeof(int), hipMemcpyDeviceToHost));
        f += v;
      }
    }
  });
  if (launches) *launches = l;
  if (groups) *groups = g;
  if (fallbacks) *fallbacks = f;
  return rc;
}
void hbm_reset_stats(hbm_engine* h) {
  for (int k = 0; k < 8; ++k) { h->ms[k] = 0; h->launches[k] = 0; h->steps[k] = 0; }
  (void)guard(h, [&] { h->E->sync(); });
  h->E->gemm_ms = h->E->gemm_flops = h->E->gemm_bytes = 0;
  h->E->gemm_launches = 0;
}
int hbm_info_L(const hbm_engine* h) { return h->E->L; }
bool hbm_have(const hbm_engine* h, int what) {
  switch (what) {
    case 0: return h->have_states;
    case 1: return h->have_psi;
    case 2: return h->have_xi;
    case 3: return h->have_xih;
  }
  return false;
}
int hbm_N(const hbm_engine* h) { return h->N; }

int hbm_denmat_decomp(hbm_engine* h, int nm, const int* rows, const int* cols, const double* const* M, double cutoff,
                      int maxm, int* kept, double* const* w, double* const* X, double* const* Y) {
  return guard(h, [&] {
    for (int i = 0; i < nm; ++i)
      if (rows[i] <= 0 || cols[i] <= 0 || rows[i] > cols[i] || rows[i] > hbm::kBtRows)
        throw hbm::Error(1, "block shape: need 0 < rows <= cols and rows <= 512");
    const auto k = h->E->decompose_dense(nm, rows, cols, M, cutoff, maxm > 0 ? maxm : 5000, w, X, Y);
    for (int i = 0; i < nm; ++i) kept[i] = k[i];
  });
}

// InitializeState on the device (ocg_ground_state): the tau schedule of
// imaginary-time steps with the state resident in one chain; per block of
// `block` steps one overlap with the block's starting state (a heap slot),
// 1 - |<prev|new>| < tol ends a stage.  Only the final state is downloaded.
// gf / gb[t]: the exp(-tau_t h) gate tables (layout glo / gsz / goff as the
// real-time ones); the real-time tables (dt0) are restored afterwards.
int hbm_ground_state(hbm_engine* h, const int* dims, const double* data, double U, int ntau, const double* taus,
                     const std::vector<std::vector<double>>& gf, const std::vector<std::vector<double>>& gb,
                     const int* glo, const int* gsz, const int* goff, int gtotal, double dt0,
                     const std::vector<double>& gf0, const std::vector<double>& gb0, int block, double tol,
                     int max_steps, int* out_dims, double* out_data, size_t cap, size_t* nelem, int* steps_done) {
  int done = 0;
  const int rc = guard(h, [&] {
    hbm::Engine& E = *h->E;
    E.set_caps(widest_of(E, dims));
    E.reserve_states(size_t(h->xih_base() + h->N + 2));
    const int prev = h->xih_base() + h->N;  // scratch slot after the trajectories
    E.upload_state(E.states[prev], dims, data);
    E.reserve_chains(std::max(E.nchain_cap, 1), false);
    std::vector<Chain*> cs{E.acquire(false)};
    E.load_many(cs, {E.states[prev].view()});
    Timer t(h, 4);
    for (int s = 0; s < ntau; ++s) {
      E.dt = taus[s];
      E.set_gates(gf[s], gb[s], glo, gsz, goff, gtotal);
      E.gcst.imag = 1;
      for (int d = 0; d < max_steps; d += block) {
        E.store_many({&E.states[prev]}, cs);
        for (int k = 0; k < block; ++k) E.step(cs, {U}, {U}, {1});
        done += block;
        const auto ov = E.overlaps({E.states[prev].view()}, {cs[0]->view()}, false);
        if (1.0 - std::abs(ov[0]) < tol) break;
      }
    }
    t.stop(done);
    const size_t tot = E.download_view(cs[0]->view(), out_dims, out_data, cap);
    if (nelem) *nelem = tot;
    E.release(cs[0]);
    if (tot > cap) throw hbm::Error(2, "output buffer too small");
  });
  const int rc2 = hbm_swap_gates(h, 0, dt0, gf0, gb0, glo, gsz, goff, gtotal);
  if (steps_done) *steps_done = done;
  return rc ? rc : rc2;
}

// ---------------------------------------------------------------------------
// Pipelined getHessian (calcHessian_*, src/OptimalControl.cpp:281-372): the
// psi chain, the rows, the dH applications and the xi chain run concurrently
// instead of one after the other, so a Hessian slice costs about one
// trajectory's latency instead of two trajectories plus the longest row.
//   main thread, engine E : one lockstep batch of the psi chain (t -> t+1) and
//                           every row that has joined (row i at its own time:
//                           per-chain controls), each row state stored for
//                           its overlap (RS slots); publishes psi_t
//   thread H, worker W[0] : psiH_i = exactApplyMPO(dH, psi_i) and normiH as
//                           psi_i appears (:256-257); publishes the row
//   thread X, worker W[1] : xi backward from the target (:392-407), then
//                           xiH_t = exactApplyMPO(dH, xi_t) (:300-303)
// then one batched launch sequence of every overlap: divT (:409-419), F (:242)
// and <xiH_j|psiH_i(j)> (:261, :272).  Same steps, decompositions, dH
// applications and overlaps as hbm_propagate + hbm_xi_dH + hbm_hessian_rows,
// and every kernel is batch-independent, so the same numbers bit for bit.
// Memory: the stored trajectories plus one state per (row, later time).
// ---------------------------------------------------------------------------
namespace {
hbm::Engine& pipe_worker(hbm_engine* h, int k) {
  hbm::Engine& E = *h->E;
  auto& W = h->W[k];
  if (W && (W->bcap != E.bcap || W->bcapw != E.bcapw)) W.reset();
  if (!W) {
    W.reset(new hbm::Engine(E.device, E.L, E.p, E.Q, E.J, E.dt, E.cutoff, E.maxm));
    W->prio_level = k == 0 ? 1 : -1;
    W->init(h->md, h->mdz, h->gf, h->gb, h->glo, h->gsz, h->goff, h->gtotal, h->gates);
    W->set_caps(E.widest);
    if (W->bcap != E.bcap || W->bcapw != E.bcapw || W->state_cap != E.state_cap)
      throw hbm::Error(3, "internal: worker engine capacities differ");
    h->w_version[k] = h->gates_version;
  }
  if (h->w_version[k] != h->gates_version) {
    W->set_gates(h->gf, h->gb, h->glo, h->gsz, h->goff, h->gtotal);
    h->w_version[k] = h->gates_version;
  }
  W->dt = E.dt;
  W->gcst.imag = 0;
  return *W;
}
// OCG_PIPE_DEBUG=1: progress lines of the three stages on stderr (diagnostic)
bool pipe_debug() {
  static const bool d = std::getenv("OCG_PIPE_DEBUG") != nullptr;
  return d;
}
#define PIPE_LOG(...)                          \
  do {                                          \
    if (pipe_debug()) {                         \
      std::fprintf(stderr, __VA_ARGS__);        \
      std::fflush(stderr);                      \
    }                                           \
  } while (0)
// first slot of the row states and the slots the pipeline needs in total
int pipe_psih_base(const hbm_engine* h, int N) { return 4 + 3 * N + 2; }
}  // namespace

double hbm_pipe_bytes(const hbm_engine* h, int N, const int* rows, int nrows) {
  double slots = pipe_psih_base(h, N) + N;
  for (int r = 0; r < nrows; ++r) slots += std::max(0, N - 2 - rows[r]);
  const hbm::Engine& E = *h->E;
  // + the context engine's nrows + 1 chains (psi and every joined row) and the two
  // workers' pools: the dH worker joins up to 8 rows (normal + wide chains), the
  // xi worker applies dH in chunks of up to min(N, 8) states
  const int wn[2] = {h->W[0] ? h->W[0]->nchain_cap : 0, h->W[1] ? h->W[1]->nchain_cap : 0};
  const int ww[2] = {h->W[0] ? h->W[0]->nchain_cap_w : 0, h->W[1] ? h->W[1]->nchain_cap_w : 0};
  const int xc = std::min(N, 8);
  return heap_growth_bytes(h, slots) + chain_growth_bytes(E, nrows + 1, E.nchain_cap, false) +
         chain_growth_bytes(E, 8, wn[0], false) + chain_growth_bytes(E, 8, ww[0], true) +
         chain_growth_bytes(E, xc, wn[1], false) + chain_growth_bytes(E, xc, ww[1], true);
}

int hbm_hessian_pipe(hbm_engine* h, const double* u, int N, const int* rows, int nrows, double* H, double* divT,
                     double* F) {
  return guard(h, [&] {
    if (!h->have_states) throw hbm::Error(4, "ocg_set_states first");
    hbm::Engine& E = *h->E;
    std::vector<int> rs(rows, rows + nrows);
    std::sort(rs.begin(), rs.end());
    hbm_prepare_N(h, N);
    h->have_psi = h->have_xi = h->have_xih = false;  // the trajectory slots are overwritten
    const int psih0 = pipe_psih_base(h, N);
    std::vector<int> rsoff(nrows + 1);
    rsoff[0] = psih0 + N;
    for (int k = 0; k < nrows; ++k) rsoff[k + 1] = rsoff[k] + (N - 2 - rs[k]);
    // a failed call gives back everything it grew — its row-state slots, the
    // context engine's chain pool, the two worker engines with their pools and
    // arenas — so that the two-phase path ocg_hessian may retry after an
    // allocation failure sees that memory free
    struct ShrinkOnError {
      hbm_engine* h;
      size_t keep;
      int chains0;
      bool ok = false;
      ~ShrinkOnError() {
        if (ok) return;
        hbm::Engine& E = *h->E;
        try {
          E.drain();
          for (auto& W : h->W)
            if (W) {
              W->drain();
              W.reset();
            }
          E.release_all();
          E.shrink_chains(chains0);
          E.shrink_states(keep);
        } catch (...) {
        }
      }
    } undo{h, std::max(E.heap_slots, size_t(h->xih_base() + N + 2)), E.nchain_cap};
    E.reserve_states(size_t(rsoff[nrows]));
    hbm::Engine& WH = pipe_worker(h, 0);
    hbm::Engine& WX = pipe_worker(h, 1);
    const int dev = E.device;
    const int B = hbm_batch(h, N);
    Timer tall(h, 5);
    std::atomic<int> psi_ready(-1), psih_ready(0), abort_(0);
    std::vector<double> nrm(nrows, 0.0);
    auto wait_for = [&](const std::atomic<int>& a, int v) {
      while (a.load(std::memory_order_acquire) < v) {
        if (abort_.load()) throw hbm::Error(3, "pipelined getHessian: another stage failed");
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    };
    std::exception_ptr ex[3];
    // X: xi_t backward from the target, then xiH_t for every t
    std::thread tx([&] {
      try {
        HCK(hipSetDevice(dev));
        hbm::Engine& W = WX;
        W.reserve_chains(std::max(W.nchain_cap, B), false);
        {
          std::vector<Chain*> c1{W.acquire(false)};
          W.load_many(c1, {E.states[1].view()});
          W.store_many({&E.states[h->xi_base() + N - 1]}, c1);
          for (int s = 0; s + 1 < N && !abort_.load(); ++s) {
            W.step(c1, {u[N - 1 - s]}, {u[N - 2 - s]}, {0});
            W.store_many({&E.states[h->xi_base() + N - 2 - s]}, c1);
            PIPE_LOG("[pipe X] xi step %d\n", s);
          }
          W.sync();
          W.release(c1[0]);
        }
        PIPE_LOG("[pipe X] xi done, xiH in batches of %d\n", B);
        for (int t0 = 0; t0 < N && !abort_.load(); t0 += B) {
          const int nb = std::min(B, N - t0);
          std::vector<View> in;
          std::vector<Chain*> out;
          std::vector<State*> ss;
          for (int i = 0; i < nb; ++i) {
            in.push_back(E.states[h->xi_base() + t0 + i].view());
            out.push_back(W.acquire(false));
            ss.push_back(&E.states[h->xih_base() + t0 + i]);
          }
          W.apply_dH(in, out);
          W.store_many(ss, out);
          W.sync();
          for (auto* c : out) W.release(c);
        }
      } catch (...) {
        ex[1] = std::current_exception();
        abort_.store(1);
        (void)hipStreamSynchronize(WX.st);
        WX.release_all();
      }
    });
    // H: psiH_i = dH psi_i and its norm as psi_i appears, up to 8 rows per batch
    std::thread th([&] {
      try {
        HCK(hipSetDevice(dev));
        hbm::Engine& W = WH;
        constexpr int kJoin = 8;
        W.reserve_chains(std::max(W.nchain_cap, kJoin), false);
        for (int next = 0; next < nrows;) {
          wait_for(psi_ready, rs[next]);
          const int avail = psi_ready.load(std::memory_order_acquire);
          int end = next;
          while (end < nrows && rs[end] <= avail && end - next < kJoin) ++end;
          std::vector<View> in;
          std::vector<Chain*> out;
          std::vector<State*> ss;
          for (int k = next; k < end; ++k) {
            in.push_back(E.states[h->psi_base() + rs[k]].view());
            out.push_back(W.acquire(false));
            ss.push_back(&E.states[psih0 + k]);
          }
          W.apply_dH(in, out);
          std::vector<View> vs;
          for (auto* c : out) vs.push_back(c->view());
          const std::vector<double> n2 = W.site_norm2(vs, 1);
          for (int k = next; k < end; ++k) nrm[k] = std::sqrt(std::max(0.0, n2[k - next]));
          W.store_many(ss, out);
          W.sync();
          for (auto* c : out) W.release(c);
          psih_ready.store(end, std::memory_order_release);
          PIPE_LOG("[pipe H] rows ready %d of %d\n", end, nrows);
          next = end;
        }
      } catch (...) {
        ex[2] = std::current_exception();
        abort_.store(1);
        (void)hipStreamSynchronize(WH.st);
        WH.release_all();
      }
    });
    // A (this thread): the psi chain and the rows in one lockstep batch
    try {
      E.reserve_chains(std::max(E.nchain_cap, nrows + 1), false);
      struct RowRun {
        Chain* c;
        int k, t;  // row index in rs, time of the chain's state
      };
      Chain* psi = E.acquire(false);
      {
        std::vector<Chain*> p1{psi};
        E.load_many(p1, {E.states[0].view()});
        E.store_many({&E.states[h->psi_base()]}, p1);
        E.sync();
      }
      psi_ready.store(0, std::memory_order_release);
      std::vector<RowRun> act;
      int joined = 0, tpsi = 0;
      while (tpsi < N - 1 || !act.empty() || joined < nrows) {
        if (abort_.load()) throw hbm::Error(3, "pipelined getHessian: another stage failed");
        const int pr = psih_ready.load(std::memory_order_acquire);
        if (joined < pr) {  // rows whose psiH is ready join the batch (row N-2: diagonal only)
          std::vector<Chain*> jc;
          std::vector<View> jv;
          std::vector<int> jk;
          for (int k = joined; k < pr; ++k) {
            if (rs[k] >= N - 2) continue;
            jc.push_back(E.acquire(false));
            jv.push_back(E.states[psih0 + k].view());
            jk.push_back(k);
          }
          E.load_many(jc, jv);
          for (size_t m = 0; m < jk.size(); ++m) act.push_back({jc[m], jk[m], rs[jk[m]]});
          joined = pr;
        }
        std::vector<Chain*> cs;
        std::vector<double> uf, ut;
        std::vector<int> fw;
        std::vector<State*> ss;
        const bool with_psi = tpsi < N - 1;
        if (with_psi) {
          cs.push_back(psi);
          uf.push_back(u[tpsi]);
          ut.push_back(u[tpsi + 1]);
          fw.push_back(1);
          ss.push_back(&E.states[h->psi_base() + tpsi + 1]);
        }
        for (auto& r : act) {  // timeStepper.step(psiH, u[j-1], u[j]) (:269), j = t + 1
          cs.push_back(r.c);
          uf.push_back(u[r.t]);
          ut.push_back(u[r.t + 1]);
          fw.push_back(1);
          ss.push_back(&E.states[rsoff[r.k] + (r.t - rs[r.k])]);
        }
        if (cs.empty()) {  // everything joined so far is done: wait for the next row, if any
          if (joined >= nrows) break;
          wait_for(psih_ready, joined + 1);
          continue;
        }
        PIPE_LOG("[pipe A] step batch %zu (psi t %d, rows %zu, joined %d)\n", cs.size(), tpsi, act.size(), joined);
        E.step(cs, uf, ut, fw);
        E.store_many(ss, cs);
        E.sync();
        if (with_psi) psi_ready.store(++tpsi, std::memory_order_release);
        for (auto& r : act) ++r.t;
        std::vector<RowRun> keep;
        for (auto& r : act) {
          if (r.t >= N - 2) E.release(r.c);
          else keep.push_back(r);
        }
        act.swap(keep);
      }
      E.release(psi);
    } catch (...) {
      ex[0] = std::current_exception();
      abort_.store(1);
    }
    PIPE_LOG("[pipe A] done, joining\n");
    tx.join();
    th.join();
    PIPE_LOG("[pipe] joined\n");
    for (auto& e : ex)
      if (e) std::rethrow_exception(e);
    for (hbm::Engine* W : {&WH, &WX}) {  // the workers' GEMM statistics belong to this context
      W->sync();
      E.gemm_ms += W->gemm_ms;
      E.gemm_flops += W->gemm_flops;
      E.gemm_bytes += W->gemm_bytes;
      E.gemm_launches += W->gemm_launches;
      W->gemm_ms = W->gemm_flops = W->gemm_bytes = 0;
      W->gemm_launches = 0;
    }
    h->have_psi = h->have_xi = h->have_xih = true;
    // overlaps: F, divT, then every <xiH_j|psiH_i(j)> in one batch
    const std::complex<double> Fc =
        E.overlaps({E.states[h->psi_base() + N - 1].view()}, {E.states[1].view()}, false)[0];
    F[0] = Fc.real();
    F[1] = Fc.imag();
    std::vector<View> xs, ys;
    for (int t = 0; t < N; ++t) {
      xs.push_back(E.states[h->xi_base() + t].view());
      ys.push_back(E.states[h->psi_base() + t].view());
    }
    const auto dvr = E.overlaps(xs, ys, true);
    for (int t = 0; t < N; ++t) { divT[2 * t] = dvr[t].real(); divT[2 * t + 1] = dvr[t].imag(); }
    auto dv = [&](int i) { return std::complex<double>(divT[2 * i], divT[2 * i + 1]); };
    const std::complex<double> Fh(F[0], F[1]);
    xs.clear();
    ys.clear();
    for (int k = 0; k < nrows; ++k) {
      xs.push_back(E.states[h->xih_base() + rs[k]].view());
      ys.push_back(E.states[psih0 + k].view());
      for (int j = rs[k] + 1; j <= N - 2; ++j) {
        xs.push_back(E.states[h->xih_base() + j].view());
        ys.push_back(E.states[rsoff[k] + (j - rs[k] - 1)].view());
      }
    }
    const auto ov = E.overlaps(xs, ys, false);
    const double dt2 = E.dt * E.dt;
    size_t e = 0;
    for (int k = 0; k < nrows; ++k) {
      const int i = rs[k];
      H[size_t(i) * N + i] = dt2 * ((Fh * ov[e++]).real() - std::norm(dv(i)));  // (:259-264)
      for (int j = i + 1; j <= N - 2; ++j) {                                     // (:266-278)
        const double v1 = (Fh * ov[e++] * nrm[k]).real();
        const double v2 = -(dv(i) * std::conj(dv(j))).real();
        const double r = dt2 * (v1 + v2);
        H[size_t(i) * N + j] = r;
        H[size_t(j) * N + i] = r;
      }
    }
    tall.stop(long(N - 1) * 2 + long(rsoff[nrows] - rsoff[0]));
    undo.ok = true;
  });
}
