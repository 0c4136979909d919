/*
 * ocmps.h — C-ABI of the MI355X-native gradient/Hessian inner loop of
 * fskovbo/OptimalControlMPS (BH_tDMRG time-stepper + OptimalControl
 * contractions), implemented by liboptimalcontrolmps_amd.so.
 *
 * Plain pointers and sizes only; no exceptions cross this boundary.  Every
 * function returns 0 on success or a nonzero OCG_E* code, with a message in
 * ocg_last_error(ctx).  The C++ facade (optimalcontrolmps/OptimalControl.hpp)
 * rethrows as std::runtime_error.  Reference citations are path:line in the
 * reference repository.
 *
 * MPS interchange format ("compact U(1) blocks", the IQMPS replacement):
 *   dims : int[(L+1)*(Q+1)]   dims[b*(Q+1)+q] = # states of bond b (between
 *          sites b and b+1; bond 0 and bond L are trivial) whose left particle
 *          count is q.  Q = number of bosons.
 *   data : double[2*nelem]    complex, interleaved (re, im); for site
 *          k = 1..L, sector q = 0..Q, occupation n = 0..p-1 with q+n <= Q and
 *          both dims nonzero: the block A_k[(q,n)] of dims[k-1][q] x
 *          dims[k][q+n] entries, row-major.
 * Every MPS handed in must be right-orthonormal with its orthogonality centre
 * at site 1 (the form BH_tDMRG::step leaves, src/BH_tDMRG.cpp:217-228).
 */
#ifndef OCMPS_H
#define OCMPS_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCG_OK 0
#define OCG_EINVAL 1    /* bad argument / shape */
#define OCG_ECAP 2      /* caller buffer too small, or problem exceeds engine capacity */
#define OCG_EHIP 3      /* HIP runtime error (no GPU, launch failure, ...) */
#define OCG_ESTATE 4    /* call order violated (e.g. rows before trajectories) */
#define OCG_ENUM 5      /* numerical failure flagged by a kernel */
#define OCG_ENOMEM 6    /* device or pinned host allocation failed (HBM engine) */

typedef struct ocg_ctx ocg_ctx;

/* Engine limits and per-context sizes (for callers sizing buffers). */
typedef struct ocg_info {
  int L, p, Q;
  size_t mps_max_nelem;   /* complex elements of the largest MPS this context can hold */
  int lds_bytes;          /* dynamic LDS of one chain workgroup */
  int block_threads;      /* threads per chain workgroup */
  int device;
  int fast_chain;         /* 1: every step runs on the one-wave padded chain (LDS engine, small bonds) */
} ocg_info;

/* --------------------------------------------------------------- context
 * Replaces BH_tDMRG(sites, J, tstep, {"Cutoff=",cutoff,"Maxm=",maxm})
 * (reference include/BH_tDMRG.hpp:34, src/BH_tDMRG.cpp:3-15): Bose-Hubbard
 * chain of L sites, local dimension p (= BoseHubbard d + 1), npart bosons,
 * hopping J, Trotter step tstep.  maxm <= 0 means ITensor's default (5000).
 * Builds the forward/backward hopping gates (initJGates, :18-58) and the
 * dH = sum_k 0.5 n_k(n_k-1) MPO data (:10-14) on `device`. */
int ocg_create(int device, int L, int p, int npart, double J, double tstep, double cutoff, int maxm,
               ocg_ctx** out);
/* As ocg_create, choosing the engine: 0 auto (the single-workgroup LDS chain
 * engine when the configuration fits it, else the HBM-resident engine),
 * 1 LDS chain engine only (OCG_ECAP if it does not fit), 2 HBM-resident
 * engine (multi-workgroup, MFMA-FP64 contractions; configurations such as
 * L=20, p=7, chi=256).  Both engines implement every entry point below with
 * the same arithmetic. */
int ocg_create_ex(int device, int L, int p, int npart, double J, double tstep, double cutoff, int maxm, int engine,
                  ocg_ctx** out);
/* number of visible HIP devices (OCG_EHIP and *n = 0 without a GPU) */
int ocg_device_count(int* n);
int ocg_destroy(ocg_ctx* ctx);
/* last error message of ctx (or of the last failed ocg_create when ctx == NULL) */
const char* ocg_last_error(const ocg_ctx* ctx);
/* writes sizeof(ocg_info) bytes of the header the library was built with
 * (ABI version 3: fast_chain is the last field); callers built against
 * another version use ocg_get_info_sz */
int ocg_get_info(const ocg_ctx* ctx, ocg_info* info);
/* as ocg_get_info, writing at most info_size bytes (the caller's sizeof(ocg_info)) */
int ocg_get_info_sz(const ocg_ctx* ctx, ocg_info* info, size_t info_size);
/* ABI version of the library (OCG_ABI_VERSION of the header it was built with).
 * Changelog: 2 ocg_info.fast_chain (round 5), OCG_ENOMEM returned by
 * ocg_hessian when OCG_HBM_PIPE=1 forces a pipeline that cannot allocate;
 * 3 ocg_get_info_sz, ocg_get_path_stats, ocg_abi_version (round 6). */
#define OCG_ABI_VERSION 3
int ocg_abi_version(void);
/* BH_tDMRG::setTstep (src/BH_tDMRG.cpp:61-65) */
int ocg_set_tstep(ocg_ctx* ctx, double tstep);
/* number of complex elements of an MPS with the given dims */
size_t ocg_mps_nelem(int L, int p, int Q, const int* dims);

/* ------------------------------------------ TimeStepper-level operations
 * Host MPS in, host MPS out (compact format above).  out_cap is the capacity
 * of out_data in complex elements; *out_nelem receives the size written. */

/* BH_tDMRG::step(psi, from, to, propagateForward) (src/BH_tDMRG.cpp:111-230) */
int ocg_step(ocg_ctx* ctx, const int* dims, const double* data, double from, double to, int forward,
             int* out_dims, double* out_data, size_t out_cap, size_t* out_nelem);
/* nsteps consecutive steps with controls u[0..nsteps] (step i: u[i] -> u[i+1]) */
int ocg_steps(ocg_ctx* ctx, const int* dims, const double* data, const double* u, int nsteps, int forward,
              int* out_dims, double* out_data, size_t out_cap, size_t* out_nelem);
/* Batched BH_tDMRG::step over n independent states, one device launch
 * (SURVEY.md §8b `ocg_step_batch`): state i = (dims + i*(L+1)*(Q+1), data[i])
 * takes one step u_from[i] -> u_to[i] in direction `forward`; the result goes
 * to (out_dims + i*(L+1)*(Q+1), out_data[i]) of capacity out_cap[i] complex
 * elements, size in out_nelem[i].  Uses scratch slots after the trajectories
 * (device psi_t / xi_t / xiH_t are left intact). */
int ocg_step_batch(ocg_ctx* ctx, int n, const int* dims, const double* const* data, const double* u_from,
                   const double* u_to, int forward, int* out_dims, double* const* out_data, const size_t* out_cap,
                   size_t* out_nelem);
/* Ground-state preparation on the device (replaces ITensor DMRG in
 * InitializeState, include/InitializeState.hpp:18-117): nsteps imaginary-time
 * Trotter steps exp(-tau H_BH(J, U)) of the state, the sweep of
 * BH_tDMRG::step with exp(-tau h) gates and exp(-tau U n(n-1)/4) phases,
 * normalised, truncated with the context's Cutoff/Maxm.  The context's
 * real-time gates and device trajectories are left as they were.  The C++
 * facade's InitializeState runs a tau schedule over this. */
int ocg_imag_steps(ocg_ctx* ctx, const int* dims, const double* data, double U, double tau, int nsteps,
                   int* out_dims, double* out_data, size_t out_cap, size_t* out_nelem);
/* InitializeState's ground state (include/InitializeState.hpp:18-117) in one
 * call with the state resident on the device: for each tau of taus[0..ntau),
 * imaginary-time steps (as ocg_imag_steps) in blocks of `block` until
 * 1 - |<state before the block|state after>| < tol or max_steps per stage; one
 * device overlap per block, no host round trip.  Returns the final state;
 * *steps_done (optional) = total steps taken.  Real-time gates and device
 * trajectories are left as they were. */
int ocg_ground_state(ocg_ctx* ctx, const int* dims, const double* data, double U, int ntau, const double* taus,
                     int block, double tol, int max_steps, int* out_dims, double* out_data, size_t out_cap,
                     size_t* out_nelem, int* steps_done);
/* overlapC(x, y) = <x|y> (with_dH = 0) or overlapC(x, propDeriv, y) = <x|dH|y>
 * (with_dH = 1) (src/OptimalControl.cpp:242, :412); out = {re, im} */
int ocg_overlap(ocg_ctx* ctx, const int* dims_x, const double* x, const int* dims_y, const double* y,
                int with_dH, double* out);
/* exactApplyMPO(propDeriv, psi, args) (src/OptimalControl.cpp:256); *norm = ||result|| */
int ocg_apply_dH(ocg_ctx* ctx, const int* dims, const double* data, int* out_dims, double* out_data,
                 size_t out_cap, size_t* out_nelem, double* norm);

/* ----------------------------------------- OptimalControl hot path
 * Device-resident trajectories for one control vector u[0..N-1].
 * OptimalControl ctor copies of psi_target / psi_init (src/OptimalControl.cpp:10-34). */
int ocg_set_states(ocg_ctx* ctx, const int* dims_target, const double* target, const int* dims_init,
                   const double* init);
/* calcPsi (which & 1, src/OptimalControl.cpp:375-390) and calcXi (which & 2,
 * :392-407); both chains run concurrently when which == 3 (calcPsiXiDivT's
 * two threads, :421-438). */
int ocg_propagate(ocg_ctx* ctx, const double* u, int N, int which);
/* overlapFactor = overlapC(psi_t[N-1], psi_target) (src/OptimalControl.cpp:242) */
int ocg_overlap_factor(ocg_ctx* ctx, double* F);
/* fid[i] = |<psi_target|psi_t[i]>|^2 (calcFidelityForAllT, :548-569) */
int ocg_fidelities(ocg_ctx* ctx, double* fid);
/* divT[i] = overlapC(xi_t[i], propDeriv, psi_t[i]) (calcDivT, :409-419); 2N doubles */
int ocg_div_t(ocg_ctx* ctx, double* divT);
/* xiHlist[i] = exactApplyMPO(propDeriv, xi_t[i], args) for all i (:300-303) */
int ocg_xi_dH(ocg_ctx* ctx);
/* calcHessianRow (:251-279) for rows[0..nrows-1] (each in 1..N-2), F and divT
 * as produced above (F: 2 doubles, divT: 2N doubles).  Writes the fidelity
 * Hessian entries (i, j>=i) and their mirrors into H (row-major N x N,
 * caller-zeroed; entries of different rows are disjoint); the regularisation
 * Hessian is the caller's.  Requires ocg_propagate(..,3) + ocg_xi_dH. */
int ocg_hessian_rows(ocg_ctx* ctx, const double* u, int N, const int* rows, int nrows, const double* F,
                     const double* divT, double* H);
/* One full getHessian(u, new_control = true) fidelity part, fused
 * (calcHessian_parallel, src/OptimalControl.cpp:281-338, without the
 * regularisation Hessian, which is the caller's): psi_t and xi_t, xiHlist,
 * divT, F and the rows[0..nrows-1] (each in 1..N-2).  Rows start as soon as
 * their psi_i is available and the <xiH_j|psiH> overlaps run as one batched
 * launch afterwards; arithmetic per row is that of ocg_hessian_rows.  H is
 * row-major N x N, caller-zeroed (rows' entries and mirrors written); divT
 * (2N doubles) and F (2) are returned for the gradient.  Leaves the same
 * device state as ocg_propagate(..,3) + ocg_xi_dH. */
int ocg_hessian(ocg_ctx* ctx, const double* u, int N, const int* rows, int nrows, double* H, double* divT,
                double* F);
/* K control vectors u[k*N .. k*N+N) in one call (IPOPT line-search trial
 * points, finite-difference probes, multi-start; no reference counterpart: the
 * reference evaluates one getHessian at a time, src/OptimalControl.cpp:281-338).
 * LDS engine: one k_pipeline launch carries all K controls' psi / xi chains,
 * xiH workers and rows (tickets keep every waiter behind its producers), then
 * one batched divT / F launch and one row-overlap launch; per control exactly
 * the arithmetic of ocg_hessian (the same H bit for bit).  HBM engine: the
 * controls in turn.  H: K row-major N x N blocks, caller-zeroed; divT: K x 2N;
 * F: K x 2.  Leaves control 0's trajectories as ocg_hessian would. */
int ocg_hessian_multi(ocg_ctx* ctx, int K, const double* u, int N, const int* rows, int nrows, double* H,
                      double* divT, double* F);
/* getAnalyticGradient's device work for one control vector (calcPsi || calcXi,
 * calcDivT and F = <psi_{N-1}|psi_target>, src/OptimalControl.cpp:204-249,
 * :375-419): divT (2N doubles, complex) and F (2 doubles).  = ocg_propagate(..,3)
 * + ocg_div_t + ocg_overlap_factor, whose trajectories it leaves on the device,
 * unless the HBM engine's stored trajectories would not fit half the free HBM
 * (config 5 at N_t = 1001): then psi and xi run as one lockstep batch that
 * meets in the middle (psi_0..psi_{N/2} and xi_{N/2+1}..xi_{N-1} stored, the
 * other halves paired as they are produced): N states instead of 2N, the same
 * N-1 dependent steps, the same numbers bit for bit, no trajectories left
 * (OCG_HBM_MID=1 / 0 forces either path). */
int ocg_gradient(ocg_ctx* ctx, const double* u, int N, double* divT, double* F);
/* The gradient's device work (calcPsi || calcXi + divT + F, the BFGS path of
 * calcFidelityGrad, src/OptimalControl.cpp:204-249) for K control vectors
 * u[k*N .. k*N+N) in one call: LDS engine, one trajectory launch of 2K chains
 * and one batched divT / F launch each (per control exactly the arithmetic of
 * ocg_propagate(..,3) + ocg_div_t + ocg_overlap_factor); HBM engine, one
 * lockstep batch of 2K chains + one batched divT / F overlap launch each when
 * the grown state heap (the context's slots + 2N per extra control) fits half
 * the free HBM (the extra slots are released afterwards), else — or when the
 * batched call fails to allocate — the controls in turn.  Either way the same
 * numbers bit for bit.  divT: K x 2N, F: K x 2; grad_k,i = dt Re(i divT_k,i F_k)
 * (plus the caller's regularisation).  Leaves control 0's trajectories. */
int ocg_gradient_multi(ocg_ctx* ctx, int K, const double* u, int N, double* divT, double* F);
/* which: 0 psi_t, 1 xi_t, 2 xiHlist; copy trajectory state t to the host.
 * Gauge: the chains skip doStep's closing position(1) (src/BH_tDMRG.cpp:206-218)
 * on every step but their last, so an intermediate psi_t / xi_t is the same
 * state with its orthogonality centre on the last gate's left site (site 2 for
 * L >= 3) instead of site 1; the final states (psi_{N-1}, xi_0) and everything
 * ocg_steps returns are in the reference's gauge. */
int ocg_get_state(ocg_ctx* ctx, int which, int t, int* dims, double* data, size_t cap, size_t* nelem);

/* ControlBasis::convertHessian (src/ControlBasis.cpp:91-116) on the device:
 * Hc (M x M) = V Hu V^T with Hu row-major N x N (host), V row-major M x N
 * (V[n][i] = S_i f_{i n}, the transposed control Jacobian).  Each entry is a
 * sequential inner product in the reference's order without fused
 * multiply-adds: bit-identical to the host restatement.  Any engine. */
int ocg_convert_hessian(ocg_ctx* ctx, const double* Hu, int N, const double* V, int M, double* Hc);

/* ITensor denmatDecomp(M, A, B, Fromleft, {"Cutoff=",cutoff,"Maxm=",maxm})
 * (called at src/BH_tDMRG.cpp:178, :191, :209) of nm independent dense
 * blocks M[i] (rows[i] x cols[i] complex, row-major, 0 < rows <= cols <= any,
 * rows <= 512), each one U(1) sector: the decomposition every two-site update
 * of the HBM engine runs (Gram M M^H, Hermitian eigensolver, truncation rule,
 * eigenvectors, factors), on caller-supplied matrices, batched in one pass.
 * kept[i] = k; A[i] (rows x k, orthonormal columns) and B[i] = A^H M (k x
 * cols), both row-major complex, caller buffers of rows*rows / rows*cols
 * complex elements (NULL: not returned); w[i] (rows doubles, NULL: not
 * returned) = the Gram eigenvalues as the eigensolver leaves them (order not
 * specified; those below ~1e-3 cutoff / rows of the trace may be unresolved).
 * HBM engine contexts only (ocg_create_ex engine 2); else OCG_EINVAL. */
int ocg_denmat_decomp(ocg_ctx* ctx, int nm, const int* rows, const int* cols, const double* const* M,
                      double cutoff, int maxm, int* kept, double* const* w, double* const* A, double* const* B);

/* ------------------------------------------------------ instrumentation
 * Per-kernel HIP-event timing on the context's stream and the algorithmic
 * traffic model of DESIGN.md §Roofline.  kind: 0 trajectory, 1 overlaps,
 * 2 dH apply, 3 Hessian rows, 4 steps, 5 fused pipeline (ocg_hessian phase 1),
 * 6 batched row overlaps (ocg_hessian phase 2), 7 the HBM engine's MFMA GEMM
 * kernel (k_gemm: HIP-event time, algorithmic bytes and flops of its tasks;
 * zeros on the LDS engine), 8 the HBM engine's getHessian path counters
 * (*launches = pipelined getHessians completed, *sweep_steps = two-phase
 * retries after a pipeline that failed with OCG_ENOMEM; never with
 * OCG_HBM_PIPE=1, which makes any pipeline failure the call's status),
 * *alg_flops = trajectory-checkpointed getHessians completed, *alg_bytes = the
 * segment length of the last one).  Sums since the last reset. */
int ocg_kernel_stats(ocg_ctx* ctx, int kind, double* total_ms, long* launches, double* alg_bytes,
                     double* alg_flops, long* sweep_steps);
int ocg_reset_stats(ocg_ctx* ctx);
/* Which paths the HBM engine's calls took since the context was created (named
 * counters; ocg_kernel_stats kind 8 returns the first four through its timing
 * fields and stays for old callers).  The caller sets out->size =
 * sizeof(ocg_path_stats); only that many bytes are written.  Zeros on the LDS
 * engine. */
typedef struct ocg_path_stats {
  size_t size;           /* set by the caller: sizeof(ocg_path_stats) of its header */
  long pipe_runs;        /* pipelined getHessians completed */
  long pipe_fallbacks;   /* two-phase reruns after a pipeline that failed with OCG_ENOMEM */
  long ckpt_runs;        /* trajectory-checkpointed getHessians completed */
  long ckpt_k;           /* segment length of the last checkpointed getHessian */
  long coop_launches;    /* multi-CU eigenvalue launches (k_heev_vals_coop) */
  long coop_groups;      /* Gram blocks reduced by a group of workgroups */
  long coop_fallbacks;   /* of those, groups that gave up a wait and were re-run on one CU */
} ocg_path_stats;
int ocg_get_path_stats(ocg_ctx* ctx, ocg_path_stats* out);
/* diagnostic builds (-DOCG_PROFILE) only: shader-clock cycles per engine phase
 * (32 slots, see engine_device.hpp Chain::pf), summed over workgroups; zeros in
 * the product build.  reset != 0 clears after reading. */
int ocg_profile(ocg_ctx* ctx, double* out32, int reset);

#ifdef __cplusplus
}
#endif
#endif /* OCMPS_H */
