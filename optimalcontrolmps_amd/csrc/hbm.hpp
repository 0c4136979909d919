// Host interface between the C-ABI (ocmps.hip) and the HBM-resident engine
// (hbm.hip).  Same argument meaning and return codes as the ocg_* entry
// points of include/ocmps.h they back; an ocg_ctx whose configuration does
// not fit the LDS chain engine (or that asked for this engine) forwards here.
#pragma once

#include <cstddef>
#include <string>
#include <vector>

struct hbm_engine;

int hbm_create(int device, int L, int p, int npart, double J, double tstep, double cutoff, int maxm,
               const std::vector<int>& md, const std::vector<int>& mdz, const std::vector<double>& gf,
               const std::vector<double>& gb, const int* glo, const int* gsz, const int* goff, int gtotal,
               const std::vector<int>& gates, hbm_engine** out, std::string& err);
void hbm_destroy(hbm_engine* h);
const char* hbm_last_error(const hbm_engine* h);
size_t hbm_mps_max_nelem(const hbm_engine* h);
int hbm_set_tstep(hbm_engine* h, double tstep, const std::vector<double>& gf, const std::vector<double>& gb,
                  const int* glo, const int* gsz, const int* goff, int gtotal);
// swap the step's gates and time mode (imag: exp(-dt H)) without touching the
// device trajectories (ocg_imag_steps switches in and back out)
int hbm_swap_gates(hbm_engine* h, int imag, double tstep, const std::vector<double>& gf,
                   const std::vector<double>& gb, const int* glo, const int* gsz, const int* goff, int gtotal);
// n states (dims[i], data[i]) take nsteps steps each, controls u[i*u_stride + s]
int hbm_steps(hbm_engine* h, int n, const int* dims, const double* const* data, const double* u, int u_stride,
              int nsteps, const int* fwd, int* out_dims, double* const* out_data, const size_t* out_cap,
              size_t* out_nelem);
int hbm_overlap(hbm_engine* h, const int* dx, const double* x, const int* dy, const double* y, int with_dH,
                double* out);
int hbm_apply_dH(hbm_engine* h, const int* dims, const double* data, int* out_dims, double* out_data, size_t cap,
                 size_t* nelem, double* norm);
int hbm_set_states(hbm_engine* h, const int* dims_target, const double* target, const int* dims_init,
                   const double* init);
int hbm_propagate(hbm_engine* h, const double* u, int N, int which);
int hbm_overlap_factor(hbm_engine* h, double* F);
int hbm_fidelities(hbm_engine* h, double* fid);
int hbm_div_t(hbm_engine* h, double* divT);
// K controls (rows of U) in one batch of 2K chains + batched divT / F (ocg_gradient_multi)
int hbm_gradient_multi(hbm_engine* h, int K, const double* U, int N, double* divT, double* F);
int hbm_xi_dH(hbm_engine* h);
int hbm_hessian_rows(hbm_engine* h, const double* u, int N, const int* rows, int nrows, const double* F,
                     const double* divT, double* H);
// divT_t and F without stored trajectories: psi || xi meeting in the middle,
// N states instead of 2 N, bit-identical to propagate + div_t + overlap_factor
int hbm_gradient_mid(hbm_engine* h, const double* u, int N, double* divT, double* F);
// getHessian's fidelity part (psi, xi, divT, F, rows) with trajectory
// checkpointing: psi_t / xi_t kept only every K steps,
// segments recomputed, xiHlist formed one segment at a time; O(N/K + K + rows
// of a batch) states instead of 3 N.  Bit-identical to the stored path.
// Leaves no device trajectories (ocg_get_state fails afterwards).
int hbm_hessian_ckpt(hbm_engine* h, const double* u, int N, const int* rows, int nrows, double* H, double* divT,
                     double* F, int K);
// bytes the stored-trajectory Hessian's 3 N + 6 state slots would newly allocate
// (0 when the context's state heap already holds them)
double hbm_traj_bytes(const hbm_engine* h, int N);
// bytes hbm_gradient_multi would newly allocate: its 3 N + 6 + 2 N (K - 1) state
// slots and 2 K chains (0 when the engine already holds them)
double hbm_gradient_multi_bytes(const hbm_engine* h, int K, int N);
int hbm_get_state(hbm_engine* h, int which, int t, int* dims, double* data, size_t cap, size_t* nelem);
// kinds 0-6 as ocg_kernel_stats (HIP-event phase times); 7: the MFMA GEMM
// kernel (k_gemm) with its algorithmic bytes and flops
int hbm_stats(hbm_engine* h, int kind, double* ms, long* launches, double* bytes, double* flops, long* steps);
// multi-CU eigenvalue launches, blocks reduced by groups, groups re-run on one CU
// (the context engine and the pipelined getHessian's workers, since creation)
int hbm_coop_stats(hbm_engine* h, long* launches, long* groups, long* fallbacks);
void hbm_reset_stats(hbm_engine* h);
bool hbm_have(const hbm_engine* h, int what);  // 0 states, 1 psi, 2 xi, 3 xiH
int hbm_N(const hbm_engine* h);
// denmatDecomp (Fromleft) of nm independent dense blocks (ocg_denmat_decomp)
int hbm_denmat_decomp(hbm_engine* h, int nm, const int* rows, const int* cols, const double* const* M, double cutoff,
                      int maxm, int* kept, double* const* w, double* const* X, double* const* Y);
// InitializeState's imaginary-time schedule with the state resident on the device (ocg_ground_state)
int hbm_ground_state(hbm_engine* h, const int* dims, const double* data, double U, int ntau, const double* taus,
                     const std::vector<std::vector<double>>& gf, const std::vector<std::vector<double>>& gb,
                     const int* glo, const int* gsz, const int* goff, int gtotal, double dt0,
                     const std::vector<double>& gf0, const std::vector<double>& gb0, int block, double tol,
                     int max_steps, int* out_dims, double* out_data, size_t cap, size_t* nelem, int* steps_done);
// getHessian's fidelity part with the psi chain + rows, the dH applications and
// the xi chain pipelined on three engines (one stream each), row states stored
// for one batched overlap pass; bit-identical to propagate + xi_dH + rows
int hbm_hessian_pipe(hbm_engine* h, const double* u, int N, const int* rows, int nrows, double* H, double* divT,
                     double* F);
// bytes hbm_hessian_pipe would newly allocate: its slots (trajectories + psiH_i +
// row states; 0 when the heap already holds them, e.g. from the last call) and the
// chain pools of the context engine (psi + every row) and of the two workers
double hbm_pipe_bytes(const hbm_engine* h, int N, const int* rows, int nrows);
