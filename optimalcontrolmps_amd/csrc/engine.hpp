// Shared host/device definitions of the MI355X tDMRG chain engine.
//
// One workgroup owns one MPS "chain" (a psi_t / xi_t trajectory, or one
// Hessian row's re-propagated psiH) resident in LDS for its whole life;
// every Trotter sweep, U(1)-block eigen-decomposition, truncation, gauge move,
// dH compression and overlap of that chain runs inside the workgroup.
// See DESIGN.md §Engine for the data layout and roofline.
#pragma once

#include <stdint.h>

#define OCG_MAXL 48      // sites
#define OCG_MAXQ1 64     // particle-number sectors (Q+1)
#define OCG_MAXP 12      // local dimension p = d+1
#define OCG_MAXGATES 48
#define OCG_MAXD (2 * OCG_MAXP)

// Kernel parameter block (passed by value).  All capacities are in complex
// (16-byte) elements unless noted.
struct OcgParams {
  int L, p, Q, Q1;          // sites, local dim, particle number, Q+1
  int nsq;                  // (L+1)*Q1 ints of bond-sector dims per slot
  int cap;                  // complex elements per MPS slot
  int site_base[OCG_MAXL + 1];  // [k] base of site k's region (k = 1..L)
  int site_cap[OCG_MAXL + 1];   // [k] capacity of site k's region
  int max_site_cap;
  int thcap;                // two-site / matricisation scratch capacity
  int ecap;                 // overlap environment capacity (per environment)
  int evcap;                // eigen-pair list capacity
  int nrot;                 // rotation-table capacity (pairs)
  double dt, cutoff;
  int maxm;
  double dH[OCG_MAXP];      // 0.5 n (n-1)
  int ngates;
  int gate_i1[OCG_MAXGATES];
  int glo[OCG_MAXD], gsz[OCG_MAXD], goff[OCG_MAXD];  // per-Δ gate blocks
  int gtotal;               // complex entries of one direction's gate table
  int lds_bytes;            // dynamic LDS of one chain workgroup
  int th2cap;               // two-site Θ elements bound (physical bonds)
  int nplan;                // decomposition plan slots in LDS (0: plans off)
  int plan_pe;              // Θ elements a plan slot can describe
  int imag;                 // 1: imaginary-time steps exp(-dt H) (ground-state preparation), 0: exp(-i dt H)
  int* err;                 // device error word of the context (bit 0: Jacobi sweep cap
                            // reached, bit 1: pipeline watchdog); checked after every launch
  const int* fplan;         // plan image of the one-wave padded chain (fast_chain.hpp), or null:
                            // every step of the kernels that step runs on it
  int fast_off;             // byte offset of its region in the dynamic LDS
  const int* oplan;         // overlap plan of the padded layout (fast_overlap.hpp), or null: the
                            // row overlaps of getHessian run on the general contraction
  int ovl_bytes;            // LDS of the padded overlap (k_row_overlaps_pad; <= fast_off)
  int ovl_dh_bytes;         // LDS of the padded <x|y> / <x|dH|y> pairs (k_overlaps_pad)
};
#define OCG_ERR_JACOBI 1
#define OCG_ERR_WATCHDOG 2

// Truncation used for gauge moves and the left-to-right half of the dH
// compression (ITensor MPS::position / orthogonalize; parity unpinned, the
// oracle uses the same value: oracle/tdmrg_oracle.hpp kGaugeCutoff).
#define OCG_GAUGE_CUTOFF 1e-14
