// Layout constants of the one-wave padded chain's plan image (host builder:
// fast_plan.hpp, device reader: fast_chain.hpp).  All entries are ints; every
// descriptor table starts 16-byte aligned and is read with b64 / b128 loads.
#pragma once

namespace ocg {
namespace fastp {

// compile-time bounds the device code unrolls to (a plan that exceeds one is
// not built, and the general chain steps)
constexpr int kMaxOps = 16;    // operations of one step
constexpr int kMaxDm = 4;      // middle-bond sector dimension of a Θ element / gauge product length
constexpr int kMaxDot = 16;    // Gram dot-product length (the larger side of a block)
constexpr int kMaxGram = 4;    // Gram block order (register Jacobi: 16-lane groups)
constexpr int kItTh = 2;       // Θ / matricisation elements per lane (<= 128)
constexpr int kItF = 4;        // factor elements per lane (<= 256)
constexpr int kItS = 4;        // gauge-product elements per lane (<= 256)
constexpr int kItMps = 4;      // padded MPS elements per lane (<= 256)

// header
enum {
  kHNp = 0,      // padded MPS complex elements
  kHNblk,        // blocks of the padded MPS
  kHBlk,         // block table: int4 {k | q << 8 | n << 16, dims index of the rows, dims index of the cols, first block of the site}
  kHLs,          // element table of the padded MPS: int4 {rows dims index | cols dims index << 16, blk | first << 16, a | c << 8, site_base[k] of the slot layout}
  kHSite,        // site element ranges [k] = first padded element of site k (k = 0..L+1)
  kHSiteN,       // per padded element of site 1: its physical index n (phases)
  kHNops,        // step operations
  kHZMps,        // complex offsets in the fast LDS region: MPS (its zero slot at index kHNp),
  kHZTh,         //   matricisation / Θ,
  kHZTg,         //   gated Θ,
  kHZW,          //   eigenvector blocks (4 groups x 16),
  kHZX,          //   factor scratch of gauge moves,
  kHZGt,         //   gate tables (forward, backward),
  kHZPh,         //   phases UF[p], UT[p]
  kHZTot,        // complex elements of the region
  kHNint,        // ints of the plan image
  kHCentre,      // orthogonality centre after a step without the closing move
  kHThZ,         // the zero slot of the Θ / gated-Θ buffers (complex index; never written)
  kHXsZ,         // the zero slot of the factor scratch
  kHOps,         // kMaxOps op offsets follow
  kHdrInts = kHOps + kMaxOps
};
// step operations
enum { kOpGate = 0, kOpGaugeR = 1, kOpGaugeL = 2 };
// op header (kOpHdr ints, 16-byte aligned; ld4 reads at offsets 0, 4, kOhGrp + 4 k)
enum {
  kOhKind = 0, kOhK, kOhDir, kOhMode,
  kOhLonely, kOhClosing, kOhNth, kOhNewBond,
  kOhMat,    // M elements: gate int2 (x1 | x2 << 16, dm | drc << 8), gauge int (source)
  kOhGate,   // gate descriptors: int4 per element
  kOhNsec, kOhT,
  kOhNgrp, kOhMaxr,  // Jacobi groups, rounds per sweep (0, 1 or 3)
  kOhO1, kOhNo1,     // order-1 sectors: int4 {M offset, length, stride, eigen slot}
  kOhEq,             // eigen slot e: int4 {s, i, eoff of s, n of s | bound << 8}
  kOhSecQ,           // sector s: q | eigen offset << 8 | order << 16 (ints)
  kOhF, kOhNf,       // factor elements: int4 (see fast_plan.hpp)
  kOhS, kOhNs,       // gauge product elements: int4 {x1 | x2 << 16, len | s2 << 16, dest, 0}
  kOhDot,            // longest Gram / order-1 dot product of the decomposition
  kOhGrp = 24,       // 4 groups x 8 ints: s, n, side, tho, R, C, eoff, 0 (16-byte aligned)
  kOpHdr = kOhGrp + 32
};

static_assert(kOhGrp % 4 == 0 && kOhNewBond < 8, "b128 reads of the op header");

// Overlap plan (fast_overlap.hpp; host builder build_overlap_plan in fast_plan.hpp):
// <X|Y> of two compact-format states contracted in the padded layout,
// E_k[q'] = sum_n X_(q'-n,n)^H E_(k-1)[q'-n] Y_(q'-n,n), every index fixed by the
// rank bounds.  Header ints, then the tables at the offsets the header holds:
constexpr int kOvMaxE = 128;  // environment elements per bond (sum over sectors of D^2)
constexpr int kOvMaxP = 6;    // local dimension (the unrolled stage-2 sum over n)
enum {
  kOvL = 0, kOvQ1, kOvP, kOvNp, kOvNblk,
  kOvMaxSite,  // largest padded site
  kOvMaxEn,    // largest environment
  kOvD,        // bounds D[(L+1) * Q1]
  kOvEo,       // environment offsets eo[(L+1) * Q1] (prefix over sectors of D^2)
  kOvEn,       // environment sizes en[L+1]
  kOvPo,       // padded block offsets within the site po[(L+2) * Q1 * p], -1: none
  kOvSb,       // site starts sb[L+2] in the padded image
  kOvElo,      // environment element lists: bond b's at elo[b] (L+2 ints)
  kOvEl,       // element x of E_b: q | c' << 8 | c << 12 | D(b, q) << 16
  kOvLs,       // per padded element, int4 (16-byte aligned):
               //   rows dims idx | cols dims idx << 16, block | first block << 16,
               //   a | c << 4 | D(k-1, q) << 8 | D(k, q+n) << 12 | eo(k-1, q) << 16, site_base[k]
  kOvBlk,      // per block: rows dims idx | cols dims idx << 16 (the compact size)
  kOvNint,     // ints of the plan
  kOvHdr = 20
};
}  // namespace fastp
}  // namespace ocg
