// TEST INFRASTRUCTURE ONLY — host emulation shim used by tests/emu/emu.cpp to
// execute the unmodified device bodies (optimalcontrolmps_amd/csrc/
// kernels.hpp) on CPU threads for debugging.  One std::thread per lane of
// the single 64-lane wave; wave intrinsics go through an exchange buffer and
// the block barrier (every call site must be wave-uniform, as on the GPU).
// Never part of the product build, never loaded by the product path.
#pragma once
#include <atomic>
#include <barrier>
#include <cmath>
#include <cstdint>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(x)
#define __align__(x) alignas(x)

struct double2 {
  double x, y;
};
inline double2 make_double2(double x, double y) { return double2{x, y}; }
struct emu_dim3 {
  unsigned x = 0, y = 0, z = 0;
};
extern thread_local emu_dim3 threadIdx, blockIdx;
extern thread_local std::barrier<>* emu_bar;   // workgroup barrier
extern thread_local std::barrier<>* emu_wbar;  // barrier of this thread's wave
extern thread_local uint64_t* emu_xbuf;        // exchange buffer of the block (one slot per thread)
inline void __syncthreads() { emu_bar->arrive_and_wait(); }
inline int atomicOr(int* p, int v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
inline int atomicAdd(int* p, int v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
inline double atomicAdd(double* p, double v) {
  std::atomic_ref<double> r(*p);
  return r.fetch_add(v);
}
template <class T>
inline T emu_xchg(T v, int src) {
  static_assert(sizeof(T) <= 8, "");
  uint64_t b = 0;
  __builtin_memcpy(&b, &v, sizeof(T));
  const unsigned w = threadIdx.x & ~63u;
  emu_xbuf[threadIdx.x] = b;
  emu_wbar->arrive_and_wait();
  uint64_t r = emu_xbuf[w + (src & 63)];
  emu_wbar->arrive_and_wait();
  T out;
  __builtin_memcpy(&out, &r, sizeof(T));
  return out;
}
template <class T>
inline T __shfl(T v, int src, int w = 64) { return emu_xchg(v, src); }
template <class T>
inline T __shfl_up(T v, unsigned d, int w = 64) {
  int l = threadIdx.x & 63;
  T r = emu_xchg(v, l >= (int)d ? l - (int)d : l);
  return r;
}
template <class T>
inline T __shfl_down(T v, unsigned d, int w = 64) {
  int l = threadIdx.x & 63;
  T r = emu_xchg(v, l + (int)d < 64 ? l + (int)d : l);
  return r;
}
template <class T>
inline T __shfl_xor(T v, int m, int w = 64) { return emu_xchg(v, (threadIdx.x & 63) ^ m); }
inline unsigned long long __ballot(int pred) {
  const unsigned w = threadIdx.x & ~63u;
  emu_xbuf[threadIdx.x] = pred ? 1 : 0;
  emu_wbar->arrive_and_wait();
  unsigned long long m = 0;
  for (int i = 0; i < 64; ++i) m |= (emu_xbuf[w + i] ? 1ULL : 0ULL) << i;
  emu_wbar->arrive_and_wait();
  return m;
}
inline int __popcll(unsigned long long m) { return __builtin_popcountll(m); }
inline double emu_rcp(double x) { return 1.0 / x; }
#define __builtin_amdgcn_rcp(x) emu_rcp(x)
inline double rsqrt(double x) { return 1.0 / std::sqrt(x); }
inline int max(int a, int b) { return a > b ? a : b; }
inline int min(int a, int b) { return a < b ? a : b; }
inline long long __double_as_longlong(double v) { long long r; __builtin_memcpy(&r, &v, 8); return r; }
inline double __longlong_as_double(long long v) { double r; __builtin_memcpy(&r, &v, 8); return r; }
inline int emu_readlane(int v, int l) { return emu_xchg(v, l); }
inline float emu_rcpf(float x) { return 1.0f / x; }
// DPP move: quad_perm (0x00-0xff), row_shr:n (0x111..0x11f), row_mirror (0x140),
// row_half_mirror (0x141), row_bcast:15 (0x142), row_bcast:31 (0x143);
// disabled rows and lanes without a source return `old`
inline int emu_update_dpp(int old, int src, int ctrl, int row_mask, int, bool) {
  const int l = threadIdx.x & 63, row = l >> 4;
  int s = -1;
  if (ctrl >= 0 && ctrl <= 0xff) s = (l & ~3) | ((ctrl >> (2 * (l & 3))) & 3);
  else if (ctrl > 0x110 && ctrl < 0x120) { int n = ctrl - 0x110; if ((l & 15) >= n) s = l - n; }
  else if (ctrl == 0x140) s = (l & ~15) | (15 - (l & 15));
  else if (ctrl == 0x141) s = (l & ~7) | (7 - (l & 7));
  else if (ctrl == 0x142) { if (row >= 1) s = row * 16 - 1; }
  else if (ctrl == 0x143) { if (row >= 2) s = 31; }
  int v = emu_xchg(src, s < 0 ? l : s);
  if (!((row_mask >> row) & 1) || s < 0) return old;
  return v;
}
#define __HIP_MEMORY_SCOPE_AGENT 0
#define __HIP_MEMORY_SCOPE_WORKGROUP 0
#define OCG_EMU 1
#define __hip_atomic_fetch_add(p, v, o, sc) __atomic_fetch_add((p), (v), __ATOMIC_SEQ_CST)
template <class T, class U>
inline void emu_atomic_store(T* p, U v) {
  T t = T(v);
  __atomic_store(p, &t, __ATOMIC_SEQ_CST);
}
#define __hip_atomic_store(p, v, o, sc) emu_atomic_store((p), (v))
#define __hip_atomic_load(p, o, sc) __atomic_load_n((p), __ATOMIC_SEQ_CST)
#define __builtin_amdgcn_s_sleep(x) ((void)0)
inline void __threadfence() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
#define __builtin_amdgcn_readlane(v, l) emu_readlane((v), (l))
#define __builtin_amdgcn_readfirstlane(v) (v)  // every use reads a wave-uniform value
#define __builtin_amdgcn_rcpf(x) emu_rcpf(x)
#define __builtin_amdgcn_update_dpp(o, s, c, r, b, bc) emu_update_dpp((o), (s), (c), (r), (b), (bc))
#define __builtin_amdgcn_fence(o, s) __atomic_thread_fence(__ATOMIC_SEQ_CST)
#define __builtin_amdgcn_wave_barrier() emu_wbar->arrive_and_wait()
inline int emu_bpermute(int addr, int v) { return emu_xchg(v, (addr >> 2) & 63); }
#define __builtin_amdgcn_ds_bpermute(a, v) emu_bpermute((a), (v))
// ds_permute: lane l pushes v to lane addr/4; a lane nobody writes reads 0
// (the last writer wins, as the hardware's highest lane)
inline int emu_permute(int addr, int v) {
  const unsigned w = threadIdx.x & ~63u;
  const int l = threadIdx.x & 63;
  emu_xbuf[threadIdx.x] = (uint64_t(uint32_t((addr >> 2) & 63)) << 32) | uint32_t(v);
  emu_wbar->arrive_and_wait();
  int r = 0;
  for (int i = 0; i < 64; ++i)
    if (int(emu_xbuf[w + i] >> 32) == l) r = int(uint32_t(emu_xbuf[w + i]));
  emu_wbar->arrive_and_wait();
  return r;
}
#define __builtin_amdgcn_ds_permute(a, v) emu_permute((a), (v))
inline int __ffsll(long long m) { return __builtin_ffsll(m); }
extern thread_local emu_dim3 gridDim;
inline double emu_rsq(double x) { return 1.0 / std::sqrt(x); }
#define __builtin_amdgcn_rsq(x) emu_rsq(x)
