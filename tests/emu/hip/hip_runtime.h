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
extern thread_local std::barrier<>* emu_bar;
extern thread_local uint64_t* emu_xbuf;  // 64-entry exchange buffer of the block
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
  emu_xbuf[threadIdx.x & 63] = b;
  emu_bar->arrive_and_wait();
  uint64_t r = emu_xbuf[src & 63];
  emu_bar->arrive_and_wait();
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
  emu_xbuf[threadIdx.x & 63] = pred ? 1 : 0;
  emu_bar->arrive_and_wait();
  unsigned long long m = 0;
  for (int i = 0; i < 64; ++i) m |= (emu_xbuf[i] ? 1ULL : 0ULL) << i;
  emu_bar->arrive_and_wait();
  return m;
}
inline int __popcll(unsigned long long m) { return __builtin_popcountll(m); }
