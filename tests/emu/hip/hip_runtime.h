// TEST INFRASTRUCTURE ONLY — host emulation shim used by tests/emu/emu.cpp to
// execute the unmodified device bodies (optimalcontrolmps_amd/csrc/
// kernels.hpp) on CPU threads for debugging.  Never part of the product
// build, never loaded by the product path.
#pragma once
#include <atomic>
#include <barrier>
#include <cmath>

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
inline void __syncthreads() { emu_bar->arrive_and_wait(); }
inline int atomicOr(int* p, int v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
inline double atomicAdd(double* p, double v) {
  std::atomic_ref<double> r(*p);
  return r.fetch_add(v);
}
