// Device-side helpers shared by the gfx950 kernels of libgmt.
// CDNA4 facts used here (see /opt/skills/guides/MI355X_MICROARCH.md):
//   * wave = 64 lanes; a 256-thread block = 4 waves = one wave per SIMD.
//   * the widest global access is 16 B/lane (global_load_dwordx4) -> fp64
//     kernels move 2 doubles per lane per instruction.
//   * workgroups are dealt round-robin over the 8 XCDs (b % 8 share one L2);
//     xcd_swizzle() below gives each XCD a contiguous range of tiles.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gmt {

typedef double d2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kNumXcd = 8;

__device__ __forceinline__ d2 ld2(const double* p) { return *reinterpret_cast<const d2*>(p); }
__device__ __forceinline__ void st2(double* p, d2 v) { *reinterpret_cast<d2*>(p) = v; }
__device__ __forceinline__ d2 ld2_nt(const double* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const d2*>(p));
}
__device__ __forceinline__ void st2_nt(double* p, d2 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<d2*>(p));
}

// Whole-wave lane shifts of a double through DPP (wave_shr:1 / wave_shl:1, a
// VALU source modifier: no LDS traffic).  bound_ctrl: the edge lane reads 0
// without an "old" operand, so no zero-initialising v_mov per shift.
__device__ __forceinline__ double dpp_from_lower(double v) {  // lane i <- lane i-1
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_from_upper(double v) {  // lane i <- lane i+1
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}

// Bijective XCD-aware remap of a linear block id: consecutive tiles (which
// share halo rows) land on the same XCD's L2.  Valid for any nblocks.
__device__ __forceinline__ int64_t xcd_swizzle(int64_t bid, int64_t nblocks) {
  const int64_t q = nblocks / kNumXcd, r = nblocks % kNumXcd;
  const int64_t xcd = bid % kNumXcd, k = bid / kNumXcd;
  // XCD `xcd` owns tiles [start, start+cnt) where the first r XCDs get q+1.
  const int64_t start = xcd * q + (xcd < r ? xcd : r);
  return start + k;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Sum over a 256-thread block; result valid in every thread.
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double s_part[kBlock / kWave];
  v = wave_sum(v);
  if ((threadIdx.x & (kWave - 1)) == 0) s_part[threadIdx.x / kWave] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < kBlock / kWave; ++i) t += s_part[i];
  __syncthreads();
  return t;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline unsigned grid_1d(int64_t nblocks) { return static_cast<unsigned>(nblocks); }

}  // namespace gmt

#define GMT_RET_LAUNCH()                                 \
  do {                                                   \
    hipError_t _e = hipGetLastError();                   \
    return static_cast<int>(_e);                         \
  } while (0)
