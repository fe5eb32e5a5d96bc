// stencil5_d1.hpp — the dim-1 (strided-axis) 5-tap derivative through the
// LDS-DMA pipeline (see stencil5.hip).  A header so csrc/bench/variant_bench.hip
// can time other chunk widths / segment lengths against the production shape.
#pragma once
#include <algorithm>
#include <utility>

#include "common.hpp"

namespace gmt {
namespace d1 {

constexpr int kP = 4;          // input rows in flight per wave
constexpr int kRS = kP + 1;    // ring: the row being read + P in flight
constexpr int kU = 5;          // unroll: window (5) and ring slots are static
static_assert(kU % 5 == 0 && kU % kRS == 0, "unroll");
constexpr uint32_t kDrop = 0x80000000u;  // buffer offset past num_records: no-op
constexpr int kNW = 4;                   // waves (adjacent strips) per workgroup

struct Args {
  int64_t nx, ny_out, ld_in, ld_out;
  int64_t nstrip, nseg;
  double c[5];  // coefficients * scale
  int seg;      // output rows per segment
  int nsteps;   // steps per segment (L + 4, padded to the unroll)
};

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const double* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), 0, bytes, 0x00020000);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// CPL 16-B chunks per lane per row: DMA j moves the strip's bytes
// [1024 j, 1024 j + 1024), lane l's piece at 16 l (columns 128 j + 2 l, +1)
template <int CPL, bool ODD>
__global__ __launch_bounds__(kNW * kWave) void stencil5_d1_dma(Args a, const double* __restrict__ in,
                                                               double* __restrict__ out, int64_t nblocks) {
  extern __shared__ d2 lds_dyn[];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  // strips fastest: the resident waves sweep a contiguous band of each row
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t ngroups = (a.nstrip + kNW - 1) / kNW;
  const int64_t seg = t / ngroups;
  const int64_t strip = (t % ngroups) * kNW + wave;
  if (strip >= a.nstrip) return;
  const int64_t ld_in = a.ld_in, ld_out = a.ld_out;
  const double c0 = a.c[0], c1 = a.c[1], c2 = a.c[2], c3 = a.c[3], c4 = a.c[4];
  const int64_t y0 = seg * a.seg;
  const int64_t L = std::min<int64_t>(a.seg, a.ny_out - y0);
  const int64_t x0 = strip * (128 * CPL);
  const uint32_t ldi8 = static_cast<uint32_t>(ld_in) * 8u, ldo8 = static_cast<uint32_t>(ld_out) * 8u;
  // loads: input rows [y0, y0 + L + 4), 16 B per lane and chunk
  const __amdgpu_buffer_rsrc_t lrs = rsrc(in + y0 * ld_in, static_cast<uint32_t>(L + 4) * ldi8);
  const uint32_t loff = static_cast<uint32_t>(x0 + 2 * lane) * 8u;
  //  stores: output rows [y0, y0 + L); a chunk's 16-B store where both
  //  columns exist, with ODD (nx odd) an 8-B store for the last column
  const __amdgpu_buffer_rsrc_t srs = rsrc(out + y0 * ld_out, static_cast<uint32_t>(L) * ldo8);
  uint32_t st16[CPL], st8[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int64_t c = x0 + 128 * j + 2 * lane;
    st16[j] = c + 1 < a.nx ? static_cast<uint32_t>(c) * 8u : kDrop;
    st8[j] = c + 1 == a.nx ? static_cast<uint32_t>(c) * 8u : kDrop;
  }
  d2(*ring)[CPL][kWave] = reinterpret_cast<d2(*)[CPL][kWave]>(lds_dyn + wave * kRS * CPL * kWave);
  // (the LDS operand is passed as char*: a d2* there makes clang drop this
  // template's host-side stub without a diagnostic)
  auto dma = [&](int s, int slot) {
#pragma unroll
    for (int j = 0; j < CPL; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, reinterpret_cast<char*>(&ring[slot][j][0]), 16,
                                               loff + 1024u * j + static_cast<uint32_t>(s) * ldi8, 0, 0, 0);
  };
  auto store = [&](int s, const d2 (&v)[CPL]) {  // output row s - 4 (out of range while s < 4)
    const uint32_t ro = static_cast<uint32_t>(s - 4) * ldo8;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v[j]), srs, st16[j] + ro, 0, 2 /* nt */);
      if constexpr (ODD) {
        const u2 lo = {static_cast<unsigned>(__double2loint(v[j].x)), static_cast<unsigned>(__double2hiint(v[j].x))};
        __builtin_amdgcn_raw_buffer_store_b64(lo, srs, st8[j] + ro, 0, 2);
      }
    }
  };
  constexpr int SPS = CPL * (ODD ? 2 : 1), DPS = CPL;
  d2 W[5][CPL];
#pragma unroll
  for (int r = 0; r < 5; ++r)
#pragma unroll
    for (int j = 0; j < CPL; ++j) W[r][j] = d2{0.0, 0.0};
  // prologue: rows 0..P-1 in flight, each after the (dropped) stores a step
  // issues, so every wait counts (SPS + DPS)(P - 1) younger operations
  // (each dummy store gets its own out-of-range row, so the compiler cannot
  // merge identical stores and break the count)
  static_for<0, kP>([&](auto I) {
    const d2 z[CPL] = {};
    store(decltype(I)::value - kP, z);
    dma(decltype(I)::value, decltype(I)::value);
  });
  for (int s0 = 0; s0 < a.nsteps; s0 += kU) {
    static_for<0, kU>([&](auto J) {
      constexpr int j = decltype(J)::value;
      const int s = s0 + j;
      wait_vmcnt<(SPS + DPS) * (kP - 1)>();  // row s (DMA'd P steps ago) has landed
#pragma unroll
      for (int k = 0; k < CPL; ++k) W[j % 5][k] = ring[j % kRS][k][lane];
      d2 o[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k)
        o[k] = c0 * W[(j + 1) % 5][k] + c1 * W[(j + 2) % 5][k] + c2 * W[(j + 3) % 5][k] +
               c3 * W[(j + 4) % 5][k] + c4 * W[j % 5][k];
      store(s, o);
      dma(s + kP, (j + kP) % kRS);  // the slot of row s - 1, read last step
    });
  }
  wait_vmcnt<0>();  // no DMA may land after the workgroup's LDS is released
}

// Register-window walk (the production dim-1 kernel since round 3): a
// workgroup = NW waves side by side, 128 columns each (one 16-B chunk per
// lane), so each input row is read as NW KiB contiguous per workgroup;
// column groups are fastest in blockIdx and not XCD-swizzled, so the
// resident workgroups walk down the same few rows of the whole width at
// once (a near-linear sweep of the array).  A ring of 5 + P rows in
// registers, P rows of plain 16-B nontemporal loads in flight.  Measured at
// the reference's dim-1 shape (524288 x 1028 -> 1024, csrc/bench/d1_walk.hip,
// profiles/r03_d1_walk.txt): 5.60-5.64 TB/s for NW = 16, P = 4, L = 128-512,
// against 5.46 TB/s for the DMA pipeline above on the same box.
// Requires an even nx and 16-B aligned rows (ld_in, ld_out even).
template <int NW, int P>
__global__ __launch_bounds__(NW * kWave) void stencil5_d1_win(int64_t nx, int64_t ny_out, int64_t ld_in,
                                                               int64_t ld_out, int64_t L, int64_t ngroups, Args c,
                                                               const double* __restrict__ in,
                                                               double* __restrict__ out) {
  constexpr int R = 5 + P;  // ring: rows o .. o+4 in use, o+5 .. o+4+P in flight
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t g = blockIdx.x % ngroups, seg = blockIdx.x / ngroups;
  const int64_t x = (g * NW + wave) * 128 + 2 * lane;
  const int64_t y0 = seg * L;
  const int64_t L1 = std::min<int64_t>(L, ny_out - y0);
  if ((g * NW + wave) * 128 >= nx || L1 <= 0) return;
  const bool valid = x < nx;  // nx even: x + 1 < nx too
  const int64_t xl = valid ? x : nx - 2;  // loads of an idle lane stay inside the row
  const d2* src = reinterpret_cast<const d2*>(in + y0 * ld_in + xl);
  d2* dst = reinterpret_cast<d2*>(out + y0 * ld_out + xl);
  const int64_t li = ld_in / 2, lo = ld_out / 2;
  const double c0 = c.c[0], c1 = c.c[1], c2 = c.c[2], c3 = c.c[3], c4 = c.c[4];
  const int64_t nin = L1 + 4;  // input rows of the segment
  d2 B[R];
  auto load = [&](int64_t r, int slot) {
    B[slot] = __builtin_nontemporal_load(src + (r < nin ? r : nin - 1) * li);  // past the end: unused
  };
  static_for<0, 4 + P>([&](auto I) { load(decltype(I)::value, decltype(I)::value); });
  for (int64_t o0 = 0; o0 < L1; o0 += R) {
    static_for<0, R>([&](auto J) {
      constexpr int j = decltype(J)::value;
      const int64_t o = o0 + j;
      load(o + 4 + P, (j + 4 + P) % R);
      if (o < L1 && valid)
        __builtin_nontemporal_store(c0 * B[j % R] + c1 * B[(j + 1) % R] + c2 * B[(j + 2) % R] +
                                        c3 * B[(j + 3) % R] + c4 * B[(j + 4) % R],
                                    dst + o * lo);
    });
  }
}

}  // namespace d1
}  // namespace gmt
