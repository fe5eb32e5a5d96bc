// K fused 5-point Jacobi sweeps per memory pass (temporal blocking), gfx950.
//
// One wave owns a 128-column strip (2 columns per lane) and walks down a
// segment of L output rows.  Time level p of row r needs level p-1 of rows
// r-1, r, r+1, which the wave computed in its three previous steps (skewed
// pipeline: at step s level p is computed for row s - 2p, so the K levels of
// a step are independent of each other):
//   step s:  level p = K..1 of row s-2p (level K is stored: 16-B buffer
//            store); issue the buffer->LDS DMA of input row s+P into the
//            ring slot that level 1 just released.
// West/east neighbours come from the adjacent lane through DPP (wave_shr /
// wave_shl); the strip edges lose one column per level, so a strip yields
// 128 - 2K output columns.  A workgroup is nw independent waves on adjacent
// strips (no barrier): their 2K overlap columns are re-read from the CU's L1.
//
// Memory pipeline: level-0 rows are DMA'd into a per-wave LDS ring of P+3
// slots (rows s-3..s-1 in use, P in flight) and read back by ds_read_b128
// when level 1 needs them: no loaded VGPR crosses the loop back edge, so
// the loop keeps P rows in flight (the round-1 register-prefetch kernel,
// jacobi5pipe.hip, copied its prefetched registers at the back edge and
// waited vmcnt(1) every 3 steps: 44% SQ_WAIT_ANY, profiles/r02_pmc/).
// One loop-invariant buffer descriptor per direction; the row is in the VGPR
// offset and the buffer range check drops every row outside the segment.
// Every step issues exactly one DMA and two stores — no branch around a
// memory instruction — so the explicit s_waitcnt vmcnt(3P+2) before the
// ring reads is exact.
//
// Arithmetic: scaled levels V_p = 4^p u_p, V_p = (W + E) + (N + S), output
// V_K * 4^-K: bitwise equal to K single sweeps u' = 0.25((W+E)+(N+S))
// unless a level value is subnormal or 4^K |u| overflows; EXACT keeps the
// 0.25 multiply per level (used by the engine when max|u| is too large).
// Dirichlet sides (halo_mask bit clear): ring cells keep their value at every
// level (RULE path, per-lane column masks + a per-row scalar test, chosen
// per wave); on halo sides the K-wide ghost ring is updated as data.
//
// Measured limits (csrc/bench/valu_rate.hip, profiles/r02_tb.md): a level
// (4 v_mov_b32_dpp + 6 v_add_f64 per 128 cells) issues at ~19.5 ns per SIMD
// at 2 waves/SIMD — DPP moves cost as much as a DADD — so the kernel is
// VALU-issue bound once K >= 12.  Sharing the strip edges between the waves
// of a workgroup through LDS (no recomputed overlap) was built and measured:
// the K exec-masked ds_write per step made it LDS-issue bound (2.0-2.4M vs
// 3.4-3.8M MLUPS), with or without the per-step barrier; removed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>

#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {
namespace tb {

constexpr int kMaxRect = 8;
constexpr int kMaxWaves = 8;
constexpr int kCols = 2 * kWave;  // columns per wave
constexpr uint32_t kDrop = 0x80000000u;  // buffer offset past num_records: no-op access

struct Args {
  int64_t r[kMaxRect][4];        // output rects: x0, nx, y0, ny (absolute; x0 even)
  int64_t nstrip[kMaxRect];      // workgroup strips per rect
  int64_t tstart[kMaxRect + 1];  // prefix sum of workgroups
  int64_t dom[4];                // interior x0, nx, y0, ny
  int64_t ld;                    // row pitch (elements, even)
  int64_t last_row;              // last allocated row (load clamp)
  int n;                         // rects
  int mask;                      // halo sides: bit0..3 = W/E/S/N
  int nw;                        // waves per workgroup
  int seg;                       // output rows per workgroup segment
  int nsteps;                    // steps per segment, padded to the unroll
  double quarter;                // 0.25 (EXACT): an SGPR operand
};

constexpr int lcm3(int n) { return n % 3 == 0 ? n : 3 * n; }

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const double* p, uint32_t bytes) {
  // 0x00020000: raw-buffer descriptor word 3 for gfx9 (32-bit data format)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), 0, bytes, 0x00020000);
}

// Per-wave LDS (dynamic, sized by the launch): the level-0 row ring,
// ring[w][slot][lane], filled by buffer->LDS DMA.
__host__ __device__ constexpr int64_t lds_bytes(int nw, int P) {
  return static_cast<int64_t>(nw) * (P + 3) * kWave * 16;
}

// s_waitcnt vmcnt(n) only (expcnt / lgkmcnt left at their maxima), as a
// compiler barrier for memory: the LDS-DMA'd rows are read by ds_read after
// it, and the compiler does not track LDS-DMA -> ds_read dependencies
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One wave: a 128-column strip (output columns [xs, xe)) and the output rows
// [ys, ye).  Skewed pipeline: at step s level p is computed for row
// yl + s - 2p (yl = ys - K), from level p-1 of the three previous steps.
template <int K, int P, bool EXACT, bool ODD, bool RULE>
__device__ __forceinline__ void run_strip(const Args& a, const double* __restrict__ u, double* __restrict__ un,
                                          d2 (*ring)[kWave], int lane, int64_t xs, int64_t xe, int64_t ys,
                                          int64_t ye) {
  constexpr int RS = P + 3;    // level-0 ring: rows s-3..s-1 in use, s..s+P-1 in flight
  constexpr int U = lcm3(RS);  // unroll: ring slots are static offsets
  // every kernel argument the loop needs, as values: the asm memory clobbers
  // below would otherwise force a reload of the kernarg segment per use
  const int64_t ld = a.ld;
  const int mask = a.mask;
  const double quarter = a.quarter;
  const int64_t dx0 = a.dom[0], dx1 = a.dom[0] + a.dom[1];
  const int64_t dy0 = a.dom[2], dy1 = a.dom[2] + a.dom[3];
  const int64_t c0 = xs - K + 2 * lane;  // this lane: columns c0, c0+1
  const int64_t yl = ys - K;             // row of step 0
  const int L = static_cast<int>(ye - ys);
  const uint32_t ld8 = static_cast<uint32_t>(ld) * 8u;

  // One loop-invariant descriptor per direction; the row lives in the VGPR
  // offset, so the buffer range check drops (stores) or zero-fills (loads)
  // every row outside the segment — no per-step scalar address math.
  //  loads: rows [yl, min(yl + L + 2K, last_row + 1)); lane column c0 (a
  //  column past the row end reads the next row: garbage outside every cone)
  const int64_t nrow_in = std::min<int64_t>(L + 2 * K, a.last_row + 1 - yl);
  const __amdgpu_buffer_rsrc_t lrs = row_rsrc(u + yl * ld, static_cast<uint32_t>(nrow_in) * ld8);
  const uint32_t loff = static_cast<uint32_t>(c0) * 8u;
  //  stores: rows [ys, ye) from column xs; a 16-B store for lanes with both
  //  columns in [xs, xe), with ODD (a rect of the launch ends at an odd
  //  column) also an 8-B store for the single lane at that edge; every other
  //  lane is offset by 2^31 (out of range for any row).  The 8-B store is not
  //  issued without ODD: dropped by every lane it still costs a TA slot, and
  //  the memory-bound passes (K <= 8) are VMEM-issue bound (93% of wave
  //  cycles in SQ_WAIT_INST_ANY, profiles/r02_pmc/).
  const __amdgpu_buffer_rsrc_t srs = row_rsrc(un + ys * ld + xs, static_cast<uint32_t>(L) * ld8);
  const bool in0 = c0 >= xs && c0 < xe, in1 = c0 + 1 >= xs && c0 + 1 < xe;
  const uint32_t st16 = (in0 && in1) ? static_cast<uint32_t>(c0 - xs) * 8u : kDrop;
  const uint32_t st8 = (in0 && !in1) ? static_cast<uint32_t>(c0 - xs) * 8u : kDrop;
  auto store_step = [&](int s, d2 v) {  // level K of step s = output row ys + s - 3K
    const uint32_t ro = static_cast<uint32_t>(s - 3 * K) * ld8;  // wraps for warm-up rows: out of range
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), srs, st16 + ro, 0, 2 /* nt */);
    if constexpr (ODD) {
      const u2 lo = {static_cast<unsigned>(__double2loint(v.x)), static_cast<unsigned>(__double2hiint(v.x))};
      __builtin_amdgcn_raw_buffer_store_b64(lo, srs, st8 + ro, 0, 2);
    }
  };
  constexpr int SPS = ODD ? 2 : 1;  // stores per step
  auto dma = [&](int s, int slot) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, &ring[slot][0], 16, loff + static_cast<uint32_t>(s) * ld8, 0, 0,
                                             0);
  };

  // Dirichlet rule (RULE only): a cell outside the interior on a side whose
  // ghost ring is fixed keeps its value at every level
  const bool gw = mask & 1, ge = mask & 2, gs = mask & 4, gn = mask & 8;
  const bool kx0 = (c0 < dx0 && !gw) || (c0 >= dx1 && !ge);
  const bool kx1 = (c0 + 1 < dx0 && !gw) || (c0 + 1 >= dx1 && !ge);

  auto level = [&](const d2& up_, const d2& c, const d2& dn, int64_t row) -> d2 {
#pragma clang fp contract(off)
    const double w = dpp_from_lower(c.y), e = dpp_from_upper(c.x);
    d2 v;
    if constexpr (EXACT) {
      v.x = quarter * ((w + c.y) + (up_.x + dn.x));
      v.y = quarter * ((c.x + e) + (up_.y + dn.y));
    } else {
      v.x = (w + c.y) + (up_.x + dn.x);
      v.y = (c.x + e) + (up_.y + dn.y);
    }
    if constexpr (RULE) {
      const bool rk = (row < dy0 && !gs) || (row >= dy1 && !gn);
      const double f = EXACT ? 1.0 : 4.0;  // a kept cell: V_p = 4 V_{p-1}
      v.x = (rk || kx0) ? c.x * f : v.x;
      v.y = (rk || kx1) ? c.y * f : v.y;
    }
    return v;
  };

  d2 W[K][3];  // W[p][slot], p = 1..K-1 (level 0 is the LDS ring)
#pragma unroll
  for (int p = 0; p < K; ++p)
#pragma unroll
    for (int j = 0; j < 3; ++j) W[p][j] = d2{0.0, 0.0};

  // prologue: rows 0..P-1 in flight, each preceded by the (dropped) stores
  // a steady-state step issues, so every wait below counts the same
  // (SPS + 1) P + SPS younger memory operations (SPS stores + 1 DMA per step)
  static_for<0, P>([&](auto I) {
    store_step(0, d2{0.0, 0.0});  // row ys - 3K: out of range
    dma(decltype(I)::value, decltype(I)::value);
  });

  auto step = [&](auto J, int s) {
    constexpr int j = decltype(J)::value;
    constexpr int cur = j % 3, s1 = (j + 2) % 3, s2 = (j + 1) % 3;  // slots of steps s (== s-3), s-1, s-2
    d2 r0, r1, r2;  // level-0 rows s-3, s-2, s-1
    static_for<0, K>([&](auto Q) {
      constexpr int p = K - decltype(Q)::value;  // K .. 1, top-down
      if constexpr (p == 3 || (K < 3 && p == K)) {
        // the DMA of row s-1 (issued at step s-1-P) has landed once at most
        // (SPS + 1) P + SPS younger memory operations are outstanding
        if constexpr (p == K) {
          wait_vmcnt<(SPS + 1) * P>();  // this step's stores are not issued yet
        } else {
          wait_vmcnt<(SPS + 1) * P + SPS>();
        }
        r0 = ring[(j + U - 3) % RS][lane];
        r1 = ring[(j + U - 2) % RS][lane];
        r2 = ring[(j + U - 1) % RS][lane];
      }
      const int64_t row = yl + s - 2 * p;
      d2 v;
      if constexpr (p == 1)
        v = level(r0, r1, r2, row);
      else
        v = level(W[p - 1][cur], W[p - 1][s2], W[p - 1][s1], row);
      if constexpr (p == K) {
        if constexpr (!EXACT) {
          v.x = __builtin_amdgcn_ldexp(v.x, -2 * K);  // exact power-of-two unscale
          v.y = __builtin_amdgcn_ldexp(v.y, -2 * K);
        }
        store_step(s, v);  // issued every step (warm-up rows are out of range)
      } else {
        W[p][cur] = v;
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    // the ring slot of row s-3 is free (its ds_reads completed before level 1
    // used them): prefetch row s+P into it
    dma(s + P, (j + P) % RS);
  };

  // One loop for the whole segment: splitting off the pipeline's warm-up
  // and drain steps (to skip the levels nobody reads there) made the
  // register allocator spill from K = 12 on (three loops carrying W).
  for (int s0 = 0; s0 < a.nsteps; s0 += U) static_for<0, U>([&](auto J) { step(J, s0 + decltype(J)::value); });
  // no LDS-DMA may land after the workgroup's LDS is released
  wait_vmcnt<0>();
}

// A workgroup = nw waves on nw adjacent 128-column strips of one segment
// (adjacent strips share their 2K overlap columns in the CU's L1 / the XCD's
// L2); every wave is independent (no barrier).
template <int K, int P, bool EXACT, bool ODD>
__global__ __launch_bounds__(kMaxWaves * kWave) __attribute__((amdgpu_waves_per_eu(2)))
void jacobi5tb_kernel(Args a, const double* __restrict__ u, double* __restrict__ un, int64_t nblocks) {
  extern __shared__ d2 lds_dyn[];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  int k = 0;
  while (k + 1 < a.n && t >= a.tstart[k + 1]) ++k;
  const int64_t lt = t - a.tstart[k];
  const int64_t ngroups = (a.nstrip[k] + a.nw - 1) / a.nw;
  const int64_t nseg = (a.r[k][3] + a.seg - 1) / a.seg;
  // dispatch order of the segment rows: the first and the last (the only
  // ones that can hold Dirichlet-rule waves at the top / bottom, ~40% more
  // VALU per step) go first, so the launch's tail is made of fast waves
  const int64_t lseg = lt / ngroups;
  const int64_t seg = nseg < 2 || lseg == 0 ? lseg : (lseg == 1 ? nseg - 1 : lseg - 1);
  const int64_t strip = (lt % ngroups) * a.nw + wave;
  if (strip >= a.nstrip[k]) return;  // whole wave: no barrier anywhere
  constexpr int64_t wout = kCols - 2 * K;
  const int64_t rx0 = a.r[k][0], rx1 = a.r[k][0] + a.r[k][1];
  const int64_t ry1 = a.r[k][2] + a.r[k][3];
  int64_t xs = rx0 + strip * wout;
  if (xs + wout > rx1) {  // last strip: shifted left to reach rx1 (even start, rounded up)
    xs = (rx1 - wout + 1) & ~int64_t(1);
    if (xs < rx0) xs = rx0;
  }
  const int64_t xe = xs + wout < rx1 ? xs + wout : rx1;
  const int64_t ys = a.r[k][2] + seg * a.seg;
  const int64_t ye = ys + a.seg < ry1 ? ys + a.seg : ry1;
  // the rule path only where a computed cell can be a fixed ring cell
  const int64_t cx0 = xs - K, cx1 = xs - K + kCols;
  const bool rule = (cx0 < a.dom[0] && !(a.mask & 1)) || (cx1 > a.dom[0] + a.dom[1] && !(a.mask & 2)) ||
                    (ys - K < a.dom[2] && !(a.mask & 4)) || (ye + K > a.dom[2] + a.dom[3] && !(a.mask & 8));
  d2(*ring)[kWave] = reinterpret_cast<d2(*)[kWave]>(lds_dyn + wave * (P + 3) * kWave);
  if (rule)
    run_strip<K, P, EXACT, ODD, true>(a, u, un, ring, lane, xs, xe, ys, ye);
  else
    run_strip<K, P, EXACT, ODD, false>(a, u, un, ring, lane, xs, xe, ys, ye);
}

}  // namespace tb
}  // namespace gmt

namespace {

using namespace gmt;
using namespace gmt::tb;

// Output rows per wave.  Short segments measured fastest on 32768^2 even
// though every segment pays the 3K-step pipeline warm-up (192-384 rows beat
// 512-1024 by 5-20%, also with the boundary segment rows dispatched first;
// gmt_kernel_bench --only=tb, profiles/r02_tb.md): K <= 12 -> 192,
// K = 14 -> 256, K = 16 -> 384.  Small domains get shorter segments so the
// launch still has ~4 waves per resident slot (8192^2: 96 rows).
int64_t default_seg_rows(int K, int64_t rows_x_strips) {
  const int64_t pref = K <= 12 ? 192 : (K <= 14 ? 256 : 384);
  constexpr int64_t kTargetWaves = 4 * 2048;  // 4 x (2 waves/SIMD x 1024 SIMDs)
  return std::max<int64_t>(64, std::min(pref, rows_x_strips / kTargetWaves));
}

template <int K, int P, bool EXACT, bool ODD>
int launch_tb(const gmt_tb_opts& o, int n_rect, const int64_t* rects, const int64_t* dom, int mask, const double* u,
              double* un, int64_t ld, int64_t nrows, hipStream_t s) {
  constexpr int U = lcm3(P + 3);
  Args a{};
  a.nw = o.wg_waves > 0 ? o.wg_waves : 4;
  a.ld = ld;
  a.last_row = nrows - 1;
  a.mask = mask;
  a.quarter = 0.25;
  for (int j = 0; j < 4; ++j) a.dom[j] = dom[j];
  constexpr int64_t wout = kCols - 2 * K;
  int64_t maxh = 0;
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    for (int j = 0; j < 4; ++j) a.r[a.n][j] = r[j];
    a.nstrip[a.n] = (r[1] + wout - 1) / wout;
    maxh = std::max(maxh, r[3]);
    ++a.n;
  }
  if (a.n == 0) return 0;
  // all strips of a rect narrower than nw strips: fewer waves per workgroup
  int64_t maxs = 0;
  for (int k = 0; k < a.n; ++k) maxs = std::max(maxs, a.nstrip[k]);
  if (a.nw > maxs) a.nw = static_cast<int>(maxs);
  // the kernel addresses a segment's rows through 32-bit buffer offsets:
  // (L + 3K + unroll + prefetch) rows of ld doubles must stay below 2^31
  const int64_t lmax = std::min<int64_t>(1 << 20, (int64_t(1) << 31) / (ld * 8) - 3 * K - 2 * U - P);
  if (lmax < 1) return static_cast<int>(hipErrorInvalidValue);
  int64_t rows_x_strips = 0;
  for (int k = 0; k < a.n; ++k) rows_x_strips += a.r[k][3] * a.nstrip[k];
  const int64_t L =
      std::min(std::min<int64_t>(o.seg_rows > 0 ? o.seg_rows : default_seg_rows(K, rows_x_strips), maxh), lmax);
  a.seg = static_cast<int>(L);
  a.nsteps = static_cast<int>((L + 3 * K + U - 1) / U * U);
  a.tstart[0] = 0;
  for (int k = 0; k < a.n; ++k) {
    const int64_t groups = (a.nstrip[k] + a.nw - 1) / a.nw;
    a.tstart[k + 1] = a.tstart[k] + groups * ((a.r[k][3] + L - 1) / L);
  }
  for (int k = a.n + 1; k <= kMaxRect; ++k) a.tstart[k] = a.tstart[a.n];
  const int64_t nb = a.tstart[a.n];
  const size_t smem = static_cast<size_t>(lds_bytes(a.nw, P));
  jacobi5tb_kernel<K, P, EXACT, ODD><<<grid_1d(nb), a.nw * kWave, smem, s>>>(a, u, un, nb);
  return static_cast<int>(hipGetLastError());
}

template <int K, int P>
int dispatch_k(const gmt_tb_opts& o, bool exact, int n_rect, const int64_t* rects, const int64_t* dom, int mask,
               const double* u, double* un, int64_t ld, int64_t nrows, hipStream_t s) {
  bool odd = false;  // some rect ends at an odd column: one lane stores a single column
  for (int k = 0; k < n_rect; ++k)
    if (rects[4 * k + 1] > 0 && rects[4 * k + 3] > 0 && ((rects[4 * k] + rects[4 * k + 1]) & 1)) odd = true;
  if (odd)
    return exact ? launch_tb<K, P, true, true>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s)
                 : launch_tb<K, P, false, true>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s);
  return exact ? launch_tb<K, P, true, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s)
               : launch_tb<K, P, false, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s);
}

}  // namespace

extern "C" int gmt_jacobi5tb(const gmt_tb_opts* opts, int n_rect, const int64_t* rects, const int64_t* dom,
                             int halo_mask, const double* u, double* un, int64_t ld, int64_t nrows, void* stream) {
  gmt_tb_opts o{};
  if (opts) o = *opts;
  const int K = o.sweeps;
  if (K < 2 || K > GMT_TB_MAX_SWEEPS || (K % 2) != 0) return static_cast<int>(hipErrorInvalidValue);
  if (n_rect < 0 || n_rect > kMaxRect) return static_cast<int>(hipErrorInvalidValue);
  if (o.wg_waves < 0 || o.wg_waves > kMaxWaves || o.seg_rows < 0) return static_cast<int>(hipErrorInvalidValue);
  if (!aligned16(u) || !aligned16(un) || (ld % 2) != 0 || ld <= 0) return static_cast<int>(hipErrorInvalidValue);
  if (static_cast<uint64_t>(ld) * 8u > 0xffffffffull) return static_cast<int>(hipErrorInvalidValue);
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    // 16-B loads: even start; the K-wide ring left of / above the rect exists
    if ((r[0] % 2) != 0 || r[0] < K || r[2] < K || r[0] + r[1] > ld || r[2] + r[3] + K > nrows)
      return static_cast<int>(hipErrorInvalidValue);
  }
  const bool exact = o.exact != 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (K) {
#define GMT_TB_CASE(KK)                                                                                   \
  case KK:                                                                                                \
    return dispatch_k<KK, 3>(o, exact, n_rect, rects, dom, halo_mask, u, un, ld, nrows, s);
    GMT_TB_CASE(2)
    GMT_TB_CASE(4)
    GMT_TB_CASE(6)
    GMT_TB_CASE(8)
    GMT_TB_CASE(10)
    GMT_TB_CASE(12)
    GMT_TB_CASE(14)
    GMT_TB_CASE(16)
#undef GMT_TB_CASE
    default:
      return static_cast<int>(hipErrorInvalidValue);
  }
}
