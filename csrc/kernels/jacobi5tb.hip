// K fused 5-point Jacobi sweeps per memory pass (temporal blocking), gfx950:
// workgroup-cooperative register pipeline.
//
// Layout of the work: a workgroup of NW waves (NW = 1..8) owns NW adjacent
// 128-column strips (2 columns per lane) and walks down a segment of L
// output rows.  Time level p of row r needs level p-1 of rows r-1, r, r+1,
// which the wave computed in its three previous steps (skewed pipeline: at
// step s level p is computed for row s - 2p, so the K levels of a step are
// independent of each other):
//   step s:  read the W/E edge values of the adjacent waves' level-(p-1)
//            centres from LDS (written at step s-2: two steps of slack);
//            level p = K..1 of row s-2p; level K is stored (16-B buffer
//            store); issue the load of input row s+P into the L0 ring slot
//            that level 1 just released; write this wave's own edge values
//            (lanes 0 and 63) to LDS; one s_barrier.
// West/east neighbours inside a wave come through DPP (wave_shr / wave_shl);
// across the waves of a workgroup they come from LDS as the DPP "old"
// operand of the edge lane, so only the two outer edges of the workgroup
// lose one column per level: a workgroup yields NW*128 - 2K output columns
// (the previous per-wave kernel, jacobi5pipe.hip, lost 2K of every 128).
//
// Memory pipeline: the level-0 rows live in a ring of P+3 slots that is also
// the prefetch queue (row s+P is loaded into the slot of row s-3), and the
// step loop is unrolled by lcm(3, P+3) so every slot index is static.  The
// loaded registers are never copied, so the loop's s_waitcnt vmcnt keeps P
// rows in flight across the back edge (rocprofv3 of jacobi5pipe.hip: its
// back-edge copies waited vmcnt(1) every 3 steps, 44% SQ_WAIT_ANY,
// profiles/r02_pmc/).  Every step issues exactly one load and two stores
// (out-of-range rows/columns are dropped by the buffer unit's range check):
// no branch around a memory instruction anywhere in the loop.
//
// Arithmetic: scaled levels V_p = 4^p u_p, V_p = (W + E) + (N + S), output
// V_K * 4^-K: bitwise equal to K single sweeps u' = 0.25((W+E)+(N+S))
// unless a level value is subnormal or 4^K |u| overflows; EXACT keeps the
// 0.25 multiply per level (used by the engine when max|u| is too large).
// Dirichlet sides (halo_mask bit clear): ring cells keep their value at every
// level (RULE path, per-lane column masks + a per-row scalar test, chosen
// per workgroup); on halo sides the K-wide ghost ring is updated as data.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
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

// lane i <- lane i-1 (lane 0 keeps `old`), lane i <- lane i+1 (lane 63 keeps `old`)
__device__ __forceinline__ double shr_old(double v, double old) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x138, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double shl_old(double v, double old) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x130, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}


// Per-workgroup LDS (dynamic, sized by the launch): the level-0 row ring of
// every wave, ring[w][slot][lane] (filled by buffer->LDS DMA), then the level
// 1..K-1 edge exchange, e[b][w][q][side] = the 2-column pair of lane 0
// (side 0) or lane 63 (side 1) of wave w's level-q value of a step s with
// s % 3 == b.
__host__ __device__ constexpr int64_t lds_bytes(int nw, int K, int P, bool share) {
  return (static_cast<int64_t>(nw) * (P + 3) * kWave + (share ? 3 * nw * K * 2 : 0)) * 16;
}

// s_waitcnt vmcnt(n) only (expcnt / lgkmcnt left at their maxima), as a
// compiler barrier for memory: the LDS-DMA'd rows are read by ds_read after
// it, and the compiler does not track LDS-DMA -> ds_read dependencies
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int K, int P, bool SHARE, bool EXACT, bool RULE>
__device__ __forceinline__ void run_strip(const Args& a, const double* __restrict__ u, double* __restrict__ un,
                                          d2* lds, int lane, int wave, int64_t xs, int64_t xe, int64_t ys,
                                          int64_t ye) {
  constexpr int RS = P + 3;    // level-0 ring: rows s-3..s-1 in use, s..s+P-1 in flight
  constexpr int U = lcm3(RS);  // unroll: ring slots and LDS edge buffers are static offsets
  constexpr int LAG = 2 * K;   // output row = level-0 row - 2K
  // every kernel argument the loop needs, as values: the asm memory clobbers
  // below would otherwise force a reload of the kernarg segment per use
  const int64_t ld = a.ld;
  const int nw = a.nw, nsteps = a.nsteps, mask = a.mask;
  const double quarter = a.quarter;
  const int64_t dx0 = a.dom[0], dx1 = a.dom[0] + a.dom[1];
  const int64_t dy0 = a.dom[2], dy1 = a.dom[2] + a.dom[3];
  const int64_t c0 = xs - K + static_cast<int64_t>(wave) * kCols + 2 * lane;  // this lane: c0, c0+1
  const int64_t yl = ys - K;  // row of step 0
  const uint32_t ld8 = static_cast<uint32_t>(ld) * 8u;

  // One loop-invariant descriptor per direction; the row lives in the VGPR
  // offset, so the buffer range check drops (stores) or zero-fills (loads)
  // every row outside the segment — no per-step scalar address math.
  //  loads: rows [yl, min(yl + L + 2K, last_row + 1)); lane column c0 (a
  //  column past the row end reads the next row: garbage outside every cone)
  const int64_t nrow_in = std::min<int64_t>((ye - ys) + 2 * K, a.last_row + 1 - yl);
  const __amdgpu_buffer_rsrc_t lrs = row_rsrc(u + yl * ld, static_cast<uint32_t>(nrow_in) * ld8);
  const uint32_t loff = static_cast<uint32_t>(c0) * 8u;
  //  stores: rows [ys, ye) from column xs; a 16-B store for lanes with both
  //  columns in [xs, xe), an 8-B store for the single lane at an odd right
  //  edge, every other lane offset by 2^31 (out of range for any row)
  const __amdgpu_buffer_rsrc_t srs = row_rsrc(un + ys * ld + xs, static_cast<uint32_t>(ye - ys) * ld8);
  const bool in0 = c0 >= xs && c0 < xe, in1 = c0 + 1 >= xs && c0 + 1 < xe;
  const uint32_t st16 = (in0 && in1) ? static_cast<uint32_t>(c0 - xs) * 8u : kDrop;
  const uint32_t st8 = (in0 && !in1) ? static_cast<uint32_t>(c0 - xs) * 8u : kDrop;
  auto store_step = [&](int s, d2 v) {  // level K of step s = output row ys + s - 3K
    const uint32_t ro = static_cast<uint32_t>(s - 3 * K) * ld8;  // wraps for warm-up rows: out of range
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), srs, st16 + ro, 0, 2 /* nt */);
    const u2 lo = {static_cast<unsigned>(__double2loint(v.x)), static_cast<unsigned>(__double2hiint(v.x))};
    __builtin_amdgcn_raw_buffer_store_b64(lo, srs, st8 + ro, 0, 2);
  };
  (void)LAG;

  // LDS: this wave's ring, ring[slot][lane], and the edge buffers
  auto ring_of = [&](int w) { return reinterpret_cast<d2(*)[kWave]>(lds + w * RS * kWave); };
  d2(*ring)[kWave] = ring_of(wave);
  d2* edges = lds + nw * RS * kWave;  // e[b][w][q][side] at ((b * nw + w) * K + q) * 2 + side
  auto dma = [&](int s, int slot) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, &ring[slot][0], 16, loff + static_cast<uint32_t>(s) * ld8, 0, 0,
                                             0);
  };

  // Dirichlet rule (RULE only): a cell outside the interior on a side whose
  // ghost ring is fixed keeps its value at every level
  const bool gw = mask & 1, ge = mask & 2, gs = mask & 4, gn = mask & 8;
  const bool kx0 = (c0 < dx0 && !gw) || (c0 >= dx1 && !ge);
  const bool kx1 = (c0 + 1 < dx0 && !gw) || (c0 + 1 >= dx1 && !ge);

  // neighbour waves (the workgroup's outer edges read their own data: those
  // columns are lost anyway)
  const int wl = wave > 0 ? wave - 1 : wave, wr = wave + 1 < nw ? wave + 1 : wave;

  auto level = [&](const d2& up_, const d2& c, const d2& dn, double eW, double eE, int64_t row) -> d2 {
#pragma clang fp contract(off)
    double w, e;
    if constexpr (SHARE) {
      w = shr_old(c.y, eW);
      e = shl_old(c.x, eE);
    } else {
      w = dpp_from_lower(c.y);
      e = dpp_from_upper(c.x);
    }
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

  // prologue: rows 0..P-1 in flight, each preceded by the two (dropped)
  // stores a steady-state step issues, so every wait below counts the same
  // 3P + 2 younger memory operations (2 stores + 1 DMA per step)
  static_for<0, P>([&](auto I) {
    store_step(0, d2{0.0, 0.0});  // row ys - 3K: out of range
    dma(decltype(I)::value, decltype(I)::value);
  });

  double Ew[K + 1], Ee[K + 1];
  auto read_edges = [&](int j, int p) {  // level p's centre = level p-1 of step s-2 (phase j)
    if (p == 1) {
      const int sl = (j + U - 2) % RS;
      Ew[1] = reinterpret_cast<const double*>(&ring_of(wl)[sl][kWave - 1])[1];
      Ee[1] = reinterpret_cast<const double*>(&ring_of(wr)[sl][0])[0];
    } else {
      const int b = (j + 1) % 3;  // LDS edge buffer written at step s-2
      Ew[p] = reinterpret_cast<const double*>(&edges[((b * nw + wl) * K + p - 1) * 2 + 1])[1];
      Ee[p] = reinterpret_cast<const double*>(&edges[((b * nw + wr) * K + p - 1) * 2 + 0])[0];
    }
  };

  auto step = [&](auto J, int s) {
    constexpr int j = decltype(J)::value;
    constexpr int cur = j % 3, s1 = (j + 2) % 3, s2 = (j + 1) % 3;  // slots of steps s (== s-3), s-1, s-2
    if constexpr (SHARE) {
      read_edges(j, K);
      if constexpr (K > 1) read_edges(j, K - 1);
    }
    d2 r0, r1, r2;  // level-0 rows s-3, s-2, s-1
    static_for<0, K>([&](auto Q) {
      constexpr int p = K - decltype(Q)::value;  // K .. 1, top-down
      if constexpr (SHARE && p - 2 >= 1) read_edges(j, p - 2);
      if constexpr (p == 3 || (K < 3 && p == K)) {
        // the DMA of row s-1 (issued at step s-1-P) has landed once at most
        // 3P+2 younger memory operations are outstanding
        if constexpr (p == K) {
          wait_vmcnt<3 * P>();  // this step's stores are not issued yet
        } else {
          wait_vmcnt<3 * P + 2>();
        }
        r0 = ring[(j + U - 3) % RS][lane];
        r1 = ring[(j + U - 2) % RS][lane];
        r2 = ring[(j + U - 1) % RS][lane];
      }
      const double eW = SHARE ? Ew[p] : 0.0, eE = SHARE ? Ee[p] : 0.0;
      const int64_t row = yl + s - 2 * p;
      d2 v;
      if constexpr (p == 1)
        v = level(r0, r1, r2, eW, eE, row);
      else
        v = level(W[p - 1][cur], W[p - 1][s2], W[p - 1][s1], eW, eE, row);
      if constexpr (p == K) {
        if constexpr (!EXACT) {
          v.x = __builtin_amdgcn_ldexp(v.x, -2 * K);  // exact power-of-two unscale
          v.y = __builtin_amdgcn_ldexp(v.y, -2 * K);
        }
        store_step(s, v);
      } else {
        W[p][cur] = v;
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    // the ring slot of row s-3 is free (its ds_reads completed before level 1
    // used them): prefetch row s+P into it
    dma(s + P, (j + P) % RS);
    if constexpr (SHARE) {
      constexpr int wb = j % 3;
      if (lane == 0 || lane == kWave - 1) {
        d2* e = &edges[(wb * nw + wave) * K * 2 + (lane == 0 ? 0 : 1)];
        static_for<1, K>([&](auto Q) { e[2 * decltype(Q)::value] = W[decltype(Q)::value][cur]; });
      }
      // LDS writes done, then the workgroup barrier (no vmcnt wait: the
      // prefetched rows stay in flight across it)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };

  for (int s0 = 0; s0 < nsteps; s0 += U) {
    static_for<0, U>([&](auto J) { step(J, s0 + decltype(J)::value); });
  }
  // no LDS-DMA may land after the workgroup's LDS is released
  wait_vmcnt<0>();
}

template <int K, int P, bool SHARE, bool EXACT>
__global__ __launch_bounds__(kMaxWaves * kWave) __attribute__((amdgpu_waves_per_eu(2)))
void jacobi5tb_kernel(Args a, const double* __restrict__ u, double* __restrict__ un, int64_t nblocks) {
  extern __shared__ d2 lds_dyn[];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  int k = 0;
  while (k + 1 < a.n && t >= a.tstart[k + 1]) ++k;
  const int64_t lt = t - a.tstart[k];
  const int64_t strip = lt % a.nstrip[k], seg = lt / a.nstrip[k];
  const int64_t wout = static_cast<int64_t>(a.nw) * kCols - 2 * K;
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
  const int64_t cx0 = xs - K, cx1 = xs - K + static_cast<int64_t>(a.nw) * kCols;
  const bool rule = (cx0 < a.dom[0] && !(a.mask & 1)) || (cx1 > a.dom[0] + a.dom[1] && !(a.mask & 2)) ||
                    (ys - K < a.dom[2] && !(a.mask & 4)) || (ye + K > a.dom[2] + a.dom[3] && !(a.mask & 8));
  if (rule)
    run_strip<K, P, SHARE, EXACT, true>(a, u, un, lds_dyn, lane, wave, xs, xe, ys, ye);
  else
    run_strip<K, P, SHARE, EXACT, false>(a, u, un, lds_dyn, lane, wave, xs, xe, ys, ye);
}

}  // namespace tb
}  // namespace gmt

namespace {

using namespace gmt;
using namespace gmt::tb;

// workgroups that fit on the device at once for a kernel / block size (cached)
int resident_workgroups(const void* fn, int block, size_t smem) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find({fn, block});
  if (it != cache.end()) return it->second;
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, smem) != hipSuccess || per_cu < 1) per_cu = 1;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  return cache[{fn, block}] = per_cu * cus;
}

template <int K, int P, bool SHARE, bool EXACT>
int launch_tb(const gmt_tb_opts& o, int n_rect, const int64_t* rects, const int64_t* dom, int mask, const double* u,
              double* un, int64_t ld, int64_t nrows, hipStream_t s) {
  constexpr int U = lcm3(P + 3);
  Args a{};
  a.nw = SHARE ? (o.wg_waves > 0 ? o.wg_waves : 4) : 1;
  a.ld = ld;
  a.last_row = nrows - 1;
  a.mask = mask;
  a.quarter = 0.25;
  for (int j = 0; j < 4; ++j) a.dom[j] = dom[j];
  const int64_t wout = static_cast<int64_t>(a.nw) * kCols - 2 * K;
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
  auto fn = reinterpret_cast<const void*>(&jacobi5tb_kernel<K, P, SHARE, EXACT>);
  const int block = a.nw * kWave;
  const size_t smem = static_cast<size_t>(lds_bytes(a.nw, K, P, SHARE));
  // segment rows: (L + 3K) a multiple of the unroll; minimise the rounds of
  // resident workgroups times the per-workgroup pipeline length
  auto tiles = [&](int64_t L) {
    int64_t t = 0;
    for (int k = 0; k < a.n; ++k) t += a.nstrip[k] * ((a.r[k][3] + L - 1) / L);
    return t;
  };
  // the kernel addresses a segment's rows through 32-bit buffer offsets:
  // (L + 3K + unroll + prefetch) rows of ld doubles must stay below 2^31
  const int64_t lmax = std::min<int64_t>(4096, (int64_t(1) << 31) / (ld * 8) - 3 * K - 2 * U - P);
  if (lmax < 1) return static_cast<int>(hipErrorInvalidValue);
  int64_t L = 0;
  if (o.seg_rows > 0) {
    L = o.seg_rows;
  } else {
    const int64_t res = resident_workgroups(fn, block, smem);
    double best = 1e300;
    for (int64_t m = 1;; ++m) {
      const int64_t cand = m * U - 3 * K;
      if (cand < 8) continue;
      if (cand > lmax || cand > maxh + U) break;
      const int64_t rounds = (tiles(cand) + res - 1) / res;
      const double cost = static_cast<double>(rounds) * static_cast<double>(std::min(cand, maxh) + 3 * K);
      if (cost < best * 0.999) {
        best = cost;
        L = cand;
      }
    }
    if (L == 0) L = std::max<int64_t>(8, U - 3 * K > 0 ? U - 3 * K : 8);
  }
  a.seg = static_cast<int>(std::min(std::min(L, maxh), lmax));
  a.nsteps = (a.seg + 3 * K + U - 1) / U * U;
  a.tstart[0] = 0;
  for (int k = 0; k < a.n; ++k) a.tstart[k + 1] = a.tstart[k] + a.nstrip[k] * ((a.r[k][3] + a.seg - 1) / a.seg);
  for (int k = a.n + 1; k <= kMaxRect; ++k) a.tstart[k] = a.tstart[a.n];
  const int64_t nb = a.tstart[a.n];
  if (smem > 64 * 1024) {  // 8-wave workgroups: 64 KiB of rings + the edge buffers
    static std::once_flag once;
    std::call_once(once, [&] {
      (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(smem));
    });
  }
  jacobi5tb_kernel<K, P, SHARE, EXACT><<<grid_1d(nb), block, smem, s>>>(a, u, un, nb);
  return static_cast<int>(hipGetLastError());
}

template <int K, int P>
int dispatch_k(const gmt_tb_opts& o, bool share, bool exact, int n_rect, const int64_t* rects, const int64_t* dom,
               int mask, const double* u, double* un, int64_t ld, int64_t nrows, hipStream_t s) {
  if (share)
    return exact ? launch_tb<K, P, true, true>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s)
                 : launch_tb<K, P, true, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s);
  return exact ? launch_tb<K, P, false, true>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s)
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
  int64_t maxw = 0;
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    // 16-B loads: even start; the K-wide ring left of / above the rect exists
    if ((r[0] % 2) != 0 || r[0] < K || r[2] < K || r[0] + r[1] > ld || r[2] + r[3] + K > nrows)
      return static_cast<int>(hipErrorInvalidValue);
    maxw = std::max(maxw, r[1]);
  }
  // workgroup width: NW waves share their edges through LDS; one wave per
  // workgroup for rects no wider than one strip (frame bands)
  const bool share = o.wg_waves != 1 && maxw > kCols - 2 * K;
  const bool exact = o.exact != 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int P = o.prefetch == 6 ? 6 : 3;
  switch (K) {
#define GMT_TB_CASE(KK)                                                                                   \
  case KK:                                                                                                \
    return P == 6 ? dispatch_k<KK, 6>(o, share, exact, n_rect, rects, dom, halo_mask, u, un, ld, nrows, s) \
                  : dispatch_k<KK, 3>(o, share, exact, n_rect, rects, dom, halo_mask, u, un, ld, nrows, s);
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
