// K fused 5-point Jacobi sweeps per memory pass, register-pipelined along y
// (wavefront temporal blocking), gfx950.
//
// Why a second temporal-blocking kernel: the LDS-tiled kernel
// (jacobi5x2.hip) re-reads every intermediate value from LDS (5 ds_read + 1
// ds_write per lattice update) and recomputes a K-cell ring per tile; at
// K = 4 it runs at ~0.75 clock per update per CU — LDS-issue bound, far
// from the HBM floor of 16/K bytes per update.
//
// Here one wave owns a 128-column strip (2 columns per lane) and walks down
// a segment of rows.  Time level p of row r is computed from level p-1 of
// rows r-1, r, r+1, which the wave computed in its three PREVIOUS steps, so
// every level lives in a 3-row register window (a skewed pipeline):
//   step s: level p of row s-2p for p = K..1 (independent of each other:
//           K-way instruction-level parallelism, no intra-step chain)
//           store level K (= u(t+K)) of row s-2K (16-B nontemporal stores)
//           level 0 <- row s of u(t) (prefetched three steps earlier)
// West/east neighbours come from the adjacent lane through DPP
// (wave_shr/wave_shl: no LDS, no barriers).  The wave edges lose one column
// per level, so a strip yields 128 - 2K output columns; a segment of L rows
// loads L + 2K rows in L + 3K steps.  Per update and sweep: 3 DADD + 1 DMUL
// + 2 DPP movs.  The three-slot register window is rotated by unrolling the
// row loop by 3 (no register moves).
//
// Same arithmetic and operand order as K single sweeps: bitwise equal.
// Dirichlet/halo rule as in jacobi5x2.hip: a ring cell outside the interior
// is updated only if that side's ghost cells belong to a neighbour
// (halo_mask bit0..3 = W/E/S/N); otherwise it keeps its (boundary) value.
// Waves whose influence cone stays inside the interior skip the rule.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

struct PipeArgs {
  int64_t r[4][4];     // output rects: x0, nx, y0, ny (absolute array coordinates, x0 even)
  int64_t nstrip[4];   // strips per rect
  int64_t wstart[5];   // prefix sum of waves (strips x segments)
  int64_t dom[4];      // interior: x0, nx, y0, ny
  int n;
  int mask;
  int seg[4];          // output rows per wave, per rect
  double quarter;      // 0.25 as a kernel argument: an SGPR operand (v_fma_f64 /
                       // v_mul_f64 with s[..]) instead of a literal that forces
                       // VOP2 v_fmac + a v_mov_b64 copy per use
};

constexpr int kPipeCols = 2 * kWave;  // columns per strip

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// FAST: the wave's whole influence cone lies inside the interior and the
// strip is full (128 - 2K output columns): no ghost rule, every load in
// range, every store a whole pair.  Then the loop has NO divergent control
// flow around memory ops — loads are unconditional (row index clamped) and
// the edge lanes' stores are dropped by the buffer unit's range check (a raw
// buffer store with an out-of-range offset is a no-op).  Branches around
// loads/stores make the waitcnt pass assume a skipped load and wait for
// vmcnt(0), which serialises every step on HBM latency; without them the
// three-row prefetch queue actually stays in flight.
// SKEW: level p of step s is row s - 2p computed from the three previous
// steps (K independent levels per step) instead of row s - p (a K-deep chain).
template <int K, bool FAST, bool SKEW>
__device__ __forceinline__ void pipe_strip(const PipeArgs& a, const double* __restrict__ u,
                                           double* __restrict__ un, int64_t ld, int lane,
                                           int64_t xs, int64_t xe, int64_t ys, int64_t ye) {
  constexpr int D = SKEW ? 2 : 1;  // row lag per level
  constexpr int LAG = D * K;       // output row = level-0 row - LAG
  const int64_t xa = xs - K;          // strip column 0 (even)
  const int64_t c0 = xa + 2 * lane;   // this lane's columns c0, c0 + 1
  const int64_t dx0 = a.dom[0], dx1 = a.dom[0] + a.dom[1];
  const int64_t dy0 = a.dom[2], dy1 = a.dom[2] + a.dom[3];
  const int64_t xlim = dx1 + K, ylim = dy1 + K;  // first column / row past the stored ring
  const bool gw = a.mask & 1, ge = a.mask & 2, gs = a.mask & 4, gn = a.mask & 8;
  // per-lane column rule (!FAST only)
  const bool rx0 = (c0 >= dx0 && c0 < dx1) || (c0 < dx0 ? gw : ge);
  const bool rx1 = (c0 + 1 >= dx0 && c0 + 1 < dx1) || (c0 + 1 < dx0 ? gw : ge);
  // load mask: whole pair, first column only, or nothing (!FAST only)
  const int lmode = c0 + 1 < xlim ? 2 : (c0 < xlim ? 1 : 0);
  // store mask
  const bool st0 = c0 >= xs && c0 < xe, st1 = c0 + 1 >= xs && c0 + 1 < xe;

  const int64_t yl = ys - K;  // row loaded at step 0
  const int nload = static_cast<int>(ye - ys) + 2 * K;
  const int nsteps = static_cast<int>(ye - ys) + K + LAG;
  const double* up = u + yl * ld + c0;

  auto load = [&](int s) -> d2 {
    if constexpr (FAST) {
      const int sc = s < nload ? s : nload - 1;  // tail: re-read the last row (unused)
      return ld2(up + static_cast<int64_t>(sc) * ld);
    } else {
      d2 v = {0.0, 0.0};
      if (s < nload && yl + s < ylim) {
        const double* p = up + static_cast<int64_t>(s) * ld;
        if (lmode == 2)
          v = ld2(p);
        else if (lmode == 1)
          v.x = p[0];
      }
      return v;
    }
  };
  const uint32_t st_off = (st0 && st1) ? static_cast<uint32_t>(c0 - xs) * 8u : 0x80000000u;
  const uint32_t st_bytes = static_cast<uint32_t>(xe - xs) * 8u;
  auto store = [&](int s, d2 v) {
    double* row = un + (yl + s - LAG) * ld;
    if constexpr (FAST) {
      // 0x00020000: raw-buffer descriptor word 3 for gfx9 (32-bit data format)
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(row + xs, 0, st_bytes, 0x00020000);
      typedef unsigned u4 __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, st_off, 0, 2 /* nt */);
    } else {
      double* q = row + c0;
      if (st0 && st1)
        st2_nt(q, v);
      else if (st0)
        q[0] = v.x;
      else if (st1)
        q[1] = v.y;
    }
  };

  d2 W[K][3];  // W[p][slot]: level p, slot = step % 3
#pragma unroll
  for (int p = 0; p < K; ++p)
#pragma unroll
    for (int j = 0; j < 3; ++j) W[p][j] = d2{0.0, 0.0};
  d2 Q[3];  // prefetch queue: row for step s sits in Q[s % 3], loaded at step s - 3
  Q[0] = load(0);
  Q[1] = load(1);
  Q[2] = load(2);

  auto level = [&](int p, int s, const d2& up_, const d2& c, const d2& dn) -> d2 {
    // no fma contraction: 6 DADD + 2 DMUL (SGPR operand) per 2 cells, and the
    // scaled values are the only ones kept live
#pragma clang fp contract(off)
    const double w = dpp_from_lower(c.y), e = dpp_from_upper(c.x);
    d2 v;
    // a.quarter == 0.25 exactly: any fma contraction of the scaling is exact
    v.x = a.quarter * ((w + c.y) + (up_.x + dn.x));
    v.y = a.quarter * ((c.x + e) + (up_.y + dn.y));
    if constexpr (!FAST) {
      const int64_t r = yl + s - D * p;  // row of this level's value
      const bool ry = (r >= dy0 && r < dy1) || (r < dy0 ? gs : gn);
      v.x = (ry && rx0) ? v.x : c.x;
      v.y = (ry && rx1) ? v.y : c.y;
    }
    return v;
  };
  // one pipeline step; returns level K of row s - LAG
  auto step = [&](auto P, int s) -> d2 {
    constexpr int cur = decltype(P)::value, s2 = (cur + 1) % 3, s1 = (cur + 2) % 3;
    d2 out;
    if constexpr (SKEW) {
      // level p-1 slots written at steps s-3 (cur), s-2 (s2), s-1 (s1); top-down
#pragma unroll
      for (int p = K; p >= 1; --p) {
        const d2 v = level(p, s, W[p - 1][cur], W[p - 1][s2], W[p - 1][s1]);
        if (p < K)
          W[p][cur] = v;
        else
          out = v;
      }
      W[0][cur] = Q[cur];
      Q[cur] = load(s + 3);
    } else {
      // level p-1 slots of steps s-2 (s2), s-1 (s1), s (cur); bottom-up
      W[0][cur] = Q[cur];
      Q[cur] = load(s + 3);
#pragma unroll
      for (int p = 1; p <= K; ++p) {
        const d2 v = level(p, s, W[p - 1][s2], W[p - 1][s1], W[p - 1][cur]);
        if (p < K)
          W[p][cur] = v;
        else
          out = v;
      }
    }
    return out;
  };
  // warm-up: steps before the first output row (ys = yl + K) produce nothing
  constexpr int WARM = K + LAG;
  using I0 = std::integral_constant<int, WARM % 3>;
  using I1 = std::integral_constant<int, (WARM + 1) % 3>;
  using I2 = std::integral_constant<int, (WARM + 2) % 3>;
  static_for<0, WARM>([&](auto S) { step(std::integral_constant<int, decltype(S)::value % 3>{}, S); });
  int s = WARM;
  for (; s + 3 <= nsteps; s += 3) {
    store(s, step(I0{}, s));
    store(s + 1, step(I1{}, s + 1));
    store(s + 2, step(I2{}, s + 2));
  }
  if (s < nsteps) store(s, step(I0{}, s));
  if (s + 1 < nsteps) store(s + 1, step(I1{}, s + 1));
}

// FAST: this launch runs only the interior full-strip waves (branch-free
// path); otherwise only the others (ghost rule, partial strips).  Two
// kernels, because a kernel's VGPR budget is the max over its paths: the
// rule path would cost the fast one a wave per SIMD (K = 8: 188 -> 142 VGPRs
// with the skewed pipeline).
// MODE 0: both paths in one kernel (A/B measurement), 1: fast waves only,
// 2: the other waves only.
template <int K, bool SKEW, int MODE>
__global__ __launch_bounds__(kBlock)
void jacobi5pipe_kernel(PipeArgs a, const double* __restrict__ u, double* __restrict__ un, int64_t ld,
                        int64_t nblocks) {
  const int lane = threadIdx.x & (kWave - 1);
  // readfirstlane: the wave index is uniform, so everything derived from it
  // (strip, rows, buffer descriptors) lives in SGPRs
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  const int64_t wid = xcd_swizzle(blockIdx.x, nblocks) * (kBlock / kWave) + wave;
  if (wid >= a.wstart[a.n]) return;  // whole wave
  int k = 0;
  while (k + 1 < a.n && wid >= a.wstart[k + 1]) ++k;
  const int64_t lt = wid - a.wstart[k];
  // strips of one segment are consecutive waves (same workgroup / XCD:
  // they share the 2K overlap columns in L2)
  const int64_t strip = lt % a.nstrip[k], seg = lt / a.nstrip[k];
  constexpr int WOUT = kPipeCols - 2 * K;
  const int64_t rx1 = a.r[k][0] + a.r[k][1], ry1 = a.r[k][2] + a.r[k][3];
  const int64_t xs = a.r[k][0] + strip * WOUT;
  const int64_t xe = xs + WOUT < rx1 ? xs + WOUT : rx1;
  const int64_t ys = a.r[k][2] + seg * a.seg[k];
  const int64_t ye = ys + a.seg[k] < ry1 ? ys + a.seg[k] : ry1;
  // influence cone of the outputs inside the interior: no ghost rule
  const bool inner = xs - K >= a.dom[0] && xe + K <= a.dom[0] + a.dom[1] && ys - K >= a.dom[2] &&
                     ye + K <= a.dom[2] + a.dom[3];
  const bool fast = inner && xe - xs == WOUT;
  if (MODE == 0) {
    if (fast)
      pipe_strip<K, true, SKEW>(a, u, un, ld, lane, xs, xe, ys, ye);
    else
      pipe_strip<K, false, SKEW>(a, u, un, ld, lane, xs, xe, ys, ye);
    return;
  }
  if (fast != (MODE == 1)) return;
  pipe_strip<K, MODE == 1, SKEW>(a, u, un, ld, lane, xs, xe, ys, ye);
}

}  // namespace gmt

// nsweeps even, 2..8; seg = output rows per wave (0 = default).
extern "C" int gmt_jacobi5xk_pipe(int nsweeps, int n_rect, const int64_t* rects, const int64_t* dom,
                                  int halo_mask, const double* u, double* un, int64_t ld, int seg,
                                  void* stream) {
  using namespace gmt;
  if (nsweeps < 2 || nsweeps > 8 || (nsweeps % 2) != 0) return static_cast<int>(hipErrorInvalidValue);
  if (n_rect < 0 || n_rect > 4) return static_cast<int>(hipErrorInvalidValue);
  if (!aligned16(u) || !aligned16(un) || (ld % 2) != 0) return static_cast<int>(hipErrorInvalidValue);
  PipeArgs a{};
  const int seg_rows = seg & 0xffff;
  a.quarter = 0.25;
  a.mask = halo_mask;
  for (int j = 0; j < 4; ++j) a.dom[j] = dom[j];
  const int wout = kPipeCols - 2 * nsweeps;
  int64_t nfast = 0, nrule = 0;
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    if ((r[0] % 2) != 0) return static_cast<int>(hipErrorInvalidValue);  // 16-B loads
    for (int j = 0; j < 4; ++j) a.r[a.n][j] = r[j];
    a.nstrip[a.n] = (r[1] + wout - 1) / wout;
    // default segment: 256 rows, halved (down to 16) while the rect would
    // give fewer than ~4096 waves — thin frame rects and small domains still
    // fill 256 CUs (the pipeline refill costs 2K extra rows per segment)
    int sg = seg_rows;
    if (sg <= 0) {
      sg = 256;
      while (sg > 16 && a.nstrip[a.n] * ((r[3] + sg - 1) / sg) < 4096) sg /= 2;
    }
    a.seg[a.n] = sg;
    const int64_t nseg = (r[3] + sg - 1) / sg;
    a.wstart[a.n + 1] = a.wstart[a.n] + a.nstrip[a.n] * nseg;
    // waves the kernel will classify as fast (same predicate as the device)
    int64_t fx = 0, fy = 0;
    for (int64_t i = 0; i < a.nstrip[a.n]; ++i) {
      const int64_t xs = r[0] + i * wout, xe = xs + wout;
      fx += xe <= r[0] + r[1] && xs - nsweeps >= dom[0] && xe + nsweeps <= dom[0] + dom[1];
    }
    for (int64_t i = 0; i < nseg; ++i) {
      const int64_t ys = r[2] + i * sg, ye = ys + sg < r[2] + r[3] ? ys + sg : r[2] + r[3];
      fy += ys - nsweeps >= dom[2] && ye + nsweeps <= dom[2] + dom[3];
    }
    nfast += fx * fy;
    nrule += a.nstrip[a.n] * nseg - fx * fy;
    ++a.n;
  }
  if (a.n == 0) return 0;
  for (int k = a.n + 1; k <= 4; ++k) a.wstart[k] = a.wstart[a.n];
  const int64_t waves = a.wstart[a.n];
  const int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned g = grid_1d(nb);
  const int sk = (seg >> 19) & 3;  // 0 = per-K default, 1 = skewed, 2 = chained pipeline
  // skewed (level-parallel) pipeline by default: fewer VGPRs for the fast
  // path at K = 6, 8 (measured, profiles/r01_pipe.md)
  const bool skew = sk == 0 ? nsweeps >= 6 : sk == 1;
  const bool single = (seg >> 21) & 1;  // one kernel for both paths (A/B)
#define GMT_PIPE(KK)                                                                        \
  do {                                                                                      \
    if (single) {                                                                           \
      if (skew) jacobi5pipe_kernel<KK, true, 0><<<g, kBlock, 0, s>>>(a, u, un, ld, nb);     \
      else jacobi5pipe_kernel<KK, false, 0><<<g, kBlock, 0, s>>>(a, u, un, ld, nb);         \
      break;                                                                                \
    }                                                                                       \
    if (nrule && skew) jacobi5pipe_kernel<KK, true, 2><<<g, kBlock, 0, s>>>(a, u, un, ld, nb);   \
    if (nrule && !skew) jacobi5pipe_kernel<KK, false, 2><<<g, kBlock, 0, s>>>(a, u, un, ld, nb); \
    if (nfast && skew) jacobi5pipe_kernel<KK, true, 1><<<g, kBlock, 0, s>>>(a, u, un, ld, nb);    \
    if (nfast && !skew) jacobi5pipe_kernel<KK, false, 1><<<g, kBlock, 0, s>>>(a, u, un, ld, nb);  \
  } while (0)
  switch (nsweeps) {
    case 2: GMT_PIPE(2); break;
    case 4: GMT_PIPE(4); break;
    case 6: GMT_PIPE(6); break;
    default: GMT_PIPE(8); break;
  }
#undef GMT_PIPE
  GMT_RET_LAUNCH();
}
