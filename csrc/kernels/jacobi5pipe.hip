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
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

// An input rect is split on the host into a fast core (full strips whose
// influence cone stays inside the interior) and up to 4 rule bands around it.
// The bands get short segments, so the few ghost-rule waves (branchy: about
// one HBM latency per step) finish in tens of microseconds instead of one
// long segment's worth (0.68 ms of a 4.2 ms pass at 256 rows per wave,
// profiles/r01_pipe.md).
constexpr int kMaxPipeRect = 24;  // 4 input rects x (2 fast + 4 rule bands)

struct PipeArgs {
  int64_t r[kMaxPipeRect][4];        // output rects: x0, nx, y0, ny (absolute array coordinates, x0 even)
  int64_t nstrip[kMaxPipeRect];      // strips per rect
  int64_t wstart[kMaxPipeRect + 1];  // prefix sum of waves (strips x segments)
  int64_t dom[4];      // interior: x0, nx, y0, ny
  int64_t wbase, wend; // this launch runs waves [wbase, wend)
  int n;
  int mask;
  int classified;      // 1: rect order = rule rects, then fast cores (no per-wave test)
  int seg[kMaxPipeRect];  // output rows per wave, per rect
  double quarter;      // 0.25 as a kernel argument: an SGPR operand (v_fma_f64 /
                       // v_mul_f64 with s[..]) instead of a literal that forces
                       // VOP2 v_fmac + a v_mov_b64 copy per use
};

constexpr int kPipeCols = 2 * kWave;  // columns per strip
constexpr int kPipeMaxK = 14;         // sweeps per pass (even): K = 14 still fits 2 waves per SIMD (254 VGPRs)

// Waves per SIMD the fast path is held to (512 VGPRs / waves).  Without the
// bound the scheduler interleaves all K independent levels of a step and the
// temporaries push K = 10 to 232 VGPRs (2 waves) instead of ~166 (3 waves).
constexpr int pipe_waves(int K, int mode) { return mode != 1 || K <= 8 ? 1 : (K <= 10 ? 3 : 2); }

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
template <int K, bool FAST, bool SKEW, bool SCALE = true>
__device__ __forceinline__ void pipe_strip(const PipeArgs& a, const double* __restrict__ u,
                                           double* __restrict__ un, int64_t ld, int lane,
                                           int64_t xs, int64_t xe, int64_t ys, int64_t ye) {
  constexpr int D = SKEW ? 2 : 1;  // row lag per level
  constexpr int LAG = D * K;       // output row = level-0 row - LAG
  const int64_t xa = xs - K;          // strip column 0 (even)
  const int64_t c0 = xa + 2 * lane;   // this lane's columns c0, c0 + 1
  const int64_t dx0 = a.dom[0], dx1 = a.dom[0] + a.dom[1];
  const int64_t dy0 = a.dom[2], dy1 = a.dom[2] + a.dom[3];
  const bool gw = a.mask & 1, ge = a.mask & 2, gs = a.mask & 4, gn = a.mask & 8;
  // per-lane column rule (!FAST only)
  const bool rx0 = (c0 >= dx0 && c0 < dx1) || (c0 < dx0 ? gw : ge);
  const bool rx1 = (c0 + 1 >= dx0 && c0 + 1 < dx1) || (c0 + 1 < dx0 ? gw : ge);
  // store mask
  const bool st0 = c0 >= xs && c0 < xe, st1 = c0 + 1 >= xs && c0 + 1 < xe;

  const int64_t yl = ys - K;  // row loaded at step 0
  const int nload = static_cast<int>(ye - ys) + 2 * K;
  const int nsteps = static_cast<int>(ye - ys) + K + LAG;
  // Both paths load unconditionally (no branch around a load, see FAST).
  // Rows past the segment's last row are clamped to it, and lanes past the
  // array row (right-edge strips) to its last column pair: those values, and
  // anything outside the ghost ring, only feed cells whose K-step cone ends
  // outside the interior — never a stored output.
  const double* up = u + yl * ld + (FAST ? c0 : (c0 < ld - 2 ? c0 : ld - 2));
  auto load = [&](int s) -> d2 {
    const int sc = s < nload ? s : nload - 1;  // tail: re-read the last row (unused)
    return ld2(up + static_cast<int64_t>(sc) * ld);
  };
  // stores through a raw buffer descriptor spanning [xs, xe) of the row: an
  // out-of-range offset (0x80000000) makes the store a no-op, so edge lanes
  // need no branch either
  constexpr uint32_t kDrop = 0x80000000u;
  const uint32_t st_off = (st0 && st1) ? static_cast<uint32_t>(c0 - xs) * 8u : kDrop;
  const uint32_t st_off0 = st0 ? static_cast<uint32_t>(c0 - xs) * 8u : kDrop;
  const uint32_t st_off1 = st1 ? static_cast<uint32_t>(c0 + 1 - xs) * 8u : kDrop;
  const uint32_t st_bytes = static_cast<uint32_t>(xe - xs) * 8u;
  auto store = [&](int s, d2 v) {
    if constexpr (FAST && SCALE) {  // level K was kept scaled by 4^K (see level)
      constexpr double kUnscale = 1.0 / static_cast<double>(1ull << (2 * K));
      v.x *= kUnscale;
      v.y *= kUnscale;
    }
    double* row = un + (yl + s - LAG) * ld;
    // 0x00020000: raw-buffer descriptor word 3 for gfx9 (32-bit data format)
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(row + xs, 0, st_bytes, 0x00020000);
    if constexpr (FAST) {
      typedef unsigned u4 __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, st_off, 0, 2 /* nt */);
    } else {
      // odd rect edges leave single-column lanes: two 8-B stores
      // (the halves are built explicitly: bit_cast of the two vector
      // elements was folded into one register pair by clang 22)
      typedef unsigned u2 __attribute__((ext_vector_type(2)));
      const double vx = v.x, vy = v.y;
      const u2 bx = {static_cast<unsigned>(__double2loint(vx)), static_cast<unsigned>(__double2hiint(vx))};
      const u2 by = {static_cast<unsigned>(__double2loint(vy)), static_cast<unsigned>(__double2hiint(vy))};
      __builtin_amdgcn_raw_buffer_store_b64(bx, r, st_off0, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b64(by, r, st_off1, 0, 2);
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
    if constexpr (FAST && SCALE) {
      // scaled levels: V_p = 4^p u_p, so V_p = (W + C) + (N + S) with no
      // multiply (scaling by a power of two commutes with every rounding
      // step: bitwise 4^p times the unscaled update, barring overflow and
      // subnormals); the output is scaled back once per stored value
      v.x = (w + c.y) + (up_.x + dn.x);
      v.y = (c.x + e) + (up_.y + dn.y);
    } else {
      // a.quarter == 0.25 exactly: any fma contraction of the scaling is exact
      v.x = a.quarter * ((w + c.y) + (up_.x + dn.x));
      v.y = a.quarter * ((c.x + e) + (up_.y + dn.y));
    }
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
        // K > 8: keep the levels in order (a fence for the scheduler only),
        // else their interleaved temporaries cost a wave per SIMD
        if constexpr (K > 8) __builtin_amdgcn_sched_barrier(0);
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
template <int K, bool SKEW, int MODE, bool SCALE = true>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(pipe_waves(K, MODE))))
void jacobi5pipe_kernel(PipeArgs a, const double* __restrict__ u, double* __restrict__ un, int64_t ld,
                        int64_t nblocks) {
  const int lane = threadIdx.x & (kWave - 1);
  // readfirstlane: the wave index is uniform, so everything derived from it
  // (strip, rows, buffer descriptors) lives in SGPRs
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  const int64_t wid = a.wbase + xcd_swizzle(blockIdx.x, nblocks) * (kBlock / kWave) + wave;
  if (wid >= a.wend) return;  // whole wave
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
  if (!a.classified && fast != (MODE == 1)) return;
  pipe_strip<K, MODE == 1, SKEW, SCALE>(a, u, un, ld, lane, xs, xe, ys, ye);
}

}  // namespace gmt

namespace {

// Split rect r into fast rects (whole strips, branch-free path) and rule
// bands (ghost rule / partial strips).  A cell may take the fast path when
// every load of its K-step cone is valid data that the kernel may update:
// interior cells, and ghost cells of sides whose ring belongs to a neighbour
// (halo_mask bit set: the caller exchanged a K-wide halo, corners included,
// and the rule would update those cells anyway).  So the fast limits are the
// interior inset by K on Dirichlet sides only.
//
// Columns: full strips of wout outputs from fx0; a leftover narrower than a
// strip becomes one more full strip shifted left to end at fx1 (its overlap
// with the previous strip is recomputed — the same operations on the same
// inputs, so the same bits, written twice).  With `ext`, a rect narrower
// than a strip may also be covered by a strip reaching outside the rect
// (still within the fast limits): the caller allows cells of the interior
// outside its rects to be rewritten with their own values, e.g. the frame
// pass after the core pass has written them.  An odd leftover column the
// shifted strip cannot reach (16-B aligned starts) goes to the rule band.
// Returns the number of fast rects (0: the whole rect is one rule band).
int split_rect(const int64_t* r, const int64_t* dom, int mask, bool ext, int K, int64_t wout,
               int64_t fast[2][4], int64_t band[4][4]) {
  const int64_t x0 = r[0], x1 = r[0] + r[1], y0 = r[2], y1 = r[2] + r[3];
  const int64_t lx = dom[0] + ((mask & 1) ? 0 : K), ux = dom[0] + dom[1] - ((mask & 2) ? 0 : K);
  const int64_t ly = dom[2] + ((mask & 4) ? 0 : K), uy = dom[2] + dom[3] - ((mask & 8) ? 0 : K);
  const int64_t fy0 = std::max(y0, ly), fy1 = std::min(y1, uy);
  int64_t fx0 = std::max(x0, lx);
  fx0 += fx0 & 1;  // even: 16-B loads
  const int64_t fx1 = std::min(x1, ux);
  if (fy1 <= fy0 || fx1 <= fx0) return 0;
  const int64_t cx1 = fx0 + (fx1 - fx0) / wout * wout;  // end of the whole strips
  // the shifted strip goes first: waves run in rect order, and its few long
  // segments must not be the launch's tail
  int nf = 0;
  int64_t xend = cx1;  // first column not covered by a fast rect
  if (cx1 < fx1) {
    // one more strip [sx, sx + wout): even start, inside the fast limits,
    // starting at or before cx1 (inside the rect unless ext)
    int64_t sx = (fx1 - wout) & ~int64_t(1);
    const int64_t lo = ext ? lx : fx0;
    if (sx < lo) sx = lo + (lo & 1);
    if (sx <= cx1 && sx + wout <= ux && sx + wout > cx1 && (ext || sx + wout <= fx1)) {
      const int64_t c[4] = {sx, wout, fy0, fy1 - fy0};
      std::copy(c, c + 4, fast[nf++]);
      xend = sx + wout;
    }
  }
  if (cx1 > fx0) {
    const int64_t c[4] = {fx0, cx1 - fx0, fy0, fy1 - fy0};
    std::copy(c, c + 4, fast[nf++]);
  }
  if (nf == 0) return 0;
  xend = std::min(xend, x1);
  const int64_t b[4][4] = {{x0, x1 - x0, y0, fy0 - y0},
                           {x0, x1 - x0, fy1, y1 - fy1},
                           {x0, fx0 - x0, fy0, fy1 - fy0},
                           {xend, x1 - xend, fy0, fy1 - fy0}};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) band[i][j] = b[i][j];
  return nf;
}

}  // namespace

// nsweeps even, 2..8; seg & 0xffff = output rows per fast-core wave (0 = default).
extern "C" int gmt_jacobi5xk_pipe(int nsweeps, int n_rect, const int64_t* rects, const int64_t* dom,
                                  int halo_mask, const double* u, double* un, int64_t ld, int seg,
                                  void* stream) {
  using namespace gmt;
  if (nsweeps < 2 || nsweeps > kPipeMaxK || (nsweeps % 2) != 0) return static_cast<int>(hipErrorInvalidValue);
  if (n_rect < 0 || n_rect > 4) return static_cast<int>(hipErrorInvalidValue);
  if (!aligned16(u) || !aligned16(un) || (ld % 2) != 0) return static_cast<int>(hipErrorInvalidValue);
  PipeArgs a{};
  const int seg_rows = seg & 0xffff;
  const int sk = (seg >> 19) & 3;         // 0 = per-K default, 1 = skewed, 2 = chained pipeline
  const bool single = (seg >> 21) & 1;    // one kernel for both paths (A/B)
  const bool nosplit = (seg >> 22) & 1;   // two kernels, per-wave classification (A/B)
  const int rule_rows = (seg >> 23) & 0x3f ? (seg >> 23) & 0x3f : (nsweeps >= 10 ? 32 : 16);
  const bool ext = (seg >> 29) & 1;       // GMT_XK_EXT: may rewrite interior cells outside the rects
  const bool classified = !single && !nosplit;
  a.quarter = 0.25;
  a.mask = halo_mask;
  a.classified = classified;
  for (int j = 0; j < 4; ++j) a.dom[j] = dom[j];
  const int64_t wout = kPipeCols - 2 * nsweeps;
  // rule rects first, then the fast cores: each kernel's waves are one range
  int64_t rl[kMaxPipeRect][4], fl[kMaxPipeRect][4];
  int nr = 0, nf = 0;
  int fgroup[kMaxPipeRect];  // fast rect -> index of the widest fast rect of its input rect
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    if ((r[0] % 2) != 0) return static_cast<int>(hipErrorInvalidValue);  // 16-B loads
    // the K-wide ring left of / above the rect must exist (relative to u)
    if (r[0] < nsweeps || r[2] < nsweeps) return static_cast<int>(hipErrorInvalidValue);
    int64_t core[2][4], band[4][4];
    const int ncore = classified ? split_rect(r, dom, halo_mask, ext, nsweeps, wout, core, band) : 0;
    if (ncore > 0) {
      const int widest = nf + (ncore == 2 && core[1][1] > core[0][1] ? 1 : 0);
      for (int c = 0; c < ncore; ++c) {
        fgroup[nf] = widest;
        std::copy(core[c], core[c] + 4, fl[nf++]);
      }
      for (auto& b : band)
        if (b[1] > 0 && b[3] > 0) std::copy(b, b + 4, rl[nr++]);
    } else {
      std::copy(r, r + 4, rl[nr++]);
    }
  }
  // default rows per wave of a rect (see add)
  auto auto_seg = [&](const int64_t* r) {
    const int64_t ns = (r[1] + wout - 1) / wout;
    int sg = nsweeps >= 6 && nsweeps < 12 ? 128 : 256;
    while (sg > 16 && ns * ((r[3] + sg - 1) / sg) < 4096) sg /= 2;
    return sg;
  };
  auto add = [&](const int64_t* r, bool rule, int sg_fast) {
    for (int j = 0; j < 4; ++j) a.r[a.n][j] = r[j];
    a.nstrip[a.n] = (r[1] + wout - 1) / wout;
    // fast core: 128 rows per wave at K = 6..10, else 256, halved (down to
    // 16) while the rect would give fewer than ~4096 waves (small domains
    // still fill 256 CUs; the pipeline refill costs 2K extra rows per
    // segment).  Rule bands: 16 rows, 32 at K >= 10 (or (seg >> 23) & 63) —
    // latency-bound waves, so many short ones (measured, profiles/r01_k12.md).
    // A shifted last strip takes its main core's length: the XCD swizzle
    // gives every XCD the same NUMBER of blocks, so a run of short-segment
    // blocks (all on one XCD) would leave the other seven a longer tail.
    int sg = rule && classified ? rule_rows : seg_rows;
    if (sg <= 0) sg = rule ? auto_seg(r) : sg_fast;
    a.seg[a.n] = sg;
    a.wstart[a.n + 1] = a.wstart[a.n] + a.nstrip[a.n] * ((r[3] + sg - 1) / sg);
    ++a.n;
  };
  for (int i = 0; i < nr; ++i) add(rl[i], true, 0);
  const int64_t nrule = a.wstart[a.n];
  for (int i = 0; i < nf; ++i) add(fl[i], false, auto_seg(fl[fgroup[i]]));
  const int64_t waves = a.wstart[a.n];
  if (waves == 0) return 0;
  for (int k = a.n + 1; k <= kMaxPipeRect; ++k) a.wstart[k] = a.wstart[a.n];
  hipStream_t s = static_cast<hipStream_t>(stream);
  constexpr int64_t wpb = kBlock / kWave;
  // skewed (level-parallel) pipeline by default: fewer VGPRs for the fast
  // path at K = 6, 8 (measured, profiles/r01_pipe.md)
  const bool skew = sk == 0 ? nsweeps >= 6 : sk == 1;
  static const bool scaled = [] {
    const char* e = std::getenv("GMT_PIPE_SCALED");
    return !(e && e[0] == '0');
  }();
  auto launch = [&](auto KC, auto MC, int64_t w0, int64_t w1) {
    constexpr int KK = decltype(KC)::value, MODE = decltype(MC)::value;
    if (w1 <= w0) return;
    a.wbase = w0;
    a.wend = w1;
    const int64_t nb = (w1 - w0 + wpb - 1) / wpb;
    if constexpr (MODE == 1) {
      if (!scaled) {  // A/B: GMT_PIPE_SCALED=0 keeps the 0.25 multiply per level
        jacobi5pipe_kernel<KK, true, MODE, false><<<grid_1d(nb), kBlock, 0, s>>>(a, u, un, ld, nb);
        return;
      }
    }
    if (skew)
      jacobi5pipe_kernel<KK, true, MODE><<<grid_1d(nb), kBlock, 0, s>>>(a, u, un, ld, nb);
    else
      jacobi5pipe_kernel<KK, false, MODE><<<grid_1d(nb), kBlock, 0, s>>>(a, u, un, ld, nb);
  };
  auto run = [&](auto KC) {
    using M0 = std::integral_constant<int, 0>;
    using M1 = std::integral_constant<int, 1>;
    using M2 = std::integral_constant<int, 2>;
    if (single) {
      launch(KC, M0{}, 0, waves);
    } else if (nosplit) {  // both kernels over every wave, each keeps its own
      launch(KC, M2{}, 0, waves);
      launch(KC, M1{}, 0, waves);
    } else {
      launch(KC, M2{}, 0, nrule);
      launch(KC, M1{}, nrule, waves);
    }
  };
  switch (nsweeps) {
    case 2: run(std::integral_constant<int, 2>{}); break;
    case 4: run(std::integral_constant<int, 4>{}); break;
    case 6: run(std::integral_constant<int, 6>{}); break;
    case 8: run(std::integral_constant<int, 8>{}); break;
    case 10: run(std::integral_constant<int, 10>{}); break;
    case 12: run(std::integral_constant<int, 12>{}); break;
    default: run(std::integral_constant<int, 14>{}); break;
  }
  GMT_RET_LAUNCH();
}
