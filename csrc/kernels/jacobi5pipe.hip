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
  int seg;             // output rows per wave
};

constexpr int kPipeCols = 2 * kWave;  // columns per strip

template <int K, bool RULE>
__device__ __forceinline__ void pipe_strip(const PipeArgs& a, const double* __restrict__ u,
                                           double* __restrict__ un, int64_t ld, int lane,
                                           int64_t xs, int64_t xe, int64_t ys, int64_t ye) {
  const int64_t xa = xs - K;          // strip column 0 (even)
  const int64_t c0 = xa + 2 * lane;   // this lane's columns c0, c0 + 1
  const int64_t dx0 = a.dom[0], dx1 = a.dom[0] + a.dom[1];
  const int64_t dy0 = a.dom[2], dy1 = a.dom[2] + a.dom[3];
  const int64_t xlim = dx1 + K, ylim = dy1 + K;  // first column / row past the stored ring
  const bool gw = a.mask & 1, ge = a.mask & 2, gs = a.mask & 4, gn = a.mask & 8;
  // per-lane column rule (RULE only)
  const bool rx0 = (c0 >= dx0 && c0 < dx1) || (c0 < dx0 ? gw : ge);
  const bool rx1 = (c0 + 1 >= dx0 && c0 + 1 < dx1) || (c0 + 1 < dx0 ? gw : ge);
  // load mask: whole pair, first column only, or nothing
  const int lmode = c0 + 1 < xlim ? 2 : (c0 < xlim ? 1 : 0);
  // store mask
  const bool st0 = c0 >= xs && c0 < xe, st1 = c0 + 1 >= xs && c0 + 1 < xe;

  // Skewed pipeline: level p at step s is row yl + s - 2p, computed from
  // level p-1 of the three PREVIOUS steps, so the K levels of one step are
  // independent (K-way ILP instead of a K-deep dependency chain); levels are
  // evaluated top-down so level p reads slot s%3 of level p-1 before level
  // p-1 overwrites it.
  const int64_t yl = ys - K;                 // row loaded at step 0
  const int nload = static_cast<int>(ye - ys) + 2 * K;
  const int nsteps = static_cast<int>(ye - ys) + 3 * K;
  const double* up = u + yl * ld + c0;
  double* op = un + (ys - 3 * K) * ld + c0;  // output row of step s: ys - 3K + s

  auto load = [&](int s) -> d2 {
    d2 v = {0.0, 0.0};
    if (s < nload && yl + s < ylim) {
      const double* p = up + static_cast<int64_t>(s) * ld;
      if (lmode == 2)
        v = ld2(p);
      else if (lmode == 1)
        v.x = p[0];
    }
    return v;
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

  auto step = [&](auto P, int s) {
    // slots of level p-1 written at steps s-3, s-2, s-1
    constexpr int cur = decltype(P)::value, s3 = cur, s2 = (cur + 1) % 3, s1 = (cur + 2) % 3;
#pragma unroll
    for (int p = K; p >= 1; --p) {
      const d2 up_ = W[p - 1][s3], c = W[p - 1][s2], dn = W[p - 1][s1];
      const double w = dpp_from_lower(c.y), e = dpp_from_upper(c.x);
      d2 v;
      v.x = 0.25 * ((w + c.y) + (up_.x + dn.x));
      v.y = 0.25 * ((c.x + e) + (up_.y + dn.y));
      if (RULE) {
        const int64_t r = yl + s - 2 * p;  // row of this level's value
        const bool ry = (r >= dy0 && r < dy1) || (r < dy0 ? gs : gn);
        v.x = (ry && rx0) ? v.x : c.x;
        v.y = (ry && rx1) ? v.y : c.y;
      }
      if (p < K) {
        W[p][cur] = v;
      } else if (s >= 3 * K) {
        double* q = op + static_cast<int64_t>(s) * ld;
        if (st0 && st1)
          st2_nt(q, v);
        else if (st0)
          q[0] = v.x;
        else if (st1)
          q[1] = v.y;
      }
    }
    W[0][cur] = Q[cur];
    Q[cur] = load(s + 3);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  for (int s = 0; s < nsteps; s += 3) {
    step(I0{}, s);
    if (s + 1 < nsteps) step(I1{}, s + 1);
    if (s + 2 < nsteps) step(I2{}, s + 2);
  }
}

// OCC: minimum waves per SIMD requested from the register allocator (1 = no
// constraint); caps the VGPR budget of the deep (K = 6, 8) pipelines.
template <int K, int OCC>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(OCC)))
void jacobi5pipe_kernel(PipeArgs a, const double* __restrict__ u, double* __restrict__ un, int64_t ld,
                        int64_t nblocks) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wid = xcd_swizzle(blockIdx.x, nblocks) * (kBlock / kWave) + threadIdx.x / kWave;
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
  const int64_t ys = a.r[k][2] + seg * a.seg;
  const int64_t ye = ys + a.seg < ry1 ? ys + a.seg : ry1;
  // influence cone of the outputs inside the interior: no ghost rule
  const bool inner = xs - K >= a.dom[0] && xe + K <= a.dom[0] + a.dom[1] && ys - K >= a.dom[2] &&
                     ye + K <= a.dom[2] + a.dom[3];
  if (inner)
    pipe_strip<K, false>(a, u, un, ld, lane, xs, xe, ys, ye);
  else
    pipe_strip<K, true>(a, u, un, ld, lane, xs, xe, ys, ye);
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
  a.seg = (seg & 0xffff) > 0 ? (seg & 0xffff) : 256;
  a.mask = halo_mask;
  for (int j = 0; j < 4; ++j) a.dom[j] = dom[j];
  const int wout = kPipeCols - 2 * nsweeps;
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    if ((r[0] % 2) != 0) return static_cast<int>(hipErrorInvalidValue);  // 16-B loads
    for (int j = 0; j < 4; ++j) a.r[a.n][j] = r[j];
    a.nstrip[a.n] = (r[1] + wout - 1) / wout;
    a.wstart[a.n + 1] = a.wstart[a.n] + a.nstrip[a.n] * ((r[3] + a.seg - 1) / a.seg);
    ++a.n;
  }
  if (a.n == 0) return 0;
  for (int k = a.n + 1; k <= 4; ++k) a.wstart[k] = a.wstart[a.n];
  const int64_t waves = a.wstart[a.n];
  const int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned g = grid_1d(nb);
  const int occ = (seg >> 16) & 0xf;  // waves-per-SIMD hint (0 = per-K default)
  bool ok = true;
#define GMT_PIPE(KK, OO) jacobi5pipe_kernel<KK, OO><<<g, kBlock, 0, s>>>(a, u, un, ld, nb)
  switch (nsweeps) {
    case 2: GMT_PIPE(2, 1); break;
    case 4: if (occ == 4) GMT_PIPE(4, 4); else GMT_PIPE(4, 1); break;
    case 6: if (occ == 3) GMT_PIPE(6, 3); else if (occ == 4) GMT_PIPE(6, 4); else GMT_PIPE(6, 1); break;
    default:
      if (occ == 3) GMT_PIPE(8, 3); else if (occ == 4) GMT_PIPE(8, 4); else GMT_PIPE(8, 1);
      break;
  }
#undef GMT_PIPE
  (void)ok;
  GMT_RET_LAUNCH();
}
