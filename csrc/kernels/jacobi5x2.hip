// Two fused 5-point Jacobi sweeps per memory pass (temporal blocking), gfx950.
//
// A single sweep is HBM-bound at 16 B per lattice update (read u, write un);
// the best single-sweep kernel runs at ~5.6 TB/s effective (jacobi5.hip v9).
// Fusing two sweeps reads u(t) once and writes u(t+2) once: 8 B per update,
// so the same bandwidth gives ~2x the lattice-update rate.  Results are
// bitwise identical to two single sweeps (same arithmetic, same order).
//
// Per workgroup (256 threads): an output tile of TX x TY points.
//   1. stage u(t) on the tile + 2-cell ring into LDS (16-B loads, rows of
//      TX + 4 doubles; reuse between neighbouring tiles is served by L2 —
//      tiles are XCD-swizzled so vertical neighbours share an XCD);
//   2. compute u(t+1) on the tile + 1-cell ring into a second LDS tile; a
//      ring cell outside the rank's interior is updated only if that side's
//      ghost cells belong to a neighbour (halo_mask), otherwise it is a fixed
//      Dirichlet ghost and keeps its value;
//   3. compute u(t+2) on the tile from LDS and stream it out with
//      nontemporal 16-B stores.
// The caller guarantees u(t) is valid on the output rect + 2 cells (ghost
// width 2, corners included when both dimensions are decomposed).
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

struct X2Args {
  int64_t r[4][4];       // output rects: x0, nx, y0, ny (absolute array coordinates)
  int64_t ntx[4];        // tiles per rect row
  int64_t tstart[5];     // prefix sum of tiles
  int64_t dom[4];        // interior: x0, nx, y0, ny (absolute)
  int n;
  int mask;              // bit0 west, bit1 east, bit2 south, bit3 north: ghost cells are real
};

template <int X2_TX, int TY>
__global__ __launch_bounds__(kBlock) void jacobi5x2_kernel(X2Args a, const double* __restrict__ u,
                                                           double* __restrict__ un, int64_t ld,
                                                           int64_t nblocks) {
  constexpr int AP = X2_TX + 4;  // LDS row pitch (doubles)
  constexpr int AR = TY + 4;
  __shared__ __attribute__((aligned(16))) double A[AR * AP];
  __shared__ __attribute__((aligned(16))) double B[AR * AP];

  const int64_t bid = xcd_swizzle(blockIdx.x, nblocks);
  int k = 0;
  while (k + 1 < a.n && bid >= a.tstart[k + 1]) ++k;
  const int64_t lt = bid - a.tstart[k];
  const int64_t ox = a.r[k][0] + (lt % a.ntx[k]) * X2_TX;
  const int64_t oy = a.r[k][2] + (lt / a.ntx[k]) * TY;
  const int64_t w = (a.r[k][0] + a.r[k][1] - ox) < X2_TX ? (a.r[k][0] + a.r[k][1] - ox) : X2_TX;
  const int64_t h = (a.r[k][2] + a.r[k][3] - oy) < TY ? (a.r[k][2] + a.r[k][3] - oy) : TY;
  const int64_t dx0 = a.dom[0], dx1 = a.dom[0] + a.dom[1], dy0 = a.dom[2], dy1 = a.dom[3] + a.dom[2];
  const int tid = threadIdx.x;

  // 1. stage u(t) on [ox-2, ox+w+2) x [oy-2, oy+h+2) (clamped to the stored ring)
  const int64_t xa = ox - 2, ya = oy - 2;
  const int pairs = static_cast<int>((w + 4 + 1) / 2);
  const int64_t xlim = dx1 + 2, ylim = dy1 + 2;
  for (int i = tid; i < (h + 4) * pairs; i += kBlock) {
    const int rr = i / pairs, cp = i - rr * pairs;
    const int64_t y = ya + rr, x = xa + 2 * cp;
    d2 v = {0.0, 0.0};
    if (y < ylim) {
      const double* p = u + y * ld + x;
      if (x + 1 < xlim)
        v = ld2(p);
      else if (x < xlim)
        v.x = p[0];
    }
    *reinterpret_cast<d2*>(&A[rr * AP + 2 * cp]) = v;
  }
  __syncthreads();

  // 2. u(t+1) on the tile + 1-cell ring
  const bool gw = a.mask & 1, ge = a.mask & 2, gs = a.mask & 4, gn = a.mask & 8;
  const int bw = static_cast<int>(w + 2);
  for (int i = tid; i < (h + 2) * bw; i += kBlock) {
    const int yy = 1 + i / bw, xx = 1 + i % bw;
    const int64_t y = ya + yy, x = xa + xx;
    const bool rx = (x >= dx0 && x < dx1) || (x < dx0 ? gw : ge);
    const bool ry = (y >= dy0 && y < dy1) || (y < dy0 ? gs : gn);
    const double* c = &A[yy * AP + xx];
    B[yy * AP + xx] = (rx && ry) ? 0.25 * ((c[-1] + c[1]) + (c[-AP] + c[AP])) : c[0];
  }
  __syncthreads();

  // 3. u(t+2) on the tile, 16-B nontemporal stores (ox even, ld even)
  const int wp = static_cast<int>((w + 1) / 2);
  for (int i = tid; i < h * wp; i += kBlock) {
    const int yy = 2 + i / wp, xx = 2 + 2 * (i % wp);
    const double* c = &B[yy * AP + xx];
    double* q = un + (ya + yy) * ld + xa + xx;
    const double o0 = 0.25 * ((c[-1] + c[1]) + (c[-AP] + c[AP]));
    if (xx + 1 < w + 2) {
      d2 o;
      o.x = o0;
      o.y = 0.25 * ((c[0] + c[2]) + (c[1 - AP] + c[1 + AP]));
      st2_nt(q, o);
    } else {
      q[0] = o0;
    }
  }
}

}  // namespace gmt

namespace gmt {
// tile = (TX << 16) | TY; 0 = default.  Measured on 1x MI355X, two sweeps of
// 32768^2 (profiles/r01_x2_tiles.md): 64x16 3.77 ms, 128x8 4.50, 64x8 4.67,
// 128x4 5.31, 128x16 6.06, 256x8 6.37, 64x4 7.30 — the LDS footprint (two
// (TY+4) x (TX+4) fp64 tiles) sets the workgroups per CU, the ring sets the
// redundant loads: 64 x 16 balances both (22 KB, 7 workgroups per CU).
struct X2Tile {
  int tx, ty;
};
static X2Tile x2_tile(int tile) {
  X2Tile t{64, 16};
  if (tile > 0) {
    t.tx = tile >> 16;
    t.ty = tile & 0xffff;
    if (tile < 0x10000) t.tx = 128;  // plain row count: 128-column tiles
  }
  const bool ok = (t.tx == 32 && (t.ty == 16 || t.ty == 32)) ||
                  (t.tx == 64 && (t.ty == 4 || t.ty == 8 || t.ty == 16 || t.ty == 24 || t.ty == 32)) ||
                  (t.tx == 128 && (t.ty == 4 || t.ty == 8 || t.ty == 16 || t.ty == 32)) ||
                  (t.tx == 256 && (t.ty == 4 || t.ty == 8));
  if (!ok) t = {64, 16};
  return t;
}
}  // namespace gmt

extern "C" int gmt_jacobi5x2(int n_rect, const int64_t* rects, const int64_t* dom, int halo_mask,
                             const double* u, double* un, int64_t ld, int tile, void* stream) {
  using namespace gmt;
  if (n_rect < 0 || n_rect > 4) return static_cast<int>(hipErrorInvalidValue);
  if (!aligned16(u) || !aligned16(un) || (ld % 2) != 0) return static_cast<int>(hipErrorInvalidValue);
  const X2Tile tl = x2_tile(tile);
  const int ty = tl.ty, X2_TX = tl.tx;
  X2Args a{};
  a.n = 0;
  a.tstart[0] = 0;
  for (int j = 0; j < 4; ++j) a.dom[j] = dom[j];
  a.mask = halo_mask;
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    if ((r[0] % 2) != 0) return static_cast<int>(hipErrorInvalidValue);  // 16-B staging
    for (int j = 0; j < 4; ++j) a.r[a.n][j] = r[j];
    a.ntx[a.n] = (r[1] + X2_TX - 1) / X2_TX;
    a.tstart[a.n + 1] = a.tstart[a.n] + a.ntx[a.n] * ((r[3] + ty - 1) / ty);
    ++a.n;
  }
  if (a.n == 0) return 0;
  for (int k = a.n + 1; k <= 4; ++k) a.tstart[k] = a.tstart[a.n];
  const int64_t nb = a.tstart[a.n];
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned g = grid_1d(nb);
#define GMT_X2(TX, TY) \
  if (X2_TX == TX && ty == TY) jacobi5x2_kernel<TX, TY><<<g, kBlock, 0, s>>>(a, u, un, ld, nb)
  GMT_X2(32, 16); else GMT_X2(32, 32);
  else GMT_X2(64, 4); else GMT_X2(64, 8); else GMT_X2(64, 16); else GMT_X2(64, 24); else GMT_X2(64, 32);
  else GMT_X2(128, 4); else GMT_X2(128, 8); else GMT_X2(128, 16); else GMT_X2(128, 32);
  else GMT_X2(256, 4); else GMT_X2(256, 8);
#undef GMT_X2
  GMT_RET_LAUNCH();
}
