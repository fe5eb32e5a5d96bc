// K fused 5-point Jacobi sweeps per memory pass (temporal blocking), gfx950.
//
// A single sweep is HBM-bound at 16 B per lattice update (read u, write un);
// the best single-sweep kernel runs at ~5.6-5.8 TB/s effective (jacobi5.hip
// v9).  Fusing K sweeps reads u(t) once and writes u(t+K) once: 16/K B per
// update.  Results are bitwise identical to K single sweeps (same arithmetic,
// same order).
//
// Per workgroup (256 threads): an output tile of TX x TY points.
//   1. stage u(t) on the tile + K-cell ring into LDS (16-B loads from an even
//      column, so the staged ring is KA = K rounded up to even columns wide in
//      x; reuse between neighbouring tiles is served by L2 — tiles are
//      XCD-swizzled so vertical neighbours share an XCD);
//   2. phases p = 1..K-1: u(t+p) on the tile + (K-p)-cell ring into the other
//      LDS buffer (ping-pong).  A ring cell outside the rank's interior is
//      updated only if that side's ghost cells belong to a neighbour
//      (halo_mask); otherwise it is a fixed Dirichlet ghost and keeps its value;
//   3. phase K: u(t+K) on the tile, streamed out with nontemporal 16-B stores.
// The caller guarantees u(t) is valid on the output rect + K cells (ghost
// width >= K, corners included when both dimensions are decomposed) and that
// KA columns left of each rect are addressable.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

struct XkArgs {
  int64_t r[4][4];       // output rects: x0, nx, y0, ny (absolute array coordinates)
  int64_t ntx[4];        // tiles per rect row
  int64_t tstart[5];     // prefix sum of tiles
  int64_t dom[4];        // interior: x0, nx, y0, ny (absolute)
  int n;
  int mask;              // bit0 west, bit1 east, bit2 south, bit3 north: ghost cells are real
};

template <int TX, int TY, int K>
__global__ __launch_bounds__(kBlock) void jacobi5xk_kernel(XkArgs a, const double* __restrict__ u,
                                                           double* __restrict__ un, int64_t ld,
                                                           int64_t nblocks) {
  constexpr int KA = (K + 1) & ~1;  // staged ring width in x (even: 16-B loads)
  constexpr int AP = TX + 2 * KA;   // LDS row pitch (doubles)
  constexpr int AR = TY + 2 * K;
  __shared__ __attribute__((aligned(16))) double L[2][AR * AP];

  const int64_t bid = xcd_swizzle(blockIdx.x, nblocks);
  int k = 0;
  while (k + 1 < a.n && bid >= a.tstart[k + 1]) ++k;
  const int64_t lt = bid - a.tstart[k];
  const int64_t ox = a.r[k][0] + (lt % a.ntx[k]) * TX;
  const int64_t oy = a.r[k][2] + (lt / a.ntx[k]) * TY;
  const int w = static_cast<int>((a.r[k][0] + a.r[k][1] - ox) < TX ? (a.r[k][0] + a.r[k][1] - ox) : TX);
  const int h = static_cast<int>((a.r[k][2] + a.r[k][3] - oy) < TY ? (a.r[k][2] + a.r[k][3] - oy) : TY);
  const int64_t dx0 = a.dom[0], dx1 = a.dom[0] + a.dom[1], dy0 = a.dom[2], dy1 = a.dom[3] + a.dom[2];
  const int tid = threadIdx.x;
  // LDS (yy, xx) <-> global (ya + yy, xa + xx)
  const int64_t xa = ox - KA, ya = oy - K;

  // tile-relative (32-bit) interior bounds; a tile whose whole K-ring lies
  // inside the interior needs no ghost-side rule (the common case)
  const int lx0 = static_cast<int>(dx0 - xa), lx1 = static_cast<int>(dx1 - xa);
  const int ly0 = static_cast<int>(dy0 - ya), ly1 = static_cast<int>(dy1 - ya);
  const bool inner = lx0 <= KA - K && lx1 >= KA + w + K && ly0 <= 0 && ly1 >= h + 2 * K;
  const bool full = w == TX && h == TY;

  // 1. stage u(t) on the tile + ring (clamped to the stored ghost ring)
  {
    const int xlim = lx1 + K, ylim = ly1 + K;  // first column / row past the stored ring
    auto stage = [&](int rr, int cp) {
      const int xx = 2 * cp;
      d2 v = {0.0, 0.0};
      if (rr < ylim) {
        const double* p = u + (ya + rr) * ld + xa + xx;
        if (xx + 1 < xlim)
          v = ld2(p);
        else if (xx < xlim)
          v.x = p[0];
      }
      *reinterpret_cast<d2*>(&L[0][rr * AP + xx]) = v;
    };
    if (full) {
      constexpr int PAIRS = AP / 2;  // compile-time divisor
      for (int i = tid; i < AR * PAIRS; i += kBlock) stage(i / PAIRS, i % PAIRS);
    } else {
      const int pairs = (w + 2 * KA + 1) / 2;
      for (int i = tid; i < (h + 2 * K) * pairs; i += kBlock) stage(i / pairs, i % pairs);
    }
  }
  __syncthreads();

  // 2. intermediate time levels, ring shrinking by one cell per sweep
  const bool gw = a.mask & 1, ge = a.mask & 2, gs = a.mask & 4, gn = a.mask & 8;
#pragma unroll
  for (int p = 1; p < K; ++p) {
    const double* S = L[(p - 1) & 1];
    double* D = L[p & 1];
    const int ring = K - p;
    const int x_off = KA - ring, y_off = K - ring;
    auto cell = [&](int yy, int xx, bool rule) {
      const double* c = &S[yy * AP + xx];
      const double v = 0.25 * ((c[-1] + c[1]) + (c[-AP] + c[AP]));
      if (rule) {
        const bool rx = (xx >= lx0 && xx < lx1) || (xx < lx0 ? gw : ge);
        const bool ry = (yy >= ly0 && yy < ly1) || (yy < ly0 ? gs : gn);
        D[yy * AP + xx] = (rx && ry) ? v : c[0];
      } else {
        D[yy * AP + xx] = v;
      }
    };
    if (full) {
      constexpr int BW = TX + 2 * (K - 1);  // widest level; narrower rings skip columns
      const int bw = TX + 2 * ring, bh = TY + 2 * ring;
      if (inner) {
        for (int i = tid; i < bh * BW; i += kBlock) {
          const int r = i / BW, cc = i % BW;
          if (cc < bw) cell(y_off + r, x_off + cc, false);
        }
      } else {
        for (int i = tid; i < bh * BW; i += kBlock) {
          const int r = i / BW, cc = i % BW;
          if (cc < bw) cell(y_off + r, x_off + cc, true);
        }
      }
    } else {
      const int bw = w + 2 * ring, bh = h + 2 * ring;
      for (int i = tid; i < bh * bw; i += kBlock) cell(y_off + i / bw, x_off + i % bw, true);
    }
    __syncthreads();
  }

  // 3. u(t+K) on the tile, 16-B nontemporal stores (ox even, ld even)
  const double* S = L[(K - 1) & 1];
  auto out = [&](int r, int cp) {
    const int yy = K + r, xx = KA + 2 * cp;
    const double* c = &S[yy * AP + xx];
    double* q = un + (ya + yy) * ld + xa + xx;
    const double o0 = 0.25 * ((c[-1] + c[1]) + (c[-AP] + c[AP]));
    if (xx + 1 < KA + w) {
      d2 o;
      o.x = o0;
      o.y = 0.25 * ((c[0] + c[2]) + (c[1 - AP] + c[1 + AP]));
      st2_nt(q, o);
    } else {
      q[0] = o0;
    }
  };
  if (full) {
    constexpr int WP = TX / 2;
    for (int i = tid; i < TY * WP; i += kBlock) out(i / WP, i % WP);
  } else {
    const int wp = (w + 1) / 2;
    for (int i = tid; i < h * wp; i += kBlock) out(i / wp, i % wp);
  }
}

// tile = (TX << 16) | TY; 0 = default.  Measured on 1x MI355X, two sweeps of
// 32768^2 (profiles/r01_x2_tiles.md): 64x16 3.77-3.94 ms, 32x32 4.02,
// 64x24 4.26, 128x8 4.50, 64x8 4.67, 64x32 4.90, 128x16 6.06 — the LDS
// footprint (two (TY+2K) x (TX+2KA) fp64 tiles) sets the workgroups per CU,
// the ring sets the redundant loads: 64 x 16 balances both (22 KB at K = 2,
// 7 workgroups per CU).
struct XkTile {
  int tx, ty;
};
static XkTile xk_tile(int tile) {
  XkTile t{64, 16};
  if (tile > 0) {
    t.tx = tile >> 16;
    t.ty = tile & 0xffff;
    if (tile < 0x10000) t.tx = 128;  // plain row count: 128-column tiles
  }
  return t;
}

template <int K>
static bool launch_k(int tx, int ty, unsigned g, hipStream_t s, const XkArgs& a, const double* u,
                     double* un, int64_t ld, int64_t nb) {
#define GMT_XK(TX, TY)                                                  \
  if (tx == TX && ty == TY) {                                           \
    jacobi5xk_kernel<TX, TY, K><<<g, kBlock, 0, s>>>(a, u, un, ld, nb); \
    return true;                                                        \
  }
  GMT_XK(32, 16) GMT_XK(32, 32) GMT_XK(64, 4) GMT_XK(64, 8) GMT_XK(64, 16) GMT_XK(64, 24)
  GMT_XK(64, 32) GMT_XK(128, 4) GMT_XK(128, 8) GMT_XK(128, 16) GMT_XK(128, 32) GMT_XK(256, 4)
  GMT_XK(256, 8)
#undef GMT_XK
  return false;
}

}  // namespace gmt

extern "C" int gmt_jacobi5xk(int nsweeps, int n_rect, const int64_t* rects, const int64_t* dom,
                             int halo_mask, const double* u, double* un, int64_t ld, int tile,
                             void* stream) {
  using namespace gmt;
  if ((tile & GMT_XK_PIPE) || (tile == 0 && nsweeps % 2 == 0))
    return gmt_jacobi5xk_pipe(nsweeps, n_rect, rects, dom, halo_mask, u, un, ld, tile & ~GMT_XK_PIPE, stream);
  if (nsweeps < 2 || nsweeps > 4) return static_cast<int>(hipErrorInvalidValue);
  if (n_rect < 0 || n_rect > 4) return static_cast<int>(hipErrorInvalidValue);
  if (!aligned16(u) || !aligned16(un) || (ld % 2) != 0) return static_cast<int>(hipErrorInvalidValue);
  const XkTile tl = xk_tile(tile);
  XkArgs a{};
  a.n = 0;
  a.tstart[0] = 0;
  for (int j = 0; j < 4; ++j) a.dom[j] = dom[j];
  a.mask = halo_mask;
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    if ((r[0] % 2) != 0) return static_cast<int>(hipErrorInvalidValue);  // 16-B staging
    // the ring left of / above the rect (x side rounded up to even) must exist
    if (r[0] < nsweeps + (nsweeps & 1) || r[2] < nsweeps) return static_cast<int>(hipErrorInvalidValue);
    for (int j = 0; j < 4; ++j) a.r[a.n][j] = r[j];
    a.ntx[a.n] = (r[1] + tl.tx - 1) / tl.tx;
    a.tstart[a.n + 1] = a.tstart[a.n] + a.ntx[a.n] * ((r[3] + tl.ty - 1) / tl.ty);
    ++a.n;
  }
  if (a.n == 0) return 0;
  for (int k = a.n + 1; k <= 4; ++k) a.tstart[k] = a.tstart[a.n];
  const int64_t nb = a.tstart[a.n];
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned g = grid_1d(nb);
  bool ok = false;
  switch (nsweeps) {
    case 2: ok = launch_k<2>(tl.tx, tl.ty, g, s, a, u, un, ld, nb); break;
    case 3: ok = launch_k<3>(tl.tx, tl.ty, g, s, a, u, un, ld, nb); break;
    default: ok = launch_k<4>(tl.tx, tl.ty, g, s, a, u, un, ld, nb); break;
  }
  if (!ok) return static_cast<int>(hipErrorInvalidValue);  // unsupported tile
  GMT_RET_LAUNCH();
}

extern "C" int gmt_jacobi5x2(int n_rect, const int64_t* rects, const int64_t* dom, int halo_mask,
                             const double* u, double* un, int64_t ld, int tile, void* stream) {
  return gmt_jacobi5xk(2, n_rect, rects, dom, halo_mask, u, un, ld, tile, stream);
}
