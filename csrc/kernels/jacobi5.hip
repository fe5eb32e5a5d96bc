// 2-D 5-point Jacobi sweep (fp64), hand-written for gfx950.
//
// This is the BASELINE.json "5-pt Jacobi" workload (an extension: the
// reference's 2-D kernels are the derivative stencils of stencil5.hip).
//   un[y][x] = c0*((u[y][x-1] + u[y][x+1]) + (u[y-1][x] + u[y+1][x])) + c1*f[y][x]
//
// Roofline: 8 B read + 8 B written per point => 16 B/pt; at the measured
// ~6.3 TB/s HBM3E stream rate that is ~390 GLUP/s on one MI355X.
//
// Variant 1 (default) — register sliding window, 2 points per lane:
//   a 256-thread block owns a 512-column x R-row tile and walks it top to
//   bottom; each lane keeps rows y-1, y, y+1 of its two columns in registers
//   (one 16-B global_load_dwordx4 per new row), so HBM sees every input row
//   once per tile (+2 halo rows per R).  The W/E neighbours are the adjacent
//   lanes' values: they come back as 8-B loads that hit the L1 line the wave
//   just fetched, costing L1 bandwidth (~15 B/clk/CU of 64) but no HBM bytes.
//   Tiles are XCD-swizzled so vertically adjacent tiles (which share halo
//   rows) sit on the same XCD L2.
// Variant 2 — LDS-tiled: the block stages (R+2) x (512+2) of u through LDS
//   once and every lane reads N/S/W/E from LDS (kept for A/B measurement).
// Variant 3 — scalar, one point per lane (reference / odd alignment).
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

static int g_jacobi_variant = 0;  // 0 = auto

constexpr int JR = 32;       // rows per tile (variant 1)
constexpr int JTX = 2 * kBlock;  // columns per tile

template <bool HAS_F, bool RESID>
__global__ __launch_bounds__(kBlock) void jacobi5_reg(int64_t x0, int64_t nx, int64_t y0,
                                                      int64_t ny, const double* __restrict__ u,
                                                      double* __restrict__ un, int64_t ld,
                                                      const double* __restrict__ f,
                                                      int64_t ldf, double c0, double c1,
                                                      double* __restrict__ partial,
                                                      int64_t nbx, int64_t nblocks) {
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t xr = (bx * kBlock + threadIdx.x) * 2;  // relative column
  const int64_t yr0 = by * JR;
  const int64_t rows = (ny - yr0) < JR ? (ny - yr0) : JR;
  double acc = 0.0;
  if (xr < nx) {
    const int64_t x = x0 + xr;
    const int64_t y = y0 + yr0;
    const double* p = u + (y - 1) * ld + x;  // row above the first output row
    double* q = un + y * ld + x;
    const double* pf = HAS_F ? f + y * ldf + x : nullptr;
    if (xr + 1 < nx) {
      d2 n = ld2(p), c = ld2(p + ld);
      auto body = [&](int64_t r) {
        const double* pc = p + (r + 1) * ld;
        const d2 s = ld2(pc + ld);
        const double w = pc[-1], e = pc[2];
        d2 o;
        o.x = c0 * ((w + c.y) + (n.x + s.x));
        o.y = c0 * ((c.x + e) + (n.y + s.y));
        if (HAS_F) o += c1 * ld2(pf + r * ldf);
        if (RESID) {
          const d2 d = o - c;
          acc += d.x * d.x + d.y * d.y;
        }
        st2(q + r * ld, o);
        n = c;
        c = s;
      };
      if (rows == JR) {
#pragma unroll 4
        for (int r = 0; r < JR; ++r) body(r);
      } else {
        for (int64_t r = 0; r < rows; ++r) body(r);
      }
    } else {  // odd last column of the region
      for (int64_t r = 0; r < rows; ++r) {
        const double* pc = p + (r + 1) * ld;
        double o = c0 * ((pc[-1] + pc[1]) + (pc[-ld] + pc[ld]));
        if (HAS_F) o += c1 * pf[r * ldf];
        if (RESID) acc += (o - pc[0]) * (o - pc[0]);
        q[r * ld] = o;
      }
    }
  }
  if (RESID) {
    acc = block_sum(acc);
    if (threadIdx.x == 0) partial[blockIdx.x] = acc;
  }
}


// Variants 4-8 — register sliding window where the W/E neighbours come from
// the adjacent LANES instead of a second and third (L1-served) global load:
// lane t holds columns 2t, 2t+1, so west of 2t is lane t-1's .y and east of
// 2t+1 is lane t+1's .x.  XCHG = 1 uses DPP wave_shr/wave_shl (a VALU
// modifier, no LDS traffic), XCHG = 2 uses __shfl (ds_bpermute), XCHG = 0
// keeps the L1 loads.  Only the two wave-edge lanes load a neighbour from
// memory.  R rows per tile; NTS = nontemporal stores of un (streamed out,
// not re-read before the next step).  Requires an even region width.
template <int R, int XCHG, bool NTS>
__global__ __launch_bounds__(kBlock) void jacobi5_lane(int64_t x0, int64_t nx, int64_t y0,
                                                       int64_t ny, const double* __restrict__ u,
                                                       double* __restrict__ un, int64_t ld,
                                                       int64_t nbx, int64_t nblocks) {
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t bx = t % nbx, by = t / nbx;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t xr = (bx * kBlock + threadIdx.x) * 2;  // relative column (nx is even)
  const bool active = xr < nx;
  const bool edge_lo = lane == 0;
  const bool edge_hi = lane == kWave - 1 || xr + 2 >= nx;
  const int64_t yr0 = by * R;
  const int64_t rows = (ny - yr0) < R ? (ny - yr0) : R;
  const int64_t x = x0 + (active ? xr : 0);
  const double* p = u + (y0 + yr0 - 1) * ld + x;  // row above the first output row
  double* q = un + (y0 + yr0) * ld + x;
  d2 n = active ? ld2(p) : d2{0.0, 0.0};
  d2 c = active ? ld2(p + ld) : d2{0.0, 0.0};
  auto body = [&](int64_t r) {
    const double* pc = p + (r + 1) * ld;
    const d2 s = active ? ld2(pc + ld) : d2{0.0, 0.0};
    double w, e;
    if (XCHG == 0) {
      w = active ? pc[-1] : 0.0;
      e = active ? pc[2] : 0.0;
    } else {
      w = XCHG == 1 ? dpp_from_lower(c.y) : __shfl_up(c.y, 1, kWave);
      e = XCHG == 1 ? dpp_from_upper(c.x) : __shfl_down(c.x, 1, kWave);
      if (active && edge_lo) w = pc[-1];
      if (active && edge_hi) e = pc[2];
    }
    if (active) {
      d2 o;
      o.x = 0.25 * ((w + c.y) + (n.x + s.x));
      o.y = 0.25 * ((c.x + e) + (n.y + s.y));
      if (NTS)
        st2_nt(q + r * ld, o);
      else
        st2(q + r * ld, o);
    }
    n = c;
    c = s;
  };
  if (rows == R) {
#pragma unroll 4
    for (int r = 0; r < R; ++r) body(r);
  } else {
    for (int64_t r = 0; r < rows; ++r) body(r);
  }
}


// Variant 9 (default) — one output pair per thread, 64 x 4 threads per block
// (128 columns x 4 rows), nontemporal stores of un.  Measured on MI355X
// (profiles/r01_sweep2.md): 3.03 ms for 32768^2 = 5.68 TB/s effective vs
// 3.38 ms for the register sliding window (v1).  Every thread is short-lived
// like a streaming copy; the vertical reuse (rows y-1, y+1 read by the
// threads of the neighbouring rows) is served by L2 because the XCD swizzle
// keeps vertically adjacent tiles on one XCD, so HBM still sees each input
// byte ~once.  Loads of u stay default-policy (nt loads cost 20% here: they
// would evict the rows the next tile row re-reads).
template <bool HAS_F, bool RESID>
__global__ __launch_bounds__(kBlock) void jacobi5_pt(int64_t x0, int64_t nx, int64_t y0,
                                                     int64_t ny, const double* __restrict__ u,
                                                     double* __restrict__ un, int64_t ld,
                                                     const double* __restrict__ f, int64_t ldf,
                                                     double c0, double c1,
                                                     double* __restrict__ partial, int64_t nbx,
                                                     int64_t nblocks) {
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t xr = (bx * kWave + (threadIdx.x & (kWave - 1))) * 2;
  const int64_t yr = by * (kBlock / kWave) + (threadIdx.x / kWave);
  double acc = 0.0;
  if (xr < nx && yr < ny) {
    const int64_t x = x0 + xr, y = y0 + yr;
    const double* pc = u + y * ld + x;
    if (xr + 1 < nx) {
      const d2 c = ld2(pc), n = ld2(pc - ld), s = ld2(pc + ld);
      const double w = pc[-1], e = pc[2];
      d2 o;
      o.x = c0 * ((w + c.y) + (n.x + s.x));
      o.y = c0 * ((c.x + e) + (n.y + s.y));
      if (HAS_F) o += c1 * ld2(f + y * ldf + x);
      if (RESID) {
        const d2 d = o - c;
        acc = d.x * d.x + d.y * d.y;
      }
      st2_nt(un + y * ld + x, o);
    } else {  // odd last column of the region
      double o = c0 * ((pc[-1] + pc[1]) + (pc[-ld] + pc[ld]));
      if (HAS_F) o += c1 * f[y * ldf + x];
      if (RESID) acc = (o - pc[0]) * (o - pc[0]);
      un[y * ld + x] = o;
    }
  }
  if (RESID) {
    acc = block_sum(acc);
    if (threadIdx.x == 0) partial[blockIdx.x] = acc;
  }
}

// LDS-tiled variant: stage (LR+2) rows x (JTX+2) columns of u, then compute.
constexpr int LR = 16;
template <bool HAS_F, bool RESID>
__global__ __launch_bounds__(kBlock) void jacobi5_lds(int64_t x0, int64_t nx, int64_t y0,
                                                      int64_t ny, const double* __restrict__ u,
                                                      double* __restrict__ un, int64_t ld,
                                                      const double* __restrict__ f,
                                                      int64_t ldf, double c0, double c1,
                                                      double* __restrict__ partial,
                                                      int64_t nbx, int64_t nblocks) {
  // +2 halo columns, padded by 2 doubles so that rows start 16-B aligned and
  // consecutive rows shift banks (row pitch 516 doubles = 4128 B).
  constexpr int P = JTX + 4;
  __shared__ double tile[(LR + 2) * P];
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t xr0 = bx * JTX, yr0 = by * LR;
  const int64_t cols = (nx - xr0) < JTX ? (nx - xr0) : JTX;
  const int64_t rows = (ny - yr0) < LR ? (ny - yr0) : LR;
  const int64_t gx = x0 + xr0, gy = y0 + yr0;
  // Stage: tile[r][c+1] = u[gy-1+r][gx+c] for c in [-1, cols], r in [0, rows+1].
  const int tid = threadIdx.x;
  for (int r = 0; r < rows + 2; ++r) {
    const double* src = u + (gy - 1 + r) * ld + gx;
    double* dst = tile + r * P + 2;  // element c lives at dst[c]; c=-1 at dst[-1]
    const int c = 2 * tid;
    if (c + 1 < cols) {
      st2(dst + c, ld2(src + c));
    } else if (c < cols) {
      dst[c] = src[c];
    }
    if (tid == 0) dst[-1] = src[-1];
    if (tid == 1) dst[cols] = src[cols];
  }
  __syncthreads();
  double acc = 0.0;
  const int c = 2 * tid;
  if (c < cols) {
    for (int r = 1; r <= rows; ++r) {
      const double* row = tile + r * P + 2;
      const int64_t gyr = gy - 1 + r;
      if (c + 1 < cols) {
        const d2 ce = *reinterpret_cast<const d2*>(row + c);
        const d2 nn = *reinterpret_cast<const d2*>(row - P + c);
        const d2 ss = *reinterpret_cast<const d2*>(row + P + c);
        const double w = row[c - 1], e = row[c + 2];
        d2 o;
        o.x = c0 * ((w + ce.y) + (nn.x + ss.x));
        o.y = c0 * ((ce.x + e) + (nn.y + ss.y));
        if (HAS_F) o += c1 * ld2(f + gyr * ldf + gx + c);
        if (RESID) {
          const d2 d = o - ce;
          acc += d.x * d.x + d.y * d.y;
        }
        st2(un + gyr * ld + gx + c, o);
      } else {
        double o = c0 * ((row[c - 1] + row[c + 1]) + (row[c - P] + row[c + P]));
        if (HAS_F) o += c1 * f[gyr * ldf + gx + c];
        if (RESID) acc += (o - row[c]) * (o - row[c]);
        un[gyr * ld + gx + c] = o;
      }
    }
  }
  if (RESID) {
    acc = block_sum(acc);
    if (threadIdx.x == 0) partial[blockIdx.x] = acc;
  }
}

struct Rects {
  int64_t r[4][4];   // x0, nx, y0, ny
  int64_t start[5];  // prefix sum of points
  int n;
};

template <bool HAS_F, bool RESID>
__global__ __launch_bounds__(kBlock) void jacobi5_scalar(Rects rs, const double* __restrict__ u,
                                                         double* __restrict__ un, int64_t ld,
                                                         const double* __restrict__ f,
                                                         int64_t ldf, double c0, double c1,
                                                         double* __restrict__ partial) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  double acc = 0.0;
  if (i < rs.start[rs.n]) {
    int k = 0;
    while (k + 1 < rs.n && i >= rs.start[k + 1]) ++k;
    const int64_t li = i - rs.start[k];
    const int64_t nxk = rs.r[k][1];
    const int64_t x = rs.r[k][0] + li % nxk, y = rs.r[k][2] + li / nxk;
    const double* pc = u + y * ld + x;
    double o = c0 * ((pc[-1] + pc[1]) + (pc[-ld] + pc[ld]));
    if (HAS_F) o += c1 * f[y * ldf + x];
    if (RESID) acc = (o - pc[0]) * (o - pc[0]);
    un[y * ld + x] = o;
  }
  if (RESID) {
    acc = block_sum(acc);
    if (threadIdx.x == 0) partial[blockIdx.x] = acc;
  }
}

// Deterministic reduction of per-block partials: level 1 sums contiguous
// chunks with up to kL2 blocks, level 2 (one block) sums those.  The
// summation order depends only on n, so results are run-to-run identical.
constexpr int64_t kL2 = 1024;
__global__ __launch_bounds__(kBlock) void sum_chunks(const double* __restrict__ partial, int64_t n,
                                                     int64_t chunk, double* __restrict__ out) {
  const int64_t lo = blockIdx.x * chunk, hi = (lo + chunk) < n ? (lo + chunk) : n;
  double acc = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) acc += partial[i];
  acc = block_sum(acc);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void sum_partials(const double* __restrict__ partial,
                                                       int64_t n, double* __restrict__ out) {
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) acc += partial[i];
  acc = block_sum(acc);
  if (threadIdx.x == 0) out[0] = acc;
}

template <bool HAS_F, bool RESID, typename... A>
static void launch_variant(int v, unsigned nb, hipStream_t s, A... args) {
  if (v == 2)
    jacobi5_lds<HAS_F, RESID><<<nb, kBlock, 0, s>>>(args...);
  else
    jacobi5_reg<HAS_F, RESID><<<nb, kBlock, 0, s>>>(args...);
}

static int64_t tiled_blocks(int v, int64_t nx, int64_t ny, int64_t* nbx) {
  const int64_t rr = (v == 2) ? LR : JR;
  *nbx = (nx + JTX - 1) / JTX;
  return *nbx * ((ny + rr - 1) / rr);
}

static Rects make_rects(int n, const int64_t* rects) {
  Rects rs{};
  rs.n = 0;
  rs.start[0] = 0;
  for (int k = 0; k < n && k < 4; ++k) {
    const int64_t nx = rects[4 * k + 1], ny = rects[4 * k + 3];
    if (nx <= 0 || ny <= 0) continue;
    for (int j = 0; j < 4; ++j) rs.r[rs.n][j] = rects[4 * k + j];
    rs.start[rs.n + 1] = rs.start[rs.n] + nx * ny;
    ++rs.n;
  }
  return rs;
}

}  // namespace gmt

extern "C" void gmt_jacobi5_set_variant(int v) { gmt::g_jacobi_variant = v; }
extern "C" int gmt_jacobi5_get_variant(void) { return gmt::g_jacobi_variant; }

namespace gmt {
static int64_t pt_blocks(int64_t nx, int64_t ny, int64_t* nbx) {
  *nbx = (nx + 2 * kWave - 1) / (2 * kWave);
  return *nbx * ((ny + kBlock / kWave - 1) / (kBlock / kWave));
}
}  // namespace gmt

// resid buffer layout: [0] result | [1, 1+nb) per-block partials | kL2 level-2 slots
extern "C" int64_t gmt_jacobi_resid_workspace(int64_t nx, int64_t ny) {
  using namespace gmt;
  int64_t nbx;
  const int64_t a = tiled_blocks(1, nx, ny, &nbx), b = tiled_blocks(2, nx, ny, &nbx);
  const int64_t c = (nx * ny + kBlock - 1) / kBlock, d = pt_blocks(nx, ny, &nbx);
  int64_t m = a > b ? a : b;
  m = m > c ? m : c;
  m = m > d ? m : d;
  return 1 + m + kL2;
}

namespace gmt {
static void reduce_partials(const double* partial, int64_t nb, double* out, hipStream_t s) {
  if (nb <= 4 * kBlock) {
    sum_partials<<<1, kBlock, 0, s>>>(partial, nb, out);
    return;
  }
  const int64_t nb2 = nb < kL2 ? nb : kL2;
  const int64_t chunk = (nb + nb2 - 1) / nb2;
  const int64_t used = (nb + chunk - 1) / chunk;
  double* l2 = const_cast<double*>(partial) + nb;
  sum_chunks<<<grid_1d(used), kBlock, 0, s>>>(partial, nb, chunk, l2);
  sum_partials<<<1, kBlock, 0, s>>>(l2, used, out);
}
}  // namespace gmt

extern "C" int gmt_jacobi5(int64_t x0, int64_t nx, int64_t y0, int64_t ny, const double* u,
                           double* un, int64_t ld, const double* f, int64_t ldf, double c0,
                           double c1, double* resid, void* stream) {
  using namespace gmt;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nx <= 0 || ny <= 0) {
    if (resid) return static_cast<int>(hipMemsetAsync(resid, 0, sizeof(double), s));
    return 0;
  }
  const bool has_f = f != nullptr;
  const bool want_r = resid != nullptr;
  int v = g_jacobi_variant;
  const bool vec_ok = aligned16(u) && aligned16(un) && (ld % 2 == 0) && (x0 % 2 == 0) &&
                      (!has_f || (aligned16(f) && ldf % 2 == 0));
  if (v == 0) v = 9;
  if (!vec_ok) v = 3;
  double* partial = want_r ? resid + 1 : nullptr;
  int64_t nb;
  if (v >= 4 && v <= 8 && !has_f && !want_r && nx % 2 == 0 && c0 == 0.25) {
    const int rr = (v == 6 || v == 7) ? 64 : (v == 8 ? 128 : 32);
    const int64_t nbx = (nx + JTX - 1) / JTX;
    nb = nbx * ((ny + rr - 1) / rr);
    const unsigned g = grid_1d(nb);
    switch (v) {
      case 4: jacobi5_lane<32, 1, false><<<g, kBlock, 0, s>>>(x0, nx, y0, ny, u, un, ld, nbx, nb); break;
      case 5: jacobi5_lane<32, 2, false><<<g, kBlock, 0, s>>>(x0, nx, y0, ny, u, un, ld, nbx, nb); break;
      case 6: jacobi5_lane<64, 1, true><<<g, kBlock, 0, s>>>(x0, nx, y0, ny, u, un, ld, nbx, nb); break;
      case 7: jacobi5_lane<64, 0, true><<<g, kBlock, 0, s>>>(x0, nx, y0, ny, u, un, ld, nbx, nb); break;
      default: jacobi5_lane<128, 1, true><<<g, kBlock, 0, s>>>(x0, nx, y0, ny, u, un, ld, nbx, nb); break;
    }
    GMT_RET_LAUNCH();
  }
  if (v == 9) {
    int64_t nbx;
    nb = pt_blocks(nx, ny, &nbx);
#define GMT_J9(HF, RS)                                                                     \
  jacobi5_pt<HF, RS><<<grid_1d(nb), kBlock, 0, s>>>(x0, nx, y0, ny, u, un, ld, f, ldf, c0, \
                                                    c1, partial, nbx, nb)
    if (has_f) { if (want_r) GMT_J9(true, true); else GMT_J9(true, false); }
    else { if (want_r) GMT_J9(false, true); else GMT_J9(false, false); }
#undef GMT_J9
    if (want_r) reduce_partials(partial, nb, resid, s);
    GMT_RET_LAUNCH();
  }
  if (v >= 4) v = 1;
  if (v == 3) {
    const int64_t rect[4] = {x0, nx, y0, ny};
    Rects rs = make_rects(1, rect);
    nb = (nx * ny + kBlock - 1) / kBlock;
#define GMT_J3(HF, RS) \
  jacobi5_scalar<HF, RS><<<grid_1d(nb), kBlock, 0, s>>>(rs, u, un, ld, f, ldf, c0, c1, partial)
    if (has_f) { if (want_r) GMT_J3(true, true); else GMT_J3(true, false); }
    else { if (want_r) GMT_J3(false, true); else GMT_J3(false, false); }
#undef GMT_J3
  } else {
    int64_t nbx;
    nb = tiled_blocks(v, nx, ny, &nbx);
#define GMT_JV(HF, RS) \
  launch_variant<HF, RS>(v, grid_1d(nb), s, x0, nx, y0, ny, u, un, ld, f, ldf, c0, c1, partial, nbx, nb)
    if (has_f) { if (want_r) GMT_JV(true, true); else GMT_JV(true, false); }
    else { if (want_r) GMT_JV(false, true); else GMT_JV(false, false); }
#undef GMT_JV
  }
  if (want_r) reduce_partials(partial, nb, resid, s);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_jacobi5_rects(int n_rect, const int64_t* rects, const double* u, double* un,
                                 int64_t ld, const double* f, int64_t ldf, double c0, double c1,
                                 void* stream) {
  using namespace gmt;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n_rect > 4) return static_cast<int>(hipErrorInvalidValue);
  Rects rs = make_rects(n_rect, rects);
  if (rs.n == 0) return 0;
  const int64_t nb = (rs.start[rs.n] + kBlock - 1) / kBlock;
  if (f)
    jacobi5_scalar<true, false><<<grid_1d(nb), kBlock, 0, s>>>(rs, u, un, ld, f, ldf, c0, c1, nullptr);
  else
    jacobi5_scalar<false, false><<<grid_1d(nb), kBlock, 0, s>>>(rs, u, un, ld, f, ldf, c0, c1, nullptr);
  GMT_RET_LAUNCH();
}
