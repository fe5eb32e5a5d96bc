// 2-D 5-point Jacobi sweep (fp64), hand-written for gfx950.
//
// This is the BASELINE.json "5-pt Jacobi" workload (an extension: the
// reference's 2-D kernels are the derivative stencils of stencil5.hip).
//   un[y][x] = c0*((u[y][x-1] + u[y][x+1]) + (u[y-1][x] + u[y+1][x])) + c1*f[y][x]
//
// Roofline: 8 B read + 8 B written per point => 16 B/pt.
//
// jacobi5_pt: one output pair per thread, 64 x 4 threads per block (128
// columns x 4 rows), nontemporal stores of un.  Measured on MI355X
// (profiles/r01_sweep2.md): 3.03 ms for 32768^2 = 5.68 TB/s effective vs
// 3.38 ms for a register sliding window.  The vertical reuse (rows y-1, y+1
// read by the threads of the neighbouring rows) is served by L2 because the
// XCD swizzle keeps vertically adjacent tiles on one XCD.  The sliding-window,
// LDS-tiled and lane-exchange variants it was chosen against live in
// csrc/bench/variant_bench.hip.  jacobi5_scalar: odd alignment and the
// frame rects.  Multi-sweep passes: jacobi5tb.hip.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

// Loads of u stay default-policy (nt loads cost 20% here: they would evict
// the rows the next tile row re-reads).
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
  const int64_t c = (nx * ny + kBlock - 1) / kBlock, d = pt_blocks(nx, ny, &nbx);
  return 1 + (c > d ? c : d) + kL2;
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
  const bool vec_ok = aligned16(u) && aligned16(un) && (ld % 2 == 0) && (x0 % 2 == 0) &&
                      (!has_f || (aligned16(f) && ldf % 2 == 0));
  double* partial = want_r ? resid + 1 : nullptr;
  int64_t nb;
  if (vec_ok) {
    int64_t nbx;
    nb = pt_blocks(nx, ny, &nbx);
#define GMT_J9(HF, RS)                                                                     \
  jacobi5_pt<HF, RS><<<grid_1d(nb), kBlock, 0, s>>>(x0, nx, y0, ny, u, un, ld, f, ldf, c0, \
                                                    c1, partial, nbx, nb)
    if (has_f) { if (want_r) GMT_J9(true, true); else GMT_J9(true, false); }
    else { if (want_r) GMT_J9(false, true); else GMT_J9(false, false); }
#undef GMT_J9
  } else {
    const int64_t rect[4] = {x0, nx, y0, ny};
    Rects rs = make_rects(1, rect);
    nb = (nx * ny + kBlock - 1) / kBlock;
#define GMT_J3(HF, RS) \
  jacobi5_scalar<HF, RS><<<grid_1d(nb), kBlock, 0, s>>>(rs, u, un, ld, f, ldf, c0, c1, partial)
    if (has_f) { if (want_r) GMT_J3(true, true); else GMT_J3(true, false); }
    else { if (want_r) GMT_J3(false, true); else GMT_J3(false, false); }
#undef GMT_J3
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
