// K9 axis sums, K10/K12 squared-difference norms, analytic fills — gfx950.
//
// Reference: gt::sum_axis_to (mpi_stencil2d_gt.cc:611,620), host
// gt::sum_squares(h_num - h_act) (mpi_stencil_gt.cc:222,
// mpi_stencil2d_gt.cc:555), the SYCL diff_norm reduction
// (mpi_stencil2d_sycl.cc:165-181) and the host analytic init loops
// (mpi_stencil2d_gt.cc:439-497).
//
// All reductions are two-pass and deterministic: pass 1 writes one partial
// per (tile), pass 2 reduces the partials in a fixed order.  No float atomics
// (run-to-run bit-identical results, which the distributed err-norm checks
// rely on).
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

// ---------------- keep_dim == 0: column sums out[x] = sum_y z[y][x]
// pass 1: block (bx, p) sums rows [p*RC, (p+1)*RC) of 512 columns into
// ws[p][x]; pass 2: out[x] = sum_p ws[p][x] (coalesced over x).
constexpr int64_t kColTargetBlocks = 4096;

__global__ __launch_bounds__(kBlock) void colsum_pass1(int64_t nx, int64_t ny,
                                                       const double* __restrict__ z, int64_t ld,
                                                       double* __restrict__ ws, int64_t nbx,
                                                       int64_t rc, bool vec) {
  const int64_t b = blockIdx.x;
  const int64_t bx = b % nbx, p = b / nbx;
  const int64_t x = (bx * kBlock + threadIdx.x) * 2;
  if (x >= nx) return;
  const int64_t y0 = p * rc;
  const int64_t y1 = (y0 + rc) < ny ? (y0 + rc) : ny;
  if (vec && x + 1 < nx) {
    d2 a0 = {0.0, 0.0}, a1 = {0.0, 0.0};
    int64_t y = y0;
    for (; y + 1 < y1; y += 2) {
      a0 += ld2(z + y * ld + x);
      a1 += ld2(z + (y + 1) * ld + x);
    }
    if (y < y1) a0 += ld2(z + y * ld + x);
    st2(ws + p * nx + x, a0 + a1);
  } else {
    for (int64_t xx = x; xx < x + 2 && xx < nx; ++xx) {
      double a = 0.0;
      for (int64_t y = y0; y < y1; ++y) a += z[y * ld + xx];
      ws[p * nx + xx] = a;
    }
  }
}

__global__ __launch_bounds__(kBlock) void colsum_pass2(int64_t nx, int64_t np,
                                                       const double* __restrict__ ws,
                                                       double* __restrict__ out) {
  const int64_t x = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (x >= nx) return;
  double a = 0.0;
  for (int64_t p = 0; p < np; ++p) a += ws[p * nx + x];
  out[x] = a;
}

// ---------------- keep_dim == 1: row sums out[y] = sum_x z[y][x]
// pass 1: block (c, y) reduces chunk c (CH elements) of row y to ws[y][c];
// pass 2: one wave per row sums its chunks.
constexpr int64_t kRowChunk = 2 * kBlock * 8;  // 4096 doubles per block

__global__ __launch_bounds__(kBlock) void rowsum_pass1(int64_t nx, int64_t ny,
                                                       const double* __restrict__ z, int64_t ld,
                                                       double* __restrict__ ws, int64_t nch,
                                                       bool vec) {
  const int64_t b = blockIdx.x;
  const int64_t c = b % nch, y = b / nch;
  const double* row = z + y * ld;
  const int64_t x0 = c * kRowChunk;
  const int64_t x1 = (x0 + kRowChunk) < nx ? (x0 + kRowChunk) : nx;
  double a = 0.0;
  if (vec) {
    d2 v = {0.0, 0.0};
    for (int64_t x = x0 + 2 * threadIdx.x; x + 1 < x1; x += 2 * kBlock) v += ld2(row + x);
    a = v.x + v.y;
    if (((x1 - x0) & 1) && threadIdx.x == 0) a += row[x1 - 1];
  } else {
    for (int64_t x = x0 + threadIdx.x; x < x1; x += kBlock) a += row[x];
  }
  a = block_sum(a);
  if (threadIdx.x == 0) ws[y * nch + c] = a;
}

__global__ __launch_bounds__(kBlock) void rowsum_pass2(int64_t ny, int64_t nch,
                                                       const double* __restrict__ ws,
                                                       double* __restrict__ out) {
  const int64_t y = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + threadIdx.x / kWave;
  if (y >= ny) return;
  const int lane = threadIdx.x & (kWave - 1);
  double a = 0.0;
  for (int64_t c = lane; c < nch; c += kWave) a += ws[y * nch + c];
  a = wave_sum(a);
  if (lane == 0) out[y] = a;
}

static void col_plan(int64_t nx, int64_t ny, int64_t* nbx, int64_t* np, int64_t* rc) {
  *nbx = (nx + 2 * kBlock - 1) / (2 * kBlock);
  int64_t p = (kColTargetBlocks + *nbx - 1) / *nbx;
  const int64_t max_p = (ny + 15) / 16;  // at least 16 rows per partial
  if (p > max_p) p = max_p;
  if (p < 1) p = 1;
  *rc = (ny + p - 1) / p;
  *np = (ny + *rc - 1) / *rc;
}

// ---------------- sum of squared differences over a 2-D region
constexpr int64_t kDiffTile = 2 * kBlock * 8;

__global__ __launch_bounds__(kBlock) void diffsq_pass1(int64_t nx, int64_t ny,
                                                       const double* __restrict__ a,
                                                       int64_t lda, const double* __restrict__ b,
                                                       int64_t ldb, double* __restrict__ ws,
                                                       int64_t nch, bool vec) {
  const int64_t blk = blockIdx.x;
  const int64_t c = blk % nch, y = blk / nch;
  const int64_t x0 = c * kDiffTile;
  const int64_t x1 = (x0 + kDiffTile) < nx ? (x0 + kDiffTile) : nx;
  const double* pa = a + y * lda;
  const double* pb = b + y * ldb;
  double acc = 0.0;
  if (vec) {
    d2 v = {0.0, 0.0};
    for (int64_t x = x0 + 2 * threadIdx.x; x + 1 < x1; x += 2 * kBlock) {
      const d2 d = ld2(pa + x) - ld2(pb + x);
      v += d * d;
    }
    acc = v.x + v.y;
    if (((x1 - x0) & 1) && threadIdx.x == 0) {
      const double d = pa[x1 - 1] - pb[x1 - 1];
      acc += d * d;
    }
  } else {
    for (int64_t x = x0 + threadIdx.x; x < x1; x += kBlock) {
      const double d = pa[x] - pb[x];
      acc += d * d;
    }
  }
  acc = block_sum(acc);
  if (threadIdx.x == 0) ws[blk] = acc;
}

// ---------------- sum of a contiguous vector (the DAXPY partial sums of
// mpi_daxpy_nvtx.cc:251-268, on the device): a fixed grid streams the
// vector with 16-B loads, one partial per workgroup, then one workgroup
// adds the partials in order — deterministic, one pass over HBM
constexpr int64_t kSumBlocks = 2048;  // 8 per CU: enough bytes in flight for HBM

__global__ __launch_bounds__(kBlock) void sum1d_pass1(int64_t n, const double* __restrict__ x,
                                                      double* __restrict__ ws, bool vec) {
  const int64_t nb = gridDim.x, b = blockIdx.x;
  double acc = 0.0;
  if (vec) {
    d2 a0 = {0.0, 0.0}, a1 = {0.0, 0.0};
    const int64_t n2 = n / 2, stride = nb * kBlock;
    int64_t i = b * kBlock + threadIdx.x;
    for (; i + stride < n2; i += 2 * stride) {
      a0 += ld2_nt(x + 2 * i);
      a1 += ld2_nt(x + 2 * (i + stride));
    }
    if (i < n2) a0 += ld2_nt(x + 2 * i);
    acc = (a0.x + a0.y) + (a1.x + a1.y);
    if ((n & 1) && b == 0 && threadIdx.x == 0) acc += x[n - 1];
  } else {
    for (int64_t i = b * kBlock + threadIdx.x; i < n; i += nb * kBlock) acc += x[i];
  }
  acc = block_sum(acc);
  if (threadIdx.x == 0) ws[b] = acc;
}

// ---------------- out[i] = sum (or max) over r of in[r * n + i], r in order:
// the reduction half of an all-reduce built from an all-gather (the ipc
// transport), the same bits on every rank
__global__ __launch_bounds__(kBlock) void slices_kernel(int op, int64_t n, int ns, const double* __restrict__ in,
                                                        double* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  double v = in[i];
  for (int r = 1; r < ns; ++r) {
    const double w = in[r * n + i];
    v = op == 0 ? v + w : fmax(v, w);
  }
  out[i] = v;
}

// ---------------- max |z| over a 2-D region (the engine's exactness guard on
// a measured field bound); same tiles and workspace as diff_sq
__device__ __forceinline__ double block_max(double v) {
  __shared__ double s_part[kBlock / kWave];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
  if ((threadIdx.x & (kWave - 1)) == 0) s_part[threadIdx.x / kWave] = v;
  __syncthreads();
  double t = s_part[0];
#pragma unroll
  for (int i = 1; i < kBlock / kWave; ++i) t = fmax(t, s_part[i]);
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(kBlock) void absmax_pass1(int64_t nx, int64_t ny, const double* __restrict__ z,
                                                       int64_t ld, double* __restrict__ ws, int64_t nch) {
  const int64_t blk = blockIdx.x;
  const int64_t c = blk % nch, y = blk / nch;
  const int64_t x0 = c * kDiffTile;
  const int64_t x1 = (x0 + kDiffTile) < nx ? (x0 + kDiffTile) : nx;
  const double* p = z + y * ld;
  double m = 0.0;
  for (int64_t x = x0 + threadIdx.x; x < x1; x += kBlock) m = fmax(m, fabs(p[x]));
  m = block_max(m);
  if (threadIdx.x == 0) ws[blk] = m;
}

__global__ __launch_bounds__(kBlock) void max_all(const double* __restrict__ ws, int64_t n,
                                                  double* __restrict__ out) {
  double m = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) m = fmax(m, ws[i]);
  m = block_max(m);
  if (threadIdx.x == 0) out[0] = m;
}

// ---------------- bitwise comparison (gmt_diff_bits): per tile the max
// |a - b| (NaN -> +inf) and the count of elements whose bits differ
__global__ __launch_bounds__(kBlock) void diffbits_pass1(int64_t nx, int64_t ny, const double* __restrict__ a,
                                                         int64_t lda, const double* __restrict__ b, int64_t ldb,
                                                         double* __restrict__ ws, int64_t nch) {
  const int64_t blk = blockIdx.x, nblk = nch * ny;
  const int64_t c = blk % nch, y = blk / nch;
  const int64_t x0 = c * kDiffTile;
  const int64_t x1 = (x0 + kDiffTile) < nx ? (x0 + kDiffTile) : nx;
  const double* pa = a + y * lda;
  const double* pb = b + y * ldb;
  double m = 0.0, n = 0.0;
  for (int64_t x = x0 + threadIdx.x; x < x1; x += kBlock) {
    const double va = pa[x], vb = pb[x];
    if (__double_as_longlong(va) != __double_as_longlong(vb)) {
      n += 1.0;
      const double d = fabs(va - vb);
      m = fmax(m, d != d ? __builtin_inf() : d);
    }
  }
  m = block_max(m);
  n = block_sum(n);
  if (threadIdx.x == 0) {
    ws[blk] = m;
    ws[nblk + blk] = n;
  }
}

// counter-based uniform [0, 1) of an integer lattice point (fill mode 5):
// splitmix64 of the packed global coordinates — the same value whatever the
// decomposition, and reproducible on the host (ops/reference.py)
__device__ __forceinline__ double lattice_uniform(int64_t gx, int64_t gy, uint64_t seed) {
  uint64_t k = (static_cast<uint64_t>(gy + (int64_t(1) << 30)) << 32) ^ static_cast<uint64_t>(gx + (int64_t(1) << 30));
  k ^= seed;
  k += 0x9E3779B97F4A7C15ull;
  k = (k ^ (k >> 30)) * 0xBF58476D1CE4E5B9ull;
  k = (k ^ (k >> 27)) * 0x94D049BB133111EBull;
  k ^= k >> 31;
  return static_cast<double>(k >> 11) * 0x1.0p-53;
}

__global__ __launch_bounds__(kBlock) void sum_all(const double* __restrict__ ws, int64_t n,
                                                  double* __restrict__ out) {
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) acc += ws[i];
  acc = block_sum(acc);
  if (threadIdx.x == 0) out[0] = acc;
}

// ---------------- analytic fills (reference fn / fn_dzdx / fn_dzdy lambdas,
// mpi_stencil2d_gt.cc:431-433)
__global__ __launch_bounds__(kBlock) void fill_poly_kernel(int mode, int64_t nx, int64_t ny,
                                                           double x0, double dx, double y0,
                                                           double dy, double* __restrict__ z,
                                                           int64_t ld) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= nx * ny) return;
  const int64_t ix = i % nx, iy = i / nx;
  double v;
  if (mode == 5) {  // x0, y0: integer global lattice origin; dx: seed
    z[iy * ld + ix] = lattice_uniform(static_cast<int64_t>(x0) + ix, static_cast<int64_t>(y0) + iy,
                                      static_cast<uint64_t>(dx));
    return;
  }
  if (mode == 4) {
    // integer lattice: x = (x0 + ix) * dx with x0 an integer index (exact
    // sum, one rounding) and no fma contraction, so a NumPy reference
    // (x*x*x + y*y on the same lattice) is bitwise equal
#pragma clang fp contract(off)
    const double x = (x0 + static_cast<double>(ix)) * dx, y = (y0 + static_cast<double>(iy)) * dy;
    z[iy * ld + ix] = x * x * x + y * y;
    return;
  }
  const double x = x0 + ix * dx, y = y0 + iy * dy;
  if (mode == 0)
    v = x * x * x + y * y;
  else if (mode == 1)
    v = 3 * x * x;
  else if (mode == 2)
    v = 2 * y;
  else
    v = x;
  z[iy * ld + ix] = v;
}

__global__ __launch_bounds__(kBlock) void poly_check_kernel(int64_t nx, int64_t ny, double x0, double dx,
                                                            double y0, double dy, double offset, double rtol,
                                                            const double* __restrict__ z, int64_t ld,
                                                            unsigned* __restrict__ bad) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  bool wrong = false;
  if (i < nx * ny) {
    const int64_t ix = i % nx, iy = i / nx;
    const double x = x0 + ix * dx, y = y0 + iy * dy;
    const double e = (x * x * x + y * y) + offset;
    const double v = z[iy * ld + ix];
    wrong = !(fabs(v - e) <= rtol * (1.0 + fabs(e)));  // NaN counts as wrong
  }
  // one atomic per wave with a mismatch
  const unsigned long long m = __ballot(wrong);
  if (m && (threadIdx.x & (kWave - 1)) == 0) atomicAdd(bad, static_cast<unsigned>(__popcll(m)));
}

__global__ __launch_bounds__(kBlock) void add_scalar_kernel(int64_t nx, int64_t ny, double v,
                                                            double* __restrict__ z, int64_t ld) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= nx * ny) return;
  z[(i / nx) * ld + i % nx] += v;
}

}  // namespace gmt

extern "C" int64_t gmt_sum_axis_workspace(int keep_dim, int64_t nx, int64_t ny) {
  using namespace gmt;
  if (keep_dim == 0) {
    int64_t nbx, np, rc;
    col_plan(nx, ny, &nbx, &np, &rc);
    return np * nx;
  }
  const int64_t nch = (nx + kRowChunk - 1) / kRowChunk;
  return ny * nch;
}

extern "C" int gmt_sum_axis(int keep_dim, int64_t nx, int64_t ny, const double* z, int64_t ld,
                            double* out, double* ws, void* stream) {
  using namespace gmt;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nx <= 0 || ny <= 0) return 0;
  const bool vec = aligned16(z) && (ld % 2 == 0);
  if (keep_dim == 0) {
    int64_t nbx, np, rc;
    col_plan(nx, ny, &nbx, &np, &rc);
    colsum_pass1<<<grid_1d(nbx * np), kBlock, 0, s>>>(nx, ny, z, ld, ws, nbx, rc,
                                                      vec && aligned16(ws) && nx % 2 == 0);
    colsum_pass2<<<grid_1d((nx + kBlock - 1) / kBlock), kBlock, 0, s>>>(nx, np, ws, out);
  } else if (keep_dim == 1) {
    const int64_t nch = (nx + kRowChunk - 1) / kRowChunk;
    rowsum_pass1<<<grid_1d(nch * ny), kBlock, 0, s>>>(nx, ny, z, ld, ws, nch, vec);
    const int64_t rows_per_block = kBlock / kWave;
    rowsum_pass2<<<grid_1d((ny + rows_per_block - 1) / rows_per_block), kBlock, 0, s>>>(
        ny, nch, ws, out);
  } else {
    return static_cast<int>(hipErrorInvalidValue);
  }
  GMT_RET_LAUNCH();
}

extern "C" int64_t gmt_diff_sq_workspace(int64_t nx, int64_t ny) {
  using namespace gmt;
  return ((nx + kDiffTile - 1) / kDiffTile) * ny;
}

extern "C" int gmt_diff_sq(int64_t nx, int64_t ny, const double* a, int64_t lda, const double* b,
                           int64_t ldb, double* out, double* ws, void* stream) {
  using namespace gmt;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nx <= 0 || ny <= 0) return static_cast<int>(hipMemsetAsync(out, 0, sizeof(double), s));
  const bool vec = aligned16(a) && aligned16(b) && lda % 2 == 0 && ldb % 2 == 0;
  const int64_t nch = (nx + kDiffTile - 1) / kDiffTile;
  diffsq_pass1<<<grid_1d(nch * ny), kBlock, 0, s>>>(nx, ny, a, lda, b, ldb, ws, nch, vec);
  sum_all<<<1, kBlock, 0, s>>>(ws, nch * ny, out);
  GMT_RET_LAUNCH();
}

extern "C" int64_t gmt_sum_workspace(int64_t n) {
  using namespace gmt;
  const int64_t nb = (n + 2 * kBlock - 1) / (2 * kBlock);
  return nb < 1 ? 1 : (nb < kSumBlocks ? nb : kSumBlocks);
}

extern "C" int gmt_sum(int64_t n, const double* x, double* out, double* ws, void* stream) {
  using namespace gmt;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n <= 0) return static_cast<int>(hipMemsetAsync(out, 0, sizeof(double), s));
  const int64_t nb = gmt_sum_workspace(n);
  sum1d_pass1<<<grid_1d(nb), kBlock, 0, s>>>(n, x, ws, aligned16(x));
  sum_all<<<1, kBlock, 0, s>>>(ws, nb, out);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_slices_reduce(int op, int64_t n, int nslices, const double* in, double* out, void* stream) {
  using namespace gmt;
  if (n < 0 || nslices < 1 || (op != 0 && op != 1)) return static_cast<int>(hipErrorInvalidValue);
  if (n == 0) return 0;
  slices_kernel<<<grid_1d((n + kBlock - 1) / kBlock), kBlock, 0, static_cast<hipStream_t>(stream)>>>(op, n, nslices,
                                                                                                  in, out);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_abs_max(int64_t nx, int64_t ny, const double* z, int64_t ld, double* out, double* ws,
                           void* stream) {
  using namespace gmt;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nx <= 0 || ny <= 0) return static_cast<int>(hipMemsetAsync(out, 0, sizeof(double), s));
  const int64_t nch = (nx + kDiffTile - 1) / kDiffTile;
  absmax_pass1<<<grid_1d(nch * ny), kBlock, 0, s>>>(nx, ny, z, ld, ws, nch);
  max_all<<<1, kBlock, 0, s>>>(ws, nch * ny, out);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_diff_bits(int64_t nx, int64_t ny, const double* a, int64_t lda, const double* b, int64_t ldb,
                             double* out, double* ws, void* stream) {
  using namespace gmt;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nx <= 0 || ny <= 0) return static_cast<int>(hipMemsetAsync(out, 0, 2 * sizeof(double), s));
  if (!a || !b || !out || !ws || lda < nx || ldb < nx) return static_cast<int>(hipErrorInvalidValue);
  const int64_t nch = (nx + kDiffTile - 1) / kDiffTile;
  diffbits_pass1<<<grid_1d(nch * ny), kBlock, 0, s>>>(nx, ny, a, lda, b, ldb, ws, nch);
  max_all<<<1, kBlock, 0, s>>>(ws, nch * ny, out);
  sum_all<<<1, kBlock, 0, s>>>(ws + nch * ny, nch * ny, out + 1);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_fill_poly(int mode, int64_t nx, int64_t ny, double x0, double dx, double y0,
                             double dy, double* z, int64_t ld, void* stream) {
  using namespace gmt;
  if (nx <= 0 || ny <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  fill_poly_kernel<<<grid_1d((nx * ny + kBlock - 1) / kBlock), kBlock, 0, s>>>(
      mode, nx, ny, x0, dx, y0, dy, z, ld);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_poly_check(int64_t nx, int64_t ny, double x0, double dx, double y0, double dy, double offset,
                              double rtol, const double* z, int64_t ld, unsigned* bad, void* stream) {
  using namespace gmt;
  if (nx <= 0 || ny <= 0) return 0;
  if (!bad || !z || ld < nx) return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  poly_check_kernel<<<grid_1d((nx * ny + kBlock - 1) / kBlock), kBlock, 0, s>>>(nx, ny, x0, dx, y0, dy, offset,
                                                                                 rtol, z, ld, bad);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_add_scalar(int64_t nx, int64_t ny, double v, double* z, int64_t ld, void* stream) {
  using namespace gmt;
  if (nx <= 0 || ny <= 0) return 0;
  if (!z || ld < nx) return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  add_scalar_kernel<<<grid_1d((nx * ny + kBlock - 1) / kBlock), kBlock, 0, s>>>(nx, ny, v, z, ld);
  GMT_RET_LAUNCH();
}

extern "C" const char* gmt_error_string(int err) {
  return hipGetErrorString(static_cast<hipError_t>(err));
}

extern "C" int gmt_device_synchronize(void) { return static_cast<int>(hipDeviceSynchronize()); }

extern "C" const char* gmt_build_info(void) {
  return "libgmt gfx950 (CDNA4) kernels: daxpy, stencil5 1d/2d (dim 1: LDS-DMA pipeline), jacobi5, "
         "jacobi5tb (1-20 fused sweeps, 4 columns per lane), ipc_exchange, signal_wait, "
         "copy2d_batched, sum_axis, sum, diff_sq, diff_bits, abs_max, fill_poly; built " __DATE__ " " __TIME__;
}
