// variant_bench — the A/B kernel variants that were measured against the
// production kernels of libgmt, kept OUT of the library (round-2 hygiene:
// no process-global variant switches in the production ABI).  Each variant
// is checked against the production entry point (gmt/kernels.h) on the same
// input, then both are timed; the table is what profiles/r01_sweep2.md and
// profiles/r02_tb.md cite.
//
//   variant_bench [--check]        --check: small shapes, correctness only
//
// Variants (all fp64):
//   daxpy  tile U4/U8 (nt x loads), tile U4/U8 (nt stores), persistent grid
//          — production: one 16-B chunk per lane, nt loads and stores
//   jacobi register sliding window (W/E from L1), LDS-tiled, lane-exchange
//          windows (DPP / shfl, 32-128 rows) — production: one output pair
//          per thread (jacobi5_pt)
//   deriv  dim 0 register window (3 overlapping loads), dim 1 register
//          window (the round-1 default, 4.92 TB/s) — production: dim 0
//          per-thread, dim 1 LDS-DMA pipeline
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../kernels/common.hpp"
#include "../kernels/stencil5_d1.hpp"
#include "gmt/kernels.h"

using namespace gmt;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)
#define GK(x)                                                                  \
  do {                                                                         \
    int e_ = (x);                                                              \
    if (e_ != 0) {                                                             \
      std::printf("gmt error %d (%s) at %s:%d\n", e_, #x, __FILE__, __LINE__); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

// ------------------------------------------------------------------ daxpy
template <int U, bool NT_LOAD_X, bool NT_STORE>
__global__ __launch_bounds__(kBlock) void daxpy_tile(int64_t n2, double a, const double* __restrict__ x,
                                                     double* __restrict__ y) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * (kBlock * U) + threadIdx.x;
  d2 xv[U], yv[U];
  if (base + (U - 1) * kBlock < n2) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * kBlock;
      xv[u] = NT_LOAD_X ? ld2_nt(x + 2 * i) : ld2(x + 2 * i);
      yv[u] = ld2(y + 2 * i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const d2 r = a * xv[u] + yv[u];
      if (NT_STORE)
        st2_nt(y + 2 * (base + u * kBlock), r);
      else
        st2(y + 2 * (base + u * kBlock), r);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * kBlock;
      if (i < n2) st2(y + 2 * i, a * ld2(x + 2 * i) + ld2(y + 2 * i));
    }
  }
}

template <int U>
__global__ __launch_bounds__(kBlock) void daxpy_persistent(int64_t n2, double a, const double* __restrict__ x,
                                                           double* __restrict__ y) {
  const int64_t chunk = static_cast<int64_t>(kBlock) * U;
  const int64_t nchunks = (n2 + chunk - 1) / chunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t base = c * chunk + threadIdx.x;
    if (base + (U - 1) * kBlock < n2) {
      d2 xv[U], yv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xv[u] = ld2(x + 2 * (base + u * kBlock));
        yv[u] = ld2(y + 2 * (base + u * kBlock));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) st2_nt(y + 2 * (base + u * kBlock), a * xv[u] + yv[u]);
    } else {
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * kBlock;
        if (i < n2) st2(y + 2 * i, a * ld2(x + 2 * i) + ld2(y + 2 * i));
      }
    }
  }
}

template <int U, bool NTX, bool NTS>
void launch_tile(int64_t n2, double a, const double* x, double* y) {
  const int64_t nb = (n2 + kBlock * U - 1) / (kBlock * U);
  daxpy_tile<U, NTX, NTS><<<grid_1d(nb), kBlock>>>(n2, a, x, y);
}

// ------------------------------------------------------------------ jacobi
constexpr int JR = 32;
constexpr int JTX = 2 * kBlock;

__global__ __launch_bounds__(kBlock) void jacobi5_reg(int64_t x0, int64_t nx, int64_t y0, int64_t ny,
                                                      const double* __restrict__ u, double* __restrict__ un,
                                                      int64_t ld, int64_t nbx, int64_t nblocks) {
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t xr = (bx * kBlock + threadIdx.x) * 2;
  const int64_t yr0 = by * JR;
  const int64_t rows = (ny - yr0) < JR ? (ny - yr0) : JR;
  if (xr + 1 >= nx) return;  // even widths only
  const double* p = u + (y0 + yr0 - 1) * ld + x0 + xr;
  double* q = un + (y0 + yr0) * ld + x0 + xr;
  d2 n = ld2(p), c = ld2(p + ld);
  for (int64_t r = 0; r < rows; ++r) {
    const double* pc = p + (r + 1) * ld;
    const d2 s = ld2(pc + ld);
    const double w = pc[-1], e = pc[2];
    d2 o;
    o.x = 0.25 * ((w + c.y) + (n.x + s.x));
    o.y = 0.25 * ((c.x + e) + (n.y + s.y));
    st2(q + r * ld, o);
    n = c;
    c = s;
  }
}

// W/E neighbours from the adjacent lanes: XCHG 1 = DPP, 2 = shfl (ds_bpermute)
template <int R, int XCHG, bool NTS>
__global__ __launch_bounds__(kBlock) void jacobi5_lane(int64_t x0, int64_t nx, int64_t y0, int64_t ny,
                                                       const double* __restrict__ u, double* __restrict__ un,
                                                       int64_t ld, int64_t nbx, int64_t nblocks) {
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t bx = t % nbx, by = t / nbx;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t xr = (bx * kBlock + threadIdx.x) * 2;
  const bool active = xr < nx;
  const bool edge_lo = lane == 0;
  const bool edge_hi = lane == kWave - 1 || xr + 2 >= nx;
  const int64_t yr0 = by * R;
  const int64_t rows = (ny - yr0) < R ? (ny - yr0) : R;
  const int64_t x = x0 + (active ? xr : 0);
  const double* p = u + (y0 + yr0 - 1) * ld + x;
  double* q = un + (y0 + yr0) * ld + x;
  d2 n = active ? ld2(p) : d2{0.0, 0.0};
  d2 c = active ? ld2(p + ld) : d2{0.0, 0.0};
  for (int64_t r = 0; r < rows; ++r) {
    const double* pc = p + (r + 1) * ld;
    const d2 s = active ? ld2(pc + ld) : d2{0.0, 0.0};
    double w = XCHG == 1 ? dpp_from_lower(c.y) : __shfl_up(c.y, 1, kWave);
    double e = XCHG == 1 ? dpp_from_upper(c.x) : __shfl_down(c.x, 1, kWave);
    if (active && edge_lo) w = pc[-1];
    if (active && edge_hi) e = pc[2];
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
  }
}

constexpr int LR = 16;
__global__ __launch_bounds__(kBlock) void jacobi5_lds(int64_t x0, int64_t nx, int64_t y0, int64_t ny,
                                                      const double* __restrict__ u, double* __restrict__ un,
                                                      int64_t ld, int64_t nbx, int64_t nblocks) {
  constexpr int P = JTX + 4;
  __shared__ double tile[(LR + 2) * P];
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t xr0 = bx * JTX, yr0 = by * LR;
  const int64_t cols = (nx - xr0) < JTX ? (nx - xr0) : JTX;
  const int64_t rows = (ny - yr0) < LR ? (ny - yr0) : LR;
  const int64_t gx = x0 + xr0, gy = y0 + yr0;
  const int tid = threadIdx.x;
  for (int r = 0; r < rows + 2; ++r) {
    const double* src = u + (gy - 1 + r) * ld + gx;
    double* dst = tile + r * P + 2;
    const int c = 2 * tid;
    if (c + 1 < cols)
      st2(dst + c, ld2(src + c));
    else if (c < cols)
      dst[c] = src[c];
    if (tid == 0) dst[-1] = src[-1];
    if (tid == 1) dst[cols] = src[cols];
  }
  __syncthreads();
  const int c = 2 * tid;
  if (c + 1 >= cols) return;
  for (int r = 1; r <= rows; ++r) {
    const double* row = tile + r * P + 2;
    const d2 ce = *reinterpret_cast<const d2*>(row + c);
    const d2 nn = *reinterpret_cast<const d2*>(row - P + c);
    const d2 ss = *reinterpret_cast<const d2*>(row + P + c);
    d2 o;
    o.x = 0.25 * ((row[c - 1] + ce.y) + (nn.x + ss.x));
    o.y = 0.25 * ((ce.x + row[c + 2]) + (nn.y + ss.y));
    st2(un + (gy - 1 + r) * ld + gx + c, o);
  }
}

// ------------------------------------------------------------------ deriv
struct Coef5 {
  double c[5];
};

// dim 1 as row streams: a block computes a U*512-column chunk of ONE output
// row from the same chunk of 5 input rows (5U independent 16-B loads per
// lane in flight); blocks are ordered rows-fastest within a chunk column so
// the 5 blocks that read an input chunk run together and share it in L2.
// ROWMAJOR: blocks sweep output row after output row instead (consecutive
// blocks walk along one row: linear streams; the 4 re-read input rows, 16 MB,
// come back from the 256 MB MALL).
template <int U, bool ROWMAJOR = false>
__global__ __launch_bounds__(kBlock) void stencil5_d1_rows(int64_t nx, int64_t ny_out, Coef5 cf, double scale,
                                                           const double* __restrict__ in, int64_t ld_in,
                                                           double* __restrict__ out, int64_t ld_out, int64_t nblocks) {
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t nchunk = nblocks / ny_out;
  const int64_t y = ROWMAJOR ? t / nchunk : t % ny_out, chunk = ROWMAJOR ? t % nchunk : t / ny_out;
  const int64_t x0 = chunk * (U * 2 * kBlock) + 2 * threadIdx.x;
  const double c0 = cf.c[0] * scale, c1 = cf.c[1] * scale, c2 = cf.c[2] * scale, c3 = cf.c[3] * scale,
               c4 = cf.c[4] * scale;
  const double* p = in + y * ld_in;
  d2 w[5][U];
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t x = x0 + u * 2 * kBlock;
      w[k][u] = x + 1 < nx ? ld2(p + k * ld_in + x) : d2{0.0, 0.0};
    }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t x = x0 + u * 2 * kBlock;
    if (x + 1 < nx) st2_nt(out + y * ld_out + x, c0 * w[0][u] + c1 * w[1][u] + c2 * w[2][u] + c3 * w[3][u] + c4 * w[4][u]);
  }
}
template <int U, bool ROWMAJOR = false>
void launch_rows(int64_t nx, int64_t ny_out, Coef5 cf, double scale, const double* in, int64_t ld_in, double* out,
                 int64_t ld_out) {
  const int64_t nchunk = (nx + U * 2 * kBlock - 1) / (U * 2 * kBlock), nb = nchunk * ny_out;
  stencil5_d1_rows<U, ROWMAJOR><<<grid_1d(nb), kBlock>>>(nx, ny_out, cf, scale, in, ld_in, out, ld_out, nb);
}

// the production dim-1 DMA pipeline at other chunk widths / segment lengths
template <int CPL>
void launch_d1(int64_t nx, int64_t ny_out, const double* c5, double scale, const double* in, int64_t ld_in,
               double* out, int64_t ld_out, int64_t L) {
  using namespace gmt::d1;
  Args a{};
  a.nx = nx;
  a.ny_out = ny_out;
  a.ld_in = ld_in;
  a.ld_out = ld_out;
  for (int k = 0; k < 5; ++k) a.c[k] = c5[k] * scale;
  a.nstrip = (nx + 128 * CPL - 1) / (128 * CPL);
  a.seg = static_cast<int>(L);
  a.nseg = (ny_out + L - 1) / L;
  a.nsteps = static_cast<int>((L + 4 + kU - 1) / kU * kU);
  const int64_t nb = (a.nstrip + kNW - 1) / kNW * a.nseg;
  const size_t smem = static_cast<size_t>(kNW) * kRS * CPL * kWave * 16;
  if (smem > 65536)
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&gmt::d1::stencil5_d1_dma<CPL, false>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(smem)));
  gmt::d1::stencil5_d1_dma<CPL, false><<<grid_1d(nb), kNW * kWave, smem>>>(a, in, out, nb);
  CK(hipGetLastError());
}
constexpr int ROWS0 = 4, ROWS1 = 32;

__global__ __launch_bounds__(kBlock) void stencil5_d0_vec(int64_t nx_out, int64_t ny, Coef5 cf, double scale,
                                                          const double* __restrict__ in, int64_t ld_in,
                                                          double* __restrict__ out, int64_t ld_out, int64_t nbx) {
  const int64_t b = blockIdx.x;
  const int64_t bx = b % nbx, by = b / nbx;
  const int64_t x = (bx * kBlock + threadIdx.x) * 2;
  if (x + 1 >= nx_out) return;  // even widths only
  const double c0 = cf.c[0] * scale, c1 = cf.c[1] * scale, c2 = cf.c[2] * scale, c3 = cf.c[3] * scale,
               c4 = cf.c[4] * scale;
  for (int r = 0; r < ROWS0; ++r) {
    const int64_t y = by * ROWS0 + r;
    if (y >= ny) break;
    const double* p = in + y * ld_in + x;
    const d2 a = ld2(p), m = ld2(p + 2), e = ld2(p + 4);
    d2 o;
    o.x = c0 * a.x + c1 * a.y + c2 * m.x + c3 * m.y + c4 * e.x;
    o.y = c0 * a.y + c1 * m.x + c2 * m.y + c3 * e.x + c4 * e.y;
    st2(out + y * ld_out + x, o);
  }
}

__global__ __launch_bounds__(kBlock) void stencil5_d1_vec(int64_t nx, int64_t ny_out, Coef5 cf, double scale,
                                                          const double* __restrict__ in, int64_t ld_in,
                                                          double* __restrict__ out, int64_t ld_out, int64_t nbx) {
  const int64_t b = blockIdx.x;
  const int64_t bx = b % nbx, by = b / nbx;
  const int64_t x = (bx * kBlock + threadIdx.x) * 2;
  if (x + 1 >= nx) return;  // even widths only
  const double c0 = cf.c[0] * scale, c1 = cf.c[1] * scale, c2 = cf.c[2] * scale, c3 = cf.c[3] * scale,
               c4 = cf.c[4] * scale;
  const int64_t y0 = by * ROWS1;
  const int64_t nrows = (ny_out - y0) < ROWS1 ? (ny_out - y0) : ROWS1;
  const double* p = in + y0 * ld_in + x;
  double* q = out + y0 * ld_out + x;
  d2 w0 = ld2(p), w1 = ld2(p + ld_in), w2 = ld2(p + 2 * ld_in), w3 = ld2(p + 3 * ld_in);
#pragma unroll 8
  for (int64_t r = 0; r < nrows; ++r) {
    const d2 w4 = ld2(p + (r + 4) * ld_in);
    st2_nt(q + r * ld_out, c0 * w0 + c1 * w1 + c2 * w2 + c3 * w3 + c4 * w4);
    w0 = w1;
    w1 = w2;
    w2 = w3;
    w3 = w4;
  }
}

// ------------------------------------------------------------------ harness
static double time_ms(int iters, const std::function<void()>& f) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) f();
  CK(hipEventRecord(e0));
  for (int k = 0; k < iters; ++k) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / iters;
}

static int g_fail = 0;

// tol: relative to max |expected| (0 = bitwise)
static void compare(const char* what, const double* got_d, const double* exp_d, size_t n, double tol) {
  std::vector<double> g(n), e(n);
  CK(hipMemcpy(g.data(), got_d, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(e.data(), exp_d, n * 8, hipMemcpyDeviceToHost));
  double worst = 0, scale = 0;
  for (size_t i = 0; i < n; ++i) {
    const double d = std::fabs(g[i] - e[i]);
    if (!(d <= worst)) worst = d;  // NaN-propagating max
    scale = std::fmax(scale, std::fabs(e[i]));
  }
  const bool ok = worst <= tol * scale;
  if (!ok) ++g_fail;
  std::printf("  check %-34s max|diff| = %.3e %s\n", what, worst, ok ? "OK" : "FAIL");
}

int main(int argc, char** argv) {
  const bool check = argc > 1 && std::strcmp(argv[1], "--check") == 0;
  const int iters = check ? 1 : 20;
  std::printf("# variant_bench (%s)\n", check ? "check" : "timing, mean of back-to-back launches");

  {  // daxpy
    const int64_t n = check ? (1 << 16) + 6 : int64_t(1) << 28, n2 = n / 2;
    double *x, *y, *y0;
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&y, n * 8));
    CK(hipMalloc(&y0, n * 8));
    GK(gmt_fill_poly(1, n, 1, 0.0, 1e-9, 0.0, 0.0, x, n, nullptr));
    GK(gmt_fill_poly(1, n, 1, 1.0, 1e-9, 0.0, 0.0, y0, n, nullptr));
    auto reset = [&] { CK(hipMemcpy(y, y0, n * 8, hipMemcpyDeviceToDevice)); };
    double* yref;
    CK(hipMalloc(&yref, n * 8));
    CK(hipMemcpy(yref, y0, n * 8, hipMemcpyDeviceToDevice));
    GK(gmt_daxpy(n2 * 2, 2.0, x, yref, nullptr));
    struct V {
      const char* name;
      std::function<void()> f;
    };
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const V vs[] = {
        {"daxpy tile U4 nt-x", [&] { launch_tile<4, true, false>(n2, 2.0, x, y); }},
        {"daxpy tile U8 nt-x", [&] { launch_tile<8, true, false>(n2, 2.0, x, y); }},
        {"daxpy persistent U4", [&] {
           const int64_t chunks = (n2 + kBlock * 4 - 1) / (kBlock * 4);
           daxpy_persistent<4><<<grid_1d(std::min<int64_t>(chunks, 8LL * cus)), kBlock>>>(n2, 2.0, x, y);
         }},
        {"daxpy tile U4 nt-store", [&] { launch_tile<4, false, true>(n2, 2.0, x, y); }},
        {"daxpy tile U8 nt-store", [&] { launch_tile<8, false, true>(n2, 2.0, x, y); }},
        {"daxpy production", [&] { GK(gmt_daxpy(n2 * 2, 2.0, x, y, nullptr)); }},
    };
    for (const V& v : vs) {
      reset();
      v.f();
      compare(v.name, y, yref, n2 * 2, 0.0);
      if (!check) {
        const double ms = time_ms(iters, v.f);
        std::printf("%-28s %9.4f ms %8.1f GB/s\n", v.name, ms, 24.0 * n2 * 2 / (ms * 1e-3) / 1e9);
      }
    }
    CK(hipFree(x));
    CK(hipFree(y));
    CK(hipFree(y0));
    CK(hipFree(yref));
  }
  {  // jacobi single sweep (Laplace form)
    const int64_t n = check ? 1000 : 32768, xo = 8, ld = ((xo + n + 1 + 63) / 64) * 64, rows = n + 2;
    double *u, *un, *uref;
    CK(hipMalloc(&u, ld * rows * 8));
    CK(hipMalloc(&un, ld * rows * 8));
    CK(hipMalloc(&uref, ld * rows * 8));
    GK(gmt_fill_poly(0, ld, rows, 0.0, 1e-5, 0.0, 1e-5, u, ld, nullptr));
    CK(hipMemset(uref, 0, ld * rows * 8));
    GK(gmt_jacobi5(xo, n, 1, n, u, uref, ld, nullptr, 0, 0.25, 0.0, nullptr, nullptr));
    auto grid = [&](int rr, int tx, int64_t* nbx) {
      *nbx = (n + tx - 1) / tx;
      return *nbx * ((n + rr - 1) / rr);
    };
    struct V {
      const char* name;
      std::function<void()> f;
    };
    int64_t nbx = 0;
    const V vs[] = {
        {"jacobi reg window", [&] {
           const int64_t nb = grid(JR, JTX, &nbx);
           jacobi5_reg<<<grid_1d(nb), kBlock>>>(xo, n, 1, n, u, un, ld, nbx, nb);
         }},
        {"jacobi LDS tile", [&] {
           const int64_t nb = grid(LR, JTX, &nbx);
           jacobi5_lds<<<grid_1d(nb), kBlock>>>(xo, n, 1, n, u, un, ld, nbx, nb);
         }},
        {"jacobi lane DPP 32", [&] {
           const int64_t nb = grid(32, JTX, &nbx);
           jacobi5_lane<32, 1, false><<<grid_1d(nb), kBlock>>>(xo, n, 1, n, u, un, ld, nbx, nb);
         }},
        {"jacobi lane shfl 32", [&] {
           const int64_t nb = grid(32, JTX, &nbx);
           jacobi5_lane<32, 2, false><<<grid_1d(nb), kBlock>>>(xo, n, 1, n, u, un, ld, nbx, nb);
         }},
        {"jacobi lane DPP 64 nt", [&] {
           const int64_t nb = grid(64, JTX, &nbx);
           jacobi5_lane<64, 1, true><<<grid_1d(nb), kBlock>>>(xo, n, 1, n, u, un, ld, nbx, nb);
         }},
        {"jacobi lane DPP 128 nt", [&] {
           const int64_t nb = grid(128, JTX, &nbx);
           jacobi5_lane<128, 1, true><<<grid_1d(nb), kBlock>>>(xo, n, 1, n, u, un, ld, nbx, nb);
         }},
        {"jacobi production", [&] {
           GK(gmt_jacobi5(xo, n, 1, n, u, un, ld, nullptr, 0, 0.25, 0.0, nullptr, nullptr));
         }},
    };
    for (const V& v : vs) {
      CK(hipMemset(un, 0, ld * rows * 8));
      v.f();
      compare(v.name, un, uref, ld * rows, 0.0);
      if (!check) {
        const double ms = time_ms(iters, v.f);
        std::printf("%-28s %9.4f ms %8.1f GB/s\n", v.name, ms, 16.0 * n * n / (ms * 1e-3) / 1e9);
      }
    }
    CK(hipFree(u));
    CK(hipFree(un));
    CK(hipFree(uref));
  }
  {  // derivative stencils: the reference's 1024 x 524288 shapes
    const int64_t a = check ? 256 : 1024, b = check ? 1000 : 512 * 1024;
    const double c[5] = {1.0 / 12, -2.0 / 3, 0.0, 2.0 / 3, -1.0 / 12};
    Coef5 cf;
    for (int k = 0; k < 5; ++k) cf.c[k] = c[k];
    double *in0, *in1, *out, *ref;
    CK(hipMalloc(&in0, (a + 4) * b * 8));
    CK(hipMalloc(&in1, (a + 4) * b * 8));  // dim 1: a + 4 rows of b columns
    CK(hipMalloc(&out, a * b * 8));
    CK(hipMalloc(&ref, a * b * 8));
    GK(gmt_fill_poly(0, a + 4, b, 0.0, 1e-3, 0.0, 1e-3, in0, a + 4, nullptr));
    GK(gmt_fill_poly(0, b, a + 4, 0.0, 1e-3, 0.0, 1e-3, in1, b, nullptr));
    // dim 0: rows of a + 4 -> a; dim 1: b columns, a + 4 rows -> a
    GK(gmt_stencil5_2d(0, a, b, c, 128.0, in0, a + 4, ref, a, nullptr));
    auto run0 = [&] {
      const int64_t nbx = (a + 2 * kBlock - 1) / (2 * kBlock);
      stencil5_d0_vec<<<grid_1d(nbx * ((b + ROWS0 - 1) / ROWS0)), kBlock>>>(a, b, cf, 128.0, in0, a + 4, out, a,
                                                                            nbx);
    };
    auto prod0 = [&] { GK(gmt_stencil5_2d(0, a, b, c, 128.0, in0, a + 4, out, a, nullptr)); };
    run0();
    compare("deriv dim0 reg window", out, ref, a * b, 1e-15);
    GK(gmt_stencil5_2d(1, b, a, c, 128.0, in1, b, ref, b, nullptr));
    auto run1 = [&] {
      const int64_t nbx = (b + 2 * kBlock - 1) / (2 * kBlock);
      stencil5_d1_vec<<<grid_1d(nbx * ((a + ROWS1 - 1) / ROWS1)), kBlock>>>(b, a, cf, 128.0, in1, b, out, b, nbx);
    };
    auto prod1 = [&] { GK(gmt_stencil5_2d(1, b, a, c, 128.0, in1, b, out, b, nullptr)); };
    // rounding differences (FMA contraction) scale with the input magnitude
    const double in_max = std::pow(b * 1e-3, 3) + std::pow((a + 4) * 1e-3, 2);
    const double tol1 = 8 * 2.3e-16 * in_max * 128.0 * 1.5;
    auto compare_abs = [&](const char* what) {
      std::vector<double> g(a * b), e(a * b);
      CK(hipMemcpy(g.data(), out, a * b * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(e.data(), ref, a * b * 8, hipMemcpyDeviceToHost));
      double worst = 0;
      for (int64_t i = 0; i < a * b; ++i) worst = std::fmax(worst, std::fabs(g[i] - e[i]));
      const bool ok = worst <= tol1;
      if (!ok) ++g_fail;
      std::printf("  check %-34s max|diff| = %.3e (tol %.1e) %s\n", what, worst, tol1, ok ? "OK" : "FAIL");
    };
    run1();
    compare_abs("deriv dim1 reg window (abs)");
    launch_rows<1>(b, a, cf, 128.0, in1, b, out, b);
    compare_abs("deriv dim1 rows U1");
    launch_rows<2>(b, a, cf, 128.0, in1, b, out, b);
    compare_abs("deriv dim1 rows U2");
    launch_rows<2, true>(b, a, cf, 128.0, in1, b, out, b);
    compare_abs("deriv dim1 rowmajor U2");
    for (int L : {64, 256}) {
      launch_d1<2>(b, a, c, 128.0, in1, b, out, b, L);
      compare_abs(L == 64 ? "deriv dim1 DMA CPL2 L64" : "deriv dim1 DMA CPL2 L256");
      launch_d1<4>(b, a, c, 128.0, in1, b, out, b, L);
      compare_abs(L == 64 ? "deriv dim1 DMA CPL4 L64" : "deriv dim1 DMA CPL4 L256");
    }
    if (!check) {
      const double bytes0 = 8.0 * ((a + 4) * b + a * b), bytes1 = bytes0;
      for (auto& [name, f] : {std::make_pair("deriv dim1 rows U1", std::function<void()>([&] { launch_rows<1>(b, a, cf, 128.0, in1, b, out, b); })),
                               std::make_pair("deriv dim1 rows U2", std::function<void()>([&] { launch_rows<2>(b, a, cf, 128.0, in1, b, out, b); })),
                               std::make_pair("deriv dim1 rows U4", std::function<void()>([&] { launch_rows<4>(b, a, cf, 128.0, in1, b, out, b); })),
                               std::make_pair("deriv dim1 rowmajor U1", std::function<void()>([&] { launch_rows<1, true>(b, a, cf, 128.0, in1, b, out, b); })),
                               std::make_pair("deriv dim1 rowmajor U2", std::function<void()>([&] { launch_rows<2, true>(b, a, cf, 128.0, in1, b, out, b); })),
                               std::make_pair("deriv dim1 rowmajor U4", std::function<void()>([&] { launch_rows<4, true>(b, a, cf, 128.0, in1, b, out, b); }))}) {
        const double ms = time_ms(iters, f);
        std::printf("%-28s %9.4f ms %8.1f GB/s\n", name, ms, bytes1 / (ms * 1e-3) / 1e9);
      }
      for (int L : {64, 128}) {
        char name[64];
        std::snprintf(name, sizeof(name), "deriv dim1 DMA CPL1 L%d", L);
        double ms = time_ms(iters, [&] { launch_d1<1>(b, a, c, 128.0, in1, b, out, b, L); });
        std::printf("%-28s %9.4f ms %8.1f GB/s\n", name, ms, bytes1 / (ms * 1e-3) / 1e9);
        std::snprintf(name, sizeof(name), "deriv dim1 DMA CPL2 L%d", L);
        ms = time_ms(iters, [&] { launch_d1<2>(b, a, c, 128.0, in1, b, out, b, L); });
        std::printf("%-28s %9.4f ms %8.1f GB/s\n", name, ms, bytes1 / (ms * 1e-3) / 1e9);
        std::snprintf(name, sizeof(name), "deriv dim1 DMA CPL4 L%d", L);
        ms = time_ms(iters, [&] { launch_d1<4>(b, a, c, 128.0, in1, b, out, b, L); });
        std::printf("%-28s %9.4f ms %8.1f GB/s\n", name, ms, bytes1 / (ms * 1e-3) / 1e9);
      }
      for (auto& [name, f, by] : {std::make_tuple("deriv dim0 reg window", std::function<void()>(run0), bytes0),
                                   std::make_tuple("deriv dim0 production", std::function<void()>(prod0), bytes0),
                                   std::make_tuple("deriv dim1 reg window", std::function<void()>(run1), bytes1),
                                   std::make_tuple("deriv dim1 production", std::function<void()>(prod1), bytes1)}) {
        const double ms = time_ms(iters, f);
        std::printf("%-28s %9.4f ms %8.1f GB/s\n", name, ms, by / (ms * 1e-3) / 1e9);
      }
    }
    CK(hipFree(in0));
    CK(hipFree(in1));
    CK(hipFree(out));
    CK(hipFree(ref));
  }
  std::printf("variant_bench %s (%d failed checks)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
