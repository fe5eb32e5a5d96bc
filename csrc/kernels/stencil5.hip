// K3/K4/K5/K11 — 5-tap first-derivative stencils, hand-written for gfx950.
//
// Reference: the gtensor expression templates stencil1d_5 / stencil2d_1d_5
// (mpi_stencil_gt.cc:54-59, mpi_stencil2d_gt.cc:84-110) and the SYCL kernel
// stencil2d_1d_5 (mpi_stencil2d_sycl.cc:53-75):
//     out[i] = scale * sum_{k=0..4} c[k] * in[i+k]
// with c = {1/12, -2/3, 0, 2/3, -1/12} (4th-order central difference).
//
// Layout: x contiguous ("dim 0"), y strided ("dim 1") — see gmt/kernels.h.
//
// dim 0 (taps along the contiguous axis): each lane produces 2 outputs from
// three overlapping 16-B loads (in[2t..2t+5]); the overlap is served by L1,
// so HBM sees each input byte once.  A block covers 512 outputs of ROWS0 rows.
//
// Variant 1 (kept for A/B; variant 2, below, is the default):
// dim 1 (taps along the strided axis): each lane owns 2 adjacent columns and
// walks down ROWS1 rows keeping a 5-row register window, so every input row
// is loaded once per column strip (+4 halo rows per strip => (R+4)/R reads).
// No LDS: the reuse is in registers, exactly where a row-walking lane needs it.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

struct Coef5 {
  double c[5];
};

constexpr int ROWS0 = 4;   // rows per block, dim-0 kernel
constexpr int ROWS1 = 32;  // rows per column strip, dim-1 kernel

__global__ __launch_bounds__(kBlock) void stencil5_d0_vec(int64_t nx_out, int64_t ny,
                                                          Coef5 cf, double scale,
                                                          const double* __restrict__ in,
                                                          int64_t ld_in,
                                                          double* __restrict__ out,
                                                          int64_t ld_out, int64_t nbx) {
  const int64_t b = blockIdx.x;
  const int64_t bx = b % nbx, by = b / nbx;
  const int64_t x = (bx * kBlock + threadIdx.x) * 2;
  if (x >= nx_out) return;
  const double c0 = cf.c[0] * scale, c1 = cf.c[1] * scale, c2 = cf.c[2] * scale,
               c3 = cf.c[3] * scale, c4 = cf.c[4] * scale;
  const int64_t y0 = by * ROWS0;
  const bool full = (x + 1 < nx_out);
#pragma unroll
  for (int r = 0; r < ROWS0; ++r) {
    const int64_t y = y0 + r;
    if (y >= ny) break;
    const double* p = in + y * ld_in + x;
    if (full) {
      const d2 a = ld2(p), m = ld2(p + 2), e = ld2(p + 4);
      d2 o;
      o.x = c0 * a.x + c1 * a.y + c2 * m.x + c3 * m.y + c4 * e.x;
      o.y = c0 * a.y + c1 * m.x + c2 * m.y + c3 * e.x + c4 * e.y;
      st2(out + y * ld_out + x, o);
    } else {
      out[y * ld_out + x] = c0 * p[0] + c1 * p[1] + c2 * p[2] + c3 * p[3] + c4 * p[4];
    }
  }
}

__global__ __launch_bounds__(kBlock) void stencil5_d1_vec(int64_t nx, int64_t ny_out,
                                                          Coef5 cf, double scale,
                                                          const double* __restrict__ in,
                                                          int64_t ld_in,
                                                          double* __restrict__ out,
                                                          int64_t ld_out, int64_t nbx) {
  const int64_t b = blockIdx.x;
  const int64_t bx = b % nbx, by = b / nbx;
  const int64_t x = (bx * kBlock + threadIdx.x) * 2;
  if (x >= nx) return;
  const double c0 = cf.c[0] * scale, c1 = cf.c[1] * scale, c2 = cf.c[2] * scale,
               c3 = cf.c[3] * scale, c4 = cf.c[4] * scale;
  const int64_t y0 = by * ROWS1;
  const int64_t nrows = (ny_out - y0) < ROWS1 ? (ny_out - y0) : ROWS1;
  const double* p = in + y0 * ld_in + x;
  double* q = out + y0 * ld_out + x;
  if (x + 1 < nx) {
    d2 w0 = ld2(p), w1 = ld2(p + ld_in), w2 = ld2(p + 2 * ld_in), w3 = ld2(p + 3 * ld_in);
    if (nrows == ROWS1) {
#pragma unroll 8
      for (int r = 0; r < ROWS1; ++r) {
        const d2 w4 = ld2(p + (r + 4) * ld_in);
        st2_nt(q + r * ld_out, c0 * w0 + c1 * w1 + c2 * w2 + c3 * w3 + c4 * w4);
        w0 = w1; w1 = w2; w2 = w3; w3 = w4;
      }
    } else {
      for (int64_t r = 0; r < nrows; ++r) {
        const d2 w4 = ld2(p + (r + 4) * ld_in);
        st2_nt(q + r * ld_out, c0 * w0 + c1 * w1 + c2 * w2 + c3 * w3 + c4 * w4);
        w0 = w1; w1 = w2; w2 = w3; w3 = w4;
      }
    }
  } else {  // odd last column
    double w0 = p[0], w1 = p[ld_in], w2 = p[2 * ld_in], w3 = p[3 * ld_in];
    for (int64_t r = 0; r < nrows; ++r) {
      const double w4 = p[(r + 4) * ld_in];
      q[r * ld_out] = c0 * w0 + c1 * w1 + c2 * w2 + c3 * w3 + c4 * w4;
      w0 = w1; w1 = w2; w2 = w3; w3 = w4;
    }
  }
}

// Per-thread kernels (variant 2; default for dim 0): one output pair per thread, 64 x 4 threads per
// block (128 columns x 4 rows), XCD-swizzled so the tiles that share input
// rows sit on one XCD's L2, nontemporal stores (the derivative is written
// once and not re-read by this kernel).  Same structure as the measured
// fastest Jacobi kernel (jacobi5.hip variant 9): short-lived threads with
// every load independent, reuse served by L1/L2 instead of registers.
template <int DIM>
__global__ __launch_bounds__(kBlock) void stencil5_pt(int64_t nx_out, int64_t ny_out, Coef5 cf,
                                                      double scale, const double* __restrict__ in,
                                                      int64_t ld_in, double* __restrict__ out,
                                                      int64_t ld_out, int64_t nbx, int64_t nblocks) {
  const int64_t t = xcd_swizzle(blockIdx.x, nblocks);
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t x = (bx * kWave + (threadIdx.x & (kWave - 1))) * 2;
  const int64_t y = by * (kBlock / kWave) + threadIdx.x / kWave;
  if (x >= nx_out || y >= ny_out) return;
  const double c0 = cf.c[0] * scale, c1 = cf.c[1] * scale, c2 = cf.c[2] * scale,
               c3 = cf.c[3] * scale, c4 = cf.c[4] * scale;
  const double* p = in + y * ld_in + x;
  if (x + 1 < nx_out) {
    d2 o;
    if (DIM == 0) {
      const d2 a = ld2(p), m = ld2(p + 2), e = ld2(p + 4);
      o.x = c0 * a.x + c1 * a.y + c2 * m.x + c3 * m.y + c4 * e.x;
      o.y = c0 * a.y + c1 * m.x + c2 * m.y + c3 * e.x + c4 * e.y;
    } else {
      o = c0 * ld2(p) + c1 * ld2(p + ld_in) + c2 * ld2(p + 2 * ld_in) + c3 * ld2(p + 3 * ld_in) +
          c4 * ld2(p + 4 * ld_in);
    }
    st2_nt(out + y * ld_out + x, o);
  } else {
    const int64_t st = DIM == 0 ? 1 : ld_in;
    out[y * ld_out + x] = c0 * p[0] + c1 * p[st] + c2 * p[2 * st] + c3 * p[3 * st] + c4 * p[4 * st];
  }
}

static int g_stencil_variant = 0;

// Generic fallback for unaligned views: one output per lane.
__global__ __launch_bounds__(kBlock) void stencil5_scalar(int dim, int64_t nx_out,
                                                          int64_t ny_out, Coef5 cf,
                                                          double scale, const double* in,
                                                          int64_t ld_in, double* out,
                                                          int64_t ld_out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= nx_out * ny_out) return;
  const int64_t x = i % nx_out, y = i / nx_out;
  const int64_t step = dim == 0 ? 1 : ld_in;
  const double* p = in + y * ld_in + x;
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 5; ++k) acc += cf.c[k] * scale * p[k * step];
  out[y * ld_out + x] = acc;
}

static Coef5 make_coef(const double* c5) {
  Coef5 c;
  for (int k = 0; k < 5; ++k) c.c[k] = c5[k];
  return c;
}

}  // namespace gmt

extern "C" void gmt_stencil5_set_variant(int v) { gmt::g_stencil_variant = v; }

extern "C" int gmt_stencil5_2d(int dim, int64_t nx_out, int64_t ny_out, const double* coef5,
                               double scale, const double* in, int64_t ld_in, double* out,
                               int64_t ld_out, void* stream) {
  using namespace gmt;
  if (nx_out <= 0 || ny_out <= 0) return 0;
  if (dim != 0 && dim != 1) return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Coef5 cf = make_coef(coef5);
  const bool vec_ok = aligned16(in) && aligned16(out) && (ld_in % 2 == 0) && (ld_out % 2 == 0);
  // default: per-thread kernel for dim 0 (taps along the contiguous axis,
  // 6.34 TB/s), register window for dim 1 (a 5-row window per lane beats
  // five L2-served row loads per thread: 1.87 vs 2.05 ms at 1024 x 524288)
  const bool pt = g_stencil_variant == 2 || (g_stencil_variant == 0 && dim == 0);
  if (vec_ok && pt) {
    const int64_t nbx = (nx_out + 2 * kWave - 1) / (2 * kWave);
    const int64_t nb = nbx * ((ny_out + kBlock / kWave - 1) / (kBlock / kWave));
    if (dim == 0)
      stencil5_pt<0><<<grid_1d(nb), kBlock, 0, s>>>(nx_out, ny_out, cf, scale, in, ld_in, out,
                                                    ld_out, nbx, nb);
    else
      stencil5_pt<1><<<grid_1d(nb), kBlock, 0, s>>>(nx_out, ny_out, cf, scale, in, ld_in, out,
                                                    ld_out, nbx, nb);
  } else if (vec_ok) {
    const int64_t nbx = (nx_out + 2 * kBlock - 1) / (2 * kBlock);
    if (dim == 0) {
      const int64_t nby = (ny_out + ROWS0 - 1) / ROWS0;
      stencil5_d0_vec<<<grid_1d(nbx * nby), kBlock, 0, s>>>(nx_out, ny_out, cf, scale, in,
                                                             ld_in, out, ld_out, nbx);
    } else {
      const int64_t nby = (ny_out + ROWS1 - 1) / ROWS1;
      stencil5_d1_vec<<<grid_1d(nbx * nby), kBlock, 0, s>>>(nx_out, ny_out, cf, scale, in,
                                                             ld_in, out, ld_out, nbx);
    }
  } else {
    const int64_t nb = (nx_out * ny_out + kBlock - 1) / kBlock;
    stencil5_scalar<<<grid_1d(nb), kBlock, 0, s>>>(dim, nx_out, ny_out, cf, scale, in, ld_in,
                                                   out, ld_out);
  }
  GMT_RET_LAUNCH();
}

extern "C" int gmt_stencil5_1d(int64_t n_out, const double* coef5, double scale,
                               const double* in, double* out, void* stream) {
  // A 1-D array is a single-row 2-D field.  Split long vectors into rows of
  // 2^16 so the dim-0 kernel's grid spreads over all CUs (each row keeps its
  // own 4-element right halo: in row r starts at r*W and reads W+4 values).
  if (n_out <= 0) return 0;
  const int64_t W = 65536;
  const int64_t rows = n_out / W;
  int err = 0;
  if (rows > 0) {
    err = gmt_stencil5_2d(0, W, rows, coef5, scale, in, W, out, W, stream);
    if (err) return err;
  }
  const int64_t rem = n_out - rows * W;
  if (rem > 0)
    err = gmt_stencil5_2d(0, rem, 1, coef5, scale, in + rows * W, rem + 4, out + rows * W,
                          rem, stream);
  return err;
}
