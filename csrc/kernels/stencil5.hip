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
// dim 0 (taps along the contiguous axis): stencil5_pt<0>, one output pair
// per thread, the overlapping loads served by L1 (6.34 TB/s effective).
//
// dim 1 (taps along the strided axis): stencil5_d1_win (even widths): 16
// waves side by side per workgroup walk 256-row segments with a register
// window, column groups fastest so the chip sweeps the array row band by row
// band (5.60-5.64 TB/s at the reference's shape, profiles/r03_d1_walk.txt);
// odd widths: stencil5_d1_dma, the round-2 LDS-DMA pipeline (5.46 TB/s on
// the same box).  The round-1 register-window kernel (now in
// csrc/bench/variant_bench.hip) issued its unrolled loads in bursts and
// drained them to vmcnt(0..3) every 8 rows: 85% of wave cycles waiting
// (rocprofv3 --pmc, profiles/r02_pmc/), 4.92 TB/s.
#include "common.hpp"
#include "gmt/kernels.h"
#include "stencil5_d1.hpp"

#include <algorithm>

namespace gmt {

struct Coef5 {
  double c[5];
};


// Per-thread kernels (dim 0 default; dim 1 fallback): one output pair per thread, 64 x 4 threads per
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

namespace {

// dim 1 through the DMA pipeline: segment rows per wave, chunks per lane
template <int CPL, bool ODD>
int launch_d1(int64_t nx, int64_t ny_out, const gmt::Coef5& cf, double scale, const double* in, int64_t ld_in,
              double* out, int64_t ld_out, int64_t L, hipStream_t s) {
  using namespace gmt::d1;
  Args a{};
  a.nx = nx;
  a.ny_out = ny_out;
  a.ld_in = ld_in;
  a.ld_out = ld_out;
  for (int k = 0; k < 5; ++k) a.c[k] = cf.c[k] * scale;
  a.nstrip = (nx + 128 * CPL - 1) / (128 * CPL);
  a.seg = static_cast<int>(L);
  a.nseg = (ny_out + L - 1) / L;
  a.nsteps = static_cast<int>((L + 4 + kU - 1) / kU * kU);
  const int64_t nb = (a.nstrip + kNW - 1) / kNW * a.nseg;
  const size_t smem = static_cast<size_t>(kNW) * kRS * CPL * gmt::kWave * 16;
  gmt::d1::stencil5_d1_dma<CPL, ODD><<<gmt::grid_1d(nb), kNW * gmt::kWave, smem, s>>>(a, in, out, nb);
  return static_cast<int>(hipGetLastError());
}

}  // namespace

extern "C" int gmt_stencil5_2d(int dim, int64_t nx_out, int64_t ny_out, const double* coef5,
                               double scale, const double* in, int64_t ld_in, double* out,
                               int64_t ld_out, void* stream) {
  using namespace gmt;
  if (nx_out <= 0 || ny_out <= 0) return 0;
  if (dim != 0 && dim != 1) return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Coef5 cf = make_coef(coef5);
  const bool vec_ok = aligned16(in) && aligned16(out) && (ld_in % 2 == 0) && (ld_out % 2 == 0);
  if (dim == 1 && vec_ok && nx_out % 2 == 0) {
    constexpr int kNWw = 16, kPw = 4;
    const int64_t L = std::min<int64_t>(256, ny_out);
    const int64_t ng = (nx_out + 128 * kNWw - 1) / (128 * kNWw), nseg = (ny_out + L - 1) / L;
    d1::Args c{};
    for (int k = 0; k < 5; ++k) c.c[k] = cf.c[k] * scale;
    d1::stencil5_d1_win<kNWw, kPw><<<grid_1d(ng * nseg), kNWw * kWave, 0, s>>>(nx_out, ny_out, ld_in, ld_out, L,
                                                                               ng, c, in, out);
    GMT_RET_LAUNCH();
  }
  if (dim == 1 && vec_ok) {
    // segment rows: the 32-bit buffer offsets must reach (L + 4 + P + U) rows
    // of the wider pitch; 128 rows amortise the 4-row input halo to 3 %
    const int64_t ld = ld_in > ld_out ? ld_in : ld_out;
    const int64_t lmax = (int64_t(1) << 31) / (ld * 8) - 4 - d1::kP - d1::kU;
    const int64_t L = std::min<int64_t>(std::min<int64_t>(128, ny_out), lmax);
    if (L >= 8) {
      if (nx_out % 2) return launch_d1<1, true>(nx_out, ny_out, cf, scale, in, ld_in, out, ld_out, L, s);
      return launch_d1<1, false>(nx_out, ny_out, cf, scale, in, ld_in, out, ld_out, L, s);
    }
  }
  if (vec_ok) {
    // one output pair per thread (dim 0: the default; dim 1: rows too long for
    // the DMA pipeline's 32-bit offsets)
    const int64_t nbx = (nx_out + 2 * kWave - 1) / (2 * kWave);
    const int64_t nb = nbx * ((ny_out + kBlock / kWave - 1) / (kBlock / kWave));
    if (dim == 0)
      stencil5_pt<0><<<grid_1d(nb), kBlock, 0, s>>>(nx_out, ny_out, cf, scale, in, ld_in, out,
                                                    ld_out, nbx, nb);
    else
      stencil5_pt<1><<<grid_1d(nb), kBlock, 0, s>>>(nx_out, ny_out, cf, scale, in, ld_in, out,
                                                    ld_out, nbx, nb);
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
