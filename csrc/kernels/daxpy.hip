// K1/K2 — fp64 DAXPY, y <- a*x + y, hand-written for gfx950.
//
// Reference behaviour: cublasDaxpy(n, &a, x, 1, y, 1) in daxpy.cu:73,
// mpi_daxpy.cc:141, mpi_daxpy_nvtx.cc:245 and gt::blas::axpy in
// mpi_daxpy_gt.cc:81 (incx = incy = 1, a = 2.0 in every caller).
//
// Design (HBM-bound, 24 B per element): each lane moves 16 B per instruction
// (global_load_dwordx4 = 2 doubles) and keeps U = 4 such loads of x and of y
// in flight before any store, so a 256-thread block owns 2048 contiguous
// doubles and a CU with 8 resident blocks has 8*256*4*32 B = 256 KiB of loads
// outstanding — well past the latency x bandwidth product of one CU
// (~2 us x 25 GB/s).  x is read exactly once: nontemporal loads keep it from
// displacing y lines in L2/MALL.  The grid is one block per 2048 elements (no
// grid-stride loop): for N = 2^28 that is 131072 blocks, far more than the
// 256 CUs need.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

template <int U>
__global__ __launch_bounds__(kBlock) void daxpy_vec_kernel(int64_t n2, double a,
                                                           const double* __restrict__ x,
                                                           double* __restrict__ y) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * (kBlock * U) + threadIdx.x;
  d2 xv[U], yv[U];
  if (base + (U - 1) * kBlock < n2) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * kBlock;
      xv[u] = ld2_nt(x + 2 * i);
      yv[u] = ld2(y + 2 * i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st2(y + 2 * (base + u * kBlock), a * xv[u] + yv[u]);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * kBlock;
      if (i < n2) st2(y + 2 * i, a * ld2(x + 2 * i) + ld2(y + 2 * i));
    }
  }
}

__global__ __launch_bounds__(kBlock) void daxpy_scalar_kernel(int64_t n, double a,
                                                              const double* __restrict__ x,
                                                              double* __restrict__ y) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) y[i] = a * x[i] + y[i];
}

}  // namespace gmt

extern "C" int gmt_daxpy(int64_t n, double a, const double* x, double* y, void* stream) {
  using namespace gmt;
  if (n <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  constexpr int U = 4;
  if (aligned16(x) && aligned16(y)) {
    const int64_t n2 = n / 2;
    if (n2 > 0) {
      const int64_t nb = (n2 + kBlock * U - 1) / (kBlock * U);
      daxpy_vec_kernel<U><<<grid_1d(nb), kBlock, 0, s>>>(n2, a, x, y);
    }
    if (n & 1) daxpy_scalar_kernel<<<1, kBlock, 0, s>>>(1, a, x + n - 1, y + n - 1);
  } else {
    const int64_t nb = (n + kBlock - 1) / kBlock;
    daxpy_scalar_kernel<<<grid_1d(nb), kBlock, 0, s>>>(n, a, x, y);
  }
  GMT_RET_LAUNCH();
}
