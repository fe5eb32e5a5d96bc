// K1/K2 — fp64 DAXPY, y <- a*x + y, hand-written for gfx950.
//
// Reference behaviour: cublasDaxpy(n, &a, x, 1, y, 1) in daxpy.cu:73,
// mpi_daxpy.cc:141, mpi_daxpy_nvtx.cc:245 and gt::blas::axpy in
// mpi_daxpy_gt.cc:81 (incx = incy = 1, a = 2.0 in every caller).
//
// HBM-bound: 24 B per element (x read, y read, y written).  128-thread
// blocks, ONE 16-B chunk of x and y per lane, nontemporal loads AND stores:
// every byte is touched once, so nothing is worth keeping in L2/MALL.
// Measured 0.974 ms at n = 2^28 = 6.62 TB/s effective vs 1.076 ms (5.99 TB/s)
// for rocblas_daxpy (profiles/r01_sweep2.md).  The tiled / persistent
// variants it was chosen against live in csrc/bench/variant_bench.hip.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

template <int B>
__global__ __launch_bounds__(B) void daxpy_stream(int64_t n2, double a, const double* __restrict__ x,
                                                  double* __restrict__ y) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * B + threadIdx.x;
  if (i < n2) st2_nt(y + 2 * i, a * ld2_nt(x + 2 * i) + ld2_nt(y + 2 * i));
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
  if (aligned16(x) && aligned16(y)) {
    const int64_t n2 = n / 2;
    if (n2 > 0) {
      constexpr int B = 128;
      daxpy_stream<B><<<grid_1d((n2 + B - 1) / B), B, 0, s>>>(n2, a, x, y);
    }
    if (n & 1) daxpy_scalar_kernel<<<1, kBlock, 0, s>>>(1, a, x + n - 1, y + n - 1);
  } else {
    const int64_t nb = (n + kBlock - 1) / kBlock;
    daxpy_scalar_kernel<<<grid_1d(nb), kBlock, 0, s>>>(n, a, x, y);
  }
  GMT_RET_LAUNCH();
}
