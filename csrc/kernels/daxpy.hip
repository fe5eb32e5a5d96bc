// K1/K2 — fp64 DAXPY, y <- a*x + y, hand-written for gfx950.
//
// Reference behaviour: cublasDaxpy(n, &a, x, 1, y, 1) in daxpy.cu:73,
// mpi_daxpy.cc:141, mpi_daxpy_nvtx.cc:245 and gt::blas::axpy in
// mpi_daxpy_gt.cc:81 (incx = incy = 1, a = 2.0 in every caller).
//
// HBM-bound: 24 B per element (x read, y read, y written).  Every lane moves
// 16 B per instruction (global_load_dwordx4 = 2 doubles).  Variants (A/B on
// gfx950 with gmt_daxpy_set_variant, measured in profiles/):
//   1  one block per 256*U*2 elements, U = 4 loads of x and y in flight per
//      lane, nontemporal x loads, plain stores (first version)
//   2  same tiling, U = 8
//   3  persistent grid (8 blocks per CU), grid-stride over U = 4 chunks,
//      nontemporal stores of y
//   4  one block per 256*U*2 elements, U = 4, plain loads, nontemporal stores
//   5  one block per 256*U*2 elements, U = 8, plain loads, nontemporal stores
//   6  (default) 128-thread blocks, ONE 16-B chunk of x and y per lane,
//      nontemporal loads AND stores: every byte is touched once, so nothing
//      is worth keeping in L2/MALL.  Measured 0.974 ms at n = 2^28 = 6.62 TB/s
//      effective vs 1.076 ms (5.99 TB/s) for rocblas_daxpy and 1.12 ms for v1
//      (profiles/r01_sweep2.md).  rocBLAS moves one double per lane.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

static int g_daxpy_variant = 0;

template <int U, bool NT_LOAD_X, bool NT_STORE>
__global__ __launch_bounds__(kBlock) void daxpy_tile(int64_t n2, double a,
                                                     const double* __restrict__ x,
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

template <int B>
__global__ __launch_bounds__(B) void daxpy_stream(int64_t n2, double a, const double* __restrict__ x,
                                                  double* __restrict__ y) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * B + threadIdx.x;
  if (i < n2) st2_nt(y + 2 * i, a * ld2_nt(x + 2 * i) + ld2_nt(y + 2 * i));
}

template <int U>
__global__ __launch_bounds__(kBlock) void daxpy_persistent(int64_t n2, double a,
                                                           const double* __restrict__ x,
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

__global__ __launch_bounds__(kBlock) void daxpy_scalar_kernel(int64_t n, double a,
                                                              const double* __restrict__ x,
                                                              double* __restrict__ y) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) y[i] = a * x[i] + y[i];
}

template <int U, bool NTX, bool NTS>
static void launch_tile(int64_t n2, double a, const double* x, double* y, hipStream_t s) {
  const int64_t nb = (n2 + kBlock * U - 1) / (kBlock * U);
  daxpy_tile<U, NTX, NTS><<<grid_1d(nb), kBlock, 0, s>>>(n2, a, x, y);
}

}  // namespace gmt

extern "C" void gmt_daxpy_set_variant(int v) { gmt::g_daxpy_variant = v; }
extern "C" int gmt_daxpy_get_variant(void) { return gmt::g_daxpy_variant; }

extern "C" int gmt_daxpy(int64_t n, double a, const double* x, double* y, void* stream) {
  using namespace gmt;
  if (n <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (aligned16(x) && aligned16(y)) {
    const int64_t n2 = n / 2;
    if (n2 > 0) {
      switch (g_daxpy_variant) {
        case 1: launch_tile<4, true, false>(n2, a, x, y, s); break;
        case 2: launch_tile<8, true, false>(n2, a, x, y, s); break;
        case 3: {
          int dev = 0, cus = 256;
          (void)hipGetDevice(&dev);
          (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
          const int64_t chunks = (n2 + kBlock * 4 - 1) / (kBlock * 4);
          const int64_t nb = chunks < 8LL * cus ? chunks : 8LL * cus;
          daxpy_persistent<4><<<grid_1d(nb), kBlock, 0, s>>>(n2, a, x, y);
          break;
        }
        case 5: launch_tile<8, false, true>(n2, a, x, y, s); break;
        case 4: launch_tile<4, false, true>(n2, a, x, y, s); break;
        default: {
          constexpr int B = 128;
          daxpy_stream<B><<<grid_1d((n2 + B - 1) / B), B, 0, s>>>(n2, a, x, y);
          break;
        }
      }
    }
    if (n & 1) daxpy_scalar_kernel<<<1, kBlock, 0, s>>>(1, a, x + n - 1, y + n - 1);
  } else {
    const int64_t nb = (n + kBlock - 1) / kBlock;
    daxpy_scalar_kernel<<<grid_1d(nb), kBlock, 0, s>>>(n, a, x, y);
  }
  GMT_RET_LAUNCH();
}
