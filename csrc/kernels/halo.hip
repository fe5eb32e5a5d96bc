// K6/K7/K8 — halo pack / unpack as ONE fused batched strided-2-D copy.
//
// Reference: gtensor slice assignments `sbuf = view(_s(n_bnd, 2*n_bnd), _all)`
// (pack, mpi_stencil2d_gt.cc:166,172,289,292), `view(_s(0,n_bnd), _all) = rbuf`
// (unpack, :239,251,357,368) and the SYCL buf_from_view / buf_to_view kernels
// (mpi_stencil2d_sycl.cc:82-116) — one launch per side per direction there.
//
// Here every side of a step (left+right, or all four faces of a 2-D
// decomposition) is packed or unpacked in a single launch: the descriptors
// travel by value in the kernel arguments, the grid is the concatenation of
// the per-descriptor block ranges, and each block finds its descriptor with a
// short scalar scan (<= 8 entries, wave-uniform).
//
// Width classes:
//  * width*elem is a multiple of 16 B and everything is 16-B aligned: each
//    lane moves 16 B (the reference's dim-0 halo is exactly 2 doubles = 16 B
//    per row, so one lane = one row, one dwordx4 load + one dwordx4 store);
//  * otherwise element-wise (e.g. the 1-double-wide W/E faces of the Jacobi
//    decomposition).
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {

struct Copy2dBatch {
  const char* src[GMT_MAX_COPY2D];
  char* dst[GMT_MAX_COPY2D];
  int64_t src_ld[GMT_MAX_COPY2D];  // in units (bytes/unit = U)
  int64_t dst_ld[GMT_MAX_COPY2D];
  int64_t width[GMT_MAX_COPY2D];   // in units
  int64_t height[GMT_MAX_COPY2D];
  int64_t block_start[GMT_MAX_COPY2D + 1];
  int n;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void copy2d_batched_kernel(Copy2dBatch b) {
  const int64_t blk = blockIdx.x;
  int k = 0;
  while (k + 1 < b.n && blk >= b.block_start[k + 1]) ++k;
  const int64_t w = b.width[k];
  const int64_t total = w * b.height[k];
  const int64_t i = (blk - b.block_start[k]) * kBlock + threadIdx.x;
  if (i >= total) return;
  int64_t row, col;
  if (w == 1) {
    row = i;
    col = 0;
  } else if (total <= 0xffffffffll) {
    // every halo face fits 32 bits: a 32-bit division (a few VALU
    // instructions) instead of the 64-bit software sequence
    const uint32_t ii = static_cast<uint32_t>(i), ww = static_cast<uint32_t>(w);
    const uint32_t r = ii / ww;
    row = r;
    col = ii - r * ww;
  } else {
    row = i / w;
    col = i - row * w;
  }
  const T* s = reinterpret_cast<const T*>(b.src[k]) + row * b.src_ld[k] + col;
  T* d = reinterpret_cast<T*>(b.dst[k]) + row * b.dst_ld[k] + col;
  *d = *s;
}

// The same copy as a grid-stride loop over few workgroups (max_wgs > 0):
// beside a pass that holds nearly every CU slot, a launch of hundreds of
// short workgroups trickles through the few free slots one dispatch at a
// time (profiles/r04_overlap.md); a few resident workgroups, each with four
// 16-B loads in flight per lane, move the same faces without waiting for
// slots to free.
template <typename T>
__global__ __launch_bounds__(kBlock) void copy2d_stride_kernel(Copy2dBatch b, int64_t total_all) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  int k = 0;
  auto at = [&](int64_t e, int& kk) -> int64_t {  // descriptor of element e (e only grows) and its offset
    while (kk + 1 < b.n && e >= b.block_start[kk + 1]) ++kk;
    return e - b.block_start[kk];
  };
  for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e0 < total_all; e0 += 4 * stride) {
    T v[4];
    T* d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = e0 + u * stride;
      d[u] = nullptr;
      if (e < total_all) {
        const int64_t i = at(e, k);
        const int64_t w = b.width[k], row = i / w, col = i - row * w;
        v[u] = *(reinterpret_cast<const T*>(b.src[k]) + row * b.src_ld[k] + col);
        d[u] = reinterpret_cast<T*>(b.dst[k]) + row * b.dst_ld[k] + col;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (d[u]) *d[u] = v[u];
    k = 0;  // e0 + 0 * stride of the next iteration may sit in an earlier descriptor than e0 + 3 * stride
  }
}

}  // namespace gmt

extern "C" int gmt_copy2d_batched(int n_desc, const gmt_copy2d_desc* descs, int elem_bytes,
                                  void* stream) {
  return gmt_copy2d_batched_wgs(n_desc, descs, elem_bytes, 0, stream);
}

extern "C" int gmt_copy2d_batched_wgs(int n_desc, const gmt_copy2d_desc* descs, int elem_bytes, int max_wgs,
                                      void* stream) {
  using namespace gmt;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n_desc < 0 || n_desc > GMT_MAX_COPY2D) return static_cast<int>(hipErrorInvalidValue);
  if (elem_bytes != 4 && elem_bytes != 8) return static_cast<int>(hipErrorInvalidValue);
  // Pick the widest unit every descriptor supports.
  int unit = 16;
  for (int k = 0; k < n_desc; ++k) {
    const gmt_copy2d_desc& d = descs[k];
    const int64_t wb = d.width * elem_bytes;
    const int64_t sb = d.src_ld * elem_bytes, db = d.dst_ld * elem_bytes;
    auto ok = [&](int u) {
      return (wb % u == 0) && (sb % u == 0 || d.height <= 1) && (db % u == 0 || d.height <= 1) &&
             (reinterpret_cast<uintptr_t>(d.src) % u == 0) &&
             (reinterpret_cast<uintptr_t>(d.dst) % u == 0);
    };
    while (unit > elem_bytes && !ok(unit)) unit /= 2;
  }
  Copy2dBatch b{};
  b.n = 0;
  b.block_start[0] = 0;
  for (int k = 0; k < n_desc; ++k) {
    const gmt_copy2d_desc& d = descs[k];
    if (d.width <= 0 || d.height <= 0) continue;
    const int64_t r = unit / elem_bytes;
    const int j = b.n;
    b.src[j] = static_cast<const char*>(d.src);
    b.dst[j] = static_cast<char*>(d.dst);
    b.src_ld[j] = d.src_ld / r;
    b.dst_ld[j] = d.dst_ld / r;
    b.width[j] = d.width / r;
    b.height[j] = d.height;
    const int64_t total = b.width[j] * b.height[j];
    b.block_start[j + 1] = b.block_start[j] + (total + kBlock - 1) / kBlock;
    ++b.n;
  }
  if (b.n == 0) return 0;
  for (int k = b.n + 1; k <= GMT_MAX_COPY2D; ++k) b.block_start[k] = b.block_start[b.n];
  const int cap = max_wgs;
  if (cap > 0) {
    // element offsets instead of block offsets
    int64_t acc = 0;
    for (int k = 0; k < b.n; ++k) {
      b.block_start[k] = acc;
      acc += b.width[k] * b.height[k];
    }
    for (int k = b.n; k <= GMT_MAX_COPY2D; ++k) b.block_start[k] = acc;
    const unsigned nb = static_cast<unsigned>(std::min<int64_t>(cap, (acc + kBlock - 1) / kBlock));
    switch (unit) {
      case 16: copy2d_stride_kernel<d2><<<nb, kBlock, 0, s>>>(b, acc); break;
      case 8: copy2d_stride_kernel<double><<<nb, kBlock, 0, s>>>(b, acc); break;
      default: copy2d_stride_kernel<float><<<nb, kBlock, 0, s>>>(b, acc); break;
    }
    GMT_RET_LAUNCH();
  }
  const unsigned nb = grid_1d(b.block_start[b.n]);
  switch (unit) {
    case 16: copy2d_batched_kernel<d2><<<nb, kBlock, 0, s>>>(b); break;
    case 8: copy2d_batched_kernel<double><<<nb, kBlock, 0, s>>>(b); break;
    default: copy2d_batched_kernel<float><<<nb, kBlock, 0, s>>>(b); break;
  }
  GMT_RET_LAUNCH();
}
