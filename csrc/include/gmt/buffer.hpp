// gmt/buffer.hpp — RAII memory in each space + column-major 2-D views.
//
// Reference containers: raw cudaMalloc/cudaMallocHost/cudaMallocManaged
// pointers (mpi_daxpy_nvtx.cc:177-199), gtensor containers in
// host/device/managed space (mpi_stencil2d_gt.cc:42-73,420-425) and the SYCL
// span2d/array2d pair (mpi_stencil2d_sycl_oo.cc:51-152) — which used 32-bit
// dims (overflows past 2^31 elements) and leaked (its destructor is
// commented out, :136-137).  Here: owning Buffer<T> frees itself, is
// move-only, and every index is size_t.
#pragma once

#include <cassert>
#include <cstddef>
#include <utility>

#include "gmt/check.hpp"

namespace gmt {

template <typename T>
class Buffer {
 public:
  Buffer() = default;
  Buffer(size_t n, int space) : n_(n), space_(space) {
    void* p = nullptr;
    GMT_CHECK("alloc", gmt_rt_malloc(&p, n * sizeof(T), space));
    p_ = static_cast<T*>(p);
  }
  ~Buffer() { reset(); }
  Buffer(const Buffer&) = delete;
  Buffer& operator=(const Buffer&) = delete;
  Buffer(Buffer&& o) noexcept { *this = std::move(o); }
  Buffer& operator=(Buffer&& o) noexcept {
    if (this != &o) {
      reset();
      p_ = o.p_;
      n_ = o.n_;
      space_ = o.space_;
      o.p_ = nullptr;
      o.n_ = 0;
    }
    return *this;
  }
  void reset() {
    if (p_) GMT_WARN("free", gmt_rt_free(p_, space_));
    p_ = nullptr;
    n_ = 0;
  }
  T* data() const { return p_; }
  size_t size() const { return n_; }
  size_t bytes() const { return n_ * sizeof(T); }
  int space() const { return space_; }
  bool host_accessible() const {
    return space_ != GMT_SPACE_DEVICE || gmt_rt_backend() == GMT_BACKEND_HOST;
  }
  T& operator[](size_t i) const { return p_[i]; }

 private:
  T* p_ = nullptr;
  size_t n_ = 0;
  int space_ = GMT_SPACE_HOST;
};

// Column-major 2-D view: element (i, j) at data[i + j*ld]; i is the
// contiguous "dim 0" of the reference (idx2, mpi_stencil2d_sycl.cc:40-43).
// In gmt/kernels.h terms: x = i, y = j, row pitch = ld.
template <typename T>
struct Span2D {
  T* data = nullptr;
  size_t nrows = 0, ncols = 0, ld = 0;

  Span2D() = default;
  Span2D(T* d, size_t r, size_t c) : data(d), nrows(r), ncols(c), ld(r) {}
  Span2D(T* d, size_t r, size_t c, size_t l) : data(d), nrows(r), ncols(c), ld(l) {}

  T& operator()(size_t i, size_t j) const {
    assert(i < nrows && j < ncols);
    return data[i + j * ld];
  }
  size_t size() const { return nrows * ncols; }
  bool contiguous() const { return ld == nrows || ncols <= 1; }
  // rows [r0, r0+nr) x cols [c0, c0+nc)
  Span2D sub(size_t r0, size_t nr, size_t c0, size_t nc) const {
    assert(r0 + nr <= nrows && c0 + nc <= ncols);
    return Span2D(data + r0 + c0 * ld, nr, nc, ld);
  }
};

}  // namespace gmt
