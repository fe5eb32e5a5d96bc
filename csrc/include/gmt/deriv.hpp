// gmt/deriv.hpp — the distributed-derivative and all-reduce tests of the
// reference, MPI-free: they run on any comm::Transport, so the MPI apps
// (csrc/apps/deriv_common.hpp) and the MPI-free engine library
// (csrc/engine/halo_bench.cpp, driven by bench.py through torch.distributed)
// share one implementation.
//
// Reference: test_deriv<S, Dim> (mpi_stencil2d_gt.cc:385-572) and
// test_sum<S, Dim> (:574-649).  Workload: z = x^3 + y^2 on a column-major
// 2-D array decomposed into 1-D slabs along `dim`, 2 ghost cells per side,
// 4th-order first derivative dz/d(dim) after every halo exchange;
// err_norm = ||numeric - analytic||_2 (the stencil is exact for cubics, so
// err_norm is round-off unless the halo exchange is wrong).  The analytic
// fill and the verification run on the GPU (gmt_fill_poly / gmt_diff_sq);
// --host-init / --host-verify restore the reference's host loops.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/halo.hpp"
#include "gmt/kernels.h"
#include "gmt/transport.hpp"
#include "gmt/util.hpp"

namespace gmt {
namespace apps {

constexpr double kDeriv5[5] = {1.0 / 12.0, -2.0 / 3.0, 0.0, 2.0 / 3.0, -1.0 / 12.0};
constexpr double kPI = 3.141592653598793;  // the reference's constant, sic

// dump(what, field, nrows, ncols, row0, nrows_to_print)
using DumpFn = std::function<void(const char*, const double*, size_t, size_t, size_t, size_t)>;

struct DerivConfig {
  int dim = 0;              // decomposed + derivative axis (0 = contiguous)
  size_t n_local = 1024;    // extent along dim per rank
  size_t n_other = 512 * 1024;
  int n_iter = 1000, n_warmup = 5;
  int space = GMT_SPACE_DEVICE;  // or GMT_SPACE_MANAGED
  bool buf = true;               // reference `use_buffers` / `stage_host`
  bool staged_is_host = true;    // dim 0 + buf means host staging (reference gt/sycl)
  comm::Kind transport = comm::Kind::Auto;  // the apps' choice (gmt/comm.hpp resolve)
  bool host_init = false, host_verify = false;
  bool realloc_per_call = false;  // emulate the gt version's per-call buffers
  bool debug_dump = false;        // rank-serialised halo-row dumps (sycl_oo DEBUG build)
  // --check: after EVERY exchange, one small kernel compares the ghost rows
  // the exchange filled with the analytic field; before every exchange the
  // whole local field is raised by 1.0 (outside the timed region), so a
  // ghost row left from an earlier exchange (a reused staging slot, a lost
  // chunk) differs by >= 1 and is counted.  The reference checks only the
  // last iteration's derivative (mpi_stencil2d_gt.cc:541-570).
  bool check = false;
};

struct DerivResult {
  double total_time = 0.0;  // seconds, this rank, timed iterations only
  double err_norm = 0.0;
  // sqrt(sum of the analytic derivative squared) over this rank's output:
  // err_norm / exact_norm is a scale-free check (the round-off of x^3 + y^2
  // at the reference's spacing grows with the non-decomposed extent)
  double exact_norm = 0.0;
  Stats iters;              // per-exchange seconds
  std::string transport;
  size_t bytes_per_exchange = 0;
  long long bad_ghosts = -1;  // --check: ghost cells that were wrong after some exchange (-1: not checked)
  int checked_exchanges = 0;
};

// GMT_CORRUPT_GHOST=R:K (fault injection for --check): rank R overwrites one
// ghost cell after its K-th exchange (counting warm-ups from 0)
inline bool corrupt_ghost_now(int rank, int it) {
  const char* e = std::getenv("GMT_CORRUPT_GHOST");
  if (!e) return false;
  const char* c = std::strchr(e, ':');
  return std::atoi(e) == rank && c && std::atoi(c + 1) == it;
}

// `dump(what, row0)` (optional) prints n_bnd rows of the field from every
// rank (the apps gather them over MPI).
inline DerivResult run_deriv_on(const DerivConfig& c, comm::Transport& tr, int rank, int ws,
                                const DumpFn& dump = nullptr) {
  const size_t n_bnd = 2;
  const size_t n_global = c.n_local * ws;
  const double ln = 8.0, delta = ln / n_global, scale = n_global / ln;
  const double start = rank * (ln / ws);
  const bool d0 = c.dim == 0;
  const size_t nrows = d0 ? c.n_local + 2 * n_bnd : c.n_other;
  const size_t ncols = d0 ? c.n_other : c.n_local + 2 * n_bnd;
  const size_t nx_out = d0 ? c.n_local : c.n_other;
  const size_t ny_out = d0 ? c.n_other : c.n_local;
  gmt_stream_t s = nullptr;
  GMT_CHECK("stream", gmt_rt_stream_create(&s, 0));

  Buffer<double> z(nrows * ncols, c.space), dz(nx_out * ny_out, c.space);
  Span2D<double> zf(z.data(), nrows, ncols);
  // interior + physical-boundary ghosts (mpi_stencil2d_gt.cc:439-497)
  const double x0 = d0 ? start : 0.0, y0 = d0 ? 0.0 : start;
  if (c.host_init) {
    std::vector<double> h(nrows * ncols, 0.0);
    auto fn = [](double x, double y) { return x * x * x + y * y; };
    const size_t gx = d0 ? n_bnd : 0, gy = d0 ? 0 : n_bnd;
    for (size_t j = 0; j < ny_out; ++j)
      for (size_t i = 0; i < nx_out; ++i)
        h[(i + gx) + (j + gy) * nrows] = fn(x0 + i * delta, y0 + j * delta);
    for (size_t k = 0; k < n_bnd; ++k) {
      const double lo = (static_cast<double>(k) - n_bnd) * delta, hi = ln + k * delta;
      for (size_t o = 0; o < (d0 ? ny_out : nx_out); ++o) {
        if (d0) {
          if (rank == 0) h[k + o * nrows] = fn(lo, o * delta);
          if (rank == ws - 1) h[(n_bnd + c.n_local + k) + o * nrows] = fn(hi, o * delta);
        } else {
          if (rank == 0) h[o + k * nrows] = fn(o * delta, lo);
          if (rank == ws - 1) h[o + (n_bnd + c.n_local + k) * nrows] = fn(o * delta, hi);
        }
      }
    }
    GMT_CHECK("z = h_z", gmt_rt_memcpy(z.data(), h.data(), z.bytes()));
  } else {
    GMT_CHECK("z = 0", gmt_rt_memset_async(z.data(), 0, z.bytes(), s));
    if (d0) {
      GMT_CHECK("fill", gmt_fill_poly(0, c.n_local, c.n_other, x0, delta, 0.0, delta,
                                      &zf(n_bnd, 0), nrows, s));
      if (rank == 0)
        GMT_CHECK("fill lo", gmt_fill_poly(0, n_bnd, c.n_other, -(double)n_bnd * delta, delta,
                                           0.0, delta, &zf(0, 0), nrows, s));
      if (rank == ws - 1)
        GMT_CHECK("fill hi", gmt_fill_poly(0, n_bnd, c.n_other, ln, delta, 0.0, delta,
                                           &zf(n_bnd + c.n_local, 0), nrows, s));
    } else {
      GMT_CHECK("fill", gmt_fill_poly(0, c.n_other, c.n_local, 0.0, delta, y0, delta,
                                      &zf(0, n_bnd), nrows, s));
      if (rank == 0)
        GMT_CHECK("fill lo", gmt_fill_poly(0, c.n_other, n_bnd, 0.0, delta,
                                           -(double)n_bnd * delta, delta, &zf(0, 0), nrows, s));
      if (rank == ws - 1)
        GMT_CHECK("fill hi", gmt_fill_poly(0, c.n_other, n_bnd, 0.0, delta, ln, delta,
                                           &zf(0, n_bnd + c.n_local), nrows, s));
    }
    GMT_CHECK("fill sync", gmt_rt_stream_synchronize(s));
  }

  Neighbors nb;
  const int lo = rank > 0 ? rank - 1 : -1, hi = rank < ws - 1 ? rank + 1 : -1;
  if (d0) {
    nb.west = lo;
    nb.east = hi;
  } else {
    nb.south = lo;
    nb.north = hi;
  }
  const int gx = d0 ? static_cast<int>(n_bnd) : 0, gy = d0 ? 0 : static_cast<int>(n_bnd);
  const bool pack_y = !d0 && c.buf;
  const int buf_space = c.space;
  auto halo = std::make_unique<Halo2D>(tr, zf, gx, gy, nb, pack_y, buf_space);

  if (c.debug_dump && d0 && dump) {
    dump("send", z.data(), nrows, ncols, n_bnd, n_bnd);
    dump("send", z.data(), nrows, ncols, nrows - 2 * n_bnd, n_bnd);
  }

  DerivResult r;
  r.transport = tr.name();
  r.bytes_per_exchange = halo->bytes_sent();
  // --check: the ghost blocks the exchange fills, in the fill's coordinates
  struct Ghost {
    double* p;
    int64_t nx, ny;
    double x0, y0;
  };
  std::vector<Ghost> ghosts;
  Buffer<unsigned> bad;
  if (c.check) {
    bad = Buffer<unsigned>(1, GMT_SPACE_DEVICE);
    GMT_CHECK("bad = 0", gmt_rt_memset_async(bad.data(), 0, sizeof(unsigned), s));
    const double lo_c = start - n_bnd * delta, hi_c = start + c.n_local * delta;
    if (d0) {
      if (lo >= 0) ghosts.push_back({&zf(0, 0), static_cast<int64_t>(n_bnd), static_cast<int64_t>(c.n_other), lo_c, 0.0});
      if (hi >= 0)
        ghosts.push_back({&zf(n_bnd + c.n_local, 0), static_cast<int64_t>(n_bnd), static_cast<int64_t>(c.n_other), hi_c, 0.0});
    } else {
      if (lo >= 0) ghosts.push_back({&zf(0, 0), static_cast<int64_t>(c.n_other), static_cast<int64_t>(n_bnd), 0.0, lo_c});
      if (hi >= 0)
        ghosts.push_back({&zf(0, n_bnd + c.n_local), static_cast<int64_t>(c.n_other), static_cast<int64_t>(n_bnd), 0.0, hi_c});
    }
  }
  for (int it = 0; it < c.n_warmup + c.n_iter; ++it) {
    if (c.check) GMT_CHECK("raise", gmt_add_scalar(nrows, ncols, 1.0, z.data(), nrows, s));
    if (c.check) GMT_CHECK("raise sync", gmt_rt_stream_synchronize(s));
    const double t0 = wtime();
    if (c.realloc_per_call) halo = std::make_unique<Halo2D>(tr, zf, gx, gy, nb, pack_y, buf_space);
    halo->exchange(s);
    const double t1 = wtime();
    if (c.check) {
      if (corrupt_ghost_now(rank, it) && !ghosts.empty())
        GMT_CHECK("corrupt", gmt_add_scalar(1, 1, 0.5, ghosts[0].p, nrows, s));
      for (const Ghost& g : ghosts)
        GMT_CHECK("ghost check", gmt_poly_check(g.nx, g.ny, g.x0, delta, g.y0, delta, static_cast<double>(it + 1),
                                                1e-9, g.p, nrows, bad.data(), s));
      ++r.checked_exchanges;
    }
    if (it >= c.n_warmup) {
      r.total_time += t1 - t0;
      r.iters.add(t1 - t0);
    }
    if (c.debug_dump && d0 && it == 0 && dump) {
      dump("ghost", z.data(), nrows, ncols, 0, n_bnd);
      dump("ghost", z.data(), nrows, ncols, nrows - n_bnd, n_bnd);
    }
    // "do some calculation" between exchanges (mpi_stencil2d_gt.cc:528-534)
    GMT_CHECK("stencil", gmt_stencil5_2d(c.dim, nx_out, ny_out, kDeriv5, scale, z.data(), nrows,
                                         dz.data(), nx_out, s));
    GMT_CHECK("stencil sync", gmt_rt_stream_synchronize(s));
  }

  // verification
  const int mode = d0 ? 1 : 2;
  {  // separable: dim 0's derivative 3x^2 varies along x only, dim 1's 2y along y only
    double a = 0.0;
    const size_t n_var = d0 ? nx_out : ny_out, n_rep = d0 ? ny_out : nx_out;
    for (size_t i = 0; i < n_var; ++i) {
      const double v = d0 ? 3 * (x0 + i * delta) * (x0 + i * delta) : 2 * (y0 + i * delta);
      a += v * v;
    }
    r.exact_norm = std::sqrt(a * static_cast<double>(n_rep));
  }
  if (c.host_verify) {
    std::vector<double> h(nx_out * ny_out);
    GMT_CHECK("h_dz = dz", gmt_rt_memcpy(h.data(), dz.data(), dz.bytes()));
    double acc = 0.0;
    for (size_t j = 0; j < ny_out; ++j)
      for (size_t i = 0; i < nx_out; ++i) {
        const double x = x0 + i * delta, y = y0 + j * delta;
        const double a = d0 ? 3 * x * x : 2 * y;
        const double d = h[i + j * nx_out] - a;
        acc += d * d;
      }
    r.err_norm = std::sqrt(acc);
  } else {
    // the analytic derivative overwrites z (no longer needed), then one reduction
    GMT_CHECK("fill exact", gmt_fill_poly(mode, nx_out, ny_out, x0, delta, y0, delta, z.data(),
                                          nx_out, s));
    const int64_t wn = gmt_diff_sq_workspace(nx_out, ny_out);
    Buffer<double> ws_buf(wn + 1, GMT_SPACE_DEVICE);
    GMT_CHECK("diff_sq", gmt_diff_sq(nx_out, ny_out, dz.data(), nx_out, z.data(), nx_out,
                                     ws_buf.data(), ws_buf.data() + 1, s));
    double acc = 0.0;
    GMT_CHECK("err D2H", gmt_rt_memcpy_async(&acc, ws_buf.data(), sizeof(double), s));
    GMT_CHECK("err sync", gmt_rt_stream_synchronize(s));
    r.err_norm = std::sqrt(acc);
  }
  if (c.check) {
    unsigned h = 0;
    GMT_CHECK("bad D2H", gmt_rt_memcpy_async(&h, bad.data(), sizeof(h), s));
    GMT_CHECK("bad sync", gmt_rt_stream_synchronize(s));
    r.bad_ghosts = h;
  }
  halo.reset();
  gmt_rt_stream_destroy(s);
  return r;
}

// test_sum: axis reduction of a PI/world_size-filled array to 1024 values,
// then a timed in-place all-reduce of them (mpi_stencil2d_gt.cc:574-649).
struct SumResult {
  double total_time = 0.0;
  Stats iters;
  double max_abs_err = 0.0;  // vs the analytic value (the reference does not check)
  std::string transport;
};

inline SumResult run_sum_on(int dim, int space, size_t n_local, size_t n_other, int n_iter,
                            int n_warmup, comm::Transport& tr, int world_size) {
  const size_t nrows = dim == 0 ? n_local : n_other, ncols = dim == 0 ? n_other : n_local;
  gmt_stream_t s = nullptr;
  GMT_CHECK("stream", gmt_rt_stream_create(&s, 0));
  Buffer<double> z(nrows * ncols, space);
  // PI/world_size everywhere: reuse the analytic-fill kernel with a constant
  // (mode 2 gives 2*y; y0 = PI/(2*ws), dy = 0)
  GMT_CHECK("fill", gmt_fill_poly(2, nrows, ncols, 0.0, 0.0, kPI / (2.0 * world_size), 0.0,
                                  z.data(), nrows, s));
  const size_t n_sum = n_local;  // keep the decomposed axis: 1024 values in both dims
  Buffer<double> sum(n_sum, space);
  const int64_t wn = gmt_sum_axis_workspace(dim, nrows, ncols);
  Buffer<double> wsb(wn > 0 ? wn : 1, GMT_SPACE_DEVICE);
  SumResult r;
  r.transport = tr.name();
  for (int it = 0; it < n_warmup + n_iter; ++it) {
    GMT_CHECK("sum_axis", gmt_sum_axis(dim, nrows, ncols, z.data(), nrows, sum.data(),
                                       wsb.data(), s));
    GMT_CHECK("sum sync", gmt_rt_stream_synchronize(s));
    const double t0 = wtime();
    tr.allreduce_sum(sum.data(), n_sum, s);
    GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
    const double t1 = wtime();
    if (it >= n_warmup) {
      r.total_time += t1 - t0;
      r.iters.add(t1 - t0);
    }
  }
  std::vector<double> h(n_sum);
  GMT_CHECK("h_sum = sum", gmt_rt_memcpy(h.data(), sum.data(), sum.bytes()));
  const double expect = kPI * static_cast<double>(n_other);
  for (double v : h) r.max_abs_err = std::max(r.max_abs_err, std::fabs(v - expect) / expect);
  gmt_rt_stream_destroy(s);
  return r;
}

}  // namespace apps
}  // namespace gmt
