// Host (CPU) implementation of the gmt/kernels.h C ABI.
//
// The CPU backend mirrors the reference's gtensor `host` device
// (/root/reference/CMakeLists.txt:59-69: the *_gt binaries compiled as plain
// C++), so that the native MPI apps and their tests run on machines with no
// GPU.  Semantics match csrc/kernels/*.hip exactly (same formulas, same
// summation structure where it matters for the err_norm checks); `stream`
// arguments are ignored — every call completes before returning.  Serial on
// purpose: several MPI ranks share the CPU in the tests, and a rank-local
// thread pool would only oversubscribe it.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <sched.h>
#include <thread>

#include <cstring>
#include <vector>

#include "gmt/kernels.h"
#include "gmt/tb_geom.h"

extern "C" {

int gmt_daxpy(int64_t n, double a, const double* x, double* y, void*) {
  for (int64_t i = 0; i < n; ++i) y[i] = a * x[i] + y[i];
  return 0;
}

int gmt_stencil5_1d(int64_t n_out, const double* c, double scale, const double* in, double* out,
                    void*) {
  const double c0 = c[0] * scale, c1 = c[1] * scale, c2 = c[2] * scale, c3 = c[3] * scale,
               c4 = c[4] * scale;
  for (int64_t i = 0; i < n_out; ++i)
    out[i] = c0 * in[i] + c1 * in[i + 1] + c2 * in[i + 2] + c3 * in[i + 3] + c4 * in[i + 4];
  return 0;
}

int gmt_stencil5_2d(int dim, int64_t nx_out, int64_t ny_out, const double* c, double scale,
                    const double* in, int64_t ld_in, double* out, int64_t ld_out, void*) {
  if (dim != 0 && dim != 1) return 1;
  const double c0 = c[0] * scale, c1 = c[1] * scale, c2 = c[2] * scale, c3 = c[3] * scale,
               c4 = c[4] * scale;
  const int64_t sx = dim == 0 ? 1 : ld_in;
  for (int64_t y = 0; y < ny_out; ++y) {
    const double* p = in + y * ld_in;
    double* q = out + y * ld_out;
    for (int64_t x = 0; x < nx_out; ++x) {
      const double* s = p + x;
      q[x] = c0 * s[0] + c1 * s[sx] + c2 * s[2 * sx] + c3 * s[3 * sx] + c4 * s[4 * sx];
    }
  }
  return 0;
}

int gmt_copy2d_batched(int n_desc, const gmt_copy2d_desc* d, int elem_bytes, void*) {
  if (n_desc < 0 || n_desc > GMT_MAX_COPY2D || (elem_bytes != 4 && elem_bytes != 8)) return 1;
  for (int k = 0; k < n_desc; ++k) {
    const char* s = static_cast<const char*>(d[k].src);
    char* t = static_cast<char*>(d[k].dst);
    const size_t row = static_cast<size_t>(d[k].width) * elem_bytes;
    for (int64_t r = 0; r < d[k].height; ++r)
      std::memmove(t + r * d[k].dst_ld * elem_bytes, s + r * d[k].src_ld * elem_bytes, row);
  }
  return 0;
}

int gmt_copy2d_batched_wgs(int n_desc, const gmt_copy2d_desc* d, int elem_bytes, int, void* s) {
  return gmt_copy2d_batched(n_desc, d, elem_bytes, s);
}

int64_t gmt_sum_axis_workspace(int, int64_t, int64_t) { return 1; }

int gmt_sum_axis(int keep_dim, int64_t nx, int64_t ny, const double* z, int64_t ld, double* out,
                 double*, void*) {
  if (keep_dim == 0) {
    for (int64_t x = 0; x < nx; ++x) out[x] = 0.0;
    for (int64_t y = 0; y < ny; ++y)
      for (int64_t x = 0; x < nx; ++x) out[x] += z[y * ld + x];
  } else if (keep_dim == 1) {
    for (int64_t y = 0; y < ny; ++y) {
      double s = 0.0;
      for (int64_t x = 0; x < nx; ++x) s += z[y * ld + x];
      out[y] = s;
    }
  } else {
    return 1;
  }
  return 0;
}

int64_t gmt_diff_sq_workspace(int64_t, int64_t) { return 1; }

int gmt_diff_sq(int64_t nx, int64_t ny, const double* a, int64_t lda, const double* b,
                int64_t ldb, double* out, double*, void*) {
  double s = 0.0;
  for (int64_t y = 0; y < ny; ++y)
    for (int64_t x = 0; x < nx; ++x) {
      const double d = a[y * lda + x] - b[y * ldb + x];
      s += d * d;
    }
  out[0] = s;
  return 0;
}

int64_t gmt_sum_workspace(int64_t) { return 1; }
int gmt_sum(int64_t n, const double* x, double* out, double*, void*) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += x[i];
  out[0] = s;
  return 0;
}

int gmt_slices_reduce(int op, int64_t n, int nslices, const double* in, double* out, void*) {
  if (n < 0 || nslices < 1 || (op != 0 && op != 1)) return 1;
  for (int64_t i = 0; i < n; ++i) {
    double v = in[i];
    for (int r = 1; r < nslices; ++r) v = op == 0 ? v + in[r * n + i] : std::max(v, in[r * n + i]);
    out[i] = v;
  }
  return 0;
}

int gmt_abs_max(int64_t nx, int64_t ny, const double* z, int64_t ld, double* out, double*, void*) {
  double m = 0.0;
  for (int64_t y = 0; y < ny; ++y)
    for (int64_t x = 0; x < nx; ++x) m = std::max(m, std::fabs(z[y * ld + x]));
  out[0] = m;
  return 0;
}

int gmt_diff_bits(int64_t nx, int64_t ny, const double* a, int64_t lda, const double* b, int64_t ldb,
                  double* out, double*, void*) {
  double m = 0.0, n = 0.0;
  for (int64_t y = 0; y < ny; ++y)
    for (int64_t x = 0; x < nx; ++x) {
      const double va = a[y * lda + x], vb = b[y * ldb + x];
      if (std::memcmp(&va, &vb, sizeof(double)) != 0) {
        n += 1.0;
        const double d = std::fabs(va - vb);
        m = std::max(m, std::isnan(d) ? HUGE_VAL : d);
      }
    }
  out[0] = m;
  out[1] = n;
  return 0;
}

// fill mode 5: the same counter-based hash as reduce.hip lattice_uniform
static double lattice_uniform(int64_t gx, int64_t gy, uint64_t seed) {
  uint64_t k = (static_cast<uint64_t>(gy + (int64_t(1) << 30)) << 32) ^ static_cast<uint64_t>(gx + (int64_t(1) << 30));
  k ^= seed;
  k += 0x9E3779B97F4A7C15ull;
  k = (k ^ (k >> 30)) * 0xBF58476D1CE4E5B9ull;
  k = (k ^ (k >> 27)) * 0x94D049BB133111EBull;
  k ^= k >> 31;
  return static_cast<double>(k >> 11) * 0x1.0p-53;
}

int gmt_poly_check(int64_t nx, int64_t ny, double x0, double dx, double y0, double dy, double offset,
                   double rtol, const double* z, int64_t ld, unsigned* bad, void*) {
  if (nx <= 0 || ny <= 0) return 0;
  if (!bad || !z || ld < nx) return 1;
  unsigned n = 0;
  for (int64_t iy = 0; iy < ny; ++iy)
    for (int64_t ix = 0; ix < nx; ++ix) {
      const double x = x0 + ix * dx, y = y0 + iy * dy;
      const double e = (x * x * x + y * y) + offset, v = z[iy * ld + ix];
      if (!(std::fabs(v - e) <= rtol * (1.0 + std::fabs(e)))) ++n;
    }
  __atomic_fetch_add(bad, n, __ATOMIC_RELAXED);
  return 0;
}

int gmt_add_scalar(int64_t nx, int64_t ny, double v, double* z, int64_t ld, void*) {
  if (nx <= 0 || ny <= 0) return 0;
  if (!z || ld < nx) return 1;
  for (int64_t iy = 0; iy < ny; ++iy)
    for (int64_t ix = 0; ix < nx; ++ix) z[iy * ld + ix] += v;
  return 0;
}

int gmt_fill_poly(int mode, int64_t nx, int64_t ny, double x0, double dx, double y0, double dy,
                  double* z, int64_t ld, void*) {
  for (int64_t j = 0; j < ny; ++j)
    for (int64_t i = 0; i < nx; ++i) {
      if (mode == 5) {
        z[j * ld + i] = lattice_uniform(static_cast<int64_t>(x0) + i, static_cast<int64_t>(y0) + j,
                                        static_cast<uint64_t>(dx));
        continue;
      }
      if (mode == 4) {  // integer lattice, see reduce.hip (built with -ffp-contract=off)
        const double xl = (x0 + static_cast<double>(i)) * dx, yl = (y0 + static_cast<double>(j)) * dy;
        z[j * ld + i] = xl * xl * xl + yl * yl;
        continue;
      }
      const double x = x0 + i * dx, y = y0 + j * dy;
      z[j * ld + i] = mode == 0 ? x * x * x + y * y : (mode == 1 ? 3 * x * x : (mode == 2 ? 2 * y : x));
    }
  return 0;
}

int64_t gmt_jacobi_resid_workspace(int64_t, int64_t) { return 2; }

static void jacobi_rect(int64_t x0, int64_t nx, int64_t y0, int64_t ny, const double* u, double* un,
                        int64_t ld, const double* f, int64_t ldf, double c0, double c1,
                        double* acc_out) {
  double acc = 0.0;
  for (int64_t y = y0; y < y0 + ny; ++y)
    for (int64_t x = x0; x < x0 + nx; ++x) {
      const double* p = u + y * ld + x;
      double o = c0 * ((p[-1] + p[1]) + (p[-ld] + p[ld]));
      if (f) o += c1 * f[y * ldf + x];
      const double d = o - p[0];
      acc += d * d;
      un[y * ld + x] = o;
    }
  if (acc_out) *acc_out = acc;
}

int gmt_jacobi5(int64_t x0, int64_t nx, int64_t y0, int64_t ny, const double* u, double* un,
                int64_t ld, const double* f, int64_t ldf, double c0, double c1, double* resid,
                void*) {
  double acc = 0.0;
  if (nx > 0 && ny > 0) jacobi_rect(x0, nx, y0, ny, u, un, ld, f, ldf, c0, c1, &acc);
  if (resid) resid[0] = acc;
  return 0;
}

int gmt_jacobi5_rects(int n_rect, const int64_t* r, const double* u, double* un, int64_t ld,
                      const double* f, int64_t ldf, double c0, double c1, void*) {
  if (n_rect > 4) return 1;
  for (int k = 0; k < n_rect; ++k)
    if (r[4 * k + 1] > 0 && r[4 * k + 3] > 0)
      jacobi_rect(r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3], u, un, ld, f, ldf, c0, c1,
                  nullptr);
  return 0;
}

static int host_xk(int K, int n_rect, const int64_t* rects, const int64_t* dom, int mask, const double* u,
                   double* un, int64_t ld) {
  const int64_t dx0 = dom[0], dx1 = dom[0] + dom[1], dy0 = dom[2], dy1 = dom[2] + dom[3];
  for (int k = 0; k < n_rect; ++k) {
    const int64_t x0 = rects[4 * k], nx = rects[4 * k + 1], y0 = rects[4 * k + 2], ny = rects[4 * k + 3];
    if (nx <= 0 || ny <= 0) continue;
    // level 0 = u on rect + K ring; each level shrinks the ring by one (same
    // ghost-side rule as the GPU kernel), the last one is written to un
    const int64_t bw = nx + 2 * K, bh = ny + 2 * K;
    std::vector<double> cur(static_cast<size_t>(bw * bh)), nxt(cur.size());
    for (int64_t j = 0; j < bh; ++j)
      for (int64_t i = 0; i < bw; ++i) {
        const int64_t y = y0 - K + j, x = x0 - K + i;
        const bool in_ring = y >= dy0 - K && y < dy1 + K && x >= dx0 - K && x < dx1 + K;
        cur[j * bw + i] = in_ring ? u[y * ld + x] : 0.0;
      }
    for (int p = 1; p <= K; ++p) {
      const int ring = K - p;
      for (int64_t j = K - ring; j < K + ny + ring; ++j)
        for (int64_t i = K - ring; i < K + nx + ring; ++i) {
          const int64_t x = x0 - K + i, y = y0 - K + j;
          const bool rx = (x >= dx0 && x < dx1) || (x < dx0 ? (mask & 1) : (mask & 2));
          const bool ry = (y >= dy0 && y < dy1) || (y < dy0 ? (mask & 4) : (mask & 8));
          const double* c = &cur[j * bw + i];
          const double v = 0.25 * ((c[-1] + c[1]) + (c[-bw] + c[bw]));
          if (p == K)
            un[y * ld + x] = v;
          else
            nxt[j * bw + i] = (rx && ry) ? v : c[0];
        }
      std::swap(cur, nxt);
    }
  }
  return 0;
}

int gmt_jacobi5tb_supported(int K) { return (K >= 1 && K <= 10) || (K > 10 && K <= GMT_TB_MAX_SWEEPS && K % 2 == 0); }
int gmt_jacobi5tb_push_supported(int K) { return gmt_jacobi5tb_supported(K) && gmt::tb::tb_push_built(K); }
int gmt_jacobi5tb_max_sweeps(int exact) { return exact ? 18 : GMT_TB_MAX_SWEEPS; }  // as the gfx950 build

// CPU backend of csrc/kernels/jacobi5tb.hip: same argument checks, reference loops
int gmt_jacobi5tb(const gmt_tb_opts* o, int n_rect, const int64_t* rects, const int64_t* dom, int mask,
                  const double* u, double* un, int64_t ld, int64_t nrows, void*) {
  const int K = o ? o->sweeps : 0;
  if (!gmt_jacobi5tb_supported(K) || n_rect < 0 || n_rect > 8 || ld <= 0) return 1;
  if (o->wg_waves < 0 || o->wg_waves > 8 || o->seg_rows < 0) return 1;
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    if (r[0] < K || r[2] < K || r[0] + r[1] + K > ld || r[2] + r[3] + K > nrows) return 1;
  }
  const bool cols = (o->signal_cols & 3) != 0;
  const bool sig = o->signal_rects > 0 || o->signal_rows > 0 || cols;
  if (o->signal_rects < 0 || o->signal_rects > n_rect || (sig && (!o->signal_count || !o->signal)) ||
      o->signal_rows < 0 || ((o->signal_rows > 0 || cols) && o->signal_rects >= n_rect) || (o->signal_cols & ~3))
    return 1;
  for (int k = 0; k < o->signal_rects + (o->signal_rows > 0 || cols ? 1 : 0); ++k)
    if (rects[4 * k + 1] <= 0 || rects[4 * k + 3] <= 0) return 1;
  if (o->signal_rows > 0) {  // the same feasibility rule as the GPU launcher
    const int rb = ((mask & 4) ? 1 : 0) + ((mask & 8) ? 1 : 0);
    if (rb == 0 || rects[4 * o->signal_rects + 3] < rb * std::max<int64_t>(32, o->signal_rows)) return 1;
  }
  const int64_t w = o->push_w;
  if (w < 0) return 1;
  if (w > 0) {  // inline halo exchange: the GPU launcher's rules (jacobi5tb.hpp launch_tb)
    bool ok = gmt::tb::tb_push_built(K) && n_rect == 1 && w <= 64 && (w & 1) == 0 && !sig && o->seg_rows == 0 && dom[1] >= w && dom[3] >= 2 * w + 2;
    for (int j = 0; ok && j < 4; ++j) ok = rects[j] == dom[j];
    const int64_t wout = gmt::tb::tb_strip_out(K);
    const auto any = [&](int d0, int d1, int d2) { return o->push[d0] || o->push[d1] || o->push[d2]; };
    if (ok && any(GMT_PUSH_W, GMT_PUSH_SW, GMT_PUSH_NW) && any(GMT_PUSH_E, GMT_PUSH_SE, GMT_PUSH_NE) &&
        (dom[1] + wout - 1) / wout < 2)
      ok = false;
    if (ok && dom[1] < wout && (dom[1] & 1)) ok = false;  // the GPU kernel's odd-edge stores
    if (!ok) return 1;
    if (o->stop && __atomic_load_n(o->stop, __ATOMIC_RELAXED) != 0) return 0;  // stopped: the pass does nothing
  }
  const int rc = host_xk(K, n_rect, rects, dom, mask, u, un, ld);
  if (rc == 0 && o->clock) {  // no shader clock on the CPU: one sample of zero cycles
    o->clock[2] += 1;
  }
  if (rc == 0 && w > 0) {
    // the faces of the output, a second time, into the neighbours' ghost cells
    const int64_t x0 = dom[0], x1 = dom[0] + dom[1], y0 = dom[2], y1 = dom[2] + dom[3];
    auto put = [&](int d, int64_t xa, int64_t xb, int64_t ya, int64_t yb) {
      double* t = const_cast<double*>(o->push[d]);
      if (!t) return;
      for (int64_t y = ya; y < yb; ++y)
        for (int64_t x = xa; x < xb; ++x) t[y * ld + x] = un[y * ld + x];
    };
    put(GMT_PUSH_S, x0, x1, y0, y0 + w);
    put(GMT_PUSH_N, x0, x1, y1 - w, y1);
    put(GMT_PUSH_W, x0, x0 + w, y0, y1);
    put(GMT_PUSH_E, x1 - w, x1, y0, y1);
    put(GMT_PUSH_SW, x0, x0 + w, y0, y0 + w);
    put(GMT_PUSH_SE, x1 - w, x1, y0, y0 + w);
    put(GMT_PUSH_NW, x0, x0 + w, y1 - w, y1);
    put(GMT_PUSH_NE, x1 - w, x1, y1 - w, y1);
  }
  if (rc == 0 && sig) __atomic_fetch_add(o->signal, uint64_t{1}, __ATOMIC_RELEASE);
  return rc;
}

// CPU backend of gmt_push_sync (csrc/kernels/ipc.hip): the same hand-over on
// memfd-shared flag words, waits bounded by GMT_WAIT_TIMEOUT_MS of wall clock
int gmt_push_sync(const uint64_t* local, uint64_t* const remote[8], int mask, uint64_t epoch, unsigned* err,
                  unsigned* stop, void*) {
  if (!local || !err || mask < 0 || mask > 255) return 1;
  for (int d = 0; d < 8; ++d)
    if (((mask >> d) & 1) && (!remote || !remote[d])) return 1;
  if (stop && __atomic_load_n(stop, __ATOMIC_RELAXED) != 0) return 0;  // stopped: no signal, no wait
  for (int d = 0; d < 8; ++d)
    if ((mask >> d) & 1) __atomic_store_n(remote[d], epoch, __ATOMIC_RELEASE);
  const char* e = std::getenv("GMT_WAIT_TIMEOUT_MS");
  const double limit = (e && std::atof(e) > 0 ? std::atof(e) : 10000.0) / 1e3;
  const auto t0 = std::chrono::steady_clock::now();
  for (int d = 0; d < 8; ++d) {
    if (!((mask >> d) & 1)) continue;
    while (__atomic_load_n(local + d, __ATOMIC_ACQUIRE) < epoch) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
        __atomic_fetch_or(err, 1u << d, __ATOMIC_RELAXED);
        if (stop) __atomic_fetch_or(stop, 1u << d, __ATOMIC_RELAXED);
        break;
      }
      std::this_thread::yield();
    }
  }
  return 0;
}

int64_t gmt_jacobi5tb_group_cols(int sweeps, int wg_waves) {
  if (!gmt_jacobi5tb_supported(sweeps)) return 0;
  // the GPU kernel's strip geometry (gmt/tb_geom.h)
  const int nw = std::min(wg_waves > 0 ? wg_waves : gmt::tb::tb_default_strips(sweeps), gmt::tb::tb_max_strips(sweeps));
  return static_cast<int64_t>(nw) * gmt::tb::tb_strip_out(sweeps);
}

// in-order CPU streams: the signal was raised before this call runs
int gmt_signal_wait(const uint64_t* signal, uint64_t* seen, unsigned* err, void*) {
  if (!signal || !seen || !err) return 1;
  const uint64_t want = __atomic_load_n(seen, __ATOMIC_RELAXED) + 1;
  if (__atomic_load_n(signal, __ATOMIC_ACQUIRE) < want) __atomic_fetch_or(err, 2u, __ATOMIC_RELAXED);
  __atomic_store_n(seen, want, __ATOMIC_RELAXED);
  return 0;
}

// the CPU backend runs every rect as one "workgroup" of one thread
int gmt_jacobi5tb_plan(const gmt_tb_opts* o, int n_rect, const int64_t* rects, const int64_t*, int, int64_t ld,
                       int64_t nrows, int64_t info[6]) {
  const int K = o ? o->sweeps : 0;
  if (!info || !gmt_jacobi5tb_supported(K) || n_rect < 0 || n_rect > 8 || ld <= 0 || nrows <= 0) return 1;
  const int64_t rows0 = n_rect > 0 ? rects[3] : 0;
  const int64_t v[6] = {n_rect, 1, 1, rows0, 1, 0};
  for (int j = 0; j < 6; ++j) info[j] = v[j];
  return 0;
}


// CPU backend of csrc/kernels/ipc.hip: the same protocol on memfd-shared
// memory between processes (flags through __atomic builtins): sends first,
// their "ready" signals, then the receives.  Waits are bounded by
// GMT_WAIT_TIMEOUT_MS (default 10 s) of wall clock, like the GPU kernel's.
int64_t gmt_ipc_table_bytes(int n_chan) {
  if (n_chan < 0) return 0;
  return static_cast<int64_t>(n_chan) * static_cast<int64_t>(sizeof(gmt_ipc_chan)) +
         (static_cast<int64_t>(n_chan) + 1) * static_cast<int64_t>(sizeof(int64_t));
}

int gmt_ipc_plan_init(gmt_ipc_plan* p, int n_send, const gmt_ipc_chan* sends, int n_recv, const gmt_ipc_chan* recvs) {
  if (!p || !p->table || n_send < 0 || n_recv < 0 || n_send + n_recv < 1) return 1;
  auto* c = static_cast<gmt_ipc_chan*>(p->table);
  for (int k = 0; k < n_send + n_recv; ++k) {
    c[k] = k < n_send ? sends[k] : recvs[k - n_send];
    if (c[k].bytes < 0 || c[k].src_run < 0 || c[k].dst_run < 0) return 1;
    if (c[k].src_run && c[k].dst_run && c[k].src_run != c[k].dst_run) return 1;
  }
  p->n_send = n_send;
  p->n_recv = n_recv;
  p->send_chunks = n_send;
  p->recv_chunks = n_recv;
  return 0;
}

int gmt_ipc_exchange(const gmt_ipc_plan* p, void*) {
  if (!p || !p->table || !p->epoch || !p->counters || !p->err || p->n_send < 0 || p->n_recv < 0 ||
      p->n_send + p->n_recv < 1)
    return 1;
  static const double limit_s = [] {
    const char* e = std::getenv("GMT_WAIT_TIMEOUT_MS");
    const long ms = e && std::atol(e) > 0 ? std::atol(e) : 10000;
    return ms * 1e-3;
  }();
  const auto* chan = static_cast<const gmt_ipc_chan*>(p->table);
  const uint64_t e = __atomic_load_n(p->epoch, __ATOMIC_ACQUIRE) + 1;
  auto run = [&](int k0, int n, uint64_t lag) {
    for (int k = k0; k < k0 + n; ++k) {
      const gmt_ipc_chan& c = chan[k];
      if (c.wait && e > lag && __atomic_load_n(p->err, __ATOMIC_RELAXED) == 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (long it = 0; __atomic_load_n(c.wait, __ATOMIC_ACQUIRE) < e - lag; ++it) {
          if (it > 1000) {
            sched_yield();
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) {
              __atomic_store_n(p->err, static_cast<unsigned>(k + 1), __ATOMIC_RELAXED);
              break;
            }
          }
        }
      }
      char* d = static_cast<char*>(c.dst) + (e & 1) * c.dst_stride;
      const char* s = static_cast<const char*>(c.src) + (e & 1) * c.src_stride;
      if (c.src_run == 0 && c.dst_run == 0) {
        std::memcpy(d, s, static_cast<size_t>(c.bytes));
      } else {  // one side strided: run by run (both runs equal the face's width)
        const int64_t run = c.src_run ? c.src_run : c.dst_run;
        for (int64_t o = 0, r = 0; o < c.bytes; o += run, ++r)
          std::memcpy(d + (c.dst_run ? r * c.dst_ld : o), s + (c.src_run ? r * c.src_ld : o),
                      static_cast<size_t>(std::min<int64_t>(run, c.bytes - o)));
      }
    }
    for (int k = k0; k < k0 + n; ++k)
      if (chan[k].signal) __atomic_store_n(chan[k].signal, e, __ATOMIC_RELEASE);
  };
  run(0, p->n_send, 2);
  run(p->n_send, p->n_recv, 0);
  __atomic_store_n(p->epoch, e, __ATOMIC_RELEASE);
  return 0;
}

// packed doubles of a strided chunk <-> its contiguous run (stage.hip strided_part)
static void strided_chunk(const gmt_stage_chunk& c, bool gather) {
  const int64_t n = c.bytes / 8;
  double* run = gather ? static_cast<double*>(c.dst) : const_cast<double*>(static_cast<const double*>(c.src));
  for (int64_t t = 0; t < n; ++t) {
    const int64_t e = c.first + t, col = e / c.rows, row = e - col * c.rows;
    double* f = c.block + row + col * c.ld;
    if (gather) run[t] = *f;
    else *f = run[t];
  }
}

// CPU backend of csrc/kernels/stage.hip: copy, then publish each chunk's flag
int gmt_stage_copy(int n_chunks, const gmt_stage_chunk* chunks, unsigned*, uint64_t* flags, uint64_t value, int wgs,
                   void*) {
  if (n_chunks < 0 || wgs < 1 || (n_chunks > 0 && (!chunks || !flags))) return 1;
  for (int k = 0; k < n_chunks; ++k) {
    if (chunks[k].rows > 0) strided_chunk(chunks[k], true);
    else if (chunks[k].bytes > 0) std::memcpy(chunks[k].dst, chunks[k].src, static_cast<size_t>(chunks[k].bytes));
    __atomic_store_n(flags + k, value, __ATOMIC_RELEASE);
  }
  return 0;
}

int gmt_stage_scatter(int n_chunks, const gmt_stage_chunk* chunks, int wgs_per_chunk, void*) {
  if (n_chunks < 0 || wgs_per_chunk < 1 || (n_chunks > 0 && !chunks)) return 1;
  for (int k = 0; k < n_chunks; ++k) {
    if (chunks[k].rows > 0) strided_chunk(chunks[k], false);
    else if (chunks[k].bytes > 0) std::memcpy(chunks[k].dst, chunks[k].src, static_cast<size_t>(chunks[k].bytes));
  }
  return 0;
}

const char* gmt_error_string(int err) {
  switch (err) {
    case 0: return "success";
    case 1: return "invalid value";
    case 2: return "out of memory";
    case 3: return "not supported by the host backend";
    case 4: return "not ready";
    default: return "unknown host-backend error";
  }
}
int gmt_device_synchronize(void) { return 0; }
const char* gmt_build_info(void) {
  return "libgmt host (CPU) backend: daxpy, stencil5 1d/2d, jacobi5, copy2d_batched, sum_axis, "
         "diff_sq, fill_poly; built " __DATE__ " " __TIME__;
}

}  // extern "C"

// the CPU backend has one "XCD": every workgroup on 0
extern "C" int gmt_xcd_of_workgroups(int n, unsigned* out, void*) {
  if (n < 1 || n > 4096 || !out) return 1;
  for (int i = 0; i < n; ++i) out[i] = 0;
  return 0;
}
