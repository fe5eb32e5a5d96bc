// gmt_kernel_bench — A/B timing of every hand-written kernel variant.
//
// Not in the reference (it has no kernels of its own).  Times
// the gfx950 kernels with hipEvents, median of --iters launches, and prints
// the effective HBM bandwidth from the kernel's compulsory bytes:
//   daxpy      24 B/elem      (variants 1-5)
//   jacobi5    16 B/point     (variants 1-8)
//   stencil5   16 B/point     (dim 0 / dim 1, the reference's derivative)
//   copy2d     16 B/elem      (halo pack of a dim-0 face: strided 16-B reads)
// CLI: gmt_kernel_bench [--daxpy-n=N] [--jacobi-n=N] [--iters=K] [--json=FILE]
//      [--only=daxpy,jacobi,stencil,pack]
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/util.hpp"

using namespace gmt;

// --sustained=1: the mean of `iters` back-to-back launches (one event pair,
// the GPU never idles: what a solver loop sees, clocks included); default:
// the median of `iters` launches each synchronised on its own
static bool g_sustained = false;

static double time_ms(gmt_stream_t s, int iters, const std::function<void()>& f) {
  gmt_event_t e0, e1;
  GMT_CHECK("event", gmt_rt_event_create(&e0, 1));
  GMT_CHECK("event", gmt_rt_event_create(&e1, 1));
  // the process's first measurement starts from an idle GPU: without a
  // longer warm-up it read 6-12% low whatever it measured (profiles/r04_shares.md)
  static bool first = true;
  if (first) {
    first = false;
    const double t0 = wtime();
    while (wtime() - t0 < 0.2) {
      for (int w = 0; w < 4; ++w) f();
      GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
    }
  }
  for (int w = 0; w < 3; ++w) f();
  if (g_sustained) {
    GMT_CHECK("rec", gmt_rt_event_record(e0, s));
    for (int k = 0; k < iters; ++k) f();
    GMT_CHECK("rec", gmt_rt_event_record(e1, s));
    GMT_CHECK("sync", gmt_rt_event_synchronize(e1));
    float ms = 0;
    GMT_CHECK("elapsed", gmt_rt_event_elapsed_ms(&ms, e0, e1));
    gmt_rt_event_destroy(e0);
    gmt_rt_event_destroy(e1);
    return ms / iters;
  }
  Stats st;
  for (int k = 0; k < iters; ++k) {
    GMT_CHECK("rec", gmt_rt_event_record(e0, s));
    f();
    GMT_CHECK("rec", gmt_rt_event_record(e1, s));
    GMT_CHECK("sync", gmt_rt_event_synchronize(e1));
    float ms = 0;
    GMT_CHECK("elapsed", gmt_rt_event_elapsed_ms(&ms, e0, e1));
    st.add(ms);
  }
  gmt_rt_event_destroy(e0);
  gmt_rt_event_destroy(e1);
  return st.median();
}

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  const int iters = static_cast<int>(cli.geti("iters", 20));
  const std::string only = cli.get("only", "daxpy,jacobi,stencil,pack");
  const std::string json = cli.get("json", "");
  g_sustained = cli.geti("sustained", 0) != 0;
  gmt_stream_t s = nullptr;
  GMT_CHECK("stream", gmt_rt_stream_create(&s, 0));
  auto report = [&](const char* kernel, int variant, const char* shape, double ms, double bytes) {
    const double gbps = bytes / (ms * 1e-3) / 1e9;
    std::printf("%-10s v%-2d %-22s %9.4f ms  %8.1f GB/s\n", kernel, variant, shape, ms, gbps);
    JsonRecord j;
    j.add("app", "gmt_kernel_bench").add("kernel", kernel).add("variant", variant).add("shape", shape)
        .add("ms", ms).add("GBps", gbps).add("backend", gmt_rt_backend_name());
    j.append_to(json);
  };
  std::printf("# gmt_kernel_bench backend=%s iters=%d (%s)\n", gmt_rt_backend_name(), iters,
              g_sustained ? "sustained mean" : "median");

  if (only.find("daxpy") != std::string::npos) {
    const size_t n = static_cast<size_t>(cli.geti("daxpy-n", 1LL << 28));
    Buffer<double> x(n, GMT_SPACE_DEVICE), y(n, GMT_SPACE_DEVICE);
    GMT_CHECK("fill", gmt_fill_poly(1, n, 1, 0.0, 1e-9, 0.0, 0.0, x.data(), n, s));
    GMT_CHECK("fill", gmt_fill_poly(1, n, 1, 1.0, 1e-9, 0.0, 0.0, y.data(), n, s));
    char shape[64];
    std::snprintf(shape, sizeof(shape), "n=%zu", n);
    double ms = time_ms(s, iters, [&] { GMT_CHECK("daxpy", gmt_daxpy(n, 1e-3, x.data(), y.data(), s)); });
    report("daxpy", 0, shape, ms, 24.0 * n);
    ms = time_ms(s, iters, [&] { GMT_CHECK("daxpy", gmt_blas_daxpy(n, 1e-3, x.data(), y.data(), s)); });
    report("rocblas", 0, shape, ms, 24.0 * n);
  }
  if (only.find("hot") != std::string::npos) {
    // --only=hot: just the production (default) configuration of the
    // temporal-blocking kernel, `iters` launches each — the target of
    // rocprofv3 --pmc passes (profiles/r02_pmc).  --hot-k=12,20 sweeps per
    // pass, --jacobi-n=32768.
    const int64_t n = cli.geti("jacobi-n", 32768);
    const std::string ks = cli.get("hot-k", "12,20");
    for (int K = 1; K <= GMT_TB_MAX_SWEEPS; ++K) {
      if (("," + ks + ",").find("," + std::to_string(K) + ",") == std::string::npos) continue;
      const int64_t g = K, xk = ((g + 7) / 8) * 8;
      const int64_t ld2 = ((xk + n + g + 63) / 64) * 64, rows = n + 2 * g;
      Buffer<double> a(static_cast<size_t>(ld2) * rows, GMT_SPACE_DEVICE), b(a.size(), GMT_SPACE_DEVICE);
      GMT_CHECK("fill", gmt_fill_poly(0, ld2, rows, 0.0, 1e-5, 0.0, 1e-5, a.data(), ld2, s));
      GMT_CHECK("fill", gmt_fill_poly(0, ld2, rows, 0.0, 1e-5, 0.0, 1e-5, b.data(), ld2, s));
      const int64_t rect[4] = {xk, n, g, n};
      gmt_tb_opts o{K, 0, 0, 0};
      const double ms = time_ms(s, iters, [&] {
        GMT_CHECK("tb", gmt_jacobi5tb(&o, 1, rect, rect, 0, a.data(), b.data(), ld2, rows, s));
      });
      char tag[64];
      std::snprintf(tag, sizeof(tag), "%lldx%lld x%d default", (long long)n, (long long)n, K);
      report("jacobi5tb", K, tag, ms, K * 16.0 * n * n);
      std::printf("%-10s    %-22s %9.1f MLUPS\n", "", tag, K * double(n) * n / (ms * 1e-3) / 1e6);
    }
  }
  if (only.find("tb") != std::string::npos) {
    // --only=tb: temporal-blocking kernel (jacobi5tb.hip),
    // --tb-k=12,14,16 --tb-nw=1,2,4,8 --tb-seg=0 --jacobi-n=32768
    // --tb-mask=0 (Dirichlet everywhere: rule workgroups at the edges)
    // --jacobi-ny=8192 --jacobi-nx=16384 (default: n x n)
    const int64_t n = cli.geti("jacobi-n", 32768);
    // --jacobi-ny / --jacobi-nx: a rectangular domain (a strong-scaling share)
    const int64_t ny = cli.geti("jacobi-ny", n), nx = cli.geti("jacobi-nx", n);
    auto list = [&](const char* key, const char* def) {
      std::vector<int> v;
      std::string str = cli.get(key, def);
      size_t p = 0;
      while (p < str.size()) {
        size_t q = str.find(',', p);
        if (q == std::string::npos) q = str.size();
        v.push_back(std::atoi(str.substr(p, q - p).c_str()));
        p = q + 1;
      }
      return v;
    };
    const int mask = static_cast<int>(cli.geti("tb-mask", 0));
    for (int K : list("tb-k", "12,14,16")) {
      const int64_t g = K, xk = ((g + 7) / 8) * 8;
      const int64_t ld2 = ((xk + nx + g + 63) / 64) * 64, rows = ny + 2 * g;
      Buffer<double> a(static_cast<size_t>(ld2) * rows, GMT_SPACE_DEVICE), b(a.size(), GMT_SPACE_DEVICE);
      GMT_CHECK("fill", gmt_fill_poly(0, ld2, rows, 0.0, 1e-5, 0.0, 1e-5, a.data(), ld2, s));
      GMT_CHECK("fill", gmt_fill_poly(0, ld2, rows, 0.0, 1e-5, 0.0, 1e-5, b.data(), ld2, s));
      const int64_t rect[4] = {xk, nx, g, ny};
      for (int nw : list("tb-nw", "0"))
        for (int P : list("tb-p", "3"))
          for (int seg : list("tb-seg", "0")) {
            gmt_tb_opts o{K, nw, seg, 0};
            const double ms = time_ms(s, iters, [&] {
              GMT_CHECK("tb", gmt_jacobi5tb(&o, 1, rect, rect, mask, a.data(), b.data(), ld2, rows, s));
            });
            char tag[96];
            std::snprintf(tag, sizeof(tag), "%lldx%lld x%d nw%d P%d seg%d m%d", (long long)ny, (long long)nx, K, nw,
                          P, seg, mask);
            report("jacobi5tb", K, tag, ms, K * 16.0 * ny * nx);
            if (cli.geti("tb-push", 0) && K % 2 == 0 && gmt_jacobi5tb_push_supported(K)) {
              // --tb-push=1: the same pass with the inline halo exchange of a
              // one-rank periodic domain (the engine's layout: every face lands
              // in the opposite ghost ring of the output), alternated with the
              // plain pass so clock drift hits both alike
              gmt_tb_opts op = o;
              double* bb = b.data();
              const int64_t dy = ny * ld2, dx = nx;
              const double* tgt[8] = {bb + dy, bb - dy, bb + dx, bb - dx, bb + dy + dx, bb + dy - dx, bb - dy + dx, bb - dy - dx};
              for (int d = 0; d < 8; ++d) op.push[d] = tgt[d];  // GMT_PUSH_S, N, W, E, SW, SE, NW, NE
              op.push_w = g;  // even K: the faces fill the g-wide ghost ring
              for (int rep = 0; rep < 2; ++rep) {
                const double mp = time_ms(s, iters, [&] {
                  GMT_CHECK("tb push", gmt_jacobi5tb(&op, 1, rect, rect, mask, a.data(), b.data(), ld2, rows, s));
                });
                const double m0 = time_ms(s, iters, [&] {
                  GMT_CHECK("tb", gmt_jacobi5tb(&o, 1, rect, rect, mask, a.data(), b.data(), ld2, rows, s));
                });
                std::printf("%-10s    %-30s push %.4f ms  plain %.4f ms  ratio %.4f\n", "", tag, mp, m0, mp / m0);
              }
            }
            int64_t pi[6] = {};
            GMT_CHECK("plan", gmt_jacobi5tb_plan(&o, 1, rect, rect, mask, ld2, rows, pi));
            std::printf("%-10s    %-30s %9.1f MLUPS  (wgs %lld resident %lld threads %lld seg %lld x %lld vgpr %lld)\n",
                        "", tag, K * double(ny) * nx / (ms * 1e-3) / 1e6, (long long)pi[0], (long long)pi[1],
                        (long long)pi[2], (long long)pi[3], (long long)pi[4], (long long)pi[5]);
          }
    }
  }
  if (only.find("jacobi") != std::string::npos) {
    const int64_t n = cli.geti("jacobi-n", 32768);
    const int64_t xo = 8, ld = ((xo + n + 1 + 63) / 64) * 64;
    Buffer<double> u(static_cast<size_t>(ld) * (n + 2), GMT_SPACE_DEVICE), un(u.size(), GMT_SPACE_DEVICE);
    GMT_CHECK("fill", gmt_fill_poly(0, ld, n + 2, 0.0, 1e-5, 0.0, 1e-5, u.data(), ld, s));
    GMT_CHECK("fill", gmt_fill_poly(0, ld, n + 2, 0.0, 1e-5, 0.0, 1e-5, un.data(), ld, s));
    char shape[64];
    std::snprintf(shape, sizeof(shape), "%lldx%lld", (long long)n, (long long)n);
    // single sweep (the K-sweep kernel: --only=tb; A/B variants: variant_bench)
    const double ms = time_ms(s, iters, [&] {
      GMT_CHECK("jacobi", gmt_jacobi5(xo, n, 1, n, u.data(), un.data(), ld, nullptr, 0, 0.25, 0.0, nullptr, s));
    });
    report("jacobi5", 0, shape, ms, 16.0 * n * n);
  }
  if (only.find("stencil") != std::string::npos) {
    // the reference's default deriv shapes: 1028 x 524288 (dim 0), 524288 x 1028 (dim 1)
    const int64_t a = 1024, b = 512 * 1024;
    Buffer<double> in(static_cast<size_t>(a + 4) * b, GMT_SPACE_DEVICE), out(static_cast<size_t>(a) * b, GMT_SPACE_DEVICE);
    GMT_CHECK("fill", gmt_fill_poly(0, a + 4, b, 0.0, 1e-3, 0.0, 1e-3, in.data(), a + 4, s));
    const double c[5] = {1.0 / 12, -2.0 / 3, 0.0, 2.0 / 3, -1.0 / 12};
    // bytes: the input (n + 4 rows / columns) read once, the output written once
    const double bytes = 8.0 * ((a + 4) * b + a * b);
    double ms = time_ms(s, iters, [&] {
      GMT_CHECK("d0", gmt_stencil5_2d(0, a, b, c, 128.0, in.data(), a + 4, out.data(), a, s));
    });
    report("stencil5", 0, "dim0 1028->1024 x 524288", ms, bytes);
    ms = time_ms(s, iters, [&] {
      GMT_CHECK("d1", gmt_stencil5_2d(1, b, a, c, 128.0, in.data(), b, out.data(), b, s));
    });
    report("stencil5", 1, "dim1 524288 x 1028->1024", ms, bytes);
  }
  if (only.find("pack") != std::string::npos) {
    // dim-0 halo faces of the reference's field: 2 rows x 524288 columns, pitch 1028
    const int64_t ld = 1028, ny = 512 * 1024;
    Buffer<double> z(static_cast<size_t>(ld) * ny, GMT_SPACE_DEVICE), b0(2 * ny, GMT_SPACE_DEVICE),
        b1(2 * ny, GMT_SPACE_DEVICE);
    gmt_copy2d_desc d[2] = {{z.data() + 2, b0.data(), ld, 2, 2, ny}, {z.data() + 1024, b1.data(), ld, 2, 2, ny}};
    const double ms = time_ms(s, iters, [&] { GMT_CHECK("pack", gmt_copy2d_batched(2, d, 8, s)); });
    report("pack", 0, "2 faces 2x524288", ms, 2.0 * 2 * 16.0 * ny);
  }
  gmt_rt_stream_destroy(s);
  return 0;
}
