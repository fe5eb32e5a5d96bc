// Shared body of `daxpy` and `daxpy_nvtx` (single process, no MPI).
//
// Reference: daxpy.cu:35-94 and daxpy_nvtx.cu (same program + NVTX ranges
// copyInput / cublasDaxpy / copyOutput and cudaProfilerStart/Stop).
// x[i] = i+1, y[i] = -(i+1), y <- 2x + y = x, so SUM = n(n+1)/2
// (524800.000000 at the reference's n = 1024).
//
// Added (not in the reference): --n=N (BASELINE config "daxpy N=2^28 fp64 on
// one MI355X"), --iters=K timed repetitions with hipEvents -> GB/s at 24 B per
// element, --rocblas to cross-check against rocBLAS (the reference's cuBLAS),
// --json=FILE.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/util.hpp"

namespace gmt {
namespace apps {

inline int daxpy_main(int argc, char** argv, bool traced) {
  Cli cli(argc, argv);
  const size_t n = static_cast<size_t>(cli.geti("n", 1024));
  const int iters = static_cast<int>(cli.geti("iters", 0));
  const bool rocblas = cli.flag("rocblas");
  const bool print_all = cli.has("print") ? cli.flag("print") : n <= 4096;
  const double a = 2.0;

  if (traced) gmt_profiler_start();
  std::vector<double> x(n), y(n);
  for (size_t i = 0; i < n; ++i) {
    x[i] = static_cast<double>(i + 1);
    y[i] = -static_cast<double>(i + 1);
  }
  Buffer<double> d_x(n, GMT_SPACE_DEVICE), d_y(n, GMT_SPACE_DEVICE);
  {
    auto r = traced ? new TraceRange("copyInput") : nullptr;
    GMT_CHECK("d_x = x", gmt_rt_memcpy(d_x.data(), x.data(), n * sizeof(double)));
    GMT_CHECK("d_y = y", gmt_rt_memcpy(d_y.data(), y.data(), n * sizeof(double)));
    delete r;
  }
  {
    auto r = traced ? new TraceRange("cublasDaxpy") : nullptr;
    if (rocblas)
      GMT_CHECK("daxpy", gmt_blas_daxpy(n, a, d_x.data(), d_y.data(), nullptr));
    else
      GMT_CHECK("daxpy", gmt_daxpy(n, a, d_x.data(), d_y.data(), nullptr));
    GMT_CHECK("daxpy sync", gmt_rt_device_synchronize());
    delete r;
  }
  {
    auto r = traced ? new TraceRange("copyOutput") : nullptr;
    GMT_CHECK("y = d_y", gmt_rt_memcpy(y.data(), d_y.data(), n * sizeof(double)));
    GMT_CHECK("y = d_y sync", gmt_rt_device_synchronize());
    delete r;
  }
  double sum = 0.0;
  for (size_t i = 0; i < n; ++i) {
    if (print_all) std::printf("%f\n", y[i]);
    sum += y[i];
  }
  std::printf("SUM = %f\n", sum);

  if (iters > 0) {
    gmt_stream_t s = nullptr;
    gmt_event_t e0, e1;
    GMT_CHECK("stream", gmt_rt_stream_create(&s, 0));
    GMT_CHECK("event", gmt_rt_event_create(&e0, 1));
    GMT_CHECK("event", gmt_rt_event_create(&e1, 1));
    for (int w = 0; w < 3; ++w) GMT_CHECK("warmup", gmt_daxpy(n, a, d_x.data(), d_y.data(), s));
    Stats st;
    for (int k = 0; k < iters; ++k) {
      GMT_CHECK("rec", gmt_rt_event_record(e0, s));
      if (rocblas)
        GMT_CHECK("daxpy", gmt_blas_daxpy(n, a, d_x.data(), d_y.data(), s));
      else
        GMT_CHECK("daxpy", gmt_daxpy(n, a, d_x.data(), d_y.data(), s));
      GMT_CHECK("rec", gmt_rt_event_record(e1, s));
      GMT_CHECK("sync", gmt_rt_event_synchronize(e1));
      float ms = 0;
      GMT_CHECK("elapsed", gmt_rt_event_elapsed_ms(&ms, e0, e1));
      st.add(ms * 1e-3);
    }
    const double bytes = 24.0 * n;
    std::printf("# DAXPY n=%zu impl=%s backend=%s: median %.4f ms min %.4f ms -> %.1f GB/s (best %.1f)\n",
                n, rocblas ? "rocblas" : "gmt", gmt_rt_backend_name(), st.median() * 1e3,
                st.min() * 1e3, bytes / st.median() / 1e9, bytes / st.min() / 1e9);
    JsonRecord j;
    j.add("app", traced ? "daxpy_nvtx" : "daxpy").add("n", n).add("impl", rocblas ? "rocblas" : "gmt")
        .add("backend", gmt_rt_backend_name()).add("iters", iters)
        .add("ms_median", st.median() * 1e3).add("ms_min", st.min() * 1e3)
        .add("GBps", bytes / st.median() / 1e9).add("sum", sum);
    j.append_to(cli.get("json", ""));
    gmt_rt_event_destroy(e0);
    gmt_rt_event_destroy(e1);
    gmt_rt_stream_destroy(s);
  }
  if (traced) gmt_profiler_stop();
  return EXIT_SUCCESS;
}

}  // namespace apps
}  // namespace gmt
