// d1_walk — HBM rate of the dim-1 (strided-axis) 5-tap derivative at the
// reference's shape (524288 columns x 1028 -> 1024 rows, fp64,
// mpi_stencil2d_gt.cc:101-110) for launch shapes that bound how many rows
// the chip touches at once (round-3 VERDICT item 6).
//
// The production kernel (LDS-DMA pipeline, stencil5_d1.hpp) walks 128-row
// segments with the XCD swizzle: every XCD works on its own row band, and
// with several segments resident per XCD the chip has ~1000 distinct 4 MiB
// rows in flight.  The variants here keep the in-flight footprint compact:
//
//   lock<NW, CPL, P>  a workgroup = NW waves side by side (NW x CPL KiB of
//                     each row), register window of 5 rows + P rows of
//                     plain 16-B loads in flight, segments of L rows, column
//                     groups fastest in blockIdx (no swizzle): with every
//                     group resident at once, the whole chip walks down
//                     the same few rows (a linear sweep of the array).
//
// Every variant is checked against a one-thread-per-point kernel with the
// same arithmetic order.  Prints ms and TB/s of compulsory bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "../kernels/common.hpp"
#include "../kernels/stencil5_d1.hpp"

using namespace gmt;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

struct C5 {
  double c[5];
};

__global__ void d1_naive(int64_t nx, int64_t ny_out, C5 c, const double* __restrict__ in,
                         double* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nx * ny_out) return;
  const int64_t y = i / nx, x = i % nx;
  const double* p = in + y * nx + x;
  out[i] = c.c[0] * p[0] + c.c[1] * p[nx] + c.c[2] * p[2 * nx] + c.c[3] * p[3 * nx] + c.c[4] * p[4 * nx];
}

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// NW waves x CPL 16-B chunks per lane: a wave covers 128 * CPL columns.
template <int NW, int CPL, int P>
__global__ __launch_bounds__(NW * 64) void d1_lock(int64_t nx, int64_t ny_out, int64_t L, int64_t ngroups, C5 c,
                                                   const double* __restrict__ in, double* __restrict__ out) {
  constexpr int R = 5 + P;  // ring: rows o .. o+4 in use, o+5 .. o+4+P in flight
  const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
  const int64_t g = blockIdx.x % ngroups, seg = blockIdx.x / ngroups;
  const int64_t x0 = (g * NW + wave) * (128 * CPL) + 2 * lane;
  const int64_t y0 = seg * L;
  const int64_t L1 = std::min<int64_t>(L, ny_out - y0);
  if (x0 >= nx || L1 <= 0) return;
  const d2* src = reinterpret_cast<const d2*>(in + y0 * nx + x0);
  d2* dst = reinterpret_cast<d2*>(out + y0 * nx + x0);
  const int64_t ld2 = nx / 2;
  const double c0 = c.c[0], c1 = c.c[1], c2 = c.c[2], c3 = c.c[3], c4 = c.c[4];
  d2 B[R][CPL];
  const int64_t nin = L1 + 4;  // input rows of the segment
  auto load = [&](int64_t r, int slot) {
    const int64_t rr = r < nin ? r : nin - 1;  // past the end: re-read the last row (unused)
#pragma unroll
    for (int j = 0; j < CPL; ++j) B[slot][j] = __builtin_nontemporal_load(src + rr * ld2 + 64 * j);
  };
  sfor<0, 4 + P>([&](auto I) { load(decltype(I)::value, decltype(I)::value); });
  for (int64_t o0 = 0; o0 < L1; o0 += R) {
    sfor<0, R>([&](auto J) {
      constexpr int j = decltype(J)::value;
      const int64_t o = o0 + j;
      load(o + 4 + P, (j + 4 + P) % R);
      if (o < L1) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const d2 v = c0 * B[j % R][k] + c1 * B[(j + 1) % R][k] + c2 * B[(j + 2) % R][k] +
                       c3 * B[(j + 3) % R][k] + c4 * B[(j + 4) % R][k];
          __builtin_nontemporal_store(v, dst + o * ld2 + 64 * k);
        }
      }
    });
  }
}

template <int CPL>
void launch_prod(int64_t nx, int64_t ny_out, const C5& c, const double* in, double* out, int64_t L) {
  using namespace gmt::d1;
  Args a{};
  a.nx = nx;
  a.ny_out = ny_out;
  a.ld_in = nx;
  a.ld_out = nx;
  for (int k = 0; k < 5; ++k) a.c[k] = c.c[k];
  a.nstrip = (nx + 128 * CPL - 1) / (128 * CPL);
  a.seg = static_cast<int>(L);
  a.nseg = (ny_out + L - 1) / L;
  a.nsteps = static_cast<int>((L + 4 + kU - 1) / kU * kU);
  const int64_t nb = (a.nstrip + kNW - 1) / kNW * a.nseg;
  const size_t smem = static_cast<size_t>(kNW) * kRS * CPL * kWave * 16;
  if (smem > 65536)
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&stencil5_d1_dma<CPL, false>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(smem)));
  stencil5_d1_dma<CPL, false><<<grid_1d(nb), kNW * kWave, smem>>>(a, in, out, nb);
  CK(hipGetLastError());
}

template <int NW, int CPL, int P>
void launch_lock(int64_t nx, int64_t ny_out, const C5& c, const double* in, double* out, int64_t L) {
  const int64_t cols = static_cast<int64_t>(NW) * 128 * CPL;
  const int64_t ng = (nx + cols - 1) / cols, nseg = (ny_out + L - 1) / L;
  d1_lock<NW, CPL, P><<<static_cast<unsigned>(ng * nseg), NW * 64>>>(nx, ny_out, L, ng, c, in, out);
  CK(hipGetLastError());
}

int main(int argc, char** argv) {
  const bool check_only = argc > 1 && std::strcmp(argv[1], "--check") == 0;
  const int64_t nx = check_only ? 8192 : 524288, ny_out = check_only ? 100 : 1024, ny_in = ny_out + 4;
  const int iters = 10;
  C5 c{{1.0 / 12, -8.0 / 12, 0.0, 8.0 / 12, -1.0 / 12}};
  double *in, *out, *ref;
  CK(hipMalloc(&in, nx * ny_in * 8));
  CK(hipMalloc(&out, nx * ny_out * 8));
  CK(hipMalloc(&ref, nx * ny_out * 8));
  {
    std::vector<double> h(nx * ny_in);
    for (int64_t i = 0; i < nx * ny_in; ++i) h[i] = std::sin(0.001 * static_cast<double>(i % 100003)) + i % 7;
    CK(hipMemcpy(in, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  }
  d1_naive<<<static_cast<unsigned>((nx * ny_out + 255) / 256), 256>>>(nx, ny_out, c, in, ref);
  CK(hipDeviceSynchronize());
  std::vector<double> hr(nx * ny_out), ho(nx * ny_out);
  CK(hipMemcpy(hr.data(), ref, hr.size() * 8, hipMemcpyDeviceToHost));
  const double bytes = static_cast<double>(nx) * (ny_in + ny_out) * 8;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int fails = 0;
  auto run = [&](const char* name, const std::function<void()>& f) {
    CK(hipMemset(out, 0, nx * ny_out * 8));
    f();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ho.data(), out, ho.size() * 8, hipMemcpyDeviceToHost));
    double err = 0;
    for (size_t i = 0; i < ho.size(); ++i) err = std::max(err, std::fabs(ho[i] - hr[i]));
    const bool ok = err <= 1e-12;
    fails += !ok;
    if (check_only) {
      std::printf("%-34s max|err| %.3g %s\n", name, err, ok ? "ok" : "FAIL");
      return;
    }
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) f();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms / iters);
      sum += ms / iters;
    }
    std::printf("%-34s %7.3f ms (mean %7.3f)  %5.2f TB/s  %s\n", name, best, sum / 3, bytes / (best * 1e-3) / 1e12,
                ok ? "" : "WRONG");
  };
  char nm[64];
  run("production DMA CPL1 L128", [&] { launch_prod<1>(nx, ny_out, c, in, out, 128); });
  for (int64_t L : {1024, 512, 256, 128}) {
    std::snprintf(nm, sizeof nm, "lock NW8 CPL1 P4 L%lld", (long long)L);
    run(nm, [&] { launch_lock<8, 1, 4>(nx, ny_out, c, in, out, L); });
    std::snprintf(nm, sizeof nm, "lock NW8 CPL1 P8 L%lld", (long long)L);
    run(nm, [&] { launch_lock<8, 1, 8>(nx, ny_out, c, in, out, L); });
    std::snprintf(nm, sizeof nm, "lock NW8 CPL2 P4 L%lld", (long long)L);
    run(nm, [&] { launch_lock<8, 2, 4>(nx, ny_out, c, in, out, L); });
    std::snprintf(nm, sizeof nm, "lock NW4 CPL2 P6 L%lld", (long long)L);
    run(nm, [&] { launch_lock<4, 2, 6>(nx, ny_out, c, in, out, L); });
    std::snprintf(nm, sizeof nm, "lock NW16 CPL1 P4 L%lld", (long long)L);
    run(nm, [&] { launch_lock<16, 1, 4>(nx, ny_out, c, in, out, L); });
  }
  std::printf("%s\n", fails ? "SOME VARIANTS WRONG" : "all variants match the naive kernel");
  return fails ? 1 : 0;
}
