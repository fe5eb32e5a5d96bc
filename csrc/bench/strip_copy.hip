// strip_copy — HBM rate of the temporal-blocking Jacobi kernel's access
// pattern without its arithmetic (gfx950).
//
// The pass reads a field of R rows x C doubles once and writes it once, but
// every wave walks DOWN a 128-column strip (one 1 KiB row piece per step)
// for L rows instead of streaming consecutive memory.  This harness copies
// an R x C array (C = 32832, the engine's 32768^2 row pitch) with:
//   linear  : each wave copies 16 consecutive 1 KiB pieces (DAXPY-like)
//   strip   : a wave per (128-column strip, L-row segment), loads P rows ahead
//             into registers, 16-B loads, 16-B nontemporal stores
//   strip2  : the same with 256-column strips (2 KiB per row and step)
// and prints TB/s of (read + write) bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);      \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

__global__ __launch_bounds__(256) void k_linear(int64_t n2, const d2* __restrict__ x, d2* __restrict__ y) {
  const int64_t base = (static_cast<int64_t>(blockIdx.x) * 256 + (threadIdx.x & ~63)) * 16 + (threadIdx.x & 63);
  d2 v[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) v[u] = base + u * 64 < n2 ? x[base + u * 64] : d2{0, 0};
#pragma unroll
  for (int u = 0; u < 16; ++u)
    if (base + u * 64 < n2) __builtin_nontemporal_store(v[u], y + base + u * 64);
}

// one wave = W pieces of 64 lanes x 16 B side by side (W = 1: 128 columns)
template <int W, int P>
__global__ __launch_bounds__(256) void k_strip(int64_t rows, int64_t ld2, int64_t nstrip, int64_t L,
                                               const d2* __restrict__ x, d2* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = static_cast<int64_t>(blockIdx.x) * 4 + threadIdx.x / 64;
  const int64_t strip = wid % nstrip, seg = wid / nstrip;
  const int64_t y0 = seg * L;
  if (y0 >= rows) return;
  const int64_t y1 = y0 + L < rows ? y0 + L : rows;
  const int64_t col = strip * 64 * W + lane;
  d2 q[P][W];
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int w = 0; w < W; ++w) q[p][w] = y0 + p < y1 ? x[(y0 + p) * ld2 + col + 64 * w] : d2{0, 0};
  for (int64_t r = y0; r < y1; r += P) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if (r + p < y1) {
#pragma unroll
        for (int w = 0; w < W; ++w) __builtin_nontemporal_store(q[p][w], y + (r + p) * ld2 + col + 64 * w);
      }
      const int64_t rn = r + p + P;
#pragma unroll
      for (int w = 0; w < W; ++w) q[p][w] = rn < y1 ? x[rn * ld2 + col + 64 * w] : d2{0, 0};
    }
  }
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? std::atoll(argv[1]) : 32768;
  const int64_t ld = 32832, ld2 = ld / 2;
  const int64_t n2 = rows * ld2;
  d2 *x, *y;
  CK(hipMalloc(&x, n2 * sizeof(d2)));
  CK(hipMalloc(&y, n2 * sizeof(d2)));
  CK(hipMemset(x, 0, n2 * sizeof(d2)));
  CK(hipMemset(y, 0, n2 * sizeof(d2)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("%-28s %8.3f ms  %6.2f TB/s\n", name, best, 2.0 * n2 * 16 / (best * 1e-3) / 1e12);
  };
  timeit("linear 16 KiB per wave", [&] { k_linear<<<(n2 + 4095) / 4096, 256>>>(n2, x, y); });
  for (int64_t L : {192, 384, 1024, 4096}) {
    char name[64];
    {
      const int64_t ns = ld2 / 64, nw = ns * ((rows + L - 1) / L);
      std::snprintf(name, sizeof(name), "strip 128 col L=%lld P=4", (long long)L);
      timeit(name, [&] { k_strip<1, 4><<<(nw + 3) / 4, 256>>>(rows, ld2, ns, L, x, y); });
      std::snprintf(name, sizeof(name), "strip 128 col L=%lld P=8", (long long)L);
      timeit(name, [&] { k_strip<1, 8><<<(nw + 3) / 4, 256>>>(rows, ld2, ns, L, x, y); });
    }
    {
      const int64_t ns = ld2 / 128, nw = ns * ((rows + L - 1) / L);
      std::snprintf(name, sizeof(name), "strip 256 col L=%lld P=4", (long long)L);
      timeit(name, [&] { k_strip<2, 4><<<(nw + 3) / 4, 256>>>(rows, ld2, ns, L, x, y); });
    }
  }
  CK(hipFree(x));
  CK(hipFree(y));
  return 0;
}
