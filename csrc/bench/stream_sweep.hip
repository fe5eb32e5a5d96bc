// stream_sweep — tuning harness for the HBM-bound kernels on gfx950.
//
// Standalone (not linked into libgmt): sweeps launch geometry and cache
// policy of (a) a plain 16-B copy (the roofline reference, MI355X guide:
// 6.29 TB/s measured float4 copy), (b) DAXPY and (c) the Jacobi sliding
// window, and prints effective GB/s.  The winners become the defaults in
// csrc/kernels/*.hip; the numbers go to profiles/.
//   build: make sweep     run: build/bench/stream_sweep [n_daxpy] [n_jacobi]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                  \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

template <bool NT>
__device__ __forceinline__ d2 ldv(const double* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const d2*>(p));
  return *reinterpret_cast<const d2*>(p);
}
template <bool NT>
__device__ __forceinline__ void stv(double* p, d2 v) {
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<d2*>(p));
  else
    *reinterpret_cast<d2*>(p) = v;
}

// ---------------------------------------------------------------- copy / daxpy
template <int B, int U, bool NTL, bool NTS, bool AXPY>
__global__ __launch_bounds__(B) void k_stream(int64_t n2, double a, const double* __restrict__ x,
                                              double* __restrict__ y) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * (B * U) + threadIdx.x;
  d2 xv[U], yv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * B;
    if (i < n2) {
      xv[u] = ldv<NTL>(x + 2 * i);
      if (AXPY) yv[u] = ldv<NTL>(y + 2 * i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * B;
    if (i < n2) stv<NTS>(y + 2 * i, AXPY ? a * xv[u] + yv[u] : xv[u]);
  }
}

template <int B, int U, bool NTL, bool NTS, bool AXPY>
__global__ __launch_bounds__(B) void k_stream_gs(int64_t n2, double a, const double* __restrict__ x,
                                                 double* __restrict__ y) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * B * U;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * (B * U) + threadIdx.x; base < n2;
       base += stride) {
    d2 xv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * B;
      if (i < n2) {
        xv[u] = ldv<NTL>(x + 2 * i);
        if (AXPY) yv[u] = ldv<NTL>(y + 2 * i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * B;
      if (i < n2) stv<NTS>(y + 2 * i, AXPY ? a * xv[u] + yv[u] : xv[u]);
    }
  }
}

// ---------------------------------------------------------------- jacobi
// block of B threads covers 2*B columns x R rows; lane owns 2 columns
template <int B, int R, bool NTS, bool SW>
__global__ __launch_bounds__(B) void k_jacobi(int64_t x0, int64_t nx, int64_t ny,
                                              const double* __restrict__ u, double* __restrict__ un,
                                              int64_t ld, int64_t nbx, int64_t nblocks) {
  int64_t t = blockIdx.x;
  if (SW) {  // XCD-aware: consecutive tiles on one XCD
    const int64_t q = nblocks / 8, r = nblocks % 8, xcd = t % 8, k = t / 8;
    t = xcd * q + (xcd < r ? xcd : r) + k;
  }
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t xr = (bx * B + threadIdx.x) * 2;
  if (xr >= nx) return;
  const int64_t y0 = 1 + by * R;
  const int64_t rows = (ny + 1 - y0) < R ? (ny + 1 - y0) : R;
  const double* p = u + (y0 - 1) * ld + x0 + xr;
  double* q = un + y0 * ld + x0 + xr;
  d2 n = ldv<false>(p), c = ldv<false>(p + ld);
  for (int64_t r = 0; r < rows; ++r) {
    const double* pc = p + (r + 1) * ld;
    const d2 s = ldv<false>(pc + ld);
    const double w = pc[-1], e = pc[2];
    d2 o;
    o.x = 0.25 * ((w + c.y) + (n.x + s.x));
    o.y = 0.25 * ((c.x + e) + (n.y + s.y));
    stv<NTS>(q + r * ld, o);
    n = c;
    c = s;
  }
}

// one output pair per thread, no register reuse: vertical reuse comes from
// L2 (rows y-1, y, y+1 are fetched by neighbouring threads of the same or
// adjacent blocks), like a plain copy kernel every thread is short-lived
template <int TY, bool NTS, bool NTL>
__global__ __launch_bounds__(64 * TY) void k_jacobi_pt(int64_t x0, int64_t nx, int64_t ny,
                                                     const double* __restrict__ u,
                                                     double* __restrict__ un, int64_t ld,
                                                     int64_t nbx, int64_t nblocks) {
  int64_t t = blockIdx.x;
  const int64_t q = nblocks / 8, r = nblocks % 8, xcd = t % 8, k = t / 8;
  t = xcd * q + (xcd < r ? xcd : r) + k;
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t xr = (bx * 64 + (threadIdx.x & 63)) * 2;
  const int64_t y = 1 + by * TY + (threadIdx.x >> 6);
  if (xr >= nx || y > ny) return;
  const double* pc = u + y * ld + x0 + xr;
  const d2 c = ldv<false>(pc), n = ldv<NTL>(pc - ld), s = ldv<NTL>(pc + ld);
  const double w = pc[-1], e = pc[2];
  d2 o;
  o.x = 0.25 * ((w + c.y) + (n.x + s.x));
  o.y = 0.25 * ((c.x + e) + (n.y + s.y));
  stv<NTS>(un + y * ld + x0 + xr, o);
}

// sliding window with an explicit software prefetch of D rows
template <int B, int R, int D, bool NTS>
__global__ __launch_bounds__(B) void k_jacobi_pf(int64_t x0, int64_t nx, int64_t ny,
                                                 const double* __restrict__ u, double* __restrict__ un,
                                                 int64_t ld, int64_t nbx, int64_t nblocks) {
  int64_t t = blockIdx.x;
  const int64_t q = nblocks / 8, rr = nblocks % 8, xcd = t % 8, k = t / 8;
  t = xcd * q + (xcd < rr ? xcd : rr) + k;
  const int64_t bx = t % nbx, by = t / nbx;
  const int64_t xr = (bx * B + threadIdx.x) * 2;
  if (xr >= nx) return;
  const int64_t y0 = 1 + by * R;
  if (y0 + R - 1 > ny) return;  // sweep harness: ny % R == 0
  const double* p = u + (y0 - 1) * ld + x0 + xr;
  double* qo = un + y0 * ld + x0 + xr;
  d2 buf[R + 2];
  double wb[R], eb[R];
#pragma unroll
  for (int i = 0; i < R + 2; ++i) buf[i] = ldv<false>(p + i * ld);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    wb[i] = p[(i + 1) * ld - 1];
    eb[i] = p[(i + 1) * ld + 2];
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    d2 o;
    o.x = 0.25 * ((wb[i] + buf[i + 1].y) + (buf[i].x + buf[i + 2].x));
    o.y = 0.25 * ((buf[i + 1].x + eb[i]) + (buf[i].y + buf[i + 2].y));
    stv<NTS>(qo + i * ld, o);
  }
  (void)D;
}

template <int B, bool NTL, bool NTS>
__global__ __launch_bounds__(B) void k_daxpy4(int64_t n4, double a, const double* __restrict__ x,
                                              double* __restrict__ y) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * B + threadIdx.x;
  if (i >= n4) return;
  const d2 x0 = ldv<NTL>(x + 4 * i), x1 = ldv<NTL>(x + 4 * i + 2);
  const d2 y0 = ldv<false>(y + 4 * i), y1 = ldv<false>(y + 4 * i + 2);
  stv<NTS>(y + 4 * i, a * x0 + y0);
  stv<NTS>(y + 4 * i + 2, a * x1 + y1);
}

// ---------------------------------------------------------------- timing
template <typename F>
static float time_ms(F f, int iters = 15) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  std::vector<float> v;
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return v[v.size() / 2];
}

static int g_cus = 256;

template <int B, int U, bool NTL, bool NTS, bool AXPY>
static void run_stream(const char* tag, int64_t n, double* x, double* y, int gs_per_cu) {
  const int64_t n2 = n / 2;
  float ms;
  if (gs_per_cu == 0) {
    const int64_t nb = (n2 + B * U - 1) / (B * U);
    ms = time_ms([&] { k_stream<B, U, NTL, NTS, AXPY><<<nb, B>>>(n2, 1.0001, x, y); });
  } else {
    const int64_t nb = static_cast<int64_t>(g_cus) * gs_per_cu;
    ms = time_ms([&] { k_stream_gs<B, U, NTL, NTS, AXPY><<<nb, B>>>(n2, 1.0001, x, y); });
  }
  CK(hipGetLastError());
  const double bytes = (AXPY ? 24.0 : 16.0) * n;
  std::printf("%-6s B=%4d U=%d ntl=%d nts=%d grid=%-5s %8.4f ms %8.1f GB/s\n", tag, B, U, NTL, NTS,
              gs_per_cu ? (std::to_string(gs_per_cu) + "/CU").c_str() : "tile", ms,
              bytes / (ms * 1e-3) / 1e9);
}

template <int B, int R, bool NTS, bool SW>
static void run_jacobi(int64_t n, int64_t ld, double* u, double* un) {
  const int64_t nbx = (n + 2 * B - 1) / (2 * B), nb = nbx * ((n + R - 1) / R);
  const float ms = time_ms([&] { k_jacobi<B, R, NTS, SW><<<nb, B>>>(8, n, n, u, un, ld, nbx, nb); });
  CK(hipGetLastError());
  std::printf("jacobi B=%4d R=%3d nts=%d swz=%d ld=%lld %8.4f ms %8.1f GB/s\n", B, R, NTS, SW,
              (long long)ld, ms, 16.0 * n * n / (ms * 1e-3) / 1e9);
}

template <int TY, bool NTS, bool NTL>
static void run_jacobi_pt(int64_t n, int64_t ld, double* u, double* un) {
  const int64_t nbx = (n + 127) / 128, nb = nbx * ((n + TY - 1) / TY);
  const float ms = time_ms([&] { k_jacobi_pt<TY, NTS, NTL><<<nb, 64 * TY>>>(8, n, n, u, un, ld, nbx, nb); });
  CK(hipGetLastError());
  std::printf("jac_pt TY=%2d nts=%d ntl=%d              %8.4f ms %8.1f GB/s\n", TY, NTS, NTL, ms,
              16.0 * n * n / (ms * 1e-3) / 1e9);
}

template <int B, int R, bool NTS>
static void run_jacobi_pf(int64_t n, int64_t ld, double* u, double* un) {
  const int64_t nbx = (n + 2 * B - 1) / (2 * B), nb = nbx * ((n + R - 1) / R);
  const float ms = time_ms([&] { k_jacobi_pf<B, R, 0, NTS><<<nb, B>>>(8, n, n, u, un, ld, nbx, nb); });
  CK(hipGetLastError());
  std::printf("jac_pf B=%4d R=%2d nts=%d              %8.4f ms %8.1f GB/s\n", B, R, NTS, ms,
              16.0 * n * n / (ms * 1e-3) / 1e9);
}

template <int B, bool NTL, bool NTS>
static void run_daxpy4(int64_t n, double* x, double* y) {
  const int64_t n4 = n / 4, nb = (n4 + B - 1) / B;
  const float ms = time_ms([&] { k_daxpy4<B, NTL, NTS><<<nb, B>>>(n4, 1.0001, x, y); });
  CK(hipGetLastError());
  std::printf("daxpy4 B=%4d ntl=%d nts=%d                %8.4f ms %8.1f GB/s\n", B, NTL, NTS, ms,
              24.0 * n / (ms * 1e-3) / 1e9);
}

static int sweep2(int64_t n, int64_t nj) {
  double *x, *y;
  CK(hipMalloc(&x, n * 8));
  CK(hipMalloc(&y, n * 8));
  CK(hipMemset(x, 0, n * 8));
  CK(hipMemset(y, 0, n * 8));
  run_stream<256, 1, false, false, false>("copy", n, x, y, 0);
  run_stream<256, 1, false, true, false>("copy", n, x, y, 0);
  run_stream<256, 1, false, false, true>("daxpy", n, x, y, 0);
  run_stream<128, 1, false, false, true>("daxpy", n, x, y, 0);
  run_stream<64, 1, false, false, true>("daxpy", n, x, y, 0);
  run_stream<128, 1, true, false, true>("daxpy", n, x, y, 0);
  run_stream<128, 1, false, true, true>("daxpy", n, x, y, 0);
  run_stream<128, 1, true, true, true>("daxpy", n, x, y, 0);
  run_stream<256, 1, true, true, true>("daxpy", n, x, y, 0);
  run_daxpy4<256, false, false>(n, x, y);
  run_daxpy4<128, false, false>(n, x, y);
  run_daxpy4<256, true, false>(n, x, y);
  run_daxpy4<256, false, true>(n, x, y);
  run_daxpy4<64, false, false>(n, x, y);
  CK(hipFree(x));
  CK(hipFree(y));
  const int64_t ld = ((8 + nj + 1 + 63) / 64) * 64;
  double *u, *un;
  CK(hipMalloc(&u, (nj + 2) * ld * 8));
  CK(hipMalloc(&un, (nj + 2) * ld * 8));
  CK(hipMemset(u, 0, (nj + 2) * ld * 8));
  CK(hipMemset(un, 0, (nj + 2) * ld * 8));
  run_jacobi<256, 32, true, true>(nj, ld, u, un);
  run_jacobi<256, 16, true, true>(nj, ld, u, un);
  run_jacobi<512, 16, true, true>(nj, ld, u, un);
  run_jacobi<1024, 16, true, true>(nj, ld, u, un);
  run_jacobi<1024, 8, true, true>(nj, ld, u, un);
  run_jacobi<1024, 32, true, true>(nj, ld, u, un);
  run_jacobi_pt<1, false, false>(nj, ld, u, un);
  run_jacobi_pt<1, true, false>(nj, ld, u, un);
  run_jacobi_pt<4, true, false>(nj, ld, u, un);
  run_jacobi_pt<4, false, false>(nj, ld, u, un);
  run_jacobi_pt<8, true, false>(nj, ld, u, un);
  run_jacobi_pt<16, true, false>(nj, ld, u, un);
  run_jacobi_pt<4, true, true>(nj, ld, u, un);
  run_jacobi_pf<256, 8, true>(nj, ld, u, un);
  run_jacobi_pf<256, 16, true>(nj, ld, u, un);
  run_jacobi_pf<128, 16, true>(nj, ld, u, un);
  run_jacobi_pf<512, 8, true>(nj, ld, u, un);
  run_jacobi_pf<64, 16, true>(nj, ld, u, un);
  CK(hipFree(u));
  CK(hipFree(un));
  return 0;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : (1LL << 28);
  const int64_t nj = argc > 2 ? std::atoll(argv[2]) : 32768;
  if (argc > 3 && argv[3][0] == '2') {
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::printf("# stream_sweep 2: n=%lld, jacobi %lld^2\n", (long long)n, (long long)nj);
    return sweep2(n, nj);
  }
  CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::printf("# stream_sweep: %d CUs, n=%lld, jacobi %lld^2\n", g_cus, (long long)n, (long long)nj);
  double *x, *y;
  CK(hipMalloc(&x, n * 8));
  CK(hipMalloc(&y, n * 8));
  CK(hipMemset(x, 0, n * 8));
  CK(hipMemset(y, 0, n * 8));
  // copy roofline
  run_stream<256, 1, false, false, false>("copy", n, x, y, 0);
  run_stream<256, 4, false, false, false>("copy", n, x, y, 0);
  run_stream<256, 4, true, true, false>("copy", n, x, y, 0);
  run_stream<256, 1, false, true, false>("copy", n, x, y, 0);
  run_stream<512, 2, false, false, false>("copy", n, x, y, 0);
  run_stream<1024, 1, false, false, false>("copy", n, x, y, 0);
  run_stream<256, 4, false, false, false>("copy", n, x, y, 4);
  run_stream<256, 2, false, false, false>("copy", n, x, y, 8);
  // daxpy
  run_stream<256, 1, false, false, true>("daxpy", n, x, y, 0);
  run_stream<256, 2, false, false, true>("daxpy", n, x, y, 0);
  run_stream<256, 4, false, false, true>("daxpy", n, x, y, 0);
  run_stream<256, 4, true, false, true>("daxpy", n, x, y, 0);
  run_stream<256, 4, false, true, true>("daxpy", n, x, y, 0);
  run_stream<256, 2, false, true, true>("daxpy", n, x, y, 0);
  run_stream<256, 1, false, true, true>("daxpy", n, x, y, 0);
  run_stream<512, 1, false, false, true>("daxpy", n, x, y, 0);
  run_stream<512, 2, false, false, true>("daxpy", n, x, y, 0);
  run_stream<1024, 1, false, false, true>("daxpy", n, x, y, 0);
  run_stream<1024, 2, false, false, true>("daxpy", n, x, y, 0);
  run_stream<256, 2, false, false, true>("daxpy", n, x, y, 4);
  run_stream<256, 2, false, false, true>("daxpy", n, x, y, 8);
  run_stream<256, 4, false, false, true>("daxpy", n, x, y, 2);
  run_stream<512, 2, false, false, true>("daxpy", n, x, y, 4);
  run_stream<1024, 1, false, false, true>("daxpy", n, x, y, 2);
  CK(hipFree(x));
  CK(hipFree(y));
  // jacobi: pitch = nj + 72 (padded like the engine) and nj + 8 + 1 -> 64-multiple
  for (int pass = 0; pass < 2; ++pass) {
    const int64_t ld = pass == 0 ? ((8 + nj + 1 + 63) / 64) * 64 : nj + 8 + 8 + 256 + 8;
    double *u, *un;
    CK(hipMalloc(&u, (nj + 2) * ld * 8));
    CK(hipMalloc(&un, (nj + 2) * ld * 8));
    CK(hipMemset(u, 0, (nj + 2) * ld * 8));
    CK(hipMemset(un, 0, (nj + 2) * ld * 8));
    run_jacobi<256, 32, false, true>(nj, ld, u, un);
    if (pass == 0) {
      run_jacobi<256, 32, false, false>(nj, ld, u, un);
      run_jacobi<256, 8, false, true>(nj, ld, u, un);
      run_jacobi<256, 16, false, true>(nj, ld, u, un);
      run_jacobi<256, 64, false, true>(nj, ld, u, un);
      run_jacobi<256, 32, true, true>(nj, ld, u, un);
      run_jacobi<128, 32, false, true>(nj, ld, u, un);
      run_jacobi<512, 32, false, true>(nj, ld, u, un);
      run_jacobi<512, 16, false, true>(nj, ld, u, un);
      run_jacobi<1024, 16, false, true>(nj, ld, u, un);
      run_jacobi<64, 64, false, true>(nj, ld, u, un);
    }
    CK(hipFree(u));
    CK(hipFree(un));
  }
  return 0;
}
