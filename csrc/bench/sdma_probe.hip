// sdma_probe — can a halo exchange run beside a pass that fills every CU?
//
// The band-first pass (csrc/engine/jacobi.cpp) hands its faces to the
// exchange while the interior still runs; an exchange made of kernels (RCCL
// p2p, the IPC copy kernels) only gets CUs when the pass's workgroups drain,
// so it cannot hide under a single-round pass.  The DMA engines need no CU:
// this harness measures, on one MI355X,
//   copy   : a K-row face (contiguous) and a K-column face (2-D, 160-B rows)
//            of a 16384 x 8192 share, hipMemcpyDeviceToDevice (blit kernels)
//            vs hipMemcpyDeviceToDeviceNoCU (DMA engines), idle GPU;
//   beside : the same copies issued while a kernel holds every CU slot for
//            ~1 ms (the copy's stream waits, with hipStreamWaitValue64, for a
//            flag the busy kernel sets once it runs): the copy's finish time
//            from the busy kernel's start, against the busy kernel's length;
//   signal : hipStreamWriteValue64 -> hipStreamWaitValue64 hand-off between
//            two streams (the stream-ordered "faces arrived" flag).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

// every workgroup spins for `ticks` of the 100 MHz real-time counter; the
// first thread of workgroup 0 raises *flag (a vector store) when it starts
__global__ __launch_bounds__(256) void busy(uint64_t ticks, uint64_t* flag, double* sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  double acc = threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) acc = acc * 0.999 + 1.0;
  if (acc == -1.0) sink[threadIdx.x] = acc;
}

static float ms(hipEvent_t a, hipEvent_t b) {
  float t;
  CK(hipEventElapsedTime(&t, a, b));
  return t;
}

int main(int argc, char** argv) {
  const int ny = argc > 1 ? std::atoi(argv[1]) : 16384, nx = argc > 2 ? std::atoi(argv[2]) : 8192;
  const int K = 20, ld = nx + 2 * K;
  const size_t bytes = static_cast<size_t>(ny + 2 * K) * ld * sizeof(double);
  double *a, *b, *sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(a, 0, bytes));
  // signal memory comes in 8-byte allocations
  uint64_t *flags, *flag2;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags), 8, hipMallocSignalMemory));
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flag2), 8, hipMallocSignalMemory));
  CK(hipMemset(flags, 0, 8));
  CK(hipMemset(flag2, 0, 8));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e[4];
  for (auto& x : e) CK(hipEventCreate(&x));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  int wv = 0;
  CK(hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, 0));
  std::printf("# %d CUs, stream wait value %d; share %d x %d (ld %d), K = %d\n", ncu, wv, ny, nx, ld, K);

  struct Face {
    const char* name;
    size_t width, height;  // bytes per row, rows
  };
  const Face faces[2] = {{"rows (N/S face, contiguous)", static_cast<size_t>(K) * ld * 8, 1},
                         {"cols (W/E face, 160-B rows)", static_cast<size_t>(K) * 8, static_cast<size_t>(ny)}};
  const hipMemcpyKind kinds[2] = {hipMemcpyDeviceToDevice, hipMemcpyDeviceToDeviceNoCU};
  const char* kname[2] = {"D2D (blit kernel)", "D2D NoCU (DMA)"};
  auto copy = [&](const Face& f, hipMemcpyKind k, hipStream_t s) {
    const size_t pitch = static_cast<size_t>(ld) * 8;
    if (f.height == 1)
      CK(hipMemcpyAsync(b + K * ld, a + K * ld, f.width, k, s));
    else
      CK(hipMemcpy2DAsync(b + K * ld + K, pitch, a + K * ld + K, pitch, f.width, f.height, k, s));
  };
  // idle GPU
  for (const Face& f : faces)
    for (int k = 0; k < 2; ++k) {
      std::vector<float> t;
      for (int r = 0; r < 23; ++r) {
        CK(hipEventRecord(e[0], s0));
        copy(f, kinds[k], s0);
        CK(hipEventRecord(e[1], s0));
        CK(hipEventSynchronize(e[1]));
        if (r >= 3) t.push_back(ms(e[0], e[1]));
      }
      std::sort(t.begin(), t.end());
      const double mb = f.width * f.height / 1e6;
      std::printf("copy   %-28s %-18s %7.1f us  %6.1f GB/s\n", f.name, kname[k], t[t.size() / 2] * 1e3,
                  mb / (t[t.size() / 2] * 1e-3) / 1e3);
    }
  // beside a kernel that holds every slot (256 threads x `per` workgroups
  // per CU): the second stream either waits for the busy kernel's flag
  // (hipStreamWaitValue64) or is simply issued 200 us after the launch;
  // "signal" issues only a hipStreamWriteValue64 there
  const uint64_t ticks = 100000;  // 1 ms
  for (int per : {8, 4})
    for (int mode = 0; mode < 2; ++mode)
      for (int fi = 0; fi < 3; ++fi)
        for (int k = 0; k < (fi < 2 ? 2 : 1); ++k) {
          std::vector<float> tc, tb;
          for (int r = 0; r < 8; ++r) {
            CK(hipMemsetAsync(flags, 0, 8, s0));
            CK(hipMemsetAsync(flag2, 0, 8, s0));
            CK(hipStreamSynchronize(s0));
            CK(hipEventRecord(e[0], s0));
            busy<<<ncu * per, 256, 0, s0>>>(ticks, flags, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(e[1], s0));
            if (mode == 0) {
              CK(hipStreamWaitValue64(s1, flags, 1, hipStreamWaitValueGte, ~0ull));
            } else {
              const auto t0 = std::chrono::steady_clock::now();
              while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200)) {
              }
            }
            if (fi < 2)
              copy(faces[fi], kinds[k], s1);
            else
              CK(hipStreamWriteValue64(s1, flag2, 1, 0));
            CK(hipEventRecord(e[2], s1));
            CK(hipEventSynchronize(e[1]));
            CK(hipEventSynchronize(e[2]));
            if (r >= 2) {
              tb.push_back(ms(e[0], e[1]));
              tc.push_back(ms(e[0], e[2]));
            }
          }
          std::sort(tc.begin(), tc.end());
          std::sort(tb.begin(), tb.end());
          std::printf("beside %d WG/CU %-9s %-28s %-18s done at %7.1f us of a %7.1f us kernel\n", per,
                      mode ? "(+200us)" : "(flag)", fi < 2 ? faces[fi].name : "signal only",
                      fi < 2 ? kname[k] : "-", tc[tc.size() / 2] * 1e3, tb[tb.size() / 2] * 1e3);
        }
  // stream-ordered flag hand-off: s0 writes, s1 waits
  {
    std::vector<float> t;
    for (int r = 0; r < 23; ++r) {
      CK(hipMemsetAsync(flag2, 0, 8, s0));
      CK(hipStreamSynchronize(s0));
      CK(hipStreamWaitValue64(s1, flag2, 1, hipStreamWaitValueGte, ~0ull));
      CK(hipEventRecord(e[3], s1));
      CK(hipEventRecord(e[0], s0));
      CK(hipStreamWriteValue64(s0, flag2, 1, 0));
      CK(hipEventSynchronize(e[3]));
      if (r >= 3) t.push_back(ms(e[0], e[3]));
    }
    std::sort(t.begin(), t.end());
    std::printf("signal write -> wait on another stream: %.1f us (median)\n", t[t.size() / 2] * 1e3);
  }
  CK(hipDeviceSynchronize());
  std::printf("ok\n");
  return 0;
}
