// valu_rate — measured issue rates on gfx950 of the instructions a
// register-pipelined Jacobi level is made of, at 1..8 waves per SIMD.
//
// A Jacobi level on 2 columns per lane needs, per 128 cells, 6 v_add_f64
// and the west/east neighbour of each pair from the adjacent lanes.  Those
// lane shifts can come from DPP moves (VALU: 2 v_mov_b32_dpp per double) or
// from ds_bpermute_b32 (the LDS crossbar: no VALU slot).  Each pattern below
// runs `iters` rounds over 8 independent cells per lane (no dependency
// between the cells of a round), so it measures issue throughput, not
// latency.  Output: ns per pattern instance per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

__device__ __forceinline__ double dpp_shr(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_shl(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double bperm(double v, int addr) {
  const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

// patterns (per cell pair = one "level" of 2 columns per lane):
//   0: 1 v_add_f64                       1: 1 v_add_f32
//   2: 2 v_mov_b32_dpp (one double)      3: 2 ds_bpermute_b32 (one double)
//   4: level, DPP both sides: 4 dpp + 6 v_add_f64
//   5: level, DPP west + bpermute east: 2 dpp + 2 bpermute + 6 v_add_f64
//   6: level, bpermute both sides: 4 bpermute + 6 v_add_f64
template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(double* out, int iters, double a) {
  constexpr int N = 8;
  double x[N], y[N];
  float f[N];
  const int lane = threadIdx.x & 63;
  const int up = ((lane + 1) & 63) * 4, dn = ((lane + 63) & 63) * 4;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    x[i] = threadIdx.x * 1e-9 + i;
    y[i] = threadIdx.x * 2e-9 + i;
    f[i] = threadIdx.x * 1e-6f + i;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if constexpr (OP == 0) {
        x[i] = x[i] + a;
      } else if constexpr (OP == 1) {
        f[i] = f[i] + static_cast<float>(a);
      } else if constexpr (OP == 2) {
        x[i] = dpp_shr(x[i]);
      } else if constexpr (OP == 3) {
        x[i] = bperm(x[i], dn);
      } else {
#pragma clang fp contract(off)
        double w, e;
        if constexpr (OP == 4) {
          w = dpp_shr(y[i]);
          e = dpp_shl(x[i]);
        } else if constexpr (OP == 5) {
          w = dpp_shr(y[i]);
          e = bperm(x[i], up);
        } else {
          w = bperm(y[i], dn);
          e = bperm(x[i], up);
        }
        const double nx = (w + y[i]) + (a + x[i]);
        const double ny = (x[i] + e) + (a + y[i]);
        x[i] = nx;
        y[i] = ny;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s += x[i] + y[i] + f[i];
  if (s == 12345.678) out[threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  double* out;
  CHECK(hipMalloc(&out, 4096 * sizeof(double)));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"v_add_f64",
                         "v_add_f32",
                         "2 v_mov_b32_dpp",
                         "2 ds_bpermute_b32",
                         "level: 4 dpp + 6 add_f64",
                         "level: 2 dpp + 2 bperm + 6 add",
                         "level: 4 bperm + 6 add_f64"};
  std::printf("# %d CUs, %d rounds x 8 instances per wave; ns per instance per SIMD\n", cus, iters);
  for (int op = 0; op < 7; ++op)
    for (int wps : {1, 2, 3, 4, 8}) {  // waves per SIMD
      const int blocks = cus * wps;     // 256-thread blocks = one wave per SIMD each
      auto launch = [&] {
        switch (op) {
          case 0: rate_kernel<0><<<blocks, 256>>>(out, iters, 1e-3); break;
          case 1: rate_kernel<1><<<blocks, 256>>>(out, iters, 1e-3); break;
          case 2: rate_kernel<2><<<blocks, 256>>>(out, iters, 1e-3); break;
          case 3: rate_kernel<3><<<blocks, 256>>>(out, iters, 1e-3); break;
          case 4: rate_kernel<4><<<blocks, 256>>>(out, iters, 1e-3); break;
          case 5: rate_kernel<5><<<blocks, 256>>>(out, iters, 1e-3); break;
          default: rate_kernel<6><<<blocks, 256>>>(out, iters, 1e-3); break;
        }
      };
      launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double inst = static_cast<double>(blocks) * 4 * iters * 8;  // pattern instances (per wave)
      const double ns = (ms * 1e6) / (inst / (cus * 4.0));
      std::printf("%-32s waves/SIMD=%d  %8.3f ms  %6.2f ns per instance per SIMD\n", names[op], wps, ms, ns);
    }
  CHECK(hipFree(out));
  return 0;
}
