// Where the dispatcher puts the waves of a workgroup (gfx950): every wave of
// a launch records its HW_ID (SIMD, CU, SH, SE) and XCC_ID while all of the
// launch's workgroups are resident (each wave idles ~50 us after its stamp),
// with 256 VGPRs per lane (two waves per SIMD, as the K-sweep kernel) and the
// dynamic LDS that sets the workgroups per CU.  Reports, for the two-stage
// strip shapes, how many SIMDs end up holding two stage-0 waves, two stage-1
// waves or one of each, with strip-major (wave w = strip w / 2, stage w % 2)
// and stage-major (strip w % nw, stage w / nw) numbering
// (profiles/r06_shared/README.md, section 2).
//
//   wave_place [strips_per_wg=1,2,4] [lds_kb_per_strip=28]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(512) void place_kernel(uint32_t* out) {
  extern __shared__ char lds[];
  const int wave = static_cast<int>(threadIdx.x) / 64;
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  if ((threadIdx.x & 63) == 0) {
    uint32_t* o = out + 2 * (blockIdx.x * (blockDim.x / 64) + wave);
    o[0] = hw;
    o[1] = xcc;
  }
  lds[threadIdx.x] = 0;
  // stay resident: ~50 us of the 100 MHz constant clock
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 5000) __builtin_amdgcn_s_sleep(10);
  // the K-sweep kernel's register footprint: every VGPR up to v255
  asm volatile("" ::: "v255");
}

int main(int argc, char** argv) {
  const int nw = argc > 1 ? std::atoi(argv[1]) : 1;
  const int kb = argc > 2 ? std::atoi(argv[2]) : 28;
  const int waves = 2 * nw;
  const size_t smem = static_cast<size_t>(nw) * kb * 1024;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&place_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(smem)) != hipSuccess)
    return 1;
  int occ = 0, cus = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(&place_kernel), waves * 64, smem);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int nb = occ * cus;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, static_cast<size_t>(nb) * waves * 8) != hipSuccess) return 1;
  place_kernel<<<nb, waves * 64, smem>>>(d);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<uint32_t> h(static_cast<size_t>(nb) * waves * 2);
  if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  std::printf("strips/wg %d, waves/wg %d, LDS %zu B/wg, %d wg/CU x %d CUs = %d workgroups\n", nw, waves, smem, occ,
              cus, nb);
  // wave index -> SIMD histogram
  std::vector<std::vector<int>> hist(waves, std::vector<int>(4, 0));
  // (xcc, se, sh, cu, simd) -> stages of the waves it holds, per numbering
  std::map<std::tuple<int, int, int, int, int>, std::vector<int>> sm, mj;
  for (int b = 0; b < nb; ++b)
    for (int w = 0; w < waves; ++w) {
      const uint32_t hw = h[2 * (static_cast<size_t>(b) * waves + w)], xcc = h[2 * (static_cast<size_t>(b) * waves + w) + 1];
      const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      ++hist[w][simd];
      const auto key = std::make_tuple(static_cast<int>(xcc & 15), se, sh, cu, simd);
      sm[key].push_back(w % 2);        // strip-major: stage w % 2
      mj[key].push_back(w / nw);       // stage-major: stage w / nw
    }
  for (int w = 0; w < waves; ++w)
    std::printf("wave %d of its workgroup -> SIMD 0..3: %d %d %d %d\n", w, hist[w][0], hist[w][1], hist[w][2],
                hist[w][3]);
  for (int m = 0; m < 2; ++m) {
    int s00 = 0, s01 = 0, s11 = 0, other = 0;
    for (const auto& kv : (m == 0 ? sm : mj)) {
      const auto& v = kv.second;
      if (v.size() != 2) {
        ++other;
        continue;
      }
      const int n1 = v[0] + v[1];
      (n1 == 0 ? s00 : n1 == 1 ? s01 : s11)++;
    }
    std::printf("%s numbering: SIMDs with two stage-0 waves %d, one of each %d, two stage-1 waves %d, other %d\n",
                m == 0 ? "strip-major" : "stage-major", s00, s01, s11, other);
  }
  (void)hipFree(d);
  return 0;
}
