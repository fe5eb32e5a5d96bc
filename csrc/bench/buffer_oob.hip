// Probe: raw-buffer range checking on gfx950 for 16-B loads/stores that
// straddle num_records (per-dword or whole-access?).  Used to decide whether
// the pipelined Jacobi kernel may clamp a lane's pair load with the buffer
// descriptor alone.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned u4 __attribute__((ext_vector_type(4)));

__global__ void probe(const unsigned* src, unsigned* out, int nrec, int off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nrec, 0x00020000);
  u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)(out + 4), 0, nrec, 0x00020000);
  u4 ones = {0xAAu, 0xBBu, 0xCCu, 0xDDu};
  __builtin_amdgcn_raw_buffer_store_b128(ones, w, off, 0, 0);
}

int main() {
  unsigned h[16];
  for (int i = 0; i < 16; ++i) h[i] = 100 + i;
  unsigned *d, *o;
  hipMalloc(&d, sizeof(h));
  hipMalloc(&o, 64 * sizeof(unsigned));
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  const int cases[][2] = {{16, 0}, {12, 0}, {8, 0}, {4, 0}, {24, 8}, {20, 8}, {16, 8}, {8, 8}, {0, 0}};
  for (auto& c : cases) {
    hipMemset(o, 0, 64 * sizeof(unsigned));
    probe<<<1, 1>>>(d, o, c[0], c[1]);
    unsigned r[16];
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    std::printf("nrec=%2d off=%2d load: %u %u %u %u   store@off: %x %x %x %x %x %x\n", c[0], c[1], r[0], r[1], r[2], r[3],
                r[4], r[5], r[6], r[7], r[8], r[9]);
  }
  return 0;
}
