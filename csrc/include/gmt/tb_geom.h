// Strip geometry of the temporal-blocking Jacobi kernel
// (csrc/kernels/jacobi5tb.hpp), shared by the gfx950 launcher, the CPU
// backend (csrc/host/kernels_host.cpp) and the engine's planners, so the
// column counts every layer reasons with are the kernel's own.
//
//   4 columns per lane = 256 columns; one wave per strip up to K = 10, two
//   waves (levels split) for even K = 12..20.
// The left margin KL is the number of window columns left of the first
// output column: K rounded up so the output starts on a lane boundary; the
// right margin mirrors it.  (The round-4 wide K = 20 strip, six columns per
// lane over four stages, is in git history: profiles/r04_wide.md.)
#pragma once

namespace gmt {
namespace tb {

constexpr int kMaxK1 = 10;  // largest single-wave K

constexpr int tb_nc(int) { return 4; }
constexpr int tb_stages(int K) { return K <= kMaxK1 ? 1 : 2; }
constexpr int tb_cols(int K) { return tb_nc(K) * 64; }
constexpr int tb_left(int K) { return (K + 3) / 4 * 4; }
constexpr int tb_strip_out(int K) { return tb_cols(K) - 2 * tb_left(K); }
// strips per workgroup: at most 512 threads; default one strip per
// workgroup for multi-stage strips, four single-wave strips otherwise
constexpr int tb_max_strips(int K) { return 8 / tb_stages(K); }
constexpr int tb_default_strips(int K) { return tb_stages(K) == 1 ? 4 : 1; }
// Sweep counts with an inline-halo (push) kernel: the face stores' two
// per-lane offsets and three descriptors spill the K = 6-10 one-wave strips
// (253-255 VGPRs without them; K = 10 since the exec-masked Dirichlet keep's
// column masks took 8 SGPRs, K = 6 since the push body is chosen per wave)
// and K = 14; the engine plans around them
constexpr bool tb_push_built(int K) { return (K < 6 || K > 10) && K != 14; }

}  // namespace tb
}  // namespace gmt
