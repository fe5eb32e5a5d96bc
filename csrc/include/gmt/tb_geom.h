// Strip geometry of the temporal-blocking Jacobi kernel
// (csrc/kernels/jacobi5tb.hpp), shared by the gfx950 launcher, the CPU
// backend (csrc/host/kernels_host.cpp) and the engine's planners, so the
// column counts every layer reasons with are the kernel's own.
//
//   narrow strips (K <= 18): 4 columns per lane = 256 columns, one wave per
//     strip up to K = 10, two waves (levels split) for even K = 12..18;
//   wide strips (K = 20): 6 columns per lane = 384 columns, four waves of
//     K/4 levels each (profiles/r04_wide.md).
// The left margin KL is the number of window columns left of the first
// output column: K rounded up so the output starts on a lane (narrow) or a
// column pair (wide) boundary; the right margin mirrors it.
#pragma once

namespace gmt {
namespace tb {

constexpr int kMaxK1 = 10;  // largest single-wave K

// The wide K = 20 kernel is bitwise-correct and cuts VALU per update by 14%,
// but on MI355X it runs 10% below the narrow one (profiles/r04_wide.md):
// built only when this is flipped (scripts/build_variant.sh A/B builds).
constexpr bool kWideK20 = false;
constexpr bool tb_wide(int K) { return kWideK20 && K == 20; }
constexpr int tb_nc(int K) { return tb_wide(K) ? 6 : 4; }
constexpr int tb_stages(int K) { return K <= kMaxK1 ? 1 : (tb_wide(K) ? 4 : 2); }
constexpr int tb_cols(int K) { return tb_nc(K) * 64; }
constexpr int tb_left(int K) { return tb_wide(K) ? (K + 1) / 2 * 2 : (K + 3) / 4 * 4; }
constexpr int tb_strip_out(int K) { return tb_cols(K) - 2 * tb_left(K); }
// strips per workgroup: at most 512 threads; default one strip per
// workgroup for multi-stage strips, four single-wave strips otherwise
constexpr int tb_max_strips(int K) { return 8 / tb_stages(K); }
constexpr int tb_default_strips(int K) { return tb_stages(K) == 1 ? 4 : 1; }
// Sweep counts with an inline-halo (push) kernel: the face stores' two
// per-lane offsets and three descriptors spill the K = 7-9 one-wave strips
// (253-255 VGPRs without them) and K = 14; the engine plans around them
constexpr bool tb_push_built(int K) { return K != 7 && K != 8 && K != 9 && K != 14; }

}  // namespace tb
}  // namespace gmt
