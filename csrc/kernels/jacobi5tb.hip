// K fused 5-point Jacobi sweeps per memory pass (temporal blocking), gfx950.
//
// One strip = 256 columns, 4 per lane, walked down a segment of L output
// rows.  Time level p of row r needs level p-1 of rows r-1, r, r+1.  Skewed
// pipeline with skew 1: at step s, level p is computed for row s-p, bottom-up
// (level 1 first), so level p reads level p-1 of the row computed earlier in
// the same step (its south neighbour) and of the two rows computed in the two
// previous steps — two register slots per level.  Level K (stored) at step s
// is row s-K; a segment takes L + 2K steps.
// West/east neighbours come from the adjacent lane through DPP (wave_shr /
// wave_shl); the strip edges lose one column per level, so a strip yields
// 256 - 2 KL output columns (KL = K rounded up to a multiple of 4, so both
// output edges fall on a lane boundary).
//
// Why 4 columns per lane (profiles/r02_tb.md, r02_pmc): the kernel is VALU
// issue bound from K ~ 10 and a DPP move costs as much as a DADD.  Per level
// a lane issues 4 DPP moves (one double from each neighbour) and 3 DADD per
// column: 16 instructions per 4 columns (13 per 3 with the round-2 192-column
// strips), and the recomputed strip overlap drops from 2K/192 to 2K/256 —
// 0.074 instead of 0.087 VALU instructions per useful update at K = 20.  The
// skew-1 pipeline is what makes 4 columns fit: 16 VGPRs per level instead of
// 24 with three slots (skew 2).  Its dependency chain per step (level p needs
// level p-1 of this step) is 2 DADD latencies per level, short against the
// 16 issue slots of a level; the DPP moves read rows of earlier steps.
//
// Level split across waves (K > kMaxK1): one wave holds at most kMaxK1
// levels at 2 waves per SIMD.  Larger K runs as 2 stages per strip: stage 0
// computes levels 1..KA from the DMA ring and writes level KA to an LDS
// hand-off ring, stage 1 (two steps behind) reads it there as its level 0 and
// computes KA+1..K; one s_barrier per step publishes the hand-off row.  A
// single memory pass fuses up to GMT_TB_MAX_SWEEPS sweeps, which is what a
// 20-step run needs to stay under the two-pass memory floor (2 x 3.3 ms at
// 32768^2).
//
// Memory pipeline: level-0 rows are DMA'd into a per-strip LDS ring of P+2
// slots (two full-wave dwordx4 DMAs per 2 KB row) and read back by level 1:
// no loaded VGPR crosses the loop back edge.  The compiler does not track
// LDS-DMA -> ds_read dependencies, so the wait is an explicit s_waitcnt
// vmcnt; every step issues the same memory instructions — no branch around
// any of them — so the count is exact.  One loop-invariant buffer descriptor
// per direction; the row is in the VGPR offset and the buffer range check
// drops (stores) or zero-fills (loads) every row outside the segment.
//
// Arithmetic: scaled levels V_p = 4^p u_p, V_p = (W + E) + (N + S), output
// V_K * 4^-K: bitwise equal to K single sweeps u' = 0.25((W+E)+(N+S))
// unless a level value is subnormal or 4^K |u| overflows; EXACT keeps the
// 0.25 multiply per level (used by the engine when max|u| is too large).
// Dirichlet sides (halo_mask bit clear): ring cells keep their value at every
// level (RULE path, per-lane column masks + a per-row test, chosen per
// wave); on halo sides the K-wide ghost ring is updated as data.
//
// This file holds the C API; the kernel is in jacobi5tb.hpp and is
// instantiated per K in jacobi5tb_k*.hip.
#include "jacobi5tb.hpp"

// every K is instantiated in its jacobi5tb_k*.hip translation unit
namespace gmt {
namespace tb {
extern template int dispatch_k<1>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<2>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<3>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<4>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<5>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<6>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<7>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<8>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<9>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<10>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<12>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<14>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<16>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<18>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
extern template int dispatch_k<20>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int,
                                      const double*, double*, int64_t, int64_t, hipStream_t, int64_t*);
}  // namespace tb
}  // namespace gmt

using namespace gmt::tb;

extern "C" int gmt_jacobi5tb_supported(int sweeps) {
  return (sweeps >= 1 && sweeps <= kMaxK1) || (sweeps > kMaxK1 && sweeps <= GMT_TB_MAX_SWEEPS && sweeps % 2 == 0);
}

// The exact (1/4 per level) K = 20 kernel needs one VGPR more than the 256 of
// 2 waves per SIMD and spills 8 B per lane (tests/test_kernel_resources.py):
// it exists for the kernel-level API, but planners use at most 18 exact sweeps.
extern "C" int gmt_jacobi5tb_push_supported(int K) { return gmt_jacobi5tb_supported(K) && tb_push_built(K); }
extern "C" int gmt_jacobi5tb_max_sweeps(int exact) { return exact ? 18 : GMT_TB_MAX_SWEEPS; }

namespace {
int jacobi5tb_run(const gmt_tb_opts* opts, int n_rect, const int64_t* rects, const int64_t* dom, int halo_mask,
                  const double* u, double* un, int64_t ld, int64_t nrows, void* stream, int64_t* info) {
  gmt_tb_opts o{};
  if (opts) o = *opts;
  const int K = o.sweeps;
  if (!gmt_jacobi5tb_supported(K)) return static_cast<int>(hipErrorInvalidValue);
  if (n_rect < 0 || n_rect > kMaxRect) return static_cast<int>(hipErrorInvalidValue);
  const bool cols = (o.signal_cols & 3) != 0;
  if (o.wg_waves < 0 || o.wg_waves > kMaxThreads / kWave || o.seg_rows < 0 || o.signal_rects < 0 || o.reserved_cus < 0 ||
      o.signal_rects > n_rect ||
      ((o.signal_rects > 0 || o.signal_rows > 0 || cols) && (!o.signal_count || !o.signal)) ||
      o.signal_rows < 0 || ((o.signal_rows > 0 || cols) && o.signal_rects >= n_rect) || (o.signal_cols & ~3))
    return static_cast<int>(hipErrorInvalidValue);
  if ((reinterpret_cast<uintptr_t>(u) & 7u) || (reinterpret_cast<uintptr_t>(un) & 7u) || ld <= 0)
    return static_cast<int>(hipErrorInvalidValue);
  if (static_cast<uint64_t>(ld) * 8u > 0xffffffffull) return static_cast<int>(hipErrorInvalidValue);
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) {
      if (k < o.signal_rects || ((o.signal_rows > 0 || cols) && k == o.signal_rects))  // signalling rects are never empty
        return static_cast<int>(hipErrorInvalidValue);
      continue;
    }
    // the K-wide ring around the rect exists
    if (r[0] < K || r[2] < K || r[0] + r[1] + K > ld || r[2] + r[3] + K > nrows)
      return static_cast<int>(hipErrorInvalidValue);
  }
  const bool exact = o.exact != 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (K) {
#define GMT_TB_CASE(KK) \
  case KK:              \
    return dispatch_k<KK>(o, exact, n_rect, rects, dom, halo_mask, u, un, ld, nrows, s, info);
    GMT_TB_CASE(1)
    GMT_TB_CASE(2)
    GMT_TB_CASE(3)
    GMT_TB_CASE(4)
    GMT_TB_CASE(5)
    GMT_TB_CASE(6)
    GMT_TB_CASE(7)
    GMT_TB_CASE(8)
    GMT_TB_CASE(9)
    GMT_TB_CASE(10)
    GMT_TB_CASE(12)
    GMT_TB_CASE(14)
    GMT_TB_CASE(16)
    GMT_TB_CASE(18)
    GMT_TB_CASE(20)
#undef GMT_TB_CASE
    default:
      return static_cast<int>(hipErrorInvalidValue);
  }
}
}  // namespace

extern "C" int gmt_jacobi5tb(const gmt_tb_opts* opts, int n_rect, const int64_t* rects, const int64_t* dom,
                             int halo_mask, const double* u, double* un, int64_t ld, int64_t nrows, void* stream) {
  return jacobi5tb_run(opts, n_rect, rects, dom, halo_mask, u, un, ld, nrows, stream, nullptr);
}

extern "C" int64_t gmt_jacobi5tb_group_cols(int sweeps, int wg_waves) {
  if (!gmt_jacobi5tb_supported(sweeps)) return 0;
  const int nw = std::min(wg_waves > 0 ? wg_waves : tb_default_strips(sweeps), tb_max_strips(sweeps));
  return static_cast<int64_t>(nw) * tb_strip_out(sweeps);
}

extern "C" int gmt_jacobi5tb_plan(const gmt_tb_opts* opts, int n_rect, const int64_t* rects, const int64_t* dom,
                                  int halo_mask, int64_t ld, int64_t nrows, int64_t info[6]) {
  if (!info) return static_cast<int>(hipErrorInvalidValue);
  // u/un only pass the alignment check: nothing is launched or dereferenced
  const double* p = reinterpret_cast<const double*>(alignof(double));
  return jacobi5tb_run(opts, n_rect, rects, dom, halo_mask, p, const_cast<double*>(p), ld, nrows, nullptr, info);
}
