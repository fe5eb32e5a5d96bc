// Temporal-blocking Jacobi kernel and its launch code (see jacobi5tb.hip for
// the design).  Included by the jacobi5tb_k*.hip translation units, each of
// which instantiates dispatch_k for a few K: the fully unrolled register
// pipelines take minutes per K to compile, so they build in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "common.hpp"
#include "gmt/kernels.h"
#include "gmt/tb_geom.h"

namespace gmt {
namespace tb {

constexpr int kMaxRect = 8;
constexpr int kMaxThreads = 512;              // 8 waves: 2 per SIMD
constexpr uint32_t kDrop = 0x80000000u;       // buffer offset past num_records: no-op access

// Unroll of the step loop: the register cycle of the pipeline.  A level's
// new row is live while its step-(s-2) row is still being read, so a step
// frees one row at the top level and the rows move up one register slot per
// step: a value's register passes through the two slots of each of the
// NL - 1 stored levels plus the spare, 2(NL - 1) + 1 steps.  Unrolling by
// exactly that lets the allocator keep every row in place (no copies at the
// back edge).
constexpr int unroll_for(int NL) { return NL > 1 ? 2 * (NL - 1) + 1 : 2; }

// Per-K shape (gmt/tb_geom.h): every step re-reads the three input rows of
// the stage's first level from LDS.  (The round-4 six-column strip with four
// stages that slid its rows — 14% less VALU, 9-10% slower at two waves per
// SIMD, profiles/r04_wide.md — lives in git history: scripts/build_variant.sh
// wide git:09d882f with GEOM='s/kWideK20 = false/kWideK20 = true/'.)
template <int K>
struct Cfg {
  static constexpr int NC = tb_nc(K);           // columns per lane
  static constexpr int S = tb_stages(K);        // waves (stages) per strip
  static constexpr int COLS = NC * kWave;
  static constexpr uint32_t ROW = COLS * 8;     // bytes of one strip row
  static constexpr int NDMA = NC / 2;           // 1-KB full-wave DMAs per row
  static constexpr int KL = tb_left(K);
  static constexpr int WOUT = tb_strip_out(K);
  static constexpr int NL = K / S;              // levels per stage
  static constexpr int U = unroll_for(NL);
  static constexpr int P = 6;                   // input rows in flight
  static constexpr int RS = P + 2;              // DMA ring slots
  static constexpr int HS = 6;                  // hand-off ring slots
  // step lag of each stage behind the previous one: 2 (the hand-off rows of
  // step s are requested before the barrier that ends step s)
  static constexpr int DLAG = 2;
  static constexpr int LAG = DLAG * (S - 1);    // the output stage's step lag
  static_assert(K % S == 0, "equal stages");
  static_assert(NC % 2 == 0 && KL % 2 == 0, "column pairs");
  static_assert(HS >= 5, "hand ring: rows of steps s-4..s");
};

// LDS per strip: the DMA ring, plus S - 1 hand-off rings
template <int K>
__host__ __device__ constexpr int64_t strip_lds() {
  using C = Cfg<K>;
  return static_cast<int64_t>(C::RS) * C::ROW + static_cast<int64_t>(C::S - 1) * C::HS * C::ROW;
}


// Shared hand-off groups (SH: gmt_tb_opts.shared; one-rect passes without
// signals).  A workgroup of NW adjacent two-stage strips writes its stage-0
// output (level NL = K/2) into ONE hand-off row of the whole group instead
// of one per strip, so a stage-1 wave can read any 256-column window of the
// group's valid level-NL columns: each stage loses NL columns per side to
// its own cone instead of the strip losing K.  Stage-0 windows are S0 =
// 256 - 2 NL apart (their valid columns [NL, 256 - NL) abut, each column
// written by exactly one wave: exec-masked hand-off stores), stage-1
// windows start O (>= NL, a lane boundary) into the group and are S1 apart,
// the last ending inside the group's valid columns.  K = 20: 4 strips,
// 920 output columns per 8 waves against 4 x 216 = 864 for four separate
// strips — 6% fewer level updates per output update.  The row is laid out
// by 4-column groups g (lane l of a window starting at group g0 holds group
// g0 + l): pair q of group g at byte q QS + 16 g, conflict-free for every
// window offset.  NL even: every ownership boundary is a column pair.
template <int K, int NW_ = 4>
struct Sh {
  static constexpr int NW = NW_;                           // strips per workgroup (2 or 4)
  static constexpr int NL = K / 2;                         // levels per stage
  static constexpr bool kOk = tb_stages(K) == 2 && NL % 2 == 0;
  static constexpr int S0 = 256 - 2 * NL;                  // stage-0 window spacing
  static constexpr int O = (NL + 3) / 4 * 4;               // first stage-1 window, from the group's
  static constexpr int S1 = (S0 * (NW - 1) - NL - O) / (NW - 1) / 4 * 4;  // stage-1 spacing
  static constexpr int GOUT = S1 * (NW - 1) + 256 - 2 * NL;  // output columns of a group
  static constexpr int ML = O + NL;                        // group window start -> output start
  // column slot of the W / E ghost column in the first / last strip's
  // windows of a pass whose rect is the interior (both stages alike: O, S0
  // and S1 are multiples of 4)
  static constexpr int kJW = (ML - 1) % 4;
  static constexpr int kJE = (GOUT + ML) % 4;
  static constexpr int kCols = S0 * (NW - 1) + 256;        // input columns of a group
  static constexpr int NG = kCols <= 512 ? 128 : 256;      // 4-column groups of a shared row
  static constexpr uint32_t QS = NG * 16;                  // pair-plane stride (bytes)
  static constexpr uint32_t ROWG = 2 * QS;                 // one shared row (bytes)
  static_assert(!kOk || (S0 % 4 == 0 && S1 > 0 && S1 <= S0 && O + S1 * (NW - 1) + 256 <= S0 * (NW - 1) + 256 - NL),
                "stage-1 windows inside the group's valid level-NL columns");
  static_assert(!kOk || (S0 * (NW - 1) + 256) / 4 <= NG, "shared row holds the group");
};

// LDS of an SH workgroup: the shared hand-off ring, then NW DMA rings
template <int K, int NW = 4>
__host__ __device__ constexpr int64_t sh_lds() {
  using C = Cfg<K>;
  return static_cast<int64_t>(C::HS) * Sh<K, NW>::ROWG + static_cast<int64_t>(NW) * C::RS * C::ROW;
}

struct Args {
  int64_t r[kMaxRect][4];        // output rects: x0, nx, y0, ny (absolute)
  int64_t nstrip[kMaxRect];      // strips per rect
  int64_t tstart[kMaxRect + 1];  // prefix sum of workgroups
  int64_t dom[4];                // interior x0, nx, y0, ny
  int64_t ld;                    // row pitch (elements)
  int64_t last_row;              // last allocated row (load clamp)
  int n;                         // rects
  int mask;                      // halo sides: bit0..3 = W/E/S/N
  // segments of rect k: an optional top edge segment of e0[k] rows and a
  // bottom one of e1[k] rows (short: the only ones whose waves can need the
  // Dirichlet rule in y), then nmid[k] interior segments of lmid[k] rows
  int64_t e0[kMaxRect], e1[kMaxRect], nmid[kMaxRect], lmid[kMaxRect];
  // the first and last strip groups (rule waves where a Dirichlet column is
  // in reach) use their own, shorter interior segments
  int64_t nmid_b[kMaxRect], lmid_b[kMaxRect];
  int nw;                        // strips per workgroup
  double quarter;                // 0.25 (EXACT): an SGPR operand
  // completion signal of the leading workgroups (gmt_tb_opts.signal_rects):
  // workgroups t < sig_wgs are dispatched first, unswizzled; the last of
  // them to finish adds 1 to *signal once its stores are visible device-wide
  int64_t sig_wgs;
  unsigned* sig_count;
  uint64_t* signal;
  int prio;                      // single-round launch: stage-0 waves at raised priority
  // row bands (gmt_tb_opts.signal_rows): rect rb_rect's segments next to a
  // halo row side (S: its first segment of every strip group, N: its last,
  // walked bottom-up) are dispatched right after the signalling rects; each
  // of their output waves adds 1 to *sig_count once its first sig_rows
  // output rows are stored.  sig_total: arrivals that raise *signal (the
  // signalling rects' workgroups + these waves); sig_dispatch: leading
  // workgroups dispatched unswizzled.
  int rb_rect;                   // -1: none
  int rb_s, rb_n;                // the rect's first / last segments are row bands
  int64_t sig_rows, sig_total, sig_dispatch;
  // edges_last > 0 (one-rect pass without signals): the first edges_last
  // tiles (the edge segments) are dispatched last on every XCD, round-robin
  // over the XCDs, after each XCD's contiguous range of the other tiles
  // (tail_swizzle); 0: every tile XCD-contiguous in tile order
  int64_t edges_last;
  int sh;                        // an SH launch (Sh<K, nw> groups of nw = 2 or 4 strips)
  int shmap;                     // waves stage-major (SH: GMT_TB_SH_MAP, default on; several
                                 // two-stage strips per workgroup: GMT_TB_STRIP_MAP, A/B)
  int col_keep;                  // the one-column Dirichlet keep (GMT_TB_COL_KEEP=0: off, A/B)
  // column bands (gmt_tb_opts.signal_cols): rect cb_rect's first (cb_lo)
  // and last (cb_hi) strip groups — every segment at full length — are
  // dispatched before everything else of the rect, and each of their
  // workgroups counts one arrival when done (they are the first of the
  // sig_wgs leading workgroups)
  int cb_rect;                   // -1: none
  int cb_lo, cb_hi;
  // inline halo exchange (gmt_tb_opts.push, the PUSH kernels): output cell
  // (x, y) of a face is stored a second time at push[d] + y * ld + x, in the
  // ghost cells of the neighbour's next input; nullptr: no neighbour that way
  const double* push[8];
  int64_t push_w;                // face width
  // PUSH: non-zero *stop (a timed-out hand-over, gmt_push_sync) makes every
  // workgroup return at entry
  const unsigned* stop;
  // shader-clock record (gmt_tb_opts.clock): sampled waves add their
  // s_memtime / s_memrealtime deltas and a count
  uint64_t* clk;
  // GMT_TB_WG_TRACE builds (scripts/build_variant.sh): per workgroup, its
  // tile, start and end (s_memrealtime, 100 MHz) and hardware ids
  uint64_t* wg_trace;
};

// Per-workgroup timeline (A/B variant builds only; the production code
// object has none of it): scripts/build_variant.sh wgt
//   's/#define GMT_TB_WG_TRACE 0/#define GMT_TB_WG_TRACE 1/', then
// GMT_TB_WG_TRACE_FILE=path [GMT_TB_WG_TRACE_LAUNCH=n] writes launch n's
// workgroups (tile, start, end, HW_ID, XCC_ID) and plan to path.
#ifndef GMT_TB_WG_TRACE
#define GMT_TB_WG_TRACE 0
#endif

// cache policy of the face stores into a neighbour's memory: system scope
// (sc0 | sc1: written through to the memory that owns them, complete when
// the wave's vmcnt drains) and streaming (nt)
constexpr int kPushAux = 1 | 2 | 16;

// NC doubles of one strip row held by a lane (its columns c0 .. c0+NC-1)
template <int NC>
struct dv {
  double c[NC];
};

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const double* p, uint32_t bytes) {
  // 0x00020000: raw-buffer descriptor word 3 for gfx9 (32-bit data format)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), 0, bytes, 0x00020000);
}

// s_waitcnt vmcnt(n) only (expcnt / lgkmcnt left at their maxima), as a
// compiler barrier for memory: the LDS-DMA'd rows are read by ds_read after
// it, and the compiler does not track LDS-DMA -> ds_read dependencies
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// hand-off rows written by this wave are visible to the workgroup after it.
// Outstanding DMAs and stores are not waited for (gfx950 has the back-off
// barrier, so s_barrier needs no vmcnt(0)).
__device__ __forceinline__ void step_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS row layout: piece q (q < NC/2) of every lane in its own 1-KB block,
// lane l's columns 2q, 2q+1 at byte 1024 q + 16 l (kPieces), so every
// ds_read_b128 / ds_write_b128 of a row is one contiguous KB: no bank
// conflicts (the row-ordered layout, lane l at 8 NC l, cost the 4-column
// kernel 2e9 conflict cycles per three 32768^2 passes, profiles/r04_wide/
// r04_c_pmc.md); the LDS-DMA fetches each piece with 16 B per lane at an
// NC*8-byte stride instead of contiguous 16 B.
constexpr bool kPieces = true;

// a lane's NC columns of an LDS row (NC / 2 ds_read_b128)
template <int NC>
__device__ __forceinline__ dv<NC> lds_row(const char* slot, int lane) {
  const d2* p = kPieces ? reinterpret_cast<const d2*>(slot) + lane : reinterpret_cast<const d2*>(slot) + (NC / 2) * lane;
  dv<NC> r;
  static_for<0, NC / 2>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    const d2 a = kPieces ? p[q * 64] : p[q];
    r.c[2 * q] = a.x;
    r.c[2 * q + 1] = a.y;
  });
  return r;
}

template <int NC>
__device__ __forceinline__ void lds_put(char* slot, int lane, const dv<NC>& v) {
  d2* p = kPieces ? reinterpret_cast<d2*>(slot) + lane : reinterpret_cast<d2*>(slot) + (NC / 2) * lane;
  static_for<0, NC / 2>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    p[kPieces ? q * 64 : q] = d2{v.c[2 * q], v.c[2 * q + 1]};
  });
}

// SH rows: a lane's NC columns at p (its group's byte in the row), pair
// plane q at p + q QS
template <int NC, uint32_t QS>
__device__ __forceinline__ dv<NC> lds_row_sh(const char* p) {
  dv<NC> r;
  static_for<0, NC / 2>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    const d2 a = *reinterpret_cast<const d2*>(p + q * QS);
    r.c[2 * q] = a.x;
    r.c[2 * q + 1] = a.y;
  });
  return r;
}

// SH stage-0 hand-off store: pair plane 0 under EXEC = m0, plane 1 under m1
// (the lanes whose column pair this strip owns in the shared row; EXEC back
// to all lanes after, and the s_nop for the SALU-writes-EXEC -> DPP hazard
// of the next step's lane shifts, as keep_cells)
template <int NC, uint32_t QS>
__device__ __forceinline__ void lds_put_sh(char* p, const dv<NC>& v, uint64_t m0, uint64_t m1) {
  static_assert(NC == 4, "four columns per lane");
  const d2 lo = d2{v.c[0], v.c[1]}, hi = d2{v.c[2], v.c[3]};
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t ad = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_char*)p));  // the LDS offset
  asm volatile(
      "s_mov_b64 exec, %[m0]\n\t"
      "ds_write_b128 %[ad], %[lo]\n\t"
      "s_mov_b64 exec, %[m1]\n\t"
      "ds_write_b128 %[ad], %[hi] offset:%[qs]\n\t"
      "s_mov_b64 exec, -1\n\t"
      "s_nop 4" ::[ad] "v"(ad),
      [lo] "v"(lo), [hi] "v"(hi), [m0] "s"(m0), [m1] "s"(m1), [qs] "i"(QS)
      : "memory");
}

template <int NC>
__device__ __forceinline__ dv<NC> dv_zero() {
  dv<NC> r;
#pragma unroll
  for (int j = 0; j < NC; ++j) r.c[j] = 0.0;
  return r;
}

__device__ __forceinline__ u4 pack2(double a, double b) {
  return u4{static_cast<unsigned>(__double2loint(a)), static_cast<unsigned>(__double2hiint(a)),
            static_cast<unsigned>(__double2loint(b)), static_cast<unsigned>(__double2hiint(b))};
}
__device__ __forceinline__ u2 pack1(double a) {
  return u2{static_cast<unsigned>(__double2loint(a)), static_cast<unsigned>(__double2hiint(a))};
}

// The Dirichlet keep of one level (RULE waves): v.c[j] = c.c[j] (exact) or
// 4 c.c[j] (scaled levels, exact in binary) on the lanes of mask
// (row kept ? all : kxm[j]); the row is kept iff x = t - tlo, as unsigned,
// is >= span = thi - tlo (t: walk coordinate, run_stage).  One asm block,
// all scalar but the four writes: the row test (s_cmp / s_cselect: a C++
// bool would come back as a VALU select), EXEC set per column and restored
// to all lanes — run_stage runs with all 64 lanes active (whole-wave
// workgroups, no divergent branch around its loop) — and an s_nop for the
// SALU-writes-EXEC -> DPP hazard of the next level's lane shifts (the
// compiler cannot see EXEC change here).  The round-4 per-cell select (a
// multiply, two v_cndmask per column and a 64-bit row compare per level)
// made rule waves ~1.8x the VALU of plain ones; this is 1.23x the VALU and
// 7 SALU per level.  (A branch past the four writes when no lane keeps —
// most levels of the edge segments of inner strips — measured 2-3% slower
// on the rectangular shares than writing under EXEC = 0:
// profiles/r05_rule_keep/.)
template <bool EXACT, int NC>
__device__ __forceinline__ void keep_cells(dv<NC>& v, const dv<NC>& c, const uint64_t (&kxm)[NC], uint32_t x,
                                           uint32_t span) {
  static_assert(NC == 4, "four columns per lane");
  uint64_t rm;
#define GMT_KEEP_ASM(OP0, OP1, OP2, OP3)                                                                          \
  asm("s_cmp_ge_u32 %[x], %[span]\n\t"                                                                          \
      "s_cselect_b64 %[rm], -1, 0\n\t"                                                                           \
      "s_or_b64 exec, %[m0], %[rm]\n\t" OP0 "\n\t"                                                              \
      "s_or_b64 exec, %[m1], %[rm]\n\t" OP1 "\n\t"                                                              \
      "s_or_b64 exec, %[m2], %[rm]\n\t" OP2 "\n\t"                                                              \
      "s_or_b64 exec, %[m3], %[rm]\n\t" OP3 "\n\t"                                                              \
      "s_mov_b64 exec, -1\n\t"                                                                                 \
      "s_nop 4"                                                                                                \
      : [v0] "+v"(v.c[0]), [v1] "+v"(v.c[1]), [v2] "+v"(v.c[2]), [v3] "+v"(v.c[3]), [rm] "=&s"(rm)            \
      : [c0] "v"(c.c[0]), [c1] "v"(c.c[1]), [c2] "v"(c.c[2]), [c3] "v"(c.c[3]), [m0] "s"(kxm[0]),             \
        [m1] "s"(kxm[1]), [m2] "s"(kxm[2]), [m3] "s"(kxm[3]), [x] "s"(x), [span] "s"(span)                    \
      : "scc")
  if constexpr (EXACT)
    GMT_KEEP_ASM("v_mov_b64 %[v0], %[c0]", "v_mov_b64 %[v1], %[c1]", "v_mov_b64 %[v2], %[c2]", "v_mov_b64 %[v3], %[c3]");
  else
    GMT_KEEP_ASM("v_mul_f64 %[v0], %[c0], 4.0", "v_mul_f64 %[v1], %[c1], 4.0", "v_mul_f64 %[v2], %[c2], 4.0",
                 "v_mul_f64 %[v3], %[c3], 4.0");
#undef GMT_KEEP_ASM
}

// The Dirichlet keep of one ghost COLUMN (RULE >= 2 waves: a window that
// holds exactly one fixed ghost column, in column slot RULE - 2 of the lane
// in m, and no fixed row): one write under EXEC = that lane.  The columns
// beyond the ghost one are garbage that nothing reads (the ghost column's
// value depends on its own cell alone), so they need no keep.  Against
// keep_cells' four writes and 7 SALU per level: 1 write and 2 SALU.  (All
// four columns are operands, as in keep_cells: with the one column alone
// the K = 20 stage-1 body spilled 17 VGPRs.)
template <bool EXACT, int J, int NC>
__device__ __forceinline__ void keep_col(dv<NC>& v, double c, uint64_t m) {
  static_assert(NC == 4, "four columns per lane");
#define GMT_KC(OP) asm("s_mov_b64 exec, %[m]\n\t" OP "\n\ts_mov_b64 exec, -1\n\ts_nop 4" \
      : [v0] "+v"(v.c[0]), [v1] "+v"(v.c[1]), [v2] "+v"(v.c[2]), [v3] "+v"(v.c[3]) : [c] "v"(c), [m] "s"(m))
  if constexpr (EXACT) {
    if constexpr (J == 0) GMT_KC("v_mov_b64 %[v0], %[c]");
    else if constexpr (J == 1) GMT_KC("v_mov_b64 %[v1], %[c]");
    else if constexpr (J == 2) GMT_KC("v_mov_b64 %[v2], %[c]");
    else GMT_KC("v_mov_b64 %[v3], %[c]");
  } else {
    if constexpr (J == 0) GMT_KC("v_mul_f64 %[v0], %[c], 4.0");
    else if constexpr (J == 1) GMT_KC("v_mul_f64 %[v1], %[c], 4.0");
    else if constexpr (J == 2) GMT_KC("v_mul_f64 %[v2], %[c], 4.0");
    else GMT_KC("v_mul_f64 %[v3], %[c], 4.0");
  }
#undef GMT_KC
}

#ifndef GMT_TB_SKIP_DEAD
#define GMT_TB_SKIP_DEAD 1
#endif

// One wave = stage J of one strip: levels PB..PE of the K-level pipeline
// (PB = J NL + 1, PE = (J + 1) NL).  Stage 0 takes level 0 from the DMA
// ring; stage J > 0 from hand-off ring J - 1 (rows written by stage J - 1;
// every stage runs two steps behind the previous one, D = 2J, so it can
// request them before the step barrier).  The last stage stores level K to
// `un`; the others write level PE to hand-off ring J.  Strip output columns
// [xs, xe), rows [ys, ye).  UP walks the segment bottom-up (a row band at the
// segment's top edge is then output first; a compile-time direction: a
// runtime one costs the unrolled body its register allocation,
// tests/test_kernel_resources.py); sig_step >= 0: once that step's row is
// stored, this (output) wave publishes a row-band arrival (Args::rb_rect).
// PUSH (inline halo exchange, output stage): bit 0 = this strip holds an x
// face (W / E columns), bit 1 = this segment holds y-face rows (S / N); both:
// the corner too.
// SH (shared hand-off group): cf is the wave's own window (stage-dependent),
// ring + hdelta + 16 lane this lane's group in the shared hand-off ring
// (stage 0 writes it under the ownership masks hm0 / hm1, stage 1 reads it;
// a wave-uniform delta from the DMA ring's lane address, so both share one
// address VGPR); otherwise cf = xs - KL and the hand-off rings are the
// strip's own.
template <int K, int J, bool EXACT, bool EDGE, int RULE, bool UP, int PUSH, int SH>
__device__ __forceinline__ void run_stage(const Args& a, const double* __restrict__ u, double* __restrict__ un,
                                          char* ring, int lane, int64_t xs, int64_t xe, int64_t ys, int64_t ye,
                                          int nsteps, int sig_step, int xd, int64_t cf, int hdelta, uint64_t hm0,
                                          uint64_t hm1) {
  using C = Cfg<K>;
  constexpr int NC = C::NC;
  constexpr int PB = J * C::NL + 1, PE = (J + 1) * C::NL;
  constexpr bool kIn = J == 0;
  constexpr bool kOut = J == C::S - 1;
  constexpr bool SYNC = C::S > 1;
  constexpr int kP = C::P, kRS = C::RS, kHS = C::HS;
  constexpr uint32_t kRow = C::ROW;
  constexpr int D = C::DLAG * J;                     // step lag behind stage 0
  // global stores per step (PUSH: one face group more per face held, and the corner)
  constexpr int kGroups = 1 + (PUSH & 1) + ((PUSH >> 1) & 1) + (PUSH == 3 ? 1 : 0);
  constexpr int SPS = kOut ? (EDGE ? NC : kGroups * (NC / 2)) : 0;
  static_assert(!(PUSH && EDGE), "inline halo exchange: no odd-edge stores");
  // DMAs per step: stage 0 loads the whole row
  constexpr bool kDma = kIn;
  constexpr int DPS = kDma ? C::NDMA : 0;
  // hand-off rings: read ring J - 1, write ring J
  char* const hand_rd = ring + kRS * kRow + (J > 0 ? J - 1 : 0) * kHS * kRow;
  char* const hand_wr = ring + kRS * kRow + J * kHS * kRow;
  // every kernel argument the loop needs, as values: the asm memory clobbers
  // below would otherwise force a reload of the kernarg segment per use
  const int64_t ld = a.ld;
  const int mask = a.mask;
  const double quarter = a.quarter;
  const int64_t dx0 = a.dom[0], dx1 = a.dom[0] + a.dom[1];
  const int64_t dy0 = a.dom[2], dy1 = a.dom[2] + a.dom[3];
  using SHG = Sh<K, SH ? SH : 4>;  // (SH: the group's strips, 2 or 4)
  static_assert(!SH || (SHG::kOk && !EDGE && PUSH == 0 && !UP), "SH: one-rect passes, plain bodies");
  constexpr uint32_t kQS = SHG::QS, kRowG = SHG::ROWG;
  char* const hsh = ring + 16 * lane + hdelta;
  const int64_t c0 = cf + NC * lane;    // this lane: columns c0 .. c0+NC-1
  const int64_t yl = ys - K;            // the window's first row
  const int L = static_cast<int>(ye - ys);
  const uint32_t ld8 = static_cast<uint32_t>(ld) * 8u;
  // row offsets of step s in the window / in the output: base + s * step
  // (bottom-up: from the last row, a negative step; rows past either end
  // wrap to offsets beyond the buffer range: zero-filled / dropped)
  constexpr bool up = UP;
  const uint32_t rstep = up ? 0u - ld8 : ld8;
  const uint32_t dbase = up ? static_cast<uint32_t>(L + 2 * K - 1) * ld8 : 0u;
  const uint32_t sbase = up ? static_cast<uint32_t>(L - 1) * ld8 : 0u;

  //  loads: rows [yl, min(yl + L + 2K, last_row + 1)), COLS * 8 contiguous
  //  bytes from column cf (a column outside the row wraps into the
  //  neighbouring row or is zero-filled: garbage outside every output cone)
  const int64_t nrow_in = std::min<int64_t>(L + 2 * K, a.last_row + 1 - yl);
  const __amdgpu_buffer_rsrc_t lrs = row_rsrc(u + yl * ld, static_cast<uint32_t>(nrow_in) * ld8);
  // piece q of lane `lane`: global columns NC*lane + 2q, +1 (kPieces) or
  // the row's bytes [1024 q + 16 lane, +16)
  const uint32_t loff = static_cast<uint32_t>(cf) * 8u + static_cast<uint32_t>(lane) * (kPieces ? NC * 8u : 16u);
  constexpr uint32_t kPieceStride = kPieces ? 16u : 1024u;
  // SH: one running row offset (the rows are requested in order, one per
  // call) advanced by an opaque v_add, with the pieces in the immediate
  // offset — the compiler otherwise keeps one offset VGPR per unrolled step
  // (~19), which the SH stage-0 body cannot spare (K = 20: 6 VGPRs spilled)
  uint32_t dmo = loff + dbase;
  auto dma = [&](int s, int slot) {
    if constexpr (kDma) {
      char* dst = ring + slot * kRow;
      if constexpr (SH) {
        (void)s;
        static_for<0, C::NDMA>([&](auto Q) {
          constexpr uint32_t q = decltype(Q)::value;
          // (the immediate offset moves the LDS destination too: M0 is
          // lowered by it)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, dst + q * (1024u - kPieceStride), 16, dmo, 0,
                                                   q * kPieceStride, 0);
        });
        asm volatile("v_add_u32 %0, %1, %0" : "+v"(dmo) : "s"(rstep));
      } else {
        const uint32_t o = dbase + static_cast<uint32_t>(s) * rstep;
        static_for<0, C::NDMA>([&](auto Q) {
          constexpr uint32_t q = decltype(Q)::value;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, dst + q * 1024u, 16, loff + q * kPieceStride + o, 0, 0, 0);
        });
      }
    }
  };
  //  stores: rows [ys, ye) from column xs.  The left output edge is a column
  //  pair boundary (KL even): 16-B stores of the lane's column pairs where
  //  both are inside, and (EDGE: a rect of the launch ends at an odd column)
  //  8-B stores of a pair's first column alone.  Lanes with nothing to store
  //  get an offset past any row (dropped).
  const __amdgpu_buffer_rsrc_t srs = row_rsrc(un + ys * ld + xs, static_cast<uint32_t>(L) * ld8);
  uint32_t stp[NC / 2], sts[NC / 2];
#pragma unroll
  for (int q = 0; q < NC / 2; ++q) {
    const int64_t ca = c0 + 2 * q;
    const bool ina = ca >= xs && ca < xe, inb = ca + 1 >= xs && ca + 1 < xe;
    stp[q] = (ina && inb) ? static_cast<uint32_t>(ca - xs) * 8u : kDrop;
    sts[q] = (ina && !inb) ? static_cast<uint32_t>(ca - xs) * 8u : kDrop;
  }
  // Inline halo exchange (PUSH, output stage; gmt_tb_opts.push): the face
  // cells of this strip's output are stored a second time, into the
  // neighbours' ghost cells — the y face this segment holds (S or N rows),
  // the x face this strip holds (xd: W or E columns; per-lane offsets xp),
  // and their corner (diagonal neighbour).  The groups of the faces this
  // wave holds (PUSH bits) are issued every step: a descriptor with nothing
  // of this wave's output in range (a row outside the face, a corner not
  // pushed) drops them in the buffer unit, with no branch in the unrolled
  // step.  Waves holding no face run PUSH = 0, the plain body.
  __amdgpu_buffer_rsrc_t prs_y = row_rsrc(un, 0), prs_x = row_rsrc(un, 0), prs_c = row_rsrc(un, 0);
  uint32_t psh = 0;  // the y face's first row relative to ys, in bytes
  uint32_t xp[NC / 2];
  if constexpr (PUSH != 0 && kOut) {
    const int64_t w = a.push_w;
    int yd = -1;
    int64_t fy0 = 0, fy1 = 0;
    // (a face is located even when only its corners are pushed)
    const bool ps = a.push[GMT_PUSH_S] || a.push[GMT_PUSH_SW] || a.push[GMT_PUSH_SE];
    const bool pn = a.push[GMT_PUSH_N] || a.push[GMT_PUSH_NW] || a.push[GMT_PUSH_NE];
    if (ps && ys < dy0 + w) {
      yd = GMT_PUSH_S;
      fy0 = ys > dy0 ? ys : dy0;
      fy1 = ye < dy0 + w ? ye : dy0 + w;
    } else if (pn && ye > dy1 - w) {
      yd = GMT_PUSH_N;
      fy0 = ys > dy1 - w ? ys : dy1 - w;
      fy1 = ye < dy1 ? ye : dy1;
    }
    auto face = [&](int d, int64_t row0, int64_t rows) {
      return row_rsrc(a.push[d] + row0 * ld + xs, static_cast<uint32_t>(rows) * ld8);
    };
    if (yd >= 0 && a.push[yd]) {
      prs_y = face(yd, fy0, fy1 - fy0);
      psh = static_cast<uint32_t>(fy0 - ys) * ld8;
    }
    if (xd >= 0) {
      if (a.push[xd]) prs_x = face(xd, ys, L);
      const int cd = yd < 0 ? -1 : (yd == GMT_PUSH_S ? (xd == GMT_PUSH_W ? GMT_PUSH_SW : GMT_PUSH_SE)
                                                      : (xd == GMT_PUSH_W ? GMT_PUSH_NW : GMT_PUSH_NE));
      if (cd >= 0 && a.push[cd]) prs_c = face(cd, fy0, fy1 - fy0);
    }
    const int64_t fx0 = xd == GMT_PUSH_W ? dx0 : dx1 - w;
#pragma unroll
    for (int q = 0; q < NC / 2; ++q) {
      const int64_t ca = c0 + 2 * q;
      xp[q] = (xd >= 0 && ca >= fx0 && ca + 1 < fx0 + w) ? stp[q] : kDrop;
    }
  }
  auto store_step = [&](int s, const dv<NC>& v) {  // level K of step s = output row s - D - 2K of the walk
    if constexpr (kOut) {
      const uint32_t ro = sbase + static_cast<uint32_t>(s - D - 2 * K) * rstep;  // warm-up rows: out of range
      static_for<0, NC / 2>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        __builtin_amdgcn_raw_buffer_store_b128(pack2(v.c[2 * q], v.c[2 * q + 1]), srs, stp[q] + ro, 0, 2 /* nt */);
      });
      if constexpr (PUSH != 0) {
        // (rows before the face wrap to offsets far past the range: the
        // segment's rows times ld8 stay below 2^31, launch_tb's lmax)
        const uint32_t ry = ro - psh;
        static_for<0, NC / 2>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          const u4 d = pack2(v.c[2 * q], v.c[2 * q + 1]);
          if constexpr (PUSH & 2) __builtin_amdgcn_raw_buffer_store_b128(d, prs_y, stp[q] + ry, 0, kPushAux);
          if constexpr (PUSH & 1) __builtin_amdgcn_raw_buffer_store_b128(d, prs_x, xp[q] + ro, 0, kPushAux);
          if constexpr (PUSH == 3) __builtin_amdgcn_raw_buffer_store_b128(d, prs_c, xp[q] + ry, 0, kPushAux);
        });
      }
      if constexpr (EDGE) {
        static_for<0, NC / 2>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          __builtin_amdgcn_raw_buffer_store_b64(pack1(v.c[2 * q]), srs, sts[q] + ro, 0, 2);
        });
      }
    }
  };

  // Dirichlet rule (RULE only): a cell outside the interior on a side whose
  // ghost ring is fixed keeps its value at every level
  const bool gw = mask & 1, ge = mask & 2, gs = mask & 4, gn = mask & 8;
  auto kept_col = [&](int64_t c) { return (c < dx0 && !gw) || (c >= dx1 && !ge); };
  // per column of the lane: the lanes whose cell is a fixed ring cell (a
  // wave-uniform 64-bit mask per column, for the exec-masked keep below)
  uint64_t kxm[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) kxm[j] = __builtin_amdgcn_ballot_w64(kept_col(c0 + j));
  // RULE >= 2: the one ghost column's lane (tb_block: slot RULE - 2)
  constexpr int kColSlot = RULE >= 2 ? RULE - 2 : 0;
  static_assert(RULE < 2 || kColSlot < NC, "column slot");
  const int64_t gcol = !gw && cf <= dx0 - 1 && dx0 - 1 < cf + C::COLS ? dx0 - 1 : dx1;
  const uint64_t kcm = RULE >= 2 ? __builtin_amdgcn_ballot_w64(c0 + kColSlot == gcol) : 0;

  // fixed ring rows, in walk coordinates t = +-(row - yanchor) (- bottom-up;
  // the walk's rows: t = s - D - p for level p of step s): kept iff t < tlo
  // or t >= thi
  // (32-bit scalar compares; 64-bit row compares would take the VALU)
  const int64_t yanchor = up ? ye - 1 + K : yl;
  const auto clamp32 = [](int64_t x) {
    return static_cast<int>(x < INT32_MIN ? int64_t{INT32_MIN} : x > INT32_MAX ? int64_t{INT32_MAX} : x);
  };
  const int tlo = up ? (gn ? INT32_MIN : clamp32(yanchor - dy1 + 1)) : (gs ? INT32_MIN : clamp32(dy0 - yanchor));
  const int thi = up ? (gs ? INT32_MAX : clamp32(yanchor - dy0 + 1)) : (gn ? INT32_MAX : clamp32(dy1 - yanchor));
  // (mod 2^32: t - tlo in [0, span) <=> tlo <= t < thi, for |t| < 2^30)
  const uint32_t span = static_cast<uint32_t>(thi) - static_cast<uint32_t>(tlo);
  auto level = [&](const dv<NC>& up_, const dv<NC>& c, const dv<NC>& dn, int t) -> dv<NC> {
#pragma clang fp contract(off)
    const double w = dpp_from_lower(c.c[NC - 1]), e = dpp_from_upper(c.c[0]);
    dv<NC> v;
    static_for<0, NC>([&](auto Q) {
#pragma clang fp contract(off)
      constexpr int j = decltype(Q)::value;
      double l, r;
      if constexpr (j == 0) l = w;
      else l = c.c[j - 1];
      if constexpr (j == NC - 1) r = e;
      else r = c.c[j + 1];
      if constexpr (EXACT) v.c[j] = quarter * ((l + r) + (up_.c[j] + dn.c[j]));
      else v.c[j] = (l + r) + (up_.c[j] + dn.c[j]);
    });
    if constexpr (RULE >= 2) {
      keep_col<EXACT, kColSlot, NC>(v, c.c[kColSlot], kcm);
    } else if constexpr (RULE == 1) {
      // a kept cell: V_p = V_{p-1} (exact) / 4 V_{p-1} (scaled levels),
      // written under EXEC = the lanes to keep: all lanes on a fixed ring
      // row, the ring-column lanes otherwise (none in most levels of most
      // rule waves)
      keep_cells<EXACT, NC>(v, c, kxm, static_cast<uint32_t>(t) - static_cast<uint32_t>(tlo), span);
    }
    return v;
  };

  constexpr int NL = PE - PB + 1;
  // W[p - PB][0 / 1]: level p (PB..PE-1) of the rows of steps s-2 / s-1
  dv<NC> W[NL > 1 ? NL - 1 : 1][2];
#pragma unroll
  for (int p = 0; p < (NL > 1 ? NL - 1 : 1); ++p)
#pragma unroll
    for (int j = 0; j < 2; ++j) W[p][j] = dv_zero<NC>();

  // prologue: rows 0..P-1 in flight, each preceded by the (dropped) stores a
  // steady-state step issues, so every wait below counts the same younger
  // memory operations
  if constexpr (kIn) {
    // (each dummy store gets its own out-of-range row so the compiler cannot
    // merge identical stores)
    static_for<0, kP>([&](auto I) {
      store_step(decltype(I)::value - kP, dv_zero<NC>());
      dma(decltype(I)::value, decltype(I)::value);
    });
  }

  // level PB-1 input rows: r0, r1, r2 = the rows of step s, read one step
  // ahead so the ds_reads are in flight across the step barrier.
  //   stage 0: input row i = DMA'd window row i, step s uses rows s-2, s-1, s;
  //   stage J > 0: input row i = the row stage J-1 wrote at its step i, step
  //   s uses rows s-2-DLAG .. s-DLAG (published by the barrier of the
  //   writer's step that wrote it).
  dv<NC> r0, r1, r2;
  auto load_rows = [&](int s) {  // the three rows of step s
    if constexpr (kIn) {
      // the DMA of row s (issued at the end of step s-P) has landed once at
      // most (SPS + DPS)(P - 1) younger memory operations are outstanding
      wait_vmcnt<(SPS + DPS) * (kP - 1)>();
      r0 = lds_row<NC>(ring + ((s + kRS - 2) % kRS) * kRow, lane);
      r1 = lds_row<NC>(ring + ((s + kRS - 1) % kRS) * kRow, lane);
      r2 = lds_row<NC>(ring + (s % kRS) * kRow, lane);
    } else {
      if constexpr (SH) {
        r0 = lds_row_sh<NC, kQS>(hsh + ((s + kHS - 4) % kHS) * kRowG);
        r1 = lds_row_sh<NC, kQS>(hsh + ((s + kHS - 3) % kHS) * kRowG);
        r2 = lds_row_sh<NC, kQS>(hsh + ((s + kHS - 2) % kHS) * kRowG);
      } else {
        r0 = lds_row<NC>(hand_rd + ((s + kHS - 4) % kHS) * kRow, lane);
        r1 = lds_row<NC>(hand_rd + ((s + kHS - 3) % kHS) * kRow, lane);
        r2 = lds_row<NC>(hand_rd + ((s + kHS - 2) % kHS) * kRow, lane);
      }
    }
  };
  load_rows(0);

  // rows of the walk: level p of step s is row yanchor +- (s - D - p)
  auto step = [&](auto Jc, int s) {
    constexpr int j = decltype(Jc)::value;
    (void)j;
    dv<NC> v = level(r0, r1, r2, s - D - PB);
    __builtin_amdgcn_sched_barrier(0);
    static_for<PB + 1, PE + 1>([&](auto Q) {
      constexpr int p = decltype(Q)::value;  // PB+1 .. PE, bottom-up
      const dv<NC> nv = level(W[p - 1 - PB][0], W[p - 1 - PB][1], v, s - D - p);
      W[p - 1 - PB][0] = W[p - 1 - PB][1];  // rows of steps s-1 and s become s-2 and s-1
      W[p - 1 - PB][1] = v;
      v = nv;
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (kOut) {
      if constexpr (!EXACT) {
#pragma unroll
        for (int q = 0; q < NC; ++q) v.c[q] = __builtin_amdgcn_ldexp(v.c[q], -2 * K);  // exact power-of-two unscale
      }
      store_step(s, v);  // issued every step (warm-up rows are out of range)
    } else if constexpr (SH) {
      lds_put_sh<NC, kQS>(hsh + (s % kHS) * kRowG, v, hm0, hm1);
    } else {
      lds_put<NC>(hand_wr + (s % kHS) * kRow, lane, v);
    }
    // the ring slot of row s-2 is free: prefetch row s+P into it
    dma(s + kP, (s + kP) % kRS);
    // hand-off row written (visible to the workgroup after the barrier),
    // then the next step's rows requested, then the barrier
    if constexpr (SYNC) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    load_rows(s + 1);
    if constexpr (SYNC) asm volatile("s_barrier" ::: "memory");
  };

  constexpr int kU = C::U;
  // The first unrolled block of a later stage (J > 0) computes nothing of
  // use: level p of step s holds walk row s - D - p, which the output cone
  // needs only from row p on (rows [p, L + 2K - p) of level p), so every
  // level PB..PE of this stage is dead for s < D + 2 PB — past the whole
  // block at K >= 12 (19 <= 2 + 2 * 11 at K = 20).  That block only keeps
  // the step barriers and, at its last step, reads the rows of step kU;
  // the loop then starts at kU with the registers as at its usual start.
  // (Its stores fall before the segment's output rows: dropped anyway; this
  // stage issues no DMA, so no vmcnt accounting changes.  Round 6: the
  // partly dead blocks compiled with their dead levels left out spilled the
  // K = 20 kernels, 20-590 VGPRs.)  GMT_TB_SKIP_DEAD 0 (A/B builds): off.
  constexpr bool kSkip0 = GMT_TB_SKIP_DEAD && !kIn && SYNC && kU <= D + 2 * PB;
  int s_first = 0;
  if constexpr (kSkip0) {
    for (int s = 0; s < kU - 1; ++s) step_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    load_rows(kU);
    asm volatile("s_barrier" ::: "memory");
    s_first = kU;
  }
  for (int s0 = s_first; s0 < nsteps; s0 += kU) {
    static_for<0, kU>([&](auto Jc) { step(Jc, s0 + decltype(Jc)::value); });
    // A row band's output wave: once the unrolled block holding step
    // sig_step is done, the band's rows are written — visible device-wide,
    // then one arrival (the last raises *signal).  Checked at the block
    // boundary, not per step: the register allocation of the unrolled body
    // has no room for a branch per step (tests/test_kernel_resources.py).
    if constexpr (kOut) {
      if (static_cast<unsigned>(sig_step - s0) < static_cast<unsigned>(kU)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (lane == 0 && __hip_atomic_fetch_add(a.sig_count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                             static_cast<unsigned>(a.sig_total - 1)) {
          __hip_atomic_store(a.sig_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(a.signal, uint64_t{1}, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
  // no LDS-DMA may land after the workgroup's LDS is released
  wait_vmcnt<0>();
}

// A workgroup = nw adjacent strips of one segment row, S waves per strip
// (adjacent strips share their overlap columns in the CU's L1 / the XCD's
// L2).  S == 1: every wave is independent (no barrier).
template <int K, bool EXACT, bool EDGE, bool PUSH, int SH>
__device__ __forceinline__ void tb_block(const Args& a, const double* __restrict__ u, double* __restrict__ un,
                                         int64_t t) {
  using C = Cfg<K>;
  constexpr int G = C::S;
  extern __shared__ d2 lds_dyn[];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  // strip of the workgroup, stage of the strip (Args::shmap: stage major,
  // wave w = strip w % nw's stage w / nw)
  const bool smaj = G > 1 && a.shmap;
  const int sl = smaj ? wave % a.nw : wave / G, stage = smaj ? wave / a.nw : wave % G;
  int k = 0;
  while (k + 1 < a.n && t >= a.tstart[k + 1]) ++k;
  const int64_t lt = t - a.tstart[k];
  const int64_t ngroups = (a.nstrip[k] + a.nw - 1) / a.nw;
  // Dispatch order: (R) the row bands of a band-first pass (Args::rb_rect:
  // every strip group's segment next to a halo row side), then every
  // workgroup that can hold Dirichlet-rule waves (~1.5x the VALU per step),
  // so the launch's tail is made of fast ones: (A) the edge segments, all
  // strip groups; (B) the interior segments' first and last strip groups;
  // (C) the rest.
  // (K) before all of them: the column bands of a band-first pass
  // (Args::cb_rect: the first / last strip group, every segment).  The
  // categories below then cover the other groups only.
  const int64_t ry0 = a.r[k][2], ry1 = a.r[k][2] + a.r[k][3];
  const int64_t e0 = a.e0[k], e1 = a.e1[k];
  const int64_t nedge = (e0 > 0) + (e1 > 0);
  const int rbs = k == a.rb_rect ? a.rb_s : 0, rbn = k == a.rb_rect ? a.rb_n : 0, rb = rbs + rbn;
  // column-band groups: 0 (cb_lo) and ngroups - 1 (cb_hi); one group when there is only one
  const int cblo = k == a.cb_rect ? a.cb_lo : 0;
  const int cbhi = k == a.cb_rect && ngroups > 1 ? a.cb_hi : 0;
  const int64_t ncb = (cblo || (k == a.cb_rect && a.cb_hi && ngroups == 1)) + cbhi;
  const int64_t nsb = nedge + a.nmid_b[k];  // segments of a boundary group
  const int64_t ng = ngroups - ncb;         // the other groups: gi = cbf + 0 .. ng - 1
  const int64_t cbf = ncb > 0 && (cblo || ngroups == 1) ? 1 : 0;
  // the other boundary groups (0 / ngroups - 1 that are not column bands)
  const bool b0 = cbf == 0, b1 = ngroups > 1 && !cbhi;
  const int64_t nbnd = (b0 ? 1 : 0) + (b1 ? 1 : 0);
  const int64_t n_cb = ncb * nsb, n_rb = rb * ng, n_ed = nedge * ng, n_bd = (a.nmid_b[k] - rb) * nbnd;
  int64_t gi, m = -1;  // m: interior segment index, -1: edge segment `edge`
  int edge = 0, dir = 1;
  bool band = false;
  auto seg_of = [&](int64_t sg, int64_t nm) {  // segment sg of a group: edge 0, mids, edge 1
    if (e0 > 0 && sg == 0) {
      edge = 0;
    } else if (sg < (e0 > 0) + nm) {
      m = sg - (e0 > 0);
    } else {
      edge = 1;
    }
  };
  if (lt < n_cb) {  // (K)
    const int64_t c = lt / nsb;
    gi = (c == 0 && cbf) ? 0 : ngroups - 1;
    seg_of(lt % nsb, a.nmid_b[k]);
  } else if (lt < n_cb + n_rb) {  // (R): S band = first interior segment, N band = last (walked bottom-up)
    const int64_t l0 = lt - n_cb;
    gi = cbf + l0 % ng;
    const bool north = l0 >= ng || !rbs;
    const int64_t nm = (gi == 0 || gi == ngroups - 1) ? a.nmid_b[k] : a.nmid[k];
    m = north ? nm - 1 : 0;
    dir = north ? -1 : 1;
    band = true;
  } else if (lt < n_cb + n_rb + n_ed) {  // (A)
    const int64_t l1 = lt - n_cb - n_rb;
    edge = (l1 / ng == 0 && e0 > 0) ? 0 : 1;
    gi = cbf + l1 % ng;
  } else if (lt < n_cb + n_rb + n_ed + n_bd) {  // (B)
    const int64_t l2 = lt - n_cb - n_rb - n_ed;
    m = rbs + l2 / nbnd;
    gi = (l2 % nbnd == 0 && b0) ? 0 : ngroups - 1;
  } else {  // (C)
    const int64_t l3 = lt - n_cb - n_rb - n_ed - n_bd;
    m = rbs + l3 / (ngroups - 2);
    gi = 1 + l3 % (ngroups - 2);
  }
  // interior segment m of nm: rows [mid m / nm, mid (m + 1) / nm) of the
  // interior part — lengths differ by one row at most.  (Round 4 cut
  // ceil(mid / nm)-row segments and left the rest to the last one: 64
  // segments of 64 rows over 4036 left 4 rows for the last, a row band
  // shorter than the rows it signals, and a band-first pass that never
  // signalled: build/bench/plan_model --check-bands.)
  const int64_t nm = (gi == 0 || gi == ngroups - 1) ? a.nmid_b[k] : a.nmid[k];
  int64_t ys, ye;
  if (m < 0) {
    ys = edge == 0 ? ry0 : ry1 - e1;
    ye = edge == 0 ? ry0 + e0 : ry1;
  } else {
    const int64_t mid = ry1 - e1 - (ry0 + e0);
    ys = ry0 + e0 + m * mid / nm;
    ye = ry0 + e0 + (m + 1) * mid / nm;
  }
  // L + 2K steps (the output stage of a split strip runs LAG steps behind)
  constexpr int kU = C::U;
  // a row band's output wave publishes its arrival at the step that stores
  // the band's last row (the first sig_rows rows of its walk)
  const int sig_step = band ? static_cast<int>(C::LAG + 2 * K + a.sig_rows - 1) : -1;
  const int nsteps = static_cast<int>((ye - ys + 2 * K + C::LAG + kU - 1) / kU * kU);
  const int64_t strip = gi * a.nw + sl;
  if (strip >= a.nstrip[k]) {  // no strip for this wave
    if constexpr (G > 1) {
      // the workgroup's per-step barriers
      for (int s = 0; s < nsteps; ++s) step_barrier();
    }
    return;
  }
  constexpr int64_t wout = C::WOUT;
  const int64_t rx0 = a.r[k][0], rx1 = a.r[k][0] + a.r[k][1];
  int64_t xs, xe, cf;  // output columns [xs, xe) of this wave's strip, its window's first column
  char* ring;          // the strip's DMA ring (and, not SH, its hand-off rings)
  int hdelta = 0;      // SH: the shared hand-off ring's lane address - the DMA ring's
  uint64_t hm0 = 0, hm1 = 0;
  if constexpr (SH) {
    // group gi: output [gx, gx + GOUT), the last one shifted left to end at
    // rx1 (launch_tb: the rect is at least GOUT wide); stage 0 of strip sl
    // reads window ga + S0 sl, stage 1 window ga + O + S1 sl and stores its
    // slice of the group's output
    using H = Sh<K, SH>;
    int64_t gx = rx0 + gi * H::GOUT;
    if (gx + H::GOUT > rx1) gx = rx1 - H::GOUT;
    const int64_t ga = gx - H::ML;
    char* const lds = reinterpret_cast<char*>(lds_dyn);
    ring = lds + C::HS * H::ROWG + sl * (C::RS * C::ROW);
    int64_t off;
    if (stage == 0) {
      off = H::S0 * sl;
      xs = ga + off;
      xe = xs;  // stores nothing
      // the level-NL columns this strip owns in the shared row: [NL, NL + S0)
      // of its window (from 0 / to 256 for the first / last strip)
      const int lo = sl == 0 ? 0 : H::NL, hi = sl == H::NW - 1 ? 256 : H::NL + H::S0;
      const int c = 4 * lane;
      hm0 = __builtin_amdgcn_ballot_w64(c >= lo && c + 1 < hi);
      hm1 = __builtin_amdgcn_ballot_w64(c + 2 >= lo && c + 3 < hi);
    } else {
      off = H::O + H::S1 * sl;
      xs = gx + H::S1 * sl;
      xe = sl < H::NW - 1 ? xs + H::S1 : gx + H::GOUT;
    }
    cf = ga + off;
    // this lane's group in the shared row: off / 4 + lane, 16 B per group and plane
    hdelta = static_cast<int>(4 * off - (ring - lds));
  } else {
    xs = rx0 + strip * wout;
    if (xs + wout > rx1) xs = rx1 - wout > rx0 ? rx1 - wout : rx0;  // last strip: shifted left to end at rx1
    xe = xs + wout < rx1 ? xs + wout : rx1;
    cf = xs - C::KL;
    ring = reinterpret_cast<char*>(lds_dyn) + sl * strip_lds<K>();
  }
  // the rule path only where a computed cell can be a fixed ring cell
  const int64_t cx0 = cf, cx1 = cx0 + C::COLS;
  const bool rule = (cx0 < a.dom[0] && !(a.mask & 1)) || (cx1 > a.dom[0] + a.dom[1] && !(a.mask & 2)) ||
                    (ys - K < a.dom[2] && !(a.mask & 4)) || (ye + K > a.dom[2] + a.dom[3] && !(a.mask & 8));
  // A rule wave whose window holds one ghost column (a W / E Dirichlet
  // side) and no fixed row runs the one-column keep (RULE 2 + the ghost's
  // column slot — compile-time for the usual rect = interior pass, so only
  // those two bodies are built; other slots take the general rule)
  int rule_kind = rule ? 1 : 0;
  // the ghost columns' slots (SH: Sh<K>; a per-strip window starts KL, a
  // multiple of 4, left of its first output column: W ghost in slot 3, E
  // ghost 256 - KL right of the last strip's window start, slot 0)
  // (SH only: in the per-strip K = 20 kernel the two extra bodies spilled
  // 12-14 VGPRs)
  constexpr bool kColBodies = SH;
  constexpr int kJW = SH ? Sh<K, SH ? SH : 4>::kJW : 3, kJE = SH ? Sh<K, SH ? SH : 4>::kJE : 0;
  if constexpr (kColBodies) {
    const bool ry = (ys - K < a.dom[2] && !(a.mask & 4)) || (ye + K > a.dom[2] + a.dom[3] && !(a.mask & 8));
    const int64_t gw0 = a.dom[0] - 1, ge0 = a.dom[0] + a.dom[1];
    const bool hw = !(a.mask & 1) && cx0 <= gw0 && gw0 < cx1, he = !(a.mask & 2) && cx0 <= ge0 && ge0 < cx1;
    if (rule && !ry && hw != he && a.col_keep) {
      const int jslot = static_cast<int>(((hw ? gw0 : ge0) - cx0) & 3);
      if (jslot == kJW || jslot == kJE) rule_kind = 2 + jslot;
    }
  }
  // one instantiation per (stage, rule path, direction); the direction is
  // bottom-up only for the N row bands
  // the x face this strip pushes (PUSH): the first strip holds the W one,
  // the last the E one (launch_tb: at least two strips when both are pushed)
  const bool pw = PUSH && (a.push[GMT_PUSH_W] || a.push[GMT_PUSH_SW] || a.push[GMT_PUSH_NW]);
  const bool pe = PUSH && (a.push[GMT_PUSH_E] || a.push[GMT_PUSH_SE] || a.push[GMT_PUSH_NE]);
  const int xd = !PUSH ? -1 : (strip == 0 && pw) ? GMT_PUSH_W : (strip == a.nstrip[k] - 1 && pe) ? GMT_PUSH_E : -1;
  // the output body by the faces this wave holds (the face stores are
  // issued every step, in range or not): most waves hold none and run the
  // plain body, the first / last strip an x face, the segments at the S / N
  // face rows a y face
  const bool py = PUSH && (((a.push[GMT_PUSH_S] || a.push[GMT_PUSH_SW] || a.push[GMT_PUSH_SE]) &&
                            ys < a.dom[2] + a.push_w) ||
                           ((a.push[GMT_PUSH_N] || a.push[GMT_PUSH_NW] || a.push[GMT_PUSH_NE]) &&
                            ye > a.dom[2] + a.dom[3] - a.push_w));
  const int pm = (xd >= 0 ? 1 : 0) | (py ? 2 : 0);
  using T = std::true_type;
  using F = std::false_type;
  auto go = [&](auto jc, auto rule_c, auto up_c, int sstep) {
    constexpr int j = decltype(jc)::value;
    auto run = [&](auto push_c) {
      run_stage<K, j, EXACT, EDGE, decltype(rule_c)::value, decltype(up_c)::value, decltype(push_c)::value, SH>(
          a, u, un, ring, lane, xs, xe, ys, ye, nsteps, sstep, xd, cf, hdelta, hm0, hm1);
    };
    using P0 = std::integral_constant<int, 0>;
    if constexpr (PUSH && j == G - 1) {
      // (two bodies: one per face group — x alone, y alone — spills the
      // kernel: 71-93 VGPRs of scratch; a wave holding any face runs all
      // three groups, the ones it does not hold dropped by their descriptors)
      if (pm != 0) run(std::integral_constant<int, 3>{});
      else run(P0{});
    } else {
      run(P0{});
    }
  };
  auto stage_go = [&](auto jc, int sstep) {
    if constexpr (!SH) {
      if (!PUSH && dir < 0) {  // (no row bands in an inline-halo pass)
        if (rule) go(jc, std::integral_constant<int, 1>{}, T{}, sstep);
        else go(jc, std::integral_constant<int, 0>{}, T{}, sstep);
        return;
      }
    }
    // (an SH pass has no row bands: top-down bodies only)
    using R0 = std::integral_constant<int, 0>;
    using R1 = std::integral_constant<int, 1>;
    if constexpr (kColBodies) {
      using RW = std::integral_constant<int, 2 + kJW>;
      using RE = std::integral_constant<int, 2 + kJE>;
      if (rule_kind == 0) go(jc, R0{}, F{}, sstep);
      else if (rule_kind == RW::value) go(jc, RW{}, F{}, sstep);
      else if (rule_kind == RE::value && RE::value != RW::value) go(jc, RE{}, F{}, sstep);
      else go(jc, R1{}, F{}, sstep);
    } else {
      if (rule) go(jc, R1{}, F{}, sstep);
      else go(jc, R0{}, F{}, sstep);
    }
  };
  if constexpr (G == 1) {
    stage_go(std::integral_constant<int, 0>{}, sig_step);
  } else {
    static_for<0, G>([&](auto Jc) {
      constexpr int j = decltype(Jc)::value;
      if (stage == j) {
        if constexpr (j == 0) {
          // a launch of one round has no later workgroups to fill the SIMDs
          // while a strip's later stages wait on its stage 0: favour the
          // producer (profiles/r02_tb.md 9.4)
          if (a.prio) __builtin_amdgcn_s_setprio(2);
        }
        stage_go(Jc, j == G - 1 ? sig_step : -1);
      }
    });
  }
}

// Tile of block b for a launch of nb blocks whose first ne tiles (the edge
// segments) go last: the hardware hands block b to XCD b % 8 as that XCD's
// (b / 8)-th block; XCD x runs its contiguous share of the nb - ne other
// tiles (in tile order, as xcd_swizzle), then its share of the edge tiles.
// Returns -1 when some XCD's block count cannot hold its share (a caller
// falls back to xcd_swizzle; tail_swizzle_ok checks it on the host).
__host__ __device__ inline int64_t tail_swizzle(int64_t b, int64_t nb, int64_t ne) {
  const int64_t nm = nb - ne;
  const int64_t x = b % kNumXcd, k = b / kNumXcd;
  const int64_t nx = nb / kNumXcd + (x < nb % kNumXcd ? 1 : 0);        // blocks of XCD x
  const int64_t qm = nm / kNumXcd, rm = nm % kNumXcd;
  const int64_t ms = qm + (x < rm ? 1 : 0);                             // its other tiles
  const int64_t mstart = x * qm + (x < rm ? x : rm);
  if (k < ms) return ne + mstart + k;
  // edge tiles: XCD x holds nx - ms of them, after the edge tiles of XCDs < x
  int64_t estart = 0;
  for (int64_t y = 0; y < x; ++y)
    estart += nb / kNumXcd + (y < nb % kNumXcd ? 1 : 0) - (qm + (y < rm ? 1 : 0));
  return estart + (k - ms);
}
inline bool tail_swizzle_ok(int64_t nb, int64_t ne) {
  if (ne <= 0 || ne >= nb) return false;
  const int64_t nm = nb - ne;
  for (int64_t x = 0; x < kNumXcd; ++x)
    if (nb / kNumXcd + (x < nb % kNumXcd ? 1 : 0) < nm / kNumXcd + (x < nm % kNumXcd ? 1 : 0)) return false;
  return true;
}

template <int K, bool EXACT, bool EDGE, bool PUSH, int SH>
__global__ __launch_bounds__(kMaxThreads) __attribute__((amdgpu_waves_per_eu(2)))
void jacobi5tb_kernel(Args a, const double* __restrict__ u, double* __restrict__ un, int64_t nblocks) {
  if constexpr (PUSH) {
    // a hand-over that timed out: the ghost cells are stale and a late
    // neighbour may still write them; the host aborts at its next sync
    if (a.stop && *a.stop != 0) return;
  }
  const int64_t ns = a.sig_wgs, nd = a.sig_dispatch;
  const int64_t b = blockIdx.x;
  // clock record: wave 0 of one workgroup in 256, from the middle of each
  // 256: its start stamps go to 16 B of LDS past the strips' rings (no
  // memory operation in front of the pipeline's exact vmcnt waits: start
  // atomics here cost a one-round 8192^2 pass 1.6%, profiles/r06_clock/),
  // the deltas go out by vector atomics once the workgroup's work is done
  extern __shared__ d2 lds_dyn[];
  uint64_t* stamp = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(lds_dyn) +
                                                (SH ? sh_lds<K, SH ? SH : 4>() : a.nw * strip_lds<K>()));
  const bool clk = a.clk && (b & 255) == 128 && threadIdx.x == 0;
  if (clk) {
    stamp[0] = __builtin_amdgcn_s_memtime();
    stamp[1] = __builtin_amdgcn_s_memrealtime();
  }
  // signalling workgroups (and row bands) first, in dispatch order over all
  // XCDs; the rest XCD-contiguous
  const int64_t t = a.edges_last > 0 ? tail_swizzle(b, nblocks, a.edges_last)
                    : b < nd ? b : nd + xcd_swizzle(b - nd, nblocks - nd);
#if GMT_TB_WG_TRACE
  const uint64_t wg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  tb_block<K, EXACT, EDGE, PUSH, SH>(a, u, un, t);
  if (clk) {
    const uint64_t m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_fetch_add(a.clk, m1 - stamp[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(a.clk + 1, r1 - stamp[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(a.clk + 2, uint64_t{1}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#if GMT_TB_WG_TRACE
  __syncthreads();
  if (threadIdx.x == 0 && a.wg_trace) {
    const uint64_t wg_t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
    const uint64_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    uint64_t* o = a.wg_trace + 4 * b;  // vector stores (a VGPR address)
    o[0] = static_cast<uint64_t>(t);
    o[1] = wg_t0;
    o[2] = wg_t1;
    o[3] = hw | (xcc << 32);
  }
#endif
  if (t < ns) {
    // every wave's stores written back past its XCD's L2, then one arrival
    // per workgroup (vector atomics on uncached memory)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(a.sig_count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
            static_cast<unsigned>(a.sig_total - 1)) {
      __hip_atomic_store(a.sig_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(a.signal, uint64_t{1}, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace tb
}  // namespace gmt
namespace {

using namespace gmt;
using namespace gmt::tb;

// Segment plan (rows per strip).  Every segment pays a 2K-step pipeline
// warm-up, so interior segments should be long; but a wave whose segment
// touches a Dirichlet row runs the rule path (~1.5x the VALU per step) for
// the whole segment, and the launch ends with its slowest round.  Measured
// (profiles/r02_tb4.md, K = 20, 32768^2): all-halo sides 4.41M MLUPS at 384
// rows and 4.61M at 1024-2048; with Dirichlet sides 3.78M at 384, falling
// to 2.38M at 4096.  So: short edge segments (max(64, K) rows) where the
// rect touches a Dirichlet row, and interior segments whose length L
// minimises rounds(L) x (L + 2K), rounds = ceil(workgroups / resident
// workgroups), over L in [128, 2048].
struct SegPlan {
  int64_t e0[kMaxRect], e1[kMaxRect], nmid[kMaxRect], lmid[kMaxRect], nmid_b[kMaxRect], lmid_b[kMaxRect];
  bool tail;  // dispatch the edge segments last on every XCD (launch_tb: Args::edges_last)
};

// Signalling rects (k < sig_rects: the boundary bands of a pass whose halo
// exchange overlaps the rest of it) get segments of max(128, 3L/4) rows and
// no edge split: their workgroups are dispatched first and end a quarter of
// a segment before the rest of their round, which is when the exchange runs
// (L/3 cost 1.5-5 % more on the 1-GPU shares: more workgroups, more 2K-step
// warm-ups; profiles/r03_band_lb).
// A row-band rect (rb_rect, gmt_tb_opts.signal_rows) keeps at least `rb`
// interior segments per strip group, each at least rb_min rows long, so its
// S and N bands are separate segments that finish early.
// The step cost of a rule-path wave relative to a plain one (the planner's
// model).  Loop census at K = 20 per 19 steps: round 4's per-cell select
// 5837 vs 3218 VALU (1.8); the exec-masked keep 3882 VALU + 1711 SALU vs
// 3150 VALU + 319 SALU (1.23x the VALU) — yet plans made with 1.2-1.5 run
// 2-10% slower than with 1.8 on every Dirichlet domain measured
// (profiles/r05_rule_keep/rule_cost_sweep.txt): a rule wave still takes
// ~1.8x a plain one's time.  GMT_TB_RULE_COST=c overrides it (A/B).
inline double tb_rule_cost() {
  static const double c = [] {
    const char* e = std::getenv("GMT_TB_RULE_COST");
    const double v = e ? std::atof(e) : 0.0;
    return v >= 1.0 && v <= 4.0 ? v : 1.8;
  }();
  return c;
}

// The step cost of a wave running the one-column Dirichlet keep (SH x-side
// rule waves: one write and 2 SALU per level, ~1.06x the VALU of a plain
// wave) relative to a plain one.  GMT_TB_RULE_COL_COST=c overrides it.
inline double tb_rule_col_cost() {
  static const double c = [] {
    const char* e = std::getenv("GMT_TB_RULE_COL_COST");
    const double v = e ? std::atof(e) : 0.0;
    return v >= 1.0 && v <= 4.0 ? v : 1.15;
  }();
  return c;
}

// The step cost of a wave running the inline-halo body (three face store
// groups per step, the ones out of range dropped) relative to a plain one:
// a one-round pass whose push waves had plain-length segments ran
// 1.11-1.14x, per-workgroup timelines put push tiles at 1.17x per step, and
// planning at 1.3 ran the application fastest on both N = 8 shares
// (profiles/r05_overlap/app_push_cost_sweep.txt).  GMT_TB_PUSH_COST=c
// overrides it.
inline double tb_push_cost() {
  static const double c = [] {
    const char* e = std::getenv("GMT_TB_PUSH_COST");
    const double v = e ? std::atof(e) : 0.0;
    return v >= 1.0 && v <= 4.0 ? v : 1.3;
  }();
  return c;
}

template <int K>
// push_sides (inline halo exchange, the one rect is the interior): the faces
// pushed, bits 1 W, 2 E, 4 S, 8 N (a corner counts for both its faces).  The
// waves holding a face run the push body: the S / N face rows get edge
// segments of their own and the W / E strips' groups shorter segments, both
// priced at tb_push_cost().  With both S and N pushed every segment holds at
// most one of the two faces (launch_tb: ny >= 2 w + 2).
SegPlan plan_segments(const Args& a, int seg_rows, int64_t lmax, int64_t resident_wgs, int sig_rects, int rb_rect = -1,
                      int rb = 0, int64_t rb_min = 0, int push_sides = 0) {
  SegPlan p{};
  const bool push_ns = (push_sides & 12) == 12;
  // A rule segment costs ~tb_rule_cost() times the steps of a plain one.  Edge segments
  // (at a Dirichlet row) are either short (64 rows: many of them pack well
  // into the tail of a multi-round launch) or "balanced" — as long as makes
  // them cost what an L-row interior segment costs, so a one-round launch
  // (the N = 8 shares, 8192^2) neither waits for them nor leaves their slots
  // idle; the makespan search tries both.  Strip groups that reach a
  // Dirichlet column run the rule path at every step: balanced segments.
  const double fr = tb_rule_cost(), fp = tb_push_cost();
  constexpr int64_t kWarm = 2 * K + Cfg<K>::LAG, kU = Cfg<K>::U;
  // a segment's rows such that its steps (whole unrolled blocks of kU) at
  // cost factor f cost at most those of an L-row plain one
  auto balanced = [](int64_t L, double f) {
    const int64_t st = (L + kWarm + kU - 1) / kU * kU;
    const int64_t blocks = static_cast<int64_t>(static_cast<double>(st) / (f * kU) + 1e-9);
    return std::max<int64_t>(64, blocks * kU - kWarm);
  };
  // per-side cost factors of rect k's waves: rule path (Dirichlet side) and
  // push body (pushed face), out[0..3] = W, E, S, N
  auto side_cost = [&](int k, double* out) {
    const int64_t ry0 = a.r[k][2], ry1 = ry0 + a.r[k][3], rx0 = a.r[k][0], rx1 = rx0 + a.r[k][1];
    const int64_t kl = a.sh ? Sh<K>::ML : Cfg<K>::KL;  // window columns left of the first output column
    const bool rule[4] = {rx0 - kl < a.dom[0] && !(a.mask & 1), rx1 + kl > a.dom[0] + a.dom[1] && !(a.mask & 2),
                          ry0 - K < a.dom[2] && !(a.mask & 4), ry1 + K > a.dom[2] + a.dom[3] && !(a.mask & 8)};
    // (the x sides' interior segments run the one-column keep)
    const double frx = a.col_keep ? tb_rule_col_cost() : fr;
    for (int d = 0; d < 4; ++d) out[d] = (rule[d] ? (d < 2 ? frx : fr) : 1.0) * ((push_sides >> d) & 1 ? fp : 1.0);
  };
  bool long_edges = false;
  auto fill = [&](int64_t L0, int64_t* wgs) {
    int64_t w = 0;
    for (int k = 0; k < a.n; ++k) {
      int64_t L = L0;
      const int64_t ny = a.r[k][3];
      if (k < sig_rects) {
        const int64_t lb = std::min<int64_t>(std::max<int64_t>(128, L - L / 4), lmax);
        p.e0[k] = p.e1[k] = 0;
        p.nmid[k] = p.nmid_b[k] = (ny + lb - 1) / lb;
        p.lmid[k] = p.lmid_b[k] = (ny + p.nmid[k] - 1) / p.nmid[k];
        w += (a.nstrip[k] + a.nw - 1) / a.nw * p.nmid[k];
        continue;
      }
      double sc[4];
      side_cost(k, sc);
      // edge segments where the row sides cost more (a Dirichlet row, a pushed face)
      const bool top = seg_rows == 0 && sc[2] > 1.0, bot = seg_rows == 0 && sc[3] > 1.0;
      const int64_t edge0 = long_edges ? balanced(L0, sc[2]) : std::max<int64_t>(64, K);
      const int64_t edge1 = long_edges ? balanced(L0, sc[3]) : std::max<int64_t>(64, K);
      p.e0[k] = p.e1[k] = 0;
      if (ny > edge0 + edge1 + 64) {  // room for edges and an interior
        p.e0[k] = top ? edge0 : 0;
        p.e1[k] = bot ? edge1 : 0;
      }
      int64_t mid = ny - p.e0[k] - p.e1[k];
      if (k == rb_rect && rb > 0) L = std::min<int64_t>(L, std::max<int64_t>(rb_min, mid / rb));
      if (push_ns) L = std::min<int64_t>(L, (mid + 1) / 2);
      p.nmid[k] = (mid + L - 1) / L;
      p.lmid[k] = (mid + p.nmid[k] - 1) / p.nmid[k];  // balanced lengths
      if (long_edges && (p.e0[k] > 0 || p.e1[k] > 0)) {
        // the edges' length follows the interior segments' final length (a
        // few fixed-point steps: both depend on each other)
        for (int it = 0; it < 4; ++it) {
          p.e0[k] = p.e0[k] > 0 ? std::min<int64_t>(balanced(p.lmid[k], sc[2]), (ny - 64) / 2) : 0;
          p.e1[k] = p.e1[k] > 0 ? std::min<int64_t>(balanced(p.lmid[k], sc[3]), (ny - 64) / 2) : 0;
          mid = ny - p.e0[k] - p.e1[k];
          p.lmid[k] = (mid + p.nmid[k] - 1) / p.nmid[k];
        }
      }
      // strip groups that can reach a Dirichlet column run the rule path
      // (tb_rule_cost() per step), the W / E strips of a push pass the push
      // body: shorter segments, so they finish with the others instead of
      // ending the launch
      const double fx = seg_rows == 0 ? std::max(sc[0], sc[1]) : 1.0;
      int64_t lb = fx > 1.0 ? balanced(p.lmid[k], fx) : p.lmid[k];
      if (k == rb_rect && rb > 0) lb = std::min<int64_t>(lb, std::max<int64_t>(rb_min, mid / rb));
      if (push_ns) lb = std::min<int64_t>(lb, (mid + 1) / 2);
      p.nmid_b[k] = (mid + lb - 1) / lb;
      p.lmid_b[k] = (mid + p.nmid_b[k] - 1) / p.nmid_b[k];
      const int64_t groups = (a.nstrip[k] + a.nw - 1) / a.nw, nbnd = groups < 2 ? groups : 2;
      w += groups * ((p.e0[k] > 0) + (p.e1[k] > 0)) + nbnd * p.nmid_b[k] + (groups - nbnd) * p.nmid[k];
    }
    *wgs = w;
  };
  int64_t wgs = 0;
  if (seg_rows > 0) {
    fill(std::min<int64_t>(seg_rows, lmax), &wgs);
    return p;
  }
  // A/B of the model's choice: GMT_TB_PLAN_L=L plans segments of L rows with
  // everything else (edges, rule groups, bands) as the model would
  static const int64_t forced_l = [] {
    const char* e = std::getenv("GMT_TB_PLAN_L");
    return e ? std::max<int64_t>(0, std::atoll(e)) : int64_t(0);
  }();
  if (forced_l > 0) {
    fill(std::min<int64_t>(std::max<int64_t>(forced_l, 64), lmax), &wgs);
    return p;
  }
  // The launch's time is its makespan: workgroups start in dispatch order
  // on the first free slot (resident_wgs of them) and run (rows + 2K + lag)
  // steps, rounded up to the unroll, rule-path ones tb_rule_cost() times
  // longer per step.
  // Round 3 priced a plan as rounds x (L + 2K), blind to the short edge and
  // boundary-group workgroups that finish early and leave their slots idle
  // for the rest of a round: 15% of a one-round 8192 x 16384 pass
  // (profiles/r04_shares.md).  The dispatch order modelled is tb_block's:
  // per rect, column bands, row bands, edge segments, boundary groups, rest,
  // on one pool of slots (the XCD-contiguous tile order is not modelled).
  constexpr int64_t u = Cfg<K>::U;
  auto steps = [&](int64_t rows) { return static_cast<double>((rows + 2 * K + Cfg<K>::LAG + u - 1) / u * u); };
  std::vector<double> dur;
  std::vector<double> slot;
  // The edges-last order (tail_swizzle): one-rect passes without signals
  // whose other tiles fill at least two rounds — short edge tiles then fill
  // the last round's tail (32768^2: +1.2%); a one-round launch gets a second
  // round of edges only and ran 4% slower (profiles/r05_wg_timeline/).
  // GMT_TB_EDGES_LAST=0 / 1 forbids / forces it (A/B).
  static const int tail_mode = [] {
    const char* e = std::getenv("GMT_TB_EDGES_LAST");
    return e ? std::atoi(e) : -1;
  }();
  const bool tail_possible = a.n == 1 && sig_rects == 0 && rb_rect < 0 && seg_rows == 0 && tail_mode != 0;
  bool tail_edges = false;
  auto makespan = [&]() {
    dur.clear();
    for (int k = 0; k < a.n; ++k) {
      const int64_t groups = (a.nstrip[k] + a.nw - 1) / a.nw, nbnd = groups < 2 ? groups : 2;
      double sc[4];
      side_cost(k, sc);
      // a workgroup's factor: the rule path if any side it touches is a
      // Dirichlet one, the push body if it holds any face; without edge
      // segments the row sides fall to the first / last interior segments
      // (modelled on all of them)
      const double fx = std::max(sc[0], sc[1]);
      const bool edges = p.e0[k] > 0 || p.e1[k] > 0;
      const double fy = edges ? 1.0 : std::max(sc[2], sc[3]);
      const double fb = std::max(fx, fy), fm = fy;
      auto edge_tiles = [&]() {
        for (int64_t g = 0; g < groups; ++g) {
          const bool bnd = g == 0 || g == groups - 1;
          if (p.e0[k] > 0) dur.push_back((bnd ? std::max(sc[2], fx) : sc[2]) * steps(p.e0[k]));
          if (p.e1[k] > 0) dur.push_back((bnd ? std::max(sc[3], fx) : sc[3]) * steps(p.e1[k]));
        }
      };
      if (!tail_edges) edge_tiles();
      for (int64_t g = 0; g < nbnd; ++g)
        for (int64_t m = 0; m < p.nmid_b[k]; ++m) dur.push_back(fb * steps(p.lmid_b[k]));
      for (int64_t g = nbnd; g < groups; ++g)
        for (int64_t m = 0; m < p.nmid[k]; ++m) dur.push_back(fm * steps(p.lmid[k]));
      if (tail_edges) edge_tiles();  // launch_tb's edges_last order (one-rect passes)
    }
    // list scheduling on the resident slots (a min-heap of free times)
    const size_t ns = static_cast<size_t>(std::max<int64_t>(1, resident_wgs));
    slot.assign(std::min(ns, dur.size()), 0.0);
    size_t used = 0;
    double end = 0.0;
    auto cmp = [](double x, double y) { return x > y; };
    for (double d : dur) {
      double t0 = 0.0;
      if (used < slot.size()) {
        slot[used++] = d;
        if (used == slot.size()) std::make_heap(slot.begin(), slot.end(), cmp);
        end = std::max(end, d);
        continue;
      }
      std::pop_heap(slot.begin(), slot.end(), cmp);
      t0 = slot.back();
      slot.back() = t0 + d;
      std::push_heap(slot.begin(), slot.end(), cmp);
      end = std::max(end, t0 + d);
    }
    return end;
  };
  // GMT_TB_PLAN_DEBUG=1: every candidate on stderr (build/bench/plan_model)
  static const bool debug = std::getenv("GMT_TB_PLAN_DEBUG") != nullptr;
  auto eval = [&](int le, int64_t L) {
    long_edges = le == 1;
    fill(L, &wgs);
    const int64_t groups0 = (a.nstrip[0] + a.nw - 1) / a.nw;
    const int64_t ne = groups0 * ((p.e0[0] > 0) + (p.e1[0] > 0));
    const bool can_tail = tail_possible && ne > 0 && wgs - ne >= 2 * resident_wgs;
    tail_edges = false;
    double cost = makespan();
    bool tail = false;
    if (can_tail && tail_mode == 1) cost = 1e300;  // forced: only the tail order
    if (can_tail) {
      tail_edges = true;
      const double ct = makespan();
      if (ct < cost - 1e-9) {
        cost = ct;
        tail = true;
      }
    }
    if (debug)
      std::fprintf(stderr, "plan le %d L %lld e %lld/%lld mid %lld x %lld b %lld x %lld wgs %lld tail %d cost %.1f\n",
                   le, (long long)L, (long long)p.e0[0], (long long)p.e1[0], (long long)p.nmid[0],
                   (long long)p.lmid[0], (long long)p.nmid_b[0], (long long)p.lmid_b[0], (long long)wgs, tail ? 1 : 0,
                   cost);
    return std::make_pair(cost, tail);
  };
  // coarse (16 rows), then every length within 16 rows of each edge mode's
  // coarse best (segment counts are integers: a plan one segment shorter
  // can tip a launch into or out of one round)
  const int64_t lhi = std::min<int64_t>(2048, lmax);
  int64_t best_l = 128;
  bool best_long = false, best_tail = false;
  double best = 1e300;
  // A/B: GMT_TB_EDGES=1 plans short edge segments only, 2 balanced ones only
  static const int edges_mode = [] {
    const char* e = std::getenv("GMT_TB_EDGES");
    return e ? std::atoi(e) : 0;
  }();
  for (int le = 0; le < 2; ++le) {
    if ((edges_mode == 1 && le == 1) || (edges_mode == 2 && le == 0)) continue;
    int64_t c0 = 128;
    double b0 = 1e300;
    for (int64_t L = 128; L <= lhi; L += 16) {
      const double cost = eval(le, L).first;
      if (cost < b0 - 1e-9) {
        b0 = cost;
        c0 = L;
      }
    }
    for (int64_t L = std::max<int64_t>(128, c0 - 15); L <= std::min(lhi, c0 + 15); ++L) {
      const auto [cost, tail] = eval(le, L);
      if (cost < best - 1e-9) {
        best = cost;
        best_l = L;
        best_long = le == 1;
        best_tail = tail;
      }
    }
  }
  long_edges = best_long;
  fill(std::min<int64_t>(best_l, lmax), &wgs);
  p.tail = best_tail;
  return p;
}

// Fills the kernel arguments and the launch shape; info (optional) gets
// {workgroups, resident workgroups, threads per workgroup, rows per interior
// segment and interior segments of the first rect, VGPRs per lane}.
template <int K, bool EXACT, bool EDGE, bool PUSH, int SH>
int launch_tb(const gmt_tb_opts& o, int n_rect, const int64_t* rects, const int64_t* dom, int mask, const double* u,
              double* un, int64_t ld, int64_t nrows, hipStream_t s, int64_t* info = nullptr) {
  using C = Cfg<K>;
  constexpr int G = C::S;
  constexpr int kMaxStrips = tb_max_strips(K);
  Args a{};
  a.nw = std::min(o.wg_waves > 0 ? o.wg_waves : tb_default_strips(K), kMaxStrips);  // multi-stage: one strip (profiles/r02_tb4/launch_shapes.txt)
  static const int col_keep = [] {
    const char* e = std::getenv("GMT_TB_COL_KEEP");
    return e ? std::atoi(e) : 1;
  }();
  a.col_keep = col_keep != 0 && SH;
  if constexpr (!SH && G > 1) {
    // several two-stage strips per workgroup: stage-major waves (all the
    // stage-0 waves first) — 32768^2 with two strips 5.24-5.25M MLUPS
    // against 4.91-4.93M for one strip per workgroup, same box
    // (profiles/r06_shared/ab_p.txt).  A large one-rect pass (more than
    // 2^28 points: several rounds) defaults to two strips; one-round passes
    // keep one (the N = 8 shares lost up to 9% with two).  GMT_TB_STRIP_MAP=0
    // keeps strip-major waves and one strip (A/B).
    static const int strip_map = [] {
      const char* e = std::getenv("GMT_TB_STRIP_MAP");
      return e ? std::atoi(e) : 1;
    }();
    if (strip_map != 0 && o.wg_waves == 0 && o.seg_rows == 0 && o.signal_rects == 0 &&
        o.signal_rows == 0 && (o.signal_cols & 3) == 0) {
      int64_t nonempty = 0, area = 0;
      for (int k = 0; k < n_rect; ++k)
        if (rects[4 * k + 1] > 0 && rects[4 * k + 3] > 0) {
          ++nonempty;
          area = rects[4 * k + 1] * rects[4 * k + 3];
        }
      if (nonempty == 1 && area > (int64_t(1) << 28)) a.nw = 2;
    }
    a.shmap = strip_map != 0 && a.nw > 1;
  }
  if constexpr (SH) {
    static_assert(Sh<K, SH>::kOk && !EDGE && !PUSH, "SH launches: plain two-stage bodies");
    a.nw = Sh<K, SH>::NW;
    a.sh = 1;
    // stage-major waves: each SIMD then holds one stage-0 and one stage-1
    // wave (the dispatcher deals a workgroup's waves to consecutive SIMDs,
    // build/bench/wave_place); strip-major put two stage-0 or two stage-1
    // waves on every SIMD: 32768^2 5.0M against 4.8M MLUPS (profiles/r06_shared/)
    static const int shmap = [] {
      const char* e = std::getenv("GMT_TB_SH_MAP");
      return e ? std::atoi(e) : 1;
    }();
    a.shmap = shmap != 0;
  }
  a.ld = ld;
  a.last_row = nrows - 1;
  a.mask = mask;
  a.quarter = 0.25;
  for (int j = 0; j < 4; ++j) a.dom[j] = dom[j];
  int push_sides = 0;  // plan_segments: faces pushed, 1 W, 2 E, 4 S, 8 N
  if constexpr (PUSH) {
    // gmt_tb_opts.push: the one rect is the interior, an even face width,
    // room for two segments clear of each other's face, no signals
    const int64_t w = o.push_w;
    bool ok = n_rect == 1 && w > 0 && w <= 64 && (w & 1) == 0 && o.signal_rects == 0 && o.signal_rows == 0 &&
              o.signal_cols == 0 && o.seg_rows == 0 && dom[1] >= w && dom[3] >= 2 * w + 2;
    for (int j = 0; ok && j < 4; ++j) ok = rects[j] == dom[j];
    if (!ok) return static_cast<int>(hipErrorInvalidValue);
    for (int d = 0; d < 8; ++d) a.push[d] = o.push[d];
    a.push_w = w;
    // (a face counts as pushed when only its corners are)
    const auto any = [&](int d0, int d1, int d2) { return o.push[d0] || o.push[d1] || o.push[d2]; };
    push_sides = (any(GMT_PUSH_W, GMT_PUSH_SW, GMT_PUSH_NW) ? 1 : 0) | (any(GMT_PUSH_E, GMT_PUSH_SE, GMT_PUSH_NE) ? 2 : 0) |
                 (any(GMT_PUSH_S, GMT_PUSH_SW, GMT_PUSH_SE) ? 4 : 0) | (any(GMT_PUSH_N, GMT_PUSH_NW, GMT_PUSH_NE) ? 8 : 0);
    // a strip pushes one x face
    if (any(GMT_PUSH_W, GMT_PUSH_SW, GMT_PUSH_NW) && any(GMT_PUSH_E, GMT_PUSH_SE, GMT_PUSH_NE) &&
        (dom[1] + C::WOUT - 1) / C::WOUT < 2)
      return static_cast<int>(hipErrorInvalidValue);
  }
  using SHG = Sh<K, SH ? SH : 4>;
  constexpr int64_t wout = SH ? SHG::GOUT : C::WOUT;  // SH: a group's columns
  int64_t maxh = 0;
  for (int k = 0; k < n_rect; ++k) {
    const int64_t* r = rects + 4 * k;
    if (r[1] <= 0 || r[3] <= 0) continue;
    if (SH && r[1] < wout) return static_cast<int>(hipErrorInvalidValue);  // (dispatch_k checks it)
    for (int j = 0; j < 4; ++j) a.r[a.n][j] = r[j];
    a.nstrip[a.n] = SH ? SHG::NW * ((r[1] + wout - 1) / wout) : (r[1] + wout - 1) / wout;
    maxh = std::max(maxh, r[3]);
    ++a.n;
  }
  if (a.n == 0) return 0;
  // all strips of a rect narrower than nw strips: fewer strips per workgroup
  int64_t maxs = 0;
  for (int k = 0; k < a.n; ++k) maxs = std::max(maxs, a.nstrip[k]);
  if (a.nw > maxs) a.nw = static_cast<int>(maxs);
  // the kernel addresses a segment's rows through 32-bit buffer offsets:
  // (L + 3K + 2 unroll + prefetch) rows of ld doubles must stay below 2^31
  const int64_t lmax = std::min<int64_t>(1 << 20, (int64_t(1) << 31) / (ld * 8) - 3 * K - C::LAG - 2 * C::U - C::P);
  if (lmax < 1) return static_cast<int>(hipErrorInvalidValue);
  (void)maxh;
  // + 16 B: the clock record's start stamps (jacobi5tb_kernel)
  const size_t smem = static_cast<size_t>(SH ? sh_lds<K, SH ? SH : 4>() : a.nw * strip_lds<K>()) + 16;
  if (smem > 65536) {  // above the default dynamic-LDS limit (gfx950 has 160 KB per CU)
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&jacobi5tb_kernel<K, EXACT, EDGE, PUSH, SH>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(smem));
    if (e != hipSuccess) return static_cast<int>(e);
  }
  // resident workgroups on the device for this shape (registers, LDS);
  // queried once per device, kernel and strips-per-workgroup (an idempotent
  // cache: a process driving several devices keeps one entry per device)
  constexpr int kMaxDev = 64;
  static std::atomic<int> resident[kMaxDev][3][kMaxThreads / kWave + 1] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::atomic<int>* slot = dev >= 0 && dev < kMaxDev ? &resident[dev][SH / 2][a.nw] : nullptr;
  int per_cu = slot ? slot->load(std::memory_order_relaxed) : 0;
  if (per_cu <= 0) {
    int occ = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(&jacobi5tb_kernel<K, EXACT, EDGE, PUSH, SH>),
                                                     a.nw * G * kWave, smem) != hipSuccess || occ < 1)
      occ = 1;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    per_cu = occ * cus;
    if (slot) slot->store(per_cu, std::memory_order_relaxed);
  }
  // a CU-masked stream: the resident workgroups of the CUs it may use
  if (o.reserved_cus > 0) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (o.reserved_cus < cus) per_cu = static_cast<int>(static_cast<int64_t>(per_cu) * (cus - o.reserved_cus) / cus);
  }
  const int sig_rects = o.signal_rects;  // non-empty rects (checked): the same indices after the compaction
  // column bands: the first rect after the signalling ones (checked non-empty)
  const int cbk = (o.signal_cols & 3) ? sig_rects : -1;
  if (cbk >= a.n) return static_cast<int>(hipErrorInvalidValue);
  // row bands: the first rect after the signalling ones (checked non-empty)
  const int rbk = o.signal_rows > 0 ? sig_rects : -1;
  const int rbs = rbk >= 0 && (mask & 4) ? 1 : 0, rbn = rbk >= 0 && (mask & 8) ? 1 : 0;
  const int64_t rb_min = std::max<int64_t>(32, o.signal_rows);
  if (rbk >= 0 && (rbk >= a.n || rbs + rbn == 0 || a.r[rbk][3] < (rbs + rbn) * rb_min))
    return static_cast<int>(hipErrorInvalidValue);
  // the plan depends only on the launch geometry: cached (the makespan
  // search costs milliseconds; the engine launches the same passes over and over)
  SegPlan sp;
  {
    std::vector<int64_t> key = {a.n, a.nw, a.mask, o.seg_rows, lmax, per_cu, sig_rects, rbk, rbs + rbn, rb_min, push_sides, SH};
    for (int k = 0; k < a.n; ++k) key.insert(key.end(), a.r[k], a.r[k] + 4);
    key.insert(key.end(), a.dom, a.dom + 4);
    static std::mutex mu;
    static std::map<std::vector<int64_t>, SegPlan> cache;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it == cache.end()) {
      if (cache.size() > 256) cache.clear();
      it = cache.emplace(key, plan_segments<K>(a, o.seg_rows, lmax, per_cu, sig_rects, rbk, rbs + rbn, rb_min, push_sides)).first;
    }
    sp = it->second;
  }
  a.tstart[0] = 0;
  for (int k = 0; k < a.n; ++k) {
    a.e0[k] = sp.e0[k];
    a.e1[k] = sp.e1[k];
    a.nmid[k] = sp.nmid[k];
    a.lmid[k] = sp.lmid[k];
    a.nmid_b[k] = sp.nmid_b[k];
    a.lmid_b[k] = sp.lmid_b[k];
    const int64_t groups = (a.nstrip[k] + a.nw - 1) / a.nw, nbnd = groups < 2 ? groups : 2;
    a.tstart[k + 1] = a.tstart[k] + groups * ((sp.e0[k] > 0) + (sp.e1[k] > 0)) + nbnd * sp.nmid_b[k] +
                      (groups - nbnd) * sp.nmid[k];
  }
  for (int k = a.n + 1; k <= kMaxRect; ++k) a.tstart[k] = a.tstart[a.n];
  const int64_t nb = a.tstart[a.n];
  a.sig_wgs = a.tstart[sig_rects];
  a.rb_rect = -1;
  a.cb_rect = -1;
  int64_t cb_groups = 0, cb_strips = 0;
  if (cbk >= 0) {
    // every segment of rect cbk's first / last strip group: its leading workgroups
    const int64_t groups = (a.nstrip[cbk] + a.nw - 1) / a.nw;
    a.cb_rect = cbk;
    a.cb_lo = (o.signal_cols & 1) ? 1 : 0;
    a.cb_hi = (o.signal_cols & 2) ? 1 : 0;
    cb_groups = groups == 1 ? 1 : a.cb_lo + a.cb_hi;
    if (groups == 1) cb_strips = a.nstrip[cbk];
    else cb_strips = (a.cb_lo ? std::min<int64_t>(a.nw, a.nstrip[cbk]) : 0) +
                     (a.cb_hi ? a.nstrip[cbk] - (groups - 1) * a.nw : 0);
    a.sig_wgs += cb_groups * ((sp.e0[cbk] > 0) + (sp.e1[cbk] > 0) + sp.nmid_b[cbk]);
  }
  a.sig_total = a.sig_wgs;
  a.sig_dispatch = a.sig_wgs;
  if (rbk >= 0) {
    // the band segments exist separately: halo row sides have no edge
    // segments, and the planner kept >= rbs + rbn interior segments of >= rb_min rows
    const int rb = rbs + rbn;
    // (the shortest segment: floor(mid / n) rows, tb_block's even split)
    const int64_t mid = a.r[rbk][3] - sp.e0[rbk] - sp.e1[rbk];
    if ((rbs && sp.e0[rbk] > 0) || (rbn && sp.e1[rbk] > 0) || sp.nmid[rbk] < rb || sp.nmid_b[rbk] < rb ||
        mid / sp.nmid[rbk] < o.signal_rows || mid / sp.nmid_b[rbk] < o.signal_rows)
      return static_cast<int>(hipErrorInvalidValue);
    a.rb_rect = rbk;
    a.rb_s = rbs;
    a.rb_n = rbn;
    a.sig_rows = o.signal_rows;
    const int64_t groups = (a.nstrip[rbk] + a.nw - 1) / a.nw;
    const bool cbr = rbk == cbk;         // column-band groups take no row bands
    a.sig_total += rb * (a.nstrip[rbk] - (cbr ? cb_strips : 0));  // one arrival per output wave (= strip) of every band
    a.sig_dispatch += rb * (groups - (cbr ? cb_groups : 0));      // rect rbk's band tiles follow the signalling ones
  }
  // (Dispatching the rule-path workgroups round-robin over the XCDs instead
  // of XCD-contiguous with the rest cost the Dirichlet 8192 x 16384 and
  // 16384 x 8192 passes 3-6%: profiles/r04_shares.md.)
  // A/B (GMT_TB_SPECIAL_RR=1): a one-rect pass without signals dispatches its
  // edge segments and boundary groups round-robin over the XCDs; XCD-contiguous
  // ranges put them all on XCD 0, which then finished 20-30% early on every
  // Dirichlet domain traced (profiles/r05_wg_timeline/)
  static const bool special_rr = [] {
    const char* e = std::getenv("GMT_TB_SPECIAL_RR");
    return e && std::atoi(e) > 0;
  }();
  // the planner's order: the edge segments of a one-rect pass without
  // signals last on every XCD (tail_swizzle), filling the launch's tail
  if (sp.tail && a.n == 1 && a.sig_dispatch == 0) {
    const int64_t groups = (a.nstrip[0] + a.nw - 1) / a.nw;
    const int64_t ne = groups * ((sp.e0[0] > 0) + (sp.e1[0] > 0));
    if (tail_swizzle_ok(nb, ne)) a.edges_last = ne;
  }
  if (special_rr && a.n == 1 && a.sig_dispatch == 0) {
    const int64_t groups = (a.nstrip[0] + a.nw - 1) / a.nw, nbnd = groups < 2 ? groups : 2;
    a.sig_dispatch = groups * ((sp.e0[0] > 0) + (sp.e1[0] > 0)) + nbnd * sp.nmid_b[0];
  }
  // GMT_TB_PRIO=0 / 1: never / always (A/B); default: one-round launches
  static const int prio_mode = [] {
    const char* e = std::getenv("GMT_TB_PRIO");
    return e ? std::atoi(e) : -1;
  }();
  a.prio = prio_mode >= 0 ? (prio_mode > 0 ? 1 : 0) : (nb <= per_cu ? 1 : 0);
  a.sig_count = o.signal_count;
  a.signal = o.signal;
  a.stop = PUSH ? o.stop : nullptr;
  a.clk = o.clock;
  if (info) {
    hipFuncAttributes fa{};
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&jacobi5tb_kernel<K, EXACT, EDGE, PUSH, SH>));
    const int64_t v[6] = {nb, per_cu, a.nw * G * kWave, a.lmid[0], a.nmid[0], fa.numRegs};
    for (int j = 0; j < 6; ++j) info[j] = v[j];
    return 0;
  }
#if GMT_TB_WG_TRACE
  static std::atomic<int> trace_launch{0};
  static uint64_t* trace_buf = nullptr;
  static int64_t trace_cap = 0;
  const char* trace_file = std::getenv("GMT_TB_WG_TRACE_FILE");
  const char* trace_at = std::getenv("GMT_TB_WG_TRACE_LAUNCH");
  const bool tracing = trace_file && trace_launch++ == (trace_at ? std::atoi(trace_at) : 50);
  if (tracing) {
    if (trace_cap < nb) {
      if (trace_buf) (void)hipFree(trace_buf);
      if (hipMalloc(&trace_buf, static_cast<size_t>(nb) * 32) != hipSuccess) return static_cast<int>(hipErrorOutOfMemory);
      trace_cap = nb;
    }
    (void)hipMemsetAsync(trace_buf, 0, static_cast<size_t>(nb) * 32, s);
    a.wg_trace = trace_buf;
  }
#endif
  jacobi5tb_kernel<K, EXACT, EDGE, PUSH, SH><<<grid_1d(nb), a.nw * G * kWave, smem, s>>>(a, u, un, nb);
#if GMT_TB_WG_TRACE
  if (tracing) {
    std::vector<uint64_t> h(static_cast<size_t>(nb) * 4);
    if (hipStreamSynchronize(s) == hipSuccess &&
        hipMemcpy(h.data(), trace_buf, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      const std::string path = std::string(trace_file) + (PUSH ? ".push" : "");
      if (FILE* f = std::fopen(path.c_str(), "w")) {
        std::fprintf(f, "# K %d nb %lld per_cu %lld nw %d n %d mask %d rect0 %lld %lld %lld %lld nstrip %lld "
                        "e0 %lld e1 %lld nmid %lld lmid %lld nmid_b %lld lmid_b %lld sig_dispatch %lld\n",
                     K, (long long)nb, (long long)per_cu, a.nw, a.n, a.mask, (long long)a.r[0][0], (long long)a.r[0][1],
                     (long long)a.r[0][2], (long long)a.r[0][3], (long long)a.nstrip[0], (long long)a.e0[0],
                     (long long)a.e1[0], (long long)a.nmid[0], (long long)a.lmid[0], (long long)a.nmid_b[0],
                     (long long)a.lmid_b[0], (long long)a.sig_dispatch);
        std::fprintf(f, "# block tile start end hw_id xcc_id\n");
        for (int64_t i = 0; i < nb; ++i)
          std::fprintf(f, "%lld %llu %llu %llu %llu %llu\n", (long long)i, (unsigned long long)h[4 * i],
                       (unsigned long long)h[4 * i + 1], (unsigned long long)h[4 * i + 2],
                       (unsigned long long)(h[4 * i + 3] & 0xffffffffu), (unsigned long long)(h[4 * i + 3] >> 32));
        std::fclose(f);
      }
    }
  }
#endif
  return static_cast<int>(hipGetLastError());
}

}  // namespace

namespace gmt {
namespace tb {

// An SH launch (Sh<K>: stage-1 windows over a shared hand-off row) for a
// pass of one rect at least a group wide, with no inline halo, completion
// signals or explicit workgroup shape.  gmt_tb_opts.shared: 1 on, -1 off,
// 0 the default (GMT_TB_SHARED=1 / 0 forces it on / off).
template <int K>
int sh_launch(const gmt_tb_opts& o, int n_rect, const int64_t* rects, int mask) {
  if constexpr (!Sh<K>::kOk) {
    return 0;
  } else {
    // GMT_TB_SHARED: 1 on wherever it applies (four-strip groups), 2 / 4 on
    // with groups of that many strips, 0 off; unset: the default
    static const int env = [] {
      const char* e = std::getenv("GMT_TB_SHARED");
      return e ? std::atoi(e) : -1;
    }();
    if (o.shared < 0 || (o.shared == 0 && env == 0)) return 0;
    if (o.push_w > 0 || o.wg_waves > 0 || o.signal_rects > 0 || o.signal_rows > 0 || (o.signal_cols & 3)) return 0;
    // the default (o.shared == 0, GMT_TB_SHARED unset): four-strip groups
    // for a rect whose x sides both exchange halos (+2-3% on the one-round
    // N = 8 shares, +2% at 32768^2); two-strip groups for a larger rect
    // (2^28 points or more: several rounds) with a Dirichlet x side — its
    // boundary groups couple only two strips to the rule strip's pace:
    // 32768^2 5.42-5.50M against 5.29-5.30M for two plain stage-major strips
    // and 5.22-5.25M for four-strip groups, same box; one-round Dirichlet
    // passes keep one strip per workgroup (profiles/r06_shared/ab_aa.txt).
    // From 2^28 points on: the N = 4 shares (8192 x 32768, three rounds)
    // gain 3-5% on every side pattern (ab_cc.txt)
    const bool dflt = o.shared == 0 && env < 0;
    int64_t area = 0, nonempty = 0;
    for (int k = 0; k < n_rect; ++k)
      if (rects[4 * k + 1] > 0 && rects[4 * k + 3] > 0) {
        ++nonempty;
        area = rects[4 * k + 1] * rects[4 * k + 3];
      }
    if (nonempty != 1) return 0;
    int w = (o.shared > 0 ? o.shared : env) == 2 ? 2 : 4;
    if (dflt) {
      if ((mask & 3) == 3) w = 4;
      else if (area >= (int64_t(1) << 28)) w = 2;
      else return 0;
    }
    const int64_t gout = w == 2 ? Sh<K, 2>::GOUT : Sh<K, 4>::GOUT;
    for (int k = 0; k < n_rect; ++k)
      if (rects[4 * k + 1] > 0 && rects[4 * k + 3] > 0 && rects[4 * k + 1] < gout) return 0;
    return w;
  }
}

template <int K>
int dispatch_k(const gmt_tb_opts& o, bool exact, int n_rect, const int64_t* rects, const int64_t* dom, int mask,
               const double* u, double* un, int64_t ld, int64_t nrows, hipStream_t s, int64_t* info) {
  if constexpr (Sh<K>::kOk) {
    const int w = sh_launch<K>(o, n_rect, rects, mask);
    if (w == 4)
      return exact ? launch_tb<K, true, false, false, 4>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info)
                   : launch_tb<K, false, false, false, 4>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info);
    if (w == 2)
      return exact ? launch_tb<K, true, false, false, 2>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info)
                   : launch_tb<K, false, false, false, 2>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info);
  }
  // a rect narrower than a strip whose width is odd ends inside a lane pair:
  // that lane stores column 0 or 2 alone (wider rects end on a lane
  // boundary: their last strip is shifted to end at the rect's edge)
  bool edge = false;
  for (int k = 0; k < n_rect; ++k)
    if (rects[4 * k + 1] > 0 && rects[4 * k + 3] > 0 && rects[4 * k + 1] < tb_strip_out(K) && rects[4 * k + 1] % 2 == 1)
      edge = true;
  if (o.push_w > 0) {  // inline halo exchange: no odd-edge stores (checked in launch_tb)
    if constexpr (tb_push_built(K)) {
      if (edge) return static_cast<int>(hipErrorInvalidValue);
      return exact ? launch_tb<K, true, false, true, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info)
                   : launch_tb<K, false, false, true, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info);
    } else {
      return static_cast<int>(hipErrorInvalidValue);
    }
  }
  if (edge)
    return exact ? launch_tb<K, true, true, false, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info)
                 : launch_tb<K, false, true, false, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info);
  return exact ? launch_tb<K, true, false, false, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info)
               : launch_tb<K, false, false, false, false>(o, n_rect, rects, dom, mask, u, un, ld, nrows, s, info);
}

}  // namespace tb
}  // namespace gmt
