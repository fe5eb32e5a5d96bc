/*
 * gmt/kernels.h — C ABI of the hand-written gfx950 kernels in libgmt.so.
 *
 * Every entry point is asynchronous on the given HIP stream (pass the raw
 * hipStream_t as `void*`; NULL = the legacy default stream) and returns a
 * hipError_t as int (0 = success). The same ABI is used by the native MPI
 * apps (csrc/apps) and by the Python package through ctypes
 * (gpu_mpi_tests_amd/_native.py), so there is exactly one kernel code path.
 *
 * Layout convention (matches the reference's column-major arrays, e.g.
 * /root/reference/mpi_stencil2d_sycl.cc:40-43 `idx2`): a 2-D field is stored
 * as `ny` rows of `ld` elements; x (the reference's "dim 0") is the contiguous
 * axis, y ("dim 1") is the strided axis. In torch terms that is a row-major
 * tensor of shape [ny, ld].
 */
#ifndef GMT_KERNELS_H
#define GMT_KERNELS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- K1/K2: y <- a*x + y (fp64).  reference: daxpy.cu:73, mpi_daxpy_gt.cc:81 */
int gmt_daxpy(int64_t n, double a, const double* x, double* y, void* stream);

/* ---- K3: 1-D 5-tap stencil, out[i] = scale * sum_k c[k]*in[i+k], k=0..4.
 *      `in` has n_out+4 elements.  reference: mpi_stencil_gt.cc:54-59 */
int gmt_stencil5_1d(int64_t n_out, const double* coef5, double scale,
                    const double* in, double* out, void* stream);

/* ---- K4/K5/K11: 2-D field, 5-tap stencil along `dim` (0 = contiguous x,
 *      1 = strided y).  `in` is (ny_out [+4 if dim==1]) rows of ld_in,
 *      holding nx_out [+4 if dim==0] valid columns.
 *      reference: mpi_stencil2d_gt.cc:84-110, mpi_stencil2d_sycl.cc:53-75 */
int gmt_stencil5_2d(int dim, int64_t nx_out, int64_t ny_out, const double* coef5,
                    double scale, const double* in, int64_t ld_in, double* out,
                    int64_t ld_out, void* stream);

/* ---- K6/K7/K8: batched strided 2-D copy (halo pack / unpack, fused L+R).
 *      Each descriptor copies `height` rows of `width` elements of
 *      `elem_bytes` (4 or 8) from src (row pitch src_ld elements) to dst
 *      (row pitch dst_ld elements).  Up to GMT_MAX_COPY2D descriptors are
 *      fused into one launch.  reference: mpi_stencil2d_gt.cc:166-174,239,251 */
#define GMT_MAX_COPY2D 8
typedef struct gmt_copy2d_desc {
  const void* src;
  void* dst;
  int64_t src_ld;
  int64_t dst_ld;
  int64_t width;
  int64_t height;
} gmt_copy2d_desc;
int gmt_copy2d_batched(int n_desc, const gmt_copy2d_desc* descs, int elem_bytes,
                       void* stream);
// The same copy by at most max_wgs workgroups in a grid-stride loop (0: one
// element per thread, the full grid) — for exchanges that run beside a pass
// holding nearly every CU slot (profiles/r04_overlap.md).
int gmt_copy2d_batched_wgs(int n_desc, const gmt_copy2d_desc* descs, int elem_bytes, int max_wgs,
                           void* stream);

/* ---- K9: axis sums of a 2-D field of nx x ny (row pitch ld).
 *      keep_dim == 0: out[x] = sum_y z[y][x]   (length nx)
 *      keep_dim == 1: out[y] = sum_x z[y][x]   (length ny)
 *      `workspace` must hold gmt_sum_axis_workspace(...) doubles.
 *      reference: mpi_stencil2d_gt.cc:611,620 (gt::sum_axis_to) */
int64_t gmt_sum_axis_workspace(int keep_dim, int64_t nx, int64_t ny);
int gmt_sum_axis(int keep_dim, int64_t nx, int64_t ny, const double* z, int64_t ld,
                 double* out, double* workspace, void* stream);

/* ---- K10/K12: out[0] = sum over the nx x ny region of (a - b)^2
 *      (NOT square-rooted, so partial results can be all-reduced).
 *      `workspace` must hold gmt_diff_sq_workspace(...) doubles.
 *      reference: mpi_stencil2d_gt.cc:555, mpi_stencil2d_sycl.cc:165-181 */
int64_t gmt_diff_sq_workspace(int64_t nx, int64_t ny);
int gmt_diff_sq(int64_t nx, int64_t ny, const double* a, int64_t lda, const double* b,
                int64_t ldb, double* out, double* workspace, void* stream);

/* ---- out[0] = sum of x[0..n) (one HBM pass, deterministic order);
 *      workspace of gmt_sum_workspace(n) doubles.  The DAXPY partial sums
 *      (reference: host loops, mpi_daxpy_nvtx.cc:251-268) */
int64_t gmt_sum_workspace(int64_t n);
int gmt_sum(int64_t n, const double* x, double* out, double* workspace, void* stream);

/* ---- out[i] = sum (op 0) or max (op 1) over r = 0..nslices-1 of
 *      in[r*n + i], in rank order (an all-gather + this = a deterministic
 *      all-reduce; out may alias slice 0 of in only if it is in[0..n)) */
int gmt_slices_reduce(int op, int64_t n, int nslices, const double* in, double* out, void* stream);

/* ---- max over the nx x ny region of |z| -> out[0]; workspace of
 *      gmt_diff_sq_workspace(nx, ny) doubles */
int gmt_abs_max(int64_t nx, int64_t ny, const double* z, int64_t ld, double* out, double* workspace,
                void* stream);

/* ---- bitwise comparison of two nx x ny regions: out[0] = max |a - b|
 *      (NaN -> +inf), out[1] = number of elements whose 64 bits differ (as a
 *      double: exact to 2^53).  Deterministic two-pass; workspace of
 *      2 * gmt_diff_sq_workspace(nx, ny) doubles.  bench.py's check of the
 *      timed run (reference: the err_norm of the timed field,
 *      mpi_stencil2d_gt.cc:541-570) */
int gmt_diff_bits(int64_t nx, int64_t ny, const double* a, int64_t lda, const double* b, int64_t ldb,
                  double* out, double* workspace, void* stream);

/* ---- analytic fill z[y][x] = (x0+i*dx)^3 + (y0+j*dy)^2 over nx x ny (device
 *      side replacement of the reference's host init loops,
 *      mpi_stencil2d_gt.cc:439-497).  mode 0: x^3+y^2 (z), 1: 3x^2 (dz/dx),
 *      2: 2y (dz/dy), 3: x (linear ramp; DAXPY inputs), 4: x^3+y^2 on the
 *      integer lattice x = (x0 + i)*dx, y = (y0 + j)*dy with x0, y0 integer
 *      indices, no fma contraction (bitwise reproducible on the host),
 *      5: uniform [0, 1) random field, a counter-based hash (splitmix64) of
 *      the integer lattice point (x0 + i, y0 + j) with seed (uint64) dx —
 *      decomposition-independent random init. */
int gmt_fill_poly(int mode, int64_t nx, int64_t ny, double x0, double dx, double y0,
                  double dy, double* z, int64_t ld, void* stream);
/* Per-exchange halo check (the apps' --check): counts the cells of the
 * nx x ny block z (pitch ld) that differ from x^3 + y^2 + offset at
 * x = x0 + i*dx, y = y0 + j*dy by more than rtol * (1 + |expected|), adding
 * the count to *bad (a device counter) — one small launch after each
 * exchange over the ghost rows it filled.  gmt_add_scalar adds v to every
 * cell of a block (the per-iteration offset that makes a stale ghost row
 * visible). */
int gmt_poly_check(int64_t nx, int64_t ny, double x0, double dx, double y0, double dy, double offset,
                   double rtol, const double* z, int64_t ld, unsigned* bad, void* stream);
int gmt_add_scalar(int64_t nx, int64_t ny, double v, double* z, int64_t ld, void* stream);

/* ---- 2-D 5-point Jacobi sweep (the BASELINE "5-pt Jacobi" extension):
 *      for y in [y0, y0+ny), x in [x0, x0+nx) (absolute array coordinates):
 *        un[y][x] = c0*(u[y][x-1]+u[y][x+1]+u[y-1][x]+u[y+1][x]) + c1*f[y][x]
 *      f may be NULL (Laplace).  If resid_partial != NULL, the kernel also
 *      accumulates sum (un-u)^2 and leaves the total in resid_partial[0]
 *      (resid_partial must hold gmt_jacobi_resid_workspace(...) doubles). */
int64_t gmt_jacobi_resid_workspace(int64_t nx, int64_t ny);
int gmt_jacobi5(int64_t x0, int64_t nx, int64_t y0, int64_t ny, const double* u,
                double* un, int64_t ld, const double* f, int64_t ldf, double c0,
                double c1, double* resid_partial, void* stream);
/* Same sweep for a list of rectangles in one launch (the boundary "frame" of
 * an overlapped step: up to 4 strips).  rect = {x0, nx, y0, ny}. */
int gmt_jacobi5_rects(int n_rect, const int64_t* rects, const double* u, double* un,
                      int64_t ld, const double* f, int64_t ldf, double c0, double c1,
                      void* stream);
/* ---- Temporal-blocking Jacobi (csrc/kernels/jacobi5tb.hip): `sweeps` fused
 *      Laplace sweeps per memory pass, un = J^sweeps(u), on up to 8 output
 *      rects {x0, nx, y0, ny} (absolute array coordinates, x0 >= sweeps,
 *      y0 >= sweeps, x0+nx+sweeps <= ld, y0+ny+sweeps <= nrows; u must hold
 *      each rect plus its sweeps-wide ring).  `dom` = the rank's interior
 *      {x0, nx, y0, ny}.  halo_mask bit0/1/2/3 = west/east/south/north ghost
 *      cells belong to a neighbour (they get the intermediate updates); a
 *      clear bit means a fixed Dirichlet ghost.  Cells of `un` outside the
 *      rects are never written.  Sweep counts: 1..10 (one wave per strip)
 *      and even 12..GMT_TB_MAX_SWEEPS (two waves per strip, levels split; K = 22
 *      and 24 exceed the register file at 2 waves per SIMD and are not built);
 *      gmt_jacobi5tb_supported() says which. */
#define GMT_TB_MAX_SWEEPS 20
typedef struct gmt_tb_opts {
  int sweeps;   /* K, see gmt_jacobi5tb_supported */
  int wg_waves; /* 256-column strips per workgroup, 1..8 (0 = default: four
                   one-stage strips for K <= 10; for K > 10 one two-stage
                   strip, two (stage-major waves) for a one-rect pass
                   larger than 2^28 points; at most 4 when K > 10) */
  int seg_rows; /* output rows per strip segment (0 = default: short edge
                   segments where a rect touches a Dirichlet row, interior
                   segments sized to fill the device's resident workgroups) */
  int exact;    /* 1: multiply by 1/4 per level (bitwise for any magnitude);
                   0: power-of-two scaled levels (bitwise unless a value is
                   subnormal or |u| * 4^K overflows) */
  /* Completion signal (0 = none): the workgroups of rects[0 .. signal_rects)
     — non-empty rects, given short segments — are dispatched first, and the
     last of them to finish adds 1 to *signal once their output is visible
     device-wide, while the rest of the launch still runs.  A stream can wait
     for it with gmt_signal_wait.  signal_count: a zeroed arrival counter
     (reset by the last arrival); both in GMT_SPACE_FLAGS memory. */
  int signal_rects;
  unsigned* signal_count;
  uint64_t* signal;
  /* Row bands (0 = none): rect signal_rects (the first rect after the
     signalling ones) keeps its S / N halo sides' segments separate, walks
     the N ones bottom-up, and dispatches all of them first; each of their
     output waves counts once toward the same signal after storing its
     first signal_rows output rows — the rect's signal_rows-deep row bands
     are ready long before the rect is.  No extra workgroups (the band
     rects of signal_rects each cost a pipeline warm-up and launch slots). */
  int signal_rows;
  /* Compute units the launch's stream may not use (a CU-masked stream, see
     gmt_rt_stream_create_cumask): the segment planner sizes the launch for
     the resident workgroups of the remaining ones (0 = every CU). */
  int reserved_cus;
  /* Column bands (0 = none; bit 0 W, bit 1 E): the first / last strip
     group of rect signal_rects — every one of its segments, full length —
     is dispatched before the rest of the launch and each of its workgroups
     counts toward the same signal when done: the rect's W / E halo columns
     are ready after the first round of workgroups, with no band rects of
     their own (no extra strips, segments or pipeline warm-ups). */
  int signal_cols;
  /* Inline halo exchange ("push", 0 = off): the pass stores its output's
     face cells a second time, straight into the ghost cells of the
     neighbours' NEXT input field — no pack, copy or exchange kernel.  For
     direction d (GMT_PUSH_S .. GMT_PUSH_NE), output cell (x, y) of a face
     goes to push[d] + (y * ld + x) doubles (the engine folds the
     neighbour's buffer and the translation into push[d]; IPC-mapped memory
     of another process or device, or this rank's own other buffer on a
     periodic axis); NULL = no neighbour that way.  Faces: rows [y0, y0 +
     push_w) to S, [y1 - push_w, y1) to N, columns [x0, x0 + push_w) to W,
     [x1 - push_w, x1) to E, their w x w intersections to the diagonals, of
     the one rect (which must be `dom`).  Needs: push_w even and <= 64;
     two strips or more when both W and E are pushed (a strip pushes one
     x face); the segment planner keeps every segment clear of one of the
     S / N faces; no completion signal options; rects of even width or
     wider than a strip (no odd-edge stores). */
  const double* push[8];
  int push_w;
  /* Inline-halo passes only (push_w > 0): a device word (NULL = none) that a
     timed-out hand-over sets (gmt_push_sync `stop`); while it is non-zero
     every workgroup of the pass returns at entry — its ghost cells are
     stale and a late neighbour may still be writing them — and the job
     fails at its next synchronisation. */
  const unsigned* stop;
  /* Shader-clock record (NULL = none): one sampled wave per 256 workgroups
     adds its s_memtime delta (shader cycles) to clock[0], its
     s_memrealtime delta (the 100 MHz constant clock) to clock[1] and 1 to
     clock[2] (device memory, zeroed by the caller): the clock the pass ran
     at is clock[0] / clock[1] x 100 MHz. */
  uint64_t* clock;
  /* Shared hand-off groups (csrc/kernels/jacobi5tb.hpp Sh<K>): K = 12, 16,
     20 passes of one rect at least a group wide (920 columns at K = 20),
     with no push, signals or wg_waves, run as workgroups of four strips
     whose stage-1 waves read windows of one shared hand-off row — 6% fewer
     level updates per output at K = 20.  Bitwise the same field.
     -1 = off, 1 = on (four-strip groups), 2 / 4 = on with groups of that
     many strips (448 / 920 output columns at K = 20), 0 = default: four-
     strip groups where both x sides exchange halos, two-strip groups for
     other rects of 2^28 points or more (GMT_TB_SHARED=0 / 1 / 2 / 4 forces it). */
  int shared;
} gmt_tb_opts;
enum { GMT_PUSH_S = 0, GMT_PUSH_N = 1, GMT_PUSH_W = 2, GMT_PUSH_E = 3,
       GMT_PUSH_SW = 4, GMT_PUSH_SE = 5, GMT_PUSH_NW = 6, GMT_PUSH_NE = 7 };
int gmt_jacobi5tb_supported(int sweeps);
/* gmt_jacobi5tb_supported and an inline-halo (gmt_tb_opts.push) kernel is built */
int gmt_jacobi5tb_push_supported(int sweeps);
/* Largest sweep count whose kernel runs without scratch: GMT_TB_MAX_SWEEPS
 * for the scaled form, 18 with exact = 1 (planners stay at or below it). */
int gmt_jacobi5tb_max_sweeps(int exact);
int gmt_jacobi5tb(const gmt_tb_opts* opts, int n_rect, const int64_t* rects, const int64_t* dom,
                  int halo_mask, const double* u, double* un, int64_t ld, int64_t nrows, void* stream);
/* The launch gmt_jacobi5tb would make, without launching: info = {workgroups,
 * resident workgroups on the device, threads per workgroup, rows per interior
 * segment and interior segments of rects[0], VGPRs per lane}. */
/* Output columns one workgroup of the fused kernel covers (strips per
 * workgroup x output columns per strip) for `sweeps` and wg_waves (0 = default). */
int64_t gmt_jacobi5tb_group_cols(int sweeps, int wg_waves);
int gmt_jacobi5tb_plan(const gmt_tb_opts* opts, int n_rect, const int64_t* rects, const int64_t* dom,
                       int halo_mask, int64_t ld, int64_t nrows, int64_t info[6]);

/* One-workgroup kernel on `stream`: waits until *signal > *seen (a
 * gmt_tb_opts completion signal), then advances *seen by one — a stream
 * ordered wait that replays correctly in a hipGraph.  Gives up after
 * GMT_WAIT_TIMEOUT_MS of device wall clock (default 10 s) and sets bit 2 of
 * *err.  All three in GMT_SPACE_FLAGS memory. */
int gmt_signal_wait(const uint64_t* signal, uint64_t* seen, unsigned* err, void* stream);

/* Hand-over between two inline-halo passes (gmt_tb_opts.push), one launch
 * on `stream` after the pushing pass: for every direction d set in `mask`,
 * stores `epoch` into *remote[d] (this rank's flag slot in the neighbour's
 * memory, IPC-mapped; system-scope release), then waits until local[d] >=
 * epoch (the neighbour's faces are in this rank's ghost cells) and acquires
 * on every XCD.  Each wait is bounded by GMT_WAIT_TIMEOUT_MS of device wall
 * clock (default 10 s); an expired one ORs 1 << d into *err (host-visible)
 * and into *stop (device memory, may be NULL: the gmt_tb_opts.stop word of
 * the following passes, which then return at once) and gives up.  While
 * *stop is non-zero the hand-over neither signals nor waits, so a stalled
 * neighbour stops the whole job within one wait instead of one per pass.
 * local / remote: GMT_SPACE_FLAGS memory. */
int gmt_push_sync(const uint64_t* local, uint64_t* const remote[8], int mask, uint64_t epoch, unsigned* err,
                  unsigned* stop, void* stream);

/* Test hook: the XCD (XCC_ID) each of n one-wave workgroups of a single
 * launch ran on, out[i] for workgroup i (device memory).  gmt_push_sync's
 * per-XCD acquire relies on workgroups i < 8 landing on 8 distinct XCDs. */
int gmt_xcd_of_workgroups(int n, unsigned* out, void* stream);

/* ---- Stream-ordered IPC exchange (csrc/kernels/ipc.hip), one launch per
 *      exchange of a persistent plan: e = *epoch + 1.  Send channel: wait
 *      until *wait >= e - 2 (receiver done with the slot), copy src -> dst +
 *      (e & 1) * dst_stride.  Receive channel: wait until *wait >= e
 *      (sender's slot ready), copy src + (e & 1) * src_stride -> dst.  When
 *      all send (receive) channels are copied, e is stored into each of their
 *      non-NULL *signal flags (system-scope release); when everything is
 *      done, *epoch = e.  Flags: GMT_SPACE_FLAGS memory; wait flags local,
 *      signal flags may be IPC-mapped memory of another process or device.
 *      Each wait is bounded by GMT_WAIT_TIMEOUT_MS of device wall clock
 *      (default 10 s); one that expires stores 1 + its channel index (sends
 *      first, then receives) into *err and gives up — the host must read
 *      *err after synchronising and treat non-zero as a failed exchange. */
typedef struct gmt_ipc_chan {
  const void* src;
  void* dst;
  int64_t bytes;
  int64_t src_stride; /* parity offsets (bytes): slot e & 1 */
  int64_t dst_stride;
  const uint64_t* wait;
  uint64_t* signal;
  /* strided side (a halo face moved in place, Transport::takes_blocks): the
     message is runs of src_run / dst_run bytes, src_ld / dst_ld bytes apart;
     run 0 = contiguous.  The staging slot side is always contiguous. */
  int64_t src_run, src_ld, dst_run, dst_ld;
} gmt_ipc_chan;
typedef struct gmt_ipc_plan {
  void* table;         /* device memory of gmt_ipc_table_bytes(n_send + n_recv) bytes */
  uint64_t* epoch;     /* device word, zero before the first exchange */
  unsigned* counters;  /* 3 device words, zero before the first exchange */
  unsigned* err;       /* host-visible (pinned) word, zero = no timeout */
  int n_send, n_recv;          /* filled by gmt_ipc_plan_init */
  int64_t send_chunks, recv_chunks;
} gmt_ipc_plan;
int64_t gmt_ipc_table_bytes(int n_chan);
/* Writes the channel table (synchronous copy) and the chunk counts; any
 * number of channels.  table/epoch/counters/err must be set by the caller. */
int gmt_ipc_plan_init(gmt_ipc_plan* plan, int n_send, const gmt_ipc_chan* sends, int n_recv,
                      const gmt_ipc_chan* recvs);
int gmt_ipc_exchange(const gmt_ipc_plan* plan, void* stream);

/* ---- Kernel-driven host staging (csrc/kernels/stage.hip): one launch copies
 *      every chunk src -> dst (device memory -> page-locked host memory the
 *      GPU maps; or the reverse): gmt_stage_copy's `wgs` workgroups each take
 *      their slice of chunk 0, then of chunk 1, ... (chunks complete in
 *      order); gmt_stage_scatter runs wgs_per_chunk per chunk.  Once chunk k is
 *      complete and visible system-wide, `value` is stored into flags[k]
 *      (GMT_SPACE_PINNED_COHERENT memory) so the host can hand chunk k to MPI
 *      while later chunks are still being copied.  The chunk table and the
 *      per-chunk arrival counters (zero between launches) are device memory.
 *      A chunk with rows > 0 is strided on its field side: it is the packed
 *      doubles [first, first + bytes/8) of a column-major block of `rows`
 *      doubles per column at pitch `ld` doubles starting at `block` (a halo
 *      face read straight out of the field: no separate pack launch, no
 *      device send buffer).  gmt_stage_copy gathers such a chunk from
 *      `block` into dst; gmt_stage_scatter writes src into `block` (a
 *      received chunk from page-locked memory straight into the ghost rows;
 *      rows == 0: a plain copy src -> dst). */
typedef struct gmt_stage_chunk {
  const void* src;
  void* dst;
  int64_t bytes;
  int64_t rows, ld, first; /* strided field side (rows == 0: contiguous) */
  double* block;
} gmt_stage_chunk;
int gmt_stage_copy(int n_chunks, const gmt_stage_chunk* chunks, unsigned* counters, uint64_t* flags,
                   uint64_t value, int wgs, void* stream);
int gmt_stage_scatter(int n_chunks, const gmt_stage_chunk* chunks, int wgs_per_chunk, void* stream);

/* One kernel per entry point: the variants the defaults were chosen against
 * are measured by csrc/bench/variant_bench.hip, not shipped in this ABI. */

/* ---- misc */
const char* gmt_error_string(int err);
int gmt_device_synchronize(void);
const char* gmt_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* GMT_KERNELS_H */
