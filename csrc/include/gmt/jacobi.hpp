// gmt/jacobi.hpp — distributed 2-D 5-point Jacobi solver (native engine).
//
// The BASELINE workload "mpi_stencil2d 32768² on 8 GPUs (2×4 decomp), halo
// exchange/interior overlap" and its single-GPU 8192² point.  The reference
// itself only times halo exchanges around a derivative stencil, serialised
// against compute (mpi_stencil2d_gt.cc:511-535); this engine is the
// MI355X-first version of that loop:
//
//   * 2-D Cartesian decomposition (py x px ranks), ghost width 1 (2 with
//     tblock), fp64;
//   * one step = halo exchange of u + one Jacobi sweep u -> un + swap;
//   * overlap: single sweeps — the interior "core" sweep runs on the compute
//     stream while the halo (fused pack kernel + RCCL/IPC/MPI transfer +
//     unpack) runs on a high-priority comm stream; the 1-2 cell boundary
//     frame is swept after the halo lands (gmt_jacobi5_rects).  Fused
//     passes run band-first: the boundary bands of the pass finish first
//     and signal, and the exchange of the pass's OUTPUT runs under the rest
//     of it (enqueue_block);
//   * graph: with a stream-ordered transport (rccl, local) both step parities
//     are captured into hipGraphs and replayed — one host call per step, so
//     small per-GPU domains (strong scaling at 8 GPUs) are not launch-bound.
//
//   * tblock: K = tsteps sweeps per kernel and per exchange (temporal
//     blocking): u(t) is read once and u(t+K) written once (gmt_jacobi5tb,
//     csrc/kernels/jacobi5tb.hip), the halo is K wide and exchanged once per pass with its
//     corners (one-phase exchange) — bitwise the same result as K single
//     sweeps.
// Storage is column-major (x contiguous) with the interior origin at x = 8
// so every interior row starts 64-B aligned and the sweep kernels take their
// 16-B vector path; the row pitch is padded to 64 doubles.
#pragma once

#include <memory>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/halo.hpp"
#include "gmt/transport.hpp"

namespace gmt {

struct JacobiConfig {
  int64_t ny_global = 8192, nx_global = 8192;  // global interior extent
  int py = 1, px = 1;                            // process grid (rank = cy*px + cx)
  bool periodic = false;                         // else Dirichlet (fixed ghost ring)
  int periodic_axes = 3;                         // with periodic: bit0 wraps x (W/E), bit1 wraps y (S/N)
  bool overlap = true;
  // overlap_auto: time a few fused passes with and without overlap at
  // construction (then restore the initial field) and keep the faster — the
  // same choice on every rank (the per-pass times are averaged over ranks).  Whether hiding the
  // exchange pays for the frame pass depends on the link (self-exchange on
  // one GPU: serial 4-8 % faster, profiles/r01_frame.md); measure it.
  bool overlap_auto = false;
  bool graph = false;
  // temporal blocking: tsteps (2-24) sweeps per memory pass (gmt_jacobi5tb;
  // odd counts above 10 round down) and per halo exchange (ghost width
  // tsteps, corners in the same
  // exchange phase) — 1/tsteps of the HBM bytes and messages per lattice
  // update.  1 = off.  tblock = true with tsteps = 0 is tsteps = 2.
  bool tblock = false;
  int tsteps = 0;
  int wg_waves = 0;                              // gmt_tb_opts.wg_waves: strips per workgroup (0 = auto)
  int seg_rows = 0;                              // gmt_tb_opts.seg_rows (0 = auto)
  // -1 / 0: power-of-two scaled levels when max|u| * 4^K stays finite (the
  // initial field bounds every later one: Jacobi averages; max|u| is
  // measured on the device at start-up), 1: always exact
  int exact = -1;
  // initial field (interior and Dirichlet ring): 0 = x^3 + y^2 on the global
  // lattice (gmt_fill_poly mode 4), 1 = uniform [0, 1) random values, a hash
  // of the global lattice point and `seed` (mode 5) — both independent of the
  // decomposition, so every process grid computes the same numbers
  int init = 0;
  uint64_t seed = 0;
  // prepare() times one pass of every fused-pass size on this rank's real
  // share (max over ranks) and plan_passes uses those costs instead of the
  // built-in table (measured on one box for one kernel revision)
  bool calibrate = false;
  // Inline halo exchange (fused passes; gmt_tb_opts.push): every pass
  // stores its output faces straight into the neighbours' ghost cells of
  // their next input (IPC mappings traded over the transport's control
  // plane; this rank's own buffers on a periodic axis), then one small
  // hand-over launch (gmt_push_sync) replaces the halo exchange.  Needs a
  // transport with a control plane (ipc) unless every neighbour is this
  // rank; off (the transport's exchange as before) when the share is too
  // small for the kernel's push rules.
  bool push = false;
};

class JacobiSolver {
 public:
  JacobiSolver(comm::Transport& t, const JacobiConfig& c);
  ~JacobiSolver();
  JacobiSolver(const JacobiSolver&) = delete;
  JacobiSolver& operator=(const JacobiSolver&) = delete;

  void step();  // one sweep, asynchronous (compute stream)
  void run(int k);  // k sweeps through the fused kernel (plan_passes) when tblock
  // cheapest sequence of fused passes (sweeps per pass <= tsteps) covering k sweeps
  std::vector<int> plan_passes(int k) const;
  void synchronize();
  // sqrt(global sum (u_{k+1} - u_k)^2) of one extra sweep (advances the solution)
  double residual();
  // one blocking halo exchange of the current field (latency measurements);
  // ordered after every pass already enqueued
  void exchange_only();
  // launch one pass of every pass type run(k) uses, then restore the initial
  // field: first-launch costs (code object, occupancy query) stay out of a
  // timed run(k)
  void prepare(int k);
  bool exact() const { return exact_; }
  // local interior, row-major [ny][nx] (host memory)
  void copy_interior(double* host) const;
  // Bitwise comparison of the current interiors of two solvers of the same
  // global problem and process grid, on the device (gmt_diff_bits):
  // out[0] = max |diff| (max over ranks), out[1] = elements whose bits differ
  // (sum over ranks).  bench.py's check of the timed run replays the timed
  // sweeps through single sweeps and compares (reference: the err_norm of the
  // timed field, mpi_stencil2d_gt.cc:541-570).  Collective.
  void compare(JacobiSolver& o, double out[2]);
  // Shader clock of the fused passes since the last clock_reset() (stream
  // ordered): one sampled wave per 256 workgroups stamps s_memtime and
  // s_memrealtime (gmt_tb_opts.clock).  out = {MHz (0 without samples or on
  // the CPU backend), samples, seconds sampled}.  GMT_CLOCK=0: no stamps.
  void clock_reset();
  void clock_read(double out[3]);
  // The launch of this rank's one-rect K-sweep pass (the serial or inline-
  // halo pass over the interior), without launching: gmt_jacobi5tb_plan's
  // {workgroups, resident workgroups, threads per workgroup, segment rows,
  // segments, VGPRs}.  Returns its error code (0: ok).
  int tb_launch_info(int K, int64_t out[6]) const;

  int64_t nx() const { return nx_; }
  int64_t ny() const { return ny_; }
  int64_t off_x() const { return ox_; }
  int64_t off_y() const { return oy_; }
  size_t bytes_per_exchange() const { return halo_[0] ? halo_[0]->bytes_sent() : 0; }
  size_t messages() const { return halo_[0] ? halo_[0]->messages() : 0; }
  bool graph_active() const { return graph_[0] != nullptr || graph2_[0] != nullptr; }
  bool tblock() const { return ks_ > 1; }
  int tsteps() const { return ks_; }
  int ghost() const { return g_; }
  bool overlap_active() const { return push_on_ || (cfg_.overlap && halo_[0] && halo_[0]->active()); }
  // the fused passes exchange their halo inline (cfg_.push took effect)
  bool push_active() const { return push_on_; }
  // the fused passes overlap band-first (enqueue_block)
  bool band_first() const { return ks_ > 1 && band_mode(ks_); }
  const Neighbors& neighbors() const { return nb_; }
  // overlap_auto: seconds per pass measured {overlap, serial} (mean over ranks), 0 if not tuned
  double tuned_overlap_s() const { return tune_s_[0]; }
  double tuned_serial_s() const { return tune_s_[1]; }
  // ms per fused pass of k sweeps: measured by prepare() with calibrate (0 if
  // not), and the built-in table's estimate for this share
  double measured_pass_ms(int k) const { return k >= 0 && k <= GMT_TB_MAX_SWEEPS ? meas_ms_[k] : 0.0; }
  double table_pass_ms(int k) const;
  double max_abs_u0() const { return umax_; }
  gmt_stream_t stream() const { return s_; }

 private:
  void enqueue_step(int parity);
  void enqueue_block(int parity, int k);  // k <= ks_ fused sweeps
  // one fused k-sweep launch on `n` output rects (gmt_jacobi5tb)
  void xk_launch(int k, int n, const int64_t* rects, int parity, int sig_rects, int sig_rows,
                 gmt_stream_t st = nullptr, int sig_cols = 0);
  // the band-first pass's rect (the interior) and its column / row bands
  bool band_rects(int k, int64_t* rects, int* sig_cols, int* sig_rows) const;
  bool band_mode(int k) const;  // the fused k-sweep pass runs band-first (overlap)
  void exchange_now(int parity);  // blocking-order halo exchange of buf_[parity] on the compute stream
  void step_block();
  void sweep_full(int parity, double* resid);
  void capture_graphs();
  void init_field();
  void autotune_overlap();
  void calibrate_costs();
  double measure_max_abs();
  int halo_mask() const;
  void split_cus();
  void setup_push();
  void maybe_corrupt(int parity);  // GMT_CORRUPT_PASS fault injection
  void push_block(int parity, int k);  // one inline-halo pass + its hand-over

  comm::Transport& t_;
  JacobiConfig cfg_;
  int64_t nx_ = 0, ny_ = 0, ox_ = 0, oy_ = 0;  // local interior + global offset
  int64_t xo_ = 8, yo_ = 1, ld_ = 0;           // interior origin (absolute), row pitch
  int g_ = 1;                                  // ghost width
  int ks_ = 1;                                 // sweeps per fused pass
  bool exact_ = false;                         // gmt_tb_opts.exact for the fused passes
  Neighbors nb_;
  Buffer<double> buf_[2];
  std::unique_ptr<Halo2D> halo_[2];
  Buffer<double> resid_ws_;
  Buffer<uint64_t> sig_;  // band-first completion signal (GMT_SPACE_FLAGS)
  bool fresh_[2] = {false, false};  // buf_[b]'s ghost ring holds the neighbours' current values
  gmt_stream_t s_ = nullptr, cs_ = nullptr;
  // band-first passes on split compute units (split_cus): the pass on sb_
  // (all but a few CUs), the exchange on cs_ (those few), so the exchange's
  // kernels start the moment the bands signal instead of waiting for the
  // pass's resident workgroups to retire
  gmt_stream_t sb_ = nullptr;
  int comm_cus_ = 0;
  // pack/unpack workgroups of the exchange a band-first pass hides
  // (Halo2D::set_pack_wgs): 0 = the full grid; GMT_PACK_WGS=N for A/B (64
  // and 128 measured no better on the N = 8 shares, profiles/r04_overlap.md)
  int beside_pack_wgs_ = 0;
  // a band-first pass was enqueued since the last synchronize(): only then
  // do the side streams and the band signal's error word need a look (a
  // D2H read and two stream syncs are ~2% of an N = 8 pass)
  bool band_ran_ = false;
  gmt_event_t ev_start_ = nullptr, ev_halo_ = nullptr, ev_band_ = nullptr;
  gmt_graph_t graph_[2] = {nullptr, nullptr};   // single sweep, per parity
  gmt_graph_t graph2_[2] = {nullptr, nullptr};  // fused ks_-sweep block, per parity
  int parity_ = 0;  // buf_[parity_] holds the current u
  int passes_ = 0;  // fused passes run() enqueued since the field was (re)initialised
  bool in_run_ = false;
  double tune_s_[2] = {0.0, 0.0};
  double meas_ms_[GMT_TB_MAX_SWEEPS + 1] = {};
  bool calibrated_ = false;
  double umax_ = 0.0;  // max |u| of the initial field over every rank
  // inline halo exchange (setup_push): per parity of the pass's INPUT, the
  // push targets (gmt_tb_opts.push) — the neighbours' other buffer with the
  // face translation folded in; the neighbours' flag slots for this rank;
  // the directions that are other ranks; the hand-over epoch
  bool push_on_ = false;
  const double* push_base_[2][8] = {};
  uint64_t* push_remote_[8] = {};
  int push_mask_ = 0;
  uint64_t push_epoch_ = 0;
  Buffer<uint64_t> push_flags_;  // [d]: written by the neighbour in direction d
  Buffer<unsigned> push_err_;    // host-visible: bit d = the wait for direction d expired
  Buffer<unsigned> push_stop_;   // device word: a wait expired, later passes return at once
  Buffer<uint64_t> clk_;         // gmt_tb_opts.clock: cycles, 100 MHz ticks, samples
  std::vector<void*> push_opened_;
};

// Balanced block split of n over p parts: offset and length of part i.
inline void block_split(int64_t n, int p, int i, int64_t* off, int64_t* len) {
  const int64_t base = n / p, rem = n % p;
  *off = i * base + (i < rem ? i : rem);
  *len = base + (i < rem ? 1 : 0);
}

// The cheapest sequence of fused passes covering k sweeps, passes of at most
// ks sweeps, cost[K] = ms of a K-sweep pass (0: no such pass; K = 1 a single
// sweep); measured costs get a 2% handicap on passes shorter than ks (clock
// noise must not displace full passes).  Full passes first, then the rest,
// largest first.  JacobiSolver::plan_passes with this rank's costs.
std::vector<int> plan_pass_sequence(int k, int ks, std::vector<double> cost, bool measured);

// Process grid minimising the halo bytes per rank; strided x faces (which
// need a pack kernel) are weighted 1.5x a contiguous y face.
void choose_dims(int world, int64_t ny, int64_t nx, int* py, int* px);

}  // namespace gmt
