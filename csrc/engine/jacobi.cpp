// Native distributed Jacobi engine (gmt/jacobi.hpp).
#include "gmt/jacobi.hpp"
#include "gmt/control.hpp"
#include "gmt/kernels.h"
#include "gmt/util.hpp"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace gmt {

namespace {
constexpr double kC0 = 0.25;  // un = 1/4 (W + E + S + N): Laplace, no source term

int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
}  // namespace

void choose_dims(int world, int64_t ny, int64_t nx, int* py, int* px) {
  double best = -1.0;
  for (int x = 1; x <= world; ++x) {
    if (world % x) continue;
    const int y = world / x;
    const double ly = static_cast<double>(ny) / y, lx = static_cast<double>(nx) / x;
    const double cost = (y > 1 ? 2 * lx : 0.0) + (x > 1 ? 1.5 * 2 * ly : 0.0);
    if (best < 0 || cost < best - 1e-9 || (std::fabs(cost - best) <= 1e-9 && y > *py)) {
      best = cost;
      *py = y;
      *px = x;
    }
  }
}

JacobiSolver::JacobiSolver(comm::Transport& t, const JacobiConfig& c) : t_(t), cfg_(c) {
  const int rank = t.rank(), world = t.size();
  watchdog_kick("jacobi: setup");
  if (c.py * c.px != world) {
    std::printf("JacobiSolver: process grid %dx%d != world size %d\n", c.py, c.px, world);
    abort_job(EXIT_FAILURE);
  }
  const int cy = rank / c.px, cx = rank % c.px;
  block_split(c.ny_global, c.py, cy, &oy_, &ny_);
  block_split(c.nx_global, c.px, cx, &ox_, &nx_);
  if (nx_ < 1 || ny_ < 1) {
    std::printf("JacobiSolver: empty local domain (%lldx%lld over %dx%d)\n",
                static_cast<long long>(c.ny_global), static_cast<long long>(c.nx_global), c.py, c.px);
    abort_job(EXIT_FAILURE);
  }
  auto at = [&](int y, int x) { return y * c.px + x; };
  const bool wx = c.periodic && (c.periodic_axes & 1), wy = c.periodic && (c.periodic_axes & 2);
  nb_.west = cx > 0 ? at(cy, cx - 1) : (wx ? at(cy, c.px - 1) : -1);
  nb_.east = cx < c.px - 1 ? at(cy, cx + 1) : (wx ? at(cy, 0) : -1);
  nb_.south = cy > 0 ? at(cy - 1, cx) : (wy ? at(c.py - 1, cx) : -1);
  nb_.north = cy < c.py - 1 ? at(cy + 1, cx) : (wy ? at(0, cx) : -1);
  // diagonal neighbours: the K-wide corner ghosts travel in the same single
  // exchange phase as the faces (gmt/halo.hpp one-phase corner mode);
  // GMT_HALO_TWO_PHASE=1 restores the two-phase exchange (A/B)
  auto wrap = [&](int v, int n, bool periodic, bool& ok) {
    if (v >= 0 && v < n) return v;
    if (!periodic) ok = false;
    return (v + n) % n;
  };
  auto diag = [&](int dy, int dx) {
    bool ok = true;
    const int y = wrap(cy + dy, c.py, wy, ok), x = wrap(cx + dx, c.px, wx, ok);
    return ok ? at(y, x) : -1;
  };
  const char* tp = std::getenv("GMT_HALO_TWO_PHASE");
  if (!(tp && tp[0] == '1')) {
    nb_.sw = diag(-1, -1);
    nb_.se = diag(-1, 1);
    nb_.nw = diag(1, -1);
    nb_.ne = diag(1, 1);
  }

  ks_ = c.tsteps > 1 ? c.tsteps : (c.tblock ? 2 : 1);
  if (ks_ > GMT_TB_MAX_SWEEPS) ks_ = GMT_TB_MAX_SWEEPS;
  while (ks_ > 1 && !gmt_jacobi5tb_supported(ks_)) --ks_;  // odd counts above 10: the next even one
  if (c.init != 0 && c.init != 1) {
    std::printf("JacobiSolver: init must be 0 (analytic) or 1 (random), got %d\n", c.init);
    abort_job(EXIT_FAILURE);
  }
  g_ = ks_;
  yo_ = g_;
  xo_ = round_up(g_, 8);  // ghost columns fit left of the interior; 64-B aligned interior
  // one row pitch on every rank (the largest share's): the inline halo
  // exchange addresses a neighbour's cells with this rank's pitch
  const int64_t nx_max = (c.nx_global + c.px - 1) / c.px;
  ld_ = round_up(xo_ + nx_max + g_, 64);
  const size_t elems = static_cast<size_t>(ld_) * (ny_ + 2 * g_);
  GMT_CHECK("stream", gmt_rt_stream_create(&s_, 0));
  // exchange stream priority: high by default; GMT_COMM_PRIORITY=0 for A/B
  const char* cp = std::getenv("GMT_COMM_PRIORITY");
  GMT_CHECK("comm stream", gmt_rt_stream_create(&cs_, cp && cp[0] == '0' ? 0 : 1));
  GMT_CHECK("event", gmt_rt_event_create(&ev_start_, 0));
  GMT_CHECK("event", gmt_rt_event_create(&ev_halo_, 0));

  // deterministic, decomposition-independent initial field and Dirichlet
  // ring: u(x, y) = x^3 + y^2 at global ghost-inclusive coordinates * h
  for (int b = 0; b < 2; ++b) buf_[b] = Buffer<double>(elems, GMT_SPACE_DEVICE);
  init_field();
  // Scaled levels (4^p u_p) are bitwise equal to the exact form while
  // max|u| * 4^K stays finite (and no level value is subnormal).  Every
  // Jacobi sweep averages, so the initial field's max|u| — measured here on
  // the device, max over ranks — bounds every later field.
  watchdog_kick("jacobi: max|u| all-reduce");
  umax_ = measure_max_abs();
  exact_ = c.exact == 1 || !(umax_ * std::ldexp(1.0, 2 * ks_) < 1e300);
  // exact passes stop at the largest K whose kernel fits the register file
  // (the ghost ring keeps its width: wider than a pass needs is harmless)
  if (ks_ > 1 && exact_)
    while (ks_ > gmt_jacobi5tb_max_sweeps(1) || !gmt_jacobi5tb_supported(ks_)) --ks_;
  resid_ws_ = Buffer<double>(gmt_jacobi_resid_workspace(nx_, ny_) + 1, GMT_SPACE_DEVICE);
  {
    const char* ce = std::getenv("GMT_CLOCK");
    if (!(ce && ce[0] == '0')) {
      clk_ = Buffer<uint64_t>(3, GMT_SPACE_DEVICE);
      clock_reset();
    }
  }
  // band-first passes: arrival counter, signal, waiter's count, error word
  sig_ = Buffer<uint64_t>(4, GMT_SPACE_FLAGS);
  for (int b = 0; b < 2; ++b) {
    Span2D<double> f(buf_[b].data() + (xo_ - g_), nx_ + 2 * g_, ny_ + 2 * g_, ld_);
    halo_[b] = std::make_unique<Halo2D>(t_, f, g_, g_, nb_, false, GMT_SPACE_DEVICE, ks_ > 1);
  }
  if (const char* e = std::getenv("GMT_PACK_WGS")) beside_pack_wgs_ = std::max(0, std::atoi(e));
  if (c.push && ks_ > 1 && halo_[0]->active()) setup_push();
  if (!push_on_ && ks_ > 1 && halo_[0]->active() && (c.overlap || c.overlap_auto)) split_cus();
  watchdog_kick("jacobi: halo plans ready");
  if (c.overlap_auto && !push_on_) autotune_overlap();
  if (c.graph) capture_graphs();
  watchdog_kick("jacobi: ready");
}

// Band-first passes run the pass and the exchange on disjoint compute units.
// A fused pass keeps every CU's wave slots full (2 waves per SIMD, one round
// of resident workgroups on the shares), so exchange kernels on a stream of
// their own — pack, RCCL or staging copies, unpack, 256-thread workgroups —
// could only start as whole CUs drained, i.e. at the end of the pass
// (profiles/r03_shares.md).  GMT_COMM_CUS = 8, 16 or 24 CUs (the same
// number from every XCD) are reserved for the exchange while band-first
// passes run; serial passes keep every CU.  Off by default: measured slower
// on one GPU (profiles/r03_shares.md, "reserved CUs").
void JacobiSolver::split_cus() {
  int cus = 0;
  if (gmt_rt_device_cu_count(&cus) != 0 || cus < 16) return;
  const char* e = std::getenv("GMT_COMM_CUS");
  const int n = e ? std::atoi(e) : 0;
  if (n <= 0 || n > 24 || n % 8 || cus != 256) return;  // MI355X: 8 XCDs x 32 CUs
  const int words = (cus + 31) / 32;
  std::vector<uint32_t> comm(words, 0u), comp(words, 0u);
  // the same number of CUs from every XCD (8 of them, 32 CUs each), whether
  // the runtime numbers CUs XCD by XCD or round-robin over the XCDs: CU
  // 33 x + 8 y is on XCD x either way (x < 8, 8 y + 7 < 32)
  for (int i = 0; i < n; ++i) {
    const int cu = ((i % 8) * 33 + (i / 8) * 8) % cus;
    comm[cu / 32] |= 1u << (cu % 32);
  }
  for (int cu = 0; cu < cus; ++cu)
    if (!(comm[cu / 32] >> (cu % 32) & 1u)) comp[cu / 32] |= 1u << (cu % 32);
  gmt_stream_t cs = nullptr, sb = nullptr;
  if (gmt_rt_stream_create_cumask(&cs, words, comm.data()) != 0) return;
  if (gmt_rt_stream_create_cumask(&sb, words, comp.data()) != 0) {
    gmt_rt_stream_destroy(cs);
    return;
  }
  GMT_CHECK("sync", gmt_rt_stream_synchronize(cs_));
  gmt_rt_stream_destroy(cs_);
  cs_ = cs;
  sb_ = sb;
  comm_cus_ = n;
  GMT_CHECK("event", gmt_rt_event_create(&ev_band_, 0));
}

void JacobiSolver::init_field() {
  const JacobiConfig& c = cfg_;
  const double h = 1.0 / (static_cast<double>(c.ny_global > c.nx_global ? c.ny_global : c.nx_global) + 1);
  for (int b = 0; b < 2; ++b) {
    GMT_CHECK("memset", gmt_rt_memset_async(buf_[b].data(), 0, buf_[b].bytes(), s_));
    // global lattice index of the first ghost column / row: ox_ - g_, oy_ - g_
    if (c.init == 1)
      GMT_CHECK("fill", gmt_fill_poly(5, nx_ + 2 * g_, ny_ + 2 * g_, static_cast<double>(ox_ - g_),
                                      static_cast<double>(c.seed), static_cast<double>(oy_ - g_), 0.0,
                                      buf_[b].data() + (xo_ - g_), ld_, s_));
    else
      GMT_CHECK("fill", gmt_fill_poly(4, nx_ + 2 * g_, ny_ + 2 * g_, static_cast<double>(ox_ - g_), h,
                                      static_cast<double>(oy_ - g_), h, buf_[b].data() + (xo_ - g_), ld_, s_));
  }
  GMT_CHECK("init sync", gmt_rt_stream_synchronize(s_));
  parity_ = 0;
  passes_ = 0;
  fresh_[0] = fresh_[1] = false;  // periodic / neighbour ghosts come from an exchange
}

double JacobiSolver::measure_max_abs() {
  const int64_t w = nx_ + 2 * g_, hgt = ny_ + 2 * g_;
  Buffer<double> ws(static_cast<size_t>(gmt_diff_sq_workspace(w, hgt)) + 1, GMT_SPACE_DEVICE);
  GMT_CHECK("abs max", gmt_abs_max(w, hgt, buf_[parity_].data() + (xo_ - g_), ld_, ws.data(), ws.data() + 1, s_));
  t_.allreduce_max(ws.data(), 1, s_);
  double m = 0.0;
  GMT_CHECK("abs max D2H", gmt_rt_memcpy_async(&m, ws.data(), sizeof(double), s_));
  GMT_CHECK("abs max sync", gmt_rt_stream_synchronize(s_));
  return m;
}

// One timed pass of every size the planner may use, on this rank's share
// with its real neighbours (a serial pass includes its exchange), max over
// ranks: the job's pass takes as long as its slowest rank.  The clock falls
// by about a quarter over the first few ms of sustained passes
// (profiles/r03_shares.md), so every pass type is launched once first (code
// object, occupancy query, clock settling), then the sizes are timed in two
// round-robin sweeps and each keeps its faster one: no size is measured only
// cold or only hot.
void JacobiSolver::calibrate_costs() {
  if (ks_ < 2) return;
  watchdog_kick("jacobi: pass-cost calibration");
  std::vector<int> ks;
  for (int K = 1; K <= ks_; ++K)
    if (K == 1 || (push_on_ ? gmt_jacobi5tb_push_supported(K) : gmt_jacobi5tb_supported(K))) ks.push_back(K);
  Buffer<double> d(ks.size(), GMT_SPACE_DEVICE);
  std::vector<double> host(ks.size(), 1e300);
  constexpr int kSweeps = 2;
  auto one = [&](int K) {
    if (K == 1) {
      step();
    } else {
      enqueue_block(parity_, K);
      parity_ ^= 1;
    }
  };
  for (int K : ks) one(K);
  synchronize();
  // enough passes per measurement for ~4 ms of GPU work: on small shares
  // (8192^2: 0.3 ms a pass) two passes were within the launch and sync
  // overhead of each other and the plan flipped between 18- and 20-sweep
  // passes from run to run (profiles/r04_shares.md)
  double t1 = wtime();
  one(ks_);
  synchronize();
  t1 = (wtime() - t1) * 1e3;
  {  // one pass count for every rank: the passes carry the exchanges
    GMT_CHECK("calib H2D", gmt_rt_memcpy(d.data(), &t1, sizeof(double)));
    t_.allreduce_max(d.data(), 1, s_);
    GMT_CHECK("calib D2H", gmt_rt_memcpy_async(&t1, d.data(), sizeof(double), s_));
    GMT_CHECK("calib sync", gmt_rt_stream_synchronize(s_));
  }
  const int kPasses = std::max(2, std::min(32, static_cast<int>(std::ceil(4.0 / std::max(t1, 1e-3)))));
  for (int sweep = 0; sweep < kSweeps; ++sweep)
    for (size_t i = 0; i < ks.size(); ++i) {
      const double t0 = wtime();
      for (int r = 0; r < kPasses; ++r) one(ks[i]);
      synchronize();
      host[i] = std::min(host[i], (wtime() - t0) / kPasses * 1e3);
    }
  GMT_CHECK("calib H2D", gmt_rt_memcpy(d.data(), host.data(), host.size() * sizeof(double)));
  t_.allreduce_max(d.data(), host.size(), s_);
  GMT_CHECK("calib D2H", gmt_rt_memcpy_async(host.data(), d.data(), host.size() * sizeof(double), s_));
  GMT_CHECK("calib sync", gmt_rt_stream_synchronize(s_));
  for (size_t i = 0; i < ks.size(); ++i) meas_ms_[ks[i]] = host[i];
  calibrated_ = true;
  // the built-in table was measured on one box for one kernel revision: say
  // so when this share disagrees with it by more than 10 %
  const double tab = table_pass_ms(ks_), got = meas_ms_[ks_];
  if (t_.rank() == 0 && tab > 0 && std::fabs(got - tab) > 0.1 * tab)
    std::fprintf(stderr, "# jacobi: measured %d-sweep pass %.3f ms vs the cost table's %.3f ms (%+.0f%%); "
                         "planning with the measured costs\n", ks_, got, tab, 100.0 * (got - tab) / tab);
  init_field();  // the timed passes advanced the solution: start over
}

void JacobiSolver::autotune_overlap() {
  if (ks_ < 2 || !halo_[0]->active()) return;  // nothing to hide
  watchdog_kick("jacobi: overlap autotune");
  Buffer<double> t(2, GMT_SPACE_DEVICE);
  double host[2] = {0.0, 0.0};
  constexpr int kPasses = 2;
  // first use of each mode's streams, untimed; then the modes in the order
  // A B B A, so the clock's fall over sustained passes (profiles/
  // r03_shares.md) does not favour the mode timed first
  for (int mode = 0; mode < 2; ++mode) {
    cfg_.overlap = mode == 0;
    enqueue_block(parity_, ks_);
    parity_ ^= 1;
  }
  synchronize();
  for (int mode : {0, 1, 1, 0}) {
    cfg_.overlap = mode == 0;
    const double t0 = wtime();
    for (int i = 0; i < kPasses; ++i) {
      enqueue_block(parity_, ks_);
      parity_ ^= 1;
    }
    synchronize();
    host[mode] += (wtime() - t0) / (2 * kPasses);
  }
  // one decision for every rank: the mode with the smaller summed time
  GMT_CHECK("tune H2D", gmt_rt_memcpy(t.data(), host, sizeof(host)));
  t_.allreduce_sum(t.data(), 2, s_);
  GMT_CHECK("tune D2H", gmt_rt_memcpy_async(host, t.data(), sizeof(host), s_));
  GMT_CHECK("tune sync", gmt_rt_stream_synchronize(s_));
  tune_s_[0] = host[0] / t_.size();
  tune_s_[1] = host[1] / t_.size();
  cfg_.overlap = host[0] <= host[1];
  init_field();  // the timed passes advanced the solution: start over
}

JacobiSolver::~JacobiSolver() {
  if (s_) gmt_rt_stream_synchronize(s_);
  for (void* b : push_opened_) GMT_WARN("ipc close", gmt_rt_ipc_close(b));
  if (cs_) gmt_rt_stream_synchronize(cs_);
  if (sb_) gmt_rt_stream_synchronize(sb_);
  for (auto& g : graph_) gmt_rt_graph_destroy(g);
  for (auto& g : graph2_) gmt_rt_graph_destroy(g);
  gmt_rt_event_destroy(ev_start_);
  gmt_rt_event_destroy(ev_halo_);
  if (ev_band_) gmt_rt_event_destroy(ev_band_);
  halo_[0].reset();
  halo_[1].reset();
  gmt_rt_stream_destroy(cs_);
  if (sb_) gmt_rt_stream_destroy(sb_);
  gmt_rt_stream_destroy(s_);
}

void JacobiSolver::sweep_full(int parity, double* resid) {
  const double* u = buf_[parity].data();
  double* un = buf_[parity ^ 1].data();
  GMT_CHECK("jacobi sweep", gmt_jacobi5(xo_, nx_, yo_, ny_, u, un, ld_, nullptr, 0, kC0, 0.0, resid, s_));
}

void JacobiSolver::enqueue_step(int parity) {
  Halo2D& h = *halo_[parity];
  fresh_[parity ^ 1] = false;
  if (!h.active()) {
    sweep_full(parity, nullptr);
    return;
  }
  if (!cfg_.overlap || nx_ < 6 || ny_ < 3) {
    h.start(s_);
    h.finish(s_);
    sweep_full(parity, nullptr);
    return;
  }
  const double* u = buf_[parity].data();
  double* un = buf_[parity ^ 1].data();
  // core: every cell whose 5-point stencil stays inside the interior; it
  // starts at an even column so the sweep keeps its 16-B vector path
  GMT_CHECK("event", gmt_rt_event_record(ev_start_, s_));
  GMT_CHECK("core sweep", gmt_jacobi5(xo_ + 2, nx_ - 4, yo_ + 1, ny_ - 2, u, un, ld_, nullptr, 0,
                                      kC0, 0.0, nullptr, s_));
  // halo on the high-priority stream, concurrent with the core sweep
  GMT_CHECK("wait", gmt_rt_stream_wait_event(cs_, ev_start_));
  h.start(cs_);
  h.finish(cs_);
  GMT_CHECK("event", gmt_rt_event_record(ev_halo_, cs_));
  GMT_CHECK("wait", gmt_rt_stream_wait_event(s_, ev_halo_));
  // boundary frame: first/last row, first/last two columns
  const int64_t y0 = yo_, y1 = yo_ + 1;
  const int64_t rects[16] = {xo_, nx_, y0,            1,       xo_,           nx_, yo_ + ny_ - 1, 1,
                             xo_, 2,   y1,            ny_ - 2, xo_ + nx_ - 2, 2,   y1,            ny_ - 2};
  GMT_CHECK("frame sweep", gmt_jacobi5_rects(4, rects, u, un, ld_, nullptr, 0, kC0, 0.0, s_));
}

int JacobiSolver::halo_mask() const {
  return (nb_.west >= 0 ? 1 : 0) | (nb_.east >= 0 ? 2 : 0) | (nb_.south >= 0 ? 4 : 0) |
         (nb_.north >= 0 ? 8 : 0);
}

void JacobiSolver::xk_launch(int K, int n, const int64_t* rects, int parity, int sig_rects, int sig_rows,
                             gmt_stream_t st, int sig_cols) {
  const double* u = buf_[parity].data();
  double* un = buf_[parity ^ 1].data();
  const int64_t dom[4] = {xo_, nx_, yo_, ny_};
  const int mask = halo_mask();
  unsigned* count = reinterpret_cast<unsigned*>(sig_.data());
  const bool sig = sig_rects > 0 || sig_rows > 0 || sig_cols != 0;
  gmt_tb_opts o{K,   cfg_.wg_waves, cfg_.seg_rows, exact_ ? 1 : 0, sig_rects, sig ? count : nullptr,
                sig ? sig_.data() + 1 : nullptr, sig_rows, st == sb_ && sb_ ? comm_cus_ : 0, sig_cols};
  o.clock = clk_.data();
  GMT_CHECK("jacobi tb", gmt_jacobi5tb(&o, n, rects, dom, mask, u, un, ld_, ny_ + 2 * g_, st ? st : s_));
}

// The bands of a band-first pass, all inside the one output rect (the
// interior): no band rects, no extra strips, segments or warm-ups.
// W/E halo sides: the rect's first / last strip group, every segment at
// full length, dispatched first; each of their workgroups signals when done
// (gmt_tb_opts.signal_cols) — with the pass's later rounds still to run.
// S/N halo sides: the other groups' segments next to those sides are row
// bands (gmt_tb_opts.signal_rows = g_: dispatched next, N ones walked
// bottom-up, each output wave signals once its first g_ rows are stored).
// (Round 3 took the W/E bands as separate rects with 3/4-length segments:
// 1.05-1.08x the serial pass on the N = 8 shares, profiles/r03_shares.md.)
// False when the domain is too small for the bands.
bool JacobiSolver::band_rects(int K, int64_t* rects, int* sig_cols, int* sig_rows) const {
  const int mask = halo_mask();
  const bool hw = mask & 1, he = mask & 2, hs = mask & 4, hn = mask & 8;
  const int64_t wb = std::max<int64_t>(gmt_jacobi5tb_group_cols(K, cfg_.wg_waves), g_);
  const int rb = (hs ? 1 : 0) + (hn ? 1 : 0);
  if (wb <= 0 || (rb > 0 && ny_ < rb * std::max<int64_t>(32, g_)) || ny_ < 64) return false;
  const int64_t r[4] = {xo_, nx_, yo_, ny_};
  std::copy(r, r + 4, rects);
  *sig_cols = (hw ? 1 : 0) | (he ? 2 : 0);
  *sig_rows = rb > 0 ? g_ : 0;
  return *sig_cols != 0 || rb > 0;
}

void JacobiSolver::exchange_now(int parity) {
  Halo2D& h = *halo_[parity];
  h.start(s_);
  h.finish(s_);
  fresh_[parity] = true;
}

// ks_ (or fewer) sweeps u(t) -> u(t+K) in one pass.
//   serial:     exchange the halo of u, then one fused launch;
//   overlap:    band-first — one launch whose boundary bands are dispatched
//               first and raise a completion signal; the comm stream waits
//               for it (gmt_signal_wait) and exchanges the halo of u(t+K)
//               while the interior workgroups still run.  The pass leaves
//               its output's halo current (fresh_), so the next pass starts
//               without an exchange.
// Every workgroup is one the serial pass would run too (plus short band
// segments): no frame pass, no redundant work (the core/frame scheme of
// round 1 cost 2-11 % per pass, profiles/r02_shares.md).
void JacobiSolver::enqueue_block(int parity, int K) {
  if (push_on_) {
    push_block(parity, K);
    return;
  }
  Halo2D& h = *halo_[parity];
  const int64_t dom[4] = {xo_, nx_, yo_, ny_};
  if (!h.active()) {
    maybe_corrupt(parity);
    xk_launch(K, 1, dom, parity, 0, 0);
    return;
  }
  if (!fresh_[parity]) exchange_now(parity);
  maybe_corrupt(parity);
  int64_t rects[4];
  int cols = 0, rows = 0;
  if (!cfg_.overlap || !band_rects(K, rects, &cols, &rows)) {
    xk_launch(K, 1, dom, parity, 0, 0);
    fresh_[parity ^ 1] = false;
    return;
  }
  // the comm stream forks before the launch (so it never waits for the whole
  // pass), and its wait kernel is enqueued after it
  band_ran_ = true;
  GMT_CHECK("event", gmt_rt_event_record(ev_start_, s_));
  GMT_CHECK("wait", gmt_rt_stream_wait_event(cs_, ev_start_));
  if (sb_) {  // the pass on the compute CUs, joined back into s_ below
    GMT_CHECK("wait", gmt_rt_stream_wait_event(sb_, ev_start_));
    xk_launch(K, 1, rects, parity, 0, rows, sb_, cols);
    GMT_CHECK("event", gmt_rt_event_record(ev_band_, sb_));
    GMT_CHECK("wait", gmt_rt_stream_wait_event(s_, ev_band_));
  } else {
    xk_launch(K, 1, rects, parity, 0, rows, nullptr, cols);
  }
  GMT_CHECK("signal wait", gmt_signal_wait(sig_.data() + 1, sig_.data() + 2,
                                           reinterpret_cast<unsigned*>(sig_.data() + 3), cs_));
  Halo2D& hn = *halo_[parity ^ 1];
  hn.set_pack_wgs(beside_pack_wgs_);  // beside the pass: few resident pack workgroups
  hn.start(cs_);
  hn.finish(cs_);
  hn.set_pack_wgs(0);
  GMT_CHECK("event", gmt_rt_event_record(ev_halo_, cs_));
  GMT_CHECK("wait", gmt_rt_stream_wait_event(s_, ev_halo_));
  fresh_[parity ^ 1] = true;
}

// ---- inline halo exchange (cfg_.push) ----
//
// Each fused pass stores its output's face cells a second time, straight
// into the ghost cells of the neighbours' next input buffer
// (gmt_tb_opts.push, csrc/kernels/jacobi5tb.hpp): the S / N faces (the
// first / last g_ rows of the interior), W / E faces (the first / last g_
// columns) and the g_ x g_ corners for the diagonal neighbours.  No pack,
// exchange or unpack launch: one hand-over launch after the pass
// (gmt_push_sync) tells every neighbour "my pass is done" and waits for
// theirs, so the next pass reads complete ghost cells and no rank writes a
// buffer its neighbour still reads (a neighbour pushes into this rank's
// buffer b^1 only during its pass p, which starts after this rank's pass
// p - 1 — the last reader of b^1 — handed over).  The round-4 traces showed
// why an exchange cannot hide beside a pass that holds every CU: its
// kernels only get registers as the pass drains (profiles/r04_overlap.md).
// Written by the pass itself, the faces cost a few store instructions per
// step of the boundary strips and segments.
namespace {
constexpr int kPushOpp[8] = {GMT_PUSH_N, GMT_PUSH_S, GMT_PUSH_E, GMT_PUSH_W,
                             GMT_PUSH_NE, GMT_PUSH_NW, GMT_PUSH_SE, GMT_PUSH_SW};
constexpr int kPushTag = 40000;  // + the direction, seen from the sender
struct PushWire {
  gmt_ipc_handle h[3];  // buf_[0], buf_[1], the flag slots
  uint64_t off[3];
  int64_t nx, ny, ld;
};
}  // namespace

void JacobiSolver::setup_push() {
  const JacobiConfig& c = cfg_;
  const int me = t_.rank();
  const int nbr[8] = {nb_.south, nb_.north, nb_.west, nb_.east, nb_.sw, nb_.se, nb_.nw, nb_.ne};
  // The kernel's rules (gmt_tb_opts.push) on the smallest share, so every
  // rank takes the same decision: an even face width, two segments clear of
  // each other's face, two strips (wider than any pass's strip output).
  const int64_t ny_min = c.ny_global / c.py, nx_min = c.nx_global / c.px;
  if ((g_ & 1) || g_ > 64 || ny_min < 2 * g_ + 2 || nx_min <= 256 || !gmt_jacobi5tb_push_supported(ks_)) return;
  bool remote = false;
  for (int d = 0; d < 8; ++d) remote = remote || (nbr[d] >= 0 && nbr[d] != me);
  comm::Control* ctl = t_.control();
  // no control plane for the mappings (rccl): the transport's exchange (the
  // same on every rank: one transport kind per job)
  if (remote && !ctl) return;
  push_flags_ = Buffer<uint64_t>(8, GMT_SPACE_FLAGS);
  GMT_CHECK("push flags", gmt_rt_memset_async(push_flags_.data(), 0, push_flags_.bytes(), s_));
  GMT_CHECK("push flags", gmt_rt_stream_synchronize(s_));
  push_err_ = Buffer<unsigned>(1, GMT_SPACE_PINNED);
  *push_err_.data() = 0;
  push_stop_ = Buffer<unsigned>(1, GMT_SPACE_DEVICE);
  GMT_CHECK("push stop", gmt_rt_memset_async(push_stop_.data(), 0, push_stop_.bytes(), s_));
  GMT_CHECK("push stop", gmt_rt_stream_synchronize(s_));
  PushWire mine;
  std::memset(&mine, 0, sizeof(mine));
  void* own[3] = {buf_[0].data(), buf_[1].data(), push_flags_.data()};
  if (remote)
    for (int i = 0; i < 3; ++i) {
      size_t off = 0;
      GMT_CHECK("ipc handle", gmt_rt_ipc_get_handle(&mine.h[i], &off, own[i]));
      mine.off[i] = off;
    }
  mine.nx = nx_;
  mine.ny = ny_;
  mine.ld = ld_;
  std::vector<PushWire> in(8);
  std::vector<comm::HostMsg> rs, ss;
  for (int d = 0; d < 8; ++d) {
    if (nbr[d] < 0 || nbr[d] == me) continue;
    rs.push_back({&in[d], sizeof(PushWire), nbr[d], kPushTag + kPushOpp[d]});
    ss.push_back({&mine, sizeof(PushWire), nbr[d], kPushTag + d});
  }
  if (!rs.empty()) ctl->exchange(rs, ss);
  std::map<std::string, void*> opened;  // a handle maps once per process
  auto open = [&](const gmt_ipc_handle& h, uint64_t off) -> char* {
    const std::string k(reinterpret_cast<const char*>(h.bytes), sizeof(h.bytes));
    auto it = opened.find(k);
    if (it == opened.end()) {
      void* base = nullptr;
      GMT_CHECK("ipc open", gmt_rt_ipc_open(&base, &h));
      push_opened_.push_back(base);
      it = opened.emplace(k, base).first;
    }
    return static_cast<char*>(it->second) + off;
  };
  for (int d = 0; d < 8; ++d) {
    if (nbr[d] < 0) continue;
    const bool self = nbr[d] == me;
    if (!self && in[d].ld != ld_) {
      std::printf("JacobiSolver: rank %d's row pitch %lld differs from rank %d's %lld\n", nbr[d],
                  static_cast<long long>(in[d].ld), me, static_cast<long long>(ld_));
      abort_job(EXIT_FAILURE);
    }
    const int64_t onx = self ? nx_ : in[d].nx, ony = self ? ny_ : in[d].ny;
    // this rank's face cell (x, y) -> the neighbour's ghost cell (x + tx, y + ty)
    const bool wside = d == GMT_PUSH_W || d == GMT_PUSH_SW || d == GMT_PUSH_NW;
    const bool eside = d == GMT_PUSH_E || d == GMT_PUSH_SE || d == GMT_PUSH_NE;
    const bool sside = d == GMT_PUSH_S || d == GMT_PUSH_SW || d == GMT_PUSH_SE;
    const bool nside = d == GMT_PUSH_N || d == GMT_PUSH_NW || d == GMT_PUSH_NE;
    const int64_t tx = wside ? onx : (eside ? -nx_ : 0);
    const int64_t ty = sside ? ony : (nside ? -ny_ : 0);
    for (int b = 0; b < 2; ++b) {
      // a pass reading buffer b writes b ^ 1: its faces go to the
      // neighbour's b ^ 1, the neighbour's input of the next pass
      const char* t = self ? reinterpret_cast<const char*>(buf_[b ^ 1].data()) : open(in[d].h[b ^ 1], in[d].off[b ^ 1]);
      push_base_[b][d] = reinterpret_cast<const double*>(
          reinterpret_cast<uintptr_t>(t) + static_cast<uintptr_t>((ty * ld_ + tx) * static_cast<int64_t>(sizeof(double))));
    }
    if (!self) {
      push_remote_[d] = reinterpret_cast<uint64_t*>(open(in[d].h[2], in[d].off[2])) + kPushOpp[d];
      push_mask_ |= 1 << d;
    }
  }
  push_on_ = true;
  cfg_.overlap = false;  // no band-first passes: the exchange is inline
}

void JacobiSolver::push_block(int parity, int K) {
  if (!fresh_[parity]) exchange_now(parity);
  maybe_corrupt(parity);
  const int64_t dom[4] = {xo_, nx_, yo_, ny_};
  gmt_tb_opts o{};
  o.sweeps = K;
  o.wg_waves = cfg_.wg_waves;
  o.exact = exact_ ? 1 : 0;
  for (int d = 0; d < 8; ++d) o.push[d] = push_base_[parity][d];
  o.push_w = g_;
  o.stop = push_stop_.data();
  o.clock = clk_.data();
  GMT_CHECK("jacobi tb (inline halo)", gmt_jacobi5tb(&o, 1, dom, dom, halo_mask(), buf_[parity].data(),
                                                     buf_[parity ^ 1].data(), ld_, ny_ + 2 * g_, s_));
  if (push_mask_) {
    fault_point_exchange(t_.rank());  // GMT_INJECT_HANG: the hand-over is this pass's exchange
    ++push_epoch_;
    GMT_CHECK("push hand-over", gmt_push_sync(push_flags_.data(), push_remote_, push_mask_, push_epoch_,
                                             push_err_.data(), push_stop_.data(), s_));
  }
  fresh_[parity ^ 1] = true;
}

int JacobiSolver::tb_launch_info(int K, int64_t out[6]) const {
  const int64_t dom[4] = {xo_, nx_, yo_, ny_};
  gmt_tb_opts o{};
  o.sweeps = K;
  o.wg_waves = cfg_.wg_waves;
  o.seg_rows = cfg_.seg_rows;
  o.exact = exact_ ? 1 : 0;
  if (push_on_) {
    for (int d = 0; d < 8; ++d) o.push[d] = push_base_[parity_][d];
    o.push_w = g_;
  }
  return gmt_jacobi5tb_plan(&o, 1, dom, dom, halo_mask(), ld_, ny_ + 2 * g_, out);
}

bool JacobiSolver::band_mode(int K) const {
  int64_t rects[4];
  int cols = 0, rows = 0;
  return cfg_.overlap && halo_[0] && halo_[0]->active() && band_rects(K, rects, &cols, &rows);
}

void JacobiSolver::step_block() {
  if (graph2_[parity_]) {
    // a band-first graph starts from a current halo (it was captured so)
    const bool band = band_mode(ks_);
    if (band && !fresh_[parity_]) exchange_now(parity_);
    band_ran_ = band_ran_ || band;
    GMT_CHECK("graph launch", gmt_rt_graph_launch(graph2_[parity_], s_));
    fresh_[parity_ ^ 1] = band;
  } else {
    enqueue_block(parity_, ks_);
  }
  parity_ ^= 1;  // u(t+ks) lives in the other buffer
}

// Measured cost of one fused pass of K sweeps (ms; gmt_kernel_bench
// --only=tb --sustained=1: back-to-back launches with the default launch
// shape and segment plan, Dirichlet sides, MI355X, profiles/r02_tb4c.md, the
// 4-column kernel) on two domain sizes.  One-wave strips (K <= 8) run at
// ~3.7-4.1 ms at 32768^2 (K = 9, 10 sit at 253-255 VGPRs); two-stage strips
// (K >= 12) are VALU bound from K ~ 16 (K = 22, 24 would exceed the register
// file at 2 waves per SIMD and spill: not built).  0 = no kernel for that K
// (odd K > 10).
namespace {
struct PassCosts {
  double points;  // lattice points of the measured domain
  double ms[GMT_TB_MAX_SWEEPS + 1];
};
constexpr PassCosts kCostLarge = {32768.0 * 32768.0,
                                  {0,    3.98, 4.13, 3.79, 3.86, 3.85, 3.68, 3.85, 3.91, 4.58, 4.57, 0,    3.63,
                                   0,    3.76, 0,    3.89, 0,    4.30, 0,    4.68}};
constexpr PassCosts kCostSmall = {8192.0 * 8192.0,
                                  {0,     0.311, 0.300, 0.294, 0.292, 0.292, 0.302, 0.287, 0.289,
                                   0.317, 0.322, 0,     0.264, 0,     0.284, 0,     0.289, 0,
                                   0.319, 0,     0.349}};
constexpr double kLaunchMs = 0.015;    // host launch + dispatch per pass
constexpr double kExchangeMs = 0.035;  // a halo exchange not hidden by the overlap
}  // namespace

double JacobiSolver::table_pass_ms(int K) const {
  if (K < 1 || K > GMT_TB_MAX_SWEEPS) return 0.0;
  // The table measured on the closer domain size, scaled to the LARGEST
  // share of the job (ceil of the global extents over the grid): every rank
  // must compute the same plan — ranks whose shares differ by a row would
  // otherwise pick different pass sequences and exchange at different sweeps
  // — and the job's pass takes as long as its largest share.
  const JacobiConfig& c = cfg_;
  const double pts = static_cast<double>((c.nx_global + c.px - 1) / c.px) *
                     static_cast<double>((c.ny_global + c.py - 1) / c.py);
  const PassCosts& tab = std::fabs(std::log(pts / kCostLarge.points)) < std::fabs(std::log(pts / kCostSmall.points))
                             ? kCostLarge
                             : kCostSmall;
  if (tab.ms[K] <= 0 || (push_on_ && K > 1 && !gmt_jacobi5tb_push_supported(K))) return 0.0;
  const bool exchanges = t_.size() > 1 || c.periodic;  // the same on every rank
  // a push pass exchanges inline (its face stores are in the table's
  // measured push costs, its hand-over is a launch): no serial exchange
  const double over = kLaunchMs + (exchanges && !c.overlap && !push_on_ ? kExchangeMs : 0.0);
  return tab.ms[K] * pts / tab.points + over;
}

std::vector<int> JacobiSolver::plan_passes(int k) const {
  if (k <= 0) return {};
  if (ks_ <= 1) return std::vector<int>(k, 1);
  // pass costs: measured on this share (prepare with calibrate; launches and
  // serial exchanges included; max over ranks), else the built-in table for
  // the job's largest share — the same costs, hence the same plan, on every rank
  std::vector<double> cost(ks_ + 1, 0.0);
  for (int K = 1; K <= ks_; ++K) cost[K] = calibrated_ ? meas_ms_[K] : table_pass_ms(K);
  return plan_pass_sequence(k, ks_, cost, calibrated_);
}

std::vector<int> plan_pass_sequence(int k, int ks, std::vector<double> cost, bool measured) {
  std::vector<int> plan;
  if (k <= 0) return plan;
  if (ks <= 1 || static_cast<int>(cost.size()) <= ks) return std::vector<int>(k, 1);
  const int ks_ = ks;
  // measured costs carry ~1-2% of clock noise: a pass shorter than ks must
  // win by more than that to displace full passes (a 1000-sweep 8192^2 plan
  // flipped between 50x20 and 5x20+50x18, the latter 1.5% slower:
  // profiles/r05_final/bench_2.json)
  if (measured)
    for (int K = 2; K < ks_; ++K) cost[K] *= 1.02;
  std::vector<double> best(k + 1, 1e300);
  std::vector<int> pick(k + 1, 0);
  best[0] = 0.0;
  for (int s = 1; s <= k; ++s)
    for (int K = 1; K <= ks_ && K <= s; ++K) {
      if (cost[K] <= 0) continue;
      const double c = best[s - K] + cost[K];
      if (c < best[s]) {
        best[s] = c;
        pick[s] = K;
      }
    }
  for (int s = k; s > 0; s -= pick[s]) plan.push_back(pick[s]);
  // full ks_ passes first (graph replays), then the rest, largest first
  std::sort(plan.begin(), plan.end(), [&](int a, int b) {
    return (a == ks_) != (b == ks_) ? a == ks_ : a > b;
  });
  return plan;
}

void JacobiSolver::run(int k) {
  in_run_ = true;
  for (int K : plan_passes(k)) {
    if (K == 1) {
      step();
    } else if (K == ks_) {
      step_block();
    } else {
      enqueue_block(parity_, K);  // eager; the ks-wide halo covers it
      parity_ ^= 1;
    }
  }
  in_run_ = false;
  watchdog_kick("jacobi steps enqueued");
}

void JacobiSolver::prepare(int k) {
  if (cfg_.calibrate && !calibrated_) calibrate_costs();
  std::vector<int> kinds;
  for (int K : plan_passes(k))
    if (std::find(kinds.begin(), kinds.end(), K) == kinds.end()) kinds.push_back(K);
  for (int K : kinds) {
    if (K == 1) {
      enqueue_step(parity_);
    } else {
      enqueue_block(parity_, K);
    }
    parity_ ^= 1;
  }
  synchronize();
  init_field();
}

void JacobiSolver::capture_graphs() {
  if (gmt_rt_backend() == GMT_BACKEND_HOST) return;  // no graphs on the CPU backend
  for (int b = 0; b < 2; ++b)
    if (halo_[b]->active() && !halo_[b]->capturable()) {
      std::printf("# jacobi: transport %s is not stream-ordered; running without hipGraphs\n",
                  t_.name());
      return;
    }
  // the first send/recv to each peer sets up connections: do that eagerly
  for (int b = 0; b < 2; ++b) {
    halo_[b]->start(cs_);
    halo_[b]->finish(cs_);
  }
  GMT_CHECK("sync", gmt_rt_stream_synchronize(cs_));
  const bool saved[2] = {fresh_[0], fresh_[1]};
  for (int p = 0; p < 4; ++p) {
    if (p >= 2 && (ks_ < 2 || push_on_)) break;  // inline-halo passes carry a per-pass epoch: eager
    // serial passes capture their exchange, band-first ones start from a
    // current halo (step_block makes sure of it)
    fresh_[0] = fresh_[1] = p >= 2 && band_mode(ks_);
    int e = gmt_rt_stream_begin_capture(s_);
    if (e == 0) {
      if (p < 2)
        enqueue_step(p);
      else
        enqueue_block(p - 2, ks_);
      e = gmt_rt_stream_end_capture(s_, p < 2 ? &graph_[p] : &graph2_[p - 2]);
    }
    fresh_[0] = saved[0];
    fresh_[1] = saved[1];
    if (e != 0) {
      std::printf("# jacobi: hipGraph capture unavailable (%s); running eagerly\n",
                  gmt_rt_error_string(e));
      for (auto* arr : {graph_, graph2_})
        for (int i = 0; i < 2; ++i) {
          gmt_rt_graph_destroy(arr[i]);
          arr[i] = nullptr;
        }
      return;
    }
  }
}

void JacobiSolver::step() {
  if (graph_[parity_])
    GMT_CHECK("graph launch", gmt_rt_graph_launch(graph_[parity_], s_));
  else
    enqueue_step(parity_);
  fresh_[parity_ ^ 1] = false;
  parity_ ^= 1;
}

void JacobiSolver::synchronize() {
  GMT_CHECK("sync", gmt_rt_stream_synchronize(s_));
  // band-first passes fork to the side streams and join back into s_ (and
  // graph replays of them run on s_), so s_ covers them; the side streams
  // are synchronised and the band signal's error word read only after an
  // eager band-first pass (serial passes use neither)
  if (band_ran_) {
    GMT_CHECK("sync", gmt_rt_stream_synchronize(cs_));
    if (sb_) GMT_CHECK("sync", gmt_rt_stream_synchronize(sb_));
    uint64_t err = 0;
    GMT_CHECK("signal D2H", gmt_rt_memcpy(&err, sig_.data() + 3, sizeof(err)));
    if (err != 0) {
      std::printf("JacobiSolver: a band-first pass timed out waiting for its boundary bands (error %llu)\n",
                  static_cast<unsigned long long>(err));
      abort_job(EXIT_FAILURE);
    }
    band_ran_ = false;
  }
  if (push_on_ && push_mask_ && *push_err_.data() != 0) {
    std::printf("JacobiSolver: an inline-halo hand-over timed out waiting for the neighbours in directions "
                "0x%x (GMT_WAIT_TIMEOUT_MS); ghost cells are stale\n", *push_err_.data());
    abort_job(EXIT_FAILURE);
  }
  // a halo exchange that timed out (IPC) left stale ghost cells: fail loudly
  for (auto& h : halo_)
    if (h) h->check();
  std::string why;
  if (!t_.ok(&why)) {
    std::printf("JacobiSolver: %s\n", why.c_str());
    abort_job(EXIT_FAILURE);
  }
  watchdog_kick("jacobi synchronize");
}

double JacobiSolver::residual() {
  if (!fresh_[parity_]) exchange_now(parity_);
  sweep_full(parity_, resid_ws_.data());
  fresh_[parity_ ^ 1] = false;
  t_.allreduce_sum(resid_ws_.data(), 1, s_);
  double r = 0.0;
  GMT_CHECK("resid D2H", gmt_rt_memcpy_async(&r, resid_ws_.data(), sizeof(double), s_));
  GMT_CHECK("resid sync", gmt_rt_stream_synchronize(s_));
  parity_ ^= 1;
  return std::sqrt(r);
}

void JacobiSolver::exchange_only() {
  Halo2D& h = *halo_[parity_];
  // the exchange packs the current field and writes its ghost ring: order it
  // after every pass already enqueued on the compute stream (on the compute
  // stream itself when the comm stream is held to a few CUs: this is the
  // blocking exchange bench.py times, and it has the GPU to itself)
  gmt_stream_t st = sb_ ? s_ : cs_;
  GMT_CHECK("event", gmt_rt_event_record(ev_start_, s_));
  GMT_CHECK("wait", gmt_rt_stream_wait_event(st, ev_start_));
  h.start(st);
  h.finish(st);
  GMT_CHECK("sync", gmt_rt_stream_synchronize(st));
  fresh_[parity_] = true;
}

// Fault injection for the check of the timed run: GMT_CORRUPT_PASS=R:P makes
// rank R, at the P-th fused pass that run() enqueued since the field was last
// initialised (bench.py: the warm-up's passes, then the timed ones), overwrite one ghost
// cell of the pass's input — after its exchange, or after the neighbour's
// inline push landed — with a wrong value, as a stale or corrupt pushed face
// cell would leave it.  The check (compare against single sweeps) must fire.
void JacobiSolver::maybe_corrupt(int parity) {
  if (!in_run_) return;  // calibration, prepare() and tuning passes do not count
  ++passes_;
  static const std::pair<int, int> spec = [] {
    const char* e = std::getenv("GMT_CORRUPT_PASS");
    int r = -1, p = -1;
    if (!e || std::sscanf(e, "%d:%d", &r, &p) != 2) r = p = -1;
    return std::make_pair(r, p);
  }();
  if (spec.first != t_.rank() || spec.second != passes_) return;
  // mid-face of the first side that has a neighbour (its ghost cells came
  // from that neighbour's exchange or push), else the west Dirichlet ring
  int64_t x = -1, y = ny_ / 2;
  if (nb_.west < 0 && nb_.east >= 0) {
    x = nx_;
  } else if (nb_.west < 0 && nb_.south >= 0) {
    x = nx_ / 2;
    y = -1;
  } else if (nb_.west < 0 && nb_.north >= 0) {
    x = nx_ / 2;
    y = ny_;
  }
  double* cell = buf_[parity].data() + (xo_ + x) + (yo_ + y) * ld_;
  GMT_CHECK("fault injection", gmt_fill_poly(3, 1, 1, 12345.0, 0.0, 0.0, 0.0, cell, ld_, s_));
  std::fprintf(stderr, "GMT FAULT INJECTION: rank %d corrupts ghost cell (x = %lld, y = %lld) of fused pass %d\n",
               t_.rank(), static_cast<long long>(x), static_cast<long long>(y), passes_);
}

void JacobiSolver::compare(JacobiSolver& o, double out[2]) {
  if (o.nx_ != nx_ || o.ny_ != ny_ || o.ox_ != ox_ || o.oy_ != oy_) {
    std::printf("JacobiSolver::compare: shares differ (%lldx%lld at %lld,%lld vs %lldx%lld at %lld,%lld)\n",
                static_cast<long long>(ny_), static_cast<long long>(nx_), static_cast<long long>(oy_),
                static_cast<long long>(ox_), static_cast<long long>(o.ny_), static_cast<long long>(o.nx_),
                static_cast<long long>(o.oy_), static_cast<long long>(o.ox_));
    abort_job(EXIT_FAILURE);
  }
  o.synchronize();
  Buffer<double> ws(2 * static_cast<size_t>(gmt_diff_sq_workspace(nx_, ny_)) + 2, GMT_SPACE_DEVICE);
  double* res = ws.data() + ws.size() - 2;
  GMT_CHECK("diff bits", gmt_diff_bits(nx_, ny_, buf_[parity_].data() + xo_ + yo_ * ld_, ld_,
                                       o.buf_[o.parity_].data() + o.xo_ + o.yo_ * o.ld_, o.ld_, res, ws.data(), s_));
  t_.allreduce_max(res, 1, s_);
  t_.allreduce_sum(res + 1, 1, s_);
  GMT_CHECK("diff bits D2H", gmt_rt_memcpy_async(out, res, 2 * sizeof(double), s_));
  GMT_CHECK("diff bits sync", gmt_rt_stream_synchronize(s_));
}

void JacobiSolver::clock_reset() {
  if (clk_.data()) GMT_CHECK("clock reset", gmt_rt_memset_async(clk_.data(), 0, clk_.bytes(), s_));
}

void JacobiSolver::clock_read(double out[3]) {
  out[0] = out[1] = out[2] = 0.0;
  if (!clk_.data()) return;
  uint64_t c[3] = {0, 0, 0};
  GMT_CHECK("clock D2H", gmt_rt_memcpy_async(c, clk_.data(), sizeof(c), s_));
  GMT_CHECK("clock sync", gmt_rt_stream_synchronize(s_));
  constexpr double kRealtimeMHz = 100.0;  // s_memrealtime: the CDNA constant 100 MHz clock
  out[0] = c[1] > 0 ? static_cast<double>(c[0]) / static_cast<double>(c[1]) * kRealtimeMHz : 0.0;
  out[1] = static_cast<double>(c[2]);
  out[2] = static_cast<double>(c[1]) / (kRealtimeMHz * 1e6);
}

void JacobiSolver::copy_interior(double* host) const {
  const double* src = buf_[parity_].data() + xo_ + yo_ * ld_;
  GMT_CHECK("interior D2H", gmt_rt_memcpy2d_async(host, nx_ * sizeof(double), src,
                                                  ld_ * sizeof(double), nx_ * sizeof(double), ny_, s_));
  GMT_CHECK("interior sync", gmt_rt_stream_synchronize(s_));
}

}  // namespace gmt
