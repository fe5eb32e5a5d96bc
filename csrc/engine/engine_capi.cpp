// C ABI of the native Jacobi engine (gmt/engine.h) for the Python package.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <memory>
#include <vector>

#include <unistd.h>

#include "gmt/control.hpp"
#include "gmt/engine.h"
#include "gmt/jacobi.hpp"
#include "gmt/kernels.h"
#include "gmt/watchdog.hpp"

namespace {
struct Handle {
  std::unique_ptr<gmt::comm::Transport> t;
  std::unique_ptr<gmt::JacobiSolver> s;
  int py = 1, px = 1;
};

}  // namespace

namespace gmt {
namespace {
// The engine runs inside a Python process: a job-wide abort (a failed check,
// the watchdog firing from its own thread while the main thread is blocked
// in a collective) must end the process at once, not run exit handlers that
// wait on the hung device or communicator; the launcher then tears the other
// ranks down.
[[noreturn]] void engine_abort(int code) {
  std::fflush(stdout);
  std::fflush(stderr);
  _exit(code);
}
}  // namespace

// Arms the hang watchdog (gmt/watchdog.hpp) for an engine entry point: a
// no-op unless GMT_TIMEOUT is set (bench.py sets a default), idempotent.
void engine_watchdog(int rank, const char* phase) {
  if (!abort_hook()) abort_hook() = &engine_abort;
  int dev = -1;
  (void)gmt_rt_get_device(&dev);
  watchdog_start(rank, dev);
  watchdog_kick(phase);
}

// Transport of an engine handle (also used by deriv_bench.cpp); nullptr when
// the request is invalid.
std::unique_ptr<comm::Transport> engine_transport(int rank, int world, int transport, const void* id) {
  if (world < 1 || rank < 0 || rank >= world) return nullptr;
  // the GPU's socket, once per process, before the first transport allocates
  static const int numa_node = [] {
    int dev = -1, node = -1;
    if (gmt_rt_get_device(&dev) == 0 && dev >= 0) (void)gmt_rt_bind_numa(dev, &node);
    return node;
  }();
  (void)numa_node;
  if (transport == GMT_ENGINE_RCCL) {
    gmt_ccl_id cid;
    std::memcpy(&cid, id, sizeof(cid));
    engine_watchdog(rank, "engine: rccl communicator init");
    auto t = comm::make_rccl_transport(rank, world, cid);
    watchdog_kick("engine: rccl communicator ready");
    return t;
  }
  if (transport == GMT_ENGINE_IPC) {
    if (!id) return nullptr;
    engine_watchdog(rank, "engine: ipc control plane connect");
    auto t = comm::make_ipc_transport(comm::make_socket_control(rank, world, static_cast<const char*>(id)));
    watchdog_kick("engine: ipc transport ready");
    return t;
  }
  if (world != 1) return nullptr;
  engine_watchdog(rank, "engine: local transport");
  return comm::make_local_transport();
}
}  // namespace gmt

extern "C" {

int gmt_engine_unique_id(void* out128) {
  gmt_ccl_id id;
  std::memset(&id, 0, sizeof(id));
  const int e = gmt_ccl_get_unique_id(&id);
  std::memcpy(out128, &id, sizeof(id));
  return e;
}

int gmt_engine_control_id(void* out128) {
  gmt::comm::make_socket_control_id(static_cast<char*>(out128));
  return 0;
}

void* gmt_engine_comm_create(int rank, int world, int transport, const void* id) {
  return gmt::engine_transport(rank, world, transport, id).release();
}
int gmt_engine_comm_allreduce_sum(void* h, double* buf, int64_t n, void* stream) {
  auto* t = static_cast<gmt::comm::Transport*>(h);
  if (!t || n < 0) return 1;
  const auto s = static_cast<gmt_stream_t>(stream);
  t->allreduce_sum(buf, static_cast<size_t>(n), s);
  GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
  std::string why;
  if (!t->ok(&why)) {
    std::printf("gmt_engine_comm_allreduce_sum: %s\n", why.c_str());
    gmt::abort_job(EXIT_FAILURE);
  }
  return 0;
}
const char* gmt_engine_comm_name(void* h) { return static_cast<gmt::comm::Transport*>(h)->name(); }
void gmt_engine_comm_destroy(void* h) { delete static_cast<gmt::comm::Transport*>(h); }

void gmt_engine_watchdog_kick(const char* phase) {
  // the phase string is kept by pointer: Python passes a bytes object that
  // may be freed, so copy it into a small ring of static slots
  static char slots[8][96];
  static std::atomic<unsigned> next{0};
  char* d = slots[next.fetch_add(1) % 8];
  std::snprintf(d, sizeof(slots[0]), "%s", phase ? phase : "python");
  gmt::watchdog_kick(d);
}
void gmt_engine_watchdog_epitaph(const char* json, int code) { gmt::watchdog_set_epitaph(json, code); }
double gmt_engine_watchdog_timeout(void) {
  return gmt::watchdog_state().armed.load() ? gmt::watchdog_state().timeout : 0.0;
}

void* gmt_engine_jacobi_create(int64_t ny, int64_t nx, int py, int px, int rank, int world,
                               int transport, const void* ccl_id, const gmt_engine_opts* opts) {
  gmt_engine_opts o{};
  if (opts) o = *opts;
  if (o.tsteps < 0 || o.tsteps > GMT_TB_MAX_SWEEPS || o.overlap < 0 || o.overlap > 2 || o.wg_waves < 0 ||
      o.wg_waves > 8 || o.seg_rows < 0 || o.exact < -1 || o.exact > 1 || o.init < 0 || o.init > 1 ||
      o.calibrate < 0 || o.calibrate > 1 || o.seed < 0 || o.seed >= (int64_t(1) << 53) || o.push < 0 || o.push > 1)
    return nullptr;
  auto* h = new Handle();
  h->t = gmt::engine_transport(rank, world, transport, ccl_id);
  if (!h->t) {
    delete h;
    return nullptr;
  }
  gmt::watchdog_kick("engine: jacobi setup");
  gmt::JacobiConfig c;
  c.ny_global = ny;
  c.nx_global = nx;
  c.py = py;
  c.px = px;
  c.periodic = o.periodic != 0;
  c.overlap = o.overlap != 0;
  c.overlap_auto = o.overlap == 2;  // time both modes, keep the faster
  c.graph = o.graph != 0;
  c.tblock = o.tsteps > 1;
  c.tsteps = o.tsteps;
  c.wg_waves = o.wg_waves;
  c.seg_rows = o.seg_rows;
  c.exact = o.exact;
  c.init = o.init;
  c.seed = static_cast<uint64_t>(o.seed);
  c.calibrate = o.calibrate != 0;
  c.push = o.push != 0;
  h->py = py;
  h->px = px;
  h->s = std::make_unique<gmt::JacobiSolver>(*h->t, c);
  gmt::watchdog_kick("engine: jacobi ready");
  return h;
}

void gmt_engine_jacobi_destroy(void* p) {
  auto* h = static_cast<Handle*>(p);
  if (!h) return;
  h->s.reset();
  h->t.reset();
  delete h;
}

int gmt_engine_jacobi_run(void* p, int steps) {
  gmt::watchdog_kick("engine: jacobi run (enqueue)");
  static_cast<Handle*>(p)->s->run(steps);
  return 0;
}
int gmt_engine_jacobi_sync(void* p) {
  gmt::watchdog_kick("engine: jacobi synchronize (waiting for the device)");
  static_cast<Handle*>(p)->s->synchronize();
  return 0;
}
double gmt_engine_jacobi_residual(void* p) { return static_cast<Handle*>(p)->s->residual(); }
int gmt_engine_jacobi_exchange(void* p) {
  gmt::watchdog_kick("engine: halo exchange");
  static_cast<Handle*>(p)->s->exchange_only();
  return 0;
}
int gmt_engine_jacobi_info(void* p, int64_t* out) {
  auto* h = static_cast<Handle*>(p);
  auto& s = *h->s;
  out[0] = s.nx();
  out[1] = s.ny();
  out[2] = s.off_x();
  out[3] = s.off_y();
  out[4] = static_cast<int64_t>(s.bytes_per_exchange());
  out[5] = static_cast<int64_t>(s.messages());
  out[6] = s.graph_active();
  out[7] = s.overlap_active();
  out[8] = h->py;
  out[9] = h->px;
  out[10] = s.tsteps();
  out[11] = static_cast<int64_t>(s.tuned_overlap_s() * 1e9);  // overlap_auto timings, ns per pass
  out[12] = static_cast<int64_t>(s.tuned_serial_s() * 1e9);
  out[13] = s.exact();
  out[14] = s.band_first();
  out[15] = s.push_active();
  return 0;
}
int gmt_engine_jacobi_tb_info(void* p, int K, int64_t* out) {
  return static_cast<Handle*>(p)->s->tb_launch_info(K, out);
}
int gmt_engine_jacobi_plan(void* p, int steps, int* out, int max) {
  const std::vector<int> plan = static_cast<Handle*>(p)->s->plan_passes(steps);
  for (int i = 0; i < static_cast<int>(plan.size()) && i < max; ++i) out[i] = plan[i];
  return static_cast<int>(plan.size());
}
int gmt_engine_jacobi_prepare(void* p, int steps) {
  static_cast<Handle*>(p)->s->prepare(steps);
  return 0;
}
int gmt_engine_jacobi_copy_interior(void* p, double* host) {
  static_cast<Handle*>(p)->s->copy_interior(host);
  return 0;
}
int gmt_engine_plan_from_costs(int k, int ks, const double* cost, int measured, int* out, int max) {
  if (k < 0 || ks < 1 || ks > GMT_TB_MAX_SWEEPS || !cost) return -1;
  const std::vector<int> plan = gmt::plan_pass_sequence(k, ks, std::vector<double>(cost, cost + ks + 1), measured != 0);
  for (int i = 0; i < static_cast<int>(plan.size()) && i < max; ++i) out[i] = plan[i];
  return static_cast<int>(plan.size());
}
int gmt_engine_jacobi_compare(void* a, void* b, double* out) {
  if (!a || !b || !out) return 1;
  gmt::watchdog_kick("engine: compare with the single-sweep replay");
  static_cast<Handle*>(a)->s->compare(*static_cast<Handle*>(b)->s, out);
  return 0;
}
int gmt_engine_jacobi_clock(void* p, int reset, double* out) {
  auto& s = *static_cast<Handle*>(p)->s;
  if (reset) {
    s.clock_reset();
    return 0;
  }
  if (!out) return 1;
  s.clock_read(out);
  return 0;
}
double gmt_engine_jacobi_stat(void* p, int what) {
  const auto& s = *static_cast<Handle*>(p)->s;
  switch (what) {
    case 0: return s.max_abs_u0();
    case 1: return s.measured_pass_ms(s.tsteps());
    case 2: return s.table_pass_ms(s.tsteps());
    default: return 0.0;
  }
}
const char* gmt_engine_backend(void) { return gmt_rt_backend_name(); }

}  // extern "C"
