// C ABI of the native Jacobi engine (gmt/engine.h) for the Python package.
#include <cstring>
#include <memory>
#include <vector>

#include "gmt/engine.h"
#include "gmt/jacobi.hpp"
#include "gmt/kernels.h"

namespace {
struct Handle {
  std::unique_ptr<gmt::comm::Transport> t;
  std::unique_ptr<gmt::JacobiSolver> s;
  int py = 1, px = 1;
};
}  // namespace

extern "C" {

int gmt_engine_unique_id(void* out128) {
  gmt_ccl_id id;
  std::memset(&id, 0, sizeof(id));
  const int e = gmt_ccl_get_unique_id(&id);
  std::memcpy(out128, &id, sizeof(id));
  return e;
}

void* gmt_engine_jacobi_create(int64_t ny, int64_t nx, int py, int px, int rank, int world,
                               int transport, const void* ccl_id, const gmt_engine_opts* opts) {
  gmt_engine_opts o{};
  if (opts) o = *opts;
  if (o.tsteps < 0 || o.tsteps > GMT_TB_MAX_SWEEPS || o.overlap < 0 || o.overlap > 2 || o.wg_waves < 0 ||
      o.wg_waves > 8 || o.seg_rows < 0 || o.exact < -1 || o.exact > 1)
    return nullptr;
  auto* h = new Handle();
  if (transport == GMT_ENGINE_RCCL) {
    gmt_ccl_id id;
    std::memcpy(&id, ccl_id, sizeof(id));
    h->t = gmt::comm::make_rccl_transport(rank, world, id);
  } else {
    if (world != 1) {
      delete h;
      return nullptr;
    }
    h->t = gmt::comm::make_local_transport();
  }
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
  h->py = py;
  h->px = px;
  h->s = std::make_unique<gmt::JacobiSolver>(*h->t, c);
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
  static_cast<Handle*>(p)->s->run(steps);
  return 0;
}
int gmt_engine_jacobi_sync(void* p) {
  static_cast<Handle*>(p)->s->synchronize();
  return 0;
}
double gmt_engine_jacobi_residual(void* p) { return static_cast<Handle*>(p)->s->residual(); }
int gmt_engine_jacobi_exchange(void* p) {
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
  return 0;
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
const char* gmt_engine_backend(void) { return gmt_rt_backend_name(); }

}  // extern "C"
