// C ABI of the native Jacobi engine (gmt/engine.h) for the Python package.
#include <cstring>
#include <memory>

#include "gmt/engine.h"
#include "gmt/jacobi.hpp"

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
                               int transport, const void* ccl_id, int flags, int variant) {
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
  c.periodic = flags & 1;
  c.overlap = (flags & 2) != 0;
  c.overlap_auto = (flags & 16) != 0;  // bit4: time both modes, keep the faster
  c.graph = (flags & 4) != 0;
  c.tblock = (flags & 8) != 0;
  c.tsteps = (flags >> 8) & 0xf;  // bits 8-11: sweeps per fused pass (0 = from bit 3)
  c.variant = variant;
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
  return 0;
}
int gmt_engine_jacobi_copy_interior(void* p, double* host) {
  static_cast<Handle*>(p)->s->copy_interior(host);
  return 0;
}
const char* gmt_engine_backend(void) { return gmt_rt_backend_name(); }

}  // extern "C"
