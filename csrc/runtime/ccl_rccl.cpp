// RCCL implementation of gmt/ccl.h — the device data plane over xGMI.
//
// Replaces the reference's GPU-aware MPI calls on device buffers
// (mpi_stencil2d_gt.cc:186-225 Irecv/Isend, :615/:624 Allreduce,
// mpi_daxpy_nvtx.cc:285-288 Allgather).  Every op is enqueued on a HIP
// stream; completion is stream-ordered, so the halo exchange can overlap
// interior compute on another stream.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include "gmt/ccl.h"

namespace {
inline hipStream_t S(gmt_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline ncclComm_t C(gmt_ccl_comm_t c) { return reinterpret_cast<ncclComm_t>(c); }
}  // namespace

extern "C" {

int gmt_ccl_available(void) { return 1; }
int gmt_ccl_emulated(void) { return 0; }
const char* gmt_ccl_error_string(int err) {
  if (err == GMT_CCL_UNAVAILABLE) return "RCCL not available in this build";
  if (err == GMT_CCL_TIMEOUT) return "communicator init timed out (a rank never joined; GMT_CCL_INIT_TIMEOUT)";
  return ncclGetErrorString(static_cast<ncclResult_t>(err));
}
int gmt_ccl_version(int* v) { return static_cast<int>(ncclGetVersion(v)); }

int gmt_ccl_get_unique_id(gmt_ccl_id* id) {
  static_assert(sizeof(ncclUniqueId) <= sizeof(gmt_ccl_id), "ncclUniqueId size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  std::memset(id, 0, sizeof(*id));
  std::memcpy(id->internal, &u, sizeof(u));
  return static_cast<int>(r);
}

// ncclCommInitRank blocks until every rank has joined.  It runs on a helper
// thread (bound to the caller's device) and the caller waits for it against
// a deadline, GMT_CCL_INIT_TIMEOUT seconds (default 300): a rank that never
// joins makes every other rank return GMT_CCL_TIMEOUT instead of hanging the
// job (the caller names itself and aborts; the stuck init thread is left
// behind, the process is about to exit).  A non-blocking communicator would
// give the same deadline but makes every later call asynchronous, including
// the grouped exchanges captured into hipGraphs.
int gmt_ccl_comm_init(gmt_ccl_comm_t* comm, int nranks, const gmt_ccl_id* id, int rank) {
  *comm = nullptr;
  ncclUniqueId u;
  std::memcpy(&u, id->internal, sizeof(u));
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const char* e = std::getenv("GMT_CCL_INIT_TIMEOUT");
  const double limit = e && std::atof(e) > 0.0 ? std::atof(e) : 300.0;
  struct State {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclSuccess;
  };
  auto st = std::make_shared<State>();
  std::thread([st, u, nranks, rank, dev] {
    ncclComm_t c = nullptr;
    ncclResult_t r = hipSetDevice(dev) == hipSuccess ? ncclCommInitRank(&c, nranks, u, rank) : ncclUnhandledCudaError;
    std::lock_guard<std::mutex> g(st->m);
    st->c = c;
    st->r = r;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lk(st->m);
  if (!st->cv.wait_for(lk, std::chrono::duration<double>(limit), [&] { return st->done; })) return GMT_CCL_TIMEOUT;
  *comm = reinterpret_cast<gmt_ccl_comm_t>(st->c);
  return static_cast<int>(st->r);
}
int gmt_ccl_comm_destroy(gmt_ccl_comm_t comm) {
  return comm ? static_cast<int>(ncclCommDestroy(C(comm))) : 0;
}
int gmt_ccl_group_start(void) { return static_cast<int>(ncclGroupStart()); }
int gmt_ccl_group_end(void) { return static_cast<int>(ncclGroupEnd()); }

int gmt_ccl_send(const void* buf, size_t bytes, int peer, gmt_ccl_comm_t comm, gmt_stream_t s) {
  return static_cast<int>(ncclSend(buf, bytes, ncclChar, peer, C(comm), S(s)));
}
int gmt_ccl_recv(void* buf, size_t bytes, int peer, gmt_ccl_comm_t comm, gmt_stream_t s) {
  return static_cast<int>(ncclRecv(buf, bytes, ncclChar, peer, C(comm), S(s)));
}
int gmt_ccl_allreduce_sum_f64(const double* send, double* recv, size_t count,
                              gmt_ccl_comm_t comm, gmt_stream_t s) {
  return static_cast<int>(ncclAllReduce(send, recv, count, ncclFloat64, ncclSum, C(comm), S(s)));
}
int gmt_ccl_allreduce_max_f64(const double* send, double* recv, size_t count,
                              gmt_ccl_comm_t comm, gmt_stream_t s) {
  return static_cast<int>(ncclAllReduce(send, recv, count, ncclFloat64, ncclMax, C(comm), S(s)));
}
int gmt_ccl_allgather(const void* send, void* recv, size_t bytes_per_rank, gmt_ccl_comm_t comm,
                      gmt_stream_t s) {
  return static_cast<int>(ncclAllGather(send, recv, bytes_per_rank, ncclChar, C(comm), S(s)));
}
int gmt_ccl_broadcast(void* buf, size_t bytes, int root, gmt_ccl_comm_t comm, gmt_stream_t s) {
  return static_cast<int>(ncclBroadcast(buf, buf, bytes, ncclChar, root, C(comm), S(s)));
}

}  // extern "C"
