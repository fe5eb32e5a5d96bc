// gmt/control.hpp — the host control plane under the device transports.
//
// The reference has one plane for everything: MPI carries both the data and
// the bookkeeping (mpi_stencil2d_gt.cc:179-225).  Here the data moves over a
// device transport (gmt/transport.hpp) and a small host control plane does
// the rest: handle exchange for HIP IPC, host-staged collectives, barriers.
// Two implementations:
//
//   mpi     MPI point-to-point + collectives (the native apps; gmt/comm.hpp)
//   socket  a full mesh of Unix-domain stream sockets between the ranks of
//           one node, named by a 128-byte id that one rank creates and the
//           launcher distributes (torch.distributed in the Python engine).
//           No MPI, so libgmt_engine.so can run the IPC transport with
//           several ranks on one GPU — the oversubscription mode of the
//           reference (mpi_daxpy.cc:43-54) — without an MPI library.
//
// Messages between a pair of ranks match by (peer, tag) in issue order, as
// MPI's do.  Collectives reduce in rank order, so every rank gets the same
// bits.  Tags below 0 are reserved for the collectives.
#pragma once

#include <cstddef>
#include <memory>
#include <vector>

namespace gmt {
namespace comm {

struct HostMsg {
  void* buf;  // host memory
  size_t bytes;
  int peer;
  int tag;  // >= 0
};

class Control {
 public:
  virtual ~Control() = default;
  virtual const char* name() const = 0;
  int rank() const { return rank_; }
  int size() const { return size_; }
  // Every receive and send progresses concurrently; returns when all are
  // done.  A receive's size must equal the matching send's.
  virtual void exchange(const std::vector<HostMsg>& recvs, const std::vector<HostMsg>& sends) = 0;
  // host-memory collectives
  virtual void allreduce_sum(double* buf, size_t n) = 0;
  virtual void allreduce_max(double* buf, size_t n) = 0;
  // recv = concat over ranks of bpr bytes; in place when send == recv + rank*bpr
  virtual void allgather(const void* send, void* recv, size_t bpr) = 0;
  virtual void barrier() = 0;

 protected:
  Control(int rank, int size) : rank_(rank), size_(size) {}
  int rank_ = 0, size_ = 1;
};

// Socket mesh of one node.  `id` is 128 bytes from make_socket_control_id on
// one rank, the same bytes on every rank.  GMT_CTL_TIMEOUT_S (default 300)
// bounds the connection set-up and every blocking wait: a peer that never
// shows up or stops answering aborts the job with a message, never a hang.
constexpr size_t kControlIdBytes = 128;
void make_socket_control_id(char* id128);
std::unique_ptr<Control> make_socket_control(int rank, int size, const char* id128);

}  // namespace comm
}  // namespace gmt
