// gmt/transport.hpp — pluggable device-data transports.
//
// The reference has exactly one transport: GPU-aware MPI fed device,
// managed or pinned pointers (mpi_stencil2d_gt.cc:179-225, :615;
// mpi_daxpy_nvtx.cc:285-288), with host staging as an in-benchmark option
// (mpi_stencil2d_gt.cc:147-176).  On an MI355X node MPI is the control plane
// and the data plane is one of:
//
//   mpi-host   face -> page-locked staging (one kernel gathers the strided
//              face, per-chunk flags) -> MPI -> one kernel scatters from
//              page-locked memory into the ghost rows (reference stage_host /
//              buf:1; works everywhere)
//   mpi-direct device/managed pointers straight to MPI — only when MPI can
//              read them: a GPU-aware MPI (GMT_MPI_GPU_AWARE=1), managed or
//              host memory, or the host backend
//   rccl       ncclSend/ncclRecv grouped per exchange on the caller's stream,
//              ncclAllReduce / ncclAllGather for collectives: xGMI links,
//              stream-ordered, one rank per GPU
//   ipc        HIP IPC: each rank maps its peers' staging slots and flags
//              once (handles traded over the host control plane,
//              gmt/control.hpp: MPI in the apps, a socket mesh in the engine)
//              and every exchange is one stream-ordered kernel that pulls the
//              peers' slots (xGMI peer read, or a same-device copy when ranks
//              share one GPU).  The one device-direct path that works with
//              several ranks per GPU.
//   local      single process: messages to self become device copies
//              (periodic boundaries on one GPU; the Python engine's CPU tests)
//
// Exchanges are PERSISTENT plans (like MPI_Send_init/MPI_Recv_init): the
// buffers are registered once, so staging memory, RCCL peers and IPC
// mappings are set up outside the timed loop — the reference re-allocates
// its buffers on every call (mpi_stencil2d_gt.cc:141-156).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "gmt/check.hpp"

namespace gmt {
namespace comm {

class Control;

// A column-major block of a field: `rows` contiguous doubles per column,
// `cols` columns at pitch `ld` doubles (a halo face in place)
struct Block {
  double* base = nullptr;
  size_t rows = 0, cols = 0, ld = 0;
};

struct Msg {
  void* buf;     // device (or managed/host) memory; nullptr with a block on a strided transport
  size_t bytes;
  int peer;      // rank in the transport's communicator
  int tag;       // matches a send on the peer with the same tag
  // the message's packed contents in place (rows x cols, packed column by
  // column): a transport with takes_blocks() reads sends from / writes
  // receives into the field directly — no separate pack / unpack launch
  Block block = {};
};

class Exchange {
 public:
  virtual ~Exchange() = default;
  // Send buffers hold valid data in stream order on `s`.  Starts the transfer.
  virtual void start(gmt_stream_t s) = 0;
  // On return the receive buffers are valid in stream order on `s`.
  virtual void wait(gmt_stream_t s) = 0;
  // Fully stream-ordered (no host blocking in start/wait): may be captured
  // into a hipGraph.
  virtual bool graph_capturable() const { return false; }
  // After the stream has been synchronised: false (and a reason) when an
  // earlier exchange failed without the host noticing — an IPC wait that
  // timed out and left stale data.  Transports that block on the host
  // report failures at once and are always ok().
  virtual bool ok(std::string* why = nullptr) const {
    (void)why;
    return true;
  }
  void run(gmt_stream_t s) {
    start(s);
    wait(s);
  }
};

enum class Kind { Auto, MpiHost, MpiDirect, Rccl, Ipc, Local };

class Transport {
 public:
  virtual ~Transport() = default;
  virtual Kind kind() const = 0;
  virtual const char* name() const = 0;
  virtual std::unique_ptr<Exchange> plan(const std::vector<Msg>& recvs,
                                         const std::vector<Msg>& sends) = 0;
  // in-place sum over all ranks of a device/managed vector, stream-ordered on s
  virtual void allreduce_sum(double* buf, size_t n, gmt_stream_t s) = 0;
  // in-place max over all ranks (device/managed vector), stream-ordered on s
  virtual void allreduce_max(double* buf, size_t n, gmt_stream_t s) = 0;
  // recv = concat over ranks of `bytes_per_rank` from each rank's send;
  // in place when send == recv + rank*bytes_per_rank
  virtual void allgather(const void* send, void* recv, size_t bytes_per_rank, gmt_stream_t s) = 0;
  // Exchange::ok for the transport's own cached plans (collectives)
  virtual bool ok(std::string* why = nullptr) const {
    (void)why;
    return true;
  }
  // the host control plane under the transport, when it has one
  virtual Control* control() { return nullptr; }
  // plans accept messages given as a field Block (buf == nullptr) and move
  // them in place (mpi-host's kernel staging: the face is gathered straight
  // into page-locked memory and scattered back out of it; ipc: the exchange
  // kernel gathers into / scatters out of its staging slots)
  virtual bool takes_blocks() const { return false; }
  // a plan writes its Block receives after its flat ones (mpi-host defers
  // the field scatters): a flat receive may then overlap a Block receive
  // and the Block wins, as the corner blocks over the y faces' stale corner
  // cells need.  Without it (ipc: every receive in one kernel, no order)
  // Halo2D sends y faces as Blocks that leave the corner cells out.
  virtual bool orders_block_receives() const { return false; }
  int rank() const { return rank_; }
  int size() const { return size_; }

 protected:
  Transport(int rank, int size) : rank_(rank), size_(size) {}
  int rank_ = 0, size_ = 1;
};

const char* kind_name(Kind k);

// RCCL over xGMI, bootstrapped from an already-distributed unique id (the
// MPI apps broadcast it with MPI_Bcast, the Python engine through
// torch.distributed).  One rank per GPU.
std::unique_ptr<Transport> make_rccl_transport(int rank, int size, const gmt_ccl_id& id);
// Single-process transport: every message must be addressed to rank 0
// (periodic self-exchange); a device-to-device copy per message.
std::unique_ptr<Transport> make_local_transport();
// HIP IPC over a host control plane (csrc/comm/transport_ipc.cpp): owning,
// or borrowing one that outlives the transport.  Same node only.
std::unique_ptr<Transport> make_ipc_transport(std::unique_ptr<Control> ctl);
std::unique_ptr<Transport> make_ipc_transport(Control& ctl);

}  // namespace comm
}  // namespace gmt
