// MPI-based transports: mpi-host, mpi-direct, ipc, and the factory that
// bootstraps rccl over MPI (gmt/comm.hpp, gmt/transport.hpp).
#include <dlfcn.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>

#include "gmt/buffer.hpp"
#include "gmt/comm.hpp"
#include "gmt/mpi.hpp"

namespace gmt {
namespace comm {

namespace {

// MPI counts are int: send doubles when possible so 8-B aligned payloads up
// to 16 GiB fit in one message (mpigatherinplace moves 1 GiB per rank).
void mpi_count(size_t bytes, MPI_Datatype* t, int* n) {
  if (bytes % 8 == 0 && bytes / 8 <= static_cast<size_t>(INT_MAX)) {
    *t = MPI_DOUBLE;
    *n = static_cast<int>(bytes / 8);
  } else if (bytes <= static_cast<size_t>(INT_MAX)) {
    *t = MPI_BYTE;
    *n = static_cast<int>(bytes);
  } else {
    std::printf("gmt::comm: message of %zu bytes exceeds one MPI message\n", bytes);
    abort_job(2);
  }
}

void isend(const void* p, size_t bytes, int peer, int tag, MPI_Comm c, MPI_Request* r) {
  MPI_Datatype t;
  int n;
  mpi_count(bytes, &t, &n);
  GMT_MPI_CHECK(MPI_Isend(p, n, t, peer, tag, c, r));
}
void irecv(void* p, size_t bytes, int peer, int tag, MPI_Comm c, MPI_Request* r) {
  MPI_Datatype t;
  int n;
  mpi_count(bytes, &t, &n);
  GMT_MPI_CHECK(MPI_Irecv(p, n, t, peer, tag, c, r));
}
void waitall(std::vector<MPI_Request>& reqs, const char* what) {
  if (reqs.empty()) return;
  std::vector<MPI_Status> st(reqs.size());
  int rv = MPI_Waitall(static_cast<int>(reqs.size()), reqs.data(), st.data());
  if (rv != MPI_SUCCESS) {
    std::printf("%s error: %d (%d)\n", what, rv, st[0].MPI_ERROR);
    abort_job(2);
  }
  reqs.clear();
}

// Host-staged collectives shared by the mpi-host and ipc transports.
void staged_allreduce(MPI_Comm c, double* buf, size_t n, gmt_stream_t s) {
  Buffer<double> h(n, GMT_SPACE_PINNED);
  GMT_CHECK("allreduce D2H", gmt_rt_memcpy_async(h.data(), buf, n * sizeof(double), s));
  GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
  GMT_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, h.data(), static_cast<int>(n), MPI_DOUBLE, MPI_SUM, c));
  GMT_CHECK("allreduce H2D", gmt_rt_memcpy_async(buf, h.data(), n * sizeof(double), s));
  GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
}
void staged_allgather(MPI_Comm c, int rank, int size, const void* send, void* recv, size_t bpr,
                      gmt_stream_t s) {
  Buffer<char> h(bpr * size, GMT_SPACE_PINNED);
  GMT_CHECK("allgather D2H", gmt_rt_memcpy_async(h.data() + rank * bpr, send, bpr, s));
  GMT_CHECK("allgather sync", gmt_rt_stream_synchronize(s));
  MPI_Datatype t;
  int n;
  mpi_count(bpr, &t, &n);
  GMT_MPI_CHECK(MPI_Allgather(MPI_IN_PLACE, 0, t, h.data(), n, t, c));
  GMT_CHECK("allgather H2D", gmt_rt_memcpy_async(recv, h.data(), bpr * size, s));
  GMT_CHECK("allgather sync", gmt_rt_stream_synchronize(s));
}

class MpiTransport : public Transport {
 protected:
  explicit MpiTransport(MPI_Comm c) : Transport(rank_of(c), size_of(c)), comm_(c) {}
  static int rank_of(MPI_Comm c) {
    int r = 0;
    MPI_Comm_rank(c, &r);
    return r;
  }
  static int size_of(MPI_Comm c) {
    int n = 1;
    MPI_Comm_size(c, &n);
    return n;
  }
  MPI_Comm comm_;
};

// ------------------------------------------------------------------ mpi-host
// Host-staged exchange, pipelined in chunks (reference: the staged path of
// mpi_stencil2d_sycl.cc:248-283 and mpi_stencil2d_gt.cc:147-176,229-252).
//   start: post every receive (one MPI_Irecv per chunk into pinned staging)
//          and enqueue every D2H chunk copy on the caller's stream, an event
//          after each; no host wait, so the caller's kernels queue right away.
//   wait:  send each chunk as soon as its D2H event has completed (MPI keeps
//          the chunks of one message in order: same peer, tag, communicator),
//          and enqueue each received chunk's H2D copy as soon as it lands, so
//          D2H, the wire and H2D of different chunks overlap.
// Receive staging is double-buffered across exchanges: the next exchange's
// receives never wait for this one's H2D copies to drain.
class MpiHostExchange : public Exchange {
 public:
  // pipeline chunk: 1 MiB (GMT_HOST_CHUNK_KB overrides, for measurement)
  static size_t chunk_bytes() {
    const char* e = std::getenv("GMT_HOST_CHUNK_KB");
    const long kb = e ? std::atol(e) : 0;
    return kb > 0 ? static_cast<size_t>(kb) << 10 : size_t(1) << 20;
  }

  MpiHostExchange(MPI_Comm c, std::vector<Msg> r, std::vector<Msg> s)
      : c_(c), recvs_(std::move(r)), sends_(std::move(s)) {
    const size_t kChunk = chunk_bytes();
    for (int set = 0; set < 2; ++set)
      for (auto& m : recvs_) rstage_[set].emplace_back(m.bytes, GMT_SPACE_PINNED);
    for (auto& m : sends_) sstage_.emplace_back(m.bytes, GMT_SPACE_PINNED);
    for (size_t i = 0; i < sends_.size(); ++i)
      for (size_t off = 0; off < sends_[i].bytes || off == 0; off += kChunk) {
        schunks_.push_back({i, off, std::min(kChunk, sends_[i].bytes - off)});
        if (sends_[i].bytes == 0) break;
      }
    for (size_t i = 0; i < recvs_.size(); ++i)
      for (size_t off = 0; off < recvs_[i].bytes || off == 0; off += kChunk) {
        rchunks_.push_back({i, off, std::min(kChunk, recvs_[i].bytes - off)});
        if (recvs_[i].bytes == 0) break;
      }
    events_.resize(schunks_.size(), nullptr);
    for (auto& e : events_) GMT_CHECK("event", gmt_rt_event_create(&e, 0));
    for (auto& e : h2d_done_) GMT_CHECK("event", gmt_rt_event_create(&e, 0));
  }
  ~MpiHostExchange() override {
    for (auto& e : events_) gmt_rt_event_destroy(e);
    for (auto& e : h2d_done_) gmt_rt_event_destroy(e);
  }
  void start(gmt_stream_t s) override {
    cur_ ^= 1;
    // the exchange before last drained this staging set with its H2D copies
    if (armed_[cur_]) GMT_CHECK("staging reuse", gmt_rt_event_synchronize(h2d_done_[cur_]));
    rreqs_.assign(rchunks_.size(), MPI_REQUEST_NULL);
    for (size_t k = 0; k < rchunks_.size(); ++k) {
      const Chunk& ch = rchunks_[k];
      const Msg& m = recvs_[ch.msg];
      irecv(rstage_[cur_][ch.msg].data() + ch.off, ch.len, m.peer, m.tag, c_, &rreqs_[k]);
    }
    for (size_t k = 0; k < schunks_.size(); ++k) {
      const Chunk& ch = schunks_[k];
      const Msg& m = sends_[ch.msg];
      if (ch.len)
        GMT_CHECK("stage D2H", gmt_rt_memcpy_async(sstage_[ch.msg].data() + ch.off,
                                                   static_cast<const char*>(m.buf) + ch.off, ch.len, s));
      GMT_CHECK("event", gmt_rt_event_record(events_[k], s));
    }
  }
  void wait(gmt_stream_t s) override {
    std::vector<MPI_Request> sreqs;
    sreqs.reserve(schunks_.size());
    size_t next = 0, pending = rchunks_.size();
    std::vector<int> idx(rchunks_.size() ? rchunks_.size() : 1);
    auto land = [&](int n) {
      for (int q = 0; q < n; ++q) {
        const Chunk& ch = rchunks_[idx[q]];
        if (ch.len)
          GMT_CHECK("stage H2D", gmt_rt_memcpy_async(static_cast<char*>(recvs_[ch.msg].buf) + ch.off,
                                                     rstage_[cur_][ch.msg].data() + ch.off, ch.len, s));
      }
      pending -= static_cast<size_t>(n);
    };
    auto send = [&](size_t k) {
      const Chunk& ch = schunks_[k];
      const Msg& m = sends_[ch.msg];
      sreqs.emplace_back();
      isend(sstage_[ch.msg].data() + ch.off, ch.len, m.peer, m.tag, c_, &sreqs.back());
    };
    while (next < schunks_.size() || pending > 0) {
      bool progress = false;
      while (next < schunks_.size() && gmt_rt_event_query(events_[next]) == 0) {
        send(next++);
        progress = true;
      }
      if (pending > 0) {
        int n = 0;
        GMT_MPI_CHECK(MPI_Testsome(static_cast<int>(rreqs_.size()), rreqs_.data(), &n, idx.data(),
                                   MPI_STATUSES_IGNORE));
        if (n > 0 && n != MPI_UNDEFINED) {
          land(n);
          progress = true;
        }
      }
      if (progress) continue;
      if (next < schunks_.size()) {  // nothing landed: block on the next D2H chunk
        GMT_CHECK("stage D2H wait", gmt_rt_event_synchronize(events_[next]));
        send(next++);
      } else {  // every chunk is sent: block on the receives
        int n = 0;
        GMT_MPI_CHECK(MPI_Waitsome(static_cast<int>(rreqs_.size()), rreqs_.data(), &n, idx.data(),
                                   MPI_STATUSES_IGNORE));
        if (n > 0 && n != MPI_UNDEFINED) land(n);
      }
    }
    waitall(sreqs, "mpi-host exchange");
    GMT_CHECK("event", gmt_rt_event_record(h2d_done_[cur_], s));
    armed_[cur_] = true;
  }

 private:
  struct Chunk {
    size_t msg, off, len;
  };
  MPI_Comm c_;
  std::vector<Msg> recvs_, sends_;
  std::vector<Buffer<char>> rstage_[2], sstage_;
  std::vector<Chunk> schunks_, rchunks_;
  std::vector<gmt_event_t> events_;
  std::vector<MPI_Request> rreqs_;
  gmt_event_t h2d_done_[2] = {nullptr, nullptr};
  bool armed_[2] = {false, false};
  int cur_ = 1;
};

class MpiHostTransport : public MpiTransport {
 public:
  explicit MpiHostTransport(MPI_Comm c) : MpiTransport(c) {}
  Kind kind() const override { return Kind::MpiHost; }
  const char* name() const override { return "mpi-host"; }
  std::unique_ptr<Exchange> plan(const std::vector<Msg>& r, const std::vector<Msg>& s) override {
    return std::make_unique<MpiHostExchange>(comm_, r, s);
  }
  void allreduce_sum(double* buf, size_t n, gmt_stream_t s) override {
    staged_allreduce(comm_, buf, n, s);
  }
  void allgather(const void* send, void* recv, size_t bpr, gmt_stream_t s) override {
    staged_allgather(comm_, rank_, size_, send, recv, bpr, s);
  }
};

// ---------------------------------------------------------------- mpi-direct
// mpi-direct hands the buffers straight to MPI.  Device memory is legal only
// with a GPU-aware MPI: refuse it otherwise, instead of letting a host-only
// MPI (MPICH ch3 here) read device addresses as host memory.  Managed and
// host memory always pass (MPI can read them).
void require_mpi_readable(const void* p, const char* what) {
  if (p == nullptr || gmt_rt_backend() == GMT_BACKEND_HOST) return;
  int space = GMT_SPACE_UNREGISTERED;
  if (gmt_rt_pointer_space(p, &space) != 0 || space != GMT_SPACE_DEVICE || mpi_gpu_aware()) return;
  std::printf("ERROR: transport mpi-direct was given device memory (%s), but this MPI is not GPU-aware "
              "(%s). Use --transport=mpi-host, rccl or ipc, or set GMT_MPI_GPU_AWARE=1 if the MPI "
              "library can read device memory.\n",
              what, mpi_gpu_aware_source());
  std::fflush(stdout);
  abort_job(EXIT_FAILURE);
}

class MpiDirectExchange : public Exchange {
 public:
  MpiDirectExchange(MPI_Comm c, std::vector<Msg> r, std::vector<Msg> s)
      : c_(c), recvs_(std::move(r)), sends_(std::move(s)) {
    for (auto& m : recvs_) require_mpi_readable(m.buf, "halo receive buffer");
    for (auto& m : sends_) require_mpi_readable(m.buf, "halo send buffer");
  }
  void start(gmt_stream_t s) override {
    // one sync covers both "send data produced" and "earlier readers of the
    // ghost cells are done" before MPI may write them
    GMT_CHECK("direct sync", gmt_rt_stream_synchronize(s));
    for (auto& m : recvs_) {
      reqs_.emplace_back();
      irecv(m.buf, m.bytes, m.peer, m.tag, c_, &reqs_.back());
    }
    for (auto& m : sends_) {
      reqs_.emplace_back();
      isend(m.buf, m.bytes, m.peer, m.tag, c_, &reqs_.back());
    }
  }
  void wait(gmt_stream_t) override { waitall(reqs_, "mpi-direct exchange"); }

 private:
  MPI_Comm c_;
  std::vector<Msg> recvs_, sends_;
  std::vector<MPI_Request> reqs_;
};

class MpiDirectTransport : public MpiTransport {
 public:
  explicit MpiDirectTransport(MPI_Comm c) : MpiTransport(c) {}
  Kind kind() const override { return Kind::MpiDirect; }
  const char* name() const override { return "mpi-direct"; }
  std::unique_ptr<Exchange> plan(const std::vector<Msg>& r, const std::vector<Msg>& s) override {
    return std::make_unique<MpiDirectExchange>(comm_, r, s);
  }
  void allreduce_sum(double* buf, size_t n, gmt_stream_t s) override {
    require_mpi_readable(buf, "all-reduce buffer");
    GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
    GMT_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, buf, static_cast<int>(n), MPI_DOUBLE, MPI_SUM, comm_));
  }
  void allgather(const void* send, void* recv, size_t bpr, gmt_stream_t s) override {
    require_mpi_readable(send, "all-gather send buffer");
    require_mpi_readable(recv, "all-gather receive buffer");
    GMT_CHECK("allgather sync", gmt_rt_stream_synchronize(s));
    MPI_Datatype t;
    int n;
    mpi_count(bpr, &t, &n);
    const bool inplace = send == static_cast<const char*>(recv) + rank_ * bpr;
    GMT_MPI_CHECK(MPI_Allgather(inplace ? MPI_IN_PLACE : send, inplace ? 0 : n, t, recv, n, t, comm_));
  }
};

// ----------------------------------------------------------------------- ipc
// handle-exchange tags: one offset per wire kind, so a pair of ranks that
// exchange messages with the same tag in both directions cannot mismatch them
constexpr int kStageTag = 10000, kFlagTag = 20000, kReadyTag = 30000;

struct IpcWire {
  gmt_ipc_handle h;
  uint64_t offset;
};

// hipIpcOpenMemHandle maps an allocation once per process: cache by handle.
class IpcCache {
 public:
  void* open(const gmt_ipc_handle& h) {
    std::string k(reinterpret_cast<const char*>(h.bytes), sizeof(h.bytes));
    auto it = map_.find(k);
    if (it != map_.end()) {
      ++it->second.refs;
      return it->second.base;
    }
    void* base = nullptr;
    GMT_CHECK("ipc open", gmt_rt_ipc_open(&base, &h));
    map_[k] = {base, 1};
    return base;
  }
  void close(void* base) {
    for (auto it = map_.begin(); it != map_.end(); ++it)
      if (it->second.base == base && --it->second.refs == 0) {
        GMT_WARN("ipc close", gmt_rt_ipc_close(base));
        map_.erase(it);
        return;
      }
  }

 private:
  struct E {
    void* base;
    int refs;
  };
  std::map<std::string, E> map_;
};

// Stream-ordered exchange over IPC-mapped memory (csrc/kernels/ipc.hip has
// the protocol).  Every send message gets two staging slots in the sender's
// memory; the receiver pulls the current slot once the sender's "ready" flag
// (in the receiver's flag memory) reaches the exchange's epoch, then marks the
// slot consumed (in the sender's flag memory).  start() and wait() are one
// kernel launch each on the caller's stream: no host synchronisation, no MPI
// traffic after construction, so the exchange can be captured into a graph.
// Several ranks may share a GPU (the IPC mappings are then same-device).
class IpcExchange : public Exchange {
 public:
  IpcExchange(MPI_Comm c, int rank, IpcCache* cache, std::vector<Msg> r, std::vector<Msg> s)
      : c_(c), rank_(rank), cache_(cache), recvs_(std::move(r)), sends_(std::move(s)) {
    const size_t nr = recvs_.size(), ns = sends_.size();
    // flags: ready[j] per receive (written by its sender), consumed[i] per send
    // (written by its receiver); control: epoch, 2 launch counters, error word
    flags_ = Buffer<uint64_t>(nr + ns + 1, GMT_SPACE_FLAGS);
    ctl_ = Buffer<uint64_t>(4, GMT_SPACE_DEVICE);  // epoch | 3 x u32 counters + u32 error
    GMT_CHECK("ipc ctl", gmt_rt_memset_async(ctl_.data(), 0, ctl_.bytes(), nullptr));
    GMT_CHECK("ipc ctl", gmt_rt_stream_synchronize(nullptr));
    for (auto& m : sends_) stage_.emplace_back(2 * (m.bytes ? m.bytes : 1), GMT_SPACE_DEVICE);

    // wiring: the receiver of send i learns {its staging, its consumed flag};
    // the sender of receive j learns {its ready flag}
    auto wire = [](void* p) {
      IpcWire w;
      size_t off = 0;
      GMT_CHECK("ipc get handle", gmt_rt_ipc_get_handle(&w.h, &off, p));
      w.offset = off;
      return w;
    };
    std::vector<IpcWire> out_stage(ns), out_cflag(ns), out_rflag(nr), in_stage(nr), in_cflag(nr), in_rflag(ns);
    std::vector<MPI_Request> reqs;
    for (size_t j = 0; j < nr; ++j) {
      if (recvs_[j].peer == rank_) continue;
      reqs.emplace_back();
      GMT_MPI_CHECK(MPI_Irecv(&in_stage[j], sizeof(IpcWire), MPI_BYTE, recvs_[j].peer, recvs_[j].tag + kStageTag,
                              c_, &reqs.back()));
      reqs.emplace_back();
      GMT_MPI_CHECK(MPI_Irecv(&in_cflag[j], sizeof(IpcWire), MPI_BYTE, recvs_[j].peer, recvs_[j].tag + kFlagTag,
                              c_, &reqs.back()));
      out_rflag[j] = wire(flags_.data() + j);
      reqs.emplace_back();
      GMT_MPI_CHECK(MPI_Isend(&out_rflag[j], sizeof(IpcWire), MPI_BYTE, recvs_[j].peer, recvs_[j].tag + kReadyTag,
                              c_, &reqs.back()));
    }
    for (size_t i = 0; i < ns; ++i) {
      if (sends_[i].peer == rank_) continue;
      reqs.emplace_back();
      GMT_MPI_CHECK(MPI_Irecv(&in_rflag[i], sizeof(IpcWire), MPI_BYTE, sends_[i].peer, sends_[i].tag + kReadyTag,
                              c_, &reqs.back()));
      out_stage[i] = wire(stage_[i].data());
      out_cflag[i] = wire(flags_.data() + nr + i);
      reqs.emplace_back();
      GMT_MPI_CHECK(MPI_Isend(&out_stage[i], sizeof(IpcWire), MPI_BYTE, sends_[i].peer, sends_[i].tag + kStageTag,
                              c_, &reqs.back()));
      reqs.emplace_back();
      GMT_MPI_CHECK(MPI_Isend(&out_cflag[i], sizeof(IpcWire), MPI_BYTE, sends_[i].peer, sends_[i].tag + kFlagTag,
                              c_, &reqs.back()));
    }
    waitall(reqs, "ipc handle exchange");
    auto open = [&](const IpcWire& w) {
      void* base = cache_->open(w.h);
      opened_.push_back(base);
      return static_cast<char*>(base) + w.offset;
    };
    // self messages (periodic single rank): the matching local buffers
    auto self_send = [&](int tag) -> int {
      for (size_t i = 0; i < ns; ++i)
        if (sends_[i].peer == rank_ && sends_[i].tag == tag) return static_cast<int>(i);
      std::printf("ipc: no self-send for tag %d\n", tag);
      abort_job(2);
    };
    auto self_recv = [&](int tag) -> int {
      for (size_t j = 0; j < nr; ++j)
        if (recvs_[j].peer == rank_ && recvs_[j].tag == tag) return static_cast<int>(j);
      std::printf("ipc: no self-receive for tag %d\n", tag);
      abort_job(2);
    };
    for (size_t i = 0; i < ns; ++i) {
      const Msg& m = sends_[i];
      gmt_ipc_chan ch{};
      ch.src = m.buf;
      ch.dst = stage_[i].data();
      ch.bytes = static_cast<int64_t>(m.bytes);
      ch.dst_stride = static_cast<int64_t>(m.bytes ? m.bytes : 1);
      ch.wait = flags_.data() + nr + i;  // the receiver has consumed slot e & 1 (exchange e - 2)
      ch.signal = m.peer == rank_ ? flags_.data() + self_recv(m.tag)
                                  : reinterpret_cast<uint64_t*>(open(in_rflag[i]));
      send_.push_back(ch);
    }
    for (size_t j = 0; j < nr; ++j) {
      const Msg& m = recvs_[j];
      gmt_ipc_chan ch{};
      if (m.peer == rank_) {
        const int i = self_send(m.tag);
        ch.src = stage_[i].data();
        ch.signal = flags_.data() + nr + i;
      } else {
        ch.src = open(in_stage[j]);
        ch.signal = reinterpret_cast<uint64_t*>(open(in_cflag[j]));
      }
      ch.src_stride = static_cast<int64_t>(m.bytes ? m.bytes : 1);
      ch.dst = m.buf;
      ch.bytes = static_cast<int64_t>(m.bytes);
      ch.wait = flags_.data() + j;  // the sender's slot for this exchange is ready
      recv_.push_back(ch);
    }
    if (send_.size() > GMT_IPC_MAX_CHAN || recv_.size() > GMT_IPC_MAX_CHAN) {
      std::printf("ipc: %zu sends / %zu receives exceed %d channels per launch\n", send_.size(), recv_.size(),
                  GMT_IPC_MAX_CHAN);
      abort_job(2);
    }
  }
  ~IpcExchange() override {
    for (void* b : opened_) cache_->close(b);
  }
  // one launch per exchange (send and receive channels in the same grid)
  void start(gmt_stream_t s) override {
    if (send_.empty() && recv_.empty()) return;
    GMT_CHECK("ipc exchange", gmt_ipc_exchange(static_cast<int>(send_.size()), send_.data(),
                                               static_cast<int>(recv_.size()), recv_.data(), epoch(), counters(),
                                               err(), s));
  }
  void wait(gmt_stream_t) override {}  // stream order: the launch in start() completes first
  bool graph_capturable() const override { return true; }

 private:
  uint64_t* epoch() { return ctl_.data(); }
  unsigned* counters() { return reinterpret_cast<unsigned*>(ctl_.data() + 1); }  // 3 words
  unsigned* err() { return reinterpret_cast<unsigned*>(ctl_.data() + 3); }

  MPI_Comm c_;
  int rank_;
  IpcCache* cache_;
  std::vector<Msg> recvs_, sends_;
  Buffer<uint64_t> flags_, ctl_;
  std::vector<Buffer<char>> stage_;
  std::vector<gmt_ipc_chan> send_, recv_;
  std::vector<void*> opened_;
};

class IpcTransport : public MpiTransport {
 public:
  explicit IpcTransport(MPI_Comm c) : MpiTransport(c) {}
  ~IpcTransport() override { gathers_.clear(); }
  Kind kind() const override { return Kind::Ipc; }
  const char* name() const override { return "ipc"; }
  std::unique_ptr<Exchange> plan(const std::vector<Msg>& r, const std::vector<Msg>& s) override {
    return std::make_unique<IpcExchange>(comm_, rank_, &cache_, r, s);
  }
  void allreduce_sum(double* buf, size_t n, gmt_stream_t s) override {
    staged_allreduce(comm_, buf, n, s);
  }
  // All-gather as one persistent IPC exchange: every rank writes its block
  // straight into every peer's receive buffer.  Plans are cached per
  // (send, recv, size) so the handle exchange happens once per buffer set.
  void allgather(const void* send, void* recv, size_t bpr, gmt_stream_t s) override {
    char* r = static_cast<char*>(recv);
    if (send != r + rank_ * bpr)
      GMT_CHECK("gather self", gmt_rt_memcpy_async(r + rank_ * bpr, send, bpr, s));
    if (size_ == 1) return;
    const auto key = std::make_tuple(send, recv, bpr);
    auto it = gathers_.find(key);
    if (it == gathers_.end()) {
      std::vector<Msg> recvs, sends;
      for (int p = 0; p < size_; ++p) {
        if (p == rank_) continue;
        recvs.push_back({r + p * bpr, bpr, p, kGatherTag});
        sends.push_back({const_cast<void*>(send), bpr, p, kGatherTag});
      }
      it = gathers_.emplace(key, plan(recvs, sends)).first;
    }
    it->second->run(s);
  }

 private:
  static constexpr int kGatherTag = 777;
  IpcCache cache_;
  std::map<std::tuple<const void*, void*, size_t>, std::unique_ptr<Exchange>> gathers_;
};

}  // namespace

Kind parse_kind(const std::string& s) {
  if (s == "auto" || s.empty()) return Kind::Auto;
  if (s == "mpi-host" || s == "host" || s == "staged") return Kind::MpiHost;
  if (s == "mpi-direct" || s == "direct" || s == "mpi") return Kind::MpiDirect;
  if (s == "rccl" || s == "nccl") return Kind::Rccl;
  if (s == "ipc" || s == "hip-ipc") return Kind::Ipc;
  if (s == "local") return Kind::Local;
  std::printf("ERROR: unknown transport '%s' (auto|mpi-host|mpi-direct|rccl|ipc)\n", s.c_str());
  abort_job(EXIT_FAILURE);
}

// GMT_MPI_GPU_AWARE=1/0 decides when set; otherwise the MPI library is asked
// through MPIX_Query_rocm_support (MPICH >= 4.1, Open MPI >= 5.0), looked up
// with dlsym so the apps link against any MPI.  Neither: not GPU-aware.
namespace {
int query_rocm_support() {  // 1 / 0, or -1 when the library has no such query
  using Query = int (*)(void);
  void* sym = dlsym(RTLD_DEFAULT, "MPIX_Query_rocm_support");
  return sym ? (reinterpret_cast<Query>(sym)() != 0 ? 1 : 0) : -1;
}
}  // namespace

bool mpi_gpu_aware() {
  const char* e = std::getenv("GMT_MPI_GPU_AWARE");
  if (e && e[0]) return e[0] == '1';
  return query_rocm_support() == 1;
}

const char* mpi_gpu_aware_source() {
  const char* e = std::getenv("GMT_MPI_GPU_AWARE");
  if (e && e[0]) return e[0] == '1' ? "GMT_MPI_GPU_AWARE=1" : "GMT_MPI_GPU_AWARE=0";
  switch (query_rocm_support()) {
    case 1: return "MPIX_Query_rocm_support() = 1";
    case 0: return "MPIX_Query_rocm_support() = 0";
    default: return "no MPIX_Query_rocm_support in this MPI, GMT_MPI_GPU_AWARE unset";
  }
}

Kind resolve(Kind k, const RankBinding& b, bool buffers_managed) {
  if (const char* e = std::getenv("GMT_TRANSPORT")) {
    if (k == Kind::Auto) k = parse_kind(e);
  }
  if (k != Kind::Auto) return k;
  if (gmt_rt_backend() == GMT_BACKEND_HOST || buffers_managed || mpi_gpu_aware())
    return Kind::MpiDirect;
  if (gmt_ccl_available() && b.ranks_per_device == 1) return Kind::Rccl;
  return Kind::Ipc;
}

std::unique_ptr<Transport> make_transport(Kind k, MPI_Comm comm, const RankBinding& b) {
  switch (resolve(k, b)) {
    case Kind::MpiHost: return std::make_unique<MpiHostTransport>(comm);
    case Kind::MpiDirect: return std::make_unique<MpiDirectTransport>(comm);
    case Kind::Rccl: {
      if (!gmt_ccl_available() && !gmt_ccl_emulated()) {
        std::printf("ERROR: transport rccl requested but this build has no RCCL (%s backend)\n",
                    gmt_rt_backend_name());
        abort_job(EXIT_FAILURE);
      }
      int worst = b.ranks_per_device;
      MPI_Allreduce(MPI_IN_PLACE, &worst, 1, MPI_INT, MPI_MAX, comm);
      if (worst > 1 && !gmt_ccl_emulated()) {  // the host emulation has no devices to share
        std::printf("ERROR: transport rccl needs one rank per GPU (%d ranks share a GPU); "
                    "use --transport=ipc or mpi-host\n", worst);
        abort_job(EXIT_FAILURE);
      }
      int rank = 0, size = 1;
      MPI_Comm_rank(comm, &rank);
      MPI_Comm_size(comm, &size);
      gmt_ccl_id id;
      std::memset(&id, 0, sizeof(id));
      if (rank == 0) GMT_CCL_CHECK("unique id", gmt_ccl_get_unique_id(&id));
      GMT_MPI_CHECK(MPI_Bcast(&id, sizeof(id), MPI_BYTE, 0, comm));
      return make_rccl_transport(rank, size, id);
    }
    case Kind::Ipc: return std::make_unique<IpcTransport>(comm);
    case Kind::Local: return make_local_transport();
    default: break;
  }
  abort_job(EXIT_FAILURE);
}

}  // namespace comm
}  // namespace gmt
