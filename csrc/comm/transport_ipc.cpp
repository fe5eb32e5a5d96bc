// The ipc transport (gmt/transport.hpp) over any host control plane
// (gmt/control.hpp): MPI in the native apps, the socket mesh in the MPI-free
// engine library.  The control plane carries only the one-time handle
// exchange and the host-staged collectives; every halo exchange is one
// stream-ordered kernel launch (csrc/kernels/ipc.hip).
//
// Reference: the reference exchanges device pointers through GPU-aware MPI
// (mpi_stencil2d_gt.cc:179-225) and runs several ranks per GPU by
// oversubscription (mpi_daxpy.cc:43-54); the same-GPU and peer-GPU direct
// path here is HIP IPC.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>

#include "gmt/buffer.hpp"
#include "gmt/control.hpp"
#include "gmt/transport.hpp"

namespace gmt {
namespace comm {

namespace {

// handle-exchange tags: one offset per wire kind, so a pair of ranks that
// exchange messages with the same tag in both directions cannot mismatch them
constexpr int kStageTag = 10000, kFlagTag = 20000, kReadyTag = 30000;

struct IpcWire {
  gmt_ipc_handle h;
  uint64_t offset;
  // the message's byte count on the side that sends this wire: both sides
  // of a message must agree (a rank whose environment picked another face
  // layout, e.g. GMT_IPC_BLOCKS, would otherwise read past the sender's
  // staging slot or fill ghost cells with the wrong bytes)
  uint64_t bytes;
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
// slot consumed (in the sender's flag memory).  start() is one kernel launch
// on the caller's stream: no host synchronisation, no control-plane traffic
// after construction, so the exchange can be captured into a graph.  Several
// ranks may share a GPU (the IPC mappings are then same-device).
class IpcExchange : public Exchange {
 public:
  IpcExchange(Control& ctl, IpcCache* cache, std::vector<Msg> r, std::vector<Msg> s)
      : rank_(ctl.rank()), cache_(cache), recvs_(std::move(r)), sends_(std::move(s)) {
    const size_t nr = recvs_.size(), ns = sends_.size();
    // flags: ready[j] per receive (written by its sender), consumed[i] per send
    // (written by its receiver); control: epoch, 3 launch counters
    flags_ = Buffer<uint64_t>(nr + ns + 1, GMT_SPACE_FLAGS);
    ctl_ = Buffer<uint64_t>(3, GMT_SPACE_DEVICE);  // epoch | 3 x u32 counters
    err_ = Buffer<unsigned>(1, GMT_SPACE_PINNED);
    *err_.data() = 0;
    GMT_CHECK("ipc ctl", gmt_rt_memset_async(ctl_.data(), 0, ctl_.bytes(), nullptr));
    GMT_CHECK("ipc ctl", gmt_rt_stream_synchronize(nullptr));
    for (auto& m : sends_) stage_.emplace_back(2 * (m.bytes ? m.bytes : 1), GMT_SPACE_DEVICE);

    // wiring: the receiver of send i learns {its staging, its consumed flag};
    // the sender of receive j learns {its ready flag}
    auto wire = [](void* p, size_t bytes) {
      IpcWire w;
      std::memset(&w, 0, sizeof(w));
      size_t off = 0;
      GMT_CHECK("ipc get handle", gmt_rt_ipc_get_handle(&w.h, &off, p));
      w.offset = off;
      w.bytes = bytes;
      return w;
    };
    std::vector<IpcWire> out_stage(ns), out_cflag(ns), out_rflag(nr), in_stage(nr), in_cflag(nr), in_rflag(ns);
    std::vector<HostMsg> hr, hs;
    for (size_t j = 0; j < nr; ++j) {
      const Msg& m = recvs_[j];
      if (m.peer == rank_) continue;
      hr.push_back({&in_stage[j], sizeof(IpcWire), m.peer, m.tag + kStageTag});
      hr.push_back({&in_cflag[j], sizeof(IpcWire), m.peer, m.tag + kFlagTag});
      out_rflag[j] = wire(flags_.data() + j, m.bytes);
      hs.push_back({&out_rflag[j], sizeof(IpcWire), m.peer, m.tag + kReadyTag});
    }
    for (size_t i = 0; i < ns; ++i) {
      const Msg& m = sends_[i];
      if (m.peer == rank_) continue;
      hr.push_back({&in_rflag[i], sizeof(IpcWire), m.peer, m.tag + kReadyTag});
      out_stage[i] = wire(stage_[i].data(), m.bytes);
      out_cflag[i] = wire(flags_.data() + nr + i, m.bytes);
      hs.push_back({&out_stage[i], sizeof(IpcWire), m.peer, m.tag + kStageTag});
      hs.push_back({&out_cflag[i], sizeof(IpcWire), m.peer, m.tag + kFlagTag});
    }
    ctl.exchange(hr, hs);
    auto agree = [&](const Msg& m, uint64_t peer_bytes, const char* what) {
      if (peer_bytes == m.bytes) return;
      std::fprintf(stderr, "ipc: rank %d %s %zu bytes (tag %d) but rank %d's side of that message has %llu bytes; "
                  "the ranks disagree on the face layout (GMT_IPC_BLOCKS must match on every rank)\n",
                  rank_, what, m.bytes, m.tag, m.peer, static_cast<unsigned long long>(peer_bytes));
      abort_job(2);
    };
    for (size_t j = 0; j < nr; ++j)
      if (recvs_[j].peer != rank_) agree(recvs_[j], in_stage[j].bytes, "receives");
    for (size_t i = 0; i < ns; ++i)
      if (sends_[i].peer != rank_) agree(sends_[i], in_rflag[i].bytes, "sends");
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
    std::vector<gmt_ipc_chan> send(ns), recv(nr);
    for (size_t i = 0; i < ns; ++i) {
      const Msg& m = sends_[i];
      gmt_ipc_chan& ch = send[i];
      ch.src = m.buf;
      if (m.block.base) {  // a halo face read in place: runs of block.rows doubles
        ch.src = m.block.base;
        ch.src_run = static_cast<int64_t>(m.block.rows * sizeof(double));
        ch.src_ld = static_cast<int64_t>(m.block.ld * sizeof(double));
      }
      ch.dst = stage_[i].data();
      ch.bytes = static_cast<int64_t>(m.bytes);
      ch.src_stride = 0;
      ch.dst_stride = static_cast<int64_t>(m.bytes ? m.bytes : 1);
      ch.wait = flags_.data() + nr + i;  // the receiver has consumed slot e & 1 (exchange e - 2)
      ch.signal = m.peer == rank_ ? flags_.data() + self_recv(m.tag)
                                  : reinterpret_cast<uint64_t*>(open(in_rflag[i]));
    }
    for (size_t j = 0; j < nr; ++j) {
      const Msg& m = recvs_[j];
      gmt_ipc_chan& ch = recv[j];
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
      if (m.block.base) {  // straight into the ghost cells
        ch.dst = m.block.base;
        ch.dst_run = static_cast<int64_t>(m.block.rows * sizeof(double));
        ch.dst_ld = static_cast<int64_t>(m.block.ld * sizeof(double));
      }
      ch.dst_stride = 0;
      ch.bytes = static_cast<int64_t>(m.bytes);
      ch.wait = flags_.data() + j;  // the sender's slot for this exchange is ready
    }
    if (ns + nr == 0) return;
    table_ = Buffer<char>(static_cast<size_t>(gmt_ipc_table_bytes(static_cast<int>(ns + nr))), GMT_SPACE_DEVICE);
    plan_.table = table_.data();
    plan_.epoch = ctl_.data();
    plan_.counters = reinterpret_cast<unsigned*>(ctl_.data() + 1);
    plan_.err = err_.data();
    GMT_CHECK("ipc plan", gmt_ipc_plan_init(&plan_, static_cast<int>(ns), send.data(), static_cast<int>(nr),
                                            recv.data()));
  }
  ~IpcExchange() override {
    for (void* b : opened_) cache_->close(b);
  }
  void start(gmt_stream_t s) override {
    if (sends_.empty() && recvs_.empty()) return;
    GMT_CHECK("ipc exchange", gmt_ipc_exchange(&plan_, s));
  }
  void wait(gmt_stream_t) override {}  // stream order: the launch in start() completes first
  bool graph_capturable() const override { return true; }
  bool ok(std::string* why) const override {
    const unsigned e = err_.data() ? __atomic_load_n(err_.data(), __ATOMIC_ACQUIRE) : 0u;
    if (e == 0) return true;
    if (why) {
      const size_t k = e - 1, ns = sends_.size();
      const bool is_send = k < ns;
      const Msg* m = is_send ? &sends_[k] : (k - ns < recvs_.size() ? &recvs_[k - ns] : nullptr);
      char buf[256];
      std::snprintf(buf, sizeof(buf),
                    "ipc exchange on rank %d: the %s of %zu bytes %s rank %d (tag %d) timed out waiting for "
                    "the peer (GMT_WAIT_TIMEOUT_MS); ghost cells are stale",
                    rank_, is_send ? "send" : "receive", m ? m->bytes : size_t(0), is_send ? "to" : "from",
                    m ? m->peer : -1, m ? m->tag : -1);
      *why = buf;
    }
    return false;
  }

 private:
  int rank_;
  IpcCache* cache_;
  std::vector<Msg> recvs_, sends_;
  Buffer<uint64_t> flags_, ctl_;
  Buffer<unsigned> err_;
  Buffer<char> table_;
  std::vector<Buffer<char>> stage_;
  std::vector<void*> opened_;
  gmt_ipc_plan plan_{};
};

class IpcTransport : public Transport {
 public:
  IpcTransport(std::unique_ptr<Control> owned, Control* ctl)
      : Transport(ctl->rank(), ctl->size()), owned_(std::move(owned)), ctl_(ctl) {}
  ~IpcTransport() override {
    gathers_.clear();
    gbuf_.clear();
  }
  Kind kind() const override { return Kind::Ipc; }
  const char* name() const override { return "ipc"; }
  // halo faces move in place: the sender's exchange kernel gathers a strided
  // face straight into its staging slot and the receiver's scatters it
  // straight into the ghost cells (no pack / unpack launches, one pass over
  // the data fewer on each side); GMT_IPC_BLOCKS=0 packs them, for A/B
  bool takes_blocks() const override {
    const char* e = std::getenv("GMT_IPC_BLOCKS");
    return !(e && e[0] == '0');
  }
  std::unique_ptr<Exchange> plan(const std::vector<Msg>& r, const std::vector<Msg>& s) override {
    return std::make_unique<IpcExchange>(*ctl_, &cache_, r, s);
  }
  // All-reduce = the IPC all-gather of every rank's vector into a gather
  // buffer (one exchange kernel), then one kernel reducing the slices in
  // rank order: stream-ordered, no host round trip, the same bits on every
  // rank.  Vectors above kDeviceReduceMax bytes go host-staged (one
  // persistent pinned buffer, the control plane's rank-ordered reduction).
  void allreduce_sum(double* buf, size_t n, gmt_stream_t s) override { reduce(buf, n, s, false); }
  void allreduce_max(double* buf, size_t n, gmt_stream_t s) override { reduce(buf, n, s, true); }
  void reduce(double* buf, size_t n, gmt_stream_t s, bool max) {
    if (size_ == 1 || n == 0) return;
    if (n * sizeof(double) > kDeviceReduceMax) return staged(buf, n, s, max);
    // transport-owned buffers keyed by the length only (the same key on every
    // rank, whatever the caller's pointers): the gather plan is created once
    // per length, collectively
    auto it = gbuf_.find(n);
    if (it == gbuf_.end()) it = gbuf_.emplace(n, Buffer<double>(n * (size_ + 1), GMT_SPACE_DEVICE)).first;
    double* g = it->second.data();
    double* mine = g + n * size_;
    GMT_CHECK("allreduce copy", gmt_rt_memcpy_async(mine, buf, n * sizeof(double), s));
    allgather(mine, g, n * sizeof(double), s);
    GMT_CHECK("slices reduce", gmt_slices_reduce(max ? 1 : 0, static_cast<int64_t>(n), size_, g, buf, s));
  }
  void staged(double* buf, size_t n, gmt_stream_t s, bool max) {
    if (size_ == 1) return;
    double* h = stage(n * sizeof(double));
    GMT_CHECK("allreduce D2H", gmt_rt_memcpy_async(h, buf, n * sizeof(double), s));
    GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
    if (max)
      ctl_->allreduce_max(h, n);
    else
      ctl_->allreduce_sum(h, n);
    GMT_CHECK("allreduce H2D", gmt_rt_memcpy_async(buf, h, n * sizeof(double), s));
    // the pinned buffer is reused by the next call: the copy must have read it
    GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
  }
  // All-gather as one persistent IPC exchange: every rank's block goes
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
  bool ok(std::string* why) const override {
    for (auto& g : gathers_)
      if (!g.second->ok(why)) return false;
    return true;
  }
  Control* control() override { return ctl_; }

 private:
  double* stage(size_t bytes) {
    if (staging_.bytes() < bytes) staging_ = Buffer<char>(bytes, GMT_SPACE_PINNED);
    return reinterpret_cast<double*>(staging_.data());
  }
  static constexpr int kGatherTag = 777;
  static constexpr size_t kDeviceReduceMax = size_t(1) << 20;  // 1 MiB vectors
  std::map<size_t, Buffer<double>> gbuf_;  // per length: size_ gathered slices + this rank's copy
  std::unique_ptr<Control> owned_;
  Control* ctl_;
  IpcCache cache_;
  Buffer<char> staging_;
  std::map<std::tuple<const void*, void*, size_t>, std::unique_ptr<Exchange>> gathers_;
};

}  // namespace

std::unique_ptr<Transport> make_ipc_transport(std::unique_ptr<Control> ctl) {
  Control* c = ctl.get();
  return std::make_unique<IpcTransport>(std::move(ctl), c);
}

std::unique_ptr<Transport> make_ipc_transport(Control& ctl) {
  return std::make_unique<IpcTransport>(nullptr, &ctl);
}

}  // namespace comm
}  // namespace gmt
