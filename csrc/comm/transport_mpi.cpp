// MPI-based transports: mpi-host, mpi-direct, ipc, and the factory that
// bootstraps rccl over MPI (gmt/comm.hpp, gmt/transport.hpp).
#include <dlfcn.h>
#include <sched.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>

#include "gmt/buffer.hpp"
#include "gmt/watchdog.hpp"
#include "gmt/comm.hpp"
#include "gmt/control.hpp"
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

// Host-staged collectives of the mpi-host transport, through one persistent
// pinned buffer (grown on demand; allocating pinned memory per call costs a
// hipHostMalloc/hipHostFree pair, far more than an 8 KiB all-reduce).
class Staging {
 public:
  char* get(size_t bytes) {
    if (buf_.bytes() < bytes) buf_ = Buffer<char>(bytes, GMT_SPACE_PINNED);
    return buf_.data();
  }

 private:
  Buffer<char> buf_;
};

void staged_allreduce(Staging& st, MPI_Comm c, double* buf, size_t n, gmt_stream_t s, MPI_Op op = MPI_SUM) {
  double* h = reinterpret_cast<double*>(st.get(n * sizeof(double)));
  GMT_CHECK("allreduce D2H", gmt_rt_memcpy_async(h, buf, n * sizeof(double), s));
  GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
  GMT_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, h, static_cast<int>(n), MPI_DOUBLE, op, c));
  GMT_CHECK("allreduce H2D", gmt_rt_memcpy_async(buf, h, n * sizeof(double), s));
  GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));  // the staging is reused next call
}
void staged_allgather(Staging& st, MPI_Comm c, int rank, int size, const void* send, void* recv, size_t bpr,
                      gmt_stream_t s) {
  char* h = st.get(bpr * size);
  GMT_CHECK("allgather D2H", gmt_rt_memcpy_async(h + rank * bpr, send, bpr, s));
  GMT_CHECK("allgather sync", gmt_rt_stream_synchronize(s));
  MPI_Datatype t;
  int n;
  mpi_count(bpr, &t, &n);
  GMT_MPI_CHECK(MPI_Allgather(MPI_IN_PLACE, 0, t, h, n, t, c));
  GMT_CHECK("allgather H2D", gmt_rt_memcpy_async(recv, h, bpr * size, s));
  GMT_CHECK("allgather sync", gmt_rt_stream_synchronize(s));
}

class MpiTransport : public Transport {
 public:
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

 protected:
  explicit MpiTransport(MPI_Comm c) : Transport(rank_of(c), size_of(c)), comm_(c) {}
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
//          D2H, the wire and H2D of different chunks overlap.  Flat chunks'
//          copies run on a stream of their own (8 MiB, ranks bound: 15.8 ->
//          20 GB/s per rank); field-block scatter kernels stay on the caller's
//          stream (on a second stream they took mpi_stencil2d_sycl from 1.3 to
//          1.9 ms: profiles/r05_xport/).
// Receive staging is double-buffered across exchanges: the next exchange's
// receives never wait for this one's H2D copies to drain.
// Device -> host leg (GMT_HOST_STAGE): "kernel" (default) — one gmt_stage_copy
// launch writes every chunk into coherent pinned memory with the CUs and
// raises a per-chunk host flag (csrc/kernels/stage.hip); "sdma" — one
// hipMemcpyAsync and one event per chunk (round 2).
class MpiHostExchange : public Exchange {
 public:
  // pipeline chunk: 1 MiB (GMT_HOST_CHUNK_KB overrides, for measurement);
  // the transport agrees on one value across ranks (receives are posted per
  // chunk, so the two sides of a message must cut it the same way)
  static size_t chunk_bytes() {
    const char* e = std::getenv("GMT_HOST_CHUNK_KB");
    const long kb = e ? std::atol(e) : 0;
    return kb > 0 ? static_cast<size_t>(kb) << 10 : size_t(1) << 20;
  }

  static bool kernel_staging() {
    const char* e = std::getenv("GMT_HOST_STAGE");
    return !(e && std::strcmp(e, "sdma") == 0);
  }

  MpiHostExchange(MPI_Comm c, size_t chunk, std::vector<Msg> r, std::vector<Msg> s)
      : c_(c), recvs_(std::move(r)), sends_(std::move(s)), kernel_(kernel_staging()) {
    const size_t kChunk = chunk;
    for (auto& m : sends_)
      if (m.block.base && !kernel_) {
        std::printf("mpi-host: a field block message needs kernel staging (GMT_HOST_STAGE=sdma given)\n");
        abort_job(EXIT_FAILURE);
      }
    for (int set = 0; set < 2; ++set)
      for (auto& m : recvs_) rstage_[set].emplace_back(m.bytes, GMT_SPACE_PINNED);
    for (auto& m : sends_) sstage_.emplace_back(m.bytes, kernel_ ? GMT_SPACE_PINNED_COHERENT : GMT_SPACE_PINNED);
    for (size_t i = 0; i < sends_.size(); ++i)
      for (size_t off = 0; off < sends_[i].bytes || off == 0; off += kChunk) {
        schunks_.push_back({i, off, std::min(kChunk, sends_[i].bytes - off)});
        if (sends_[i].bytes == 0) break;
      }
    for (size_t i = 0; i < recvs_.size(); ++i) {
      for (size_t off = 0; off < recvs_[i].bytes || off == 0; off += kChunk) {
        rchunks_.push_back({i, off, std::min(kChunk, recvs_[i].bytes - off)});
        if (recvs_[i].bytes == 0) break;
      }
      (recvs_[i].block.base ? any_block_recv_ : any_flat_recv_) = true;
    }
    if (kernel_ && !schunks_.empty()) {
      const size_t n = schunks_.size();
      std::vector<gmt_stage_chunk> t(n);
      for (size_t k = 0; k < n; ++k) {
        const Chunk& ch = schunks_[k];
        const Msg& m = sends_[ch.msg];
        // a field block is gathered in place (the pack and the D2H leg in one
        // pass); a flat buffer is copied
        t[k] = stage_chunk(m, m.buf ? static_cast<const char*>(m.buf) + ch.off : nullptr,
                           sstage_[ch.msg].data() + ch.off, ch);
      }
      table_ = Buffer<gmt_stage_chunk>(n, GMT_SPACE_DEVICE);
      GMT_CHECK("stage table", gmt_rt_memcpy(table_.data(), t.data(), n * sizeof(gmt_stage_chunk)));
      counters_ = Buffer<unsigned>(n, GMT_SPACE_DEVICE);
      GMT_CHECK("stage counters", gmt_rt_memset_async(counters_.data(), 0, counters_.bytes(), nullptr));
      GMT_CHECK("stage counters", gmt_rt_stream_synchronize(nullptr));
      flags_ = Buffer<uint64_t>(n, GMT_SPACE_PINNED_COHERENT);
      for (size_t k = 0; k < n; ++k) flags_.data()[k] = 0;
    } else {
      events_.resize(schunks_.size(), nullptr);
      for (auto& e : events_) GMT_CHECK("event", gmt_rt_event_create(&e, 0));
    }
    if (any_block_recv_ && !rchunks_.empty()) {
      // per staging set: the scatter descriptors of every receive chunk
      // (field blocks straight out of page-locked memory)
      const size_t n = rchunks_.size();
      for (int set = 0; set < 2; ++set) {
        std::vector<gmt_stage_chunk> t(n);
        for (size_t k = 0; k < n; ++k) {
          const Chunk& ch = rchunks_[k];
          const Msg& m = recvs_[ch.msg];
          t[k] = stage_chunk(m, rstage_[set][ch.msg].data() + ch.off,
                             m.buf ? static_cast<char*>(m.buf) + ch.off : nullptr, ch);
        }
        rtable_[set] = Buffer<gmt_stage_chunk>(n, GMT_SPACE_DEVICE);
        GMT_CHECK("scatter table", gmt_rt_memcpy(rtable_[set].data(), t.data(), n * sizeof(gmt_stage_chunk)));
      }
    }
    for (auto& e : h2d_done_) GMT_CHECK("event", gmt_rt_event_create(&e, 0));
    // flat receive chunks go to the device on a stream of their own (SDMA
    // copies that start as a chunk lands, instead of queueing behind the
    // staging kernel on the caller's stream; field blocks keep their scatter
    // kernels on the caller's stream: profiles/r05_xport/)
    const char* rs = std::getenv("GMT_HOST_RECV_STREAM");  // A/B: 0 = the caller's stream
    if (any_flat_recv_ && !(rs && std::atoi(rs) == 0)) {
      GMT_CHECK("stream", gmt_rt_stream_create(&hs_, 1));
      GMT_CHECK("event", gmt_rt_event_create(&before_, 0));
      GMT_CHECK("event", gmt_rt_event_create(&flat_done_, 0));
    }
    // the staging poll gives up after this long WITHOUT a chunk staged (the
    // clock restarts at every staged chunk).  The first chunk also waits for
    // whatever the stream holds ahead of the staging kernel, so the default
    // is the hang watchdog's timeout (GMT_TIMEOUT), at least 10 s; an
    // explicit GMT_WAIT_TIMEOUT_MS wins
    const char* w = std::getenv("GMT_WAIT_TIMEOUT_MS");
    const double wd = watchdog_state().timeout;
    wait_limit_s_ = w && std::atof(w) > 0 ? std::atof(w) / 1e3 : std::max(10.0, wd);
  }
  ~MpiHostExchange() override {
    if (trace_ && !tr_.empty()) trace_dump();
    for (auto& e : events_) gmt_rt_event_destroy(e);
    for (auto& e : h2d_done_) gmt_rt_event_destroy(e);
    if (hs_) {
      gmt_rt_event_destroy(before_);
      gmt_rt_event_destroy(flat_done_);
      gmt_rt_stream_destroy(hs_);
    }
  }
  void start(gmt_stream_t s) override {
    if (trace_) trace_start();
    cur_ ^= 1;
    // the exchange before last drained this staging set with its H2D copies
    if (armed_[cur_]) GMT_CHECK("staging reuse", gmt_rt_event_synchronize(h2d_done_[cur_]));
    if (hs_) {  // the flat copies write device buffers the caller's earlier work may read
      GMT_CHECK("event", gmt_rt_event_record(before_, s));
      GMT_CHECK("stream wait", gmt_rt_stream_wait_event(hs_, before_));
    }
    rreqs_.assign(rchunks_.size(), MPI_REQUEST_NULL);
    for (size_t k = 0; k < rchunks_.size(); ++k) {
      const Chunk& ch = rchunks_[k];
      const Msg& m = recvs_[ch.msg];
      irecv(rstage_[cur_][ch.msg].data() + ch.off, ch.len, m.peer, m.tag, c_, &rreqs_[k]);
    }
    if (kernel_) {
      // kStageWgs workgroups sweep the chunks in order (2 x 16 B in flight per lane)
      ++epoch_;
      GMT_CHECK("stage D2H", gmt_stage_copy(static_cast<int>(schunks_.size()), table_.data(), counters_.data(),
                                            flags_.data(), epoch_, kStageWgs, s));
      return;
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
    std::vector<size_t> deferred;
    // a received chunk: a flat message gets its H2D copy; a field block is
    // scattered from page-locked memory into the ghost cells by one launch
    // — after every flat copy when the exchange has both (a flat y face
    // carries the sender's stale corner ghosts; the corner blocks must land
    // last, gmt/halo.hpp)
    auto land_one = [&](size_t k) {
      const Chunk& ch = rchunks_[k];
      const Msg& m = recvs_[ch.msg];
      if (!ch.len) return;
      if (m.block.base) {
        if (any_flat_recv_) deferred.push_back(k);
        else GMT_CHECK("stage scatter", gmt_stage_scatter(1, rtable_[cur_].data() + k, kScatterWgs, s));
        return;
      }
      GMT_CHECK("stage H2D", gmt_rt_memcpy_async(static_cast<char*>(m.buf) + ch.off,
                                                 rstage_[cur_][ch.msg].data() + ch.off, ch.len, hs_ ? hs_ : s));
    };
    auto land = [&](int n) {
      for (int q = 0; q < n; ++q) land_one(static_cast<size_t>(idx[q]));
      pending -= static_cast<size_t>(n);
      if (trace_) tr_.back().landed.push_back(MPI_Wtime());
    };
    auto send = [&](size_t k) {
      const Chunk& ch = schunks_[k];
      const Msg& m = sends_[ch.msg];
      if (trace_) tr_.back().staged.push_back(MPI_Wtime());
      sreqs.emplace_back();
      isend(sstage_[ch.msg].data() + ch.off, ch.len, m.peer, m.tag, c_, &sreqs.back());
    };
    // chunk k of the send staging is complete (kernel: its host flag; sdma: its event)
    auto staged = [&](size_t k) {
      return kernel_ ? __atomic_load_n(flags_.data() + k, __ATOMIC_ACQUIRE) >= epoch_
                     : gmt_rt_event_query(events_[k]) == 0;
    };
    if (trace_) tr_.back().wait = MPI_Wtime();
    double t0 = MPI_Wtime();
    long polls = 0;
    while (next < schunks_.size() || pending > 0) {
      bool progress = false;
      while (next < schunks_.size() && staged(next)) {
        send(next++);
        progress = true;
        t0 = MPI_Wtime();
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
        if (!kernel_) {
          GMT_CHECK("stage D2H wait", gmt_rt_event_synchronize(events_[next]));
          send(next++);
          continue;
        }
        // poll its host flag (and the receives) again: bounded by wall
        // clock, the stream's error state checked, the core yielded now and
        // then (ranks share the host's cores with MPI progress)
        if ((++polls & 1023) == 0) {
          const int q = gmt_rt_stream_query(s);
          if (q != 0 && q != 1) {
            std::printf("mpi-host: the staging stream failed before chunk %zu of %zu was staged: %s\n", next,
                        schunks_.size(), gmt_rt_error_string(q));
            abort_job(EXIT_FAILURE);
          }
          if (MPI_Wtime() - t0 > wait_limit_s_) {
            std::printf("mpi-host: chunk %zu of %zu never staged within %.1f s (GMT_WAIT_TIMEOUT_MS)\n", next,
                        schunks_.size(), wait_limit_s_);
            abort_job(EXIT_FAILURE);
          }
          sched_yield();
        }
        continue;
      }
      // every chunk is sent: block on the receives
      int n = 0;
      GMT_MPI_CHECK(MPI_Waitsome(static_cast<int>(rreqs_.size()), rreqs_.data(), &n, idx.data(),
                                 MPI_STATUSES_IGNORE));
      if (n > 0 && n != MPI_UNDEFINED) land(n);
    }
    if (hs_) {  // the flat copies joined back into the caller's stream
      GMT_CHECK("event", gmt_rt_event_record(flat_done_, hs_));
      GMT_CHECK("stream wait", gmt_rt_stream_wait_event(s, flat_done_));
    }
    if (!deferred.empty()) {  // the field blocks, after every flat copy
      std::sort(deferred.begin(), deferred.end());
      for (size_t a = 0; a < deferred.size();) {  // runs of consecutive chunks: one launch each
        size_t b = a + 1;
        while (b < deferred.size() && deferred[b] == deferred[b - 1] + 1) ++b;
        GMT_CHECK("stage scatter", gmt_stage_scatter(static_cast<int>(b - a), rtable_[cur_].data() + deferred[a],
                                                     kScatterWgs, s));
        a = b;
      }
    }
    if (trace_) tr_.back().recvd = MPI_Wtime();
    waitall(sreqs, "mpi-host exchange");
    GMT_CHECK("event", gmt_rt_event_record(h2d_done_[cur_], s));
    armed_[cur_] = true;
    if (trace_) tr_.back().end = MPI_Wtime();
  }

 private:
  // GMT_HOST_TRACE=DIR: host timestamps of every exchange (start, wait
  // entry, each chunk staged and sent, each receive chunk landed, all
  // received, sends complete), written to DIR/host_trace_r<rank>.txt when
  // the plan is destroyed — the phases of a slow exchange against a fast one
  struct Trace {
    double start = 0, wait = 0, recvd = 0, end = 0;
    std::vector<double> staged, landed;
  };
  void trace_start() {
    tr_.emplace_back();
    tr_.back().start = MPI_Wtime();
  }
  void trace_dump() {
    int rank = 0;
    MPI_Comm_rank(c_, &rank);
    const std::string path = std::string(trace_) + "/host_trace_r" + std::to_string(rank) + ".txt";
    FILE* f = std::fopen(path.c_str(), "a");
    if (!f) return;
    std::fprintf(f, "# exchange start(s) wait+ first_staged+ last_staged+ first_landed+ last_landed+ recvd+ end+ "
                    "(us after start) chunks=%zu/%zu bytes=%zu\n", schunks_.size(), rchunks_.size(), total_bytes());
    for (size_t i = 0; i < tr_.size(); ++i) {
      const Trace& t = tr_[i];
      auto us = [&](double v) { return v > 0 ? (v - t.start) * 1e6 : -1.0; };
      std::fprintf(f, "%zu %.6f %.1f %.1f %.1f %.1f %.1f %.1f %.1f\n", i, t.start, us(t.wait),
                   us(t.staged.empty() ? 0 : t.staged.front()), us(t.staged.empty() ? 0 : t.staged.back()),
                   us(t.landed.empty() ? 0 : t.landed.front()), us(t.landed.empty() ? 0 : t.landed.back()),
                   us(t.recvd), us(t.end));
    }
    std::fclose(f);
  }
  size_t total_bytes() const {
    size_t b = 0;
    for (auto& m : sends_) b += m.bytes;
    return b;
  }
  const char* trace_ = std::getenv("GMT_HOST_TRACE");
  std::vector<Trace> tr_;

 public:

 private:
  struct Chunk {
    size_t msg, off, len;
  };
  // the staging descriptor of chunk ch of message m: flat (rows 0) or the
  // packed doubles [off/8, (off+len)/8) of the message's field block
  static gmt_stage_chunk stage_chunk(const Msg& m, const void* src, void* dst, const Chunk& ch) {
    gmt_stage_chunk t{src, dst, static_cast<int64_t>(ch.len), 0, 0, 0, nullptr};
    if (m.block.base) {
      t.rows = static_cast<int64_t>(m.block.rows);
      t.ld = static_cast<int64_t>(m.block.ld);
      t.first = static_cast<int64_t>(ch.off / sizeof(double));
      t.block = m.block.base;
    }
    return t;
  }
  static constexpr int kStageWgs = 256;  // one per CU: enough posted writes in flight to fill the host link
  static constexpr int kScatterWgs = 32;
  MPI_Comm c_;
  std::vector<Msg> recvs_, sends_;
  bool kernel_;
  bool any_block_recv_ = false, any_flat_recv_ = false;
  Buffer<gmt_stage_chunk> table_;
  Buffer<gmt_stage_chunk> rtable_[2];
  Buffer<unsigned> counters_;
  Buffer<uint64_t> flags_;  // per send chunk: the exchange (epoch) whose data it holds
  uint64_t epoch_ = 0;
  std::vector<Buffer<char>> rstage_[2], sstage_;
  std::vector<Chunk> schunks_, rchunks_;
  std::vector<gmt_event_t> events_;
  std::vector<MPI_Request> rreqs_;
  gmt_event_t h2d_done_[2] = {nullptr, nullptr};
  gmt_stream_t hs_ = nullptr;  // flat receive chunks' H2D copies
  gmt_event_t before_ = nullptr, flat_done_ = nullptr;
  bool armed_[2] = {false, false};
  int cur_ = 1;
  double wait_limit_s_ = 10.0;
};

class MpiHostTransport : public MpiTransport {
 public:
  explicit MpiHostTransport(MPI_Comm c) : MpiTransport(c) {
    const unsigned long long mine = MpiHostExchange::chunk_bytes();
    unsigned long long lo = mine, hi = mine;
    GMT_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, &lo, 1, MPI_UNSIGNED_LONG_LONG, MPI_MIN, c));
    GMT_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, &hi, 1, MPI_UNSIGNED_LONG_LONG, MPI_MAX, c));
    if (lo != hi && rank_ == 0)
      std::printf("# mpi-host: GMT_HOST_CHUNK_KB differs between ranks (%llu..%llu KiB); using %llu KiB\n",
                  lo >> 10, hi >> 10, hi >> 10);
    chunk_ = static_cast<size_t>(hi);
  }
  Kind kind() const override { return Kind::MpiHost; }
  const char* name() const override { return "mpi-host"; }
  // GMT_HOST_BLOCKS=0: pack / unpack halo faces through device buffers (the
  // round-3 five-hop path, for A/B) instead of staging them in place
  bool takes_blocks() const override {
    const char* e = std::getenv("GMT_HOST_BLOCKS");
    return MpiHostExchange::kernel_staging() && !(e && e[0] == '0');
  }
  bool orders_block_receives() const override { return true; }
  std::unique_ptr<Exchange> plan(const std::vector<Msg>& r, const std::vector<Msg>& s) override {
    return std::make_unique<MpiHostExchange>(comm_, chunk_, r, s);
  }
  void allreduce_sum(double* buf, size_t n, gmt_stream_t s) override {
    staged_allreduce(staging_, comm_, buf, n, s);
  }
  void allreduce_max(double* buf, size_t n, gmt_stream_t s) override {
    staged_allreduce(staging_, comm_, buf, n, s, MPI_MAX);
  }
  void allgather(const void* send, void* recv, size_t bpr, gmt_stream_t s) override {
    staged_allgather(staging_, comm_, rank_, size_, send, recv, bpr, s);
  }

 private:
  Staging staging_;
  size_t chunk_ = size_t(1) << 20;
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
  void allreduce_max(double* buf, size_t n, gmt_stream_t s) override {
    require_mpi_readable(buf, "all-reduce buffer");
    GMT_CHECK("allreduce sync", gmt_rt_stream_synchronize(s));
    GMT_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, buf, static_cast<int>(n), MPI_DOUBLE, MPI_MAX, comm_));
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

// ------------------------------------------------------- MPI control plane
// gmt/control.hpp over MPI: the ipc transport's handle exchange and
// host-staged collectives in the native apps.
class MpiControl : public Control {
 public:
  explicit MpiControl(MPI_Comm c) : Control(MpiTransport::rank_of(c), MpiTransport::size_of(c)), c_(c) {}
  const char* name() const override { return "mpi"; }
  void exchange(const std::vector<HostMsg>& recvs, const std::vector<HostMsg>& sends) override {
    std::vector<MPI_Request> reqs;
    reqs.reserve(recvs.size() + sends.size());
    for (auto& m : recvs) {
      reqs.emplace_back();
      irecv(m.buf, m.bytes, m.peer, m.tag, c_, &reqs.back());
    }
    for (auto& m : sends) {
      reqs.emplace_back();
      isend(m.buf, m.bytes, m.peer, m.tag, c_, &reqs.back());
    }
    waitall(reqs, "control exchange");
  }
  void allreduce_sum(double* buf, size_t n) override {
    GMT_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, buf, static_cast<int>(n), MPI_DOUBLE, MPI_SUM, c_));
  }
  void allreduce_max(double* buf, size_t n) override {
    GMT_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, buf, static_cast<int>(n), MPI_DOUBLE, MPI_MAX, c_));
  }
  void allgather(const void* send, void* recv, size_t bpr) override {
    MPI_Datatype t;
    int n;
    mpi_count(bpr, &t, &n);
    const bool inplace = send == static_cast<const char*>(recv) + rank_ * bpr;
    GMT_MPI_CHECK(MPI_Allgather(inplace ? MPI_IN_PLACE : send, inplace ? 0 : n, t, recv, n, t, c_));
  }
  void barrier() override { GMT_MPI_CHECK(MPI_Barrier(c_)); }

 private:
  MPI_Comm c_;
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
    case Kind::Ipc: return make_ipc_transport(std::make_unique<MpiControl>(comm));
    case Kind::Local: return make_local_transport();
    default: break;
  }
  abort_job(EXIT_FAILURE);
}

}  // namespace comm
}  // namespace gmt
