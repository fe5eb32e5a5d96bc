// MPI-free transports: rccl (bootstrapped from a distributed unique id) and
// local (single process).  See gmt/transport.hpp.
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "gmt/transport.hpp"

namespace gmt {
namespace comm {

namespace {

// ---------------------------------------------------------------------- rccl
class RcclExchange : public Exchange {
 public:
  RcclExchange(gmt_ccl_comm_t cc, std::vector<Msg> r, std::vector<Msg> s)
      : cc_(cc), recvs_(std::move(r)), sends_(std::move(s)) {
    // Within one group, messages between a pair of ranks are matched in
    // issue order: sort both sides by (peer, tag) so the k-th send to B is
    // B's k-th receive from us.
    auto key = [](const Msg& a, const Msg& b) {
      return a.peer != b.peer ? a.peer < b.peer : a.tag < b.tag;
    };
    std::sort(recvs_.begin(), recvs_.end(), key);
    std::sort(sends_.begin(), sends_.end(), key);
  }
  void start(gmt_stream_t s) override {
    GMT_CCL_CHECK("group start", gmt_ccl_group_start());
    for (auto& m : recvs_) GMT_CCL_CHECK("recv", gmt_ccl_recv(m.buf, m.bytes, m.peer, cc_, s));
    for (auto& m : sends_) GMT_CCL_CHECK("send", gmt_ccl_send(m.buf, m.bytes, m.peer, cc_, s));
    GMT_CCL_CHECK("group end", gmt_ccl_group_end());
  }
  void wait(gmt_stream_t) override {}  // stream-ordered on s already
  bool graph_capturable() const override { return true; }

 private:
  gmt_ccl_comm_t cc_;
  std::vector<Msg> recvs_, sends_;
};

class RcclTransport : public Transport {
 public:
  RcclTransport(int rank, int size, const gmt_ccl_id& id) : Transport(rank, size) {
    if (!gmt_ccl_available() && !gmt_ccl_emulated()) {
      std::printf("ERROR: transport rccl requested but this build has no RCCL (%s backend)\n",
                  gmt_rt_backend_name());
      abort_job(EXIT_FAILURE);
    }
    const int e = gmt_ccl_comm_init(&cc_, size_, &id, rank_);
    if (e != 0) {
      char host[256] = "?";
      gethostname(host, sizeof(host) - 1);
      std::fprintf(stderr, "GMT: rank %d of %d (host %s): RCCL communicator init failed: %s (%d)\n", rank_, size_,
                   host, gmt_ccl_error_string(e), e);
      abort_job(e == GMT_CCL_TIMEOUT ? 124 : EXIT_FAILURE);
    }
  }
  ~RcclTransport() override { gmt_ccl_comm_destroy(cc_); }
  Kind kind() const override { return Kind::Rccl; }
  const char* name() const override { return "rccl"; }
  std::unique_ptr<Exchange> plan(const std::vector<Msg>& r, const std::vector<Msg>& s) override {
    return std::make_unique<RcclExchange>(cc_, r, s);
  }
  void allreduce_sum(double* buf, size_t n, gmt_stream_t s) override {
    GMT_CCL_CHECK("allreduce", gmt_ccl_allreduce_sum_f64(buf, buf, n, cc_, s));
  }
  void allreduce_max(double* buf, size_t n, gmt_stream_t s) override {
    GMT_CCL_CHECK("allreduce max", gmt_ccl_allreduce_max_f64(buf, buf, n, cc_, s));
  }
  void allgather(const void* send, void* recv, size_t bpr, gmt_stream_t s) override {
    GMT_CCL_CHECK("allgather", gmt_ccl_allgather(send, recv, bpr, cc_, s));
  }

 private:
  gmt_ccl_comm_t cc_ = nullptr;
};

// --------------------------------------------------------------------- local
class LocalExchange : public Exchange {
 public:
  LocalExchange(const std::vector<Msg>& r, const std::vector<Msg>& s) {
    for (auto& m : s) {
      const Msg* dst = nullptr;
      for (auto& q : r)
        if (q.tag == m.tag && q.peer == m.peer) dst = &q;
      if (m.peer != 0 || !dst || dst->bytes != m.bytes) {
        std::printf("local transport: message to rank %d tag %d has no matching receive\n",
                    m.peer, m.tag);
        abort_job(EXIT_FAILURE);
      }
      pairs_.push_back({dst->buf, m.buf, m.bytes});
    }
  }
  void start(gmt_stream_t s) override {
    for (auto& p : pairs_) GMT_CHECK("local copy", gmt_rt_memcpy_async(p.dst, p.src, p.bytes, s));
  }
  void wait(gmt_stream_t) override {}
  bool graph_capturable() const override { return true; }

 private:
  struct Pair {
    void* dst;
    const void* src;
    size_t bytes;
  };
  std::vector<Pair> pairs_;
};

class LocalTransport : public Transport {
 public:
  LocalTransport() : Transport(0, 1) {}
  Kind kind() const override { return Kind::Local; }
  const char* name() const override { return "local"; }
  std::unique_ptr<Exchange> plan(const std::vector<Msg>& r, const std::vector<Msg>& s) override {
    return std::make_unique<LocalExchange>(r, s);
  }
  void allreduce_sum(double*, size_t, gmt_stream_t) override {}
  void allreduce_max(double*, size_t, gmt_stream_t) override {}
  void allgather(const void* send, void* recv, size_t bpr, gmt_stream_t s) override {
    if (send != recv) GMT_CHECK("local gather", gmt_rt_memcpy_async(recv, send, bpr, s));
  }
};

}  // namespace

const char* kind_name(Kind k) {
  switch (k) {
    case Kind::MpiHost: return "mpi-host";
    case Kind::MpiDirect: return "mpi-direct";
    case Kind::Rccl: return "rccl";
    case Kind::Ipc: return "ipc";
    case Kind::Local: return "local";
    default: return "auto";
  }
}

std::unique_ptr<Transport> make_rccl_transport(int rank, int size, const gmt_ccl_id& id) {
  return std::make_unique<RcclTransport>(rank, size, id);
}

std::unique_ptr<Transport> make_local_transport() { return std::make_unique<LocalTransport>(); }

}  // namespace comm
}  // namespace gmt
