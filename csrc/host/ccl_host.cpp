// Host-backend implementation of gmt/ccl.h: the RCCL data-plane semantics
// (point-to-point send/recv grouped per exchange, all-reduce, all-gather,
// broadcast) emulated between processes of one node over Unix-domain
// sockets, so the code paths that run on RCCL over xGMI on an MI355X node —
// the transports' grouped halo exchange (transport_core.cpp RcclExchange),
// the native Jacobi engine at N ranks, bench.py's multi-rank path — run and
// are checked on a CPU-only box with any number of ranks.
//
// Semantics mirrored from RCCL/NCCL:
//   * a unique id created on one rank and distributed out of band (MPI_Bcast
//     in the apps, torch.distributed in Python) names the communicator;
//   * inside gmt_ccl_group_start/end the sends and receives progress
//     concurrently (no ordering deadlock); messages between a pair of ranks
//     match in issue order; sizes must agree (checked: every message carries
//     its length);
//   * sends/receives to self are allowed (periodic domains);
//   * collectives give bitwise-identical results on every rank (reduction in
//     rank order).
// gmt_ccl_available() stays 0 — automatic transport selection never picks the
// emulation; gmt_ccl_emulated() == 1 lets an explicit "rccl" request run.
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <random>
#include <string>
#include <vector>

#include "gmt/ccl.h"

namespace {

enum : int {
  kOk = 0,
  kErrSys = 9002,       // socket / system call failure
  kErrArg = 9003,       // invalid argument
  kErrTimeout = GMT_CCL_TIMEOUT,  // a peer did not connect / progress
  kErrMismatch = 9005,  // message sizes of a send/recv pair differ
};

constexpr int kTimeoutMs = 120000;
// communicator set-up deadline: GMT_CCL_INIT_TIMEOUT seconds (default 120)
int init_timeout_ms() {
  const char* e = std::getenv("GMT_CCL_INIT_TIMEOUT");
  const double s = e ? std::atof(e) : 0.0;
  return s > 0.0 ? static_cast<int>(s * 1000.0) : kTimeoutMs;
}

struct Op {
  bool send;
  char* buf;
  size_t bytes;
  int peer;
  uint64_t hdr = 0;
  size_t hdr_done = 0, done = 0;
};

}  // namespace

struct gmt_ccl_comm_s {
  int rank = 0, n = 1;
  std::vector<int> fd;  // per peer (-1 for self)
};

namespace {

thread_local int g_depth = 0;
thread_local std::vector<std::pair<gmt_ccl_comm_t, Op>> g_ops;
thread_local char g_err[256] = "";

int fail(int code, const char* what) {
  std::snprintf(g_err, sizeof(g_err), "%s: %s", what, code == kErrSys ? std::strerror(errno) : "");
  return code;
}

std::string sock_name(const gmt_ccl_id* id, int rank) {
  char tok[96];
  std::memcpy(tok, id->internal, sizeof(tok));
  tok[sizeof(tok) - 1] = 0;
  return std::string(tok) + "-" + std::to_string(rank);
}

socklen_t make_addr(const std::string& name, sockaddr_un* a) {
  std::memset(a, 0, sizeof(*a));
  a->sun_family = AF_UNIX;
  // abstract namespace: leading NUL, no file system entry to clean up
  std::memcpy(a->sun_path + 1, name.data(), std::min(name.size(), sizeof(a->sun_path) - 2));
  return static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + name.size());
}

double now_ms() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

bool full_io(int fd, void* p, size_t n, bool wr) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t k = wr ? ::send(fd, c, n, MSG_NOSIGNAL) : ::recv(fd, c, n, 0);
    if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    if (k <= 0) return false;
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

// Progress a set of operations of one communicator to completion.  Per peer
// only the oldest send and the oldest receive are active (issue-order
// matching); all peers progress concurrently under poll().
int progress(gmt_ccl_comm_t c, std::vector<Op>& ops) {
  // self messages: k-th send to self -> k-th receive from self
  std::vector<Op*> ss, sr;
  for (auto& o : ops)
    if (o.peer == c->rank) (o.send ? ss : sr).push_back(&o);
  if (ss.size() != sr.size()) return fail(kErrMismatch, "unmatched send/recv to self");
  for (size_t i = 0; i < ss.size(); ++i) {
    if (ss[i]->bytes != sr[i]->bytes) return fail(kErrMismatch, "send/recv to self size mismatch");
    if (ss[i]->bytes) std::memmove(sr[i]->buf, ss[i]->buf, ss[i]->bytes);
  }
  std::vector<std::deque<Op*>> sq(c->n), rq(c->n);
  size_t pending = 0;
  for (auto& o : ops) {
    if (o.peer == c->rank) continue;
    o.hdr = o.send ? o.bytes : 0;
    (o.send ? sq : rq)[o.peer].push_back(&o);
    ++pending;
  }
  double t_last = now_ms();
  std::vector<pollfd> pf;
  std::vector<int> who;
  while (pending) {
    pf.clear();
    who.clear();
    for (int p = 0; p < c->n; ++p) {
      short ev = (sq[p].empty() ? 0 : POLLOUT) | (rq[p].empty() ? 0 : POLLIN);
      if (ev) {
        pf.push_back({c->fd[p], ev, 0});
        who.push_back(p);
      }
    }
    const int r = ::poll(pf.data(), pf.size(), 1000);
    if (r < 0 && errno != EINTR) return fail(kErrSys, "poll");
    if (r <= 0) {
      if (now_ms() - t_last > kTimeoutMs) return fail(kErrTimeout, "peer made no progress");
      continue;
    }
    t_last = now_ms();
    for (size_t i = 0; i < pf.size(); ++i) {
      const int p = who[i];
      if (pf[i].revents & (POLLERR | POLLNVAL)) return fail(kErrSys, "peer socket error");
      if ((pf[i].revents & POLLOUT) && !sq[p].empty()) {
        Op* o = sq[p].front();
        if (o->hdr_done < sizeof(o->hdr)) {
          const ssize_t k = ::send(c->fd[p], reinterpret_cast<char*>(&o->hdr) + o->hdr_done,
                                   sizeof(o->hdr) - o->hdr_done, MSG_NOSIGNAL | MSG_DONTWAIT);
          if (k < 0 && errno != EAGAIN && errno != EINTR) return fail(kErrSys, "send header");
          if (k > 0) o->hdr_done += static_cast<size_t>(k);
        }
        if (o->hdr_done == sizeof(o->hdr) && o->done < o->bytes) {
          const ssize_t k = ::send(c->fd[p], o->buf + o->done, o->bytes - o->done,
                                   MSG_NOSIGNAL | MSG_DONTWAIT);
          if (k < 0 && errno != EAGAIN && errno != EINTR) return fail(kErrSys, "send");
          if (k > 0) o->done += static_cast<size_t>(k);
        }
        if (o->hdr_done == sizeof(o->hdr) && o->done == o->bytes) {
          sq[p].pop_front();
          --pending;
        }
      }
      if ((pf[i].revents & (POLLIN | POLLHUP)) && !rq[p].empty()) {
        Op* o = rq[p].front();
        if (o->hdr_done < sizeof(o->hdr)) {
          const ssize_t k = ::recv(c->fd[p], reinterpret_cast<char*>(&o->hdr) + o->hdr_done,
                                   sizeof(o->hdr) - o->hdr_done, MSG_DONTWAIT);
          if (k == 0) return fail(kErrSys, "peer closed the connection");
          if (k < 0 && errno != EAGAIN && errno != EINTR) return fail(kErrSys, "recv header");
          if (k > 0) o->hdr_done += static_cast<size_t>(k);
          if (o->hdr_done == sizeof(o->hdr) && o->hdr != o->bytes) {
            std::snprintf(g_err, sizeof(g_err), "rank %d expects %zu bytes from rank %d, got %llu",
                          c->rank, o->bytes, p, static_cast<unsigned long long>(o->hdr));
            return kErrMismatch;
          }
        }
        if (o->hdr_done == sizeof(o->hdr) && o->done < o->bytes) {
          const ssize_t k = ::recv(c->fd[p], o->buf + o->done, o->bytes - o->done, MSG_DONTWAIT);
          if (k == 0) return fail(kErrSys, "peer closed the connection");
          if (k < 0 && errno != EAGAIN && errno != EINTR) return fail(kErrSys, "recv");
          if (k > 0) o->done += static_cast<size_t>(k);
        }
        if (o->hdr_done == sizeof(o->hdr) && o->done == o->bytes) {
          rq[p].pop_front();
          --pending;
        }
      }
    }
  }
  return kOk;
}

int enqueue(gmt_ccl_comm_t c, bool send, const void* buf, size_t bytes, int peer) {
  if (!c || peer < 0 || peer >= c->n || (bytes && !buf)) return fail(kErrArg, "send/recv argument");
  Op o{send, const_cast<char*>(static_cast<const char*>(buf)), bytes, peer};
  if (g_depth > 0) {
    g_ops.emplace_back(c, o);
    return kOk;
  }
  std::vector<Op> one{o};
  return progress(c, one);
}

// Run a batch of operations as one group (collectives).
int run_group(gmt_ccl_comm_t c, std::vector<Op>& ops) { return progress(c, ops); }

}  // namespace

extern "C" {

int gmt_ccl_available(void) { return 0; }
int gmt_ccl_emulated(void) { return 1; }

const char* gmt_ccl_error_string(int err) {
  switch (err) {
    case kOk: return "success";
    case GMT_CCL_UNAVAILABLE: return "not available";
    default: return g_err[0] ? g_err : "host ccl error";
  }
}

int gmt_ccl_version(int* v) {
  *v = 0;
  return kOk;
}

int gmt_ccl_get_unique_id(gmt_ccl_id* id) {
  std::memset(id, 0, sizeof(*id));
  std::random_device rd;
  const unsigned long long r = (static_cast<unsigned long long>(rd()) << 32) ^ rd();
  std::snprintf(id->internal, 96, "gmtccl-%d-%016llx", static_cast<int>(getpid()), r);
  return kOk;
}

int gmt_ccl_comm_init(gmt_ccl_comm_t* out, int nranks, const gmt_ccl_id* id, int rank) {
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks || std::strncmp(id->internal, "gmtccl-", 7) != 0)
    return fail(kErrArg, "comm_init: bad rank/size or unique id");
  auto* c = new gmt_ccl_comm_s;
  c->rank = rank;
  c->n = nranks;
  c->fd.assign(nranks, -1);
  auto bail = [&](int code, const char* what) {
    const int e = fail(code, what);
    for (int f : c->fd)
      if (f >= 0) ::close(f);
    delete c;
    return e;
  };
  int lfd = -1;
  if (rank < nranks - 1) {  // higher ranks connect to us
    lfd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_un a;
    const socklen_t al = make_addr(sock_name(id, rank), &a);
    if (lfd < 0 || ::bind(lfd, reinterpret_cast<sockaddr*>(&a), al) != 0 || ::listen(lfd, nranks) != 0) {
      if (lfd >= 0) ::close(lfd);
      return bail(kErrSys, "comm_init: listen");
    }
  }
  // connect to every lower rank (retry until its listener exists), then say who we are
  for (int p = 0; p < rank; ++p) {
    sockaddr_un a;
    const socklen_t al = make_addr(sock_name(id, p), &a);
    const double t0 = now_ms();
    for (;;) {
      const int f = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
      if (f < 0) return bail(kErrSys, "comm_init: socket");
      if (::connect(f, reinterpret_cast<sockaddr*>(&a), al) == 0) {
        c->fd[p] = f;
        break;
      }
      ::close(f);
      if (now_ms() - t0 > init_timeout_ms()) {
        if (lfd >= 0) ::close(lfd);
        return bail(kErrTimeout, "comm_init: lower rank never listened");
      }
      ::usleep(2000);
    }
    int32_t me = rank;
    if (!full_io(c->fd[p], &me, sizeof(me), true)) return bail(kErrSys, "comm_init: hello");
  }
  // accept every higher rank
  for (int k = rank + 1; k < nranks; ++k) {
    pollfd pf{lfd, POLLIN, 0};
    if (::poll(&pf, 1, init_timeout_ms()) <= 0) {
      ::close(lfd);
      return bail(kErrTimeout, "comm_init: higher rank never connected");
    }
    const int f = ::accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
    int32_t who = -1;
    if (f < 0 || !full_io(f, &who, sizeof(who), false) || who <= rank || who >= nranks || c->fd[who] >= 0) {
      if (f >= 0) ::close(f);
      ::close(lfd);
      return bail(kErrSys, "comm_init: accept");
    }
    c->fd[who] = f;
  }
  if (lfd >= 0) ::close(lfd);
  for (int f : c->fd)
    if (f >= 0) ::fcntl(f, F_SETFL, ::fcntl(f, F_GETFL) | O_NONBLOCK);
  *out = c;
  return kOk;
}

int gmt_ccl_comm_destroy(gmt_ccl_comm_t c) {
  if (!c) return kOk;
  for (int f : c->fd)
    if (f >= 0) ::close(f);
  delete c;
  return kOk;
}

int gmt_ccl_group_start(void) {
  ++g_depth;
  return kOk;
}

int gmt_ccl_group_end(void) {
  if (g_depth <= 0) return fail(kErrArg, "group_end without group_start");
  if (--g_depth > 0) return kOk;
  // one progress loop per communicator, in first-use order
  std::vector<std::pair<gmt_ccl_comm_t, Op>> ops;
  ops.swap(g_ops);
  std::vector<gmt_ccl_comm_t> comms;
  for (auto& e : ops)
    if (std::find(comms.begin(), comms.end(), e.first) == comms.end()) comms.push_back(e.first);
  for (auto* c : comms) {
    std::vector<Op> mine;
    for (auto& e : ops)
      if (e.first == c) mine.push_back(e.second);
    const int r = progress(c, mine);
    if (r != kOk) return r;
  }
  return kOk;
}

int gmt_ccl_send(const void* buf, size_t bytes, int peer, gmt_ccl_comm_t c, gmt_stream_t) {
  return enqueue(c, true, buf, bytes, peer);
}

int gmt_ccl_recv(void* buf, size_t bytes, int peer, gmt_ccl_comm_t c, gmt_stream_t) {
  return enqueue(c, false, buf, bytes, peer);
}

int gmt_ccl_allgather(const void* send, void* recv, size_t bpr, gmt_ccl_comm_t c, gmt_stream_t) {
  if (!c) return fail(kErrArg, "allgather: comm");
  char* r = static_cast<char*>(recv);
  const char* mine = static_cast<const char*>(send);
  if (mine != r + c->rank * bpr && bpr) std::memmove(r + c->rank * bpr, mine, bpr);
  std::vector<Op> ops;
  for (int p = 0; p < c->n; ++p) {
    if (p == c->rank) continue;
    ops.push_back(Op{true, r + c->rank * bpr, bpr, p});
    ops.push_back(Op{false, r + p * bpr, bpr, p});
  }
  return run_group(c, ops);
}

static int allreduce(const double* send, double* recv, size_t count, gmt_ccl_comm_t c, bool max) {
  if (!c) return fail(kErrArg, "allreduce: comm");
  std::vector<double> all(count * static_cast<size_t>(c->n));
  const int r = gmt_ccl_allgather(send, all.data(), count * sizeof(double), c, nullptr);
  if (r != kOk) return r;
  // rank order: every rank computes the same bits
  for (size_t i = 0; i < count; ++i) {
    double v = all[i];
    for (int p = 1; p < c->n; ++p) {
      const double w = all[p * count + i];
      v = max ? (w > v ? w : v) : v + w;
    }
    recv[i] = v;
  }
  return kOk;
}

int gmt_ccl_allreduce_sum_f64(const double* send, double* recv, size_t count, gmt_ccl_comm_t c,
                              gmt_stream_t) {
  return allreduce(send, recv, count, c, false);
}

int gmt_ccl_allreduce_max_f64(const double* send, double* recv, size_t count, gmt_ccl_comm_t c,
                              gmt_stream_t) {
  return allreduce(send, recv, count, c, true);
}

int gmt_ccl_broadcast(void* buf, size_t bytes, int root, gmt_ccl_comm_t c, gmt_stream_t) {
  if (!c || root < 0 || root >= c->n) return fail(kErrArg, "broadcast: root");
  std::vector<Op> ops;
  if (c->rank == root) {
    for (int p = 0; p < c->n; ++p)
      if (p != root) ops.push_back(Op{true, static_cast<char*>(buf), bytes, p});
  } else {
    ops.push_back(Op{false, static_cast<char*>(buf), bytes, root});
  }
  return run_group(c, ops);
}

}  // extern "C"
