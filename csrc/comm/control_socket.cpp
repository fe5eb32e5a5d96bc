// Socket control plane (gmt/control.hpp): a full mesh of abstract-namespace
// Unix stream sockets between the ranks of one node.  Used by the MPI-free
// engine library for the IPC transport's handle exchange and its
// host-staged collectives; the data itself never crosses these sockets.
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <random>
#include <string>
#include <utility>

#include "gmt/check.hpp"
#include "gmt/control.hpp"

namespace gmt {
namespace comm {

namespace {

constexpr int kTagGather = -1, kTagBarrier = -2;

double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

double timeout_s() {
  const char* e = std::getenv("GMT_CTL_TIMEOUT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0 ? v : 300.0;
}

socklen_t make_addr(const std::string& name, sockaddr_un* a) {
  std::memset(a, 0, sizeof(*a));
  a->sun_family = AF_UNIX;
  const size_t n = std::min(name.size(), sizeof(a->sun_path) - 2);
  // abstract namespace: leading NUL, nothing to unlink afterwards
  std::memcpy(a->sun_path + 1, name.data(), n);
  return static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + n);
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

struct Header {
  int32_t tag;
  uint32_t magic;
  uint64_t bytes;
};
constexpr uint32_t kMagic = 0x474d5443;  // "GMTC"

class SocketControl : public Control {
 public:
  SocketControl(int rank, int size, const char* id)
      : Control(rank, size), fd_(size, -1), in_(size), closed_(size, false) {
    timeout_ = timeout_s();
    char tok[kControlIdBytes];
    std::memcpy(tok, id, sizeof(tok));
    tok[sizeof(tok) - 1] = 0;
    if (std::strncmp(tok, "gmtctl-", 7) != 0 || rank < 0 || rank >= size) {
      std::printf("gmt control: bad id or rank %d of %d\n", rank, size);
      abort_job(EXIT_FAILURE);
    }
    // "gmtctl-<pid>-<nonce>-<secret>": names from the public part, the
    // secret in every hello (an id without one authenticates with "")
    std::string base(tok), secret;
    const size_t cut = base.find('-', base.find('-', 7) + 1);
    if (cut != std::string::npos) {
      secret = base.substr(cut + 1);
      base.resize(cut);
    }
    char want[64] = {0};
    std::snprintf(want, sizeof(want), "%s", secret.c_str());
    auto name = [&](int r) { return base + "-" + std::to_string(r); };
    int lfd = -1;
    if (rank < size - 1) {  // higher ranks connect to us
      lfd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
      sockaddr_un a;
      const socklen_t al = make_addr(name(rank), &a);
      if (lfd < 0 || ::bind(lfd, reinterpret_cast<sockaddr*>(&a), al) != 0 || ::listen(lfd, size) != 0)
        fail("listen");
    }
    const double t0 = now_s();
    for (int p = 0; p < rank; ++p) {  // connect to every lower rank (retry until it listens)
      sockaddr_un a;
      const socklen_t al = make_addr(name(p), &a);
      for (;;) {
        const int f = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
        if (f < 0) fail("socket");
        if (::connect(f, reinterpret_cast<sockaddr*>(&a), al) == 0) {
          fd_[p] = f;
          break;
        }
        ::close(f);
        if (now_s() - t0 > timeout_) fail("rank never listened", p);
        ::usleep(2000);
      }
      int32_t me = rank;
      if (!full_io(fd_[p], &me, sizeof(me), true) || !full_io(fd_[p], want, sizeof(want), true)) fail("hello", p);
    }
    for (int k = rank + 1; k < size; ++k) {  // accept every higher rank
      pollfd pf{lfd, POLLIN, 0};
      if (::poll(&pf, 1, static_cast<int>(timeout_ * 1000)) <= 0) fail("a higher rank never connected");
      const int f = ::accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      if (f < 0) fail("accept");
      // only this user's processes, and only with the job's secret
      ucred cr{};
      socklen_t cl = sizeof(cr);
      if (::getsockopt(f, SOL_SOCKET, SO_PEERCRED, &cr, &cl) != 0 || cr.uid != ::geteuid()) {
        ::close(f);
        --k;  // not a rank of this job: keep waiting for the real one
        continue;
      }
      int32_t who = -1;
      char got[64] = {0};
      if (!full_io(f, &who, sizeof(who), false) || !full_io(f, got, sizeof(got), false) ||
          std::memcmp(got, want, sizeof(want)) != 0) {
        ::close(f);
        --k;
        continue;
      }
      if (who <= rank || who >= size || fd_[who] >= 0) fail("accept");
      fd_[who] = f;
    }
    if (lfd >= 0) ::close(lfd);
    for (int f : fd_)
      if (f >= 0) ::fcntl(f, F_SETFL, ::fcntl(f, F_GETFL) | O_NONBLOCK);
  }
  ~SocketControl() override {
    for (int f : fd_)
      if (f >= 0) ::close(f);
  }
  const char* name() const override { return "socket"; }

  void exchange(const std::vector<HostMsg>& recvs, const std::vector<HostMsg>& sends) override {
    for (auto& m : recvs)
      if (m.tag < 0) fail_tag(m.tag);
    for (auto& m : sends)
      if (m.tag < 0) fail_tag(m.tag);
    run(recvs, sends);
  }

  void allgather(const void* send, void* recv, size_t bpr) override {
    char* r = static_cast<char*>(recv);
    if (send != r + rank_ * bpr && bpr) std::memmove(r + rank_ * bpr, send, bpr);
    std::vector<HostMsg> rs, ss;
    for (int p = 0; p < size_; ++p) {
      if (p == rank_) continue;
      rs.push_back({r + p * bpr, bpr, p, kTagGather});
      ss.push_back({r + rank_ * bpr, bpr, p, kTagGather});
    }
    run(rs, ss);
  }
  void allreduce_sum(double* buf, size_t n) override { reduce(buf, n, false); }
  void allreduce_max(double* buf, size_t n) override { reduce(buf, n, true); }
  void barrier() override {
    std::vector<char> b(static_cast<size_t>(size_));
    std::vector<HostMsg> rs, ss;
    for (int p = 0; p < size_; ++p) {
      if (p == rank_) continue;
      rs.push_back({&b[p], 1, p, kTagBarrier});
      ss.push_back({&b[rank_], 1, p, kTagBarrier});
    }
    run(rs, ss);
  }

 private:
  // one incoming message being read from a peer's socket
  struct In {
    Header h{};
    size_t hdr_done = 0, done = 0;
    std::vector<char> body;
    std::map<int, std::deque<std::vector<char>>> early;  // complete, not yet asked for
  };
  struct Out {
    Header h;
    const char* buf;
    size_t hdr_done = 0, done = 0;
  };

  [[noreturn]] void fail(const char* what, int peer = -1) const {
    std::printf("gmt control (socket): rank %d of %d: %s%s%s (%s)\n", rank_, size_, what,
                peer >= 0 ? ", peer " : "", peer >= 0 ? std::to_string(peer).c_str() : "",
                errno ? std::strerror(errno) : "no system error");
    abort_job(EXIT_FAILURE);
  }
  [[noreturn]] void fail_tag(int tag) const {
    std::printf("gmt control: tag %d is reserved (tags must be >= 0)\n", tag);
    abort_job(EXIT_FAILURE);
  }

  void reduce(double* buf, size_t n, bool max) {
    std::vector<double> all(n * static_cast<size_t>(size_));
    allgather(buf, all.data(), n * sizeof(double));
    for (size_t i = 0; i < n; ++i) {  // rank order: the same bits everywhere
      double v = all[i];
      for (int p = 1; p < size_; ++p) {
        const double w = all[p * n + i];
        v = max ? (w > v ? w : v) : v + w;
      }
      buf[i] = v;
    }
  }

  // Deliver a complete message to the oldest matching receive, or keep it.
  static bool deliver(std::deque<const HostMsg*>& want, int tag, std::vector<char>& body, int rank, int peer) {
    for (auto it = want.begin(); it != want.end(); ++it)
      if ((*it)->tag == tag) {
        if ((*it)->bytes != body.size()) {
          std::printf("gmt control: rank %d expects %zu bytes (tag %d) from rank %d, got %zu\n", rank,
                      (*it)->bytes, tag, peer, body.size());
          abort_job(EXIT_FAILURE);
        }
        if (!body.empty()) std::memcpy((*it)->buf, body.data(), body.size());
        want.erase(it);
        return true;
      }
    return false;
  }

  void run(const std::vector<HostMsg>& recvs, const std::vector<HostMsg>& sends) {
    std::vector<std::deque<const HostMsg*>> want(size_);
    std::vector<std::deque<Out>> out(size_);
    size_t pending = 0;
    for (auto& m : recvs) {
      if (m.peer < 0 || m.peer >= size_) fail("receive from a rank outside the job", m.peer);
      want[m.peer].push_back(&m);
    }
    // messages to self: k-th send with a tag -> k-th receive with that tag
    for (auto& m : sends) {
      if (m.peer < 0 || m.peer >= size_) fail("send to a rank outside the job", m.peer);
      if (m.peer != rank_) {
        out[m.peer].push_back({Header{m.tag, kMagic, m.bytes}, static_cast<const char*>(m.buf)});
        continue;
      }
      std::vector<char> body(static_cast<const char*>(m.buf), static_cast<const char*>(m.buf) + m.bytes);
      if (!deliver(want[rank_], m.tag, body, rank_, rank_)) fail("send to self without a matching receive");
    }
    if (!want[rank_].empty()) fail("receive from self without a matching send");
    // receives that arrived during an earlier call
    for (int p = 0; p < size_; ++p) {
      for (auto it = want[p].begin(); it != want[p].end();) {
        auto e = in_[p].early.find((*it)->tag);
        if (e != in_[p].early.end() && !e->second.empty()) {
          std::vector<char> body = std::move(e->second.front());
          e->second.pop_front();
          const HostMsg* m = *it;
          std::deque<const HostMsg*> one{m};
          deliver(one, m->tag, body, rank_, p);
          it = want[p].erase(it);
        } else {
          ++it;
        }
      }
      pending += want[p].size() + out[p].size();
    }
    double t_last = now_s();
    std::vector<pollfd> pf;
    std::vector<int> who;
    while (pending) {
      pf.clear();
      who.clear();
      for (int p = 0; p < size_; ++p) {
        if (p == rank_) continue;
        if (closed_[p]) {
          if (!want[p].empty() || !out[p].empty()) fail("peer closed the connection", p);
          continue;
        }
        // always read: a peer blocked sending to us must drain before it reads
        pf.push_back({fd_[p], static_cast<short>(POLLIN | (out[p].empty() ? 0 : POLLOUT)), 0});
        who.push_back(p);
      }
      const int r = ::poll(pf.data(), pf.size(), 1000);
      if (r < 0 && errno != EINTR) fail("poll");
      if (r <= 0) {
        if (now_s() - t_last > timeout_) {
          for (int p = 0; p < size_; ++p)
            if (!want[p].empty() || !out[p].empty()) fail("no progress within GMT_CTL_TIMEOUT_S", p);
        }
        continue;
      }
      for (size_t i = 0; i < pf.size(); ++i) {
        const int p = who[i];
        if (pf[i].revents & (POLLERR | POLLNVAL)) fail("socket error", p);
        if ((pf[i].revents & POLLOUT) && !out[p].empty()) {
          Out& o = out[p].front();
          if (o.hdr_done < sizeof(Header)) {
            const ssize_t k = ::send(fd_[p], reinterpret_cast<char*>(&o.h) + o.hdr_done, sizeof(Header) - o.hdr_done,
                                     MSG_NOSIGNAL | MSG_DONTWAIT);
            if (k < 0 && errno != EAGAIN && errno != EINTR) fail("send", p);
            if (k > 0) o.hdr_done += static_cast<size_t>(k), t_last = now_s();
          }
          if (o.hdr_done == sizeof(Header) && o.done < o.h.bytes) {
            const ssize_t k = ::send(fd_[p], o.buf + o.done, o.h.bytes - o.done, MSG_NOSIGNAL | MSG_DONTWAIT);
            if (k < 0 && errno != EAGAIN && errno != EINTR) fail("send", p);
            if (k > 0) o.done += static_cast<size_t>(k), t_last = now_s();
          }
          if (o.hdr_done == sizeof(Header) && o.done == o.h.bytes) {
            out[p].pop_front();
            --pending;
          }
        }
        if (pf[i].revents & (POLLIN | POLLHUP)) {
          In& m = in_[p];
          for (;;) {  // read as much as is there
            if (m.hdr_done < sizeof(Header)) {
              const ssize_t k = ::recv(fd_[p], reinterpret_cast<char*>(&m.h) + m.hdr_done,
                                       sizeof(Header) - m.hdr_done, MSG_DONTWAIT);
              if (k == 0) {  // orderly shutdown: an error only if we still need this peer
                if (m.hdr_done) fail("peer closed the connection inside a message", p);
                closed_[p] = true;
                break;
              }
              if (k < 0) {
                if (errno != EAGAIN && errno != EINTR) fail("recv", p);
                break;
              }
              m.hdr_done += static_cast<size_t>(k);
              t_last = now_s();
              if (m.hdr_done < sizeof(Header)) continue;
              if (m.h.magic != kMagic) fail("corrupt message header", p);
              m.body.assign(m.h.bytes, 0);
              m.done = 0;
            }
            if (m.done < m.h.bytes) {
              const ssize_t k = ::recv(fd_[p], m.body.data() + m.done, m.h.bytes - m.done, MSG_DONTWAIT);
              if (k == 0) fail("peer closed the connection", p);
              if (k < 0) {
                if (errno != EAGAIN && errno != EINTR) fail("recv", p);
                break;
              }
              m.done += static_cast<size_t>(k);
              t_last = now_s();
            }
            if (m.done == m.h.bytes) {
              if (deliver(want[p], m.h.tag, m.body, rank_, p))
                --pending;
              else
                m.early[m.h.tag].push_back(std::move(m.body));
              m.hdr_done = 0;
              m.done = 0;
              m.body.clear();
            }
          }
        }
      }
    }
  }

  std::vector<int> fd_;
  std::vector<In> in_;
  std::vector<bool> closed_;
  double timeout_ = 300.0;
};

}  // namespace

// id = "gmtctl-<pid>-<name nonce>-<secret>": the abstract socket names use
// only the part before the secret (they are visible to every local user in
// /proc/net/unix); every hello carries the secret, which only the job's
// ranks received (over the launcher's own channel)
void make_socket_control_id(char* id) {
  std::memset(id, 0, kControlIdBytes);
  std::random_device rd;
  auto r64 = [&] { return (static_cast<unsigned long long>(rd()) << 32) ^ rd(); };
  const unsigned long long n = r64(), s0 = r64(), s1 = r64();
  std::snprintf(id, kControlIdBytes, "gmtctl-%d-%016llx-%016llx%016llx", static_cast<int>(getpid()), n, s0, s1);
}

std::unique_ptr<Control> make_socket_control(int rank, int size, const char* id) {
  return std::make_unique<SocketControl>(rank, size, id);
}

}  // namespace comm
}  // namespace gmt
