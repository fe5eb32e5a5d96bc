// gmt/watchdog.hpp — hang detection and fault injection for the native apps.
//
// The reference has no failure detection: a lost message leaves every rank
// blocked in MPI_Waitall forever (mpi_stencil2d_gt.cc:229-246), and the
// SURVEY (§5.3) asks the rebuild to stay fail-fast and optionally add "a
// --timeout watchdog thread for hung exchanges".
//
// Watchdog: a detached thread that aborts the whole job (abort_job ->
// MPI_Abort in the MPI apps) when the process makes no progress for
// `timeout` seconds.  Progress points call watchdog_kick(phase): every
// completed halo exchange, every engine step, every app phase.  The abort
// message names rank, host, device and the last phase reached, so a hung
// exchange is attributed to the rank that stopped.  Armed by `--timeout=S`
// on any app command line or GMT_TIMEOUT=S in the environment (the larger
// wins); off by default.
//
// Fault injection: GMT_INJECT_HANG=R[:N] makes rank R stop forever at its
// (N+1)-th halo exchange (default N = 0) — the test for the watchdog and for
// the job-wide teardown (tests/test_native_apps.py).
#pragma once

#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "gmt/check.hpp"

namespace gmt {

struct WatchdogState {
  std::atomic<double> last{0.0};
  std::atomic<const char*> phase{"startup"};
  std::atomic<bool> armed{false};
  double timeout = 0.0;   // seconds; set from the command line / env
  int rank = -1, device = -1;
  long long hang_rank = -2, hang_after = 0;  // fault injection
  std::atomic<long long> exchanges{0};
  // Last words (watchdog_set_epitaph): a JSON object written to stdout, with
  // a "watchdog" field naming the stall, before the process exits with
  // epitaph_code instead of 124 — a result already measured is not lost to a
  // later phase that hangs.  Empty text: exit with the code, print nothing.
  std::atomic<const char*> epitaph{nullptr};
  std::atomic<int> epitaph_code{124};
};

// intentionally leaked: the detached thread may outlive static destruction
inline WatchdogState& watchdog_state() {
  static WatchdogState* s = [] {
    auto* w = new WatchdogState;
    if (const char* e = std::getenv("GMT_TIMEOUT")) w->timeout = std::atof(e);
    if (const char* e = std::getenv("GMT_INJECT_HANG")) {
      w->hang_rank = std::atoll(e);
      if (const char* c = std::strchr(e, ':')) w->hang_after = std::atoll(c + 1);
    }
    return w;
  }();
  return *s;
}

inline double watchdog_now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1.0e-9;
}

// `--timeout=S` (parsed by Cli) raises the timeout; it never lowers the env's
inline void watchdog_set_timeout(double seconds) {
  WatchdogState& w = watchdog_state();
  if (seconds > w.timeout) w.timeout = seconds;
}

inline void watchdog_kick(const char* phase = nullptr) {
  WatchdogState& w = watchdog_state();
  if (phase) w.phase.store(phase, std::memory_order_relaxed);
  if (w.armed.load(std::memory_order_relaxed)) w.last.store(watchdog_now(), std::memory_order_relaxed);
}

// Arms the watchdog (no-op when no timeout is configured or already armed).
inline void watchdog_start(int rank, int device) {
  WatchdogState& w = watchdog_state();
  w.rank = rank;
  w.device = device;
  if (w.timeout <= 0.0 || w.armed.exchange(true)) return;
  w.last.store(watchdog_now());
  std::thread([&w] {
    const double period = w.timeout < 4.0 ? w.timeout / 4.0 : 1.0;
    for (;;) {
      timespec ts{static_cast<time_t>(period), static_cast<long>((period - static_cast<long>(period)) * 1e9)};
      nanosleep(&ts, nullptr);
      const double idle = watchdog_now() - w.last.load(std::memory_order_relaxed);
      if (idle > w.timeout) {
        char host[256] = "?";
        gethostname(host, sizeof(host) - 1);
        std::fprintf(stderr,
                     "GMT WATCHDOG: rank %d host %s device %d: no progress for %.1f s "
                     "(timeout %.1f s, last phase '%s'); aborting the job\n",
                     w.rank, host, w.device, idle, w.timeout, w.phase.load());
        if (const char* ep = w.epitaph.load()) {
          const size_t n = std::strlen(ep);
          const char* close = n ? std::strrchr(ep, '}') : nullptr;
          if (close) {
            // raw write(2): the main thread may hold stdio's lock
            char tail[512];
            const int m = std::snprintf(tail, sizeof(tail),
                                        "%s\"watchdog\": \"rank %d: no progress for %.1f s in phase '%s'\"}\n",
                                        close == ep + 1 ? "" : ", ", w.rank, idle, w.phase.load());
            ssize_t rc = write(1, ep, static_cast<size_t>(close - ep));
            rc = write(1, tail, static_cast<size_t>(m > 0 && m < static_cast<int>(sizeof(tail)) ? m : 0));
            (void)rc;
          }
          abort_job(w.epitaph_code.load());
        }
        abort_job(124);
      }
    }
  }).detach();
}

// Replaces the epitaph (a copy is kept; the previous one is leaked on
// purpose: the watchdog thread may be reading it).  nullptr: none, the
// watchdog exits 124 again.
inline void watchdog_set_epitaph(const char* json, int code) {
  WatchdogState& w = watchdog_state();
  w.epitaph_code.store(code);
  w.epitaph.store(json ? strdup(json) : nullptr);
}

// Fault injection point (halo exchange start): rank `hang_rank` stops here
// forever once it has completed `hang_after` exchanges.
inline void fault_point_exchange(int rank) {
  WatchdogState& w = watchdog_state();
  if (w.hang_rank != rank) {
    return;
  }
  if (w.exchanges.fetch_add(1) < w.hang_after) return;
  std::fprintf(stderr, "GMT FAULT INJECTION: rank %d hangs in the halo exchange\n", rank);
  std::fflush(stderr);
  for (;;) pause();
}

}  // namespace gmt
