// gmt/numa_bind.hpp — run a rank on the CPUs of its GPU's NUMA node.
//
// An MI355X node has two sockets, four GPUs on each (numa_node of the PCI
// device).  A rank that floats to the other socket reaches its GPU, and the
// pinned staging buffers it allocates, over the socket link.  The host-staged
// exchange runs at 7 or 16 GB/s per rank from run to run; this header tests
// whether rank placement is the cause.
// bind_numa_near() sets every thread of the process to the node's CPUs
// (intersected with the allowed set), before the transport allocates its
// buffers, so first-touch and pinned pages land on the GPU's side too.
// Measured neutral: the slow mode shows up with and without the binding
// (profiles/r04_xport/README.md), so it is opt-in: GMT_NUMA_BIND=1.  Linux
// sysfs only; a missing node (-1) or an empty intersection change nothing.
#pragma once

#include <dirent.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace gmt {

// "0-63,128-191" -> set; false on a malformed list
inline bool parse_cpulist(const char* s, cpu_set_t* set) {
  CPU_ZERO(set);
  while (*s && *s != '\n') {
    char* end = nullptr;
    const long a = std::strtol(s, &end, 10);
    if (end == s || a < 0) return false;
    long b = a;
    s = end;
    if (*s == '-') {
      b = std::strtol(s + 1, &end, 10);
      if (end == s + 1 || b < a) return false;
      s = end;
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(static_cast<int>(c), set);
    if (*s == ',') ++s;
  }
  return true;
}

inline int read_int_file(const char* path, int fallback) {
  FILE* f = std::fopen(path, "r");
  if (!f) return fallback;
  int v = fallback;
  if (std::fscanf(f, "%d", &v) != 1) v = fallback;
  std::fclose(f);
  return v;
}

// Returns the node bound to, or -1 (nothing changed).
inline int bind_numa_near(int pci_domain, int pci_bus, int pci_device) {
  const char* env = std::getenv("GMT_NUMA_BIND");
  if (!env || std::atoi(env) == 0) return -1;
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node", pci_domain, pci_bus,
                pci_device);
  const int node = read_int_file(path, -1);
  if (node < 0) return -1;
  std::snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  char buf[4096] = {0};
  const bool got = std::fgets(buf, sizeof(buf), f) != nullptr;
  std::fclose(f);
  cpu_set_t near, allowed, want;
  if (!got || !parse_cpulist(buf, &near) || sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return -1;
  CPU_AND(&want, &near, &allowed);
  if (CPU_COUNT(&want) == 0 || CPU_EQUAL(&want, &allowed)) return CPU_COUNT(&want) ? node : -1;
  // every existing thread (runtime helpers included); threads started later inherit
  DIR* d = opendir("/proc/self/task");
  if (!d) return sched_setaffinity(0, sizeof(want), &want) == 0 ? node : -1;
  int bound = 0;
  while (dirent* e = readdir(d)) {
    const int tid = std::atoi(e->d_name);
    if (tid > 0 && sched_setaffinity(tid, sizeof(want), &want) == 0) ++bound;
  }
  closedir(d);
  return bound > 0 ? node : -1;
}

}  // namespace gmt
