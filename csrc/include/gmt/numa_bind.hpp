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

// ---- rank pinning (default on the GPU backend; GMT_PIN=0: off)
//
// Round 5 traced the host-staged exchange's bimodal slow mode to unpinned
// ranks: `mpirun -bind-to core` removed it in 12 of 12 runs
// (profiles/r05_xport/README.md).  The reference's Summit launch binds its
// resource sets the same way (summit/run.sh:30: jsrun).  So every rank pins
// itself to ONE physical core (all its hardware threads) near its GPU:
//   * the candidate CPUs are the GPU's NUMA node's CPUs within the allowed
//     set (a launcher's binding is only ever narrowed, never widened), all
//     allowed CPUs when the node is unknown or the intersection is empty;
//   * the ranks whose GPUs share that node take consecutive physical cores
//     of it in local-rank order — like `-bind-to core`, which put two ranks
//     on neighbouring cores (one CCD, one L3).  Spreading them over the node
//     instead halved the host-staged exchange: 7.1-7.6 GB/s per rank
//     against 14.9-15.6 unpinned (profiles/r06_pin/);
//   * nothing changes when the allowed set is already one core.
// node_of_rank[i]: the NUMA node of local rank i's GPU (-1 unknown).
// Returns the first CPU of the core pinned to, or -1 (nothing changed).
inline bool cpu_siblings(int cpu, cpu_set_t* set) {
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", cpu);
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  char buf[256] = {0};
  const bool got = std::fgets(buf, sizeof(buf), f) != nullptr;
  std::fclose(f);
  return got && parse_cpulist(buf, set);
}

inline bool node_cpus(int node, cpu_set_t* set) {
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  char buf[4096] = {0};
  const bool got = std::fgets(buf, sizeof(buf), f) != nullptr;
  std::fclose(f);
  return got && parse_cpulist(buf, set);
}

inline int pci_numa_node(int pci_domain, int pci_bus, int pci_device) {
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node", pci_domain, pci_bus,
                pci_device);
  return read_int_file(path, -1);
}

inline int set_all_threads_affinity(const cpu_set_t& want) {
  DIR* d = opendir("/proc/self/task");
  if (!d) return sched_setaffinity(0, sizeof(want), &want) == 0 ? 1 : 0;
  int bound = 0;
  while (dirent* e = readdir(d)) {
    const int tid = std::atoi(e->d_name);
    if (tid > 0 && sched_setaffinity(tid, sizeof(want), &want) == 0) ++bound;
  }
  closedir(d);
  return bound;
}

inline int pin_rank_core(int local_rank, int local_size, const int* node_of_rank) {
  cpu_set_t allowed;
  if (local_rank < 0 || local_rank >= local_size || sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return -1;
  // GMT_PIN_NEAR=0 (A/B): consecutive cores from the start of the allowed
  // set, whatever the GPU's node (what `mpirun -bind-to core` does)
  static const bool near_only = [] {
    const char* e = std::getenv("GMT_PIN_NEAR");
    return !(e && e[0] == '0');
  }();
  const int node = near_only ? node_of_rank[local_rank] : -1;
  cpu_set_t cand = allowed;
  if (node >= 0) {
    cpu_set_t near, both;
    if (node_cpus(node, &near)) {
      CPU_AND(&both, &near, &allowed);
      if (CPU_COUNT(&both) > 0) cand = both;
    }
  }
  // physical cores of the candidates: the first allowed CPU of each SMT
  // sibling set.  A sibling list wider than 4 is not an SMT group (a
  // virtualised topology reported 32: pinning two ranks to "cores" 0 and 32
  // put them 32 CPUs apart and halved the host-staged exchange,
  // profiles/r06_pin/): each CPU is then a core of its own.
  auto siblings = [](int c, cpu_set_t* sib) {
    if (!cpu_siblings(c, sib) || CPU_COUNT(sib) > 4 || !CPU_ISSET(c, sib)) {
      CPU_ZERO(sib);
      CPU_SET(c, sib);
    }
  };
  int cores[CPU_SETSIZE];
  int nc = 0;
  cpu_set_t seen;
  CPU_ZERO(&seen);
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &cand) || CPU_ISSET(c, &seen)) continue;
    cpu_set_t sib;
    siblings(c, &sib);
    for (int s = 0; s < CPU_SETSIZE; ++s)
      if (CPU_ISSET(s, &sib)) CPU_SET(s, &seen);
    cores[nc++] = c;
  }
  if (nc == 0) return -1;
  // this rank's index among the local ranks whose GPUs share its node
  int idx = 0;
  for (int r = 0; r < local_rank; ++r) idx += !near_only || node_of_rank[r] == node ? 1 : 0;
  const int core = cores[idx % nc];
  cpu_set_t want, sib;
  siblings(core, &sib);
  CPU_AND(&want, &sib, &allowed);
  if (CPU_COUNT(&want) == 0 || CPU_EQUAL(&want, &allowed)) return -1;
  return set_all_threads_affinity(want) > 0 ? core : -1;
}

// This process's node-local rank and rank count as the launcher exported
// them (hydra, Open MPI, torchrun, Slurm), for pinning BEFORE MPI_Init:
// false when none is set.
inline bool launcher_local_rank(int* rank, int* size) {
  static const char* const kVars[][2] = {{"MPI_LOCALRANKID", "MPI_LOCALNRANKS"},
                                         {"OMPI_COMM_WORLD_LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_SIZE"},
                                         {"LOCAL_RANK", "LOCAL_WORLD_SIZE"},
                                         {"SLURM_LOCALID", "SLURM_NTASKS_PER_NODE"}};
  for (const auto& v : kVars) {
    const char* r = std::getenv(v[0]);
    const char* n = std::getenv(v[1]);
    if (r && n && *r && *n) {
      *rank = std::atoi(r);
      *size = std::atoi(n);
      return *size > 0 && *rank >= 0 && *rank < *size;
    }
  }
  return false;
}

// GMT_PIN: "0" off, "1" on; unset: on for the GPU backend (default_on)
inline bool pin_enabled(bool default_on) {
  const char* e = std::getenv("GMT_PIN");
  if (!e || !*e) return default_on;
  return std::atoi(e) != 0;
}

}  // namespace gmt
