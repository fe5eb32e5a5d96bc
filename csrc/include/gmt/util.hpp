// gmt/util.hpp — timers, statistics, roctx ranges, CLI parsing, JSON records.
//
// Reference: MPI_Wtime and clock_gettime(CLOCK_MONOTONIC) timers
// (mpi_daxpy_nvtx.cc:168,242-249,275-291,327; mpi_stencil2d_gt.cc:512-526),
// NVTX ranges + cudaProfilerStart/Stop (daxpy_nvtx.cu:65-105,
// mpi_daxpy_nvtx.cc:167-328) and positional argv parsing
// (mpi_stencil2d_gt.cc:660-665, mpi_stencil2d_sycl.cc:389-399).
// Added here: min/median/mean statistics, `--key=value` options next to the
// reference's positional arguments, and machine-readable JSON lines
// (`--json FILE`) for the bench runner.
#pragma once

#include <time.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "gmt/rt.h"
#include "gmt/watchdog.hpp"

namespace gmt {

inline double wtime() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1.0e-9;
}

struct Stats {
  std::vector<double> v;
  void add(double x) { v.push_back(x); }
  size_t n() const { return v.size(); }
  double sum() const {
    double s = 0;
    for (double x : v) s += x;
    return s;
  }
  double mean() const { return v.empty() ? 0.0 : sum() / v.size(); }
  double min() const { return v.empty() ? 0.0 : *std::min_element(v.begin(), v.end()); }
  double max() const { return v.empty() ? 0.0 : *std::max_element(v.begin(), v.end()); }
  double median() const {
    if (v.empty()) return 0.0;
    std::vector<double> s(v);
    std::sort(s.begin(), s.end());
    const size_t m = s.size() / 2;
    return s.size() % 2 ? s[m] : 0.5 * (s[m - 1] + s[m]);
  }
};

// RAII roctx range (NVTX nvtxRangePushA/Pop equivalent).  Names are kept
// identical to the reference's NVTX ranges for cross-platform comparison.
struct TraceRange {
  explicit TraceRange(const char* name) { gmt_trace_push(name); }
  ~TraceRange() { gmt_trace_pop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

// Positional arguments (reference CLI) + GNU-style long options.
struct Cli {
  std::vector<std::string> pos;
  std::map<std::string, std::string> opt;

  Cli(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
        const size_t eq = a.find('=');
        if (eq == std::string::npos) {
          // "--flag": a bare option never consumes the next token, so the
          // reference's positional arguments stay unambiguous
          opt[a.substr(2)] = "1";
        } else {
          opt[a.substr(2, eq - 2)] = a.substr(eq + 1);
        }
      } else {
        pos.push_back(a);
      }
    }
    // every app accepts --timeout=S: hang watchdog (gmt/watchdog.hpp)
    if (has("timeout")) watchdog_set_timeout(getd("timeout", 0.0));
  }
  bool has(const std::string& k) const { return opt.count(k) != 0; }
  std::string get(const std::string& k, const std::string& d) const {
    auto it = opt.find(k);
    return it == opt.end() ? d : it->second;
  }
  long long geti(const std::string& k, long long d) const {
    auto it = opt.find(k);
    return it == opt.end() ? d : std::atoll(it->second.c_str());
  }
  double getd(const std::string& k, double d) const {
    auto it = opt.find(k);
    return it == opt.end() ? d : std::atof(it->second.c_str());
  }
  bool flag(const std::string& k) const {
    auto it = opt.find(k);
    return it != opt.end() && it->second != "0";
  }
  const char* positional(size_t i) const { return i < pos.size() ? pos[i].c_str() : nullptr; }
};

// One flat JSON object per line, appended to a file (bench runner input).
class JsonRecord {
 public:
  JsonRecord& add(const std::string& k, const std::string& v) {
    std::string e;
    for (char c : v) {
      if (c == '"' || c == '\\') e += '\\';
      e += c;
    }
    items_.push_back("\"" + k + "\": \"" + e + "\"");
    return *this;
  }
  JsonRecord& add(const std::string& k, const char* v) { return add(k, std::string(v)); }
  JsonRecord& add(const std::string& k, double v) {
    char b[64];
    if (std::isfinite(v))
      std::snprintf(b, sizeof(b), "%.9g", v);
    else
      std::snprintf(b, sizeof(b), "null");
    items_.push_back("\"" + k + "\": " + b);
    return *this;
  }
  JsonRecord& add(const std::string& k, long long v) {
    items_.push_back("\"" + k + "\": " + std::to_string(v));
    return *this;
  }
  JsonRecord& add(const std::string& k, int v) { return add(k, static_cast<long long>(v)); }
  JsonRecord& add(const std::string& k, size_t v) { return add(k, static_cast<long long>(v)); }
  JsonRecord& add(const std::string& k, bool v) {
    items_.push_back("\"" + k + "\": " + (v ? "true" : "false"));
    return *this;
  }
  std::string str() const {
    std::string s = "{";
    for (size_t i = 0; i < items_.size(); ++i) s += (i ? ", " : "") + items_[i];
    return s + "}";
  }
  void append_to(const std::string& path) const {
    if (path.empty()) return;
    FILE* f = std::fopen(path.c_str(), "a");
    if (!f) return;
    std::fprintf(f, "%s\n", str().c_str());
    std::fclose(f);
  }

 private:
  std::vector<std::string> items_;
};

}  // namespace gmt
