// plan_model — the temporal-blocking kernel's segment planner, on the host.
//
// Prints the segment plan plan_segments<K> (csrc/kernels/jacobi5tb.hpp)
// picks for a domain and halo mask, with the makespan model's terms: edge
// segments at Dirichlet rows, interior segments, the strip groups that reach
// a Dirichlet column, the workgroup count against the resident slots.  No
// GPU needed (the planner is host code; the resident-workgroup count is an
// argument, 1024 = 4 two-stage K = 20 workgroups per CU on 256 CUs).
//
//   build/bench/plan_model [ny nx mask [resident]] ...   (K = 20, one rect = the interior)
//   GMT_PLAN_PUSH=S: plan as an inline-halo pass pushing faces S (bits 1 W, 2 E, 4 S, 8 N)
#include <cstdio>
#include <cstdlib>

#include "jacobi5tb.hpp"

int main(int argc, char** argv) {
  struct Case {
    int64_t ny, nx;
    int mask;
    int64_t resident;
  };
  std::vector<Case> cases;
  for (int i = 1; i + 2 < argc; i += 4)
    cases.push_back({std::atoll(argv[i]), std::atoll(argv[i + 1]), std::atoi(argv[i + 2]),
                     i + 3 < argc ? std::atoll(argv[i + 3]) : 1024});
  if (cases.empty())
    cases = {{32768, 32768, 0, 1024}, {32768, 32768, 15, 1024}, {8192, 8192, 0, 1024}, {8192, 8192, 15, 1024},
             {8192, 16384, 0, 1024},  {16384, 8192, 0, 1024},   {8192, 16384, 5, 1024}, {16384, 8192, 6, 1024}};
  constexpr int K = 20;
  using C = Cfg<K>;
  for (const Case& c : cases) {
    Args a{};
    a.nw = 1;
    a.n = 1;
    const int64_t x0 = 24, y0 = K;
    a.r[0][0] = x0;
    a.r[0][1] = c.nx;
    a.r[0][2] = y0;
    a.r[0][3] = c.ny;
    a.nstrip[0] = (c.nx + C::WOUT - 1) / C::WOUT;
    a.dom[0] = x0;
    a.dom[1] = c.nx;
    a.dom[2] = y0;
    a.dom[3] = c.ny;
    a.mask = c.mask;
    const int64_t ld = (x0 + c.nx + K + 63) / 64 * 64;
    const int64_t lmax = std::min<int64_t>(1 << 20, (int64_t(1) << 31) / (ld * 8) - 3 * K - C::LAG - 2 * C::U - C::P);
    const char* ps = std::getenv("GMT_PLAN_PUSH");
    const SegPlan p = plan_segments<K>(a, 0, lmax, c.resident, 0, -1, 0, 0, ps ? std::atoi(ps) : 0);
    const int64_t g = a.nstrip[0], nb = g < 2 ? g : 2;
    const int64_t wgs = g * ((p.e0[0] > 0) + (p.e1[0] > 0)) + nb * p.nmid_b[0] + (g - nb) * p.nmid[0];
    std::printf("%6lld x %6lld mask %2d: edges %lld / %lld rows, interior %lld x %lld rows, rule groups %lld x %lld rows, "
                "%lld workgroups on %lld slots\n",
                (long long)c.ny, (long long)c.nx, c.mask, (long long)p.e0[0], (long long)p.e1[0], (long long)p.nmid[0],
                (long long)p.lmid[0], (long long)p.nmid_b[0], (long long)p.lmid_b[0], (long long)wgs,
                (long long)c.resident);
  }
  return 0;
}
