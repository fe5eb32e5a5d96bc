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
//   build/bench/plan_model --check-bands: for every built K, a sweep of shares
//     and halo masks planned as band-first passes (row bands of g = 20 rows on
//     the halo row sides, the engine's JacobiSolver::band_rects): every row
//     band segment (the first / last interior segment of every strip group)
//     must hold at least the signalled rows, or its output wave never counts
//     its arrival and the pass never signals.  Exit 1 on a violation.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "jacobi5tb.hpp"

namespace {
// launch_tb's set-up of a one-rect pass over the interior, host side
template <int K>
bool check_bands(int64_t ny, int64_t nx, int mask, int64_t resident, int64_t g, bool verbose) {
  using C = Cfg<K>;
  Args a{};
  a.nw = std::min(tb_default_strips(K), tb_max_strips(K));
  a.n = 1;
  const int64_t x0 = 24, y0 = K;
  const int64_t r[4] = {x0, nx, y0, ny};
  for (int j = 0; j < 4; ++j) a.r[0][j] = a.dom[j] = r[j];
  a.nstrip[0] = (nx + C::WOUT - 1) / C::WOUT;
  if (a.nw > a.nstrip[0]) a.nw = static_cast<int>(a.nstrip[0]);
  a.mask = mask;
  const int rbs = (mask & 4) ? 1 : 0, rbn = (mask & 8) ? 1 : 0, rb = rbs + rbn;
  if (rb == 0 || ny < rb * std::max<int64_t>(32, g) || ny < 64) return true;  // band_rects: no row bands
  const int64_t rb_min = std::max<int64_t>(32, g);
  const int64_t ld = (x0 + nx + K + 63) / 64 * 64;
  const int64_t lmax = std::min<int64_t>(1 << 20, (int64_t(1) << 31) / (ld * 8) - 3 * K - C::LAG - 2 * C::U - C::P);
  const SegPlan p = plan_segments<K>(a, 0, lmax, resident, 0, 0, rb, rb_min);
  const int64_t mid = ny - p.e0[0] - p.e1[0];
  // launch_tb's own feasibility rule (a plan it refuses fails loudly, not a hang)
  if ((rbs && p.e0[0] > 0) || (rbn && p.e1[0] > 0) || p.nmid[0] < rb || p.nmid_b[0] < rb ||
      mid / p.nmid[0] < g || mid / p.nmid_b[0] < g) {
    if (verbose)
      std::printf("K %2d %6lld x %6lld mask %2d: refused by launch_tb\n", K, (long long)ny, (long long)nx, mask);
    return true;
  }
  bool ok = true;
  for (int bnd = 0; bnd < 2; ++bnd) {
    const int64_t nm = bnd ? p.nmid_b[0] : p.nmid[0], lm = bnd ? p.lmid_b[0] : p.lmid[0];
    // tb_block: segment m covers rows [mid m / nm, mid (m + 1) / nm) of the
    // interior part; S band m = 0, N band m = nm - 1
    const int64_t first = mid / nm, last = mid - (nm - 1) * mid / nm;
    if ((rbs && first < g) || (rbn && last < g) || last < 1) {
      ok = false;
      std::printf("K %2d %6lld x %6lld mask %2d: %s groups: %lld segments of %lld rows over %lld: S band %lld, "
                  "N band %lld rows < %lld signalled\n",
                  K, (long long)ny, (long long)nx, mask, bnd ? "boundary" : "inner", (long long)nm, (long long)lm,
                  (long long)mid, (long long)first, (long long)last, (long long)g);
    }
  }
  if (verbose && ok)
    std::printf("K %2d %6lld x %6lld mask %2d: ok (e %lld/%lld mid %lld x %lld bnd %lld x %lld)\n", K, (long long)ny,
                (long long)nx, mask, (long long)p.e0[0], (long long)p.e1[0], (long long)p.nmid[0], (long long)p.lmid[0],
                (long long)p.nmid_b[0], (long long)p.lmid_b[0]);
  return ok;
}

template <int K>
int sweep_bands(bool verbose) {
  int bad = 0;
  const int64_t sizes[] = {96, 157, 313, 640, 1000, 2048, 4096, 4100, 8192, 12345, 16384};
  const int masks[] = {4, 8, 12, 5, 6, 9, 10, 13, 14, 15};
  for (int64_t ny : sizes)
    for (int64_t nx : {850, 4096, 8192, 16384})
      for (int m : masks)
        for (int64_t res : {1024, 2048, 512})
          if (!check_bands<K>(ny, nx, m, res, 20, verbose)) ++bad;
  return bad;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "--check-swizzle") == 0) {
    // tail_swizzle is a permutation of the tiles wherever tail_swizzle_ok holds
    int bad = 0, checked = 0;
    for (int64_t nb = 2; nb < 4000; nb += (nb < 200 ? 1 : 37))
      for (int64_t ne = 1; ne < nb; ne += (ne < 40 ? 1 : 13)) {
        if (!tail_swizzle_ok(nb, ne)) continue;
        std::vector<char> seen(nb, 0);
        for (int64_t b = 0; b < nb; ++b) {
          const int64_t t = tail_swizzle(b, nb, ne);
          if (t < 0 || t >= nb || seen[t]++) { ++bad; break; }
        }
        ++checked;
      }
    std::printf("tail_swizzle: %d of %d launch shapes not a permutation\n", bad, checked);
    return bad ? 1 : 0;
  }
  if (argc > 1 && std::strcmp(argv[1], "--check-bands") == 0) {
    const bool v = argc > 2;
    int bad = 0;
    bad += sweep_bands<2>(v) + sweep_bands<3>(v) + sweep_bands<4>(v) + sweep_bands<5>(v) + sweep_bands<6>(v);
    bad += sweep_bands<7>(v) + sweep_bands<8>(v) + sweep_bands<9>(v) + sweep_bands<10>(v) + sweep_bands<12>(v);
    bad += sweep_bands<14>(v) + sweep_bands<16>(v) + sweep_bands<18>(v) + sweep_bands<20>(v);
    std::printf("band plans: %d violations\n", bad);
    return bad ? 1 : 0;
  }
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
  // GMT_PLAN_SH=1: the shared hand-off group launch (Sh<K>, one 8-wave
  // workgroup per CU: 256 slots unless given)
  const bool sh = std::getenv("GMT_PLAN_SH") && std::atoi(std::getenv("GMT_PLAN_SH")) != 0;
  for (Case c : cases) {
    if (sh && c.resident == 1024) c.resident = 256;
    Args a{};
    a.nw = sh ? Sh<K>::NW : 1;
    a.sh = sh ? 1 : 0;
    a.col_keep = 1;
    a.n = 1;
    const int64_t x0 = 24, y0 = K;
    a.r[0][0] = x0;
    a.r[0][1] = c.nx;
    a.r[0][2] = y0;
    a.r[0][3] = c.ny;
    a.nstrip[0] = sh ? Sh<K>::NW * ((c.nx + Sh<K>::GOUT - 1) / Sh<K>::GOUT) : (c.nx + C::WOUT - 1) / C::WOUT;
    a.dom[0] = x0;
    a.dom[1] = c.nx;
    a.dom[2] = y0;
    a.dom[3] = c.ny;
    a.mask = c.mask;
    const int64_t ld = (x0 + c.nx + K + 63) / 64 * 64;
    const int64_t lmax = std::min<int64_t>(1 << 20, (int64_t(1) << 31) / (ld * 8) - 3 * K - C::LAG - 2 * C::U - C::P);
    const char* ps = std::getenv("GMT_PLAN_PUSH");
    const SegPlan p = plan_segments<K>(a, 0, lmax, c.resident, 0, -1, 0, 0, ps ? std::atoi(ps) : 0);
    const int64_t g = (a.nstrip[0] + a.nw - 1) / a.nw, nb = g < 2 ? g : 2;
    const int64_t wgs = g * ((p.e0[0] > 0) + (p.e1[0] > 0)) + nb * p.nmid_b[0] + (g - nb) * p.nmid[0];
    std::printf("%6lld x %6lld mask %2d: edges %lld / %lld rows, interior %lld x %lld rows, rule groups %lld x %lld rows, "
                "%lld workgroups on %lld slots%s\n",
                (long long)c.ny, (long long)c.nx, c.mask, (long long)p.e0[0], (long long)p.e1[0], (long long)p.nmid[0],
                (long long)p.lmid[0], (long long)p.nmid_b[0], (long long)p.lmid_b[0], (long long)wgs,
                (long long)c.resident, p.tail ? ", edges last" : "");
  }
  return 0;
}
