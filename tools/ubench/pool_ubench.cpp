// Dispatch cost of the host worker pool (hyperopt_amd/csrc/tpe_pool.cpp):
// parallel_for of n jobs that each spin for `work_ns`, back to back, median
// wall time per call.  Build (host only):
//   g++ -O2 -std=c++17 -I include tools/ubench/pool_ubench.cpp hyperopt_amd/csrc/tpe_pool.cpp -pthread -o /tmp/pool_ubench
// Usage: TPE_HOST_THREADS=16 /tmp/pool_ubench [work_ns]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../hyperopt_amd/csrc/tpe_pool.h"

namespace {
using clk = std::chrono::steady_clock;

struct Ctx { int64_t work_ns; };

void job(void* c, int) {
  const int64_t ns = ((Ctx*)c)->work_ns;
  const auto t0 = clk::now();
  while (std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count() < ns) {
  }
}
}  // namespace

int main(int argc, char** argv) {
  Ctx c{argc > 1 ? atoll(argv[1]) : 0};
  for (int n : {2, 4, 8, 10, 16, 32, 64, 256, 1000}) {
    std::vector<double> t;
    for (int it = 0; it < 3000; ++it) {
      const auto a = clk::now();
      tpe_pool::parallel_for(n, job, &c);
      t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
      // a short host gap between dispatches, as between a suggest's phases
      const auto g = clk::now();
      while (std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - g).count() < 5000) {
      }
    }
    std::sort(t.begin() + 500, t.end());
    const size_t m = 500 + (t.size() - 500) / 2, p9 = 500 + (t.size() - 500) * 9 / 10;
    printf("n %3d work %5lld ns: median %7.2f us  p90 %7.2f us  (ideal %.2f)\n", n, (long long)c.work_ns, t[m], t[p9],
           1e-3 * c.work_ns * ((n + tpe_pool::workers()) / (tpe_pool::workers() + 1)));
  }
  return 0;
}
