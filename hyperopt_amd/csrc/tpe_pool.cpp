// tpe_pool.cpp — resident worker threads of the host runtime (tpe_pool.h).
//
// A suggest's host work is a handful of per-label jobs of 5-30 us each, so the
// pool is built for latency: workers spin on a generation word for a while
// after their last job (a back-to-back suggest loop finds them awake), then
// sleep on a condition variable.  Jobs are claimed by compare-and-swap on a
// (generation << 32 | next index) word, so a worker that wakes late can never
// run a job of a generation it did not read the job function of.
#include "tpe_pool.h"

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/tpe_hip.h"

namespace {

constexpr int kMaxThreads = 16;

inline void cpu_relax() { __builtin_ia32_pause(); }

struct Pool {
  std::mutex busy;                          // held by the dispatching caller
  std::mutex m;                             // sleep / wake
  std::condition_variable cv;
  std::atomic<uint64_t> next{0};            // generation << 32 | next job index
  std::atomic<int> n{0};
  std::atomic<void (*)(void*, int)> fn{nullptr};
  std::atomic<void*> ctx{nullptr};
  std::atomic<uint32_t> stamp{0};           // generation whose fn / ctx / n are written (0: being written)
  std::atomic<int> left{0};                 // jobs of the current generation not yet returned
  std::atomic<int> sleepers{0};
  std::atomic<bool> stop{false};
  std::atomic<bool> retired{false};         // replaced by tpe_host_threads: dispatch nothing more to it
  std::atomic<int> refs{1};                 // holders: g_pool's slot + every get_pool caller not yet done
  uint32_t gen = 0;                         // dispatcher's generation counter
  int64_t spin_ns = 200000;
  std::vector<std::thread> th;
};

// claim and run jobs of generation `g` until none is left
void run_jobs(Pool* p, uint32_t g) {
  // (seqlock: the job fields are g's only if g's stamp is there before and after)
  if (p->stamp.load(std::memory_order_acquire) != g) return;
  void (*fn)(void*, int) = p->fn.load(std::memory_order_relaxed);
  void* ctx = p->ctx.load(std::memory_order_relaxed);
  const int n = p->n.load(std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_acquire);
  if (p->stamp.load(std::memory_order_relaxed) != g) return;
  uint64_t v = p->next.load(std::memory_order_acquire);
  for (;;) {
    if ((uint32_t)(v >> 32) != g || (int)(uint32_t)v >= n) return;
    if (!p->next.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel, std::memory_order_acquire)) continue;
    fn(ctx, (int)(uint32_t)v);
    p->left.fetch_sub(1, std::memory_order_acq_rel);
    v = p->next.load(std::memory_order_acquire);
  }
}

void worker(Pool* p) {
  uint32_t seen = (uint32_t)(p->next.load() >> 32);
  for (;;) {
    // spin for a while, then sleep until the generation moves
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t g = seen;
    int k = 0;
    while (!p->stop.load(std::memory_order_relaxed)) {
      g = (uint32_t)(p->next.load(std::memory_order_acquire) >> 32);
      if (g != seen) break;
      cpu_relax();
      if (++k == 256) {
        k = 0;
        if (std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() >
            p->spin_ns) {
          std::unique_lock<std::mutex> lk(p->m);
          p->sleepers.fetch_add(1);
          while (!p->stop.load() && (uint32_t)(p->next.load() >> 32) == seen) p->cv.wait(lk);
          p->sleepers.fetch_sub(1);
        }
      }
    }
    if (p->stop.load()) return;
    seen = g;
    run_jobs(p, g);
  }
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

std::mutex g_mu;                 // pool creation / teardown
Pool* g_pool = nullptr;
int g_threads = -1;              // total threads incl. the caller (-1: not yet read from the environment)

void after_fork_child() {        // the workers do not exist in the child: start over (the old pool leaks)
  new (&g_mu) std::mutex();
  g_pool = nullptr;
}

// drops one reference: the last holder frees the pool (its workers were
// joined when it was retired: the slot's reference is dropped after that)
void release(Pool* p) {
  if (p && p->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete p;
}

// joins the workers of a retired pool; a concurrent parallel_for that took its
// pointer from get_pool before the swap holds a reference and finds it retired
// under `busy`, so the pool is freed by whichever of them releases it last
void stop_pool(Pool* p) {
  {
    std::lock_guard<std::mutex> lk(p->m);
    p->stop.store(true);
  }
  p->cv.notify_all();
  for (auto& t : p->th) t.join();
  p->th.clear();
}

int total_threads() {            // under g_mu
  if (g_threads < 0) {
    static bool atfork = [] { return pthread_atfork(nullptr, nullptr, after_fork_child) == 0; }();
    (void)atfork;
    int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;                       // (the CPUs this process may run on, when restricted)
    if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) hw = std::min(hw, (int)CPU_COUNT(&set));
    // (16: a GPU's share of the host's CPUs; the large levels of configs 4 and 5
    // fit and pack their labels on them, a 4-label suggest uses what it needs;
    // ranks sharing the host under torchrun take their share of its CPUs)
    int dflt = 16;
    const int lws = env_int("LOCAL_WORLD_SIZE", 1);
    if (lws > 1) dflt = std::min(dflt, std::max(2, hw / lws));
    g_threads = std::min({env_int("TPE_HOST_THREADS", dflt), hw, kMaxThreads});
  }
  return g_threads;
}

Pool* get_pool() {
  std::lock_guard<std::mutex> lk(g_mu);
  const int t = total_threads();
  if (t <= 1) return nullptr;
  if (!g_pool) {
    Pool* p = new Pool();
    p->spin_ns = (int64_t)std::max(0, env_int("TPE_POOL_SPIN_US", 200)) * 1000;
    for (int i = 0; i < t - 1; ++i) p->th.emplace_back(worker, p);
    g_pool = p;
  }
  g_pool->refs.fetch_add(1, std::memory_order_relaxed);     // (the caller's; release() when done)
  return g_pool;
}

}  // namespace

namespace tpe_pool {

void parallel_for(int n, void (*fn)(void*, int), void* ctx) {
  Pool* const held = n >= 2 ? get_pool() : nullptr;
  Pool* p = held;
  std::unique_lock<std::mutex> own;
  if (p) {
    own = std::unique_lock<std::mutex>(p->busy, std::try_to_lock);
    if (!own.owns_lock()) {
      p = nullptr;
    } else if (p->retired.load()) {                 // replaced since get_pool: run here
      own.unlock();
      p = nullptr;
    }
  }
  if (!p) {
    for (int i = 0; i < n; ++i) fn(ctx, i);
    release(held);
    return;
  }
  uint32_t g = ++p->gen;
  if (g == 0) g = p->gen = 1;                       // (0 marks a job being written)
  p->stamp.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  p->fn.store(fn, std::memory_order_relaxed);
  p->ctx.store(ctx, std::memory_order_relaxed);
  p->n.store(n, std::memory_order_relaxed);
  p->left.store(n, std::memory_order_relaxed);
  p->stamp.store(g, std::memory_order_release);
  p->next.store((uint64_t)g << 32);                 // publishes the job (seq_cst)
  if (p->sleepers.load()) {
    { std::lock_guard<std::mutex> lk(p->m); }
    p->cv.notify_all();
  }
  run_jobs(p, g);
  while (p->left.load(std::memory_order_acquire) > 0) cpu_relax();
  own.unlock();
  release(held);
}

int workers() {
  std::lock_guard<std::mutex> lk(g_mu);
  return std::max(0, total_threads() - 1);
}

}  // namespace tpe_pool

extern "C" int tpe_host_threads(int32_t n, int32_t* previous) {
  if (n > kMaxThreads) return TPE_E_ARG;
  Pool* old = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    const int prev = total_threads();
    if (previous) *previous = prev;
    if (n < 0) return TPE_OK;                        // query only
    if (n != prev) {
      old = g_pool;
      g_pool = nullptr;
      g_threads = std::max(1, (int)n);
    }
  }
  if (old) {
    {
      std::lock_guard<std::mutex> busy(old->busy);   // a dispatch in flight finishes first
      old->retired.store(true);                      // later dispatchers holding `old` run serially
    }
    stop_pool(old);
    release(old);                                    // (g_pool's reference)
  }
  return TPE_OK;
}
