// tpe_pool.cpp — resident worker threads of the host runtime (tpe_pool.h).
//
// A suggest's host work is a handful of per-label jobs of 1-30 us each, so the
// pool is built for dispatch latency: workers spin on a control word for a while
// after their last job (a back-to-back suggest loop finds them awake), then
// sleep on a condition variable.  A dispatch touches few shared cache lines:
// the caller publishes the job and, in the same 64-bit control word, its
// generation and the set of PARTICIPANTS — itself and the workers that are
// awake (spinning), at most one per job.  Participant r runs job r straight
// away (no claim) and reports completion in its own cache line.  The jobs past
// the participants' (a wide dispatch: a thousand labels' fits) are claimed by
// compare-and-swap on a word that carries the generation and the job count —
// by the participants and by every other worker, the ones woken from sleep
// included — and counted down as they return.  A generation cannot end before
// every participant has reported and every claimed job has returned, so no
// worker ever runs a job of a generation it was not given.
#include "tpe_pool.h"

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/tpe_hip.h"

namespace {

constexpr int kMaxThreads = 16;          // caller + 15 workers (participant masks: bits 1..15)

inline void cpu_relax() { __builtin_ia32_pause(); }

struct alignas(64) Slot {
  std::atomic<uint32_t> done{0};         // the last generation this worker finished as a participant
  std::atomic<int> awake{0};             // spinning (1) or about to sleep / asleep (0)
};

struct Pool {
  std::mutex busy;                          // held by the dispatching caller
  std::mutex m;                             // sleep / wake
  std::condition_variable cv;
  // the job and its control word share one cache line: a worker that sees the
  // new generation has the job's fields with it
  alignas(64) std::atomic<uint64_t> ctl{0}; // generation << 32 | participant mask (bit w: worker w)
  void (*fn)(void*, int) = nullptr;
  void* ctx = nullptr;
  int n = 0;
  int n_part = 0;                           // participants, the caller included
  // the jobs past the participants' first ones, claimed by compare-and-swap on
  // (generation mod 2^24, job count, next job) — by the participants and by any
  // other worker, awake or woken, so a wide dispatch uses every thread; a claim
  // can only succeed while its generation's jobs are not all taken
  alignas(64) std::atomic<uint64_t> next{0};
  alignas(64) std::atomic<int> left{0};     // claimed jobs not yet returned
  alignas(64) std::atomic<int> sleepers{0};
  std::atomic<bool> stop{false};
  std::atomic<bool> retired{false};         // replaced by tpe_host_threads: dispatch nothing more to it
  std::atomic<int> refs{1};                 // holders: g_pool's slot + every get_pool caller not yet done
  uint32_t gen = 0;                         // dispatcher's generation counter
  int n_workers = 0;
  int64_t spin_ns = 200000;
  Slot slot[kMaxThreads];
  std::vector<std::thread> th;
};

constexpr int kJobBits = 20;                // jobs per dispatch < 2^20 (more: run serially)
inline uint64_t claim_word(uint32_t g, int n, int i) {
  return (uint64_t)(g & 0xFFFFFFu) << (2 * kJobBits) | (uint64_t)n << kJobBits | (uint64_t)i;
}

// claim and run the jobs of generation g past the participants' first ones, a
// guided share at a time (the remaining jobs / twice the threads, at least one):
// a thousand one-microsecond jobs (config 5's label fits and fills) would
// otherwise pass the claim word's cache line between the threads once a job
void claim_jobs(Pool* p, uint32_t g) {
  const int share = 2 * (p->n_workers + 1);
  uint64_t v = p->next.load(std::memory_order_acquire);
  for (;;) {
    if ((uint32_t)(v >> (2 * kJobBits)) != (g & 0xFFFFFFu)) return;
    const int i = (int)(v & ((1u << kJobBits) - 1)), n = (int)((v >> kJobBits) & ((1u << kJobBits) - 1));
    if (i >= n) return;
    const int b = std::max(1, (n - i) / share);
    if (!p->next.compare_exchange_weak(v, v + (uint64_t)b, std::memory_order_acq_rel, std::memory_order_acquire))
      continue;
    // (the claim holds the generation open: its job fields are current)
    for (int j = i; j < i + b; ++j) p->fn(p->ctx, j);
    p->left.fetch_sub(b, std::memory_order_acq_rel);
    v = p->next.load(std::memory_order_acquire);
  }
}

void worker(Pool* p, int id) {
  Slot& me = p->slot[id];
  uint32_t seen = (uint32_t)(p->ctl.load() >> 32);
  for (;;) {
    // spin for a while, then sleep until the generation moves
    me.awake.store(1);
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t c = 0;
    int k = 0;
    while (!p->stop.load(std::memory_order_relaxed)) {
      c = p->ctl.load(std::memory_order_acquire);
      if ((uint32_t)(c >> 32) != seen) break;
      cpu_relax();
      if (++k == 256) {
        k = 0;
        if (std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() >
            p->spin_ns) {
          me.awake.store(0);                // (seq_cst: before the generation check under the lock)
          std::unique_lock<std::mutex> lk(p->m);
          p->sleepers.fetch_add(1);
          while (!p->stop.load() && (uint32_t)(p->ctl.load() >> 32) == seen) p->cv.wait(lk);
          p->sleepers.fetch_sub(1);
          lk.unlock();
          me.awake.store(1);
        }
      }
    }
    if (p->stop.load()) return;
    const uint32_t g = (uint32_t)(c >> 32);
    const uint32_t mask = (uint32_t)c;
    seen = g;
    if (mask >> id & 1) {
      // a participant: its own job (the job fields were written before the
      // control word; they stay until every participant has reported), then claims
      const int rank = 1 + __builtin_popcount(mask & ((1u << id) - 1));
      if (rank < p->n) p->fn(p->ctx, rank);
      claim_jobs(p, g);
      me.done.store(g, std::memory_order_release);
    } else {
      claim_jobs(p, g);                     // (nothing when every job has a participant)
    }
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

// CPUs the process's cgroup quota allows (cgroup v2 cpu.max, else v1
// cfs_quota_us / cfs_period_us), 0 when unlimited or unknown: a container's CPU
// share is a quota, which neither hardware_concurrency nor the affinity mask
// shows — and workers that spin past it are descheduled for a whole CFS period
// (the two-rank rehearsal's 80-ms steps)
int cgroup_cpus() {
  long long quota = -1, period = 0;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0) quota = atoll(q);
    fclose(f);
  } else if (FILE* g = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    if (fscanf(g, "%lld", &quota) != 1) quota = -1;
    fclose(g);
    if (FILE* h = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (fscanf(h, "%lld", &period) != 1) period = 0;
      fclose(h);
    }
  }
  if (quota <= 0 || period <= 0) return 0;
  return (int)std::max<long long>(1, quota / period);
}

int total_threads() {            // under g_mu
  if (g_threads < 0) {
    static bool atfork = [] { return pthread_atfork(nullptr, nullptr, after_fork_child) == 0; }();
    (void)atfork;
    int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;                       // (the CPUs this process may run on, when restricted)
    if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) hw = std::min(hw, (int)CPU_COUNT(&set));
    if (const int q = cgroup_cpus()) hw = std::min(hw, q);
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
    // (a lone rank's workers spin 2 ms: a wake from sleep costs the first
    // suggest after a pause ~60 us and the steady loop ~5 us of its p50 at 200 us
    // (tools/g15.sh); ranks sharing the host's CPU quota keep 200 us)
    const int spin_us = env_int("LOCAL_WORLD_SIZE", 1) > 1 ? 200 : 2000;
    p->spin_ns = (int64_t)std::max(0, env_int("TPE_POOL_SPIN_US", spin_us)) * 1000;
    p->n_workers = t - 1;
    for (int i = 1; i < t; ++i) p->th.emplace_back(worker, p, i);
    g_pool = p;
  }
  g_pool->refs.fetch_add(1, std::memory_order_relaxed);     // (the caller's; release() when done)
  return g_pool;
}

}  // namespace

namespace tpe_pool {

void parallel_for(int n, void (*fn)(void*, int), void* ctx) {
  // TPE_POOL_TRACE=1: every dispatch's job count and the participants it
  // found awake, on stderr (diagnostic)
  static const bool trace = [] { const char* e = getenv("TPE_POOL_TRACE"); return e && e[0] == '1'; }();
  if (trace) {
    int awake = 0;
    if (g_pool)
      for (int w = 1; w <= g_pool->n_workers; ++w) awake += g_pool->slot[w].awake.load(std::memory_order_relaxed);
    fprintf(stderr, "[tpe_pool] dispatch n=%d awake=%d\n", n, awake);
  }
  Pool* const held = n >= 2 && n < (1 << kJobBits) ? get_pool() : nullptr;
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
  if (g == 0) g = p->gen = 1;                       // (0: no generation yet)
  // participants: the caller and up to n - 1 awake workers
  uint32_t mask = 0;
  int part = 1;
  for (int w = 1; w <= p->n_workers && part < n; ++w)
    if (p->slot[w].awake.load(std::memory_order_relaxed)) { mask |= 1u << w; ++part; }
  p->fn = fn;
  p->ctx = ctx;
  p->n = n;
  p->n_part = part;
  p->left.store(n - part, std::memory_order_relaxed);
  p->next.store(claim_word(g, n, part), std::memory_order_relaxed);
  p->ctl.store((uint64_t)g << 32 | mask);           // publishes the job (seq_cst)
  if (p->sleepers.load()) {                         // (a participant may have gone to sleep; helpers)
    { std::lock_guard<std::mutex> lk(p->m); }
    p->cv.notify_all();
  }
  fn(ctx, 0);
  claim_jobs(p, g);
  for (int w = 1; w <= p->n_workers; ++w)
    if (mask >> w & 1)
      while (p->slot[w].done.load(std::memory_order_acquire) != g) cpu_relax();
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
