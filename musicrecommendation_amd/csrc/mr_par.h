// mr_par.h — host-side fork/join helpers for the index builders (TSV ingest,
// mr_load's transposes and tile-major CSR). Plain std::thread fan-out per
// phase: every phase is a bulk pass over tens of millions of entries, so a
// spawn (~30 us per thread) is noise next to it, and small inputs run inline.
#ifndef MR_PAR_H
#define MR_PAR_H

#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <new>
#include <thread>
#include <utility>
#include <vector>

namespace mr_par {

// Cores this process may really use: the affinity mask, capped by a cgroup v2
// CPU quota (on the GPU box hardware_concurrency() shows the whole machine
// while the job gets a 16-core share), then shared with the other ranks of a
// one-process-per-GPU launch on this node (torchrun's LOCAL_WORLD_SIZE: 8
// ranks on a 16-core share get 2 threads each, not 16 each) unless the
// launcher already pinned each rank to its own CPU set. MR_THREADS overrides.
inline int usable_cores() {
  static const int n = [] {
    if (const char* e = std::getenv("MR_THREADS")) {
      const int t = std::atoi(e);
      if (t > 0) return std::min(t, 256);
    }
    int local_ranks = 1;
    if (const char* e = std::getenv("LOCAL_WORLD_SIZE")) local_ranks = std::max(1, std::atoi(e));
    int aff = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) aff = CPU_COUNT(&set);
    int quota = 0;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long per = 0;
      if (std::fscanf(f, "%31s %lld", q, &per) == 2 && q[0] != 'm' && per > 0)
        quota = (int)std::max(1LL, std::atoll(q) / per);
      std::fclose(f);
    }
    int t = aff > 0 ? aff : 1;
    // the ranks share the node's cores only when this rank's mask covers the
    // whole share (the quota, else the machine); a launcher that pinned each
    // rank to its own CPU set already split them
    const int share = quota > 0 ? quota : (int)std::thread::hardware_concurrency();
    const bool shared_mask = t >= share;
    if (quota > 0) t = std::min(t, quota);
    if (shared_mask) t /= local_ranks;
    return std::max(1, std::min(t, 256));
  }();
  return n;
}

// f(lo, hi, worker) over [0, n) cut into at most `threads` contiguous ranges of
// at least `grain` items; inline when one range suffices.
template <class F>
void parallel_for(int64_t n, F&& f, int64_t grain = 1 << 16, int threads = 0) {
  if (n <= 0) return;
  int T = threads > 0 ? threads : usable_cores();
  T = (int)std::max<int64_t>(1, std::min<int64_t>(T, (n + grain - 1) / std::max<int64_t>(1, grain)));
  if (T == 1) {
    f((int64_t)0, n, 0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; ++t) th.emplace_back([&, t] { f(n * t / T, n * (t + 1) / T, t); });
  f((int64_t)0, n / T, 0);
  for (auto& x : th) x.join();
}

// f(i, worker) for i in [0, n), items handed out dynamically in blocks of
// `block` (for work of uneven cost per item, e.g. CSR rows of power-law length).
template <class F>
void parallel_dynamic(int64_t n, int64_t block, F&& f, int threads = 0) {
  if (n <= 0) return;
  int T = threads > 0 ? threads : usable_cores();
  T = (int)std::max<int64_t>(1, std::min<int64_t>(T, (n + block - 1) / block));
  std::atomic<int64_t> next{0};
  auto body = [&](int w) {
    for (;;) {
      const int64_t a = next.fetch_add(block, std::memory_order_relaxed);
      if (a >= n) break;
      const int64_t b = std::min(n, a + block);
      for (int64_t i = a; i < b; ++i) f(i, w);
    }
  };
  if (T == 1) {
    body(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; ++t) th.emplace_back(body, t);
  body(0);
  for (auto& x : th) x.join();
}

// Allocator that default-initialises (no zero fill: the builders write every
// element, in parallel) and asks for transparent huge pages on large blocks
// (one fault per 2 MB instead of per 4 KB for the 100-MB-class arrays).
template <class T>
struct fill_alloc {
  using value_type = T;
  fill_alloc() = default;
  template <class U>
  fill_alloc(const fill_alloc<U>&) {}
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes >= ((size_t)8 << 20)) {
      void* p = nullptr;
      if (posix_memalign(&p, (size_t)2 << 20, bytes) != 0) throw std::bad_alloc();
      (void)madvise(p, bytes, MADV_HUGEPAGE);
      return static_cast<T*>(p);
    }
    if (void* p = std::malloc(std::max<size_t>(1, bytes))) return static_cast<T*>(p);
    throw std::bad_alloc();
  }
  void deallocate(T* p, size_t) { std::free(p); }
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
  bool operator==(const fill_alloc&) const { return true; }
  bool operator!=(const fill_alloc&) const { return false; }
};
template <class T>
using buffer = std::vector<T, fill_alloc<T>>;

// Phase timer of a host builder: prints "<label> <phase> <ms>" on stderr when
// the environment variable `env` is set (MR_INGEST_TRACE, MR_LOAD_TRACE).
struct PhaseTrace {
  const char* label;
  bool on;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  PhaseTrace(const char* env, const char* l) : label(l), on(std::getenv(env) != nullptr) {}
  void operator()(const char* phase) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "%s %-12s %8.1f ms\n", label, phase, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

// In-place exclusive prefix sum a[0..n) -> a[i] = sum(a[0..i)); returns the
// total. Two passes over per-range sums when n is large.
template <class T>
T exclusive_scan(T* a, int64_t n) {
  const int64_t grain = 1 << 20;
  const int R = (int)std::max<int64_t>(1, std::min<int64_t>(usable_cores(), n / grain));
  if (R == 1) {
    T s = 0;
    for (int64_t i = 0; i < n; ++i) {
      const T x = a[i];
      a[i] = s;
      s += x;
    }
    return s;
  }
  std::vector<T> part(R + 1, 0);
  parallel_for(
      n,
      [&](int64_t lo, int64_t hi, int w) {
        T s = 0;
        for (int64_t i = lo; i < hi; ++i) s += a[i];
        part[w + 1] = s;
      },
      1, R);
  for (int r = 0; r < R; ++r) part[r + 1] += part[r];
  parallel_for(
      n,
      [&](int64_t lo, int64_t hi, int w) {
        T s = part[w];
        for (int64_t i = lo; i < hi; ++i) {
          const T x = a[i];
          a[i] = s;
          s += x;
        }
      },
      1, R);
  return part[R];
}

}  // namespace mr_par

#endif  // MR_PAR_H
