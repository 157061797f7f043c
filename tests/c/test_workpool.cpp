// WorkPool (emqx_amd/csrc/workpool.h): every run executes its job once on the caller and once on
// each of t - 1 workers, runs never overlap, and no wake-up is lost, with and without the spin
// window (spin 0: every wait blocks; a long spin: no wait blocks; the default in between).
#include "../../emqx_amd/csrc/workpool.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>

int main() {
  auto& pool = emqx::WorkPool::get();
  std::mt19937 rng(7);
  const uint32_t spins[] = {0u, 200u, 20000u, 5u};
  long total = 0;
  for (uint32_t spin : spins) {
    pool.set_spin_us(spin);
    for (int r = 0; r < 600; ++r) {
      const unsigned t = 1 + rng() % 16;
      std::atomic<int> calls{0}, inside{0};
      bool overlap = false;
      std::atomic<bool> bad{false};
      const std::function<void()> job = [&] {
        if (inside.fetch_add(1) >= static_cast<int>(t)) bad = true;
        calls.fetch_add(1);
        inside.fetch_sub(1);
      };
      pool.run(job, t);
      // the pool may hold fewer workers than asked only if a thread could not start
      if (calls.load() != static_cast<int>(t) || bad.load()) overlap = true;
      if (overlap) {
        std::fprintf(stderr, "spin %u run %d: %d calls for t=%u\n", spin, r, calls.load(), t);
        return 1;
      }
      total += calls.load();
      if (r % 100 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 400));  // let workers sleep
    }
  }
  // runs from several caller threads at once (serialised by the pool's run lock): no deadlock,
  // and ThreadSanitizer (the second build of this test) sees no race
  std::vector<std::thread> callers;
  std::atomic<long> calls{0};
  for (int c = 0; c < 4; ++c)
    callers.emplace_back([&] {
      for (int r = 0; r < 200; ++r) {
        const std::function<void()> job = [&] { calls.fetch_add(1); };
        pool.run(job, 8);
      }
    });
  for (auto& th : callers) th.join();
  if (calls.load() != 4L * 200 * 8) {
    std::fprintf(stderr, "concurrent callers: %ld job calls, want %d\n", calls.load(), 4 * 200 * 8);
    return 1;
  }
  std::printf("workpool ok: %ld job calls\n", total);
  return 0;
}
