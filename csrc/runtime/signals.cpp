// Async-signal-safe preemption flags.
//
// Replaces the reference's raise-in-handler design (reference utils.py:93-97,
// registered at train.py:89-90), where SIGUSR1/SIGTERM became a Python
// exception at an arbitrary bytecode boundary (torn optimizer
// steps, off-by-one resume). Here the sigaction handler only performs
// lock-free atomic stores; the trainer polls the flag at step boundaries and
// dispatches through the same exit-policy matrix (10 / 15 / -1).
#include "runtime.h"

#include <pthread.h>
#include <signal.h>
#include <string.h>

#include <atomic>

namespace ftrt {
namespace {
std::atomic<int> g_first{0};          // first signal received since clear()
std::atomic<uint64_t> g_mask{0};      // bitmask of all received signals
std::atomic<uint64_t> g_count{0};     // total deliveries
static_assert(std::atomic<int>::is_always_lock_free, "need lock-free int atomics");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "need lock-free u64 atomics");

void handler(int signum) {
  int expected = 0;
  g_first.compare_exchange_strong(expected, signum, std::memory_order_acq_rel);
  if (signum > 0 && signum < 64) g_mask.fetch_or(1ull << signum, std::memory_order_acq_rel);
  g_count.fetch_add(1, std::memory_order_acq_rel);
}
}  // namespace

void signals_install(const std::vector<int>& signums) {
  for (int s : signums) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = handler;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_RESTART;
    if (sigaction(s, &sa, nullptr) != 0) throw std::runtime_error("sigaction failed");
  }
}

void signals_restore_default(const std::vector<int>& signums) {
  for (int s : signums) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = SIG_DFL;
    sigemptyset(&sa.sa_mask);
    sigaction(s, &sa, nullptr);
  }
}

int signals_pending() { return g_first.load(std::memory_order_acquire); }
uint64_t signals_mask() { return g_mask.load(std::memory_order_acquire); }
uint64_t signals_count() { return g_count.load(std::memory_order_acquire); }

void signals_clear() {
  g_first.store(0, std::memory_order_release);
  g_mask.store(0, std::memory_order_release);
}

// Block / unblock delivery to the calling thread (used around the final save so a
// late SIGTERM cannot interrupt a checkpoint publish).
void signals_block(const std::vector<int>& signums, bool block) {
  sigset_t set;
  sigemptyset(&set);
  for (int s : signums) sigaddset(&set, s);
  pthread_sigmask(block ? SIG_BLOCK : SIG_UNBLOCK, &set, nullptr);
}

}  // namespace ftrt
