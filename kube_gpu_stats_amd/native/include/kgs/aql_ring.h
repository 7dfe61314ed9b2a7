// Bounded slot reservation on a single-producer AQL queue (the counter reader's
// private READ queue, native/counters/pmc_aqlprofile.cpp).
//
// The HSA idiom `idx = add_write_index(q, 1); while (idx - read_index >= size) {}`
// has two faults for a monitoring agent: it spins forever when the command
// processor stops consuming (a wedged CP — exactly when the exporter must keep
// reporting), and it reserves the slot *before* there is room, so giving up
// would leave a hole the CP stalls on.  Here the producer checks for room first
// and reserves only then (the queue has one producer: HSA_QUEUE_TYPE_SINGLE, one
// sampler thread per device), waits at most until `deadline_ns`, and gives up
// early when `abort` is raised (Sampler::stop()).  Header-only and templated on
// the queue accessors so the policy is unit-tested against a fake queue whose
// read index never advances (native/tests/test_core.cpp).
#pragma once

#include <atomic>
#include <cstdint>

namespace kgs {

enum class SlotResult : int { kOk = 0, kTimeout = -1, kAborted = -2 };

// read_index() / write_index(): the queue's indices; commit(idx): publish
// write index idx + 1 (the slot at idx is ours); now_ns(): monotonic clock;
// pause(): what to do between polls (a pause instruction / short sleep).
template <class ReadIdx, class WriteIdx, class Commit, class Now, class Pause>
SlotResult reserve_slot(uint64_t size, int64_t deadline_ns, const std::atomic<int>* abort, ReadIdx read_index,
                        WriteIdx write_index, Commit commit, Now now_ns, Pause pause, uint64_t& idx_out) {
  const uint64_t idx = write_index();
  uint64_t spins = 0;
  while (idx - read_index() >= size) {
    if (abort && abort->load(std::memory_order_relaxed)) return SlotResult::kAborted;
    // The clock is read every 64 polls: a full queue is the rare case, and the
    // common one (room right away) never reads it.
    if ((++spins & 63) == 0 && now_ns() >= deadline_ns) return SlotResult::kTimeout;
    pause();
  }
  commit(idx);
  idx_out = idx;
  return SlotResult::kOk;
}

}  // namespace kgs
