// Slot plan of the counter reader's batched publication (--pmc-batch,
// native/counters/pmc_aqlprofile.cpp read_batched).
//
// A counter READ leaves its results in the GPU's L2 until a cache writeback
// pushes them to the host; that writeback is about half of what a READ costs a
// training step (profiles/r3/README.md r3e / r3g).  With a batch of B the READs go
// round 2B pre-built slots in two halves.  Slot h*B + B-1 is half h's publisher:
// its IB writes the L2 back and its AQL header carries the system-scope release
// fence; the other slots do neither.  Packets on the queue run in order, so when
// a publisher completes, every READ of its half is visible on the host and the
// half is folded in submit order.
//
// The plan also bounds how long a sample waits to be published: a READ takes the
// publisher slot at once — closing its half early — when the next READ would be
// due `publish_ns` or more after the half's first one.  At 8 kHz (125 µs ticks)
// with B = 8 and 1 ms that never fires and the L2 is written back 1000 times a
// second instead of 8000; at a quiet GPU's 100 Hz, or any --hz <= 1 kHz, every
// READ publishes and a sample is one tick late, as without batching.
//
// The price is the delay line: after each (re)start of the rotation (a START, a
// quiet GPU turning busy) about B calls return no sample (kPmcPending) while the
// first half fills.  Nothing is lost but resolution — the counters are
// cumulative, so the next sample's interval covers those ticks.
//
// Pure bookkeeping, single-threaded (one sampler thread per device), header-only
// so the policy is unit-tested without a GPU (native/tests/test_core.cpp).
#pragma once

#include <cstdint>

namespace kgs {

class BatchPlan {
 public:
  static constexpr int kMaxBatch = 16;

  // batch in [2, kMaxBatch]; publish_ns <= 0: only a half's B-th READ publishes.
  void configure(int batch, int64_t publish_ns) {
    b_ = batch < 2 ? 2 : (batch > kMaxBatch ? kMaxBatch : batch);
    publish_ns_ = publish_ns;
    reset();
  }
  void reset() {
    count_[0] = count_[1] = 0;
    closed_[0] = closed_[1] = false;
    first_ns_[0] = first_ns_[1] = 0;
    next_ = 0;
    last_ = -1;
    last_ns_ = -1;
  }

  int batch() const { return b_; }
  int nslots() const { return 2 * b_; }
  bool is_publisher(int slot) const { return slot % b_ == b_ - 1; }
  int publisher(int half) const { return half * b_ + b_ - 1; }
  // The half the next READ goes into.  If it is closed (its publisher was
  // submitted and it was not collected yet), the caller waits for that publisher
  // and collects the half before submitting.
  int current_half() const { return next_ / b_; }
  bool closed(int half) const { return closed_[half]; }
  int last() const { return last_; }  // slot of the last READ submitted, -1 none

  // The slot for a READ submitted at now_ns.  The tick interval is the time
  // since the previous READ; with none yet (after a reset) the READ publishes.
  int next_slot(int64_t now_ns) const {
    const int h = next_ / b_;
    if (is_publisher(next_) || publish_ns_ <= 0) return next_;
    const int64_t interval = last_ns_ < 0 ? publish_ns_ + 1 : now_ns - last_ns_;
    const int64_t waited = count_[h] == 0 ? 0 : now_ns - first_ns_[h];
    return waited + interval >= publish_ns_ ? publisher(h) : next_;
  }

  // Record the READ submitted into `slot` (the value next_slot returned) at now_ns.
  void submitted(int slot, int64_t now_ns) {
    const int h = slot / b_;
    if (count_[h] == 0) first_ns_[h] = now_ns;
    ++count_[h];
    if (is_publisher(slot)) {
      closed_[h] = true;
      next_ = (h ^ 1) * b_;
    } else {
      next_ = slot + 1;
    }
    last_ = slot;
    last_ns_ = now_ns;
  }

  // Slots of a closed half in submit order (its non-publishers from the half's
  // first slot on, then the publisher).  Returns how many were written to out.
  int slots(int half, int* out) const {
    int n = 0;
    for (int j = 0; j < count_[half] - 1; ++j) out[n++] = half * b_ + j;
    out[n++] = publisher(half);
    return n;
  }
  void collected(int half) {
    count_[half] = 0;
    closed_[half] = false;
  }

  // Which closed halves to fold before the next READ, oldest first (ADVICE r3:
  // folding them out of order hands the caller samples whose time and cumulative
  // counts go backwards).  When both halves are closed, the current half — the one
  // the next READ goes into — closed first: the other closed after it and is the
  // newer.  A current half that is closed must be folded (wait[i] = true: block on
  // its publisher) before its slots are reused; the other is folded only if its
  // publisher is already done (`other_done`).  Returns how many entries of
  // half/wait were written (0..2).
  int collect_order(bool other_done, int* half, bool* wait) const {
    const int cur = current_half(), other = cur ^ 1;
    int n = 0;
    if (closed_[cur]) {
      half[n] = cur;
      wait[n++] = true;
    }
    if (closed_[other] && other_done) {
      half[n] = other;
      wait[n++] = false;
    }
    return n;
  }

 private:
  int b_ = 2;
  int64_t publish_ns_ = 0;
  int count_[2] = {0, 0};        // READs submitted into each half since it was collected
  bool closed_[2] = {false, false};
  int64_t first_ns_[2] = {0, 0};  // submit time of each half's first READ
  int next_ = 0;
  int last_ = -1;
  int64_t last_ns_ = -1;
};

}  // namespace kgs
