// Single-writer / multi-reader publication primitives for the sampler → scrape
// hand-off (SURVEY.md §2.3 "producer/consumer pipeline", §5.2).
//
// The writer (one sampler thread per GPU) never blocks and never allocates.
// Readers (the HTTP renderer, Python snapshot calls) retry on a torn read.
// The payload is copied word-by-word through relaxed atomics so the protocol is
// data-race-free under the C++ memory model (and therefore TSAN-clean), not just
// "works on x86".
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <type_traits>

namespace kgs {

namespace detail {
template <class T>
constexpr size_t words_of() { return (sizeof(T) + sizeof(uint64_t) - 1) / sizeof(uint64_t); }
}  // namespace detail

template <class T>
class Seqlock {
  static_assert(std::is_trivially_copyable<T>::value, "Seqlock payload must be POD");
  static constexpr size_t kWords = detail::words_of<T>();

 public:
  Seqlock() {
    for (auto& w : data_) w.store(0, std::memory_order_relaxed);
  }

  // Writer side: exactly one thread.
  void store(const T& v) {
    uint64_t buf[kWords] = {};
    std::memcpy(buf, &v, sizeof(T));
    const uint64_t s = seq_.load(std::memory_order_relaxed);
    seq_.store(s + 1, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);
    for (size_t i = 0; i < kWords; ++i) data_[i].store(buf[i], std::memory_order_relaxed);
    seq_.store(s + 2, std::memory_order_release);
  }

  // Reader side: any number of threads.  Returns false if never written.
  // `version`, if given, receives the number of completed stores the copy came
  // from (SampleRing uses it to tell a slot's current lap from a newer one).
  bool load(T& out, int max_spins = 1 << 20, uint64_t* version = nullptr) const {
    uint64_t buf[kWords];
    for (int spin = 0; spin < max_spins; ++spin) {
      const uint64_t s0 = seq_.load(std::memory_order_acquire);
      if (s0 & 1) continue;
      for (size_t i = 0; i < kWords; ++i) buf[i] = data_[i].load(std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_acquire);
      const uint64_t s1 = seq_.load(std::memory_order_relaxed);
      if (s0 == s1) {
        if (s0 == 0) return false;
        std::memcpy(&out, buf, sizeof(T));
        if (version) *version = s0 >> 1;
        return true;
      }
    }
    return false;
  }

  uint64_t version() const { return seq_.load(std::memory_order_acquire) >> 1; }

 private:
  alignas(64) std::atomic<uint64_t> seq_{0};
  std::atomic<uint64_t> data_[kWords];
};

// Fixed-capacity history ring of seqlocked slots.  The writer publishes slot
// `head % N` and then advances `head`; a reader walking back from `head` gets
// every slot that was not overwritten while it read (torn slots are skipped).
//
// Generation check: entry e (0-based push index) lives in slot e % N and is that
// slot's (e / N + 1)-th store.  A reader that was descheduled long enough for
// the writer to lap it finds a *newer* entry in the slot — untorn, but the wrong
// one — and the slot's store count tells it so.  Binary searches over the ring
// (Sampler::window_busy / window_pmc) rely on entries being time-ordered, so a
// lapped slot reads as absent, never as a newer sample under an old index.
template <class T, size_t N>
class SampleRing {
  static_assert((N & (N - 1)) == 0, "capacity must be a power of two");

 public:
  void push(const T& v) {
    const uint64_t h = head_.load(std::memory_order_relaxed);
    slots_[h & (N - 1)].store(v);
    head_.store(h + 1, std::memory_order_release);
  }

  uint64_t head() const { return head_.load(std::memory_order_acquire); }
  static constexpr size_t capacity() { return N; }

  // The i-th most recent entry (0 = newest) as of this call's `head`; false if
  // absent, torn, or already overwritten by a later lap of the writer.
  bool at(uint64_t i, T& out) const { return at_from(head(), i, out); }

  // Same, relative to a head value the caller read once (a consistent view
  // across several lookups of one search).
  bool at_from(uint64_t h, uint64_t i, T& out) const {
    if (i >= h || i >= N - 1) return false;
    return load_entry(h - 1 - i, out);
  }

  // Number of entries a reader can walk back over (one slot of slack for the writer).
  size_t available() const {
    const uint64_t h = head();
    return static_cast<size_t>(h < N - 1 ? h : N - 1);
  }

  // Visit the most recent entries newest-first, one seqlock load at a time,
  // until `fn(entry)` returns false; returns the number visited.  A scrape that
  // needs the last second of a ring reads only that second, not the whole ring.
  template <class F>
  size_t visit_recent(F&& fn) const {
    const uint64_t h = head();
    T v;
    size_t n = 0;
    for (uint64_t i = 0; i < h && i < N - 1; ++i) {
      if (!load_entry(h - 1 - i, v)) continue;
      ++n;
      if (!fn(static_cast<const T&>(v))) break;
    }
    return n;
  }

  // Copy up to `max` most recent entries (newest first) into out[]; returns count.
  size_t recent(T* out, size_t max) const {
    const uint64_t h = head();
    size_t n = 0;
    for (uint64_t i = 0; i < max && i < h && i < N - 1; ++i) {
      if (load_entry(h - 1 - i, out[n])) ++n;
    }
    return n;
  }

 private:
  // Entry `e` (push index), only if its slot still holds that lap.
  bool load_entry(uint64_t e, T& out) const {
    uint64_t ver = 0;
    if (!slots_[e & (N - 1)].load(out, 4, &ver)) return false;
    return ver == e / N + 1;
  }

  alignas(64) std::atomic<uint64_t> head_{0};
  Seqlock<T> slots_[N];
};

}  // namespace kgs
