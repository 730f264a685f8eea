// SlotRing — FIFO allocator of payload-ring slots (the pinned / shared-memory buffer of decoded
// request payloads that the GPU workers DMA from).
//
// `alloc(n)` hands out the next n slots in ring order, so a batch received from the FIFO dispatch
// queue is (almost always) one contiguous run -> one H2D copy. `free` marks slots and advances the
// head over the freed prefix. A ring can cover a sub-range [base, base+n) of a larger shared
// buffer: every ingest process owns one partition of the node's ring.
#pragma once

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace ai4e {

class SlotRing {
 public:
  SlotRing(int64_t nslots, int64_t base) : n_(nslots), base_(base), freed_(static_cast<size_t>(nslots), 0) {
    if (nslots <= 0) throw std::invalid_argument("SlotRing needs at least one slot");
  }

  // Blocks up to timeout_s (< 0: forever) for n free slots; empty result on timeout.
  std::vector<int64_t> alloc(int64_t n, double timeout_s) {
    if (n > n_) throw std::invalid_argument("request larger than the ring");
    std::unique_lock<std::mutex> lk(mu_);
    auto ok = [&] { return closed_ || n_ - used_ >= n; };
    if (timeout_s < 0) {
      cv_.wait(lk, ok);
    } else if (!cv_.wait_until(lk, std::chrono::system_clock::now() +
                                       std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                           std::chrono::duration<double>(timeout_s)),
                               ok)) {
      return {};
    }
    if (closed_) return {};
    std::vector<int64_t> out(static_cast<size_t>(n));
    const int64_t start = (head_ + used_) % n_;
    for (int64_t i = 0; i < n; ++i) out[static_cast<size_t>(i)] = base_ + (start + i) % n_;
    used_ += n;
    return out;
  }

  // Returns the number of slots freed. Slots outside this ring, slots not currently allocated (outside
  // [head, head + used)) and slots already freed are ignored: a stale or duplicated free can never
  // latch a mark that would later let the head run over a live slot.
  size_t free(const std::vector<int64_t>& slots) {
    std::lock_guard<std::mutex> g(mu_);
    size_t k = 0;
    for (int64_t s : slots) {
      const int64_t i = s - base_;
      if (i < 0 || i >= n_) continue;
      if ((i - head_ + n_) % n_ >= used_) continue;  // not allocated
      if (freed_[static_cast<size_t>(i)]) continue;   // double free
      freed_[static_cast<size_t>(i)] = 1;
      ++k;
    }
    while (used_ && freed_[static_cast<size_t>(head_)]) {
      freed_[static_cast<size_t>(head_)] = 0;
      head_ = (head_ + 1) % n_;
      --used_;
    }
    cv_.notify_all();
    return k;
  }

  bool owns(int64_t slot) const { return slot >= base_ && slot < base_ + n_; }
  int64_t used() {
    std::lock_guard<std::mutex> g(mu_);
    return used_;
  }
  int64_t capacity() const { return n_; }
  int64_t base() const { return base_; }
  void close() {
    std::lock_guard<std::mutex> g(mu_);
    closed_ = true;
    cv_.notify_all();
  }

 private:
  const int64_t n_, base_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<uint8_t> freed_;
  int64_t head_ = 0, used_ = 0;
  bool closed_ = false;
};

}  // namespace ai4e
