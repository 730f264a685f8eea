// DispatchQueue — per-endpoint FIFO with the Service Bus semantics the reference relies on
// (BackendQueueProcessor.cs:27-81, host.json peek-lock / abandon / max delivery count,
// deploy_servicebus_queue.sh:35): receive (peek-lock), complete, abandon(+delay), lock expiry ->
// redelivery, max delivery -> dead letter; plus a batching receive (max_n / linger) for the GPU
// scheduler. Lock expiry is checked by a scan of the in-flight set at most every
// min(50 ms, lock/2), so the per-receive cost does not grow with the number of messages in flight.
#pragma once

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <queue>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "common.h"

namespace ai4e {

struct Message {
  uint64_t seq = 0;
  std::string task_id;
  int64_t ref = -1;        // payload slot (pinned ring index) or -1
  std::string body;        // request body (used when no slot)
  int delivery_count = 0;
  double enqueued_at = 0;  // CLOCK_MONOTONIC
  double visible_at = 0;   // scheduled redelivery
  double lock_until = 0;
};

class DispatchQueue {
 public:
  DispatchQueue(std::string name, int max_delivery_count, double lock_duration_s, size_t max_size)
      : name_(std::move(name)), max_delivery_(max_delivery_count), lock_s_(lock_duration_s), max_size_(max_size) {}

  const std::string& name() const { return name_; }

  // Returns false (backpressure) when the queue is at max_size or closed.
  bool send(const std::string& task_id, int64_t ref, const std::string& body) {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_ || full_locked()) return false;
    Message m;
    m.seq = ++seq_;
    m.task_id = task_id;
    m.ref = ref;
    m.body = body;
    m.enqueued_at = mono_now();
    ready_.push_back(std::move(m));
    cv_.notify_one();
    return true;
  }

  size_t send_many(const std::vector<std::string>& ids, const std::vector<int64_t>& refs) {
    if (!refs.empty() && refs.size() != ids.size()) throw std::invalid_argument("ids/refs length mismatch");
    std::lock_guard<std::mutex> g(mu_);
    size_t n = 0;
    const double now = mono_now();
    for (size_t i = 0; i < ids.size(); ++i) {
      if (closed_ || full_locked()) break;
      Message m;
      m.seq = ++seq_;
      m.task_id = ids[i];
      m.ref = refs.empty() ? -1 : refs[i];
      m.enqueued_at = now;
      ready_.push_back(std::move(m));
      ++n;
    }
    cv_.notify_all();
    return n;
  }

  // Peek-lock receive with dynamic batching: wait up to `timeout_s` for the first message, then
  // up to `linger_s` more for the batch to fill to `max_n`. Returns locked messages.
  std::vector<Message> receive(size_t max_n, double timeout_s, double linger_s) {
    std::vector<Message> out;
    std::unique_lock<std::mutex> lk(mu_);
    const double deadline = mono_now() + timeout_s;
    for (;;) {
      promote_locked(mono_now());
      if (!ready_.empty() || closed_) break;
      const double now = mono_now();
      if (now >= deadline) return out;
      double wake = deadline;
      if (!scheduled_.empty()) wake = std::min(wake, scheduled_.top().visible_at);
      if (!inflight_.empty() && lock_s_ > 0) wake = std::min(wake, next_scan_);
      wait_s(lk, wake - now);
    }
    if (linger_s > 0 && ready_.size() < max_n && !closed_) {
      const double ldl = mono_now() + linger_s;
      while (ready_.size() < max_n && !closed_) {
        const double now = mono_now();
        if (now >= ldl) break;
        wait_s(lk, ldl - now);
        promote_locked(mono_now());
      }
    }
    const double now = mono_now();
    out.reserve(std::min(max_n, ready_.size()));
    while (!ready_.empty() && out.size() < max_n) {
      Message m = std::move(ready_.front());
      ready_.pop_front();
      m.delivery_count += 1;
      m.lock_until = now + lock_s_;
      out.push_back(m);
      inflight_.emplace(m.seq, std::move(m));
    }
    return out;
  }

  size_t complete(const std::vector<uint64_t>& seqs) {
    std::lock_guard<std::mutex> g(mu_);
    size_t n = 0;
    for (auto s : seqs) n += inflight_.erase(s);
    return n;
  }

  // Abandon (BackendQueueProcessor.cs:54-64): redeliver after the delay, or dead-letter when the
  // delivery count reached max_delivery. Returns "requeued" / "deadlettered" / "unknown".
  std::string abandon(uint64_t seq, double delay_s) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = inflight_.find(seq);
    if (it == inflight_.end()) return "unknown";
    Message m = std::move(it->second);
    inflight_.erase(it);
    return requeue_locked(std::move(m), delay_s);
  }

  std::vector<std::string> take_deadletters() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> out;
    out.reserve(dead_.size());
    for (auto& m : dead_) out.push_back(m.task_id);
    dead_.clear();
    return out;
  }

  void close() {
    std::lock_guard<std::mutex> g(mu_);
    closed_ = true;
    cv_.notify_all();
  }
  bool closed() {
    std::lock_guard<std::mutex> g(mu_);
    return closed_;
  }

  struct Stats {
    size_t ready, scheduled, inflight;
    uint64_t deadlettered, sent;
  };
  Stats stats() {
    std::lock_guard<std::mutex> g(mu_);
    return {ready_.size(), scheduled_.size(), inflight_.size(), dead_total_, seq_};
  }
  size_t depth() {
    std::lock_guard<std::mutex> g(mu_);
    return ready_.size() + scheduled_.size();
  }

  // Wake every blocked receiver (scheduler shutdown).
  void kick() { cv_.notify_all(); }

  // Lock duration for later receives; <= 0 disables lock expiry. A queue drained by the NodeScheduler
  // runs with expiry off: the scheduler detects dead workers by heartbeat and requeues their batches
  // itself, and an expiry-redelivery of a batch the first worker still holds would hand its ring
  // slots to a second worker while the first may still complete them.
  void set_lock_duration(double s) {
    std::lock_guard<std::mutex> g(mu_);
    lock_s_ = s;
    for (auto& kv : inflight_) kv.second.lock_until = s > 0 ? mono_now() + s : 0;
  }
  double lock_duration() {
    std::lock_guard<std::mutex> g(mu_);
    return lock_s_;
  }

 private:
  struct Later {
    bool operator()(const Message& a, const Message& b) const { return a.visible_at > b.visible_at; }
  };

  bool full_locked() const { return max_size_ && ready_.size() + scheduled_.size() >= max_size_; }

  std::string requeue_locked(Message m, double delay_s) {
    if (max_delivery_ > 0 && m.delivery_count >= max_delivery_) {
      dead_.push_back(std::move(m));
      ++dead_total_;
      return "deadlettered";
    }
    m.visible_at = mono_now() + delay_s;
    if (delay_s <= 0) {
      ready_.push_back(std::move(m));
    } else {
      scheduled_.push(std::move(m));
    }
    cv_.notify_one();
    return "requeued";
  }

  void promote_locked(double now) {
    while (!scheduled_.empty() && scheduled_.top().visible_at <= now) {
      ready_.push_back(scheduled_.top());
      scheduled_.pop();
    }
    // Lock expiry: a receiver that died (or hung) loses its messages, which are redelivered.
    if (lock_s_ <= 0 || inflight_.empty() || now < next_scan_) return;
    next_scan_ = now + std::min(0.05, lock_s_ / 2);
    std::vector<uint64_t> expired;
    for (auto& kv : inflight_)
      if (kv.second.lock_until <= now) expired.push_back(kv.first);
    for (auto s : expired) {
      auto it = inflight_.find(s);
      Message m = std::move(it->second);
      inflight_.erase(it);
      requeue_locked(std::move(m), 0);
    }
  }

  // Timed wait on the system clock: pthread_cond_timedwait (the steady-clock overload maps to
  // pthread_cond_clockwait, which ThreadSanitizer in this toolchain does not intercept and then
  // reports as a double lock — tools/tsan_check.sh keeps this core race-clean).
  void wait_s(std::unique_lock<std::mutex>& lk, double seconds) {
    cv_.wait_until(lk, std::chrono::system_clock::now() +
                           std::chrono::duration_cast<std::chrono::system_clock::duration>(
                               std::chrono::duration<double>(std::max(0.0, seconds))));
  }

  std::string name_;
  int max_delivery_;
  double lock_s_;
  size_t max_size_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Message> ready_;
  std::priority_queue<Message, std::vector<Message>, Later> scheduled_;
  std::unordered_map<uint64_t, Message> inflight_;
  double next_scan_ = 0;
  std::vector<Message> dead_;
  uint64_t seq_ = 0, dead_total_ = 0;
  bool closed_ = false;
};

}  // namespace ai4e
