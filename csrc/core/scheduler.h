// NodeScheduler — the node's dispatch loop in native code: dispatch queue -> dynamic batch ->
// per-GPU worker process -> results + task-state transitions, with no Python (and no GIL) on the
// per-batch path.
//
// It is the single-node replacement for the reference's per-endpoint BackendQueueProcessor
// (ProcessManager/BackendQueueProcessor/BackendQueueProcessor.cs:27-81: receive -> POST ->
// complete / abandon on 429) *and* for its replica scaling (APIs/Charts/templates/async-gpu/
// autoscaler.yaml, routing.yml ROUND_ROBIN): every GPU worker process owns one connection; for
// each connection a dispatcher thread pulls up to max_batch peek-locked messages when its GPU has
// a free pipeline slot (least-loaded placement by construction) and a reader thread retires the
// worker's results. Messages on a connection use multiprocessing.Connection framing (4-byte
// big-endian length + payload), so the Python side of a worker is plain Connection.send_bytes /
// recv_bytes. Payload = u32 type + fields (little-endian):
//
//   READY  (w->s) i32 rank, i32 pinned, utf-8 JSON info
//   HB     (w->s) f64 t, u64 hbm_used, u64 hbm_total, f64 gpu_busy_ms, u64 batches, u64 xgmi_tx, u64 xgmi_rx,
//                 f64 gfx_mhz, f64 power_w (GPU telemetry; 0 = unavailable)
//   DONE   (w->s) u64 bid, u32 n, u32 row_bytes, f64 stage[5], u8 status[n] (padded to 8), rows
//   BATCH  (s->w) u64 bid, u32 n, u32 0, i64 slots[n]
//   STOP   (s->w)
//   SUBMIT (w->s) u32 n, u32 0, i64 slots[n]      (a remote ingest shard enqueued n payloads)
//   FREE   (s->w) u32 n, u32 0, i64 slots[n]      (slots of that shard's partition are free again)
//   SUBMIT_IDS (w->s) u32 n, u32 trace_len, u32 id_len, u32 flags, u64 token, i64 slots[n],
//          char ids[n][id_len], trace   (an ingest front-end process enqueued n payloads under task ids it
//          minted; flags bit 0: answer with SUBMITTED once the tasks exist, so its HTTP reply never races them)
//   SUBMITTED (s->w) u64 token, u32 n_created, u32 0
//   SUBMIT_MULTI (w->s) u32 nreq, u64 token, then per request u32 n, u32 trace_len, u32 id_len, u32 0, i64 slots[n],
//          char ids[n][id_len], trace   (a front-end's group commit: the requests of several client connections)
//   SUBMITTED_MULTI (s->w) u64 token, u32 nreq, u32 created[nreq]
//   STAGE  (w->s) u64 bid, u32 stage, u32 0        (ensemble hop: AddPipelineTask for the batch)
//
// Item status in DONE: 0 ok, 1 invalid payload (failed, not retried), 2 model error (failed,
// "Task failed - try again" as ai4e_service.py:208-211), 3 retry (abandoned with the retry delay;
// dead-lettered after max delivery -> failed with a reason).
// Failure detection (survey §5.3): a closed connection or a heartbeat older than hb_timeout marks
// the worker dead; its in-flight batches go back to the queue and the rank is reported to Python
// (`wait_failed`) which restarts or removes the process.
#pragma once

#include <arpa/inet.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "dispatch_queue.h"
#include "slot_ring.h"
#include "task_store.h"

namespace ai4e {

// Timed condition waits on the system clock (see DispatchQueue::wait_s: TSAN-interceptable).
template <class Pred>
inline bool cv_wait_s(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, double seconds, Pred pred) {
  return cv.wait_until(lk,
                       std::chrono::system_clock::now() + std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                                              std::chrono::duration<double>(std::max(0.0, seconds))),
                       pred);
}

enum : uint32_t {
  F_READY = 1, F_HB = 2, F_DONE = 3, F_BATCH = 4, F_STOP = 5, F_SUBMIT = 6, F_FREE = 7, F_STAGE = 8, F_SUBMIT_IDS = 9,
  F_SUBMITTED = 10, F_SUBMIT_MULTI = 11, F_SUBMITTED_MULTI = 12
};
enum : uint8_t { IT_OK = 0, IT_INVALID = 1, IT_ERROR = 2, IT_RETRY = 3 };

static const char* kFailInvalid = "Task failed - invalid payload";
static const char* kFailError = "Task failed - try again";
static const char* kFailMaxRetries = "Task failed - maximum retries exceeded";
static const char* kRequeued = "Awaiting service availability. Worker failed; requeued.";
static const char* kPublishFailed = "Failed - unable to send to backend service.";

struct SchedConfig {
  size_t max_batch = 250;
  double linger_s = 0.0005;
  // linger while the worker already has a batch in flight: its GPU is busy anyway, so a fuller batch costs no
  // throughput (single-image arrivals otherwise leave as many small batches, each run in a padded graph bucket)
  double busy_linger_s = 0.0;
  int depth = 2;               // batches in flight per worker
  double retry_delay_s = 1.0;  // abandon delay for IT_RETRY items
  double hb_timeout_s = 10.0;
  double poll_s = 0.02;        // queue wait per dispatcher iteration
};

struct WorkerStats {
  int rank = -1;
  bool ready = false, alive = false, pinned = false;
  uint64_t batches = 0, images = 0, failed_items = 0, retried_items = 0;
  size_t outstanding = 0;
  double last_hb_age_s = 0, gpu_busy_ms = 0, gfx_mhz = 0, power_w = 0;
  uint64_t hbm_used = 0, hbm_total = 0, xgmi_tx = 0, xgmi_rx = 0;
  std::string info;
};

class NodeScheduler {
 public:
  NodeScheduler(std::shared_ptr<TaskStore> store, std::shared_ptr<DispatchQueue> queue, std::string endpoint,
                int64_t ring_slots, SchedConfig cfg)
      : store_(std::move(store)), queue_(std::move(queue)), endpoint_(std::move(endpoint)), ring_slots_(ring_slots),
        cfg_(cfg), hist_(12, 0) {}
  ~NodeScheduler() {
    stop();
    if (stat_) {
      munmap(stat_, sizeof(ShardStat));
      if (!stat_name_.empty()) shm_unlink(("/" + stat_name_).c_str());
    }
    if (tags_) munmap(tags_, static_cast<size_t>(ring_slots_) * kTagBytes);
  }

  // Durable payloads (a task journal is configured): the payload ring itself outlives a crash of the serving tree
  // (POSIX shm that nothing unlinks on a crash), and this tag array — kTagBytes per ring slot, the id of the task
  // whose payload the slot holds — lets a restarted node find each unfinished task's payload there
  // (runtime/durable_ring.py). Tags are written before a task is acknowledged (the journal record is flushed to
  // the kernel first too), so every acknowledged task has its record and its payload on a crash; the reference's
  // equivalent is the Redis "{TaskId}_ORIG" body of CacheConnectorUpsert.cs:125-176.
  static constexpr size_t kTagBytes = 48;
  bool set_slot_tags(const std::string& name) {
    if (tags_ || name.empty() || name.find('/') != std::string::npos) return false;
    const int fd = shm_open(("/" + name).c_str(), O_RDWR, 0);
    if (fd < 0) return false;
    void* p = mmap(nullptr, static_cast<size_t>(ring_slots_) * kTagBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) return false;
    tags_ = static_cast<char*>(p);
    return true;
  }

  // Shard load published in a small POSIX shm block (the native ingest front-ends map it read-write): tasks queued
  // into this scheduler, tasks that reached a terminal state (completed, failed, dead-lettered), items out at the GPU
  // workers and the live dispatch workers, so a front-end's latency-budget admission projects the shard's whole
  // backlog over its service rate instead of its own partition's share (which, with several front-ends and 250-image
  // requests, is mostly bodies still uploading and batch-quantization noise), and routes around a shard with no live
  // worker. Every front-end owns one `fe_pending` word (admitted bodies still uploading); the scheduler zeroes it
  // when that front-end's connection closes, so a front-end killed mid-upload never leaves phantom backlog behind.
  static constexpr int kStatFrontends = 56;
  struct ShardStat {
    std::atomic<uint64_t> enq;       // [0]
    std::atomic<uint64_t> done;      // [1] terminal outcomes
    std::atomic<uint64_t> pending;   // [2] bodies uploading at front-ends without a word of their own
    std::atomic<uint64_t> live;      // [3] dispatch workers that are ready
    std::atomic<uint64_t> inflight;  // [4] items handed to GPU workers, not yet finished or requeued
    // [5] microseconds the shard has had items in flight at its workers, closed intervals; [6] CLOCK_MONOTONIC
    // microseconds at which the open interval began (0: none open). Finished items per busy second is the shard's
    // capacity at the batches it forms, whatever the load (ingestd admission)
    std::atomic<uint64_t> busy_us;
    std::atomic<uint64_t> busy_since_us;
    std::atomic<uint64_t> batches;  // [7] batches finished (or returned) by the workers
    std::atomic<uint64_t> fe_pending[kStatFrontends];  // [8 + i] front-end i (scheduler rank kFrontendRank0 + i)
  };
  static_assert(sizeof(ShardStat) == 512, "ShardStat is mapped as 512 bytes by csrc/ingest/ingestd.cpp");
  static constexpr int kFrontendRank0 = 1 << 20;  // runtime/worker_pool.py FRONTEND_RANK0
  bool open_stat(const std::string& name) {
    if (stat_ || name.empty() || name.find('/') != std::string::npos) return false;
    const int fd = shm_open(("/" + name).c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) return false;
    void* p = MAP_FAILED;
    if (ftruncate(fd, sizeof(ShardStat)) == 0)
      p = mmap(nullptr, sizeof(ShardStat), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) {
      shm_unlink(("/" + name).c_str());
      return false;
    }
    stat_ = new (p) ShardStat{};
    stat_->live.store(static_cast<uint64_t>(live_.load()));
    stat_name_ = name;
    return true;
  }
  // Unlink the counters' name (the mapping stays valid for everyone who has it): on a clean stop.
  void unlink_stat() {
    if (!stat_name_.empty()) shm_unlink(("/" + stat_name_).c_str());
    stat_name_.clear();
  }
  // (tests / stats) the published counters: enq, done, pending (all front-ends), live, inflight
  std::vector<uint64_t> stat_counters() {
    std::vector<uint64_t> out(6, 0);
    if (!stat_) {
      out[3] = static_cast<uint64_t>(live_.load());
      return out;
    }
    out[0] = stat_->enq.load();
    out[1] = stat_->done.load();
    out[2] = stat_->pending.load();
    for (int i = 0; i < kStatFrontends; ++i) out[2] += stat_->fe_pending[i].load();
    out[3] = stat_->live.load();
    out[4] = stat_->inflight.load();
    const uint64_t t0 = stat_->busy_since_us.load();
    const uint64_t now = static_cast<uint64_t>(mono_now() * 1e6);
    out[5] = stat_->busy_us.load() + (t0 && now > t0 ? now - t0 : 0);
    return out;
  }

  // Competing consumers across control-plane shards (the reference's replicas all consume ONE Service Bus queue:
  // BackendQueueProcessor.cs:54-64, host.json:3-11 — an abandoned or orphaned message goes to whichever consumer is
  // alive). A shard's dispatchers take batches from a peer's queue (a) first, whenever that peer has no live
  // dispatch worker (its workers died past max_restarts, or it was resized to zero), and (b) when their own queue
  // stayed empty for a whole poll while the peer holds at least a full batch. A stolen batch stays the peer's: its
  // messages complete / abandon on the peer's queue, its slots go back to the peer's ring partitions and its
  // terminal counts to the peer's ShardStat.
  void set_peers(const std::vector<std::shared_ptr<NodeScheduler>>& peers) {
    std::lock_guard<std::mutex> g(mu_);
    peers_.clear();
    for (auto& p : peers)
      if (p.get() != this) peers_.push_back(p);
  }
  void set_steal(bool orphans, bool idle) {
    steal_orphans_.store(orphans);
    steal_idle_.store(idle);
  }
  int live_workers() const { return live_.load(); }
  uint64_t stolen_items() const { return stolen_.load(); }

  // Partition of the payload ring freed in this process (the ingest ring of the gateway).
  void add_local_ring(std::shared_ptr<SlotRing> ring) {
    std::lock_guard<std::mutex> g(mu_);
    local_rings_.push_back(std::move(ring));
  }
  // Partition [base, base+len) is owned by the ingest shard on `rank`'s connection.
  void add_remote_partition(int64_t base, int64_t len, int rank) {
    std::lock_guard<std::mutex> g(mu_);
    remote_parts_.push_back({base, len, rank});
  }
  // Ensemble stages: STAGE k from a worker moves the batch's tasks to stage_endpoints[k].
  void set_stage_endpoints(std::vector<std::string> eps, std::vector<std::string> statuses) {
    std::lock_guard<std::mutex> g(mu_);
    stage_eps_ = std::move(eps);
    stage_status_ = std::move(statuses);
  }
  void enable_completion_feed(bool on) {
    std::lock_guard<std::mutex> g(feed_mu_);
    feed_on_ = on;
  }
  // Control-plane shard: tasks this scheduler creates are minted in these task-store lock domains only
  // (round-robin per batch). Empty (the default): any domain, the store's own round-robin.
  void set_store_shards(std::vector<int> shards) {
    std::lock_guard<std::mutex> g(mu_);
    store_shards_ = std::move(shards);
  }

  // Takes ownership of `fd` (a connected stream socket). dispatch=false: ingest-only connection.
  void attach(int rank, int fd, bool dispatch) {
    {
      std::lock_guard<std::mutex> g(fail_mu_);
      if (stopped_) {  // shutting down: never start threads nobody will join
        ::close(fd);
        return;
      }
    }
    std::unique_ptr<Worker> old;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = workers_.find(rank);
      if (it != workers_.end()) old = std::move(it->second);
      workers_.erase(rank);
    }
    if (old) join_worker(*old);
    auto w = std::make_unique<Worker>();
    w->rank = rank;
    w->fd = fd;
    w->dispatch = dispatch;
    w->alive = true;
    w->last_hb = mono_now();
    Worker* raw = w.get();
    {
      std::lock_guard<std::mutex> g(mu_);
      workers_[rank] = std::move(w);
    }
    raw->reader = std::thread([this, raw] { reader_loop(*raw); });
    if (dispatch) raw->dispatcher = std::thread([this, raw] { dispatch_loop(*raw); });
  }

  // Graceful retire: stop dispatching to `rank`, wait (<= timeout) for its batches, send STOP.
  void detach(int rank, double timeout_s) {
    Worker* w = nullptr;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = workers_.find(rank);
      if (it == workers_.end()) return;
      w = it->second.get();
    }
    {
      std::unique_lock<std::mutex> lk(w->mu);
      w->draining = true;
      set_live(*w, false);
      w->cv.notify_all();
      cv_wait_s(w->cv, lk, timeout_s, [&] { return w->out.empty() || !w->alive; });
    }
    send_simple(*w, F_STOP);
    mark_dead(*w, "retired", false);
    std::unique_ptr<Worker> own;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = workers_.find(rank);
      if (it != workers_.end()) own = std::move(it->second);
      workers_.erase(rank);
    }
    if (own) join_worker(*own);
  }

  // Ranks whose worker died since the last call (blocks up to timeout_s for the first one).
  std::vector<int> wait_failed(double timeout_s) {
    std::unique_lock<std::mutex> lk(fail_mu_);
    cv_wait_s(fail_cv_, lk, timeout_s, [&] { return !failed_.empty() || stopped_; });
    std::vector<int> out(failed_.begin(), failed_.end());
    failed_.clear();
    return out;
  }

  // In-process ingest (gateway): create tasks for payloads already written to `slots`.
  std::vector<std::string> submit(const std::vector<int64_t>& slots, const std::string& trace) {
    return enqueue(slots, trace);
  }

  // Tasks whose records already exist (explicit-TaskId upsert, journal replay) queued on this shard; returns how many
  // were queued (the rest hit backpressure).
  size_t send_existing(const std::vector<std::string>& ids, const std::vector<int64_t>& slots) {
    tag_slots(ids, slots);
    if (store_->journaled()) store_->flush();
    const size_t sent = queue_->send_many(ids, slots);
    if (stat_) stat_->enq.fetch_add(sent);
    return sent;
  }

  std::vector<std::string> wait_completed(double timeout_s) {
    std::unique_lock<std::mutex> lk(feed_mu_);
    cv_wait_s(feed_cv_, lk, timeout_s, [&] { return !feed_.empty() || stopped_; });
    std::vector<std::string> out(std::make_move_iterator(feed_.begin()), std::make_move_iterator(feed_.end()));
    feed_.clear();
    return out;
  }

  std::vector<WorkerStats> worker_stats() {
    std::vector<WorkerStats> out;
    std::lock_guard<std::mutex> g(mu_);
    const double now = mono_now();
    for (auto& kv : workers_) {
      Worker& w = *kv.second;
      std::lock_guard<std::mutex> wg(w.mu);
      WorkerStats s;
      s.rank = w.rank;
      s.ready = w.ready;
      s.alive = w.alive;
      s.pinned = w.pinned;
      s.batches = w.batches;
      s.images = w.images;
      s.failed_items = w.failed_items;
      s.retried_items = w.retried_items;
      s.outstanding = w.out.size();
      s.last_hb_age_s = now - w.last_hb;
      s.gpu_busy_ms = w.gpu_busy_ms;
      s.hbm_used = w.hbm_used;
      s.hbm_total = w.hbm_total;
      s.xgmi_tx = w.xgmi_tx;
      s.xgmi_rx = w.xgmi_rx;
      s.gfx_mhz = w.gfx_mhz;
      s.power_w = w.power_w;
      s.info = w.info;
      out.push_back(s);
    }
    return out;
  }

  // Batch-size histogram: bucket i counts batches of size in (2^(i-1), 2^i].
  std::vector<uint64_t> batch_histogram() {
    std::lock_guard<std::mutex> g(hist_mu_);
    return hist_;
  }
  uint64_t images_done() const { return images_done_.load(); }

  void stop() {
    halted_.store(true);
    {
      std::lock_guard<std::mutex> g(fail_mu_);
      stopped_ = true;
    }
    fail_cv_.notify_all();
    feed_cv_.notify_all();
    for (;;) {  // until no worker is left (an attach racing with stop is refused after stopped_)
      std::vector<std::unique_ptr<Worker>> ws;
      {
        std::lock_guard<std::mutex> g(mu_);
        for (auto& kv : workers_) ws.push_back(std::move(kv.second));
        workers_.clear();
      }
      if (ws.empty()) break;
      for (auto& w : ws) {
        send_simple(*w, F_STOP);
        mark_dead(*w, "stopped", false);
      }
      queue_->kick();
      for (auto& w : ws) join_worker(*w);
    }
  }

 private:
  struct Outstanding {
    std::vector<std::string> ids;
    std::vector<uint64_t> seqs;
    std::vector<int64_t> slots;
    std::shared_ptr<NodeScheduler> src;  // the peer shard whose queue the batch came from (null: this one)
  };
  struct Worker {
    int rank = -1;
    int fd = -1;
    bool dispatch = true;
    std::thread reader, dispatcher;
    std::mutex send_mu;
    std::mutex mu;  // guards everything below
    std::condition_variable cv;
    std::atomic<bool> alive{false};
    bool ready = false, draining = false, pinned = false;
    bool live_counted = false;  // counted in live_ (a ready dispatch worker)
    double last_hb = 0;
    std::unordered_map<uint64_t, Outstanding> out;
    uint64_t batches = 0, images = 0, failed_items = 0, retried_items = 0;
    double gpu_busy_ms = 0, gfx_mhz = 0, power_w = 0;
    uint64_t hbm_used = 0, hbm_total = 0, xgmi_tx = 0, xgmi_rx = 0;
    std::string info;
  };
  struct RemotePart {
    int64_t base, len;
    int rank;
  };

  // ------------------------------------------------------------------ framing
  static bool read_exact(int fd, void* buf, size_t n) {
    char* p = static_cast<char*>(buf);
    while (n) {
      ssize_t k = ::recv(fd, p, n, 0);
      if (k == 0) return false;
      if (k < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      p += k;
      n -= static_cast<size_t>(k);
    }
    return true;
  }
  static bool write_all(int fd, const void* buf, size_t n) {
    const char* p = static_cast<const char*>(buf);
    while (n) {
      ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
      if (k < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      p += k;
      n -= static_cast<size_t>(k);
    }
    return true;
  }
  // Buffered frame reader of one connection: one recv() usually brings several small frames (SUBMIT_IDS of many
  // front-end requests, heartbeats, DONE headers), each then parsed without a syscall of its own.
  struct FrameReader {
    int fd;
    std::vector<char> buf = std::vector<char>(1 << 18);
    size_t pos = 0, end = 0;
    bool fill(size_t need) {  // at least `need` unread bytes buffered
      if (end - pos >= need) return true;
      if (pos) {
        std::memmove(buf.data(), buf.data() + pos, end - pos);
        end -= pos;
        pos = 0;
      }
      if (need > buf.size()) buf.resize(need);
      while (end < need) {
        const ssize_t k = ::recv(fd, buf.data() + end, buf.size() - end, 0);
        if (k == 0) return false;
        if (k < 0) {
          if (errno == EINTR) continue;
          return false;
        }
        end += static_cast<size_t>(k);
      }
      return true;
    }
    bool next(std::string& out) {
      if (!fill(4)) return false;
      int32_t be;
      std::memcpy(&be, buf.data() + pos, 4);
      int64_t len = static_cast<int32_t>(ntohl(static_cast<uint32_t>(be)));
      size_t hdr = 4;
      if (len == -1) {  // multiprocessing's >2 GiB form: 8-byte big-endian length follows
        if (!fill(12)) return false;
        uint64_t be8;
        std::memcpy(&be8, buf.data() + pos + 4, 8);
        len = static_cast<int64_t>(be64toh(be8));
        hdr = 12;
      }
      if (len < 4) return false;
      if (static_cast<size_t>(len) > (1u << 20)) {  // a large frame (a DONE of big result rows): straight into `out`
        out.resize(static_cast<size_t>(len));
        const size_t have = std::min(end - pos - hdr, out.size());
        std::memcpy(out.data(), buf.data() + pos + hdr, have);
        pos = end = 0;
        return have == out.size() || read_exact(fd, out.data() + have, out.size() - have);
      }
      if (!fill(hdr + static_cast<size_t>(len))) return false;
      out.assign(buf.data() + pos + hdr, static_cast<size_t>(len));
      pos += hdr + static_cast<size_t>(len);
      return true;
    }
  };
  bool send_frame(Worker& w, const std::string& payload) {
    std::lock_guard<std::mutex> g(w.send_mu);
    if (w.fd < 0) return false;
    uint32_t be = htonl(static_cast<uint32_t>(payload.size()));
    struct iovec iov[2] = {{&be, 4}, {const_cast<char*>(payload.data()), payload.size()}};
    size_t left = 4 + payload.size();
    int idx = 0;
    while (left) {  // one sendmsg for the length prefix and the payload (partial writes resume mid-iovec)
      msghdr mh{};
      mh.msg_iov = iov + idx;
      mh.msg_iovlen = static_cast<size_t>(2 - idx);
      const ssize_t k = ::sendmsg(w.fd, &mh, MSG_NOSIGNAL);
      if (k < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      size_t kk = static_cast<size_t>(k);
      left -= kk;
      while (idx < 2 && kk >= iov[idx].iov_len) {
        kk -= iov[idx].iov_len;
        ++idx;
      }
      if (idx < 2) {
        iov[idx].iov_base = static_cast<char*>(iov[idx].iov_base) + kk;
        iov[idx].iov_len -= kk;
      }
    }
    return true;
  }
  bool send_simple(Worker& w, uint32_t type) {
    std::string p(4, '\0');
    std::memcpy(p.data(), &type, 4);
    return send_frame(w, p);
  }
  bool send_slots(Worker& w, uint32_t type, uint64_t bid, const std::vector<int64_t>& slots, bool with_bid) {
    std::string p;
    p.resize(4 + (with_bid ? 8 : 0) + 8 + slots.size() * 8);
    char* q = p.data();
    std::memcpy(q, &type, 4);
    q += 4;
    if (with_bid) {
      std::memcpy(q, &bid, 8);
      q += 8;
    }
    const uint32_t n = static_cast<uint32_t>(slots.size()), z = 0;
    std::memcpy(q, &n, 4);
    std::memcpy(q + 4, &z, 4);
    q += 8;
    if (!slots.empty()) std::memcpy(q, slots.data(), slots.size() * 8);
    return send_frame(w, p);
  }

  // ------------------------------------------------------------------ slots / tasks
  void free_slots(const std::vector<int64_t>& slots) {
    if (slots.empty()) return;
    std::vector<std::shared_ptr<SlotRing>> locals;
    std::vector<RemotePart> parts;
    {
      std::lock_guard<std::mutex> g(mu_);
      locals = local_rings_;
      parts = remote_parts_;
    }
    for (auto& r : locals) r->free(slots);
    for (const auto& p : parts) {
      std::vector<int64_t> mine;
      for (int64_t s : slots)
        if (s >= p.base && s < p.base + p.len) mine.push_back(s);
      if (mine.empty()) continue;
      std::lock_guard<std::mutex> g(mu_);  // keeps the worker alive while its FREE frame is sent
      auto it = workers_.find(p.rank);
      if (it != workers_.end()) send_slots(*it->second, F_FREE, 0, mine, false);
    }
  }

  std::vector<std::string> enqueue(const std::vector<int64_t>& slots, const std::string& trace) {
    int shard = -1;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!store_shards_.empty()) shard = store_shards_[store_rr_++ % store_shards_.size()];
    }
    auto ids = shard < 0 ? store_->create_many(endpoint_, slots.size(), "created", trace)
                         : store_->create_many_in(static_cast<size_t>(shard), endpoint_, slots.size(), "created", trace);
    tag_slots(ids, slots);
    if (store_->journaled()) store_->flush();  // (the caller acknowledges these ids once this returns)
    const size_t sent = queue_->send_many(ids, slots);
    if (stat_) stat_->enq.fetch_add(sent);
    if (sent < ids.size()) {  // backpressure / closed: CacheConnectorUpsert.cs:181-199
      std::vector<std::string> rest(ids.begin() + static_cast<long>(sent), ids.end());
      std::vector<int64_t> rs(slots.begin() + static_cast<long>(sent), slots.end());
      store_->transition_many(rest, "failed", kPublishFailed);
      free_slots(rs);
      feed(rest);
    }
    return ids;
  }

  // SUBMIT_IDS: the front-end already answered its clients with these ids; a payload whose id could not be
  // created (duplicate) or queued is dropped and its slot freed.
  // SUBMIT_MULTI: every request's records (each with its own trace), then ONE tag pass, journal flush and queue
  // send for all of them. Returns the tasks created per request.
  std::vector<uint32_t> enqueue_ids_multi(std::vector<std::vector<int64_t>>& slots, std::vector<std::vector<std::string>>& ids,
                                          const std::vector<std::string>& traces) {
    std::vector<uint32_t> created(slots.size(), 0);
    std::vector<int64_t> all_slots, drop;
    std::vector<std::string> all_ids;
    for (size_t r = 0; r < slots.size(); ++r) {
      auto ok = store_->create_ids(endpoint_, ids[r], "created", traces[r]);
      for (size_t i = 0; i < ids[r].size(); ++i) {
        if (!ok[i]) {
          drop.push_back(slots[r][i]);
          continue;
        }
        all_ids.push_back(std::move(ids[r][i]));
        all_slots.push_back(slots[r][i]);
        ++created[r];
      }
    }
    free_slots(drop);
    tag_slots(all_ids, all_slots);
    if (store_->journaled()) store_->flush();
    const size_t sent = queue_->send_many(all_ids, all_slots);
    if (stat_) stat_->enq.fetch_add(sent);
    if (sent < all_ids.size()) {
      std::vector<std::string> rest(all_ids.begin() + static_cast<long>(sent), all_ids.end());
      std::vector<int64_t> rs(all_slots.begin() + static_cast<long>(sent), all_slots.end());
      store_->transition_many(rest, "failed", kPublishFailed);
      free_slots(rs);
      feed(rest);
    }
    return created;
  }

  size_t enqueue_ids(std::vector<int64_t> slots, std::vector<std::string> ids, const std::string& trace) {
    auto ok = store_->create_ids(endpoint_, ids, "created", trace);
    std::vector<int64_t> drop;
    size_t k = 0;
    for (size_t i = 0; i < ids.size(); ++i) {
      if (!ok[i]) {
        drop.push_back(slots[i]);
        continue;
      }
      if (k != i) {  // (a self move-assignment would empty the string)
        ids[k] = std::move(ids[i]);
        slots[k] = slots[i];
      }
      ++k;
    }
    ids.resize(k);
    slots.resize(k);
    free_slots(drop);
    tag_slots(ids, slots);
    if (store_->journaled()) store_->flush();  // (the front-end acknowledges these ids on SUBMITTED)
    const size_t sent = queue_->send_many(ids, slots);
    if (stat_) stat_->enq.fetch_add(sent);
    if (sent < ids.size()) {
      std::vector<std::string> rest(ids.begin() + static_cast<long>(sent), ids.end());
      std::vector<int64_t> rs(slots.begin() + static_cast<long>(sent), slots.end());
      store_->transition_many(rest, "failed", kPublishFailed);
      free_slots(rs);
      feed(rest);
    }
    return ids.size();
  }

  void tag_slots(const std::vector<std::string>& ids, const std::vector<int64_t>& slots) {
    if (!tags_) return;
    for (size_t i = 0; i < ids.size() && i < slots.size(); ++i) {
      if (slots[i] < 0 || slots[i] >= ring_slots_) continue;
      char* t = tags_ + static_cast<size_t>(slots[i]) * kTagBytes;
      const size_t n = std::min(ids[i].size(), kTagBytes - 1);
      std::memcpy(t, ids[i].data(), n);
      std::memset(t + n, 0, kTagBytes - n);
    }
  }

  // A connection with a declared ring partition (torchrun rank, ingest front-end) may only submit slots of
  // that partition; connections without one (spawned local workers do not submit) are not restricted.
  bool in_partition(int rank, const std::vector<int64_t>& slots) {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& pt : remote_parts_) {
      if (pt.rank != rank) continue;
      for (int64_t s : slots)
        if (s < pt.base || s >= pt.base + pt.len) return false;
      return true;
    }
    return true;
  }

  void feed(const std::vector<std::string>& ids) {
    {
      std::lock_guard<std::mutex> g(feed_mu_);
      if (!feed_on_) return;
      feed_.insert(feed_.end(), ids.begin(), ids.end());
    }
    feed_cv_.notify_all();
  }

  // Requeue (or dead-letter) items; returns ids that were dead-lettered (already failed).
  void requeue(const std::vector<std::string>& ids, const std::vector<uint64_t>& seqs,
               const std::vector<int64_t>& slots, double delay_s, const char* status) {
    if (ids.empty()) return;
    store_->transition_many(ids, "created", status);
    std::vector<std::string> dead;
    std::vector<int64_t> dead_slots;
    for (size_t i = 0; i < seqs.size(); ++i) {
      if (queue_->abandon(seqs[i], delay_s) == "deadlettered") {
        dead.push_back(ids[i]);
        dead_slots.push_back(slots[i]);
      }
    }
    queue_->take_deadletters();  // drained here: the scheduler fails them itself
    if (!dead.empty()) {
      if (stat_) stat_->done.fetch_add(dead.size());
      store_->transition_many(dead, "failed", kFailMaxRetries);
      free_slots(dead_slots);
      feed(dead);
    }
  }

  void set_live(Worker& w, bool on) {  // (w.mu held)
    if (w.live_counted == on) return;
    w.live_counted = on;
    const int v = live_.fetch_add(on ? 1 : -1) + (on ? 1 : -1);
    if (stat_) stat_->live.store(static_cast<uint64_t>(std::max(0, v)));
  }
  NodeScheduler& owner(const Outstanding& o) { return o.src ? *o.src : *this; }
  void add_inflight(NodeScheduler& own, size_t n, bool add) {
    if (!own.stat_ || !n) return;
    std::lock_guard<std::mutex> g(own.busy_mu_);  // (per batch: the 0 <-> busy transitions stay paired)
    const uint64_t now = static_cast<uint64_t>(mono_now() * 1e6);
    if (add) {
      if (own.stat_->inflight.fetch_add(n) == 0) own.stat_->busy_since_us.store(now);
      return;
    }
    own.stat_->batches.fetch_add(1);
    if (own.stat_->inflight.fetch_sub(n) == n) {
      const uint64_t t0 = own.stat_->busy_since_us.exchange(0);
      if (t0 && now > t0) own.stat_->busy_us.fetch_add(now - t0);
    }
  }

  void mark_dead(Worker& w, const char* why, bool report) {
    if (!w.alive.exchange(false)) return;
    std::unordered_map<uint64_t, Outstanding> out;
    {
      std::lock_guard<std::mutex> g(w.mu);
      out.swap(w.out);
      set_live(w, false);
      w.cv.notify_all();
    }
    for (auto& kv : out) {
      NodeScheduler& own = owner(kv.second);
      add_inflight(own, kv.second.ids.size(), false);
      own.requeue(kv.second.ids, kv.second.seqs, kv.second.slots, 0.0, kRequeued);
    }
    {
      std::lock_guard<std::mutex> g(w.send_mu);
      if (w.fd >= 0) ::shutdown(w.fd, SHUT_RDWR);
    }
    if (report) {
      {
        std::lock_guard<std::mutex> g(fail_mu_);
        failed_.push_back(w.rank);
        fail_reasons_.push_back(why);
      }
      fail_cv_.notify_all();
    }
  }

  void join_worker(Worker& w) {
    mark_dead(w, "joined", false);
    if (w.dispatcher.joinable()) w.dispatcher.join();
    if (w.reader.joinable()) w.reader.join();
    std::lock_guard<std::mutex> g(w.send_mu);
    if (w.fd >= 0) ::close(w.fd);
    w.fd = -1;
  }

  // ------------------------------------------------------------------ threads
  void dispatch_loop(Worker& w) {
    while (w.alive) {
      bool busy = false;
      {
        std::unique_lock<std::mutex> lk(w.mu);
        cv_wait_s(w.cv, lk, 0.05, [&] {
          return !w.alive || (w.ready && !w.draining && w.out.size() < static_cast<size_t>(cfg_.depth));
        });
        if (!w.alive) break;
        if (w.ready && mono_now() - w.last_hb > cfg_.hb_timeout_s) {
          lk.unlock();
          mark_dead(w, "heartbeat timeout", true);
          break;
        }
        if (!w.ready || w.draining || w.out.size() >= static_cast<size_t>(cfg_.depth)) continue;
        busy = !w.out.empty();
      }
      if (queue_->closed()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        continue;
      }
      std::shared_ptr<NodeScheduler> src;
      auto msgs = take_orphaned(src);
      if (msgs.empty()) {
        msgs = queue_->receive(cfg_.max_batch, cfg_.poll_s,
                               busy ? std::max(cfg_.linger_s, cfg_.busy_linger_s) : cfg_.linger_s);
        if (msgs.empty()) msgs = take_idle(src);
      }
      if (msgs.empty()) continue;
      NodeScheduler& own = src ? *src : *this;
      Outstanding o;
      o.src = src;
      std::vector<std::string> bad;
      std::vector<uint64_t> bad_seqs;
      o.ids.reserve(msgs.size());
      o.seqs.reserve(msgs.size());
      o.slots.reserve(msgs.size());
      for (auto& m : msgs) {
        // poison guard: a message without a valid payload slot (e.g. recovered after a restart
        // with its ring slot gone) fails on its own instead of poisoning the batch
        if (m.ref < 0 || m.ref >= own.ring_slots_) {
          bad.push_back(m.task_id);
          bad_seqs.push_back(m.seq);
          continue;
        }
        o.ids.push_back(std::move(m.task_id));
        o.seqs.push_back(m.seq);
        o.slots.push_back(m.ref);
      }
      if (!bad.empty()) {
        store_->transition_many(bad, "failed", kFailInvalid);
        own.queue_->complete(bad_seqs);
        if (own.stat_) own.stat_->done.fetch_add(bad.size());
        feed(bad);
      }
      if (o.ids.empty()) continue;
      store_->transition_many(o.ids, "running", "running");
      {
        std::lock_guard<std::mutex> g(hist_mu_);
        size_t b = 0;
        while ((size_t{1} << b) < o.ids.size() && b + 1 < hist_.size()) ++b;
        ++hist_[b];
      }
      const uint64_t bid = next_bid_.fetch_add(1);
      std::vector<int64_t> slots = o.slots;
      const size_t nitems = o.ids.size();
      bool died = false;
      {
        std::lock_guard<std::mutex> g(w.mu);
        died = !w.alive;
        if (!died) {
          add_inflight(own, nitems, true);
          w.out.emplace(bid, std::move(o));
        }
      }
      if (died) {  // died while we were receiving: hand the batch straight back
        own.requeue(o.ids, o.seqs, o.slots, 0.0, kRequeued);
        break;
      }
      if (!send_slots(w, F_BATCH, bid, slots, true)) {
        mark_dead(w, "send failed", true);
        break;
      }
    }
  }

  std::vector<std::shared_ptr<NodeScheduler>> live_peers() {
    std::vector<std::shared_ptr<NodeScheduler>> ps;
    std::lock_guard<std::mutex> g(mu_);
    ps.reserve(peers_.size());
    for (auto& wp : peers_)
      if (auto p = wp.lock())
        if (!p->halted_.load()) ps.push_back(std::move(p));
    return ps;
  }
  // (a) a peer shard without a live dispatch worker: its queued work is ours to finish, before our own
  std::vector<Message> take_orphaned(std::shared_ptr<NodeScheduler>& src) {
    if (!steal_orphans_.load() || peers_empty_()) return {};
    auto ps = live_peers();
    const size_t k = ps.size(), start = k ? steal_rr_.fetch_add(1) % k : 0;
    for (size_t i = 0; i < k; ++i) {
      auto& p = ps[(start + i) % k];
      if (p->live_.load() > 0 || p->queue_->depth() == 0) continue;
      auto m = p->queue_->receive(cfg_.max_batch, 0.0, 0.0);
      if (!m.empty()) {
        stolen_.fetch_add(m.size());
        src = p;
        return m;
      }
    }
    return {};
  }
  // (b) our queue stayed empty for a whole poll: help the peer with the deepest backlog of at least a full batch
  std::vector<Message> take_idle(std::shared_ptr<NodeScheduler>& src) {
    if (!steal_idle_.load() || peers_empty_()) return {};
    std::shared_ptr<NodeScheduler> best;
    size_t best_depth = 0;
    for (auto& p : live_peers()) {
      const size_t d = p->queue_->depth();
      if (d >= cfg_.max_batch && d > best_depth) {
        best_depth = d;
        best = p;
      }
    }
    if (!best) return {};
    auto m = best->queue_->receive(cfg_.max_batch, 0.0, 0.0);
    if (!m.empty()) {
      stolen_.fetch_add(m.size());
      src = best;
    }
    return m;
  }
  bool peers_empty_() {
    std::lock_guard<std::mutex> g(mu_);
    return peers_.empty();
  }

  void reader_loop(Worker& w) {
    std::string f;
    FrameReader rd{w.fd};
    while (true) {
      if (!rd.next(f)) {
        // an ingest front-end that went away (killed mid-upload) leaves no admitted-body backlog behind
        if (!w.dispatch && stat_ && w.rank >= kFrontendRank0 && w.rank - kFrontendRank0 < kStatFrontends)
          stat_->fe_pending[w.rank - kFrontendRank0].store(0);
        if (w.alive) mark_dead(w, "connection lost", true);
        return;
      }
      uint32_t type;
      std::memcpy(&type, f.data(), 4);
      const char* p = f.data() + 4;
      const size_t len = f.size() - 4;
      switch (type) {
        case F_READY: {
          std::lock_guard<std::mutex> g(w.mu);
          if (len >= 8) {
            int32_t pinned;
            std::memcpy(&pinned, p + 4, 4);
            w.pinned = pinned != 0;
            w.info.assign(p + 8, len - 8);
          }
          w.ready = true;
          w.last_hb = mono_now();
          if (w.dispatch && !w.draining && w.alive) set_live(w, true);
          w.cv.notify_all();
          break;
        }
        case F_HB: {
          std::lock_guard<std::mutex> g(w.mu);
          w.last_hb = mono_now();
          if (len >= 40) {
            std::memcpy(&w.hbm_used, p + 8, 8);
            std::memcpy(&w.hbm_total, p + 16, 8);
            std::memcpy(&w.gpu_busy_ms, p + 24, 8);
          }
          if (len >= 56) {
            std::memcpy(&w.xgmi_tx, p + 40, 8);
            std::memcpy(&w.xgmi_rx, p + 48, 8);
          }
          if (len >= 72) {
            std::memcpy(&w.gfx_mhz, p + 56, 8);
            std::memcpy(&w.power_w, p + 64, 8);
          }
          break;
        }
        case F_DONE:
          on_done(w, p, len);
          break;
        case F_SUBMIT: {
          if (len < 8) break;  // malformed: ignore
          uint32_t n;
          std::memcpy(&n, p, 4);
          if (len < 8 + n * 8ull) break;
          std::vector<int64_t> slots(n);
          if (n) std::memcpy(slots.data(), p + 8, n * 8ull);
          if (!in_partition(w.rank, slots)) break;  // slots outside the sender's ring partition
          enqueue(slots, std::string());
          break;
        }
        case F_SUBMIT_IDS: {
          if (len < 24) break;
          uint32_t n, tl, il, flags;
          uint64_t token;
          std::memcpy(&n, p, 4);
          std::memcpy(&tl, p + 4, 4);
          std::memcpy(&il, p + 8, 4);
          std::memcpy(&flags, p + 12, 4);
          std::memcpy(&token, p + 16, 8);
          if (len < 24 + n * (8ull + il) + tl) break;  // malformed: ignore
          std::vector<int64_t> slots(n);
          if (n) std::memcpy(slots.data(), p + 24, n * 8ull);
          if (!in_partition(w.rank, slots)) break;
          std::vector<std::string> ids(n);
          const char* q = p + 24 + n * 8ull;
          for (uint32_t i = 0; i < n; ++i) ids[i].assign(q + i * static_cast<size_t>(il), il);
          const uint32_t created = static_cast<uint32_t>(
              enqueue_ids(std::move(slots), std::move(ids), std::string(q + n * static_cast<size_t>(il), tl)));
          if (flags & 1u) {
            std::string ack(20, '\0');
            const uint32_t t = F_SUBMITTED, z = 0;
            std::memcpy(&ack[0], &t, 4);
            std::memcpy(&ack[4], &token, 8);
            std::memcpy(&ack[12], &created, 4);
            std::memcpy(&ack[16], &z, 4);
            send_frame(w, ack);
          }
          break;
        }
        case F_SUBMIT_MULTI: {
          if (len < 12) break;
          uint32_t nreq;
          uint64_t token;
          std::memcpy(&nreq, p, 4);
          std::memcpy(&token, p + 4, 8);
          std::vector<std::vector<int64_t>> slots;
          std::vector<std::vector<std::string>> ids;
          std::vector<std::string> traces;
          slots.reserve(nreq);
          ids.reserve(nreq);
          traces.reserve(nreq);
          size_t off = 12;
          bool bad = false;
          for (uint32_t r = 0; r < nreq && !bad; ++r) {
            if (len < off + 16) {
              bad = true;
              break;
            }
            uint32_t n, tl, il;
            std::memcpy(&n, p + off, 4);
            std::memcpy(&tl, p + off + 4, 4);
            std::memcpy(&il, p + off + 8, 4);
            off += 16;
            if (len < off + n * (8ull + il) + tl) {
              bad = true;
              break;
            }
            std::vector<int64_t> sl(n);
            if (n) std::memcpy(sl.data(), p + off, n * 8ull);
            off += n * 8ull;
            std::vector<std::string> rid(n);
            for (uint32_t i = 0; i < n; ++i) rid[i].assign(p + off + i * static_cast<size_t>(il), il);
            off += n * static_cast<size_t>(il);
            traces.emplace_back(p + off, tl);
            off += tl;
            if (!in_partition(w.rank, sl)) {  // (outside the sender's partition: this request creates nothing)
              sl.clear();
              rid.clear();
            }
            slots.push_back(std::move(sl));
            ids.push_back(std::move(rid));
          }
          if (bad) break;  // malformed: ignore
          const auto created = enqueue_ids_multi(slots, ids, traces);
          std::string ack(16 + 4 * created.size(), '\0');
          const uint32_t t = F_SUBMITTED_MULTI, nr = static_cast<uint32_t>(created.size());
          std::memcpy(&ack[0], &t, 4);
          std::memcpy(&ack[4], &token, 8);
          std::memcpy(&ack[12], &nr, 4);
          if (nr) std::memcpy(&ack[16], created.data(), 4ull * nr);
          send_frame(w, ack);
          break;
        }
        case F_STAGE: {
          if (len < 12) break;  // malformed: ignore
          uint64_t bid;
          uint32_t stage;
          std::memcpy(&bid, p, 8);
          std::memcpy(&stage, p + 8, 4);
          on_stage(w, bid, stage);
          break;
        }
        default:
          break;
      }
    }
  }

  void on_stage(Worker& w, uint64_t bid, uint32_t stage) {
    std::vector<std::string> ids;
    {
      std::lock_guard<std::mutex> g(w.mu);
      auto it = w.out.find(bid);
      if (it == w.out.end()) return;
      ids = it->second.ids;
    }
    std::string ep, st;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stage >= stage_eps_.size()) return;
      ep = stage_eps_[stage];
      st = stage_status_[stage];
    }
    store_->retarget_many(ids, ep, st);
  }

  void on_done(Worker& w, const char* p, size_t len) {
    if (len < 16 + 40) return;
    uint64_t bid;
    uint32_t n, row_bytes;
    std::memcpy(&bid, p, 8);
    std::memcpy(&n, p + 8, 4);
    std::memcpy(&row_bytes, p + 12, 4);
    auto res = std::make_shared<ResultBatch>();
    std::memcpy(res->stage, p + 16, 40);
    res->row_bytes = row_bytes;
    res->worker = w.rank;
    const char* status = p + 56;
    const size_t spad = (static_cast<size_t>(n) + 7) / 8 * 8;
    const size_t need = 56 + spad + static_cast<size_t>(n) * row_bytes;
    Outstanding o;
    {
      std::lock_guard<std::mutex> g(w.mu);
      auto it = w.out.find(bid);
      if (it == w.out.end()) return;  // batch was already requeued (worker declared dead)
      o = std::move(it->second);
      w.out.erase(it);
    }
    NodeScheduler& own = owner(o);
    add_inflight(own, o.ids.size(), false);
    if (len < need || n != o.ids.size()) {  // malformed: treat the batch as a model error
      std::vector<uint8_t> none(o.ids.size(), 0);
      store_->finish_many(o.ids, nullptr, none, "completed", kFailError);
      own.queue_->complete(o.seqs);
      own.free_slots(o.slots);
      if (own.stat_) own.stat_->done.fetch_add(o.ids.size());
      feed(o.ids);
    } else {
      res->data.assign(status + spad, static_cast<size_t>(n) * row_bytes);
      std::vector<uint8_t> ok(n);
      std::vector<std::string> done_ids, invalid, retry;
      std::vector<uint64_t> done_seqs, retry_seqs;
      std::vector<int64_t> free_s, retry_slots;
      bool any_err = false;
      for (uint32_t i = 0; i < n; ++i) {
        const uint8_t s = static_cast<uint8_t>(status[i]);
        if (s == IT_RETRY) {
          retry.push_back(o.ids[i]);
          retry_seqs.push_back(o.seqs[i]);
          retry_slots.push_back(o.slots[i]);
          continue;
        }
        ok[i] = s == IT_OK;
        if (s == IT_INVALID) invalid.push_back(o.ids[i]);
        if (s == IT_ERROR) any_err = true;
        done_seqs.push_back(o.seqs[i]);
        free_s.push_back(o.slots[i]);
      }
      std::shared_ptr<const ResultBatch> cres = res;
      if (retry.empty()) {
        store_->finish_many(o.ids, cres, ok, "completed", kFailError);
      } else {  // finish only the non-retried items (retried ones keep their slot and message)
        std::vector<std::string> fin;
        std::vector<uint8_t> fok;
        std::shared_ptr<ResultBatch> sub = std::make_shared<ResultBatch>();
        *sub = *res;
        sub->data.clear();
        for (uint32_t i = 0; i < n; ++i) {
          if (static_cast<uint8_t>(status[i]) == IT_RETRY) continue;
          fin.push_back(o.ids[i]);
          fok.push_back(ok[i]);
          sub->data.append(res->data, static_cast<size_t>(i) * row_bytes, row_bytes);
        }
        store_->finish_many(fin, sub, fok, "completed", kFailError);
      }
      if (!invalid.empty()) store_->transition_many(invalid, "failed", kFailInvalid);
      own.queue_->complete(done_seqs);
      own.free_slots(free_s);
      if (!retry.empty()) own.requeue(retry, retry_seqs, retry_slots, cfg_.retry_delay_s,
                                      "Awaiting service availability. Batch failed; retrying.");
      size_t nfail = 0;
      for (uint32_t i = 0; i < n; ++i) nfail += status[i] == IT_INVALID || status[i] == IT_ERROR;
      (void)any_err;
      {
        std::lock_guard<std::mutex> g(w.mu);
        w.batches += 1;
        w.images += n - retry.size() - nfail;
        w.failed_items += nfail;
        w.retried_items += retry.size();
      }
      images_done_.fetch_add(n - retry.size());
      if (own.stat_) own.stat_->done.fetch_add(n - retry.size());
      std::vector<std::string> fed;
      fed.reserve(n);
      for (uint32_t i = 0; i < n; ++i)
        if (static_cast<uint8_t>(status[i]) != IT_RETRY) fed.push_back(o.ids[i]);
      feed(fed);
    }
    w.cv.notify_all();
  }

  std::shared_ptr<TaskStore> store_;
  std::shared_ptr<DispatchQueue> queue_;
  std::string endpoint_;
  int64_t ring_slots_;
  SchedConfig cfg_;
  std::mutex mu_;
  std::map<int, std::unique_ptr<Worker>> workers_;
  std::vector<std::shared_ptr<SlotRing>> local_rings_;
  std::vector<RemotePart> remote_parts_;
  std::vector<std::string> stage_eps_, stage_status_;
  std::vector<int> store_shards_;
  size_t store_rr_ = 0;
  std::vector<std::weak_ptr<NodeScheduler>> peers_;
  std::atomic<bool> steal_orphans_{true}, steal_idle_{true}, halted_{false};
  std::atomic<size_t> steal_rr_{0};
  std::atomic<uint64_t> stolen_{0};
  std::atomic<int> live_{0};
  std::atomic<uint64_t> next_bid_{1};
  std::atomic<uint64_t> images_done_{0};
  ShardStat* stat_ = nullptr;
  std::mutex busy_mu_;  // (add_inflight: busy-interval bookkeeping)
  std::string stat_name_;
  char* tags_ = nullptr;
  std::mutex fail_mu_;
  std::condition_variable fail_cv_;
  std::vector<int> failed_;
  std::vector<std::string> fail_reasons_;
  bool stopped_ = false;
  std::mutex feed_mu_;
  std::condition_variable feed_cv_;
  std::deque<std::string> feed_;
  bool feed_on_ = false;
  std::mutex hist_mu_;
  std::vector<uint64_t> hist_;
};

}  // namespace ai4e
