// TaskStore — the reference's Redis task cache (CacheConnectorUpsert.cs:92-176,
// CacheConnectorGet.cs:56-65, CurrentProcessingUpsert.cs:102-104, QueueLogger.cs:21-47) as one
// in-process object.
//
// Layout is built for the node-scale hot path (8 GPUs x ~70k tasks/s, three mutations per task):
//  * records live in a node-based hash map, so a record's address is stable and the per-state
//    indexes are intrusive doubly-linked lists threaded through the records: ZADD/ZREM are O(1)
//    pointer moves, ZCARD is a counter, ZRANGE walks the list (insertion order == score order,
//    since scores are the wall-clock second of the mutation);
//  * a task is in exactly one "{EndpointPath}_{BackendStatus}" set at a time (the reference's
//    running/completed/failed ZREMs, plus removal from _created for tasks failed before they ran);
//  * status strings are shared (one allocation per batch transition), timestamps are stored as
//    epoch seconds and formatted on read;
//  * model results are attached to the record (one shared buffer per GPU batch, a row per task),
//    so eviction of finished tasks (TTL, oldest first) also frees their results.
// All methods take the store mutex once per call (batch calls: once per batch).
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace ai4e {

enum : int { ST_CREATED = 0, ST_RUNNING = 1, ST_COMPLETED = 2, ST_FAILED = 3 };

struct TaskRec;

struct IndexList {
  TaskRec* head = nullptr;
  TaskRec* tail = nullptr;
  size_t n = 0;
  bool touched = false;  // the Redis key "exists" for KEYS (the reference's ZREM also creates nothing,
                         // but the python executable spec keeps touched keys; both agree here)
};

struct PathIndex {
  std::string path;
  std::deque<IndexList> lists;  // by backend-state id; a deque so growth keeps list addresses stable
};

// One GPU batch's outputs: item-major rows (row r = every output of task r, concatenated).
struct ResultBatch {
  std::string data;
  uint32_t row_bytes = 0;
  // worker-side stage times (CLOCK_MONOTONIC s) + GPU durations (ms): recv, launch, done, h2d_ms, compute_ms
  double stage[5] = {0, 0, 0, 0, 0};
  int32_t worker = -1;
};

struct TaskRec {
  const std::string* idp = nullptr;               // the record's key in the map (node-stable)
  std::shared_ptr<const std::string> endpoint;    // shared by every task of a batch
  const std::string& id() const { return *idp; }
  PathIndex* pidx = nullptr;
  IndexList* list = nullptr;
  TaskRec* prev = nullptr;
  TaskRec* next = nullptr;
  std::shared_ptr<const std::string> status;
  std::string trace;  // B3 trace context "traceid/spanid" (optional)
  double wall = 0;    // epoch seconds of the last mutation (the Timestamp field)
  double score = 0;
  double t_created = 0, t_running = 0, t_finished = 0;  // CLOCK_MONOTONIC
  int state = -1;
  bool pub = false;
  std::shared_ptr<const ResultBatch> res;
  uint32_t row = 0;
};

// Append-only journal shared by the shards (its own lock; taken while a shard lock is held).
struct Journal {
  FILE* f = nullptr;
  bool paused = false;
  std::mutex mu;
  void write(const std::string& line) {
    std::lock_guard<std::mutex> g(mu);
    if (f && !paused) std::fwrite(line.data(), 1, line.size(), f);
  }
};

// Which shard owns a task id: its last character (hex digit value, else the byte) modulo the shard
// count. Ids minted by the store carry their shard in that digit; upstream ids spread by it.
inline size_t shard_of(const std::string& id, size_t nshards) {
  if (id.empty() || nshards <= 1) return 0;
  const unsigned char c = static_cast<unsigned char>(id.back());
  const unsigned v = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                     : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : c;
  return v % nshards;
}

// One lock domain of the task store: records, per-(path, state) indexes, _ORIG bodies.
class StoreShard {
 public:
  StoreShard(size_t shard = 0, size_t nshards = 1, Journal* journal = nullptr)
      : shard_(shard), nshards_(nshards), journal_(journal) {
    for (const char* s : {"created", "running", "completed", "failed"}) state_id(s);
    recs_.reserve((1 << 20) / nshards);  // a node's worth of in-flight + retained tasks without rehash stalls
  }
  StoreShard(const StoreShard&) = delete;
  StoreShard& operator=(const StoreShard&) = delete;

  // A fresh UUID whose last hex digit routes to this shard.
  std::string mint_id() {
    std::string id = uuid_.next();
    if (nshards_ > 1) {
      static const char* hex = "0123456789abcdef";
      const unsigned d = static_cast<unsigned>(shard_) + static_cast<unsigned>(nshards_) * (uuid_rnd_++ & 1);
      id.back() = hex[d & 15];
    }
    return id;
  }

  // CacheConnectorUpsert (CacheConnectorUpsert.cs:92-176): returns the serialized task (Body
  // nulled) and the body to publish (the original "{TaskId}_ORIG" body on a pipeline re-publish).
  std::pair<std::string, std::optional<std::string>> upsert(std::string task_id, const std::string& status,
                                                            const std::string& backend_status,
                                                            const std::string& endpoint,
                                                            const std::optional<std::string>& body,
                                                            bool publish_to_grid) {
    std::lock_guard<std::mutex> g(mu_);
    if (task_id.find_first_not_of(" \t\r\n") == std::string::npos) task_id = mint_id();
    const double wnow = wall_now(), mnow = mono_now();
    auto ins = recs_.try_emplace(task_id);
    TaskRec& r = ins.first->second;
    if (ins.second) {
      r.idp = &ins.first->first;
      r.t_created = mnow;
    }
    PathIndex* p = path_index(absolute_path(endpoint));
    r.endpoint = shared_endpoint(endpoint);
    r.status = std::make_shared<const std::string>(status);
    r.pub = publish_to_grid;
    r.wall = wnow;
    move_to(r, p, state_id(backend_status), wnow, mnow);
    std::optional<std::string> publish_body;
    if (publish_to_grid) {
      if (body && !body->empty()) {
        orig_[task_id] = *body;
        publish_body = *body;
      } else {  // subsequent pipeline call: reuse "{TaskId}_ORIG"
        auto it = orig_.find(task_id);
        publish_body = it == orig_.end() ? std::string() : it->second;
      }
    }
    journal_write(r, publish_to_grid && body && !body->empty() ? &*body : nullptr);
    return {serialize(r), publish_body};
  }

  // Hot path: n new tasks for one endpoint (BackendStatus "created").
  std::vector<std::string> create_many(const std::string& endpoint, size_t n, const std::string& status,
                                       const std::string& trace = std::string()) {
    std::vector<std::string> ids;
    ids.reserve(n);
    std::lock_guard<std::mutex> g(mu_);
    const double wnow = wall_now(), mnow = mono_now();
    PathIndex* p = path_index(absolute_path(endpoint));
    auto st = std::make_shared<const std::string>(status);
    auto ep = shared_endpoint(endpoint);
    for (size_t i = 0; i < n; ++i) {
      std::string id = mint_id();
      auto ins = recs_.try_emplace(id);
      if (!ins.second) {  // 2^-122 collision: draw again
        --i;
        continue;
      }
      TaskRec& r = ins.first->second;
      r.idp = &ins.first->first;
      r.endpoint = ep;
      r.status = st;
      r.pub = true;
      r.wall = wnow;
      r.t_created = mnow;
      r.trace = trace;
      move_to(r, p, ST_CREATED, wnow, mnow);
      journal_write(r, nullptr);
      ids.push_back(std::move(id));
    }
    return ids;
  }

  // create_many with ids minted by the caller (an ingest front-end process); an id already present is
  // left untouched and reported as not created (ok[i] = 0).
  std::vector<uint8_t> create_ids(const std::string& endpoint, const std::vector<std::string>& ids,
                                  const std::string& status, const std::string& trace = std::string()) {
    std::vector<uint8_t> ok(ids.size(), 0);
    std::lock_guard<std::mutex> g(mu_);
    const double wnow = wall_now(), mnow = mono_now();
    PathIndex* p = path_index(absolute_path(endpoint));
    auto st = std::make_shared<const std::string>(status);
    auto ep = shared_endpoint(endpoint);
    for (size_t i = 0; i < ids.size(); ++i) {
      auto ins = recs_.try_emplace(ids[i]);
      if (!ins.second) continue;
      TaskRec& r = ins.first->second;
      r.idp = &ins.first->first;
      r.endpoint = ep;
      r.status = st;
      r.pub = true;
      r.wall = wnow;
      r.t_created = mnow;
      r.trace = trace;
      move_to(r, p, ST_CREATED, wnow, mnow);
      journal_write(r, nullptr);
      ok[i] = 1;
    }
    return ok;
  }

  // Hot path: move tasks to running / completed / failed (any backend state) in one lock.
  size_t transition_many(const std::vector<std::string>& ids, const std::string& backend_status,
                         const std::string& status) {
    std::lock_guard<std::mutex> g(mu_);
    const double wnow = wall_now(), mnow = mono_now();
    const int sid = state_id(backend_status);
    auto st = std::make_shared<const std::string>(status);
    size_t n = 0;
    for (const auto& id : ids) {
      auto it = recs_.find(id);
      if (it == recs_.end()) continue;
      TaskRec& r = it->second;
      r.status = st;
      r.wall = wnow;
      move_to(r, r.pidx, sid, wnow, mnow);
      journal_write(r, nullptr);
      ++n;
    }
    return n;
  }

  // Pipeline hop (AddPipelineTask, distributed_api_task.py:67-100 -> CacheConnectorUpsert.cs:144-176):
  // the same TaskIds re-targeted at the next endpoint, then marked running there.
  size_t retarget_many(const std::vector<std::string>& ids, const std::string& endpoint, const std::string& status) {
    std::lock_guard<std::mutex> g(mu_);
    const double wnow = wall_now(), mnow = mono_now();
    PathIndex* p = path_index(absolute_path(endpoint));
    auto st = std::make_shared<const std::string>(status);
    auto ep = shared_endpoint(endpoint);
    size_t n = 0;
    for (const auto& id : ids) {
      auto it = recs_.find(id);
      if (it == recs_.end()) continue;
      TaskRec& r = it->second;
      r.endpoint = ep;
      r.status = st;
      r.wall = wnow;
      move_to(r, p, ST_CREATED, wnow, mnow);
      journal_write(r, nullptr);
      move_to(r, p, ST_RUNNING, wnow, mnow);
      journal_write(r, nullptr);
      ++n;
    }
    return n;
  }

  // Finish a batch: attach results (row r of `res` to ids[r]) and set per-task final states.
  // ok[r] != 0 -> completed with `status_ok`, else failed with `status_fail`.
  void finish_many(const std::vector<std::string>& ids, const std::shared_ptr<const ResultBatch>& res,
                   const std::vector<uint8_t>& ok, const std::string& status_ok, const std::string& status_fail,
                   const std::vector<uint32_t>* rows = nullptr) {
    std::lock_guard<std::mutex> g(mu_);
    const double wnow = wall_now(), mnow = mono_now();
    auto sok = std::make_shared<const std::string>(status_ok);
    auto sfail = std::make_shared<const std::string>(status_fail);
    for (size_t i = 0; i < ids.size(); ++i) {
      auto it = recs_.find(ids[i]);
      if (it == recs_.end()) continue;
      TaskRec& r = it->second;
      const bool good = ok.empty() || ok[rows ? (*rows)[i] : i];
      r.status = good ? sok : sfail;
      r.wall = wnow;
      if (good && res) {
        r.res = res;
        r.row = rows ? (*rows)[i] : static_cast<uint32_t>(i);
      }
      move_to(r, r.pidx, good ? ST_COMPLETED : ST_FAILED, wnow, mnow);
      journal_write(r, nullptr);
    }
  }

  // BackendQueueProcessor.UpdateTaskStatus (BackendQueueProcessor.cs:83-133): Status text only.
  bool set_status_text(const std::string& id, const std::string& status) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = recs_.find(id);
    if (it == recs_.end()) return false;
    it->second.status = std::make_shared<const std::string>(status);
    it->second.wall = wall_now();
    journal_write(it->second, nullptr);
    return true;
  }

  bool set_trace(const std::string& id, const std::string& trace) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = recs_.find(id);
    if (it == recs_.end()) return false;
    it->second.trace = trace;
    return true;
  }

  std::optional<std::string> get(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = recs_.find(id);
    if (it == recs_.end()) return std::nullopt;
    return serialize(it->second);
  }

  // Copy of one record's public fields (bindings turn it into a dict without holding the lock).
  struct View {
    std::string id, timestamp, status, backend_status, endpoint, path, trace;
    bool pub = false;
    double t_created = 0, t_running = 0, t_finished = 0;
    std::shared_ptr<const ResultBatch> res;
    uint32_t row = 0;
  };
  std::optional<View> view(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = recs_.find(id);
    if (it == recs_.end()) return std::nullopt;
    const TaskRec& r = it->second;
    View v;
    v.id = r.id();
    v.timestamp = dotnet_timestamp(r.wall);
    v.status = r.status ? *r.status : std::string();
    v.backend_status = state_names_[r.state];
    v.endpoint = *r.endpoint;
    v.path = r.pidx->path;
    v.trace = r.trace;
    v.pub = r.pub;
    v.t_created = r.t_created;
    v.t_running = r.t_running;
    v.t_finished = r.t_finished;
    v.res = r.res;
    v.row = r.row;
    return v;
  }

  std::optional<std::string> get_orig_body(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = orig_.find(id);
    if (it == orig_.end()) return std::nullopt;
    return it->second;
  }

  // Seconds from create to finish (or to running) for each id that got there.
  std::vector<double> latencies(const std::vector<std::string>& ids, bool to_running) {
    std::vector<double> out;
    out.reserve(ids.size());
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& id : ids) {
      auto it = recs_.find(id);
      if (it == recs_.end()) continue;
      const TaskRec& r = it->second;
      const double end = to_running ? r.t_running : r.t_finished;
      if (end > 0) out.push_back(end - r.t_created);
    }
    return out;
  }

  // Create->finish latency of every task of `path` that finished in [t0, t1] (CLOCK_MONOTONIC).
  std::vector<double> latencies_window(const std::string& path, double t0, double t1) {
    std::vector<double> out;
    std::lock_guard<std::mutex> g(mu_);
    auto pit = paths_.find(path);
    if (pit == paths_.end()) return out;
    for (int s : {ST_COMPLETED, ST_FAILED}) {
      const IndexList& l = pit->second->lists[s];
      for (TaskRec* r = l.head; r; r = r->next)
        if (r->t_finished >= t0 && r->t_finished <= t1) out.push_back(r->t_finished - r->t_created);
    }
    return out;
  }

  size_t zcard(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    const IndexList* l = find_list(key);
    return l ? l->n : 0;
  }

  std::vector<std::pair<double, std::string>> zrange_scored(const std::string& key, size_t limit) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::pair<double, std::string>> out;
    const IndexList* l = find_list(key);
    if (!l) return out;
    for (TaskRec* r = l->head; r && out.size() < limit; r = r->next) out.emplace_back(r->score, r->id());
    return out;
  }

  // Redis "KEYS *{suffix}" over the index namespace (QueueLogger.cs:21-47).
  std::vector<std::string> keys_with_suffix(const std::string& suffix) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> out;
    for (const auto& kv : paths_) {
      const PathIndex& p = *kv.second;
      for (size_t s = 0; s < p.lists.size(); ++s) {
        if (!p.lists[s].touched) continue;
        std::string k = p.path + "_" + state_names_[s];
        if (k.size() >= suffix.size() && k.compare(k.size() - suffix.size(), suffix.size(), suffix) == 0)
          out.push_back(std::move(k));
      }
    }
    std::sort(out.begin(), out.end());
    return out;
  }

  // Drop completed/failed records finished more than max_age_s ago, oldest first: the finished
  // lists are in finish order, so this costs O(evicted), not O(store).
  // `max_finished` caps the finished records kept per (path, state) regardless of age (a node at
  // ~550k tasks/s cannot keep an hour of results): the oldest beyond the cap go first.
  size_t evict_finished(double max_age_s, size_t max_finished = SIZE_MAX) {
    std::lock_guard<std::mutex> g(mu_);
    const double cutoff = mono_now() - max_age_s;
    size_t n = 0;
    for (auto& kv : paths_) {
      for (int s : {ST_COMPLETED, ST_FAILED}) {
        IndexList& l = kv.second->lists[s];
        while (l.head && l.head->t_finished > 0 && (l.head->t_finished <= cutoff || l.n > max_finished)) {
          TaskRec* r = l.head;
          unlink(*r);
          orig_.erase(r->id());
          recs_.erase(recs_.find(r->id()));  // by iterator: the key lives in the node being erased
          ++n;
        }
      }
    }
    return n;
  }

  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return recs_.size();
  }

  // Journal replay: each line is a full record image (+ optional _ORIG body). `parse` turns one
  // JSON line into fields (bindings supply the Python json module; the core stays JSON-free).
  struct JournalLine {
    std::string id, timestamp, status, backend_status, endpoint;
    bool pub = false;
    double score = 0;
    std::optional<std::string> orig;
  };
  // Apply one journal line (replay; the journal is paused by the caller).
  void replay_line(const JournalLine& jl, double mnow) {
    std::lock_guard<std::mutex> g(mu_);
    auto ins = recs_.try_emplace(jl.id);
    TaskRec& r = ins.first->second;
    if (ins.second) {
      r.idp = &ins.first->first;
      r.t_created = mnow;
    }
    r.endpoint = shared_endpoint(jl.endpoint);
    r.status = std::make_shared<const std::string>(jl.status);
    r.pub = jl.pub;
    r.wall = jl.score;
    const int sid = state_id(jl.backend_status);
    PathIndex* p = path_index(absolute_path(jl.endpoint));
    if (r.list) unlink(r);
    r.pidx = p;
    r.state = sid;
    r.score = jl.score;
    link_tail(r, &p->lists[sid]);
    // finished records get a finish time, so TTL eviction applies to them too
    r.t_finished = (sid == ST_COMPLETED || sid == ST_FAILED) ? mnow : 0;
    if (jl.orig) orig_[r.id()] = *jl.orig;
  }

  const std::string& state_name(int s) const { return state_names_[s]; }

 private:
  // Endpoint strings are interned: a batch of tasks shares one allocation.
  std::shared_ptr<const std::string> shared_endpoint(const std::string& e) {
    auto it = endpoints_.find(e);
    if (it != endpoints_.end()) return it->second;
    auto p = std::make_shared<const std::string>(e);
    if (endpoints_.size() < 65536) endpoints_.emplace(e, p);
    return p;
  }

  int state_id(const std::string& s) {
    auto it = state_ids_.find(s);
    if (it != state_ids_.end()) return it->second;
    const int id = static_cast<int>(state_names_.size());
    state_names_.push_back(s);
    state_ids_.emplace(s, id);
    for (auto& kv : paths_) kv.second->lists.resize(state_names_.size());
    return id;
  }

  PathIndex* path_index(const std::string& path) {
    auto it = paths_.find(path);
    if (it != paths_.end()) return it->second.get();
    auto p = std::make_unique<PathIndex>();
    p->path = path;
    p->lists.resize(state_names_.size());
    PathIndex* raw = p.get();
    paths_.emplace(path, std::move(p));
    return raw;
  }

  const IndexList* find_list(const std::string& key) const {
    const auto us = key.rfind('_');
    if (us == std::string::npos) return nullptr;
    auto pit = paths_.find(key.substr(0, us));
    auto sit = state_ids_.find(key.substr(us + 1));
    if (pit == paths_.end() || sit == state_ids_.end()) return nullptr;
    return &pit->second->lists[sit->second];
  }

  static void unlink(TaskRec& r) {
    IndexList* l = r.list;
    if (!l) return;
    (r.prev ? r.prev->next : l->head) = r.next;
    (r.next ? r.next->prev : l->tail) = r.prev;
    r.prev = r.next = nullptr;
    r.list = nullptr;
    --l->n;
  }
  static void link_tail(TaskRec& r, IndexList* l) {
    r.prev = l->tail;
    r.next = nullptr;
    (l->tail ? l->tail->next : l->head) = &r;
    l->tail = &r;
    r.list = l;
    ++l->n;
    l->touched = true;
  }

  // ZADD "{path}_{state}" + the ZREMs of CacheConnectorUpsert.cs:125-142 (single membership).
  void move_to(TaskRec& r, PathIndex* p, int sid, double wnow, double mnow) {
    if (r.list) unlink(r);
    r.pidx = p;
    r.state = sid;
    r.score = static_cast<double>(static_cast<int64_t>(wnow));
    link_tail(r, &p->lists[sid]);
    if (sid == ST_RUNNING) {
      p->lists[ST_CREATED].touched = true;
      r.t_running = mnow;
    } else if (sid == ST_COMPLETED || sid == ST_FAILED) {
      p->lists[ST_RUNNING].touched = p->lists[ST_CREATED].touched = true;
      r.t_finished = mnow;
    } else if (sid == ST_CREATED) {
      for (int s : {ST_RUNNING, ST_COMPLETED, ST_FAILED}) p->lists[s].touched = true;
      r.t_finished = 0;
      r.res.reset();
    }
  }

  std::string serialize(const TaskRec& r) const {
    std::string out;
    out.reserve(256);
    out += "{\"TaskId\":";
    json_escape_into(out, r.id());
    out += ",\"Timestamp\":";
    json_escape_into(out, dotnet_timestamp(r.wall));
    out += ",\"Status\":";
    json_escape_into(out, r.status ? *r.status : std::string());
    out += ",\"BackendStatus\":";
    json_escape_into(out, state_names_[r.state]);
    out += ",\"Endpoint\":";
    json_escape_into(out, *r.endpoint);
    out += ",\"Body\":null,\"PublishToGrid\":";
    out += r.pub ? "true" : "false";
    out += ",\"EndpointPath\":";
    json_escape_into(out, r.pidx->path);
    out += "}";
    return out;
  }

  void journal_write(const TaskRec& r, const std::string* orig) {
    if (!journal_ || !journal_->f) return;
    std::string line = serialize(r);
    line.pop_back();
    line += ",\"_score\":" + std::to_string(static_cast<int64_t>(r.score));
    if (orig) {
      line += ",\"_orig\":";
      json_escape_into(line, *orig);
    }
    line += "}\n";
    journal_->write(line);
  }

  std::mutex mu_;
  size_t shard_, nshards_;
  Journal* journal_;
  Uuid4 uuid_;
  uint32_t uuid_rnd_ = 0;
  std::unordered_map<std::string, TaskRec> recs_;  // node-based: record addresses are stable
  std::unordered_map<std::string, std::shared_ptr<const std::string>> endpoints_;
  std::unordered_map<std::string, std::unique_ptr<PathIndex>> paths_;
  std::unordered_map<std::string, int> state_ids_;
  std::vector<std::string> state_names_;
  std::unordered_map<std::string, std::string> orig_;
};

// JournalLine is declared inside StoreShard's public section (replay parser output).
using JournalLine = StoreShard::JournalLine;

// TaskStore — the sharded store: ids route to one of S lock domains (shard_of), batches minted by
// create_many live in one shard (round-robin per call), so a node's ingest, dispatcher and reader
// threads contend on different locks; index queries (ZCARD, ZRANGE, KEYS) merge the shards.
class TaskStore {
 public:
  using View = StoreShard::View;
  using JournalLine = StoreShard::JournalLine;

  explicit TaskStore(std::string journal_path = "", size_t nshards = 8) : nshards_(std::max<size_t>(1, nshards)) {
    if (!journal_path.empty()) {
      journal_.f = std::fopen(journal_path.c_str(), "a");
      if (!journal_.f) throw std::runtime_error("cannot open journal " + journal_path);
    }
    for (size_t i = 0; i < nshards_; ++i) shards_.push_back(std::make_unique<StoreShard>(i, nshards_, &journal_));
  }
  ~TaskStore() {
    if (journal_.f) std::fclose(journal_.f);
  }
  TaskStore(const TaskStore&) = delete;
  TaskStore& operator=(const TaskStore&) = delete;

  size_t nshards() const { return nshards_; }
  StoreShard& shard_for(const std::string& id) { return *shards_[shard_of(id, nshards_)]; }

  std::pair<std::string, std::optional<std::string>> upsert(std::string task_id, const std::string& status,
                                                            const std::string& backend_status,
                                                            const std::string& endpoint,
                                                            const std::optional<std::string>& body,
                                                            bool publish_to_grid) {
    StoreShard& sh = task_id.find_first_not_of(" \t\r\n") == std::string::npos ? next_shard() : shard_for(task_id);
    return sh.upsert(std::move(task_id), status, backend_status, endpoint, body, publish_to_grid);
  }

  std::vector<std::string> create_many(const std::string& endpoint, size_t n, const std::string& status,
                                       const std::string& trace = std::string()) {
    return next_shard().create_many(endpoint, n, status, trace);
  }
  // The same in lock domain `shard` (mod nshards): a control-plane shard (one NodeScheduler per GPU) mints every id
  // in the store shards it owns, so shards never contend on each other's locks and an id names its owner.
  std::vector<std::string> create_many_in(size_t shard, const std::string& endpoint, size_t n, const std::string& status,
                                          const std::string& trace = std::string()) {
    return shards_[shard % nshards_]->create_many(endpoint, n, status, trace);
  }
  size_t shard_index(const std::string& id) const { return shard_of(id, nshards_); }

  std::vector<uint8_t> create_ids(const std::string& endpoint, const std::vector<std::string>& ids,
                                  const std::string& status, const std::string& trace = std::string()) {
    std::vector<uint8_t> ok(ids.size(), 0);
    for_groups(ids, [&](StoreShard& sh, const std::vector<std::string>& g, const std::vector<uint32_t>* pos) {
      auto r = sh.create_ids(endpoint, g, status, trace);
      for (size_t i = 0; i < r.size(); ++i) ok[pos ? (*pos)[i] : i] = r[i];
    });
    return ok;
  }

  size_t transition_many(const std::vector<std::string>& ids, const std::string& backend_status,
                         const std::string& status) {
    size_t n = 0;
    for_groups(ids, [&](StoreShard& sh, const std::vector<std::string>& g, const std::vector<uint32_t>*) {
      n += sh.transition_many(g, backend_status, status);
    });
    return n;
  }

  size_t retarget_many(const std::vector<std::string>& ids, const std::string& endpoint, const std::string& status) {
    size_t n = 0;
    for_groups(ids, [&](StoreShard& sh, const std::vector<std::string>& g, const std::vector<uint32_t>*) {
      n += sh.retarget_many(g, endpoint, status);
    });
    return n;
  }

  void finish_many(const std::vector<std::string>& ids, const std::shared_ptr<const ResultBatch>& res,
                   const std::vector<uint8_t>& ok, const std::string& status_ok, const std::string& status_fail) {
    for_groups(ids, [&](StoreShard& sh, const std::vector<std::string>& g, const std::vector<uint32_t>* rows) {
      sh.finish_many(g, res, ok, status_ok, status_fail, rows);
    });
  }

  bool set_status_text(const std::string& id, const std::string& status) {
    return shard_for(id).set_status_text(id, status);
  }
  bool set_trace(const std::string& id, const std::string& trace) { return shard_for(id).set_trace(id, trace); }
  std::optional<std::string> get(const std::string& id) { return shard_for(id).get(id); }
  std::optional<StoreShard::View> view(const std::string& id) { return shard_for(id).view(id); }
  std::optional<std::string> get_orig_body(const std::string& id) { return shard_for(id).get_orig_body(id); }

  std::vector<double> latencies(const std::vector<std::string>& ids, bool to_running) {
    std::vector<double> out;
    out.reserve(ids.size());
    for_groups(ids, [&](StoreShard& sh, const std::vector<std::string>& g, const std::vector<uint32_t>*) {
      auto v = sh.latencies(g, to_running);
      out.insert(out.end(), v.begin(), v.end());
    });
    return out;
  }
  std::vector<double> latencies_window(const std::string& path, double t0, double t1) {
    std::vector<double> out;
    for (auto& sh : shards_) {
      auto v = sh->latencies_window(path, t0, t1);
      out.insert(out.end(), v.begin(), v.end());
    }
    return out;
  }

  size_t zcard(const std::string& key) {
    size_t n = 0;
    for (auto& sh : shards_) n += sh->zcard(key);
    return n;
  }
  // ZRANGE over the shards: merged by score (the wall-clock second of the last mutation).
  std::vector<std::string> zrange(const std::string& key, size_t limit) {
    std::vector<std::pair<double, std::string>> all;
    for (auto& sh : shards_) {
      auto v = sh->zrange_scored(key, limit);
      all.insert(all.end(), std::make_move_iterator(v.begin()), std::make_move_iterator(v.end()));
    }
    std::stable_sort(all.begin(), all.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    std::vector<std::string> out;
    for (auto& e : all) {
      if (out.size() >= limit) break;
      out.push_back(std::move(e.second));
    }
    return out;
  }
  std::vector<std::string> keys_with_suffix(const std::string& suffix) {
    std::vector<std::string> out;
    for (auto& sh : shards_) {
      auto v = sh->keys_with_suffix(suffix);
      out.insert(out.end(), v.begin(), v.end());
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
  }

  int64_t incrby(const std::string& key, int64_t delta) {
    std::lock_guard<std::mutex> g(cmu_);
    return counters_[key] += delta;
  }
  std::optional<int64_t> get_counter(const std::string& key) {
    std::lock_guard<std::mutex> g(cmu_);
    auto it = counters_.find(key);
    if (it == counters_.end()) return std::nullopt;
    return it->second;
  }
  std::map<std::string, int64_t> counters() {
    std::lock_guard<std::mutex> g(cmu_);
    return {counters_.begin(), counters_.end()};
  }

  size_t evict_finished(double max_age_s, size_t max_finished = SIZE_MAX) {
    size_t n = 0;
    const size_t per = max_finished == SIZE_MAX ? SIZE_MAX : (max_finished + nshards_ - 1) / nshards_;
    for (auto& sh : shards_) n += sh->evict_finished(max_age_s, per);
    return n;
  }
  size_t size() {
    size_t n = 0;
    for (auto& sh : shards_) n += sh->size();
    return n;
  }
  void flush() {
    std::lock_guard<std::mutex> g(journal_.mu);
    if (journal_.f) std::fflush(journal_.f);
  }
  bool journaled() const { return journal_.f != nullptr; }

  template <class Parse>
  size_t replay(const std::string& path, Parse parse) {
    std::ifstream in(path);
    if (!in) return 0;
    {
      std::lock_guard<std::mutex> g(journal_.mu);
      journal_.paused = true;  // do not re-journal while replaying
    }
    std::string line;
    size_t n = 0;
    const double mnow = mono_now();
    while (std::getline(in, line)) {
      if (line.empty()) continue;
      JournalLine jl;
      if (!parse(line, jl)) continue;  // torn tail line after a crash
      shard_for(jl.id).replay_line(jl, mnow);
      ++n;
    }
    std::lock_guard<std::mutex> g(journal_.mu);
    journal_.paused = false;
    return n;
  }

 private:
  StoreShard& next_shard() { return *shards_[rr_.fetch_add(1, std::memory_order_relaxed) % nshards_]; }

  // Calls fn(shard, ids of that shard, original positions or null) once per shard touched, in order.
  template <class Fn>
  void for_groups(const std::vector<std::string>& ids, Fn fn) {
    if (ids.empty()) return;
    const size_t s0 = shard_of(ids[0], nshards_);
    bool one = true;
    for (const auto& id : ids)
      if (shard_of(id, nshards_) != s0) {
        one = false;
        break;
      }
    if (one) {  // the common case: a batch minted by one create_many call
      fn(*shards_[s0], ids, nullptr);
      return;
    }
    std::vector<std::vector<std::string>> g(nshards_);
    std::vector<std::vector<uint32_t>> pos(nshards_);
    for (size_t i = 0; i < ids.size(); ++i) {
      const size_t s = shard_of(ids[i], nshards_);
      g[s].push_back(ids[i]);
      pos[s].push_back(static_cast<uint32_t>(i));
    }
    for (size_t s = 0; s < nshards_; ++s)
      if (!g[s].empty()) fn(*shards_[s], g[s], &pos[s]);
  }

  size_t nshards_;
  Journal journal_;
  std::vector<std::unique_ptr<StoreShard>> shards_;
  std::atomic<size_t> rr_{0};
  std::mutex cmu_;
  std::unordered_map<std::string, int64_t> counters_;
};

}  // namespace ai4e
