// ai4e_core — native control plane of the MI355X serving platform.
//
// Replaces the reference's Redis-backed task cache + Service Bus transport
// (ProcessManager/CacheManager/CacheConnectorUpsert.cs:40-213,
//  ProcessManager/CacheManager/CacheConnectorGet.cs:27-73,
//  ProcessManager/BackendQueueProcessor/BackendQueueProcessor.cs:27-81,
//  ProcessManager/RequestReporter/CurrentProcessingUpsert.cs:99-110,
//  ProcessManager/Libraries/QueueLogger.cs:21-47)
// with one in-process C++ object per concern:
//
//   TaskStore      task records + "{EndpointPath}_{BackendStatus}" ordered
//                  indexes + "{TaskId}_ORIG" bodies + INCRBY counters, all
//                  mutated atomically under one lock (the reference's Redis
//                  MULTI/EXEC), optional append-only journal for restart.
//   DispatchQueue  per-endpoint FIFO with Service-Bus semantics: receive
//                  (peek-lock), complete, abandon(+delay), lock expiry ->
//                  redelivery, max-delivery -> dead letter; plus a dynamic
//                  batching receive (max_n / linger) for the GPU workers.
//
// Every blocking call releases the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <ctime>
#include <deque>
#include <fstream>
#include <map>
#include <mutex>
#include <optional>
#include <queue>
#include <random>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace ai4e {

// ---------------------------------------------------------------- utilities
static double wall_now() {
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}
static double mono_now() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// .NET DateTime.UtcNow.ToString() under the en-US culture: "M/d/yyyy h:mm:ss tt".
static std::string dotnet_timestamp(double epoch_s) {
  std::time_t t = static_cast<std::time_t>(epoch_s);
  std::tm tm{};
  gmtime_r(&t, &tm);
  int h12 = tm.tm_hour % 12;
  if (h12 == 0) h12 = 12;
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%d/%d/%04d %d:%02d:%02d %s", tm.tm_mon + 1, tm.tm_mday,
                tm.tm_year + 1900, h12, tm.tm_min, tm.tm_sec, tm.tm_hour < 12 ? "AM" : "PM");
  return buf;
}

class Uuid4 {
 public:
  Uuid4() {
    std::random_device rd;
    s0_ = (static_cast<uint64_t>(rd()) << 32) ^ rd() ^ static_cast<uint64_t>(mono_now() * 1e9);
    s1_ = (static_cast<uint64_t>(rd()) << 32) ^ rd();
    if (!s0_ && !s1_) s1_ = 0x9E3779B97F4A7C15ull;
  }
  std::string next() {
    uint64_t a = step(), b = step();
    a = (a & 0xFFFFFFFFFFFF0FFFull) | 0x0000000000004000ull;  // version 4
    b = (b & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;  // variant 10
    char buf[37];
    std::snprintf(buf, sizeof(buf), "%08x-%04x-%04x-%04x-%012llx", static_cast<unsigned>(a >> 32),
                  static_cast<unsigned>((a >> 16) & 0xFFFF), static_cast<unsigned>(a & 0xFFFF),
                  static_cast<unsigned>(b >> 48),
                  static_cast<unsigned long long>(b & 0xFFFFFFFFFFFFull));
    return buf;
  }

 private:
  uint64_t step() {  // xorshift128+
    uint64_t x = s0_;
    const uint64_t y = s1_;
    s0_ = y;
    x ^= x << 23;
    s1_ = x ^ y ^ (x >> 17) ^ (y >> 26);
    return s1_ + y;
  }
  uint64_t s0_, s1_;
};

static void json_escape_into(std::string& out, const std::string& s) {
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
}

// System.Uri.AbsolutePath for "scheme://host[:port]/path?query" (path only, "/" if empty).
static std::string absolute_path(const std::string& endpoint) {
  auto p = endpoint.find("://");
  size_t start = 0;
  if (p != std::string::npos) {
    start = endpoint.find('/', p + 3);
    if (start == std::string::npos) return "/";
  } else if (endpoint.empty() || endpoint[0] != '/') {
    return endpoint.empty() ? "/" : "/" + endpoint;
  }
  auto q = endpoint.find_first_of("?#", start);
  return endpoint.substr(start, q == std::string::npos ? std::string::npos : q - start);
}

static const char* kStates[] = {"created", "running", "completed", "failed"};

// ---------------------------------------------------------------- TaskStore
struct TaskRecord {
  std::string task_id, timestamp, status, backend_status, endpoint, endpoint_path;
  bool publish_to_grid = false;
  double t_created = 0, t_running = 0, t_finished = 0;  // monotonic seconds (latency accounting)
};

struct SortedSet {  // Redis ZSET subset: ZADD / ZREM / ZCARD / ZRANGE
  std::unordered_map<std::string, double> score;
  std::set<std::pair<double, std::string>> order;
  void add(const std::string& id, double s) {
    auto it = score.find(id);
    if (it != score.end()) {
      order.erase({it->second, id});
      it->second = s;
    } else {
      score.emplace(id, s);
    }
    order.emplace(s, id);
  }
  bool rem(const std::string& id) {
    auto it = score.find(id);
    if (it == score.end()) return false;
    order.erase({it->second, id});
    score.erase(it);
    return true;
  }
  size_t size() const { return score.size(); }
};

class TaskStore {
 public:
  explicit TaskStore(std::string journal_path = "") : journal_path_(std::move(journal_path)) {
    if (!journal_path_.empty()) open_journal();
  }
  ~TaskStore() {
    if (journal_) std::fclose(journal_);
  }

  // CacheConnectorUpsert semantics (CacheConnectorUpsert.cs:92-176). Returns the serialized task
  // (Body nulled) and the body that must be published (original body for a pipeline re-publish).
  std::pair<std::string, std::optional<std::string>> upsert(
      std::string task_id, const std::string& status, const std::string& backend_status,
      const std::string& endpoint, const std::optional<std::string>& body, bool publish_to_grid) {
    std::lock_guard<std::mutex> g(mu_);
    if (task_id.find_first_not_of(" \t\r\n") == std::string::npos) task_id = uuid_.next();
    const double wnow = wall_now(), mnow = mono_now();
    TaskRecord& r = records_[task_id];
    if (r.task_id.empty()) {
      r.t_created = mnow;
    } else {
      // Pipeline hop to another endpoint: the task leaves the previous endpoint's state index
      // (the reference leaves it behind in "{old}_{state}", inflating that queue's depth metric).
      const std::string new_path = absolute_path(endpoint);
      if (new_path != r.endpoint_path) index_[r.endpoint_path + "_" + r.backend_status].rem(task_id);
    }
    r.task_id = task_id;
    r.timestamp = dotnet_timestamp(wnow);
    r.status = status;
    r.backend_status = backend_status;
    r.endpoint = endpoint;
    r.endpoint_path = absolute_path(endpoint);
    r.publish_to_grid = publish_to_grid;
    apply_index(r, wnow, mnow);
    std::optional<std::string> publish_body;
    if (publish_to_grid) {
      if (body && !body->empty()) {
        orig_[task_id] = *body;
        publish_body = *body;
      } else {  // subsequent pipeline call: reuse "{TaskId}_ORIG"
        auto it = orig_.find(task_id);
        publish_body = it == orig_.end() ? std::optional<std::string>(std::string())
                                         : std::optional<std::string>(it->second);
      }
    }
    journal_write(r, publish_to_grid && body && !body->empty() ? &*body : nullptr);
    return {serialize(r), publish_body};
  }

  // Hot path: create n tasks for one endpoint (status "created"), no per-task body.
  std::vector<std::string> create_many(const std::string& endpoint, size_t n, const std::string& status) {
    std::vector<std::string> ids;
    ids.reserve(n);
    std::lock_guard<std::mutex> g(mu_);
    const double wnow = wall_now(), mnow = mono_now();
    const std::string ts = dotnet_timestamp(wnow), path = absolute_path(endpoint);
    SortedSet& created = index_[path + "_created"];
    for (size_t i = 0; i < n; ++i) {
      std::string id = uuid_.next();
      TaskRecord& r = records_[id];
      r.task_id = id;
      r.timestamp = ts;
      r.status = status;
      r.backend_status = "created";
      r.endpoint = endpoint;
      r.endpoint_path = path;
      r.publish_to_grid = true;
      r.t_created = mnow;
      created.add(id, static_cast<double>(static_cast<int64_t>(wnow)));
      journal_write(r, nullptr);
      ids.push_back(std::move(id));
    }
    return ids;
  }

  // Hot path: move tasks to running / completed / failed with one lock acquisition.
  size_t transition_many(const std::vector<std::string>& ids, const std::string& backend_status,
                         const std::string& status) {
    std::lock_guard<std::mutex> g(mu_);
    const double wnow = wall_now(), mnow = mono_now();
    const std::string ts = dotnet_timestamp(wnow);
    size_t n = 0;
    for (const auto& id : ids) {
      auto it = records_.find(id);
      if (it == records_.end()) continue;
      TaskRecord& r = it->second;
      r.timestamp = ts;
      r.status = status;
      r.backend_status = backend_status;
      apply_index(r, wnow, mnow);
      journal_write(r, nullptr);
      ++n;
    }
    return n;
  }

  // BackendQueueProcessor.UpdateTaskStatus (BackendQueueProcessor.cs:83-133): set Status text only.
  bool set_status_text(const std::string& id, const std::string& status) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = records_.find(id);
    if (it == records_.end()) return false;
    it->second.status = status;
    it->second.timestamp = dotnet_timestamp(wall_now());
    journal_write(it->second, nullptr);
    return true;
  }

  std::optional<std::string> get(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = records_.find(id);
    if (it == records_.end()) return std::nullopt;
    return serialize(it->second);
  }

  std::optional<py::dict> get_record(const std::string& id) {
    TaskRecord r;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = records_.find(id);
      if (it == records_.end()) return std::nullopt;
      r = it->second;
    }
    py::dict d;
    d["TaskId"] = r.task_id;
    d["Timestamp"] = r.timestamp;
    d["Status"] = r.status;
    d["BackendStatus"] = r.backend_status;
    d["Endpoint"] = r.endpoint;
    d["Body"] = py::none();
    d["PublishToGrid"] = r.publish_to_grid;
    d["EndpointPath"] = r.endpoint_path;
    return d;
  }

  std::optional<std::string> get_orig_body(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = orig_.find(id);
    if (it == orig_.end()) return std::nullopt;
    return it->second;
  }

  // Seconds from create to finish (or to running if finished==false) for each finished id.
  std::vector<double> latencies(const std::vector<std::string>& ids, bool to_running) {
    std::vector<double> out;
    out.reserve(ids.size());
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& id : ids) {
      auto it = records_.find(id);
      if (it == records_.end()) continue;
      const TaskRecord& r = it->second;
      const double end = to_running ? r.t_running : r.t_finished;
      if (end > 0) out.push_back(end - r.t_created);
    }
    return out;
  }

  size_t zcard(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(key);
    return it == index_.end() ? 0 : it->second.size();
  }

  std::vector<std::string> zrange(const std::string& key, size_t limit) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> out;
    auto it = index_.find(key);
    if (it == index_.end()) return out;
    for (const auto& e : it->second.order) {
      if (out.size() >= limit) break;
      out.push_back(e.second);
    }
    return out;
  }

  // Redis "KEYS *{suffix}" over the index namespace (QueueLogger.cs:21-47).
  std::vector<std::string> keys_with_suffix(const std::string& suffix) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> out;
    for (const auto& kv : index_) {
      const std::string& k = kv.first;
      if (k.size() >= suffix.size() && k.compare(k.size() - suffix.size(), suffix.size(), suffix) == 0)
        out.push_back(k);
    }
    std::sort(out.begin(), out.end());
    return out;
  }

  int64_t incrby(const std::string& key, int64_t delta) {
    std::lock_guard<std::mutex> g(mu_);
    return counters_[key] += delta;
  }
  std::optional<int64_t> get_counter(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = counters_.find(key);
    if (it == counters_.end()) return std::nullopt;
    return it->second;
  }
  std::map<std::string, int64_t> counters() {
    std::lock_guard<std::mutex> g(mu_);
    return {counters_.begin(), counters_.end()};
  }

  // Drop completed/failed records finished more than max_age_s ago (bounded memory for serving).
  size_t evict_finished(double max_age_s) {
    std::lock_guard<std::mutex> g(mu_);
    const double cutoff = mono_now() - max_age_s;
    size_t n = 0;
    for (auto it = records_.begin(); it != records_.end();) {
      const TaskRecord& r = it->second;
      if (r.t_finished > 0 && r.t_finished <= cutoff) {
        index_[r.endpoint_path + "_" + r.backend_status].rem(r.task_id);
        orig_.erase(r.task_id);
        it = records_.erase(it);
        ++n;
      } else {
        ++it;
      }
    }
    return n;
  }

  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return records_.size();
  }

  void flush() {
    std::lock_guard<std::mutex> g(mu_);
    if (journal_) std::fflush(journal_);
  }

  // Rebuild state from a journal (each line = full record image + optional ORIG body).
  size_t replay(const std::string& path) {
    std::ifstream in(path);
    if (!in) return 0;
    py::gil_scoped_acquire acq;
    py::module_ json = py::module_::import("json");
    std::string line;
    size_t n = 0;
    std::lock_guard<std::mutex> g(mu_);
    FILE* saved = journal_;
    journal_ = nullptr;  // do not re-journal while replaying
    while (std::getline(in, line)) {
      if (line.empty()) continue;
      py::dict d;
      try {
        d = json.attr("loads")(line);
      } catch (...) {
        continue;  // torn tail line after a crash
      }
      TaskRecord& r = records_[d["TaskId"].cast<std::string>()];
      const std::string old_state = r.backend_status, old_path = r.endpoint_path;
      r.task_id = d["TaskId"].cast<std::string>();
      r.timestamp = d["Timestamp"].cast<std::string>();
      r.status = d["Status"].cast<std::string>();
      r.backend_status = d["BackendStatus"].cast<std::string>();
      r.endpoint = d["Endpoint"].cast<std::string>();
      r.endpoint_path = absolute_path(r.endpoint);
      r.publish_to_grid = d["PublishToGrid"].cast<bool>();
      if (!old_state.empty()) index_[old_path + "_" + old_state].rem(r.task_id);
      index_[r.endpoint_path + "_" + r.backend_status].add(r.task_id, d["_score"].cast<double>());
      if (d.contains("_orig") && !d["_orig"].is_none()) orig_[r.task_id] = d["_orig"].cast<std::string>();
      ++n;
    }
    journal_ = saved;
    return n;
  }

 private:
  void apply_index(TaskRecord& r, double wnow, double mnow) {
    const double score = static_cast<double>(static_cast<int64_t>(wnow));
    const std::string& p = r.endpoint_path;
    index_[p + "_" + r.backend_status].add(r.task_id, score);
    if (r.backend_status == "running") {
      index_[p + "_created"].rem(r.task_id);
      r.t_running = mnow;
    } else if (r.backend_status == "completed" || r.backend_status == "failed") {
      index_[p + "_running"].rem(r.task_id);
      // Intended behaviour (reference only clears _running): a task failed before it ever ran
      // must not linger in _created either, or queue-depth metrics over-count forever.
      index_[p + "_created"].rem(r.task_id);
      r.t_finished = mnow;
    } else if (r.backend_status == "created") {
      // Re-publish (pipeline hop / 429 requeue) to a possibly new endpoint.
      for (const char* s : {"running", "completed", "failed"}) index_[p + "_" + s].rem(r.task_id);
      r.t_finished = 0;
    }
  }

  static std::string serialize(const TaskRecord& r) {
    std::string out;
    out.reserve(256);
    out += "{\"TaskId\":";
    json_escape_into(out, r.task_id);
    out += ",\"Timestamp\":";
    json_escape_into(out, r.timestamp);
    out += ",\"Status\":";
    json_escape_into(out, r.status);
    out += ",\"BackendStatus\":";
    json_escape_into(out, r.backend_status);
    out += ",\"Endpoint\":";
    json_escape_into(out, r.endpoint);
    out += ",\"Body\":null,\"PublishToGrid\":";
    out += r.publish_to_grid ? "true" : "false";
    out += ",\"EndpointPath\":";
    json_escape_into(out, r.endpoint_path);
    out += "}";
    return out;
  }

  void open_journal() {
    journal_ = std::fopen(journal_path_.c_str(), "a");
    if (!journal_) throw std::runtime_error("cannot open journal " + journal_path_);
  }

  void journal_write(const TaskRecord& r, const std::string* orig) {
    if (!journal_) return;
    std::string line = serialize(r);
    line.pop_back();
    line += ",\"_score\":" + std::to_string(static_cast<int64_t>(wall_now()));
    if (orig) {
      line += ",\"_orig\":";
      json_escape_into(line, *orig);
    }
    line += "}\n";
    std::fwrite(line.data(), 1, line.size(), journal_);
  }

  std::mutex mu_;
  Uuid4 uuid_;
  std::unordered_map<std::string, TaskRecord> records_;
  std::unordered_map<std::string, SortedSet> index_;
  std::unordered_map<std::string, std::string> orig_;
  std::unordered_map<std::string, int64_t> counters_;
  std::string journal_path_;
  FILE* journal_ = nullptr;
};

// ------------------------------------------------------------- DispatchQueue
struct Message {
  uint64_t seq = 0;
  std::string task_id;
  int64_t ref = -1;          // payload slot (pinned ring index) or -1
  std::string body;          // request body (used when no slot)
  int delivery_count = 0;
  double enqueued_at = 0;    // monotonic
  double visible_at = 0;     // monotonic (scheduled redelivery)
  double lock_until = 0;
};

class DispatchQueue {
 public:
  DispatchQueue(std::string name, int max_delivery_count, double lock_duration_s, size_t max_size)
      : name_(std::move(name)),
        max_delivery_(max_delivery_count),
        lock_s_(lock_duration_s),
        max_size_(max_size) {}

  const std::string& name() const { return name_; }

  // Returns false (backpressure) when the queue is at max_size.
  bool send(const std::string& task_id, int64_t ref, const std::string& body) {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_ || (max_size_ && ready_.size() + scheduled_.size() >= max_size_)) return false;
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
      if (closed_ || (max_size_ && ready_.size() + scheduled_.size() >= max_size_)) break;
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
    const double t0 = mono_now();
    auto deadline = t0 + timeout_s;
    for (;;) {
      promote_locked(mono_now());
      if (!ready_.empty() || closed_) break;
      double now = mono_now();
      if (now >= deadline) return out;
      double wake = deadline;
      if (!scheduled_.empty()) wake = std::min(wake, scheduled_.top().visible_at);
      if (!inflight_.empty()) wake = std::min(wake, now + 0.05);
      wait_s(lk, wake - now);
    }
    if (linger_s > 0 && ready_.size() < max_n && !closed_) {
      const double ldl = mono_now() + linger_s;
      while (ready_.size() < max_n && !closed_) {
        double now = mono_now();
        if (now >= ldl) break;
        wait_s(lk, ldl - now);
        promote_locked(mono_now());
      }
    }
    const double now = mono_now();
    while (!ready_.empty() && out.size() < max_n) {
      Message m = std::move(ready_.front());
      ready_.pop_front();
      m.delivery_count += 1;
      m.lock_until = now + lock_s_;
      inflight_.emplace(m.seq, m);
      out.push_back(std::move(m));
    }
    return out;
  }

  size_t complete(const std::vector<uint64_t>& seqs) {
    std::lock_guard<std::mutex> g(mu_);
    size_t n = 0;
    for (auto s : seqs) n += inflight_.erase(s);
    return n;
  }

  // Abandon (BackendQueueProcessor.cs:54-64): redeliver after delay, or dead-letter when the
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

  py::dict stats() {
    std::lock_guard<std::mutex> g(mu_);
    py::dict d;
    d["name"] = name_;
    d["ready"] = ready_.size();
    d["scheduled"] = scheduled_.size();
    d["inflight"] = inflight_.size();
    d["deadlettered"] = dead_total_;
    d["sent"] = seq_;
    return d;
  }
  size_t depth() {
    std::lock_guard<std::mutex> g(mu_);
    return ready_.size() + scheduled_.size();
  }

 private:
  struct Later {
    bool operator()(const Message& a, const Message& b) const { return a.visible_at > b.visible_at; }
  };

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
    if (!inflight_.empty() && lock_s_ > 0) {
      std::vector<uint64_t> expired;
      for (auto& kv : inflight_)
        if (kv.second.lock_until <= now) expired.push_back(kv.first);
      for (auto s : expired) {
        Message m = std::move(inflight_[s]);
        inflight_.erase(s);
        requeue_locked(std::move(m), 0);
      }
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
  std::vector<Message> dead_;
  uint64_t seq_ = 0, dead_total_ = 0;
  bool closed_ = false;
};

}  // namespace ai4e

PYBIND11_MODULE(_ai4e_core, m) {
  using namespace ai4e;
  m.doc() = "Native task store + dispatch queue for the MI355X AI4E serving platform";
  m.def("dotnet_timestamp", &dotnet_timestamp);
  m.def("absolute_path", &absolute_path);
  m.def("uuid4", []() {
    static Uuid4 u;
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    return u.next();
  });

  py::class_<TaskStore>(m, "TaskStore")
      .def(py::init<std::string>(), py::arg("journal_path") = "")
      .def("upsert", &TaskStore::upsert, py::arg("task_id"), py::arg("status"), py::arg("backend_status"),
           py::arg("endpoint"), py::arg("body") = std::nullopt, py::arg("publish_to_grid") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("create_many", &TaskStore::create_many, py::arg("endpoint"), py::arg("n"),
           py::arg("status") = "created", py::call_guard<py::gil_scoped_release>())
      .def("transition_many", &TaskStore::transition_many, py::arg("ids"), py::arg("backend_status"),
           py::arg("status"), py::call_guard<py::gil_scoped_release>())
      .def("set_status_text", &TaskStore::set_status_text, py::call_guard<py::gil_scoped_release>())
      .def("get", &TaskStore::get, py::call_guard<py::gil_scoped_release>())
      .def("get_record", &TaskStore::get_record)
      .def("get_orig_body", &TaskStore::get_orig_body)
      .def("latencies", &TaskStore::latencies, py::arg("ids"), py::arg("to_running") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("zcard", &TaskStore::zcard)
      .def("zrange", &TaskStore::zrange, py::arg("key"), py::arg("limit") = static_cast<size_t>(-1))
      .def("keys_with_suffix", &TaskStore::keys_with_suffix)
      .def("incrby", &TaskStore::incrby)
      .def("get_counter", &TaskStore::get_counter)
      .def("counters", &TaskStore::counters)
      .def("evict_finished", &TaskStore::evict_finished, py::call_guard<py::gil_scoped_release>())
      .def("size", &TaskStore::size)
      .def("flush", &TaskStore::flush)
      .def("replay", &TaskStore::replay, py::call_guard<py::gil_scoped_release>());

  py::class_<Message>(m, "Message")
      .def_readonly("seq", &Message::seq)
      .def_readonly("task_id", &Message::task_id)
      .def_readonly("ref", &Message::ref)
      .def_property_readonly("body", [](const Message& msg) { return py::bytes(msg.body); })
      .def_readonly("delivery_count", &Message::delivery_count)
      .def_readonly("enqueued_at", &Message::enqueued_at);

  py::class_<DispatchQueue>(m, "DispatchQueue")
      .def(py::init<std::string, int, double, size_t>(), py::arg("name"), py::arg("max_delivery_count") = 1440,
           py::arg("lock_duration_s") = 300.0, py::arg("max_size") = 0)
      .def_property_readonly("name", &DispatchQueue::name)
      .def("send", &DispatchQueue::send, py::arg("task_id"), py::arg("ref") = -1, py::arg("body") = "",
           py::call_guard<py::gil_scoped_release>())
      .def("send_many", &DispatchQueue::send_many, py::arg("ids"), py::arg("refs") = std::vector<int64_t>{},
           py::call_guard<py::gil_scoped_release>())
      .def("receive", &DispatchQueue::receive, py::arg("max_n") = 1, py::arg("timeout_s") = 0.0,
           py::arg("linger_s") = 0.0, py::call_guard<py::gil_scoped_release>())
      .def("complete", &DispatchQueue::complete, py::call_guard<py::gil_scoped_release>())
      .def("abandon", &DispatchQueue::abandon, py::arg("seq"), py::arg("delay_s") = 0.0,
           py::call_guard<py::gil_scoped_release>())
      .def("take_deadletters", &DispatchQueue::take_deadletters)
      .def("close", &DispatchQueue::close)
      .def("stats", &DispatchQueue::stats)
      .def("depth", &DispatchQueue::depth);
}
