// ai4e_ingestd — native ingest front-end of the gateway (the C++ form of runtime/frontend.py).
//
// One process listens on the public port beside the serving process (SO_REUSEPORT: the kernel spreads
// connections over every listener) and takes the async POSTs of the GPU endpoints itself:
//
//   * binary batches (application/x-ai4e-batch, n x item bytes) and raw single payloads
//     (application/octet-stream of exactly one item) are recv()'d STRAIGHT into slots of this process's
//     partition of the endpoint's shared payload ring — one kernel->ring copy, no parse, no decode;
//   * task ids are minted here (uuid4, last hex digit = store shard, as ingest.IngestShard.mint_ids) and handed
//     to the node scheduler with the slots (SUBMIT_IDS over the ingest connection, acknowledged with
//     SUBMITTED once the tasks exist); slots come back with FREE when the tasks finish;
//   * everything else (task status / result / trace, sync routes, encoded images, requests carrying an
//     upstream taskId, chunked bodies) is proxied to the serving process's internal listener.
//
// Admission matches the gateway (gateway/server.py, gateway/security.py): subscription keys (401), the
// route's max_concurrent (429), draining after SIGTERM (503), content type (401), length (413; proxied bodies too,
// with a global 1 GiB cap as aiohttp's client_max_size, chunked bodies counted as they arrive).
//
// TLS (the reference's Istio gateway on :443 with a mounted certificate, Cluster/networking/secure_routing_base.yml):
// with "tls CERT KEY" in the config every client connection is a TLS 1.2+ session (OpenSSL; kernel TLS offload
// where the kernel has it), and the ingest path SSL_read()s the request body straight into the ring slots — the
// decryption is the one copy. The connection to the serving process's internal listener stays plain TCP on
// loopback.
//
// Threads: one acceptor, one thread per client connection (blocking I/O, keep-alive), one reader per
// scheduler connection. The process exits when a scheduler connection closes (the serving process is gone)
// or 5 s after SIGTERM.
//
// Config: a line-oriented file written by runtime/native_frontend.py (see parse_config).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <openssl/err.h>
#include <openssl/ssl.h>

#include "../core/common.h"
#include "../core/jpeg_coef.h"
#include "../core/slot_ring.h"

namespace {

constexpr uint32_t F_STOP = 5, F_FREE = 7, F_SUBMIT_IDS = 9, F_SUBMITTED = 10, F_SUBMIT_MULTI = 11,
                   F_SUBMITTED_MULTI = 12;
const char* kBatchType = "application/x-ai4e-batch";
const char* kRawType = "application/octet-stream";
const char* kKeyHeader = "ocp-apim-subscription-key";
const char* kMissingKey =
    "Access denied due to missing subscription key. Make sure to include subscription key when making requests "
    "to an API.";
const char* kInvalidKey =
    "Access denied due to invalid subscription key. Make sure to provide a valid key for an active subscription.";

std::atomic<bool> g_draining{false};
SSL_CTX* g_tls = nullptr;                     // non-null: client connections are TLS sessions
constexpr int64_t kMaxBody = int64_t{1} << 30;  // global request-body cap (aiohttp client_max_size of the gateway)
constexpr int64_t kMaxUpstreamBody = int64_t{1} << 34;  // responses of the (trusted) serving process

// ------------------------------------------------------------------ socket helpers
bool write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

bool read_exact(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k == 0) return false;
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

std::string lower(std::string s) {
  for (auto& ch : s) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  return s;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t"), b = s.find_last_not_of(" \t\r");
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char ch : s) {
    if (ch == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(ch);
    }
  }
  out.push_back(cur);
  return out;
}

std::string hexid(std::mt19937_64& rng, int bits) {
  static const char* hx = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < bits / 64; ++i) {
    uint64_t v = rng();
    for (int k = 15; k >= 0; --k) s.push_back(hx[(v >> (4 * k)) & 0xF]);
  }
  return s;
}

// ------------------------------------------------------------------ scheduler connection (one per endpoint)
// multiprocessing.Connection framing on a socketpair: 4-byte big-endian length, then the frame.
struct Ack {
  bool done = false;
  uint32_t n = 0;
  std::vector<uint32_t> per;  // SUBMITTED_MULTI: tasks created per request of the frame
};

// One request's ingest waiting to be submitted (group commit: the connection threads of a shard queue their
// requests and one of them — whoever finds no frame in flight — sends every queued request in ONE SUBMIT_MULTI frame
// and hands each its own created count from the one SUBMITTED_MULTI answer)
struct PendingSubmit {
  const std::vector<int64_t>* sl;
  const std::vector<std::string>* ids;
  std::string trace;
  int64_t created = -2;  // -2 pending, -1 ack timed out, else tasks created
  bool leader = false;   // this request's thread sends the next group
  std::condition_variable cv;  // its own wake-up (no herd: one notify per waiter)
};

struct Shard {
  int idx = 0, fd = -1;
  std::string endpoint, endpoint_path, shape_str;
  int64_t nslots = 0, item = 0, base = 0, len = 0;
  int out_h = 0, out_w = 0, out_c = 0;  // the model input (shape_str)
  int64_t max_batch = 0;                // the workers' batch size (0: unknown)
  uint8_t* ring = nullptr;
  // the ring's key for slots holding prepared JPEG frames (its tail, csrc/core/jpeg_layout.h RingTail; 0: the ring's
  // workers do not decode them, JPEG bodies go to the serving process)
  uint64_t jpeg_key = 0;
  std::unique_ptr<ai4e::SlotRing> slots;
  std::mutex send_mu, ack_mu;
  std::condition_variable ack_cv;
  std::unordered_map<uint64_t, Ack> acks;
  std::atomic<uint64_t> token{1}, shard_ctr{0};
  std::mutex id_mu;
  ai4e::Uuid4 uuid;
  // last hex digits the ids of this scheduler shard may end in (= the task-store lock domains it owns;
  // default 0-7: any domain of the 8-way store)
  std::string digits = "01234567";
  // service rate of this partition (slots coming back FREE per second, EWMA over ~50 ms samples): the
  // latency-budget admission projects a new request's queue wait as (slots in use + n) / rate
  std::atomic<int64_t> freed{0};
  std::mutex rate_mu;
  double rate = 0.0, rate_t = 0.0;
  int64_t rate_n = 0;
  bool rate_sat = false;

  // the scheduler shard's load counters (NodeScheduler::ShardStat, "stat NAME" on the shard line), 64 words:
  // [0] queued, [1] finished (terminal), [2] bodies uploading (front-ends without a word of their own), [3] live
  // dispatch workers, [4] items out at the GPU workers, [8 + i] bodies uploading at front-end i; null = estimate
  // from this partition alone
  std::atomic<uint64_t>* st = nullptr;
  static constexpr int kStatWords = 64, kStatFe0 = 8, kStatFrontends = 56;

  bool live() const { return !st || st[3].load(std::memory_order_relaxed) > 0; }
  // tasks of the shard not yet finished, plus every front-end's admitted bodies still uploading
  double backlog() const {
    const uint64_t e = st[0].load(std::memory_order_relaxed), d = st[1].load(std::memory_order_relaxed);
    uint64_t up = st[2].load(std::memory_order_relaxed);
    for (int i = 0; i < kStatFrontends; ++i) up += st[kStatFe0 + i].load(std::memory_order_relaxed);
    return (e > d ? static_cast<double>(e - d) : 0.0) + static_cast<double>(up);
  }
  // items queued behind the GPU workers' pipelines (not yet handed to a worker)
  bool queued() const {
    const uint64_t e = st[0].load(std::memory_order_relaxed), d = st[1].load(std::memory_order_relaxed),
                   f = st[4].load(std::memory_order_relaxed);
    return e > d + f;
  }
  // ... or admitted bodies still uploading: work that will have to wait for the pipelines too
  bool waiting() const {
    if (queued()) return true;
    uint64_t up = st[2].load(std::memory_order_relaxed);
    for (int i = 0; i < kStatFrontends; ++i) up += st[kStatFe0 + i].load(std::memory_order_relaxed);
    return up > 0;
  }

  // The shard's capacity in items per second at the batches it actually forms. A completion-rate sample taken while
  // tasks waited in the queue at both ends (the workers never starved) measures that capacity and is averaged in;
  // a sample from a shard that ran out of work only measures the demand, a lower bound: it can raise the estimate,
  // never lower it. (Round 5 held the smoothed rate's peak and let it decay 10 %/s, so a route whose clients were
  // slower than the GPU — single images — read as a slow GPU and throttled itself to 0.59x.)
  // Busy time published by the scheduler (words 5-6: microseconds with items in flight at the workers): finished items
  // per busy second is the capacity at the batches the shard forms, at any load. Used once the workers have been
  // busy for 20 ms of a sample; the completion-rate rules below are the fallback.
  double busy_s() const {
    const uint64_t b = st[5].load(std::memory_order_relaxed), t0 = st[6].load(std::memory_order_relaxed);
    const uint64_t now = static_cast<uint64_t>(ai4e::mono_now() * 1e6);
    return static_cast<double>(b + (t0 && now > t0 ? now - t0 : 0)) * 1e-6;
  }
  double rate_busy0 = 0.0;
  int64_t rate_bn = 0, rate_bb = 0;
  double service_rate() {
    std::unique_lock<std::mutex> g(rate_mu, std::try_to_lock);
    if (!g.owns_lock()) return rate_seen.load(std::memory_order_relaxed);  // (another thread is sampling)
    if (st) {
      // a backlog drains in full batches: with the workers' batch size known, the capacity is max_batch batches per
      // busy second of a batch (a light load forms small batches that each cost about a full one: their items per
      // busy second understate what a backlog would get); else finished items per busy second
      const double b = busy_s();
      const int64_t n = static_cast<int64_t>(st[1].load(std::memory_order_relaxed));
      const int64_t nb = static_cast<int64_t>(st[7].load(std::memory_order_relaxed));
      if (rate_busy0 == 0.0 && rate_bn == 0) {
        rate_busy0 = b;
        rate_bn = n;
        rate_bb = nb;
      } else if (b - rate_busy0 >= 0.02 && n > rate_bn) {
        const double r = max_batch > 0 && nb > rate_bb
                             ? std::max(static_cast<double>(n - rate_bn),
                                        static_cast<double>(max_batch) * static_cast<double>(nb - rate_bb)) /
                                   (b - rate_busy0)
                             : static_cast<double>(n - rate_bn) / (b - rate_busy0);
        busy_rate = busy_rate == 0.0 ? r : 0.7 * busy_rate + 0.3 * r;
        rate_busy0 = b;
        rate_bn = n;
        rate_bb = nb;
      }
      if (busy_rate > 0.0) {
        rate_seen.store(busy_rate, std::memory_order_relaxed);
        return busy_rate;
      }
    }
    const double t = ai4e::mono_now();
    const int64_t n = st ? static_cast<int64_t>(st[1].load(std::memory_order_relaxed)) : freed.load();
    const bool sat = st ? queued() : false;
    if (rate_t == 0.0) {
      rate_t = t;
      rate_n = n;
      rate_sat = sat;
    } else if (t - rate_t >= 0.05) {
      const double r = static_cast<double>(n - rate_n) / (t - rate_t);
      const uint64_t nref = refused.exchange(0, std::memory_order_relaxed);
      if (n > rate_n) {
        if (!st) {
          rate = rate == 0.0 ? r : 0.7 * rate + 0.3 * r;
        } else if (rate_sat && sat) {
          rate = rate == 0.0 ? r : 0.7 * rate + 0.3 * r;
        } else if (r > rate) {
          rate = r;
        } else if (nref > 0) {
          rate *= 1.5;  // (below)
        }
      } else if (nref > 0 && !sat) {
        // refusing while the workers ran out of queued work: the estimate is below the capacity (e.g. one learned
        // from the first batches after a start, when the demand set the completion rate) and the refusals keep the
        // samples unsaturated, so it could never rise; probe upward until samples saturate again
        rate *= 1.5;
      }
      rate_t = t;
      rate_n = n;
      rate_sat = sat;
    }
    rate_seen.store(rate, std::memory_order_relaxed);
    return rate;
  }
  std::atomic<double> rate_seen{0.0};
  std::atomic<uint64_t> refused{0};  // 429s answered since the last rate sample
  double busy_rate = 0.0;            // items per busy second (0: no busy-time sample yet)

  // request-body upload rate of this front-end (bytes/s, EWMA over completed bodies): a request's tasks only join
  // the queue once its body has arrived, by when the shard has worked off nbytes / upload_bw of its backlog
  std::mutex up_mu;
  double upload_bw = 0.0;
  void note_upload(double bytes, double secs) {
    if (secs <= 0.0 || bytes < 65536.0) return;
    std::lock_guard<std::mutex> g(up_mu);
    const double bw = bytes / secs;
    upload_bw = upload_bw == 0.0 ? bw : 0.8 * upload_bw + 0.2 * bw;
  }

  // projected queue wait of n more items (nbytes of body) once they are queued: the shard's backlog over its
  // capacity, minus what drains while this body uploads; or this partition's slots in use over its FREE rate when
  // the shard publishes no counters. Nothing waiting behind the GPU workers' pipelines means no queue wait at all,
  // whatever the estimate (a shard whose demand never reached its capacity has only a lower bound of it).
  double projected_wait(int64_t n, double nbytes) {
    const double rate = service_rate();
    if (rate <= 0.0) return 0.0;
    if (st) {
      if (!waiting()) return 0.0;
      double up = 0.0;
      {
        std::lock_guard<std::mutex> g(up_mu);
        if (upload_bw > 0.0) up = nbytes / upload_bw;
      }
      return std::max(0.0, (backlog() + static_cast<double>(n)) / rate - up);
    }
    return static_cast<double>(slots->used() + n) / rate;
  }
  // this front-end's admitted-bodies word in the shard's counters
  std::atomic<uint64_t>* pending_word(int fe) {
    if (!st) return nullptr;
    return fe >= 0 && fe < kStatFrontends ? &st[kStatFe0 + fe] : &st[2];
  }

  bool send_frame(std::string& f) {  // (f: 4 bytes reserved up front for the length prefix)
    const uint32_t be = htonl(static_cast<uint32_t>(f.size() - 4));
    std::memcpy(&f[0], &be, 4);
    std::lock_guard<std::mutex> g(send_mu);
    return write_all(fd, f.data(), f.size());  // one write per frame
  }

  std::vector<std::string> mint(size_t n) {
    static const char* hx = "0123456789abcdef";
    (void)hx;
    const char d = digits[shard_ctr.fetch_add(1) % digits.size()];
    std::vector<std::string> ids(n);
    std::lock_guard<std::mutex> g(id_mu);
    for (auto& s : ids) {
      s = uuid.next();
      s.back() = d;
    }
    return ids;
  }

  // SUBMIT_IDS: u32 type, u32 n, u32 trace_len, u32 id_len, u32 ack, u64 token | i64 slots[n] | ids | trace
  uint64_t submit(const std::vector<int64_t>& sl, const std::vector<std::string>& ids, const std::string& trace) {
    const uint64_t tok = token.fetch_add(1);
    {
      std::lock_guard<std::mutex> g(ack_mu);
      acks[tok] = Ack{};
    }
    const uint32_t n = static_cast<uint32_t>(sl.size()), tl = static_cast<uint32_t>(trace.size()),
                   il = ids.empty() ? 0 : static_cast<uint32_t>(ids[0].size()), ack = 1;
    std::string f(4, '\0');  // (length prefix, filled by send_frame)
    f.reserve(32 + 8 * n + il * n + tl);
    auto put32 = [&](uint32_t v) { f.append(reinterpret_cast<const char*>(&v), 4); };
    put32(F_SUBMIT_IDS);
    put32(n);
    put32(tl);
    put32(il);
    put32(ack);
    f.append(reinterpret_cast<const char*>(&tok), 8);
    f.append(reinterpret_cast<const char*>(sl.data()), 8 * sl.size());
    for (auto& s : ids) f += s;
    f += trace;
    if (!send_frame(f)) std::_Exit(0);  // the serving process is gone
    return tok;
  }

  // Group commit (see PendingSubmit): queue this request; the first thread to find no frame in flight sends every
  // queued request in one frame and waits for its answer, then the next group goes. Under load one scheduler frame and
  // one answer carry many requests (one scheduler wake-up, one journal flush, one queue notify for all of them)
  // instead of one frame and one answer each; alone, a request goes out at once as before.
  std::mutex gc_mu;
  std::vector<PendingSubmit*> gc_q;
  bool gc_busy = false;
  int64_t submit_wait(const std::vector<int64_t>& sl, const std::vector<std::string>& ids, std::string trace,
                      double timeout_s) {
    PendingSubmit me;
    me.sl = &sl;
    me.ids = &ids;
    me.trace = std::move(trace);
    std::unique_lock<std::mutex> lk(gc_mu);
    gc_q.push_back(&me);
    if (!gc_busy) {
      gc_busy = true;
      me.leader = true;
    }
    while (!me.leader && me.created == -2) me.cv.wait(lk);
    if (me.created != -2) return me.created;  // a leader sent it
    std::vector<PendingSubmit*> group;  // leader: everything queued so far (this request included)
    group.swap(gc_q);
    lk.unlock();
    std::vector<int64_t> got;
    if (group.size() == 1) {
      got.push_back(wait_ack(submit(*me.sl, *me.ids, me.trace), timeout_s));
    } else {
      got = wait_ack_multi(submit_multi(group), group.size(), timeout_s);
    }
    lk.lock();
    for (size_t i = 0; i < group.size(); ++i) {
      group[i]->created = got[i];
      if (group[i] != &me) group[i]->cv.notify_one();
    }
    if (!gc_q.empty()) {  // hand the lead to the oldest request that queued meanwhile
      gc_q.front()->leader = true;
      gc_q.front()->cv.notify_one();
    } else {
      gc_busy = false;
    }
    return me.created;
  }

  // SUBMIT_MULTI: u32 type, u32 nreq, u64 token | per request: u32 n, u32 trace_len, u32 id_len, u32 0,
  // i64 slots[n], ids, trace
  uint64_t submit_multi(const std::vector<PendingSubmit*>& group) {
    const uint64_t tok = token.fetch_add(1);
    {
      std::lock_guard<std::mutex> g(ack_mu);
      acks[tok] = Ack{};
    }
    size_t bytes = 20;
    for (auto* p : group)
      bytes += 16 + 8 * p->sl->size() + (p->ids->empty() ? 0 : p->ids->size() * (*p->ids)[0].size()) + p->trace.size();
    std::string f(4, '\0');  // (length prefix, filled by send_frame)
    f.reserve(bytes);
    auto put32 = [&](uint32_t v) { f.append(reinterpret_cast<const char*>(&v), 4); };
    put32(F_SUBMIT_MULTI);
    put32(static_cast<uint32_t>(group.size()));
    f.append(reinterpret_cast<const char*>(&tok), 8);
    for (auto* p : group) {
      const uint32_t n = static_cast<uint32_t>(p->sl->size());
      put32(n);
      put32(static_cast<uint32_t>(p->trace.size()));
      put32(p->ids->empty() ? 0 : static_cast<uint32_t>((*p->ids)[0].size()));
      put32(0);
      f.append(reinterpret_cast<const char*>(p->sl->data()), 8 * p->sl->size());
      for (auto& id : *p->ids) f += id;
      f += p->trace;
    }
    if (!send_frame(f)) std::_Exit(0);  // the serving process is gone
    return tok;
  }

  std::vector<int64_t> wait_ack_multi(uint64_t tok, size_t nreq, double timeout_s) {
    std::unique_lock<std::mutex> lk(ack_mu);
    const auto deadline = std::chrono::system_clock::now() + std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                                                  std::chrono::duration<double>(timeout_s));
    const bool ok = ack_cv.wait_until(lk, deadline, [&] { return acks[tok].done; });
    std::vector<int64_t> out(nreq, -1);
    if (ok)
      for (size_t i = 0; i < nreq && i < acks[tok].per.size(); ++i) out[i] = acks[tok].per[i];
    acks.erase(tok);
    return out;
  }

  // -1: timed out (the tasks may still be created), else tasks created
  int64_t wait_ack(uint64_t tok, double timeout_s) {
    std::unique_lock<std::mutex> lk(ack_mu);
    // system_clock deadline (pthread_cond_timedwait), as SlotRing: libtsan does not intercept the steady-clock
    // pthread_cond_clockwait that wait_for compiles to, and would report the waiter's re-lock as a double lock
    const auto deadline = std::chrono::system_clock::now() + std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                                                  std::chrono::duration<double>(timeout_s));
    bool ok = ack_cv.wait_until(lk, deadline, [&] { return acks[tok].done; });
    int64_t n = ok ? acks[tok].n : -1;
    acks.erase(tok);
    return n;
  }

  void reader() {
    std::vector<char> in(1 << 16);  // frames from the scheduler, several per recv()
    size_t pos = 0, end = 0;
    auto fill = [&](size_t need) {
      if (end - pos >= need) return true;
      if (pos) {
        std::memmove(in.data(), in.data() + pos, end - pos);
        end -= pos;
        pos = 0;
      }
      if (need > in.size()) in.resize(need);
      while (end < need) {
        ssize_t k;
        do {
          k = ::recv(fd, in.data() + end, in.size() - end, 0);
        } while (k < 0 && errno == EINTR);
        if (k <= 0) return false;
        end += static_cast<size_t>(k);
      }
      return true;
    };
    std::vector<char> buf;
    while (true) {
      if (!fill(4)) break;
      uint32_t be;
      std::memcpy(&be, in.data() + pos, 4);
      int32_t n = static_cast<int32_t>(ntohl(be));
      uint64_t len = static_cast<uint64_t>(n);
      size_t hdr = 4;
      if (n == -1) {
        if (!fill(12)) break;
        uint64_t be8;
        std::memcpy(&be8, in.data() + pos + 4, 8);
        len = be64toh(be8);
        hdr = 12;
      }
      if (!fill(hdr + len)) break;
      buf.assign(in.data() + pos + hdr, in.data() + pos + hdr + len);
      pos += hdr + len;
      if (len < 4) continue;
      uint32_t type;
      std::memcpy(&type, buf.data(), 4);
      if (type == F_FREE && len >= 12) {  // u32 type, u32 n, u32 pad, i64 slots[n]
        uint32_t cnt;
        std::memcpy(&cnt, buf.data() + 4, 4);
        std::vector<int64_t> s(cnt);
        if (12 + 8ull * cnt <= len) {
          std::memcpy(s.data(), buf.data() + 12, 8ull * cnt);
          slots->free(s);
          freed.fetch_add(cnt);
        }
      } else if (type == F_SUBMITTED && len >= 20) {  // u32 type, u64 token, u32 n, u32 pad
        uint64_t tok;
        uint32_t cnt;
        std::memcpy(&tok, buf.data() + 4, 8);
        std::memcpy(&cnt, buf.data() + 12, 4);
        std::lock_guard<std::mutex> g(ack_mu);
        auto it = acks.find(tok);
        if (it != acks.end()) {
          it->second.done = true;
          it->second.n = cnt;
        }
        ack_cv.notify_all();
      } else if (type == F_SUBMITTED_MULTI && len >= 16) {  // u32 type, u64 token, u32 nreq, u32 created[nreq]
        uint64_t tok;
        uint32_t nreq;
        std::memcpy(&tok, buf.data() + 4, 8);
        std::memcpy(&nreq, buf.data() + 12, 4);
        if (16 + 4ull * nreq <= len) {
          std::lock_guard<std::mutex> g(ack_mu);
          auto it = acks.find(tok);
          if (it != acks.end()) {
            it->second.per.resize(nreq);
            if (nreq) std::memcpy(it->second.per.data(), buf.data() + 16, 4ull * nreq);
            it->second.done = true;
          }
          ack_cv.notify_all();
        }
      } else if (type == F_STOP) {
        break;
      }
    }
    std::_Exit(0);  // scheduler connection closed: nothing left to serve
  }
};

struct Route {
  std::string prefix, mode;
  std::vector<int> shards;  // the endpoint's control-plane shards (one scheduler per GPU); empty: proxied
  std::atomic<uint64_t> rr{0};
  int64_t max_content_length = 0, max_concurrent = -1;
  std::vector<std::string> content_types, keys;
  std::atomic<int64_t> inflight{0};
};

struct Config {
  std::string host = "127.0.0.1";
  int port = 0;
  std::string internal_host = "127.0.0.1";
  int internal_port = 0;
  double ack_timeout = 30.0, alloc_timeout = 60.0;
  double max_queue_s = 0.0;  // latency budget of an ingested request's queue wait (0: no budget, wait for slots)
  double hold_s = -1.0;      // longest wait at the door before a 429 (< 0: one budget)
  int ready_fd = -1;  // "ready FD": one byte written once the public socket listens (the parent hands the port over)
  int frontend_index = -1;  // "frontend_index I": this process's word in every shard's counters
  std::vector<std::string> keys;
  std::vector<std::unique_ptr<Shard>> shards;
  std::vector<std::unique_ptr<Route>> routes;  // longest prefix first
};

Config g_cfg;

// "listen H P" | "internal H P" | "key K" | "tls CERT KEY" | "ack_timeout S" | "alloc_timeout S" | "ready FD"
// "shard IDX FD SHM NSLOTS ITEM BASE LEN ENDPOINT SHAPE" | "route PREFIX MODE SHARD MCL MC TYPES|- KEYS|-"
void parse_config(const char* path) {
  std::ifstream in(path);
  if (!in) {
    std::fprintf(stderr, "ai4e_ingestd: cannot read %s\n", path);
    std::exit(2);
  }
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    std::string kw;
    ls >> kw;
    if (kw == "listen") {
      ls >> g_cfg.host >> g_cfg.port;
    } else if (kw == "internal") {
      ls >> g_cfg.internal_host >> g_cfg.internal_port;
    } else if (kw == "key") {
      std::string k;
      ls >> k;
      g_cfg.keys.push_back(k);
    } else if (kw == "tls") {
      std::string cert, key;
      ls >> cert >> key;
      g_tls = SSL_CTX_new(TLS_server_method());
      if (!g_tls || SSL_CTX_set_min_proto_version(g_tls, TLS1_2_VERSION) != 1 ||
          SSL_CTX_use_certificate_chain_file(g_tls, cert.c_str()) != 1 ||
          SSL_CTX_use_PrivateKey_file(g_tls, key.c_str(), SSL_FILETYPE_PEM) != 1 || SSL_CTX_check_private_key(g_tls) != 1) {
        std::fprintf(stderr, "ai4e_ingestd: cannot load TLS certificate %s / key %s\n", cert.c_str(), key.c_str());
        ERR_print_errors_fp(stderr);
        std::exit(2);
      }
      SSL_CTX_set_mode(g_tls, SSL_MODE_AUTO_RETRY);
#ifdef SSL_OP_ENABLE_KTLS
      SSL_CTX_set_options(g_tls, SSL_OP_ENABLE_KTLS);  // kernel TLS offload where available (no-op otherwise)
#endif
    } else if (kw == "ack_timeout") {
      ls >> g_cfg.ack_timeout;
    } else if (kw == "alloc_timeout") {
      ls >> g_cfg.alloc_timeout;
    } else if (kw == "ready") {
      ls >> g_cfg.ready_fd;
    } else if (kw == "frontend_index") {
      ls >> g_cfg.frontend_index;
    } else if (kw == "hold_ms") {
      double ms = 0;
      ls >> ms;
      g_cfg.hold_s = ms / 1e3;
    } else if (kw == "max_queue_ms") {
      double ms = 0;
      ls >> ms;
      g_cfg.max_queue_s = ms / 1e3;
    } else if (kw == "shard") {
      auto s = std::make_unique<Shard>();
      std::string shm;
      ls >> s->idx >> s->fd >> shm >> s->nslots >> s->item >> s->base >> s->len >> s->endpoint >> s->shape_str;
      std::string dg, stat;
      if (ls >> dg && !dg.empty() && dg != "-") s->digits = dg;
      const bool have_stat = static_cast<bool>(ls >> stat);
      int64_t mb = 0;
      if (have_stat && (ls >> mb) && mb > 0) s->max_batch = mb;
      if (have_stat && !stat.empty() && stat != "-") {
        const int sfd = shm_open(("/" + stat).c_str(), O_RDWR, 0);
        void* sp = sfd >= 0 ? mmap(nullptr, Shard::kStatWords * 8, PROT_READ | PROT_WRITE, MAP_SHARED, sfd, 0)
                            : MAP_FAILED;
        if (sfd >= 0) ::close(sfd);
        if (sp != MAP_FAILED) s->st = static_cast<std::atomic<uint64_t>*>(sp);  // (else: partition estimate)
      }
      s->endpoint_path = ai4e::absolute_path(s->endpoint);
      int mfd = shm_open(("/" + shm).c_str(), O_RDWR, 0);
      if (mfd < 0) {
        std::perror("ai4e_ingestd: shm_open");
        std::exit(2);
      }
      const size_t ring_bytes = static_cast<size_t>(s->nslots * s->item);
      struct stat sb{};
      const bool tail = fstat(mfd, &sb) == 0 && static_cast<size_t>(sb.st_size) >= ring_bytes + sizeof(ai4e::RingTail);
      const size_t map_bytes = ring_bytes + (tail ? sizeof(ai4e::RingTail) : 0);
      void* p = mmap(nullptr, map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, mfd, 0);
      ::close(mfd);
      if (p == MAP_FAILED) {
        std::perror("ai4e_ingestd: mmap");
        std::exit(2);
      }
      s->ring = static_cast<uint8_t*>(p);
      if (tail) {
        ai4e::RingTail t;
        std::memcpy(&t, s->ring + ring_bytes, sizeof(t));
        if (t.magic == ai4e::kRingTailMagic) s->jpeg_key = t.key;
      }
      if (std::sscanf(s->shape_str.c_str(), "(%d,%d,%d)", &s->out_h, &s->out_w, &s->out_c) != 3) s->jpeg_key = 0;
      s->slots = std::make_unique<ai4e::SlotRing>(s->len, s->base);
      g_cfg.shards.push_back(std::move(s));
    } else if (kw == "route") {
      auto r = std::make_unique<Route>();
      std::string types, keys, shards;
      ls >> r->prefix >> r->mode >> shards >> r->max_content_length >> r->max_concurrent >> types >> keys;
      for (auto& v : split(shards, ','))
        if (!v.empty() && std::atoi(v.c_str()) >= 0) r->shards.push_back(std::atoi(v.c_str()));
      if (types != "-")
        for (auto& t : split(types, ',')) r->content_types.push_back(t);
      if (keys != "-")
        for (auto& k : split(keys, ',')) r->keys.push_back(k);
      g_cfg.routes.push_back(std::move(r));
    }
  }
  std::sort(g_cfg.routes.begin(), g_cfg.routes.end(),
            [](const std::unique_ptr<Route>& a, const std::unique_ptr<Route>& b) {
              return a->prefix.size() > b->prefix.size();
            });
}

// ------------------------------------------------------------------ HTTP
struct Request {
  std::string method, target, path, query, version;
  std::vector<std::pair<std::string, std::string>> headers;  // original case, in order
  std::map<std::string, std::string> h;                       // lower-case name -> value
  int64_t content_length = -1;
  bool chunked = false, keep_alive = true;
  std::string get(const char* k) const {
    auto it = h.find(k);
    return it == h.end() ? std::string() : it->second;
  }
};

struct Conn {
  int fd;
  SSL* ssl = nullptr;     // TLS session of a client connection (g_tls), else plain recv/send
  std::vector<char> buf;  // bytes received past the current parse point
  size_t pos = 0, end = 0;
  int upstream = -1;      // keep-alive connection to the internal listener
  std::mt19937_64 rng{std::random_device{}()};

  explicit Conn(int f) : fd(f), buf(1 << 16) {}
  ~Conn() {
    if (upstream >= 0) ::close(upstream);
    if (ssl) SSL_free(ssl);
  }
  // one read of up to n bytes (> 0), 0 = closed / error
  ssize_t recv_some(void* dst, size_t n) {
    if (ssl) {
      const int k = SSL_read(ssl, dst, static_cast<int>(std::min<size_t>(n, 1u << 30)));
      return k > 0 ? k : 0;
    }
    ssize_t k;
    do {
      k = ::recv(fd, dst, n, 0);
    } while (k < 0 && errno == EINTR);
    return k > 0 ? k : 0;
  }
  bool read_exact(void* p, size_t n) {
    if (!ssl) return ::read_exact(fd, p, n);
    char* d = static_cast<char*>(p);
    while (n) {
      const ssize_t k = recv_some(d, n);
      if (k <= 0) return false;
      d += k;
      n -= static_cast<size_t>(k);
    }
    return true;
  }
  bool send_all(const void* p, size_t n) {
    if (!ssl) return write_all(fd, p, n);
    const char* d = static_cast<const char*>(p);
    while (n) {
      const int k = SSL_write(ssl, d, static_cast<int>(std::min<size_t>(n, 1u << 30)));
      if (k <= 0) return false;
      d += k;
      n -= static_cast<size_t>(k);
    }
    return true;
  }
  size_t avail() const { return end - pos; }
  bool fill() {
    if (pos == end) pos = end = 0;
    if (end == buf.size()) {
      if (pos > 0) {
        std::memmove(buf.data(), buf.data() + pos, end - pos);
        end -= pos;
        pos = 0;
      } else {
        buf.resize(buf.size() * 2);
      }
    }
    const ssize_t k = recv_some(buf.data() + end, buf.size() - end);
    if (k <= 0) return false;
    end += static_cast<size_t>(k);
    return true;
  }
  // read exactly n body bytes into dst (buffered bytes first, then straight from the socket)
  bool body_into(uint8_t* dst, size_t n) {
    size_t take = std::min(n, avail());
    if (take) {
      std::memcpy(dst, buf.data() + pos, take);
      pos += take;
      dst += take;
      n -= take;
    }
    return n == 0 || read_exact(dst, n);
  }
  bool discard(size_t n) {
    std::vector<char> tmp(1 << 16);
    size_t take = std::min(n, avail());
    pos += take;
    n -= take;
    while (n) {
      size_t k = std::min(n, tmp.size());
      if (!read_exact(tmp.data(), k)) return false;
      n -= k;
    }
    return true;
  }
  bool line(std::string& out) {  // one CRLF line (for chunked bodies)
    while (true) {
      char* b = buf.data() + pos;
      char* e = static_cast<char*>(std::memchr(b, '\n', avail()));
      if (e) {
        out.assign(b, e);
        if (!out.empty() && out.back() == '\r') out.pop_back();
        pos += static_cast<size_t>(e - b) + 1;
        return true;
      }
      if (!fill()) return false;
    }
  }
};

bool read_head(Conn& c, Request& r) {
  size_t scanned = 0;
  while (true) {
    const char* b = c.buf.data() + c.pos;
    size_t n = c.avail();
    for (size_t i = scanned >= 3 ? scanned - 3 : 0; i + 3 < n; ++i) {
      if (b[i] == '\r' && b[i + 1] == '\n' && b[i + 2] == '\r' && b[i + 3] == '\n') {
        std::string head(b, i);
        c.pos += i + 4;
        std::istringstream hs(head);
        std::string l;
        std::getline(hs, l);
        if (!l.empty() && l.back() == '\r') l.pop_back();
        std::istringstream rl(l);
        rl >> r.method >> r.target >> r.version;
        if (r.method.empty() || r.target.empty()) return false;
        auto q = r.target.find('?');
        r.path = q == std::string::npos ? r.target : r.target.substr(0, q);
        r.query = q == std::string::npos ? "" : r.target.substr(q + 1);
        while (std::getline(hs, l)) {
          if (!l.empty() && l.back() == '\r') l.pop_back();
          auto colon = l.find(':');
          if (colon == std::string::npos) continue;
          std::string k = trim(l.substr(0, colon)), v = trim(l.substr(colon + 1));
          r.headers.emplace_back(k, v);
          r.h[lower(k)] = v;
        }
        std::string cl = r.get("content-length");
        if (!cl.empty()) r.content_length = std::strtoll(cl.c_str(), nullptr, 10);
        r.chunked = lower(r.get("transfer-encoding")).find("chunked") != std::string::npos;
        std::string conn = lower(r.get("connection"));
        r.keep_alive = r.version == "HTTP/1.1" ? conn.find("close") == std::string::npos
                                               : conn.find("keep-alive") != std::string::npos;
        return true;
      }
    }
    scanned = n;
    if (n > (1 << 20)) return false;  // header too large
    if (!c.fill()) return false;
  }
}

const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 202: return "Accepted";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 404: return "Not Found";
    case 411: return "Length Required";
    case 413: return "Request Entity Too Large";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

bool respond(Conn& c, int code, const std::string& ctype, const std::string& body, bool keep_alive,
             const std::string& extra_headers = "") {
  std::string h = "HTTP/1.1 " + std::to_string(code) + " " + reason(code) + "\r\nContent-Type: " + ctype +
                  "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n" + extra_headers +
                  (keep_alive ? "" : "Connection: close\r\n") + "Server: ai4e-ingestd\r\n\r\n";
  if (c.ssl) return c.send_all((h + body).data(), h.size() + body.size());  // one TLS record run
  struct iovec iov[2] = {{const_cast<char*>(h.data()), h.size()}, {const_cast<char*>(body.data()), body.size()}};
  size_t total = h.size() + body.size(), sent = 0;
  int idx = 0;
  while (sent < total) {
    ssize_t k = ::writev(c.fd, iov + idx, 2 - idx);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    sent += static_cast<size_t>(k);
    size_t kk = static_cast<size_t>(k);
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

std::string message_json(const std::string& m) {
  std::string out = "{\"message\":";
  ai4e::json_escape_into(out, m);
  return out + "}";
}

// application/x-www-form-urlencoded decoding of a query component (%XX, '+' = space), as aiohttp's request.query
std::string url_decode(const std::string& v) {
  std::string out;
  out.reserve(v.size());
  auto hex = [](char ch) {
    return ch >= '0' && ch <= '9' ? ch - '0' : ch >= 'a' && ch <= 'f' ? ch - 'a' + 10 : ch >= 'A' && ch <= 'F' ? ch - 'A' + 10 : -1;
  };
  for (size_t i = 0; i < v.size(); ++i) {
    if (v[i] == '+') {
      out.push_back(' ');
    } else if (v[i] == '%' && i + 2 < v.size() && hex(v[i + 1]) >= 0 && hex(v[i + 2]) >= 0) {
      out.push_back(static_cast<char>(hex(v[i + 1]) * 16 + hex(v[i + 2])));
      i += 2;
    } else {
      out.push_back(v[i]);
    }
  }
  return out;
}

std::string query_param(const std::string& q, const std::string& name) {
  for (auto& kv : split(q, '&')) {
    auto eq = kv.find('=');
    if (eq != std::string::npos && url_decode(kv.substr(0, eq)) == name) return url_decode(kv.substr(eq + 1));
  }
  return "";
}

bool ct_equal(const std::string& a, const std::string& b) {  // constant time per candidate
  if (a.size() != b.size()) return false;
  unsigned char d = 0;
  for (size_t i = 0; i < a.size(); ++i) d |= static_cast<unsigned char>(a[i] ^ b[i]);
  return d == 0;
}

// nullptr = allowed, else the APIM-style 401 message. Only the API routes are checked here: route-less paths
// (task management, control routes) are proxied and the serving process's key policy decides (gateway/server.py).
const char* check_key(const Request& r, const Route* route) {
  if (!route) return nullptr;
  std::vector<const std::string*> allowed;
  for (auto& k : g_cfg.keys) allowed.push_back(&k);
  if (route)
    for (auto& k : route->keys) allowed.push_back(&k);
  if (allowed.empty()) return nullptr;
  std::string key = r.get(kKeyHeader);
  if (key.empty()) key = query_param(r.query, "subscription-key");
  if (key.empty()) return kMissingKey;
  bool ok = false;
  for (auto* a : allowed) ok |= ct_equal(key, *a);
  return ok ? nullptr : kInvalidKey;
}

Route* match(const std::string& path) {
  for (auto& r : g_cfg.routes) {
    const std::string& p = r->prefix;
    std::string pre = p;
    while (!pre.empty() && pre.back() == '/') pre.pop_back();
    if (path == p || path.compare(0, pre.size() + 1, pre + "/") == 0) return r.get();
  }
  return nullptr;
}

// ------------------------------------------------------------------ proxy to the serving process
int connect_internal() {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(g_cfg.internal_port));
  inet_pton(AF_INET, g_cfg.internal_host.c_str(), &a.sin_addr);
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    ::close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}

// 0 = body read, -1 = connection error, 413 = the body (declared length, or chunks so far) exceeds `limit`
// bytes: nothing beyond the limit is allocated or read.
int read_body(Conn& c, const Request& r, std::string& body, int64_t limit) {
  if (r.chunked) {
    while (true) {
      std::string l;
      if (!c.line(l)) return -1;
      if (l.size() > 32) return 413;  // a chunk-size line this long is not a size we would accept
      errno = 0;
      const unsigned long long n = std::strtoull(l.c_str(), nullptr, 16);
      if (errno == ERANGE || n > static_cast<unsigned long long>(limit) ||
          body.size() + n > static_cast<unsigned long long>(limit))
        return 413;
      if (n == 0) {
        do {
          if (!c.line(l)) return -1;
        } while (!l.empty());
        return 0;
      }
      size_t off = body.size();
      body.resize(off + static_cast<size_t>(n));
      if (!c.body_into(reinterpret_cast<uint8_t*>(&body[off]), static_cast<size_t>(n))) return -1;
      if (!c.line(l)) return -1;
    }
  }
  if (r.content_length > limit) return 413;
  if (r.content_length > 0) {
    body.resize(static_cast<size_t>(r.content_length));
    return c.body_into(reinterpret_cast<uint8_t*>(&body[0]), body.size()) ? 0 : -1;
  }
  return 0;
}

bool is_hop(const std::string& k) {
  static const char* hop[] = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te",
                              "trailers", "transfer-encoding", "upgrade", "content-length", "expect"};
  std::string l = lower(k);
  for (auto* h : hop)
    if (l == h) return true;
  return false;
}

bool too_large(Conn& c, int64_t limit) {  // answered before the body is read: the connection closes after
  respond(c, 413, "application/json",
          message_json("Request content too large. Must be smaller than: " + std::to_string(limit)), false);
  return false;
}

// `prebody`: the request's body, already read (a JPEG the GPU path does not take, csrc ingest_jpeg)
bool proxy(Conn& c, const Request& r, const Route* route, const std::string* prebody = nullptr) {
  const int64_t limit = route && route->max_content_length > 0 ? std::min(route->max_content_length, kMaxBody) : kMaxBody;
  std::string body;
  if (prebody) {
    body = *prebody;
  } else {
    // a client waiting for 100-continue before its body (the load generator from 64 KiB) would otherwise stall
    // until its own timeout; the body then goes upstream whole, without the Expect header
    if (lower(r.get("expect")) == "100-continue" && r.content_length > 0 &&
        !c.send_all("HTTP/1.1 100 Continue\r\n\r\n", 25))
      return false;
    const int rb = read_body(c, r, body, limit);
    if (rb == 413) return too_large(c, limit);
    if (rb != 0) return false;
  }
  std::string req = r.method + " " + r.target + " HTTP/1.1\r\n";
  for (auto& kv : r.headers)
    if (!is_hop(kv.first)) req += kv.first + ": " + kv.second + "\r\n";
  req += "Content-Length: " + std::to_string(body.size()) + "\r\nConnection: keep-alive\r\n\r\n";
  for (int attempt = 0; attempt < 2; ++attempt) {  // a kept-alive upstream may have been closed meanwhile
    if (c.upstream < 0 && (c.upstream = connect_internal()) < 0) break;
    if (!write_all(c.upstream, req.data(), req.size()) || !write_all(c.upstream, body.data(), body.size())) {
      ::close(c.upstream);
      c.upstream = -1;
      continue;
    }
    Conn up(c.upstream);
    Request resp;
    // (the upstream's status line parses with method = version, target = code)
    if (!read_head(up, resp)) {
      ::close(c.upstream);
      c.upstream = -1;
      up.fd = -1;
      if (attempt == 0) continue;
      break;
    }
    std::string rbody;
    bool ok;
    const int status = std::atoi(resp.target.c_str());
    if (status < 200 || status == 204 || status == 304 || r.method == "HEAD") {
      ok = true;  // no body by definition
    } else if (resp.chunked || resp.content_length >= 0) {
      ok = read_body(up, resp, rbody, kMaxUpstreamBody) == 0;
    } else {  // no length: until the upstream closes
      rbody.assign(up.buf.data() + up.pos, up.avail());
      up.pos = up.end;
      while (up.fill()) {
        rbody.append(up.buf.data() + up.pos, up.avail());
        up.pos = up.end;
      }
      ok = true;
      ::close(c.upstream);
      c.upstream = -1;
    }
    up.fd = -1;  // (the Conn wrapper does not own the upstream socket)
    if (!ok) {
      if (c.upstream >= 0) ::close(c.upstream);
      c.upstream = -1;
      break;
    }
    if (lower(resp.get("connection")).find("close") != std::string::npos && c.upstream >= 0) {
      ::close(c.upstream);
      c.upstream = -1;
    }
    const int code = status;
    std::string extra, ctype = "application/octet-stream";
    for (auto& kv : resp.headers) {
      std::string l = lower(kv.first);
      if (is_hop(kv.first) || l == "content-encoding" || l == "server" || l == "date") continue;
      if (l == "content-type") {
        ctype = kv.second;
        continue;
      }
      extra += kv.first + ": " + kv.second + "\r\n";
    }
    return respond(c, code, ctype, rbody, r.keep_alive, extra);
  }
  return respond(c, 502, "application/json", message_json("gateway unreachable"), false) && false;
}

// ------------------------------------------------------------------ ingest
std::string task_json(const std::string& tid, const Shard& s) {
  std::string out = "{\"TaskId\":\"" + tid + "\",\"Timestamp\":";
  ai4e::json_escape_into(out, ai4e::dotnet_timestamp(ai4e::wall_now()));
  out += ",\"Status\":\"created\",\"BackendStatus\":\"created\",\"Endpoint\":";
  ai4e::json_escape_into(out, s.endpoint);
  out += ",\"Body\":null,\"PublishToGrid\":true,\"EndpointPath\":";
  ai4e::json_escape_into(out, s.endpoint_path);
  return out + "}";
}

std::string py_list(const std::vector<std::string>& v) {  // Python's repr of a list of str
  std::string out = "[";
  for (size_t i = 0; i < v.size(); ++i) out += (i ? ", '" : "'") + v[i] + "'";
  return out + "]";
}

constexpr int64_t kDrainMax = 1 << 20;  // refused bodies read and dropped to keep a non-Expect connection

// mode: 0 one raw item, 1 a binary batch, 2 one JPEG frame (prepared into its slot for the workers' GPU decode,
// runtime/jpeg_gpu.py; a frame the GPU path does not take goes to the serving process with its body)
bool ingest(Conn& c, const Request& r, Route& route, Shard& s, int mode) {
  const bool batch = mode == 1, jpeg = mode == 2;
  const int64_t nbytes = r.content_length;
  const bool ka = r.keep_alive;
  auto reject = [&](int code, const std::string& msg) {  // answer without reading the body: close after
    respond(c, code, "application/json", message_json(msg), false);
    return false;
  };
  if (g_draining.load()) return reject(503, "Service is terminating, please try again later.");
  if (route.max_concurrent >= 0 && route.inflight.load() + 1 > route.max_concurrent)
    return reject(429, "Service is busy, please try again later.");
  struct Guard {
    std::atomic<int64_t>& v;
    explicit Guard(std::atomic<int64_t>& x) : v(x) { v.fetch_add(1); }
    ~Guard() { v.fetch_sub(1); }
  } guard(route.inflight);
  std::string ctype = lower(trim(split(r.get("content-type"), ';')[0]));
  if (!route.content_types.empty() &&
      std::find(route.content_types.begin(), route.content_types.end(), ctype) == route.content_types.end())
    return reject(401, "Content-type must be " + py_list(route.content_types));
  if (nbytes > kMaxBody) return reject(413, "Request content too large (" + std::to_string(nbytes) + ")");
  if (route.max_content_length > 0 && nbytes > route.max_content_length)
    return reject(413, "Request content too large (" + std::to_string(nbytes) +
                           "). Must be smaller than: " + std::to_string(route.max_content_length));
  if (!jpeg && (nbytes <= 0 || nbytes % s.item))
    return reject(400, "batch payload must be a multiple of " + std::to_string(s.item) + " bytes (uint8 " +
                           s.shape_str + ")");
  const int64_t n = jpeg ? 1 : nbytes / s.item;
  if (n > s.len)
    return reject(413, "batch of " + std::to_string(n) + " items exceeds the ingest partition (" +
                           std::to_string(s.len) + " slots)");
  if (g_cfg.max_queue_s > 0.0) {
    // latency-budgeted admission (the reference's busy path: BackendQueueProcessor.cs:54-64 answers 429 and the
    // message is retried later; ai4e_service.py:122-125): a request whose projected queue wait exceeds the budget is
    // refused with 429 + Retry-After instead of queueing behind a deep ring
    double wait = s.projected_wait(n, static_cast<double>(nbytes));
    // A request only a little over the budget waits at the door — before its body is read and before any task
    // exists — for the backlog to drain, instead of a 429 and a client back-off round trip: at saturation with many
    // small clients almost every refusal is of this kind (projected wait a few ms past the budget), and the refused
    // client would be back within those milliseconds anyway. The wait shows in the client's request latency, not in
    // any task's queue wait.
    const double hold_max = g_cfg.hold_s >= 0.0 ? g_cfg.hold_s : g_cfg.max_queue_s;
    double held = 0.0;
    while (wait > g_cfg.max_queue_s && held + (wait - g_cfg.max_queue_s) <= hold_max) {
      const double d = std::max(2e-4, wait - g_cfg.max_queue_s);
      std::this_thread::sleep_for(std::chrono::microseconds(static_cast<long>(d * 1e6)));
      held += d;
      wait = s.projected_wait(n, static_cast<double>(nbytes));
    }
    if (wait > g_cfg.max_queue_s) {
      s.refused.fetch_add(1, std::memory_order_relaxed);
      static const bool dbg = std::getenv("AI4E_INGESTD_DEBUG") != nullptr;
      static std::atomic<int> dbg_n{0};
      if (dbg && s.st && dbg_n.fetch_add(1) % 500 == 0)
        std::fprintf(stderr, "ingestd 429: wait %.2f ms backlog %.0f rate %.0f enq %llu done %llu inflight %llu\n",
                     wait * 1e3, s.backlog(), s.rate, static_cast<unsigned long long>(s.st[0].load()),
                     static_cast<unsigned long long>(s.st[1].load()), static_cast<unsigned long long>(s.st[4].load()));
      // the hint: the time for the backlog above the budget to drain (>= 1 ms), at most twice the budget (a request
      // refused on a stale estimate is judged again soon). A hint of a whole budget starved the batch route (16
      // clients, 250 images each: 78k -> 67k images/s); clients back off exponentially on repeated refusals instead
      // (csrc/ingest/http_load.cpp)
      const double retry_s = std::min(2.0 * g_cfg.max_queue_s, std::max(0.001, wait - g_cfg.max_queue_s));
      const std::string h = "Retry-After: " + std::to_string(static_cast<int>(std::ceil(retry_s))) +
                            "\r\nx-ai4e-retry-after-ms: " + std::to_string(static_cast<int>(std::ceil(retry_s * 1e3))) +
                            "\r\n";
      // An Expect: 100-continue client (the load generator sends it for bodies of 64 KiB or more) sends no body after
      // a final answer, so its connection stays usable: a refusal costs a header round trip. Any other client's body
      // is on its way: one under kDrainMax is read and dropped (measured: closing instead made every refusal a
      // reconnect + a new connection thread, and the single-image route fell from 48k to 23k images/s); a larger
      // one is refused unread and the connection closed.
      if (lower(r.get("expect")) != "100-continue") {
        if (nbytes <= kDrainMax && c.discard(static_cast<size_t>(nbytes)))
          return respond(c, 429, "application/json", message_json("Service is busy, please try again later."), ka, h);
        respond(c, 429, "application/json", message_json("Service is busy, please try again later."), false, h);
        ::shutdown(c.fd, SHUT_WR);
        return false;
      }
      return respond(c, 429, "application/json", message_json("Service is busy, please try again later."), ka, h);
    }
  }
  // admitted: until its tasks exist the body counts as the shard's backlog for every front-end's admission
  struct Pending {
    std::atomic<uint64_t>* p;
    uint64_t n;
    ~Pending() {
      if (p) p->fetch_sub(n);
    }
  } pending{g_cfg.max_queue_s > 0.0 ? s.pending_word(g_cfg.frontend_index) : nullptr, static_cast<uint64_t>(n)};
  if (pending.p) pending.p->fetch_add(pending.n);
  if (lower(r.get("expect")) == "100-continue" && !c.send_all("HTTP/1.1 100 Continue\r\n\r\n", 25)) return false;
  std::vector<int64_t> sl = s.slots->alloc(n, g_cfg.alloc_timeout);
  if (sl.empty()) {  // no ring slot in time: nothing was created
    if (!c.discard(static_cast<size_t>(nbytes))) return false;
    return respond(c, 429, "application/json", message_json("Service is busy, please try again later."), ka);
  }
  const double t_up = ai4e::mono_now();
  if (jpeg) {
    // body -> scratch -> headers + unstuffed scan into the slot (~0.2 ms), marked with the ring's key
    thread_local std::string jbody;
    thread_local std::unique_ptr<ai4e::JpegCoefDecoder> dec;
    if (!dec) dec = std::make_unique<ai4e::JpegCoefDecoder>();
    jbody.resize(static_cast<size_t>(nbytes));
    if (!c.body_into(reinterpret_cast<uint8_t*>(jbody.data()), jbody.size())) {
      s.slots->free(sl);
      return false;
    }
    uint8_t* slot = s.ring + sl[0] * s.item;
    const size_t cap = static_cast<size_t>(s.item) - sizeof(ai4e::JpegSlotTrailer);
    size_t used = 0;
    const bool ok = s.item > static_cast<int64_t>(sizeof(ai4e::JpegScanHeader) + sizeof(ai4e::JpegSlotTrailer)) &&
                    dec->prepare(reinterpret_cast<const uint8_t*>(jbody.data()), jbody.size(), slot, cap, &used) ==
                        ai4e::JpegCoefDecoder::kOk &&
                    ai4e::jpeg_gpu_plan_ok(*reinterpret_cast<const ai4e::JpegScanHeader*>(slot), s.out_h, s.out_w,
                                           s.out_c);
    if (!ok) {  // decoded on the CPU by the serving process
      s.slots->free(sl);
      return proxy(c, r, &route, &jbody);
    }
    ai4e::JpegSlotTrailer tr{ai4e::kJpegSlotMagic, s.jpeg_key, static_cast<uint32_t>(used), 0, 0};
    std::memcpy(slot + s.item - sizeof(tr), &tr, sizeof(tr));
    static const bool dbg = std::getenv("AI4E_INGESTD_DEBUG") != nullptr;
    static std::atomic<int> dbg_n{0};
    if (dbg && dbg_n.fetch_add(1) < 4) std::fprintf(stderr, "ingestd jpeg: %zu bytes prepared into slot %lld\n", used,
                                                    static_cast<long long>(sl[0]));
  }
  // body -> ring: one recv per contiguous slot run
  for (size_t i = 0; !jpeg && i < sl.size();) {
    size_t j = i + 1;
    while (j < sl.size() && sl[j] == sl[j - 1] + 1) ++j;
    if (!c.body_into(s.ring + sl[i] * s.item, static_cast<size_t>((j - i) * s.item))) {
      s.slots->free(sl);
      return false;
    }
    i = j;
  }
  s.note_upload(static_cast<double>(nbytes), ai4e::mono_now() - t_up);
  // B3: a child span of the caller's (utils/tracing.py b3_from_headers / b3_pack)
  std::string trace_id = r.get("x-b3-traceid"), parent = r.get("x-b3-spanid"), sampled = r.get("x-b3-sampled");
  if (trace_id.empty()) trace_id = hexid(c.rng, 128);
  std::string span = hexid(c.rng, 64);
  if (sampled.empty()) sampled = "1";
  std::string b3 = "x-b3-traceid: " + trace_id + "\r\nx-b3-spanid: " + span + "\r\nx-b3-parentspanid: " + parent +
                   "\r\nx-b3-sampled: " + sampled + "\r\n";
  std::vector<std::string> ids = s.mint(static_cast<size_t>(n));
  const int64_t created = s.submit_wait(sl, ids, trace_id + "/" + span + "/" + parent, g_cfg.ack_timeout);
  if (batch) {
    std::string body = "{\"TaskIds\":[";
    for (size_t i = 0; i < ids.size(); ++i) body += (i ? ",\"" : "\"") + ids[i] + "\"";
    body += "]";
    if (created < 0) body += ",\"message\":\"accepted, not yet acknowledged\"";
    body += "}";
    return respond(c, created < 0 ? 202 : 200, "application/json", body, ka, b3);
  }
  if (created == 0)
    return respond(c, 500, "application/json", message_json("Task insert failed."), ka, b3);
  std::string accept = r.get("accept");
  if (accept.empty() || accept.find("application/json") != std::string::npos ||
      accept.find("*/*") != std::string::npos)
    return respond(c, created < 0 ? 202 : 200, "application/json", task_json(ids[0], s), ka, b3);
  return respond(c, created < 0 ? 202 : 200, "text/plain; charset=utf-8", "TaskId: " + ids[0], ka, b3);
}

// The control-plane shard of an endpoint that takes the next request: among the shards with a live GPU worker, the
// one with the smallest backlog (the scheduler's published counters: tasks not finished + bodies uploading), else the
// smallest share of this front-end's partition in use; ties round-robin. A shard without a live worker is only
// picked when no shard has one (its peers drain its queue: NodeScheduler competing consumers).
Shard* pick_shard(Route& route) {
  const size_t k = route.shards.size();
  if (k == 0) return nullptr;
  if (k == 1) return g_cfg.shards[static_cast<size_t>(route.shards[0])].get();
  const size_t start = static_cast<size_t>(route.rr.fetch_add(1) % k);
  Shard* best = nullptr;
  double best_load = 0.0;
  bool best_live = false;
  for (size_t i = 0; i < k; ++i) {
    Shard* s = g_cfg.shards[static_cast<size_t>(route.shards[(start + i) % k])].get();
    const bool live = s->live();
    const double load = s->st ? s->backlog() + static_cast<double>(s->slots->used())
                              : static_cast<double>(s->slots->used()) / static_cast<double>(std::max<int64_t>(1, s->len));
    if (!best || (live && !best_live) || (live == best_live && load < best_load)) {
      best = s;
      best_load = load;
      best_live = live;
    }
  }
  return best;
}

void serve_requests(Conn& c);
std::atomic<int> g_conns{0};
constexpr int kMaxConns = 4096;  // one thread each; beyond this new connections are answered 503 and closed

void serve_conn(int fd) {
  struct Count {
    Count() { g_conns.fetch_add(1); }
    ~Count() { g_conns.fetch_sub(1); }
  } count;
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int rcv = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof(rcv));
  struct timeval idle {300, 0};  // an idle keep-alive connection (or a stalled body) releases its thread
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &idle, sizeof(idle));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &idle, sizeof(idle));
  Conn c(fd);
  if (g_tls) {
    c.ssl = SSL_new(g_tls);
    if (!c.ssl || SSL_set_fd(c.ssl, fd) != 1 || SSL_accept(c.ssl) != 1) {
      ERR_clear_error();
      ::close(fd);
      return;
    }
  }
  try {
    serve_requests(c);
  } catch (const std::exception& e) {  // (bad_alloc, length_error, ...): this connection ends, the process stays
    std::fprintf(stderr, "ai4e_ingestd: connection dropped: %s\n", e.what());
  }
  if (c.ssl) SSL_shutdown(c.ssl);
  ::close(fd);
}

void serve_requests(Conn& c) {
  while (true) {
    Request r;
    if (!read_head(c, r)) break;
    Route* route = match(r.path);
    if (r.path != "/" && r.path != "/openapi.json") {
      if (const char* msg = check_key(r, route)) {
        std::string body = "{\"statusCode\":401,\"message\":";
        ai4e::json_escape_into(body, msg);
        body += "}";
        bool drained = !r.chunked && r.content_length <= (1 << 20) &&
                       c.discard(static_cast<size_t>(std::max<int64_t>(0, r.content_length)));
        if (!respond(c, 401, "application/json", body, r.keep_alive && drained) || !r.keep_alive || !drained) break;
        continue;
      }
    }
    bool ok;
    std::string ctype = lower(trim(split(r.get("content-type"), ';')[0]));
    Shard* s = route ? pick_shard(*route) : nullptr;
    const bool ingestible = s && route->mode == "async" && (r.method == "POST" || r.method == "PUT") &&
                            r.get("taskid").empty() && !r.chunked && r.content_length >= 0;
    if (ingestible && ctype == kBatchType && r.content_length > 0) {
      ok = ingest(c, r, *route, *s, 1);
    } else if (ingestible && ctype == kRawType && r.content_length == s->item) {
      ok = ingest(c, r, *route, *s, 0);
    } else if (ingestible && s->jpeg_key && r.content_length > 0 &&
               (ctype == "image/jpeg" || ctype == "image/jpg" || ctype == "image/pjpeg")) {
      ok = ingest(c, r, *route, *s, 2);
    } else {
      ok = proxy(c, r, route);  // encoded images, task API, sync routes, ... -> the serving process
    }
    if (!ok || !r.keep_alive) break;
  }
}

int listen_on(const std::string& host, int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, host == "0.0.0.0" || host.empty() ? "0.0.0.0" : host.c_str(), &a.sin_addr) != 1)
    a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(fd, 1024) != 0) {
    std::perror("ai4e_ingestd: bind/listen");
    std::exit(3);
  }
  return fd;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: ai4e_ingestd CONFIG\n");
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  parse_config(argv[1]);
  struct sigaction sa{};
  sa.sa_handler = [](int) {  // drain: refuse new ingest (503), let in-flight requests finish, then exit
    g_draining.store(true);
    alarm(5);
  };
  sigaction(SIGTERM, &sa, nullptr);
  struct sigaction al{};
  al.sa_handler = [](int) { std::_Exit(0); };
  sigaction(SIGALRM, &al, nullptr);
  for (auto& s : g_cfg.shards) std::thread([p = s.get()] { p->reader(); }).detach();
  int lfd = listen_on(g_cfg.host, g_cfg.port);
  if (g_cfg.ready_fd >= 0) {
    const char one = 'R';
    (void)!::write(g_cfg.ready_fd, &one, 1);
    ::close(g_cfg.ready_fd);
  }
  std::fprintf(stderr, "ai4e_ingestd pid %d on %s:%d (%zu endpoints, %zu routes)\n", getpid(), g_cfg.host.c_str(),
               g_cfg.port, g_cfg.shards.size(), g_cfg.routes.size());
  while (true) {
    int fd = ::accept(lfd, nullptr, nullptr);
    if (fd < 0) {
      if (errno == EINTR) continue;
      continue;
    }
    if (g_conns.load() >= kMaxConns) {
      if (g_tls) {  // (no handshake for a connection we are not going to serve)
        ::close(fd);
        continue;
      }
      static const char busy[] =
          "HTTP/1.1 503 Service Unavailable\r\nContent-Type: application/json\r\nContent-Length: 54\r\n"
          "Connection: close\r\n\r\n{\"message\":\"Service is busy, please try again later.\"}";
      write_all(fd, busy, sizeof(busy) - 1);
      ::close(fd);
      continue;
    }
    std::thread(serve_conn, fd).detach();
  }
}
