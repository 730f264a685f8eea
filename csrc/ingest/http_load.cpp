// ai4e_http_load — HTTP/1.1 keep-alive load generator for the REST benchmarks (runtime/node_bench.py
// http_phase). A Python client tops out near the rate it is supposed to measure (one aiohttp process moves
// ~1-2 GB/s of request bodies); this one sends a prebuilt request (headers + body, one writev) per
// round trip from one thread per connection, parses the status line / Content-Length of the answer and
// collects the task ids it hands back, so the server side is what the benchmark measures. It reports its
// own CPU time (user + system) so a reader can tell whether the client was the ceiling.
//
//   ai4e_http_load HOST PORT PATH CONTENT_TYPE BODY_FILE CONNS SECONDS START_AT_EPOCH IDS_OUT [HEADER...]
//
// HOST = "tls:ADDR" speaks HTTPS (TLS 1.2+, OpenSSL, no certificate verification: a load generator against the
// platform's own front door); each request is then one SSL_write of the prebuilt head + body.
//
// Prints one JSON line: requests, ok, errors, busy (429s, retried after the server's Retry-After), t0, t1 (epoch s),
// bytes_sent, cpu_user_s, cpu_sys_s.
// IDS_OUT receives one task id per line (TaskId / TaskIds of every 2xx answer).
// Bodies of 64 KiB or more are sent as careful clients (curl: past 1 MiB) send them: `Expect: 100-continue` first, the
// body only after `100 Continue`, so a request the server's admission refuses (429) costs a header round trip, not
// the upload of the body, and the connection stays open (a refusal the server closes: the client dials again).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <csignal>
#include <cstdlib>
#include <random>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <openssl/err.h>
#include <openssl/ssl.h>

namespace {

SSL_CTX* g_tls = nullptr;

// one client connection: plain TCP or a TLS session over it
struct Link {
  int fd = -1;
  SSL* ssl = nullptr;
  void close() {
    if (ssl) {
      SSL_free(ssl);
      ssl = nullptr;
    }
    if (fd >= 0) ::close(fd);
    fd = -1;
  }
  ssize_t recv_some(char* p, size_t n) {
    if (ssl) {
      const int k = SSL_read(ssl, p, static_cast<int>(n));
      return k > 0 ? k : 0;
    }
    return ::recv(fd, p, n, 0);
  }
};

double now() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

struct Result {
  long requests = 0, ok = 0, errors = 0, busy = 0;
  double bytes = 0;
  std::vector<std::string> ids;
  std::vector<float> lat_ms;  // per admitted request: first attempt -> 2xx, 429 back-offs and retries included
};

bool send_all(int fd, const struct iovec* iov0, int cnt) {
  std::vector<struct iovec> iov(iov0, iov0 + cnt);
  size_t idx = 0;
  while (idx < iov.size()) {
    ssize_t k = ::writev(fd, iov.data() + idx, static_cast<int>(iov.size() - idx));
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    size_t kk = static_cast<size_t>(k);
    while (idx < iov.size() && kk >= iov[idx].iov_len) kk -= iov[idx++].iov_len;
    if (idx < iov.size()) {
      iov[idx].iov_base = static_cast<char*>(iov[idx].iov_base) + kk;
      iov[idx].iov_len -= kk;
    }
  }
  return true;
}

// Reads one response; returns the status (0 on a broken connection) and its body.
int read_response(Link& l, std::string& buf, std::string& body, double* retry_ms = nullptr, bool* closes = nullptr) {
  size_t hend;
  while ((hend = buf.find("\r\n\r\n")) == std::string::npos) {
    char tmp[65536];
    ssize_t k = l.recv_some(tmp, sizeof(tmp));
    if (k <= 0) return 0;
    buf.append(tmp, static_cast<size_t>(k));
  }
  int status = std::atoi(buf.c_str() + 9);
  size_t clen = 0;
  std::string head = buf.substr(0, hend);
  for (auto& ch : head) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  auto p = head.find("content-length:");
  if (p != std::string::npos) clen = std::strtoull(head.c_str() + p + 15, nullptr, 10);
  if (closes) *closes = head.find("connection: close") != std::string::npos;
  if (retry_ms) {  // 429: the server's projected wait (x-ai4e-retry-after-ms, else Retry-After seconds)
    *retry_ms = 0;
    auto q = head.find("x-ai4e-retry-after-ms:");
    if (q != std::string::npos) {
      *retry_ms = std::atof(head.c_str() + q + 22);
    } else if ((q = head.find("retry-after:")) != std::string::npos) {
      *retry_ms = 1e3 * std::atof(head.c_str() + q + 12);
    }
  }
  while (buf.size() < hend + 4 + clen) {
    char tmp[65536];
    ssize_t k = l.recv_some(tmp, sizeof(tmp));
    if (k <= 0) return 0;
    buf.append(tmp, static_cast<size_t>(k));
  }
  body = buf.substr(hend + 4, clen);
  buf.erase(0, hend + 4 + clen);
  return status;
}

void extract_ids(const std::string& body, std::vector<std::string>& out) {
  // {"TaskIds":["a","b",...]} or {"TaskId":"a",...}
  auto p = body.find("\"TaskIds\"");
  if (p != std::string::npos) {
    size_t e = body.find(']', p);
    size_t q = body.find('[', p);
    while (q != std::string::npos && q < e) {
      size_t a = body.find('"', q + 1);
      if (a == std::string::npos || a > e) break;
      size_t b = body.find('"', a + 1);
      out.emplace_back(body.substr(a + 1, b - a - 1));
      q = b;
    }
    return;
  }
  p = body.find("\"TaskId\"");
  if (p != std::string::npos) {
    size_t a = body.find('"', body.find(':', p) + 1);
    size_t b = body.find('"', a + 1);
    out.emplace_back(body.substr(a + 1, b - a - 1));
  }
}

int dial_tcp(const char* host, int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  inet_pton(AF_INET, host, &a.sin_addr);
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    ::close(fd);
    return -1;
  }
  int one = 1, snd = 4 << 20;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &snd, sizeof(snd));
  struct timeval tv {30, 0};  // a stalled server ends the run with errors instead of hanging it
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  return fd;
}

Link dial(const char* host, int port) {
  Link l;
  l.fd = dial_tcp(host, port);
  if (l.fd >= 0 && g_tls) {
    l.ssl = SSL_new(g_tls);
    if (!l.ssl || SSL_set_fd(l.ssl, l.fd) != 1 || SSL_connect(l.ssl) != 1) {
      ERR_clear_error();
      l.close();
    }
  }
  return l;
}

bool send_bytes(Link& l, const char* p, size_t n) {
  if (!l.ssl) {
    struct iovec one = {const_cast<char*>(p), n};
    return send_all(l.fd, &one, 1);
  }
  size_t off = 0;
  while (off < n) {
    const int k = SSL_write(l.ssl, p + off, static_cast<int>(std::min<size_t>(n - off, 1u << 30)));
    if (k <= 0) return false;
    off += static_cast<size_t>(k);
  }
  return true;
}

bool send_req(Link& l, const struct iovec* iov, const std::string& whole) {
  if (!l.ssl) return send_all(l.fd, iov, 2);
  size_t off = 0;
  while (off < whole.size()) {
    const int k = SSL_write(l.ssl, whole.data() + off, static_cast<int>(std::min<size_t>(whole.size() - off, 1u << 30)));
    if (k <= 0) return false;
    off += static_cast<size_t>(k);
  }
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);  // (a refused body the server closed on: the send fails, the answer is still read)
  if (argc < 10) {
    std::fprintf(stderr,
                 "usage: ai4e_http_load HOST PORT PATH CONTENT_TYPE BODY_FILE CONNS SECONDS START_AT IDS_OUT "
                 "[HEADER...]\n");
    return 2;
  }
  const char* host = argv[1];
  if (std::strncmp(host, "tls:", 4) == 0) {
    host += 4;
    g_tls = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_min_proto_version(g_tls, TLS1_2_VERSION);
    SSL_CTX_set_verify(g_tls, SSL_VERIFY_NONE, nullptr);
    SSL_CTX_set_mode(g_tls, SSL_MODE_AUTO_RETRY);
  }
  const int port = std::atoi(argv[2]);
  const std::string path = argv[3], ctype = argv[4];
  std::ifstream bf(argv[5], std::ios::binary);
  std::string body((std::istreambuf_iterator<char>(bf)), std::istreambuf_iterator<char>());
  const int conns = std::atoi(argv[6]);
  const double seconds = std::atof(argv[7]), start_at = std::atof(argv[8]);
  const char* ids_out = argv[9];
  std::string head = "POST " + path + " HTTP/1.1\r\nHost: " + std::string(host) + ":" + std::to_string(port) +
                     "\r\nContent-Type: " + ctype + "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
  for (int i = 10; i < argc; ++i) head += std::string(argv[i]) + "\r\n";
  // (curl sends Expect for bodies past 1 MiB; 64 KiB here, so a refused camera frame costs its headers, not its body)
  const char* emin = std::getenv("AI4E_HTTP_EXPECT_MIN");  // (bytes; A/B knob)
  const bool expect = body.size() >= (emin ? std::strtoull(emin, nullptr, 10) : (64u << 10));
  if (expect) head += "Expect: 100-continue\r\n";
  head += "\r\n";
  const std::string whole = g_tls ? head + body : std::string();  // (TLS: one SSL_write per request)

  std::vector<Result> res(static_cast<size_t>(conns));
  while (now() < start_at) std::this_thread::sleep_for(std::chrono::microseconds(200));
  const double t0 = now(), t_end = t0 + seconds;
  std::vector<std::thread> th;
  for (int c = 0; c < conns; ++c) {
    th.emplace_back([&, c] {
      Result& r = res[static_cast<size_t>(c)];
      Link l = dial(host, port);
      // a refused request waits the server's hint, doubled for every further refusal in a row (capped at 100 ms),
      // with +-25 % jitter so refused clients do not all return at once; an admitted request resets it
      std::mt19937 rng(static_cast<unsigned>(c) * 7919u + 17u);
      int refusals = 0;
      const int64_t ok0 = -1;
      int64_t seen_ok = ok0;
      double t_first = -1.0;  // start of the current logical request (kept across its 429 retries)
      auto backoff = [&](double hint_ms) {
        if (static_cast<int64_t>(r.ok) != seen_ok) refusals = 0;
        seen_ok = static_cast<int64_t>(r.ok);
        const double base = std::max(0.5, hint_ms) * static_cast<double>(1u << std::min(refusals, 8));
        ++refusals;
        const double ms = std::min(100.0, base) * std::uniform_real_distribution<double>(0.75, 1.25)(rng);
        std::this_thread::sleep_for(std::chrono::microseconds(static_cast<long>(ms * 1e3)));
      };
      std::string buf, rbody;
      struct iovec iov[2] = {{const_cast<char*>(head.data()), head.size()},
                             {const_cast<char*>(body.data()), body.size()}};
      while (l.fd >= 0 && now() < t_end) {
        if (t_first < 0) t_first = now();
        if (expect) {
          // headers, then the body only once the server's admission let the request in
          double retry_ms = 0;
          bool closes = false;
          int st = send_bytes(l, head.data(), head.size()) ? read_response(l, buf, rbody, &retry_ms, &closes) : 0;
          if (st == 100) {
            ++r.requests;
            r.bytes += static_cast<double>(head.size() + body.size());
            st = send_bytes(l, body.data(), body.size()) ? read_response(l, buf, rbody, &retry_ms) : 0;
          } else if (st != 0) {
            ++r.requests;
            r.bytes += static_cast<double>(head.size());
          }
          if (st >= 200 && st < 300) {
            ++r.ok;
            extract_ids(rbody, r.ids);
            r.lat_ms.push_back(static_cast<float>((now() - t_first) * 1e3));
            t_first = -1.0;
            continue;
          }
          if (st == 429) {
            ++r.busy;
            backoff(retry_ms);
          } else {
            ++r.errors;
          }
          if (st == 0 || closes) {  // (a refusal the server closed: dial again; a keep-alive one is reused)
            l.close();
            buf.clear();
            l = dial(host, port);
          }
          continue;
        }
        const bool sent = send_req(l, iov, whole);
        ++r.requests;
        r.bytes += static_cast<double>(head.size() + body.size());
        double retry_ms = 0;
        bool closes = false;
        // (a send cut short may still have its answer waiting: the server refuses an unread body with 429 and closes)
        int st = read_response(l, buf, rbody, &retry_ms, &closes);
        if (!sent && st != 429) st = 0;
        if (st == 429 && (closes || !sent)) {  // refused unread: back off, then dial again
          ++r.busy;
          backoff(retry_ms);
          l.close();
          buf.clear();
          l = dial(host, port);
          continue;
        }
        if (st == 0) {
          l.close();
          buf.clear();
          l = dial(host, port);
          ++r.errors;
          continue;
        }
        if (st >= 200 && st < 300) {
          ++r.ok;
          extract_ids(rbody, r.ids);
          r.lat_ms.push_back(static_cast<float>((now() - t_first) * 1e3));
          t_first = -1.0;
        } else if (st == 429) {  // admission refused: back off for the server's projected wait, then retry
          ++r.busy;
          backoff(retry_ms);
        } else {
          ++r.errors;
        }
      }
      l.close();
    });
  }
  for (auto& t : th) t.join();
  const double t1 = now();
  Result tot;
  FILE* f = std::fopen(ids_out, "w");
  for (auto& r : res) {
    tot.requests += r.requests;
    tot.ok += r.ok;
    tot.errors += r.errors;
    tot.busy += r.busy;
    tot.bytes += r.bytes;
    if (f)
      for (auto& id : r.ids) std::fprintf(f, "%s\n", id.c_str());
  }
  if (f) std::fclose(f);
  FILE* lf = std::fopen((std::string(ids_out) + ".lat").c_str(), "w");  // request latencies, ms, one per line
  if (lf) {
    for (auto& r : res)
      for (float v : r.lat_ms) std::fprintf(lf, "%.3f\n", v);
    std::fclose(lf);
  }
  struct rusage ru {};
  getrusage(RUSAGE_SELF, &ru);
  std::printf(
      "{\"requests\": %ld, \"ok\": %ld, \"errors\": %ld, \"busy\": %ld, \"t0\": %.6f, \"t1\": %.6f, \"bytes_sent\": %.0f, "
      "\"cpu_user_s\": %.3f, \"cpu_sys_s\": %.3f, \"connections\": %d}\n",
      tot.requests, tot.ok, tot.errors, tot.busy, t0, t1, tot.bytes, ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6,
      ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6, conns);
  return 0;
}
