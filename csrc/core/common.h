// Shared helpers of the native control plane: clocks, UUIDs, JSON escaping, .NET-style
// timestamps and System.Uri.AbsolutePath (ProcessManager/Classes/APITask.cs:19-26).
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <ctime>
#include <random>
#include <string>

namespace ai4e {

inline double wall_now() {
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}
// CLOCK_MONOTONIC: shared by every process of the node, so worker-side stage times
// (time.monotonic() in Python) are directly comparable with the scheduler's.
inline double mono_now() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// .NET DateTime.UtcNow.ToString() under the en-US culture: "M/d/yyyy h:mm:ss tt"
// (CacheConnectorUpsert.cs:102). Formatting is lazy (records keep the epoch seconds) and cached
// per second per thread, so a batch transition costs no formatting at all.
inline std::string dotnet_timestamp(double epoch_s) {
  thread_local int64_t cached_sec = INT64_MIN;
  thread_local std::string cached;
  const int64_t sec = static_cast<int64_t>(epoch_s);
  if (sec == cached_sec) return cached;
  std::time_t t = static_cast<std::time_t>(sec);
  std::tm tm{};
  gmtime_r(&t, &tm);
  int h12 = tm.tm_hour % 12;
  if (h12 == 0) h12 = 12;
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%d/%d/%04d %d:%02d:%02d %s", tm.tm_mon + 1, tm.tm_mday, tm.tm_year + 1900, h12,
                tm.tm_min, tm.tm_sec, tm.tm_hour < 12 ? "AM" : "PM");
  cached_sec = sec;
  cached = buf;
  return cached;
}

// Version-4 UUIDs from a per-store xorshift128+ (the reference uses Guid.NewGuid(),
// CacheConnectorUpsert.cs:92-100); hex formatting by table, no snprintf on the hot path.
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
    static const char* hex = "0123456789abcdef";
    std::string s(36, '-');
    int pos = 0;
    auto put = [&](uint64_t v, int nibbles) {
      for (int i = nibbles - 1; i >= 0; --i) {
        if (pos == 8 || pos == 13 || pos == 18 || pos == 23) ++pos;
        s[pos++] = hex[(v >> (4 * i)) & 0xF];
      }
    };
    put(a, 16);
    put(b, 16);
    return s;
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

inline void json_escape_into(std::string& out, const std::string& s) {
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
inline std::string absolute_path(const std::string& endpoint) {
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

}  // namespace ai4e
