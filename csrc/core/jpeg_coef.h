// JpegCoef — baseline JPEG entropy decoding to quantized DCT coefficients, for on-GPU reconstruction of camera-trap
// frames (survey §5.8(4) / §7.5.4; runtime/jpeg_gpu.py, csrc/kernels/jpeg.hip).
//
// A camera-trap client posts JPEG frames (the reference's detection API takes image files:
// APIs/Charts/camera-trap/detection-async/prod-values.yaml). Decoding them on CPU threads costs ~8 ms per 3-MP frame
// (PIL/libjpeg-turbo, DCT-domain 1/2 scale + resize), which caps one node far below its GPUs' detection rate. Here a
// CPU thread does only the serial part — Huffman decoding — and writes the coefficients compactly into the request's
// payload-ring slot; dequantization, the scaled IDCT, chroma upsampling, YCbCr -> RGB and the resize to the model input
// run as HIP kernels inside the worker's graph.
//
// Scope: baseline and extended-sequential Huffman JPEG (SOF0 / SOF1), 8-bit, 1 or 3 components, any sampling factors
// up to 2x2, restart intervals. Progressive / arithmetic / 12-bit files return an error (the caller falls back to the
// CPU decoder).
//
// Slot layout (little-endian):
//   u32 magic 'JCO1', u32 width, u32 height, u32 ncomp, u32 hmax, u32 vmax, u32 nblocks, u32 data_bytes
//   per component c < 3 (8 u32 each): h, v, blocks_w, blocks_h, first block index, quant table (0..3), 0, 0
//   u16 quant[4][64] (natural order)
//   u32 block[nblocks]  (a component's blocks row-major): byte offset into the data area | (nonzero count << 24)
//   data: per block, its nonzero coefficients as (u8 natural index, i16 value) triples, DC first when nonzero
//         (blocks are stored in MCU order, so a block's triples are found through its offset, not its neighbour's)
//
// prepare() is the GPU-Huffman variant (csrc/kernels/jpeg.hip decodes the entropy-coded data itself): the CPU parses
// the headers, builds GPU lookup tables and copies the scan with its 0xFF00 stuffing removed. Layout: JpegScanHeader,
// then the unstuffed scan bytes, then 64 bytes of 0xFF padding.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "jpeg_layout.h"

namespace ai4e {

struct JpegCoefHeader {
  uint32_t magic, width, height, ncomp, hmax, vmax, nblocks, data_bytes;
  uint32_t comp[3][8];
  uint16_t quant[4][64];
};
static_assert(sizeof(JpegCoefHeader) == 32 + 96 + 512, "JpegCoefHeader layout");
static constexpr uint32_t kJpegCoefMagic = 0x314f434a;  // "JCO1"


static const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Whether a prepared frame can be decoded on the GPU for a (out_h, out_w, out_c) model input bit-identically to the CPU
// path (runtime/decode.py decode_image: PIL's draft scale, libjpeg's per-component IDCT sizes with no upsampling left
// over, no reducing_gap pre-reduction in the resize). Mirrors runtime/jpeg_gpu.py plan_frame.
inline bool jpeg_gpu_plan_ok(const JpegScanHeader& H, int out_h, int out_w, int out_c) {
  if (out_c != 3 || out_h <= 0 || out_w <= 0 || H.magic != kJpegScanMagic) return false;
  const int W = static_cast<int>(H.width), Ht = static_cast<int>(H.height);
  int s = 1;
  if (W >= 2 * out_w || Ht >= 2 * out_h) {
    const int sc = std::min(W / out_w, Ht / out_h);
    s = sc >= 8 ? 8 : sc >= 4 ? 4 : sc >= 2 ? 2 : 1;
  }
  const int src_w = (W + s - 1) / s, src_h = (Ht + s - 1) / s;
  if (static_cast<int>(static_cast<double>(src_w) / out_w / 2.0) > 1 ||
      static_cast<int>(static_cast<double>(src_h) / out_h / 2.0) > 1)
    return false;
  const int min_s = 8 / s;
  for (uint32_t c = 0; c < H.ncomp; ++c) {
    const int h = static_cast<int>(H.comp[c][0]), v = static_cast<int>(H.comp[c][1]);
    const int hm = static_cast<int>(H.hmax), vm = static_cast<int>(H.vmax);
    int ss = min_s;
    while (ss < 8 && (hm * min_s) % (h * ss * 2) == 0 && (vm * min_s) % (v * ss * 2) == 0) ss *= 2;
    if ((hm * min_s) != h * ss || (vm * min_s) != v * ss) return false;  // would need upsampling
  }
  return true;
}

class JpegCoefDecoder {
 public:
  // Bytes the slot layout of a frame of at most `max_w` x `max_h` pixels needs in the worst case (every coefficient
  // nonzero, 4:4:4); callers size ring slots with a realistic fraction of it and handle kNoRoom.
  static size_t header_bytes(uint32_t nblocks) { return sizeof(JpegCoefHeader) + 4ull * nblocks; }

  enum Status { kOk = 0, kUnsupported = 1, kCorrupt = 2, kNoRoom = 3 };

  // Decode `data` into `out` (capacity `cap` bytes). Returns a Status; `*used` = bytes written.
  Status decode(const uint8_t* data, size_t len, uint8_t* out, size_t cap, size_t* used) {
    gpu_ = false;
    return parse(data, len, out, cap, used);
  }
  // Headers + GPU tables + unstuffed scan for the on-GPU Huffman decoder (JpegScanHeader layout).
  Status prepare(const uint8_t* data, size_t len, uint8_t* out, size_t cap, size_t* used) {
    gpu_ = true;
    return parse(data, len, out, cap, used);
  }

 private:
  bool gpu_ = false;
  Status parse(const uint8_t* data, size_t len, uint8_t* out, size_t cap, size_t* used) {
    p_ = data;
    end_ = data + len;
    *used = 0;
    restart_ = 0;
    have_frame_ = false;
    for (auto& t : dc_) t.ok = false;
    for (auto& t : ac_) t.ok = false;
    if (len < 4 || p_[0] != 0xFF || p_[1] != 0xD8) return kCorrupt;
    p_ += 2;
    for (;;) {
      int m = next_marker();
      if (m < 0) return kCorrupt;
      if (m == 0xD9) return kCorrupt;  // EOI before any scan
      if (m == 0xC0 || m == 0xC1) {
        if (!read_sof()) return kUnsupported;
        continue;
      }
      if ((m >= 0xC2 && m <= 0xC3) || (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xCC)) return kUnsupported;
      if (m == 0xC4) {
        if (!read_dht()) return kCorrupt;
        continue;
      }
      if (m == 0xDB) {
        if (!read_dqt()) return kCorrupt;
        continue;
      }
      if (m == 0xDD) {
        if (seg_len() != 4) return kCorrupt;
        restart_ = (p_[2] << 8) | p_[3];
        p_ += 4;
        continue;
      }
      if (m == 0xDA) {
        if (!have_frame_) return kCorrupt;
        return gpu_ ? emit_scan(out, cap, used) : scan(out, cap, used);
      }
      // APPn, COM, anything else with a length: skip (an Adobe APP14 with transform 0 marks RGB / CMYK samples: the
      // YCbCr reconstruction does not apply, CPU path)
      const int l = seg_len();
      if (m == 0xEE && l >= 14 && p_ + l <= end_ && std::memcmp(p_ + 2, "Adobe", 5) == 0 && p_[13] == 0)
        return kUnsupported;
      if (l < 2 || p_ + l > end_) return kCorrupt;
      p_ += l;
    }
  }

  // 9-bit lookahead with the value folded in where the code and its value bits fit in 9 bits (most coefficients):
  // kind 0 = coefficient (run, val, len = code + value bits), 1 = code only (val = value size, len = code length),
  // 2 = end of block, 3 = run of 16 zeros, 4 = code longer than 9 bits
  struct Fast {  // 4 bytes: a 2048-entry table is 8 KB (both AC tables stay in L1)
    int16_t val;
    uint8_t run_len;  // run << 4 ... run in the high nibble is not enough for len 0..27: see len/kind below
    uint8_t len_kind;  // len (5 bits) | kind << 5
  };
  static inline int f_len(const Fast& f) { return f.len_kind & 31; }
  static inline int f_kind(const Fast& f) { return f.len_kind >> 5; }
  static inline int f_run(const Fast& f) { return f.run_len; }
  static constexpr int kLook = 11;  // lookahead bits (11: 96 % of this file's coefficients decode in one lookup)
  struct Huff {
    bool ok = false;
    Fast fast[1 << kLook];
    uint16_t look[1 << kLook];  // lookahead: (length << 8) | symbol, 0 = longer code
    int32_t maxcode[18];
    int32_t valptr[17];
    int32_t mincode[17];
    uint8_t vals[256];
    uint8_t counts[16];
  };
  struct Comp {
    int id, h, v, tq, td, ta, bw, bh, first;
  };

  const uint8_t* p_;
  const uint8_t* end_;
  int restart_ = 0;
  bool have_frame_ = false;
  uint32_t width_ = 0, height_ = 0;
  int ncomp_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
  Comp comp_[3];
  uint16_t quant_[4][64] = {};
  Huff dc_[4], ac_[4];

  int seg_len() const { return (end_ - p_ >= 2) ? ((p_[0] << 8) | p_[1]) : -1; }
  int next_marker() {
    while (p_ < end_ && *p_ != 0xFF) ++p_;  // (garbage between segments)
    while (p_ < end_ && *p_ == 0xFF) ++p_;
    if (p_ >= end_) return -1;
    return *p_++;
  }
  bool read_sof() {
    const int l = seg_len();
    if (l < 8 || p_ + l > end_) return false;
    const uint8_t* s = p_ + 2;
    if (s[0] != 8) return false;  // 8-bit only
    height_ = (s[1] << 8) | s[2];
    width_ = (s[3] << 8) | s[4];
    ncomp_ = s[5];
    if ((ncomp_ != 1 && ncomp_ != 3) || width_ == 0 || height_ == 0 || l != 8 + 3 * ncomp_) return false;
    hmax_ = vmax_ = 1;
    for (int c = 0; c < ncomp_; ++c) {
      comp_[c].id = s[6 + 3 * c];
      comp_[c].h = s[7 + 3 * c] >> 4;
      comp_[c].v = s[7 + 3 * c] & 15;
      comp_[c].tq = s[8 + 3 * c];
      if (comp_[c].h < 1 || comp_[c].h > 2 || comp_[c].v < 1 || comp_[c].v > 2 || comp_[c].tq > 3) return false;
      hmax_ = std::max(hmax_, comp_[c].h);
      vmax_ = std::max(vmax_, comp_[c].v);
    }
    if (ncomp_ == 3 && comp_[0].id == 'R' && comp_[1].id == 'G' && comp_[2].id == 'B') return false;  // RGB JPEG
    mcux_ = static_cast<int>((width_ + 8 * hmax_ - 1) / (8 * hmax_));
    mcuy_ = static_cast<int>((height_ + 8 * vmax_ - 1) / (8 * vmax_));
    int first = 0;
    for (int c = 0; c < ncomp_; ++c) {
      comp_[c].bw = mcux_ * comp_[c].h;
      comp_[c].bh = mcuy_ * comp_[c].v;
      comp_[c].first = first;
      first += comp_[c].bw * comp_[c].bh;
    }
    if (ncomp_ == 1) {  // a single-component scan is not interleaved: blocks cover the image exactly
      comp_[0].h = comp_[0].v = hmax_ = vmax_ = 1;
      mcux_ = static_cast<int>((width_ + 7) / 8);
      mcuy_ = static_cast<int>((height_ + 7) / 8);
      comp_[0].bw = mcux_;
      comp_[0].bh = mcuy_;
    }
    have_frame_ = true;
    p_ += l;
    return true;
  }
  bool read_dqt() {
    const int l = seg_len();
    if (l < 2 || p_ + l > end_) return false;
    const uint8_t* s = p_ + 2;
    const uint8_t* e = p_ + l;
    while (s < e) {
      const int pq = *s >> 4, tq = *s & 15;
      ++s;
      if (tq > 3 || s + 64 * (pq ? 2 : 1) > e) return false;
      for (int k = 0; k < 64; ++k) {
        quant_[tq][kZigzag[k]] = pq ? static_cast<uint16_t>((s[2 * k] << 8) | s[2 * k + 1]) : s[k];
      }
      s += 64 * (pq ? 2 : 1);
    }
    p_ += l;
    return true;
  }
  bool read_dht() {
    const int l = seg_len();
    if (l < 2 || p_ + l > end_) return false;
    const uint8_t* s = p_ + 2;
    const uint8_t* e = p_ + l;
    while (s < e) {
      if (s + 17 > e) return false;
      const int tc = *s >> 4, th = *s & 15;
      if (tc > 1 || th > 3) return false;
      Huff& h = tc ? ac_[th] : dc_[th];
      const uint8_t* counts = s + 1;
      int total = 0;
      for (int i = 0; i < 16; ++i) total += counts[i];
      if (total > 256 || s + 17 + total > e) return false;
      std::memcpy(h.vals, s + 17, static_cast<size_t>(total));
      std::memcpy(h.counts, counts, 16);
      // canonical codes
      int code = 0, k = 0;
      std::memset(h.look, 0, sizeof(h.look));
      for (int len = 1; len <= 16; ++len) {
        h.valptr[len] = k;
        h.mincode[len] = code;
        for (int i = 0; i < counts[len - 1]; ++i) {
          if (len <= kLook) {  // every kLook-bit pattern starting with this code
            const int shift = kLook - len;
            for (int j = 0; j < (1 << shift); ++j) h.look[(code << shift) | j] = static_cast<uint16_t>((len << 8) | h.vals[k]);
          }
          ++code;
          ++k;
        }
        h.maxcode[len] = counts[len - 1] ? code - 1 : -1;
        code <<= 1;
      }
      h.maxcode[17] = 0x7fffffff;
      for (int pfx = 0; pfx < (1 << kLook); ++pfx) {
        Fast& f = h.fast[pfx];
        std::memset(&f, 0, sizeof(f));
        const uint16_t e = h.look[pfx];
        auto set = [&](int kind, int len) { f.len_kind = static_cast<uint8_t>(len | (kind << 5)); };
        if (!e) {
          set(4, 0);
          continue;
        }
        const int L = e >> 8, sym = e & 0xFF;
        const int r = tc ? sym >> 4 : 0, sz = tc ? sym & 15 : sym;
        if (tc && sz == 0) {
          set(r == 15 ? 3 : 2, L);
          continue;
        }
        f.run_len = static_cast<uint8_t>(r);
        if (sz == 0) {  // DC difference 0
          set(0, L);
          f.val = 0;
        } else if (L + sz <= kLook) {
          set(0, L + sz);
          f.val = static_cast<int16_t>(extend((pfx >> (kLook - L - sz)) & ((1 << sz) - 1), sz));
        } else {
          set(1, L);
          f.val = static_cast<int16_t>(sz);
        }
      }
      h.ok = true;
      s += 17 + total;
    }
    p_ += l;
    return true;
  }

  // ---- bit reader over the entropy-coded segment (0xFF00 stuffing; a marker ends the data: zeros after it). A local
  // of scan() (never the decoder's members): the coefficient stores go through a uint8_t pointer, which may alias any
  // member, so member state would be reloaded from memory after every store.
  struct BitReader {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t bits = 0;
    int nbits = 0;
    bool hit_marker = false;

    inline void fill() {
      // fast path: the next 8 bytes hold no 0xFF (no stuffing, no marker): take as many whole bytes as fit at once
      if (!hit_marker && end - p >= 8 && nbits <= 56) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        const uint64_t x = ~w;
        if (((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull) == 0) {
          const int k = (64 - nbits) >> 3;  // 1..8 bytes
          const int top = nbits + 8 * k;    // bits valid after the load (<= 64)
          const uint64_t be = __builtin_bswap64(w);
          bits |= (be >> nbits) & (top >= 64 ? ~0ull : ~(~0ull >> top));
          nbits += 8 * k;
          p += k;
          return;
        }
      }
      while (nbits <= 56) {
        uint64_t b = 0;
        if (!hit_marker && p < end) {
          b = *p;
          if (b == 0xFF) {
            const uint8_t n = p + 1 < end ? p[1] : 0xD9;
            if (n == 0x00) {
              p += 2;
            } else {
              hit_marker = true;  // a marker: leave it for the caller
              b = 0;
            }
          } else {
            ++p;
          }
        }
        bits |= b << (56 - nbits);
        nbits += 8;
      }
    }
    inline int peek() const { return static_cast<int>(bits >> (64 - kLook)); }
    inline void skip(int n) {
      bits <<= n;
      nbits -= n;
    }
    inline int getbits(int n) {  // n in 1..16
      const int v = static_cast<int>(bits >> (64 - n));
      skip(n);
      return v;
    }
    inline int decode_sym(const Huff& h) {
      if (nbits < 16) fill();
      const uint16_t e = h.look[peek()];
      if (e) {
        skip(e >> 8);
        return e & 0xFF;
      }
      int len = kLook + 1;
      int code = static_cast<int>(bits >> (64 - len));
      while (len <= 16 && code > h.maxcode[len]) {
        ++len;
        code = static_cast<int>(bits >> (64 - len));
      }
      if (len > 16) return -1;
      skip(len);
      return h.vals[h.valptr[len] + code - h.mincode[len]];
    }
    bool restart() {  // byte-align and step over the RSTn marker
      bits = 0;
      nbits = 0;
      hit_marker = false;
      while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
      if (p + 1 >= end) return false;
      p += 2;
      return true;
    }
  };
  static inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

  static void gpu_table(const Huff& h, bool ac, GpuHuff* g) {
    std::memset(g, 0, sizeof(GpuHuff));
    std::memcpy(g->vals, h.vals, 256);
    int code = 0, k = 0;
    for (int len = 1; len <= 16; ++len) {
      g->valoff[len] = k - code;
      for (int i = 0; i < h.counts[len - 1]; ++i, ++code, ++k) {
        if (len > kGpuLook) continue;
        const int sym = h.vals[k];
        const int r = ac ? sym >> 4 : 0, sz = ac ? sym & 15 : sym;
        const int shift = kGpuLook - len;
        for (int j = 0; j < (1 << shift); ++j) {
          const int pfx = (code << shift) | j;
          uint32_t kind, n, val = 0;
          if (ac && sz == 0) {
            kind = r == 15 ? 3 : 2;
            n = static_cast<uint32_t>(len);
          } else if (len + sz <= kGpuLook) {
            kind = 0;
            n = static_cast<uint32_t>(len + sz);
            val = sz ? static_cast<uint16_t>(static_cast<int16_t>(extend((pfx >> (shift - sz)) & ((1 << sz) - 1), sz)))
                     : 0u;
          } else {
            kind = 1;
            n = static_cast<uint32_t>(len);
            val = static_cast<uint32_t>(sz);
          }
          g->fast[pfx] = val | (static_cast<uint32_t>(ac ? r : 0) << 16) | (n << 20) | (kind << 25);
        }
      }
      g->maxcode[len] = h.counts[len - 1] ? code - 1 : -1;
      code <<= 1;
    }
    g->maxcode[17] = 0x7fffffff;
    for (int pfx = 0; pfx < (1 << kGpuLook); ++pfx)
      if (!g->fast[pfx]) g->fast[pfx] = 4u << 25;  // longer code (or none): slow path
  }

  Status emit_scan(uint8_t* out, size_t cap, size_t* used) {
    const int l = seg_len();
    if (l < 6 || p_ + l > end_) return kCorrupt;
    const uint8_t* s = p_ + 2;
    const int ns = s[0];
    if (ns != ncomp_ || l != 6 + 2 * ns) return kUnsupported;
    if (restart_) return kUnsupported;  // restart intervals: the CPU path
    for (int i = 0; i < ns; ++i) {
      const int cid = s[1 + 2 * i];
      int c = -1;
      for (int k = 0; k < ncomp_; ++k)
        if (comp_[k].id == cid) c = k;
      if (c != i) return kUnsupported;
      comp_[c].td = s[2 + 2 * i] >> 4;
      comp_[c].ta = s[2 + 2 * i] & 15;
      if (comp_[c].td > 3 || comp_[c].ta > 3 || !dc_[comp_[c].td].ok || !ac_[comp_[c].ta].ok) return kCorrupt;
      if (comp_[c].td > 1 || comp_[c].ta > 1) return kUnsupported;  // (the GPU layout carries tables 0 and 1)
    }
    if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0) return kUnsupported;
    p_ += l;
    if (cap < sizeof(JpegScanHeader) + kJpegScanPad) return kNoRoom;
    auto* H = reinterpret_cast<JpegScanHeader*>(out);
    std::memset(H, 0, offsetof(JpegScanHeader, dc));
    H->magic = kJpegScanMagic;
    H->width = width_;
    H->height = height_;
    H->ncomp = static_cast<uint32_t>(ncomp_);
    H->hmax = static_cast<uint32_t>(hmax_);
    H->vmax = static_cast<uint32_t>(vmax_);
    uint32_t nblocks = 0, bpm = 0;
    for (int c = 0; c < ncomp_; ++c) {
      uint32_t* w = H->comp[c];
      w[0] = static_cast<uint32_t>(comp_[c].h);
      w[1] = static_cast<uint32_t>(comp_[c].v);
      w[2] = static_cast<uint32_t>(comp_[c].bw);
      w[3] = static_cast<uint32_t>(comp_[c].bh);
      w[4] = static_cast<uint32_t>(comp_[c].first);
      w[5] = static_cast<uint32_t>(comp_[c].tq);
      w[6] = static_cast<uint32_t>(comp_[c].td);
      w[7] = static_cast<uint32_t>(comp_[c].ta);
      nblocks += static_cast<uint32_t>(comp_[c].bw * comp_[c].bh);
      for (int by = 0; by < comp_[c].v; ++by)
        for (int bx = 0; bx < comp_[c].h; ++bx) {
          H->blk_comp[bpm] = static_cast<uint8_t>(c);
          H->blk_dy[bpm] = static_cast<uint8_t>(by);
          H->blk_dx[bpm] = static_cast<uint8_t>(bx);
          ++bpm;
        }
    }
    H->nblocks = nblocks;
    H->mcux = static_cast<uint32_t>(mcux_);
    H->mcuy = static_cast<uint32_t>(mcuy_);
    H->bpm = bpm;
    std::memcpy(H->quant, quant_, sizeof(quant_));
    for (int t = 0; t < 2; ++t) {
      if (dc_[t].ok) gpu_table(dc_[t], false, &H->dc[t]);
      else std::memset(&H->dc[t], 0, sizeof(GpuHuff));
      if (ac_[t].ok) gpu_table(ac_[t], true, &H->ac[t]);
      else std::memset(&H->ac[t], 0, sizeof(GpuHuff));
    }
    // unstuff: copy runs between 0xFF bytes; FF 00 -> FF; any other marker ends the entropy-coded data
    uint8_t* dst = out + sizeof(JpegScanHeader);
    uint8_t* const dend = out + cap - kJpegScanPad;
    const uint8_t* p = p_;
    for (;;) {
      const uint8_t* ff = static_cast<const uint8_t*>(std::memchr(p, 0xFF, static_cast<size_t>(end_ - p)));
      const uint8_t* run_end = ff ? ff : end_;
      const size_t n = static_cast<size_t>(run_end - p);
      if (n > static_cast<size_t>(dend - dst)) return kNoRoom;
      std::memcpy(dst, p, n);
      dst += n;
      if (!ff || ff + 1 >= end_) break;
      if (ff[1] == 0x00) {
        if (dst >= dend) return kNoRoom;
        *dst++ = 0xFF;
        p = ff + 2;
        continue;
      }
      if (ff[1] == 0xFF) {  // fill bytes before a marker
        p = ff + 1;
        continue;
      }
      break;  // a marker (EOI, or RSTn in a file without DRI: treated as the end)
    }
    const size_t nbytes = static_cast<size_t>(dst - (out + sizeof(JpegScanHeader)));
    std::memset(dst, 0xFF, kJpegScanPad);
    H->scan_bytes = static_cast<uint32_t>(nbytes);
    H->total_bits = static_cast<uint32_t>(std::min<size_t>(nbytes * 8, 0xFFFFFFF0u));
    *used = sizeof(JpegScanHeader) + nbytes + kJpegScanPad;
    return kOk;
  }

  Status scan(uint8_t* out, size_t cap, size_t* used) {
    const int l = seg_len();
    if (l < 6 || p_ + l > end_) return kCorrupt;
    const uint8_t* s = p_ + 2;
    const int ns = s[0];
    if (ns != ncomp_ || l != 6 + 2 * ns) return kUnsupported;  // non-interleaved multi-scan files: CPU path
    for (int i = 0; i < ns; ++i) {
      const int cid = s[1 + 2 * i];
      int c = -1;
      for (int k = 0; k < ncomp_; ++k)
        if (comp_[k].id == cid) c = k;
      if (c != i) return kUnsupported;
      comp_[c].td = s[2 + 2 * i] >> 4;
      comp_[c].ta = s[2 + 2 * i] & 15;
      if (comp_[c].td > 3 || comp_[c].ta > 3 || !dc_[comp_[c].td].ok || !ac_[comp_[c].ta].ok) return kCorrupt;
    }
    if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0) return kUnsupported;  // Ss, Se, Ah/Al
    p_ += l;

    uint32_t nblocks = 0;
    for (int c = 0; c < ncomp_; ++c) nblocks += static_cast<uint32_t>(comp_[c].bw * comp_[c].bh);
    const size_t hdr = header_bytes(nblocks);
    if (cap < hdr) return kNoRoom;
    auto* H = reinterpret_cast<JpegCoefHeader*>(out);
    std::memset(H, 0, sizeof(JpegCoefHeader));
    H->magic = kJpegCoefMagic;
    H->width = width_;
    H->height = height_;
    H->ncomp = static_cast<uint32_t>(ncomp_);
    H->hmax = static_cast<uint32_t>(hmax_);
    H->vmax = static_cast<uint32_t>(vmax_);
    H->nblocks = nblocks;
    for (int c = 0; c < ncomp_; ++c) {
      uint32_t* w = H->comp[c];
      w[0] = static_cast<uint32_t>(comp_[c].h);
      w[1] = static_cast<uint32_t>(comp_[c].v);
      w[2] = static_cast<uint32_t>(comp_[c].bw);
      w[3] = static_cast<uint32_t>(comp_[c].bh);
      w[4] = static_cast<uint32_t>(comp_[c].first);
      w[5] = static_cast<uint32_t>(comp_[c].tq);
    }
    std::memcpy(H->quant, quant_, sizeof(quant_));
    uint32_t* offs = reinterpret_cast<uint32_t*>(out + sizeof(JpegCoefHeader));
    uint8_t* data = out + hdr;
    const size_t dcap = cap - hdr;
    size_t dpos = 0;

    BitReader br{p_, end_};
    int pred[3] = {0, 0, 0};
    const int nmcu = mcux_ * mcuy_;
    int todo = restart_;
    for (int m = 0; m < nmcu; ++m) {
      if (restart_ && todo == 0) {
        if (!br.restart()) return kCorrupt;
        pred[0] = pred[1] = pred[2] = 0;
        todo = restart_;
      }
      const int my = m / mcux_, mx = m - my * mcux_;
      for (int c = 0; c < ncomp_; ++c) {
        const Comp& C = comp_[c];
        const Huff& dc = dc_[C.td];
        const Huff& ac = ac_[C.ta];
        for (int by = 0; by < C.v; ++by)
          for (int bx = 0; bx < C.h; ++bx) {
            const int row = my * C.v + by, col = mx * C.h + bx;
            const uint32_t bi = static_cast<uint32_t>(C.first + row * C.bw + col);
            if (dcap - dpos < 3 * 64 || dpos >= (1u << 24)) return kNoRoom;
            const size_t b0 = dpos;
            // DC
            if (br.nbits < 32) br.fill();
            int diff;
            {
              const Fast& f = dc.fast[br.peek()];
              if (f_kind(f) == 0) {
                br.skip(f_len(f));
                diff = f.val;
              } else {
                const int t = f_kind(f) == 1 ? (br.skip(f_len(f)), f.val) : br.decode_sym(dc);
                if (t < 0 || t > 11) return kCorrupt;
                diff = 0;
                if (t) {
                  if (br.nbits < t) br.fill();
                  diff = extend(br.getbits(t), t);
                }
              }
            }
            pred[c] += diff;
            if (pred[c]) {
              data[dpos] = 0;
              const int16_t v = static_cast<int16_t>(pred[c]);
              std::memcpy(data + dpos + 1, &v, 2);
              dpos += 3;
            }
            // AC
            for (int k = 1; k < 64;) {
              if (br.nbits < 32) br.fill();
              const Fast& f = ac.fast[br.peek()];
              int16_t v;
              if (f_kind(f) == 0) {  // the common case: code and value bits in one lookup
                br.skip(f_len(f));
                k += f_run(f);
                v = f.val;
              } else if (f_kind(f) == 2) {  // EOB
                br.skip(f_len(f));
                break;
              } else if (f_kind(f) == 3) {  // ZRL
                br.skip(f_len(f));
                k += 16;
                continue;
              } else {
                int r, sz;
                if (f_kind(f) == 1) {
                  br.skip(f_len(f));
                  r = f_run(f);
                  sz = f.val;
                } else {
                  const int rs = br.decode_sym(ac);
                  if (rs < 0) return kCorrupt;
                  r = rs >> 4;
                  sz = rs & 15;
                  if (sz == 0) {
                    if (r != 15) break;  // EOB
                    k += 16;
                    continue;
                  }
                }
                k += r;
                if (br.nbits < sz) br.fill();
                v = static_cast<int16_t>(extend(br.getbits(sz), sz));
              }
              if (k > 63) return kCorrupt;
              data[dpos] = kZigzag[k];
              std::memcpy(data + dpos + 1, &v, 2);
              dpos += 3;
              ++k;
            }
            offs[bi] = static_cast<uint32_t>(b0) | (static_cast<uint32_t>((dpos - b0) / 3) << 24);
          }
      }
      --todo;
    }
    H->data_bytes = static_cast<uint32_t>(dpos);
    *used = hdr + dpos;
    return kOk;
  }
};

}  // namespace ai4e
