// The per-thread core of the on-GPU Huffman decoder (csrc/kernels/jpeg.hip): decode the symbols whose codes start in
// one span of the entropy-coded bits, from a given decoder state.
//
// Parallel decoding (self-synchronising Huffman codes): the scan's bits are cut into spans of `span_bits`; thread t
// owns the symbols whose codes START in span t. Its entry state (bit position of the first such code, coefficient
// index z, block index inside the MCU) is the exit state of thread t-1, which is unknown until t-1 is decoded. So:
//   pass 0: thread t guesses (t * span_bits, z 0, block 0) and decodes its span; a wrong guess usually falls into
//           step with the true symbol stream within a few dozen bits, so its exit state is usually already right;
//   pass k: thread t re-decodes from thread t-1's exit state of pass k-1 (only if that state changed in pass k-1);
//           when no exit state changes, every state is the sequential decoder's (induction from thread 0, which always
//           starts at the true state);
//   prefix: exclusive sums over threads of (blocks completed, DC differences per component) give each thread its
//           first block index and DC predictors;
//   write:  every thread decodes its span once more from its (now exact) entry state and stores the coefficients
//           (zigzag order, DC undifferenced) into the dense [block][64] array, with each block's written length.
// Host and device share this code: the CPU build (tests/native/jpeg_span_emul.cpp) runs the same passes sequentially
// against the CPU decoder's output. Needs AI4E_HD (__host__ __device__ for hipcc, empty for g++) defined by the
// includer.
#pragma once

#include <cstdint>

#include "jpeg_layout.h"

// Address space of the decoder's global-memory operands: the kernels define it as the global space, so the scan words,
// slow-path tables and coefficient stores compile to global_* instructions, which count only in vmcnt. As flat_*
// operations they also count in lgkmcnt, and every LDS table lookup's lgkmcnt(0) wait then waited for the prefetched
// scan word too (the prefetch hid nothing). Host builds: the default address space.
#ifndef AI4E_GAS
#define AI4E_GAS
#endif

namespace ai4e {

// exit state: bit position (32) | z (8) | block in MCU (8) | valid (bit 63)
AI4E_HD inline uint64_t jspan_pack(uint32_t pos, int z, int cp) {
  return static_cast<uint64_t>(pos) | (static_cast<uint64_t>(z) << 32) | (static_cast<uint64_t>(cp) << 40) |
         (1ull << 63);
}
AI4E_HD inline uint32_t jspan_pos(uint64_t s) { return static_cast<uint32_t>(s); }
AI4E_HD inline int jspan_z(uint64_t s) { return static_cast<int>((s >> 32) & 0xFF); }
AI4E_HD inline int jspan_cp(uint64_t s) { return static_cast<int>((s >> 40) & 0xFF); }

struct JSpanTables {
  const uint32_t* lut;     // [4][1 << kGpuLook]: DC tables 0-1, AC tables 0-1 (LDS on the GPU)
  const AI4E_GAS GpuHuff* huff;  // dc[2], ac[2] of the JpegScanHeader (slow path: codes longer than kGpuLook)
  const uint8_t* blk_tab;  // per MCU block: dc table | ac table << 2 | component << 4
  const uint8_t* natural;  // zigzag -> natural order, 80 entries (64..79 -> 63, as libjpeg's jpeg_natural_order)
  const AI4E_GAS uint32_t* words;  // the unstuffed scan as 32-bit words (big-endian bytes), padded with 0xFF
  uint32_t nwords;
  int bpm;
};

struct JSpanResult {
  uint64_t exit;
  int32_t nblk;   // blocks completed
  int32_t dc[3];  // DC differences summed per component
  int32_t bad;    // invalid codes met (0 for a valid stream decoded from a true state)
};

// kWrite: store coefficients (coef: int16 [total][64] in ZIGZAG order, natural positions being the IDCT's business;
// q0 = index of the block the span starts in, pred = DC predictors at the span's start) and, for every block the span
// finishes, blen[q] = length of the written zigzag prefix (the span that started the block may have written its first
// coefficients: the entry state's z bounds them); stops after the last block.
template <bool kWrite>
AI4E_HD inline void jspan_decode(const JSpanTables& T, uint32_t pos, int z, int cp, uint32_t end, JSpanResult& r,
                                 AI4E_GAS int16_t* coef = nullptr, int32_t q0 = 0, const int32_t* pred_in = nullptr,
                                 int32_t total = 0, AI4E_GAS uint8_t* blen = nullptr) {
  r.exit = jspan_pack(pos, z, cp);
  if (kWrite && q0 >= total) {  // a span past the last block (the scan's padding)
    r.nblk = 0;
    r.dc[0] = r.dc[1] = r.dc[2] = 0;
    r.bad = 0;
    return;
  }
  const int32_t pred0 = kWrite ? pred_in[0] : 0, pred1 = kWrite ? pred_in[1] : 0, pred2 = kWrite ? pred_in[2] : 0;
  int32_t dc0 = 0, dc1 = 0, dc2 = 0;
  r.nblk = 0;
  r.bad = 0;
  // 64-bit window, MSB = the bit at `pos`; nb valid bits
  uint32_t wi = pos >> 5;
  // raw (big-endian) scan word; the index is clamped, not the loaded value, so nothing consumes a load before its
  // bits are needed (reads stay inside the 64-byte 0xFF pad: a span never decodes more than a code past its end)
  auto raw = [&](uint32_t i) -> uint32_t { return T.words[i < T.nwords ? i : T.nwords - 1]; };
  auto word = [&](uint32_t i) -> uint64_t { return static_cast<uint64_t>(__builtin_bswap32(raw(i))); };
  uint64_t buf = (word(wi) << 32) << (pos & 31);
  int nb = 32 - static_cast<int>(pos & 31);
  ++wi;
  buf |= word(wi) << (32 - nb);
  nb += 32;
  ++wi;
  // the next word is loaded one refill ahead and byte-swapped only when used: its global-memory latency overlaps the
  // ~5 symbols decoded from the current window instead of stalling the refill
  uint32_t nxt = raw(wi);
  int bt = T.blk_tab[cp];
  int32_t q = q0;
  int lz = z > 0 ? z - 1 : 0;  // highest zigzag index written in the current block (bound for the part before us)
  while (pos < end) {
    if (nb < 32) {
      buf |= static_cast<uint64_t>(__builtin_bswap32(nxt)) << (32 - nb);
      nb += 32;
      nxt = raw(++wi);
    }
    const int dct = bt & 1, act = 2 + ((bt >> 2) & 1), comp = (bt >> 4) & 3;
    const int tab = z == 0 ? dct : act;
    const uint32_t e = T.lut[(tab << kGpuLook) | static_cast<uint32_t>(buf >> (64 - kGpuLook))];
    int kind = static_cast<int>(e >> 25);
    int n = static_cast<int>((e >> 20) & 31);
    int run = static_cast<int>((e >> 16) & 15);
    int val = static_cast<int16_t>(e & 0xFFFF);
    int sz = kind == 1 ? val : 0;
    if (kind == 4 || n == 0) {  // code longer than the lookahead
      const AI4E_GAS GpuHuff& h = T.huff[tab];
      int len = kGpuLook + 1;
      int code = static_cast<int>(buf >> (64 - len));
      while (len <= 16 && code > h.maxcode[len]) {
        ++len;
        code = static_cast<int>(buf >> (64 - len));
      }
      if (len > 16) {  // no such code: a wrong (speculative) state, or a corrupt stream
        ++r.bad;
        buf <<= 1;
        nb -= 1;
        pos += 1;
        z = 0;
        continue;
      }
      const int sym = h.vals[(code + h.valoff[len]) & 0xFF];
      n = len;
      if (z == 0) {
        kind = 1;
        run = 0;
        sz = sym > 15 ? 15 : sym;
      } else {
        run = sym >> 4;
        sz = sym & 15;
        kind = sz ? 1 : (run == 15 ? 3 : 2);
      }
    }
    // code (+ folded value) bits, then the value bits of a kind-1 symbol
    buf <<= n;
    nb -= n;
    pos += static_cast<uint32_t>(n);
    if (kind == 1) {
      if (sz) {
        if (nb < sz) {  // (never: >= 16 bits remain after a code of <= 16)
          buf |= static_cast<uint64_t>(__builtin_bswap32(nxt)) << (32 - nb);
          nb += 32;
          nxt = raw(++wi);
        }
        const int v = static_cast<int>(buf >> (64 - sz));
        val = v < (1 << (sz - 1)) ? v - (1 << sz) + 1 : v;
        buf <<= sz;
        nb -= sz;
        pos += static_cast<uint32_t>(sz);
      } else {
        val = 0;
      }
    }
    if (z == 0) {  // DC difference (selects, not an indexed array: the array would live in scratch on the GPU)
      dc0 += comp == 0 ? val : 0;
      dc1 += comp == 1 ? val : 0;
      dc2 += comp == 2 ? val : 0;
      if (kWrite) {
        const int p = comp == 0 ? pred0 + dc0 : (comp == 1 ? pred1 + dc1 : pred2 + dc2);
        coef[static_cast<int64_t>(q) * 64] = static_cast<int16_t>(p);
        lz = 0;
      }
      z = 1;
    } else if (kind == 2) {
      z = 64;
    } else if (kind == 3) {
      z += 16;
    } else {
      z += run;
      if (kWrite) {  // zigzag positions past 63 land on 63, as libjpeg's jpeg_natural_order[64..79]
        lz = z > 63 ? 63 : z;
        coef[static_cast<int64_t>(q) * 64 + lz] = static_cast<int16_t>(val);
      }
      z += 1;
    }
    if (z >= 64) {
      if (kWrite) blen[q] = static_cast<uint8_t>(lz + 1);
      z = 0;
      ++r.nblk;
      ++q;
      cp = cp + 1 == T.bpm ? 0 : cp + 1;
      bt = T.blk_tab[cp];
      if (kWrite && q >= total) break;
    }
  }
  r.exit = jspan_pack(pos, z, cp);
  r.dc[0] = dc0;
  r.dc[1] = dc1;
  r.dc[2] = dc2;
}

}  // namespace ai4e
