// CPU emulation of the on-GPU Huffman decoder's passes (csrc/kernels/jpeg.hip) over one prepared frame: the same
// per-thread span decoder (csrc/core/jpeg_span.h) run thread by thread, pass by pass. Used by tests/test_jpeg_gpu.py to
// check the parallel decode (speculation, sync passes, prefix, write) against the sequential CPU decoder on any host.
//
//   jpeg_span_emul <prepared.bin> <span_bits> <coef_out.bin> [sync_passes]
//     -> prints "passes P unsynced0 U ... fixup F": without sync_passes the passes run until nothing changes; with it,
//        exactly that many run and the fix-up walk (huff_fixup_kernel) finishes the rest sequentially
#define AI4E_HD
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../csrc/core/jpeg_span.h"

using namespace ai4e;

static const uint8_t kZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                                41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                                30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> buf;
  uint8_t tmp[65536];
  size_t n;
  while ((n = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
  std::fclose(f);
  const int S = std::atoi(argv[2]);
  const int max_passes = argc > 4 ? std::atoi(argv[4]) : 1 << 30;
  const auto* H = reinterpret_cast<const JpegScanHeader*>(buf.data());
  if (H->magic != kJpegScanMagic) return 3;
  std::vector<uint32_t> lut(4 << kGpuLook);
  for (int t = 0; t < 2; ++t) {
    std::memcpy(&lut[t << kGpuLook], H->dc[t].fast, sizeof(H->dc[t].fast));
    std::memcpy(&lut[(2 + t) << kGpuLook], H->ac[t].fast, sizeof(H->ac[t].fast));
  }
  uint8_t nat[80], btab[16];
  for (int i = 0; i < 80; ++i) nat[i] = i < 64 ? kZz[i] : 63;
  for (uint32_t k = 0; k < H->bpm; ++k) {
    const int c = H->blk_comp[k];
    btab[k] = static_cast<uint8_t>(H->comp[c][6] | (H->comp[c][7] << 2) | (c << 4));
  }
  const size_t scan_words = (H->scan_bytes + kJpegScanPad) / 4;
  std::vector<uint32_t> words(scan_words);
  std::memcpy(words.data(), buf.data() + sizeof(JpegScanHeader), scan_words * 4);
  JSpanTables T{lut.data(), H->dc, btab, nat, words.data(), static_cast<uint32_t>(scan_words), static_cast<int>(H->bpm)};
  const uint32_t bits = H->total_bits;
  const int nt = static_cast<int>((bits + S - 1) / S);
  std::vector<uint64_t> ex[2] = {std::vector<uint64_t>(nt), std::vector<uint64_t>(nt)};
  std::vector<uint32_t> chg[2] = {std::vector<uint32_t>(nt), std::vector<uint32_t>(nt)};
  std::vector<int32_t> counts(4 * nt);
  auto end_of = [&](int t) { return std::min<uint32_t>(static_cast<uint32_t>(t + 1) * S, bits); };
  // pass 0
  for (int t = 0; t < nt; ++t) {
    JSpanResult r;
    jspan_decode<false>(T, static_cast<uint32_t>(t) * S, 0, 0, end_of(t), r);
    ex[0][t] = r.exit;
    chg[0][t] = 1;
    counts[4 * t] = r.nblk;
    for (int c = 0; c < 3; ++c) counts[4 * t + 1 + c] = r.dc[c];
  }
  int pass = 1, unsynced0 = -1;
  long redecoded = 0;
  for (;; ++pass) {
    const int in = (pass - 1) & 1, out = pass & 1;
    int changed = 0;
    ex[out][0] = ex[in][0];
    chg[out][0] = 0;
    for (int t = 1; t < nt; ++t) {
      if (pass >= 2 && !chg[in][t - 1]) {
        ex[out][t] = ex[in][t];
        chg[out][t] = 0;
        continue;
      }
      const uint64_t s = ex[in][t - 1];
      ++redecoded;
      JSpanResult r;
      jspan_decode<false>(T, jspan_pos(s), jspan_z(s), jspan_cp(s), end_of(t), r);
      ex[out][t] = r.exit;
      chg[out][t] = r.exit != ex[in][t];
      changed += chg[out][t];
      counts[4 * t] = r.nblk;
      for (int c = 0; c < 3; ++c) counts[4 * t + 1 + c] = r.dc[c];
    }
    if (pass == 1) unsynced0 = changed;
    if (!changed || pass >= max_passes) break;
  }
  const int last = pass & 1;
  // fix-up walk (huff_fixup_kernel)
  int fixed = 0;
  {
    bool dirty = false;
    for (int t = 1; t < nt; ++t) {
      if (!dirty && !chg[last][t - 1]) continue;
      chg[last][t - 1] = 0;
      const uint64_t s = ex[last][t - 1];
      JSpanResult r;
      jspan_decode<false>(T, jspan_pos(s), jspan_z(s), jspan_cp(s), end_of(t), r);
      dirty = r.exit != ex[last][t];
      ex[last][t] = r.exit;
      counts[4 * t] = r.nblk;
      for (int c = 0; c < 3; ++c) counts[4 * t + 1 + c] = r.dc[c];
      ++fixed;
    }
  }
  // exclusive prefix
  int32_t acc[4] = {0, 0, 0, 0};
  for (int t = 0; t < nt; ++t)
    for (int k = 0; k < 4; ++k) {
      const int32_t v = counts[4 * t + k];
      counts[4 * t + k] = acc[k];
      acc[k] += v;
    }
  const int32_t total = static_cast<int32_t>(H->nblocks);
  std::vector<int16_t> coef(static_cast<size_t>(total) * 64, 0);
  std::vector<uint8_t> blen(static_cast<size_t>(total), 0);
  int bad = 0;
  for (int t = 0; t < nt; ++t) {
    const uint64_t s = t ? ex[last][t - 1] : jspan_pack(0, 0, 0);
    JSpanResult r;
    jspan_decode<true>(T, jspan_pos(s), jspan_z(s), jspan_cp(s), end_of(t), r, coef.data(), counts[4 * t],
                       &counts[4 * t + 1], total, blen.data());
    bad += r.bad;
  }
  // zigzag -> natural (the kernels' IDCT does this on load); every coefficient must lie inside its block's length
  std::vector<int16_t> natural(coef.size(), 0);
  int beyond = 0;
  for (int32_t q = 0; q < total; ++q)
    for (int k = 0; k < 64; ++k) {
      const int16_t v = coef[static_cast<size_t>(q) * 64 + k];
      natural[static_cast<size_t>(q) * 64 + kZz[k]] = v;
      if (v && k >= blen[q]) ++beyond;
    }
  coef.swap(natural);
  bad += beyond;
  FILE* o = std::fopen(argv[3], "wb");
  std::fwrite(coef.data(), 2, coef.size(), o);
  std::fclose(o);
  std::printf("passes %d unsynced0 %d threads %d bad %d blocks %d redecoded %ld (%.2f spans/thread) fixup %d\n", pass,
              unsynced0, nt, bad, acc[0], redecoded, static_cast<double>(redecoded) / nt, fixed);
  return 0;
}
