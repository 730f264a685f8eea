// Slot layout of a JPEG frame prepared for the on-GPU decoder: shared by the CPU preparer (csrc/core/jpeg_coef.h) and
// the HIP kernels (csrc/kernels/jpeg.hip). Plain data only, no host or device code.
#pragma once

#include <cstddef>
#include <cstdint>

namespace ai4e {

// GPU Huffman table: a 10-bit lookahead with the value bits folded in where code + value fit, plus the canonical-code
// slow path for longer codes. fast entry: bits 0-15 value (int16; for kind 1 the value size), 16-19 run, 20-24 bits
// consumed, 25-27 kind (0 value complete, 1 code only (value bits follow), 2 EOB, 3 ZRL, 4 longer code -> slow path).
static constexpr int kGpuLook = 10;
struct GpuHuff {
  uint32_t fast[1 << kGpuLook];
  int32_t maxcode[18];  // by code length (17: sentinel)
  int32_t valoff[18];   // symbol index = code + valoff[len]
  uint8_t vals[256];
};
static_assert(sizeof(GpuHuff) % 16 == 0, "GpuHuff alignment");

struct JpegScanHeader {
  uint32_t magic, width, height, ncomp, hmax, vmax, nblocks, scan_bytes;
  uint32_t comp[3][8];  // h, v, blocks_w, blocks_h, first block (planar), tq, td, ta
  uint32_t mcux, mcuy, bpm, restart, total_bits, pad[3];
  uint8_t blk_comp[16];  // block k of an MCU -> component
  uint8_t blk_dy[16];    // block k of an MCU -> row / column inside the component's MCU footprint
  uint8_t blk_dx[16];
  uint8_t pad2[16];
  uint16_t quant[4][64];  // natural order
  GpuHuff dc[2], ac[2];   // baseline tables 0 and 1 (a scan naming table 2 or 3 is decoded on the CPU)
};
static_assert(sizeof(JpegScanHeader) % 16 == 0, "JpegScanHeader alignment");
static constexpr uint32_t kJpegScanMagic = 0x3153434a;  // "JCS1"
static constexpr size_t kJpegScanPad = 64;

// A payload-ring slot that holds a prepared frame (instead of decoded pixels) ends with this trailer; `key` is the
// ring's secret (RingTail, written by the ring's creator), so a raw payload (which always fills its whole slot) can
// never be taken for one.
struct JpegSlotTrailer {
  uint64_t magic;
  uint64_t key;
  uint32_t used;  // prepared bytes at the start of the slot
  uint32_t pad;
  uint64_t pad2;
};
static_assert(sizeof(JpegSlotTrailer) == 32, "JpegSlotTrailer layout");
static constexpr uint64_t kJpegSlotMagic = 0x3153504a45344941ull;  // "AI4EJPS1"
// after the ring's slots: magic, key (0: the ring's workers do not decode prepared frames)
struct RingTail {
  uint64_t magic;
  uint64_t key;
  uint64_t pad[6];
};
static_assert(sizeof(RingTail) == 64, "RingTail layout");
static constexpr uint64_t kRingTailMagic = 0x474e495245344941ull;  // "AI4ERING"

// One frame of a decode batch (built by runtime/jpeg_gpu.py; device addresses).
struct JpegFrameDesc {
  uint64_t scan;          // JpegScanHeader + unstuffed scan (16-byte aligned)
  uint64_t coef;          // int16 [nblocks][64], MCU order, zigzag order; zero between batches (the IDCT clears it)
  uint64_t blen;          // uint8 [nblocks]: coefficients written per block (zigzag prefix; 0 between batches)
  uint64_t exit[2];       // uint64 [nthreads] span exit states (ping-pong over the sync passes)
  uint64_t chg[2];        // uint32 [nthreads] exit state changed in that pass
  uint64_t counts;        // int32 [nthreads][4]: blocks completed, DC sums -> exclusive prefixes
  uint64_t planes;        // uint8 component planes at the output scale
  uint64_t rows;          // uint8 [src_h][out_w][out_c] after the horizontal pass
  uint64_t out;           // uint8 [out_h][out_w][out_c]
  uint64_t hk, hb, vk, vb;  // PIL fixed-point resample coefficients int32 [n][ks] and bounds int32 [n][2]
  uint64_t status;        // uint32: bit 0 sync did not converge, bit 1 corrupt data
  int32_t nthreads, span_bits, hks, vks;
  int32_t ssize[3], plane_off[3], plane_pitch[3];
  int32_t src_w, src_h, out_w, out_h, out_c, kbase1, kbase2;
};
static_assert(sizeof(JpegFrameDesc) % 8 == 0, "JpegFrameDesc alignment");

}  // namespace ai4e
