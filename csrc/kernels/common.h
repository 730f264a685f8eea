// Shared helpers for the gfx950 (CDNA4, MI355X) kernels. Wave64 everywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

#define AI4E_API extern "C" __attribute__((visibility("default")))

// Error codes returned by the C ABI launchers (0 = ok).
enum { AI4E_OK = 0, AI4E_EINVAL = 1, AI4E_ELAUNCH = 2 };

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// Round-to-nearest-even float -> bf16 bits (NaN kept quiet): the compiler emits the gfx950 hardware
// conversion (v_cvt_pk_bf16_f32), one VALU op per PAIR of values instead of ~6 integer ops per value.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const bf16x2_t v = {static_cast<__bf16>(lo), static_cast<__bf16>(hi)};
  return __builtin_bit_cast(uint32_t, v);
}

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef short i16x2_t __attribute__((ext_vector_type(2)));

// ReLU on two packed bf16 (sign bit set -> 0; relu(round(x)) == round(relu(x))): one v_pk_max_i16.
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2_t, v), (i16x2_t){0, 0}));
}

// bf16x2(relu(lo, hi)): v_cvt_pk_bf16_f32 + v_pk_max_i16.
__device__ __forceinline__ uint32_t pack_relu_bf16x2(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return relu_bf16x2(__builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t)));
}

// (a + r.lo, b + r.hi) for two packed bf16 r without unpacking: v_dot2c_f32_bf16 against (1, 0) / (0, 1).
// The selector constants go through an opaque s_mov: hipcc otherwise encodes bf16x2 (1, 0) = 0x00003f80 as
// the inline constant 1.0, which the hardware reads as 0x3f800000 = (0, 1) (measured: wrong half added).
__device__ __forceinline__ uint32_t bf16_sel_lo() {
  uint32_t v;
  asm("s_mov_b32 %0, 0x3f80" : "=s"(v));
  return v;
}
__device__ __forceinline__ uint32_t bf16_sel_hi() {
  uint32_t v;
  asm("s_mov_b32 %0, 0x3f800000" : "=s"(v));
  return v;
}
__device__ __forceinline__ float add_bf16_lo(uint32_t r, float a) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, r), __builtin_bit_cast(bf16x2_t, bf16_sel_lo()),
                                         a, false);
}
__device__ __forceinline__ float add_bf16_hi(uint32_t r, float a) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, r), __builtin_bit_cast(bf16x2_t, bf16_sel_hi()),
                                         a, false);
}

// bf16x2 of two floats (v_cvt_pk_bf16_f32), no ReLU.
__device__ __forceinline__ uint32_t cvt_bf16x2(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// Conv epilogue for 8 consecutive channels: f (+ 8 packed-bf16 residual values) -> 8 bf16 (ReLU optional);
// the residual is added from its packed form (dot2), ReLU runs on the packed result.
__device__ __forceinline__ uint4 epilogue8_bf16(const float (&f)[8], bool has_res, const uint4& r, bool relu) {
  float g[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) g[k] = f[k];
  if (has_res) {
    g[0] = add_bf16_lo(r.x, g[0]); g[1] = add_bf16_hi(r.x, g[1]);
    g[2] = add_bf16_lo(r.y, g[2]); g[3] = add_bf16_hi(r.y, g[3]);
    g[4] = add_bf16_lo(r.z, g[4]); g[5] = add_bf16_hi(r.z, g[5]);
    g[6] = add_bf16_lo(r.w, g[6]); g[7] = add_bf16_hi(r.w, g[7]);
  }
  uint4 o = make_uint4(cvt_bf16x2(g[0], g[1]), cvt_bf16x2(g[2], g[3]), cvt_bf16x2(g[4], g[5]), cvt_bf16x2(g[6], g[7]));
  if (relu) {
    o.x = relu_bf16x2(o.x); o.y = relu_bf16x2(o.y); o.z = relu_bf16x2(o.z); o.w = relu_bf16x2(o.w);
  }
  return o;
}

__device__ __forceinline__ void unpack_bf16x2(uint32_t v, float& lo, float& hi) {
  lo = __uint_as_float(v << 16);
  hi = __uint_as_float(v & 0xffff0000u);
}

// ---- element-type traits of the K1 path: bf16 (default) or fp16 (F16 = true) activations and weights.
// Both feed the same-rate gfx950 MFMA (v_mfma_f32_16x16x32_bf16 / _f16, fp32 accumulate); fp16 keeps 10
// mantissa bits against bf16's 7 (the detector -> classifier ensemble runs its classifier in fp16).
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

template <bool F16>
__device__ __forceinline__ f32x4_t mfma_16x16x32(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                  0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <bool F16>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  if constexpr (F16) {
    const f32x2_t v = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_t));
  } else {
    return pack_bf16x2(lo, hi);
  }
}

template <bool F16>
__device__ __forceinline__ void unpack2(uint32_t v, float& lo, float& hi) {
  if constexpr (F16) {
    const f16x2_t h = __builtin_bit_cast(f16x2_t, v);
    lo = static_cast<float>(h[0]);
    hi = static_cast<float>(h[1]);
  } else {
    unpack_bf16x2(v, lo, hi);
  }
}

// f16 twins of add_bf16_lo/hi: (a + r.lo / r.hi) through v_dot2_f32_f16 against (1, 0) / (0, 1) (selectors
// through an opaque s_mov, as for bf16: hipcc would encode 0x3c00 as an inline float constant)
__device__ __forceinline__ uint32_t f16_sel_lo() {
  uint32_t v;
  asm("s_mov_b32 %0, 0x3c00" : "=s"(v));
  return v;
}
__device__ __forceinline__ uint32_t f16_sel_hi() {
  uint32_t v;
  asm("s_mov_b32 %0, 0x3c000000" : "=s"(v));
  return v;
}

// (a + r.lo / r.hi) of packed bf16 / fp16 r (dot2 against a (1, 0) / (0, 1) selector)
template <bool F16>
__device__ __forceinline__ float add_lo(uint32_t r, float a) {
  if constexpr (F16)
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, r), __builtin_bit_cast(f16x2_t, f16_sel_lo()), a, false);
  else
    return add_bf16_lo(r, a);
}
template <bool F16>
__device__ __forceinline__ float add_hi(uint32_t r, float a) {
  if constexpr (F16)
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, r), __builtin_bit_cast(f16x2_t, f16_sel_hi()), a, false);
  else
    return add_bf16_hi(r, a);
}
// relu(lo, hi) packed to bf16 / fp16 (sign-bit ReLU on the packed halves, valid for both formats)
template <bool F16>
__device__ __forceinline__ uint32_t pack_relu2(float lo, float hi) {
  return relu_bf16x2(pack2<F16>(lo, hi));
}

template <bool F16>
__device__ __forceinline__ uint4 epilogue8(const float (&f)[8], bool has_res, const uint4& r, bool relu) {
  if constexpr (!F16) {
    return epilogue8_bf16(f, has_res, r, relu);
  } else {
    float g[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = f[k];
    if (has_res) {
      const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        g[2 * q] = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, rr[q]), __builtin_bit_cast(f16x2_t, f16_sel_lo()),
                                          g[2 * q], false);
        g[2 * q + 1] = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, rr[q]),
                                              __builtin_bit_cast(f16x2_t, f16_sel_hi()), g[2 * q + 1], false);
      }
    }
    uint4 o = make_uint4(pack2<true>(g[0], g[1]), pack2<true>(g[2], g[3]), pack2<true>(g[4], g[5]),
                         pack2<true>(g[6], g[7]));
    if (relu) {  // sign bit set -> 0, as for bf16 (v_pk_max_i16)
      o.x = relu_bf16x2(o.x); o.y = relu_bf16x2(o.y); o.z = relu_bf16x2(o.z); o.w = relu_bf16x2(o.w);
    }
    return o;
  }
}

// Bijective XCD-aware remap of a linear workgroup id: the dispatcher places workgroup b on XCD
// (b % 8); give each XCD a contiguous run of logical tiles so neighbouring tiles (which share an
// operand panel) hit the same private L2 (cdna_hip_programming.md §5.5 T1).
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int xcd = b & 7, q = nb >> 3, r = nb & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

static inline int ai4e_cdiv(long a, long b) { return static_cast<int>((a + b - 1) / b); }
