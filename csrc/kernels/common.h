// Shared device helpers for the consensus kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace cml {

constexpr int kWave = 64;

using bf16 = __hip_bfloat16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
// Round-to-nearest-even f32->bf16; hipcc lowers the cast to v_cvt_pk_bf16_f32 (keeps NaN a NaN).
__device__ __forceinline__ uint16_t f2bf(float f) {
  bf16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// ---------------------------------------------------------------- packed bf16 pairs (one VGPR)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

// {bf16(lo), bf16(hi)} in one v_cvt_pk_bf16_f32 (RNE, bit-identical to two f2bf); f2bf per value
// makes hipcc emit two conversions plus a shift and an or.
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  const f32x2 v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
// ReLU of two packed bf16 as one v_pk_max_i16: negative values (sign bit set) are negative as
// int16 and become +0; equal to rounding max(v, 0) except that a positive NaN stays NaN.
__device__ __forceinline__ uint32_t relu_pk(uint32_t w) {
  const i16x2 z = {0, 0};
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2, w), z));
}
// max(x sc + bi, 0) of the two bf16 in w (fp32 fma per element as v_pk_fma_f32, RNE to bf16):
// 5 VALU instructions per pair instead of 9.
__device__ __forceinline__ uint32_t bnrelu_pk(uint32_t w, f32x2 sc, f32x2 bi) {
  const f32x2 x = {__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
  const f32x2 y = __builtin_elementwise_fma(x, sc, bi);
  return relu_pk(pk_bf16(y.x, y.y));
}
// the two bf16 of w kept where their mask bits (bit 2i, 2i + 1 of `bits`) are set, else +0: v_bfe_i32
// sign-extends each bit to a full mask, v_bfi_b32 joins the halves (inline asm: hipcc otherwise
// turns the one-bit extracts into compare + select pairs)
template <int I>
__device__ __forceinline__ uint32_t mask_pk(uint32_t w, uint32_t bits) {
  uint32_t lo, hi, m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(lo) : "v"(bits), "i"(2 * I));
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(hi) : "v"(bits), "i"(2 * I + 1));
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(m) : "v"(0xffffu), "v"(lo), "v"(hi));
  return w & m;
}

// ---------------------------------------------------------------- vector loads of VEC elements
// VEC elements of T starting at p -> float out[VEC]. Vector widths: 16 B per lane where possible.
template <typename T, int VEC>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float (&out)[VEC]);

template <>
__device__ __forceinline__ void load_vec<bf16, 8>(const bf16* __restrict__ p, float (&o)[8]) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void load_vec<bf16, 4>(const bf16* __restrict__ p, float (&o)[4]) {
  uint2 u = *reinterpret_cast<const uint2*>(p);
  o[0] = __uint_as_float(u.x << 16);
  o[1] = __uint_as_float(u.x & 0xffff0000u);
  o[2] = __uint_as_float(u.y << 16);
  o[3] = __uint_as_float(u.y & 0xffff0000u);
}
template <>
__device__ __forceinline__ void load_vec<bf16, 2>(const bf16* __restrict__ p, float (&o)[2]) {
  uint32_t u = *reinterpret_cast<const uint32_t*>(p);
  o[0] = __uint_as_float(u << 16);
  o[1] = __uint_as_float(u & 0xffff0000u);
}
template <>
__device__ __forceinline__ void load_vec<bf16, 1>(const bf16* __restrict__ p, float (&o)[1]) {
  o[0] = bf2f(*reinterpret_cast<const uint16_t*>(p));
}
template <>
__device__ __forceinline__ void load_vec<float, 8>(const float* __restrict__ p, float (&o)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <>
__device__ __forceinline__ void load_vec<float, 4>(const float* __restrict__ p, float (&o)[4]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
}
template <>
__device__ __forceinline__ void load_vec<float, 2>(const float* __restrict__ p, float (&o)[2]) {
  float2 a = *reinterpret_cast<const float2*>(p);
  o[0] = a.x; o[1] = a.y;
}
template <>
__device__ __forceinline__ void load_vec<float, 1>(const float* __restrict__ p, float (&o)[1]) {
  o[0] = *p;
}

template <int VEC>
__device__ __forceinline__ void store_f32(float* __restrict__ p, const float (&v)[VEC]) {
  if constexpr (VEC % 4 == 0) {
#pragma unroll
    for (int i = 0; i < VEC; i += 4)
      *reinterpret_cast<float4*>(p + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) p[i] = v[i];
  }
}

template <int VEC>
__device__ __forceinline__ void store_bf16(bf16* __restrict__ p, const float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    uint4 u;
    u.x = f2bf(v[0]) | (uint32_t(f2bf(v[1])) << 16);
    u.y = f2bf(v[2]) | (uint32_t(f2bf(v[3])) << 16);
    u.z = f2bf(v[4]) | (uint32_t(f2bf(v[5])) << 16);
    u.w = f2bf(v[6]) | (uint32_t(f2bf(v[7])) << 16);
    *reinterpret_cast<uint4*>(p) = u;
  } else if constexpr (VEC == 4) {
    uint2 u;
    u.x = f2bf(v[0]) | (uint32_t(f2bf(v[1])) << 16);
    u.y = f2bf(v[2]) | (uint32_t(f2bf(v[3])) << 16);
    *reinterpret_cast<uint2*>(p) = u;
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<uint32_t*>(p) = f2bf(v[0]) | (uint32_t(f2bf(v[1])) << 16);
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) reinterpret_cast<uint16_t*>(p)[i] = f2bf(v[i]);
  }
}

// ---------------------------------------------------------------- Batcher odd-even merge sort
// Compile-time network over a[NP][VEC] of E (sorts every column independently, ascending).
// NP is a power of two; all indices fold to constants, so a[][] stays in VGPRs. E is float
// (v_min_f32/v_max_f32: one coordinate per instruction) or u16x2 order-preserving bf16 keys
// (v_pk_min_u16/v_pk_max_u16: two coordinates per instruction, half the VGPRs).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float vmin(float x, float y) { return fminf(x, y); }
__device__ __forceinline__ float vmax(float x, float y) { return fmaxf(x, y); }
__device__ __forceinline__ u16x2 vmin(u16x2 x, u16x2 y) { return __builtin_elementwise_min(x, y); }
__device__ __forceinline__ u16x2 vmax(u16x2 x, u16x2 y) { return __builtin_elementwise_max(x, y); }

template <typename E, int VEC>
__device__ __forceinline__ void cswap(E (&x)[VEC], E (&y)[VEC]) {
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    E lo = vmin(x[v], y[v]);
    E hi = vmax(x[v], y[v]);
    x[v] = lo;
    y[v] = hi;
  }
}

template <typename E, int NP, int VEC, int LO, int HI, int R>
struct OEMerge {
  static __device__ __forceinline__ void run(E (&a)[NP][VEC]) {
    constexpr int STEP = R * 2;
    if constexpr (STEP < HI - LO) {
      OEMerge<E, NP, VEC, LO, HI, STEP>::run(a);
      OEMerge<E, NP, VEC, LO + R, HI, STEP>::run(a);
#pragma unroll
      for (int i = LO + R; i < HI - R; i += STEP) cswap<E, VEC>(a[i], a[i + R]);
    } else {
      cswap<E, VEC>(a[LO], a[LO + R]);
    }
  }
};

template <typename E, int NP, int VEC, int LO, int HI>
struct OESort {
  static __device__ __forceinline__ void run(E (&a)[NP][VEC]) {
    if constexpr (HI - LO >= 1) {
      constexpr int MID = LO + (HI - LO) / 2;
      OESort<E, NP, VEC, LO, MID>::run(a);
      OESort<E, NP, VEC, MID + 1, HI>::run(a);
      OEMerge<E, NP, VEC, LO, HI, 1>::run(a);
    }
  }
};

template <typename E, int NP, int VEC>
__device__ __forceinline__ void sort_columns(E (&a)[NP][VEC]) {
  OESort<E, NP, VEC, 0, NP - 1>::run(a);
}

// ---------------------------------------------------------------- bf16 sort keys
// Two bf16 per 32-bit word -> two unsigned 16-bit keys whose integer order is the value order:
// the classic float radix key (negative: ~w, positive: w | 0x8000), rotated down by 127 so that
// the negative NaNs (keys 0..126) wrap above +inf; one v_pk_min_u16 against the +inf key then
// maps every NaN to +inf (the rules' NaN -> +inf convention). Exhaustively checked over all 65536
// bf16 patterns in tests/test_reference.py::test_bf16_key_roundtrip (numpy model of these ops).
constexpr unsigned short kKeyInf = 0xFF01;   // key of +inf: (0x7F80 | 0x8000) - 127

__device__ __forceinline__ u16x2 bf16_key(uint32_t w) {
  const u16x2 x = __builtin_bit_cast(u16x2, w);
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const u16x2 sgn = __builtin_bit_cast(u16x2, __builtin_bit_cast(s16x2, x) >> 15);
  const u16x2 k = (x ^ (sgn | static_cast<unsigned short>(0x8000))) - static_cast<unsigned short>(127);
  return vmin(k, u16x2{kKeyInf, kKeyInf});
}

__device__ __forceinline__ void bf16_unkey(u16x2 k, float& lo, float& hi) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const u16x2 uk = k + static_cast<unsigned short>(127);
  const u16x2 sgn = __builtin_bit_cast(u16x2, __builtin_bit_cast(s16x2, uk) >> 15);
  const uint32_t w = __builtin_bit_cast(uint32_t, uk ^ (~sgn | static_cast<unsigned short>(0x8000)));
  lo = __uint_as_float(w << 16);
  hi = __uint_as_float(w & 0xffff0000u);
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// ---------------------------------------------------------------- erf GELU
// erf by Abramowitz-Stegun 7.1.26 (|error| < 1.5e-7, far below bf16 resolution) instead of ocml's
// erff: 2 transcendentals (rcp, exp), and the exp(-x^2 / 2) term is shared with the derivative's
// density. Used by the GEMM epilogues (gemm.hip) and the standalone GELU backward (transformer.hip).
__device__ __forceinline__ float erf_as(float z, float e) {   // e = exp(-z^2)
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float r = fmaf(-p * t, e, 1.f);
  return copysignf(r, z);
}
__device__ __forceinline__ float gelu_f(float x) {
  const float z = x * 0.70710678118654752f;
  const float e = __expf(-z * z);
  return 0.5f * x * (1.f + erf_as(z, e));
}
// d gelu / dx = Phi(x) + x phi(x)
__device__ __forceinline__ float dgelu_f(float x) {
  const float z = x * 0.70710678118654752f;
  const float e = __expf(-z * z);
  return fmaf(0.5f, erf_as(z, e), 0.5f) + x * 0.3989422804014327f * e;
}

}  // namespace cml
