// Short-sequence multi-head attention (BERT: S <= 128, head dim 64, no mask) on MFMA, forward and
// backward, reading the fused QKV projection [B, S, 3, H, 64] and writing O as [B, S, H * 64] —
// the layouts of the surrounding GEMMs, so no split / transpose copies exist on either side.
//
// Why: the ROCm SDPA kernels spend 17.6 us (forward) + 60 us (backward) per BERT attention call
// of [32 x 12 heads x 128 x 64] (profiles/r01_prof16_bert_fused_kernels.md, ~10 % of the step)
// for ~1.6 / 4 GFLOP and ~20 / 50 MB: a whole (batch, head) problem fits in one workgroup's LDS
// at S = 128, so one workgroup per (b, h) does everything with exact (non-online) softmax.
//
// MFMA: v_mfma_f32_32x32x16_bf16. Lane l (r = l & 31, h = l >> 5): A[r][8h + j], B[8h + j][r]
// (j = 0..7), C[(i & 3) + 8 (i >> 2) + 4h][r] (i = 0..15). Accumulator tiles are fed straight back
// as the B operand of the next product over their row index (k-step u of a tile uses registers
// 8u..8u+7, i.e. rows 16u + 8 (j >> 2) + 4h + (j & 3)); the other operand is read from LDS with
// that same k permutation.
//
// Forward, workgroup = S / 32 waves, wave w owns queries 32w..32w+31:
//   S^T = K Q^T            (A = K rows from LDS, B = Q rows from global)   -> keys in registers
//   exact softmax per query (max / sum over 4 x 16 registers + one lane^32 exchange), lse saved
//   O^T = V^T P^T          (A = V^T from LDS, B = P^T accumulators)
// Backward, wave w owns keys 32w..32w+31 (all queries):
//   S = Q K^T, dP = dO V^T (A = Q / dO rows from LDS, B = K / V rows from global)
//   P = exp(S scale - lse), dS = P (dP - D), D = rowsum(dO * O)
//   dV^T += dO^T P, dK^T += Q^T dS       (A = dO^T / Q^T from LDS, B = accumulators)
//   dS -> LDS; barrier; wave w then owns queries 32w..: dQ^T = K^T dS^T (A = K^T, B = dS rows)
#include <math.h>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kHD = 64;            // head dim
constexpr int kRS = kHD + 8;       // LDS row stride (elements) of [S][64] images: 144 B
__host__ __device__ constexpr int tstride(int S) { return S + 8; }   // [64][S] images

__device__ __forceinline__ f32x16 mfma(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8_t ld_frag(const uint16_t* p) {   // 16-B aligned
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}
// two runs of 4 contiguous elements (k permutation of an accumulator operand)
__device__ __forceinline__ bf16x8_t ld_frag_2x4(const uint16_t* p0, const uint16_t* p1) {
  const uint2 a = *reinterpret_cast<const uint2*>(p0);
  const uint2 b = *reinterpret_cast<const uint2*>(p1);
  return __builtin_bit_cast(bf16x8_t, make_uint4(a.x, a.y, b.x, b.y));
}
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
}
// registers 8u..8u+7 of an accumulator (times s) as a bf16 operand fragment
__device__ __forceinline__ bf16x8_t acc_frag(const f32x16& x, int u, float s) {
  const int o = 8 * u;
  return __builtin_bit_cast(bf16x8_t, make_uint4(pack2(x[o] * s, x[o + 1] * s),
                                                 pack2(x[o + 2] * s, x[o + 3] * s),
                                                 pack2(x[o + 4] * s, x[o + 5] * s),
                                                 pack2(x[o + 6] * s, x[o + 7] * s)));
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// accumulator row of register i for lane half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// ------------------------------------------------------------------------------------- forward
template <int NT>
__global__ __launch_bounds__(64 * NT) void attn_fwd_kernel(const bf16* __restrict__ qkv,
                                                          bf16* __restrict__ out,
                                                          float* __restrict__ lse, int H,
                                                          float scale) {
  constexpr int S = 32 * NT;
  constexpr int TS = tstride(S);
  __shared__ __attribute__((aligned(16))) uint16_t Ks[S * kRS];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[kHD * TS];
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int64_t rs = 3LL * H * kHD;                         // qkv row stride
  const uint16_t* base = reinterpret_cast<const uint16_t*>(qkv) + static_cast<int64_t>(b) * S * rs;
  const uint16_t* qg = base + hh * kHD;
  const uint16_t* kg = base + (H + hh) * kHD;
  const uint16_t* vg = base + (2 * H + hh) * kHD;
  for (int idx = threadIdx.x; idx < S * 8; idx += 64 * NT) {
    const int row = idx >> 3, c = (idx & 7) * 8;
    *reinterpret_cast<uint4*>(&Ks[row * kRS + c]) = *reinterpret_cast<const uint4*>(kg + row * rs + c);
    const uint4 v = *reinterpret_cast<const uint4*>(vg + row * rs + c);
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      Vt[(c + 2 * e) * TS + row] = static_cast<uint16_t>(w4[e] & 0xffffu);
      Vt[(c + 2 * e + 1) * TS + row] = static_cast<uint16_t>(w4[e] >> 16);
    }
  }
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int q = 32 * w + r;
  bf16x8_t qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qf[ks] = ld_frag(qg + q * rs + 16 * ks + 8 * h);
  __syncthreads();
  // S^T tiles: acc[kt][i] = S^T[key 32kt + acc_row(i, h)][query q]
  f32x16 acc[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    acc[kt] = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      acc[kt] = mfma(ld_frag(&Ks[(32 * kt + r) * kRS + 16 * ks + 8 * h]), qf[ks], acc[kt]);
  }
  // exact softmax over the S keys of query q (this lane: half of them; lane ^ 32: the rest)
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) m = fmaxf(m, acc[kt][i]);
  m = fmaxf(m, __shfl_xor(m, 32, 64)) * scale;
  float l = 0.f;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = __expf(fmaf(acc[kt][i], scale, -m));
      acc[kt][i] = p;
      l += p;
    }
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  if (h == 0) lse[static_cast<int64_t>(bh) * S + q] = m + __logf(l);
  // O^T = V^T P^T over 2 d-tiles
  f32x16 o[2] = {zero16(), zero16()};
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8_t pb = acc_frag(acc[kt], u, inv);
      const int k0 = 32 * kt + 16 * u + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const uint16_t* vr = &Vt[(32 * dt + r) * TS + k0];
        o[dt] = mfma(ld_frag_2x4(vr, vr + 8), pb, o[dt]);
      }
    }
  // O[q][d]: registers 4g..4g+3 are 4 consecutive d of query q
  uint16_t* og = reinterpret_cast<uint16_t*>(out) + (static_cast<int64_t>(b) * S + q) * H * kHD + hh * kHD;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * h;
      *reinterpret_cast<uint2*>(og + d) =
          make_uint2(pack2(o[dt][4 * g], o[dt][4 * g + 1]), pack2(o[dt][4 * g + 2], o[dt][4 * g + 3]));
    }
}

// ------------------------------------------------------------------------------------ backward
template <int NT>
__global__ __launch_bounds__(64 * NT) void attn_bwd_kernel(const bf16* __restrict__ qkv,
                                                          const bf16* __restrict__ out,
                                                          const bf16* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          bf16* __restrict__ dqkv, int H,
                                                          float scale) {
  constexpr int S = 32 * NT;
  constexpr int TS = tstride(S);
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Qs = smem;                    // [S][kRS]   Q rows
  uint16_t* dOs = Qs + S * kRS;           // [S][kRS]   dO rows
  uint16_t* Qt = dOs + S * kRS;           // [64][TS]   Q^T
  uint16_t* dOt = Qt + kHD * TS;          // [64][TS]   dO^T
  uint16_t* Kt = dOt + kHD * TS;          // [64][TS]   K^T
  uint16_t* dSs = Kt + kHD * TS;          // [S][TS]    dS (query rows, key columns)
  float* Dq = reinterpret_cast<float*>(dSs + S * TS);   // [S] rowsum(dO * O)
  float* Lq = Dq + S;                                    // [S] logsumexp
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int64_t rs = 3LL * H * kHD;
  const int64_t os = static_cast<int64_t>(H) * kHD;      // O / dO row stride
  const uint16_t* base = reinterpret_cast<const uint16_t*>(qkv) + static_cast<int64_t>(b) * S * rs;
  const uint16_t* qg = base + hh * kHD;
  const uint16_t* kg = base + (H + hh) * kHD;
  const uint16_t* vg = base + (2 * H + hh) * kHD;
  const uint16_t* og = reinterpret_cast<const uint16_t*>(out) + static_cast<int64_t>(b) * S * os + hh * kHD;
  const uint16_t* dog = reinterpret_cast<const uint16_t*>(dout) + static_cast<int64_t>(b) * S * os + hh * kHD;
  for (int idx = threadIdx.x; idx < S * 8; idx += 64 * NT) {
    const int row = idx >> 3, c = (idx & 7) * 8;
    const uint4 qv = *reinterpret_cast<const uint4*>(qg + row * rs + c);
    const uint4 dv = *reinterpret_cast<const uint4*>(dog + row * os + c);
    const uint4 kv = *reinterpret_cast<const uint4*>(kg + row * rs + c);
    const uint4 ov = *reinterpret_cast<const uint4*>(og + row * os + c);
    *reinterpret_cast<uint4*>(&Qs[row * kRS + c]) = qv;
    *reinterpret_cast<uint4*>(&dOs[row * kRS + c]) = dv;
    const uint32_t q4[4] = {qv.x, qv.y, qv.z, qv.w}, d4[4] = {dv.x, dv.y, dv.z, dv.w};
    const uint32_t k4[4] = {kv.x, kv.y, kv.z, kv.w}, o4[4] = {ov.x, ov.y, ov.z, ov.w};
    float dot = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      Qt[(c + 2 * e) * TS + row] = static_cast<uint16_t>(q4[e] & 0xffffu);
      Qt[(c + 2 * e + 1) * TS + row] = static_cast<uint16_t>(q4[e] >> 16);
      dOt[(c + 2 * e) * TS + row] = static_cast<uint16_t>(d4[e] & 0xffffu);
      dOt[(c + 2 * e + 1) * TS + row] = static_cast<uint16_t>(d4[e] >> 16);
      Kt[(c + 2 * e) * TS + row] = static_cast<uint16_t>(k4[e] & 0xffffu);
      Kt[(c + 2 * e + 1) * TS + row] = static_cast<uint16_t>(k4[e] >> 16);
      dot = fmaf(__uint_as_float(d4[e] << 16), __uint_as_float(o4[e] << 16), dot);
      dot = fmaf(__uint_as_float(d4[e] & 0xffff0000u), __uint_as_float(o4[e] & 0xffff0000u), dot);
    }
    // the 8 chunks of a row are 8 consecutive lanes (64 * NT is a multiple of 8)
    dot += __shfl_xor(dot, 1, 64);
    dot += __shfl_xor(dot, 2, 64);
    dot += __shfl_xor(dot, 4, 64);
    if ((idx & 7) == 0) {
      Dq[row] = dot;
      Lq[row] = lse[static_cast<int64_t>(bh) * S + row];
    }
  }
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int key = 32 * w + r;
  bf16x8_t kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = ld_frag(kg + key * rs + 16 * ks + 8 * h);
    vf[ks] = ld_frag(vg + key * rs + 16 * ks + 8 * h);
  }
  __syncthreads();
  f32x16 dk[2] = {zero16(), zero16()}, dv[2] = {zero16(), zero16()};
#pragma unroll
  for (int qt = 0; qt < NT; ++qt) {
    f32x16 s = zero16(), dp = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      s = mfma(ld_frag(&Qs[(32 * qt + r) * kRS + 16 * ks + 8 * h]), kf[ks], s);
      dp = mfma(ld_frag(&dOs[(32 * qt + r) * kRS + 16 * ks + 8 * h]), vf[ks], dp);
    }
    // s[i] = S[query 32qt + acc_row(i, h)][key]: P and dS in place
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = 32 * qt + acc_row(i, h);
      const float p = __expf(fmaf(s[i], scale, -Lq[qi]));
      s[i] = p;
      dp[i] = p * (dp[i] - Dq[qi]);
      dSs[qi * TS + key] = f2bf(dp[i]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8_t pb = acc_frag(s, u, 1.f);
      const bf16x8_t sb = acc_frag(dp, u, 1.f);
      const int q0 = 32 * qt + 16 * u + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const uint16_t* dor = &dOt[(32 * dt + r) * TS + q0];
        const uint16_t* qr = &Qt[(32 * dt + r) * TS + q0];
        dv[dt] = mfma(ld_frag_2x4(dor, dor + 8), pb, dv[dt]);
        dk[dt] = mfma(ld_frag_2x4(qr, qr + 8), sb, dk[dt]);
      }
    }
  }
  // dK (scaled) and dV: registers 4g..4g+3 are 4 consecutive d of this wave's key
  uint16_t* dbase = reinterpret_cast<uint16_t*>(dqkv) + static_cast<int64_t>(b) * S * rs;
  uint16_t* dkg = dbase + (H + hh) * kHD + key * rs;
  uint16_t* dvg = dbase + (2 * H + hh) * kHD + key * rs;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * h;
      *reinterpret_cast<uint2*>(dkg + d) =
          make_uint2(pack2(dk[dt][4 * g] * scale, dk[dt][4 * g + 1] * scale),
                     pack2(dk[dt][4 * g + 2] * scale, dk[dt][4 * g + 3] * scale));
      *reinterpret_cast<uint2*>(dvg + d) =
          make_uint2(pack2(dv[dt][4 * g], dv[dt][4 * g + 1]), pack2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]));
    }
  __syncthreads();   // every wave's dS columns are in LDS
  // dQ^T = K^T dS^T for queries 32w..32w+31 (this wave now owns queries)
  const int q = 32 * w + r;
  f32x16 dq[2] = {zero16(), zero16()};
#pragma unroll
  for (int ks = 0; ks < S / 16; ++ks) {
    const bf16x8_t sb = ld_frag(&dSs[q * TS + 16 * ks + 8 * h]);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) dq[dt] = mfma(ld_frag(&Kt[(32 * dt + r) * TS + 16 * ks + 8 * h]), sb, dq[dt]);
  }
  uint16_t* dqg = dbase + hh * kHD + q * rs;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * h;
      *reinterpret_cast<uint2*>(dqg + d) =
          make_uint2(pack2(dq[dt][4 * g] * scale, dq[dt][4 * g + 1] * scale),
                     pack2(dq[dt][4 * g + 2] * scale, dq[dt][4 * g + 3] * scale));
    }
}

template <int NT>
constexpr size_t bwd_smem() {
  return (2 * (32 * NT) * kRS + 3 * kHD * tstride(32 * NT) + (32 * NT) * tstride(32 * NT)) * 2 +
         2 * (32 * NT) * sizeof(float);
}

}  // namespace

hipError_t launch_attn_fwd(const void* qkv, void* out, float* lse, int B, int S, int H,
                           float scale, hipStream_t st) {
  if (B < 1 || H < 1 || S % 32 || S < 32 || S > 128) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(B * H));
  auto* q = reinterpret_cast<const bf16*>(qkv);
  auto* o = reinterpret_cast<bf16*>(out);
  switch (S / 32) {
    case 1: attn_fwd_kernel<1><<<grid, 64, 0, st>>>(q, o, lse, H, scale); break;
    case 2: attn_fwd_kernel<2><<<grid, 128, 0, st>>>(q, o, lse, H, scale); break;
    case 3: attn_fwd_kernel<3><<<grid, 192, 0, st>>>(q, o, lse, H, scale); break;
    default: attn_fwd_kernel<4><<<grid, 256, 0, st>>>(q, o, lse, H, scale); break;
  }
  return hipGetLastError();
}

hipError_t launch_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse,
                           void* dqkv, int B, int S, int H, float scale, hipStream_t st) {
  if (B < 1 || H < 1 || S % 32 || S < 32 || S > 128) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(B * H));
  auto* q = reinterpret_cast<const bf16*>(qkv);
  auto* o = reinterpret_cast<const bf16*>(out);
  auto* d = reinterpret_cast<const bf16*>(dout);
  auto* g = reinterpret_cast<bf16*>(dqkv);
#define CML_AB(NT)                                                                           \
  do {                                                                                       \
    static bool attr_set = false;                                                            \
    if (!attr_set) {                                                                         \
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(attn_bwd_kernel<NT>), \
                                         hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                         static_cast<int>(bwd_smem<NT>()));                  \
      if (e != hipSuccess) return e;                                                         \
      attr_set = true;                                                                       \
    }                                                                                        \
    attn_bwd_kernel<NT><<<grid, 64 * NT, bwd_smem<NT>(), st>>>(q, o, d, lse, g, H, scale);    \
  } while (0)
  switch (S / 32) {
    case 1: CML_AB(1); break;
    case 2: CML_AB(2); break;
    case 3: CML_AB(3); break;
    default: CML_AB(4); break;
  }
#undef CML_AB
  return hipGetLastError();
}

}  // namespace cml
