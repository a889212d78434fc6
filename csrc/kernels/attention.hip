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
//   O^T = V^T P^T          (A = V^T by transposed reads of the V row image, B = P^T accumulators)
// Backward (attn_bwd2_kernel), wave w owns keys 32w..32w+31 (all queries):
//   S = Q K^T, dP = dO V^T (A = Q / dO rows from LDS, B = K rows from LDS / V rows from global)
//   P = exp(S scale - lse), dS = P (dP - D), D = rowsum(dO * O)
//   dV^T += dO^T P, dK^T += Q^T dS       (A = dO^T / Q^T by transposed reads, B = accumulators)
//   dS^T -> LDS (over Q, dO); barrier; wave w then owns queries 32w..:
//   dQ^T = K^T dS^T        (both operands by transposed reads)
// Transposed operands come from ds_read_b64_tr_b16 on the same swizzled row images that the row
// reads use (sw64 / sw256e below), so staging is 16-B loads + ds_write_b128 only. The first
// backward (attn_bwd_kernel, CML_ATTN_BWD_V1=1) kept [64][S] transposed copies built with 2-B LDS
// writes: 122 KB of LDS, one workgroup per CU.
#include <math.h>

#include <cstdlib>

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

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ int sw64(int r, int c) {
  const int k = (r >> 1) & 7;
  return r * 128 + 16 * (c ^ (((k & 1) << 2) | (k >> 1)));
}
__device__ __forceinline__ int sw64e(int r, int col) { return sw64(r, col >> 3) + 2 * (col & 7); }
__device__ __forceinline__ int sw256e(int r, int col) {
  return r * 256 + 16 * ((col >> 3) ^ (((r & 3) << 2) | ((r >> 2) & 3))) + 2 * (col & 7);
}
__device__ __forceinline__ uint2 tr_rd(const char* p) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p)));
}
// X^T operand fragment of an [rows = k][64 cols = m] image (lane: m = m0 + (lane & 31)):
// elements 0-3 = X[ka + q][m], 4-7 = X[kb + q][m] (q = 0..3)
__device__ __forceinline__ bf16x8_t trfrag64(const char* img, int ka, int kb, int m0, int lane) {
  const int q = (lane >> 2) & 3, col = m0 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const uint2 lo = tr_rd(img + sw64e(ka + q, col)), hi = tr_rd(img + sw64e(kb + q, col));
  return __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
}
__device__ __forceinline__ bf16x8_t trfrag256(const char* img, int ka, int kb, int m0, int lane) {
  const int q = (lane >> 2) & 3, col = m0 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const uint2 lo = tr_rd(img + sw256e(ka + q, col)), hi = tr_rd(img + sw256e(kb + q, col));
  return __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

// ------------------------------------------------------------------------------------- forward
template <int NT>
__global__ __launch_bounds__(64 * NT) void attn_fwd_kernel(const bf16* __restrict__ qkv,
                                                          bf16* __restrict__ out,
                                                          float* __restrict__ lse, int H,
                                                          float scale) {
  constexpr int S = 32 * NT;
  // K and V as swizzled [S][64] row images (sw64); V^T is read by ds_read_b64_tr_b16
  __shared__ __attribute__((aligned(16))) char Ks[S * 128];
  __shared__ __attribute__((aligned(16))) char Vs[S * 128];
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int64_t rs = 3LL * H * kHD;                         // qkv row stride
  const uint16_t* base = reinterpret_cast<const uint16_t*>(qkv) + static_cast<int64_t>(b) * S * rs;
  const uint16_t* qg = base + hh * kHD;
  const uint16_t* kg = base + (H + hh) * kHD;
  const uint16_t* vg = base + (2 * H + hh) * kHD;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int q = 32 * w + r;
  bf16x8_t qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qf[ks] = ld_frag(qg + q * rs + 16 * ks + 8 * h);
#pragma unroll
  for (int it = 0; it < S * 8 / (64 * NT); ++it) {
    const int idx = threadIdx.x + it * 64 * NT;
    const int row = idx >> 3, c = idx & 7;
    const uint4 kv = *reinterpret_cast<const uint4*>(kg + row * rs + 8 * c);
    const uint4 vv = *reinterpret_cast<const uint4*>(vg + row * rs + 8 * c);
    *reinterpret_cast<uint4*>(Ks + sw64(row, c)) = kv;
    *reinterpret_cast<uint4*>(Vs + sw64(row, c)) = vv;
  }
  __syncthreads();
  // S^T tiles: acc[kt][i] = S^T[key 32kt + acc_row(i, h)][query q]
  f32x16 acc[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    acc[kt] = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      acc[kt] = mfma(*reinterpret_cast<const bf16x8_t*>(Ks + sw64(32 * kt + r, 2 * ks + h)), qf[ks],
                     acc[kt]);
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
  // O^T = V^T P^T over 2 d-tiles (V^T fragments by transposed reads of the V rows)
  f32x16 o[2] = {zero16(), zero16()};
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8_t pb = acc_frag(acc[kt], u, inv);
      const int k0 = 32 * kt + 16 * u + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) o[dt] = mfma(trfrag64(Vs, k0, k0 + 8, 32 * dt, lane), pb, o[dt]);
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

// ------------------------------------------------------------------------- backward, version 2
// Same products as attn_bwd_kernel, with every transposed operand read by ds_read_b64_tr_b16 from
// the ROW image it is also read from by rows (no [64][S] transposed copies, no 2-B LDS writes):
//   Q, dO, K   [S][64] images with 128-B rows; chunk c of row r at 16 (c ^ f((r >> 1) & 7)),
//              f(k) = ((k & 1) << 2) | (k >> 1): the 16 rows of a ds_read_b128 lane group hit 16
//              distinct bank slots (f is a bijection), and the 4 rows of a transposed read
//              (rows 4n .. 4n + 3, 4 chunks) too (rows 4n + 2, 4n + 3 flip bit 2 of the chunk)
//   dS^T       [S keys][S queries] with 256-B rows (chunk ^ ((row & 3) << 2 | (row >> 2) & 3)):
//              each lane writes 4 consecutive queries of its key (8 B) after phase 1 (dS is held
//              in registers as bf16 meanwhile) into the space of Q and dO, which are dead by then.
// LDS 3 S 128 B + 2 S 4 B (49 KB at S = 128, was 122 KB): two workgroups per CU, so one
// workgroup's load phase overlaps the other's MFMAs.
template <int NT>
constexpr size_t bwd2_smem() { return 3 * (32 * NT) * 128 + 2 * (32 * NT) * sizeof(float); }

template <int NT>
__global__ __launch_bounds__(64 * NT, 2) void attn_bwd2_kernel(const bf16* __restrict__ qkv,
                                                              const bf16* __restrict__ out,
                                                              const bf16* __restrict__ dout,
                                                              const float* __restrict__ lse,
                                                              bf16* __restrict__ dqkv, int H,
                                                              float scale) {
  constexpr int S = 32 * NT;
  extern __shared__ __attribute__((aligned(16))) char smem2[];
  char* Qs = smem2;                    // [S][64]
  char* dOs = Qs + S * 128;            // [S][64]
  char* Ks = dOs + S * 128;            // [S][64]
  char* dSt = smem2;                   // [S keys][S queries], over Q and dO after phase 1
  float* Dq = reinterpret_cast<float*>(Ks + S * 128);   // [S] rowsum(dO * O)
  float* Lq = Dq + S;                                   // [S] logsumexp
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int64_t rs = 3LL * H * kHD;
  const int64_t os = static_cast<int64_t>(H) * kHD;
  const uint16_t* base = reinterpret_cast<const uint16_t*>(qkv) + static_cast<int64_t>(b) * S * rs;
  const uint16_t* qg = base + hh * kHD;
  const uint16_t* kg = base + (H + hh) * kHD;
  const uint16_t* vg = base + (2 * H + hh) * kHD;
  const uint16_t* og = reinterpret_cast<const uint16_t*>(out) + static_cast<int64_t>(b) * S * os + hh * kHD;
  const uint16_t* dog = reinterpret_cast<const uint16_t*>(dout) + static_cast<int64_t>(b) * S * os + hh * kHD;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int key = 32 * w + r;
  // this wave's V rows (B operand of dP), issued first so their latency overlaps the staging
  bf16x8_t vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) vf[ks] = ld_frag(vg + key * rs + 16 * ks + 8 * h);
  // staging: S rows x 8 chunks of Q, dO, K (16-B loads and ds_write_b128), D = rowsum(dO * O)
#pragma unroll
  for (int it = 0; it < S * 8 / (64 * NT); ++it) {
    const int idx = threadIdx.x + it * 64 * NT;
    const int row = idx >> 3, c = idx & 7;
    const uint4 qv = *reinterpret_cast<const uint4*>(qg + row * rs + 8 * c);
    const uint4 dv = *reinterpret_cast<const uint4*>(dog + row * os + 8 * c);
    const uint4 kv = *reinterpret_cast<const uint4*>(kg + row * rs + 8 * c);
    const uint4 ov = *reinterpret_cast<const uint4*>(og + row * os + 8 * c);
    *reinterpret_cast<uint4*>(Qs + sw64(row, c)) = qv;
    *reinterpret_cast<uint4*>(dOs + sw64(row, c)) = dv;
    *reinterpret_cast<uint4*>(Ks + sw64(row, c)) = kv;
    const uint32_t d4[4] = {dv.x, dv.y, dv.z, dv.w}, o4[4] = {ov.x, ov.y, ov.z, ov.w};
    float dot = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      dot = fmaf(__uint_as_float(d4[e] << 16), __uint_as_float(o4[e] << 16), dot);
      dot = fmaf(__uint_as_float(d4[e] & 0xffff0000u), __uint_as_float(o4[e] & 0xffff0000u), dot);
    }
    dot += __shfl_xor(dot, 1, 64);   // the 8 chunks of a row are 8 consecutive lanes
    dot += __shfl_xor(dot, 2, 64);
    dot += __shfl_xor(dot, 4, 64);
    if (c == 0) {
      Dq[row] = dot;
      Lq[row] = lse[static_cast<int64_t>(bh) * S + row];
    }
  }
  __syncthreads();
  bf16x8_t kf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    kf[ks] = *reinterpret_cast<const bf16x8_t*>(Ks + sw64(key, 2 * ks + h));
  f32x16 dk[2] = {zero16(), zero16()}, dv[2] = {zero16(), zero16()};
  uint2 dsr[NT][4];   // dS of this wave's key as bf16: registers 4g..4g+3 of query tile qt
#pragma unroll
  for (int qt = 0; qt < NT; ++qt) {
    f32x16 s = zero16(), dp = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int qr = 32 * qt + r;
      s = mfma(*reinterpret_cast<const bf16x8_t*>(Qs + sw64(qr, 2 * ks + h)), kf[ks], s);
      dp = mfma(*reinterpret_cast<const bf16x8_t*>(dOs + sw64(qr, 2 * ks + h)), vf[ks], dp);
    }
    // s[i] = S[query 32 qt + acc_row(i, h)][key]: P and dS in place
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = 32 * qt + acc_row(i, h);
      const float p = __expf(fmaf(s[i], scale, -Lq[qi]));
      s[i] = p;
      dp[i] = p * (dp[i] - Dq[qi]);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
      dsr[qt][g] = make_uint2(pack2(dp[4 * g], dp[4 * g + 1]), pack2(dp[4 * g + 2], dp[4 * g + 3]));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8_t pb = acc_frag(s, u, 1.f);
      const bf16x8_t sb = __builtin_bit_cast(
          bf16x8_t, make_uint4(dsr[qt][2 * u].x, dsr[qt][2 * u].y, dsr[qt][2 * u + 1].x,
                               dsr[qt][2 * u + 1].y));
      const int q0 = 32 * qt + 16 * u + 4 * h;   // k rows of registers 8u..8u+7: q0 + {0-3, 8-11}
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        dv[dt] = mfma(trfrag64(dOs, q0, q0 + 8, 32 * dt, lane), pb, dv[dt]);
        dk[dt] = mfma(trfrag64(Qs, q0, q0 + 8, 32 * dt, lane), sb, dk[dt]);
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
  __syncthreads();   // every wave is done with Q and dO: dS^T goes over them
#pragma unroll
  for (int qt = 0; qt < NT; ++qt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<uint2*>(dSt + sw256e(key, 32 * qt + 8 * g + 4 * h)) = dsr[qt][g];
  __syncthreads();
  // dQ^T = K^T dS^T for queries 32 w .. 32 w + 31 (this wave now owns queries)
  const int q = 32 * w + r;
  f32x16 dq[2] = {zero16(), zero16()};
#pragma unroll
  for (int ks = 0; ks < S / 16; ++ks) {
    const int k0 = 16 * ks + 8 * h;
    const bf16x8_t sb = trfrag256(dSt, k0, k0 + 4, 32 * w, lane);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) dq[dt] = mfma(trfrag64(Ks, k0, k0 + 4, 32 * dt, lane), sb, dq[dt]);
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
#define CML_AB2(NT)                                                                          \
  do {                                                                                       \
    static bool attr_set = false;                                                            \
    if (!attr_set) {                                                                         \
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(attn_bwd2_kernel<NT>), \
                                         hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                         static_cast<int>(bwd2_smem<NT>()));                 \
      if (e != hipSuccess) return e;                                                         \
      attr_set = true;                                                                       \
    }                                                                                        \
    attn_bwd2_kernel<NT><<<grid, 64 * NT, bwd2_smem<NT>(), st>>>(q, o, d, lse, g, H, scale);  \
  } while (0)
  static const bool v1 = [] {
    const char* e = std::getenv("CML_ATTN_BWD_V1");
    return e && e[0] == '1';
  }();
  if (v1) {
    switch (S / 32) {
      case 1: CML_AB(1); break;
      case 2: CML_AB(2); break;
      case 3: CML_AB(3); break;
      default: CML_AB(4); break;
    }
  } else {
    switch (S / 32) {
      case 1: CML_AB2(1); break;
      case 2: CML_AB2(2); break;
      case 3: CML_AB2(3); break;
      default: CML_AB2(4); break;
    }
  }
#undef CML_AB
#undef CML_AB2
  return hipGetLastError();
}

}  // namespace cml
