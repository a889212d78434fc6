// Flash attention for head dim 128 with grouped-query heads (Llama-3-8B: 32 q / 8 kv heads,
// causal, S up to 8192), forward and backward on v_mfma_f32_32x32x16_bf16, gfx950 / CDNA4.
//
// Layouts (the neighbours' layouts, so nothing is transposed or copied around the kernels):
//   q [B, H, S, 128], k / v [B, KV, S, 128]     head-major, from the QKV split + RoPE kernel
//   o [B, S, H, 128]                            = the output projection's input rows
//   lse [B, H, S] fp32                          log2-domain: m + log2(l) of the scores times
//                                               scale * log2(e) (the kernels use exp2)
//   dsum [B, H, S] fp32                         D = rowsum(dO * O), written by the dQ kernel
//   dq [B, H, S, 128]; dk / dv [B, H, S, 128]   per QUERY head: the group sum over the H / KV
//                                               heads of a kv head is fused into the RoPE
//                                               backward (launch_rope_bwd, grp > 1)
//
// MFMA 32x32x16 bf16: lane l (r = l & 31, h = l >> 5) holds A[r][8h + j], B[8h + j][r]
// (j = 0..7) and C[(i & 3) + 8 (i >> 2) + 4h][r] (i = 0..15). Every product is oriented so that
// the next product sums over the accumulator's ROW index, so accumulators are fed back as B
// operands with no lane movement (registers 8u..8u+7 = rows 16u + 8 (j >> 2) + 4h + (j & 3));
// the other operand is then read from LDS in that same k order with ds_read_b64_tr_b16.
//
// Forward (fa_fwd_kernel), workgroup = 4 waves x 32 queries, K / V in 64-key tiles:
//   S^T = K Q^T          A = K rows (LDS), B = Q^T (this lane's query row, registers)
//                        -> each lane holds 16 keys of ONE query: the softmax row statistics are
//                           lane-local (one lane ^ 32 exchange for the tile max)
//   online softmax in the log2 domain, O^T rescaled by a lane-local alpha
//   O^T += V^T P^T        A = V^T (transposed reads of the V rows), B = P^T accumulators
// Backward, two kernels (no atomics: deterministic, and the dQ kernel needs no fp32 scratch):
//   fa_dq_kernel   (query-major, as the forward)  S^T = K Q^T, dP^T = V dO^T, D = rowsum(dO O)
//                  computed in the prologue, dS^T = P^T (dP^T - D), dQ^T += K^T dS^T
//   fa_dkdv_kernel (key-major, 4 waves x 32 keys) S = Q K^T, dP = dO V^T (Q / dO rows from LDS,
//                  K / V of the lane's key in registers), dV^T += dO^T P, dK^T += Q^T dS
// Staging: 16-B global_load_lds (LDS-DMA) into two buffers; [rows][128] bf16 images with 256-B
// rows, chunk ch of row r at 16 (ch ^ ((r & 3) << 2 | (r >> 2) & 3)): conflict-free for the
// ds_read_b128 row reads and the transposed reads of the 32x32x16 operands. LDS-DMA writes
// lane-linear, so the swizzle is applied to each lane's SOURCE address. One barrier per tile:
// wait + barrier (tile t landed, tile t - 1 consumed by every wave), then the DMA of tile t + 1
// is issued into the other buffer and runs under tile t's MFMAs.
// Work order: workgroup ids are remapped so that the 8 groups of ids that share an XCD take
// contiguous (batch, head) ranges (the 4 query heads of a kv head read its K / V from one L2),
// heaviest causal blocks first. Causal tiles that are fully masked for a wave are skipped
// wave-uniformly (the barrier count stays uniform).
//
// Replaces ROCm SDPA's AOTriton kernels (attn_fwd / bwd_kernel_dk_dv / bwd_kernel_dq /
// bwd_preprocess: 84 ms of the 4 x 2048 Llama-3-8B step, profiles/r04_12/llama_kernels.md).
#include <math.h>

#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

constexpr int kD = 128;                 // head dim
constexpr int kBQ = 128;                // queries (forward, dQ) / keys (dK dV) per workgroup
constexpr int kBK = 64;                 // rows per staged tile
constexpr int kImg = kBK * 256;         // one [64][128] bf16 image: 16 KB
constexpr int kThreads = 256;

struct FaArgs {
  const uint16_t* q;      // [B, H, S, 128]
  const uint16_t* k;      // [B, KV, S, 128]
  const uint16_t* v;
  const uint16_t* o;      // [B, S, H, 128]
  const uint16_t* dout;   // [B, S, H, 128]
  uint16_t* out;          // forward: o; backward: dq [B, H, S, 128]
  uint16_t* dk;           // [B, H, S, 128]
  uint16_t* dv;
  float* lse;             // [B, H, S]
  float* dsum;            // [B, H, S]
  int B, H, KV, S;
  float c;                // scale * log2(e)
  float scale;
  float thr;              // forward: deferred-rescale threshold (log2 units), see fa_fwd_kernel
};

__device__ __forceinline__ f32x16 mfma(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// accumulator row of register i for lane half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
__device__ __forceinline__ int swz_f(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
// byte offset of 16-B chunk ch / of element col of row `row` in a [rows][256 B] image
__device__ __forceinline__ int sw(int row, int ch) { return row * 256 + 16 * (ch ^ swz_f(row)); }
__device__ __forceinline__ int swe(int row, int col) { return sw(row, col >> 3) + 2 * (col & 7); }
__device__ __forceinline__ bf16x8_t rowfrag(const char* img, int row, int ch) {
  return *reinterpret_cast<const bf16x8_t*>(img + sw(row, ch));
}
__device__ __forceinline__ uint2 tr_rd(const char* p) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p)));
}
// transposed operand of an image X [rows = k][128 cols = m]: elements 0-3 = X[ka + q][m],
// 4-7 = X[kb + q][m] (q = 0..3), m = m0 + (lane & 31)
__device__ __forceinline__ bf16x8_t trfrag(const char* img, int ka, int kb, int m0, int lane) {
  const int q = (lane >> 2) & 3, col = m0 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const uint2 lo = tr_rd(img + swe(ka + q, col)), hi = tr_rd(img + swe(kb + q, col));
  return __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
}
// registers 8u..8u+7 of an accumulator as a bf16 operand fragment
__device__ __forceinline__ bf16x8_t acc_frag(const f32x16& x, int u) {
  const int o = 8 * u;
  return __builtin_bit_cast(bf16x8_t, make_uint4(pk_bf16(x[o], x[o + 1]), pk_bf16(x[o + 2], x[o + 3]),
                                                 pk_bf16(x[o + 4], x[o + 5]),
                                                 pk_bf16(x[o + 6], x[o + 7])));
}
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// One row of 128 outputs times sc as bf16: o[dt][4g..4g+3] = elements 32 dt + 8 g + 4 h + 0..3
// of the lane's row (lanes r and r + 32 hold one row). permlane32_swap pairs groups g, g + 1 so
// each lane stores 16 contiguous bytes (8 dwordx4 per lane instead of 16 dwordx2; the store tail
// is issue-bound). Every lane must execute it (a cross-lane op): `ok` only gates the stores.
__device__ __forceinline__ void store_row(uint16_t* row, const f32x16 (&o)[4], float sc, int h,
                                          bool ok) {
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      uint32_t a0 = pk_bf16(o[dt][4 * g] * sc, o[dt][4 * g + 1] * sc);
      uint32_t a1 = pk_bf16(o[dt][4 * g + 2] * sc, o[dt][4 * g + 3] * sc);
      uint32_t b0 = pk_bf16(o[dt][4 * g + 4] * sc, o[dt][4 * g + 5] * sc);
      uint32_t b1 = pk_bf16(o[dt][4 * g + 6] * sc, o[dt][4 * g + 7] * sc);
      const auto x = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto y = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      a0 = x[0]; b0 = x[1];
      a1 = y[0]; b1 = y[1];
      if (ok) *reinterpret_cast<uint4*>(row + 32 * dt + 8 * g + 8 * h) = make_uint4(a0, a1, b0, b1);
    }
}

// rows [row0, row0 + ROWS) of a [S][ld] bf16 tensor (rows past S clamped to S - 1) into an
// image: ROWS / 4 LDS-DMA wave-instructions of 4 rows x 256 B, wave w of NW issues w, w + NW, ..
template <int NW = 4, int ROWS = kBK>
__device__ __forceinline__ void stage(const uint16_t* g, int64_t ld, int row0, int S, char* img,
                                      int w, int lane) {
#pragma unroll
  for (int s = 0; s < ROWS / 4 / NW; ++s) {
    const int i = w + NW * s;
    const int row = 4 * i + (lane >> 4);
    const int ch = (lane & 15) ^ swz_f(row);
    int gr = row0 + row;
    gr = gr < S ? gr : S - 1;
    __builtin_amdgcn_global_load_lds((g_void*)(g + gr * ld + 8 * ch), (lds_void*)(img + 1024 * i),
                                     16, 0, 0);
  }
}

// workgroup id -> (row block, batch * head): ids sharing an XCD (id % 8) take a contiguous head
// range; blocks in decreasing (heavy_last) or increasing order of causal work
__device__ __forceinline__ void work_item(int nblk, int BH, bool heavy_last, int& blk, int& bh) {
  const int id = blockIdx.x;
  int slot, hb;
  if ((BH & 7) == 0) {
    const int hp = BH >> 3;
    slot = (id >> 3) / hp;
    hb = (id & 7) * hp + (id >> 3) % hp;
  } else {
    slot = id / BH;
    hb = id % BH;
  }
  blk = heavy_last ? nblk - 1 - slot : slot;
  bh = hb;
}

// ------------------------------------------------------------------------------------- forward
// NWV waves x 32 queries per workgroup: 4 (two workgroups per CU) or 8 (one; each staged K / V
// tile feeds twice the queries, half the L2 -> LDS traffic per FLOP)
template <bool CAUSAL, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, 8 / NWV) void fa_fwd_kernel(FaArgs a) {
  constexpr int BQ = 32 * NWV;
  extern __shared__ __attribute__((aligned(16))) char smem[];   // 2 x (K image, V image)
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int S = a.S;
  int qb, bh;
  work_item((S + BQ - 1) / BQ, a.B * a.H, CAUSAL, qb, bh);
  const int b = bh / a.H, hh = bh - b * a.H, kvh = hh / (a.H / a.KV);
  const int q0 = qb * BQ, qrow = q0 + 32 * w + r, qmin = q0 + 32 * w;
  const int64_t kvoff = (static_cast<int64_t>(b) * a.KV + kvh) * S * kD;
  const uint16_t* kg = a.k + kvoff;
  const uint16_t* vg = a.v + kvoff;
  const int kend = CAUSAL ? min(S, q0 + BQ) : S;
  const int nt = (kend + kBK - 1) / kBK;

  stage<NWV>(kg, kD, 0, S, smem, w, lane);
  stage<NWV>(vg, kD, 0, S, smem + kImg, w, lane);
  bf16x8_t qf[8];   // B operand of S^T = K Q^T: Q[qrow][16 ks + 8 h + j]
  {
    const uint16_t* qp = a.q + (static_cast<int64_t>(bh) * S + min(qrow, S - 1)) * kD + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *reinterpret_cast<const bf16x8_t*>(qp + 16 * ks);
  }
  f32x16 o[4] = {zero16(), zero16(), zero16(), zero16()};
  float m = -INFINITY, l = 0.f;
  for (int t = 0; t < nt; ++t) {
    const char* kimg = smem + (t & 1) * 2 * kImg;
    const char* vimg = kimg + kImg;
    // tile t landed (this wave's DMAs: a barrier does not wait for global_load_lds, and hipcc
    // inserts no wait here -- its alias analysis separates the two buffers), then every wave's;
    // every wave is done with tile t - 1's buffer
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < nt) {
      char* nb = smem + ((t + 1) & 1) * 2 * kImg;
      stage<NWV>(kg, kD, (t + 1) * kBK, S, nb, w, lane);
      stage<NWV>(vg, kD, (t + 1) * kBK, S, nb + kImg, w, lane);
    }
    const int k0 = t * kBK;
    if (CAUSAL && k0 > qmin + 31) continue;   // every key of the tile is after every query
    // S^T: s0 = keys k0 + 0..31, s1 = keys k0 + 32..63 (rows), query qrow (lane)
    f32x16 s0 = zero16(), s1 = zero16();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      s0 = mfma(rowfrag(kimg, r, 2 * ks + h), qf[ks], s0);
      s1 = mfma(rowfrag(kimg, 32 + r, 2 * ks + h), qf[ks], s1);
    }
    if (CAUSAL ? (k0 + kBK - 1 > qmin) : (k0 + kBK > S)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = k0 + acc_row(i, h);
        if ((CAUSAL && key > qrow) || key >= S) s0[i] = -INFINITY;
        if ((CAUSAL && key + 32 > qrow) || key + 32 >= S) s1[i] = -INFINITY;
      }
    }
    float mt = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) mt = fmaxf(mt, fmaxf(s0[i], s1[i]));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * a.c;
    // deferred rescale: the running max m moves (and O, l are rescaled) only when some row's
    // tile max exceeds it by more than thr (log2 units), so exponentiated scores stay <= 2^thr
    // (fp32 O / l accumulators, bf16 P keeps its relative precision); the first tile always
    // sets m (finite from then on: key 0 is visible to every query). thr = 0: the textbook
    // rescale at every max increase.
    if (__any(mt > m + a.thr)) {
      const float mn = fmaxf(m, mt);
      const float alpha = fexp2(m - mn);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
    }
    float ls = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s0[i] = fexp2(fmaf(s0[i], a.c, -m));
      s1[i] = fexp2(fmaf(s1[i], a.c, -m));
      ls += s0[i] + s1[i];
    }
    l += ls;
    // O^T += V^T P^T over the 64 keys (4 k-steps of 16)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8_t p0 = acc_frag(s0, u), p1 = acc_frag(s1, u);
      const int ka = 16 * u + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        o[dt] = mfma(trfrag(vimg, ka, ka + 8, 32 * dt, lane), p0, o[dt]);
        o[dt] = mfma(trfrag(vimg, 32 + ka, 40 + ka, 32 * dt, lane), p1, o[dt]);
      }
    }
  }
  l += __shfl_xor(l, 32, 64);
  store_row(a.out + ((static_cast<int64_t>(b) * S + min(qrow, S - 1)) * a.H + hh) * kD, o, 1.f / l,
            h, qrow < S);
  if (h == 0 && qrow < S) a.lse[static_cast<int64_t>(bh) * S + qrow] = m + __log2f(l);
}

// ------------------------------------------------------------------------------ backward: dQ
template <bool CAUSAL, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, 8 / NWV) void fa_dq_kernel(FaArgs a) {
  constexpr int BQ = 32 * NWV;
  extern __shared__ __attribute__((aligned(16))) char smem[];   // 2 x (K image, V image)
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int S = a.S;
  int qb, bh;
  work_item((S + BQ - 1) / BQ, a.B * a.H, CAUSAL, qb, bh);
  const int b = bh / a.H, hh = bh - b * a.H, kvh = hh / (a.H / a.KV);
  const int q0 = qb * BQ, qrow = q0 + 32 * w + r, qmin = q0 + 32 * w;
  const int qc = min(qrow, S - 1);
  const int64_t kvoff = (static_cast<int64_t>(b) * a.KV + kvh) * S * kD;
  const uint16_t* kg = a.k + kvoff;
  const uint16_t* vg = a.v + kvoff;
  const int kend = CAUSAL ? min(S, q0 + BQ) : S;
  const int nt = (kend + kBK - 1) / kBK;

  stage<NWV>(kg, kD, 0, S, smem, w, lane);
  stage<NWV>(vg, kD, 0, S, smem + kImg, w, lane);
  bf16x8_t qf[8], df[8];
  float dsum;
  {
    const uint16_t* qp = a.q + (static_cast<int64_t>(bh) * S + qc) * kD + 8 * h;
    const int64_t orow = ((static_cast<int64_t>(b) * S + qc) * a.H + hh) * kD + 8 * h;
    const uint16_t* dp = a.dout + orow;
    const uint16_t* op = a.o + orow;
    float part = 0.f;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      qf[ks] = *reinterpret_cast<const bf16x8_t*>(qp + 16 * ks);
      const uint4 dv = *reinterpret_cast<const uint4*>(dp + 16 * ks);
      const uint4 ov = *reinterpret_cast<const uint4*>(op + 16 * ks);
      df[ks] = __builtin_bit_cast(bf16x8_t, dv);
      const uint32_t d4[4] = {dv.x, dv.y, dv.z, dv.w}, o4[4] = {ov.x, ov.y, ov.z, ov.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        part = fmaf(__uint_as_float(d4[e] << 16), __uint_as_float(o4[e] << 16), part);
        part = fmaf(__uint_as_float(d4[e] & 0xffff0000u), __uint_as_float(o4[e] & 0xffff0000u), part);
      }
    }
    dsum = part + __shfl_xor(part, 32, 64);
    if (h == 0 && qrow < S) a.dsum[static_cast<int64_t>(bh) * S + qrow] = dsum;
  }
  const float lse = a.lse[static_cast<int64_t>(bh) * S + qc];
  f32x16 dq[4] = {zero16(), zero16(), zero16(), zero16()};
  for (int t = 0; t < nt; ++t) {
    const char* kimg = smem + (t & 1) * 2 * kImg;
    const char* vimg = kimg + kImg;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile t landed (see fa_fwd_kernel)
    __syncthreads();
    if (t + 1 < nt) {
      char* nb = smem + ((t + 1) & 1) * 2 * kImg;
      stage<NWV>(kg, kD, (t + 1) * kBK, S, nb, w, lane);
      stage<NWV>(vg, kD, (t + 1) * kBK, S, nb + kImg, w, lane);
    }
    const int k0 = t * kBK;
    if (CAUSAL && k0 > qmin + 31) continue;
    f32x16 s0 = zero16(), s1 = zero16(), p0 = zero16(), p1 = zero16();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      s0 = mfma(rowfrag(kimg, r, 2 * ks + h), qf[ks], s0);
      s1 = mfma(rowfrag(kimg, 32 + r, 2 * ks + h), qf[ks], s1);
      p0 = mfma(rowfrag(vimg, r, 2 * ks + h), df[ks], p0);
      p1 = mfma(rowfrag(vimg, 32 + r, 2 * ks + h), df[ks], p1);
    }
    const bool edge = CAUSAL ? (k0 + kBK - 1 > qmin) : (k0 + kBK > S);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float e0 = fexp2(fmaf(s0[i], a.c, -lse)), e1 = fexp2(fmaf(s1[i], a.c, -lse));
      if (edge) {
        const int key = k0 + acc_row(i, h);
        if ((CAUSAL && key > qrow) || key >= S) e0 = 0.f;
        if ((CAUSAL && key + 32 > qrow) || key + 32 >= S) e1 = 0.f;
      }
      s0[i] = e0 * (p0[i] - dsum);   // dS^T
      s1[i] = e1 * (p1[i] - dsum);
    }
    // dQ^T += K^T dS^T (K^T by transposed reads of the K rows)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8_t d0 = acc_frag(s0, u), d1 = acc_frag(s1, u);
      const int ka = 16 * u + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dq[dt] = mfma(trfrag(kimg, ka, ka + 8, 32 * dt, lane), d0, dq[dt]);
        dq[dt] = mfma(trfrag(kimg, 32 + ka, 40 + ka, 32 * dt, lane), d1, dq[dt]);
      }
    }
  }
  store_row(a.out + (static_cast<int64_t>(bh) * S + min(qrow, S - 1)) * kD, dq, a.scale, h,
            qrow < S);
}

// --------------------------------------------------------------------------- backward: dK, dV
// 8 waves x 32 keys = 256 keys per workgroup (two waves per SIMD); the block's V rows sit in LDS
// for the whole kernel (B operand of dP = dO V^T by row reads), the lane's K row in registers.
// LDS: V image (64 KB) + 2 x (Q image, dO image, lse [64], D [64]) = 130 KB, one workgroup per CU.
constexpr int kKVKeys = 256;
constexpr int kKVThreads = 512;
constexpr int kKVBuf = 2 * kImg + 512;
constexpr int kVImg = kKVKeys * 256;

template <bool CAUSAL>
__global__ __launch_bounds__(kKVThreads, 2) void fa_dkdv_kernel(FaArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* vimg = smem;
  char* bufs = smem + kVImg;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int S = a.S;
  int kb, bh;
  work_item((S + kKVKeys - 1) / kKVKeys, a.B * a.H, false, kb, bh);
  const int b = bh / a.H, hh = bh - b * a.H, kvh = hh / (a.H / a.KV);
  const int kb0 = kb * kKVKeys, key = kb0 + 32 * w + r, kmin = kb0 + 32 * w;
  const int64_t kvoff = (static_cast<int64_t>(b) * a.KV + kvh) * S * kD;
  const uint16_t* qg = a.q + static_cast<int64_t>(bh) * S * kD;
  const int64_t ld_o = static_cast<int64_t>(a.H) * kD;
  const uint16_t* dog = a.dout + static_cast<int64_t>(b) * S * ld_o + hh * kD;
  const float* lseg = a.lse + static_cast<int64_t>(bh) * S;
  const float* dsg = a.dsum + static_cast<int64_t>(bh) * S;
  const int qstart = CAUSAL ? kb0 : 0;
  const int nt = (S - qstart + kBK - 1) / kBK;

  auto stage_all = [&](int t, char* buf) {
    const int row0 = qstart + t * kBK;
    stage<8>(qg, kD, row0, S, buf, w, lane);
    stage<8>(dog, ld_o, row0, S, buf + kImg, w, lane);
    if (w < 2) {   // lse (wave 0) / D (wave 1) of the tile's 64 queries: one 4-B DMA per lane
      const float* src = (w == 0 ? lseg : dsg) + min(row0 + lane, S - 1);
      __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(buf + 2 * kImg + 256 * w), 4, 0, 0);
    }
  };
  stage<8, kKVKeys>(a.v + kvoff, kD, kb0, S, vimg, w, lane);
  stage_all(0, bufs);
  bf16x8_t kf[8];   // B operand K^T [d][key] = this lane's key row
  {
    const uint16_t* kp = a.k + kvoff + static_cast<int64_t>(min(key, S - 1)) * kD + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) kf[ks] = *reinterpret_cast<const bf16x8_t*>(kp + 16 * ks);
  }
  f32x16 dk[4] = {zero16(), zero16(), zero16(), zero16()};
  f32x16 dv[4] = {zero16(), zero16(), zero16(), zero16()};
  for (int t = 0; t < nt; ++t) {
    const char* buf = bufs + (t & 1) * kKVBuf;
    const char* qimg = buf;
    const char* dimg = buf + kImg;
    const float* lsel = reinterpret_cast<const float*>(buf + 2 * kImg);
    const float* dsl = lsel + 64;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile t landed (see fa_fwd_kernel)
    __syncthreads();
    if (t + 1 < nt) stage_all(t + 1, bufs + ((t + 1) & 1) * kKVBuf);
    const int q0 = qstart + t * kBK;
#pragma unroll 1
    for (int qs = 0; qs < 2; ++qs) {
      const int qq0 = q0 + 32 * qs;
      // causal: a sub-tile whose every query is before every key of the wave contributes nothing
      if (!CAUSAL || qq0 + 31 >= kmin) {
        f32x16 s = zero16(), dp = zero16();
        // the V rows are loop-invariant: an opaque base keeps them LDS reads (hoisted, they
        // would pin 32 more VGPRs for the whole loop)
        int vrow = 32 * w + r;
        asm volatile("" : "+v"(vrow));
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          s = mfma(rowfrag(qimg, 32 * qs + r, 2 * ks + h), kf[ks], s);
          dp = mfma(rowfrag(dimg, 32 * qs + r, 2 * ks + h), rowfrag(vimg, vrow, 2 * ks + h), dp);
        }
        // s[i] = S[query qq0 + acc_row(i, h)][key]; registers 4g..4g+3: 4 consecutive queries
        const bool edge = (CAUSAL && qq0 < kmin + 31) || qq0 + 32 > S;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ql = 32 * qs + 8 * g + 4 * h;
          const float4 L = *reinterpret_cast<const float4*>(lsel + ql);
          const float4 Dd = *reinterpret_cast<const float4*>(dsl + ql);
          const float Lv[4] = {L.x, L.y, L.z, L.w}, Dv[4] = {Dd.x, Dd.y, Dd.z, Dd.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e;
            float p = fexp2(fmaf(s[i], a.c, -Lv[e]));
            if (edge) {
              const int qi = qq0 + 8 * g + 4 * h + e;
              if ((CAUSAL && qi < key) || qi >= S) p = 0.f;
            }
            s[i] = p;
            dp[i] = p * (dp[i] - Dv[e]);
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bf16x8_t pb = acc_frag(s, u), sb = acc_frag(dp, u);
          const int ka = 32 * qs + 16 * u + 4 * h;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            dv[dt] = mfma(trfrag(dimg, ka, ka + 8, 32 * dt, lane), pb, dv[dt]);
            dk[dt] = mfma(trfrag(qimg, ka, ka + 8, 32 * dt, lane), sb, dk[dt]);
          }
        }
      }
    }
  }
  const int64_t row = (static_cast<int64_t>(bh) * S + min(key, S - 1)) * kD;
  store_row(a.dk + row, dk, a.scale, h, key < S);
  store_row(a.dv + row, dv, 1.f, h, key < S);
}

typedef void (*FaKernel)(FaArgs);

hipError_t launch_fa(FaKernel kern, const FaArgs& a, int smem, hipStream_t st, int rows = kBQ,
                     int threads = kThreads) {
  // dynamic LDS above the default limit: set once per kernel
  static const void* done[16] = {};
  const void* f = reinterpret_cast<const void*>(kern);
  bool set = false;
  for (const void* d : done) set = set || d == f;
  if (!set) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    if (e != hipSuccess) return e;
    for (const void*& d : done)
      if (d == nullptr) {
        d = f;
        break;
      }
  }
  const int nblk = (a.S + rows - 1) / rows;
  const dim3 grid(static_cast<unsigned>(nblk * a.B * a.H));
  kern<<<grid, threads, smem, st>>>(a);
  return hipGetLastError();
}

// queries per workgroup of the forward and dQ kernels: CML_FA_WAVES = 8 (256, default: each staged
// K / V tile feeds twice the queries; backward 0.574-0.580 vs 0.588-0.590 ms per Llama-3-8B layer,
// forward within 1 %, profiles/r06_24/fa_*.jsonl) or 4 (128)
int fa_waves() {
  static const int w = [] {
    const char* e = std::getenv("CML_FA_WAVES");
    return e && std::atoi(e) == 4 ? 4 : 8;
  }();
  return w;
}

bool fa_shape_ok(int B, int H, int KV, int S) {
  return B >= 1 && H >= 1 && KV >= 1 && H % KV == 0 && S >= 1 &&
         static_cast<int64_t>((S + kBQ - 1) / kBQ) * B * H < (1LL << 31);
}

}  // namespace

hipError_t launch_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B,
                            int H, int KV, int S, float scale, bool causal, hipStream_t st,
                            float rescale_thr) {
  if (!fa_shape_ok(B, H, KV, S)) return hipErrorInvalidValue;
  FaArgs a{};
  a.q = static_cast<const uint16_t*>(q);
  a.k = static_cast<const uint16_t*>(k);
  a.v = static_cast<const uint16_t*>(v);
  a.out = static_cast<uint16_t*>(o);
  a.lse = lse;
  a.B = B; a.H = H; a.KV = KV; a.S = S;
  a.scale = scale;
  a.c = scale * 1.4426950408889634f;
  a.thr = rescale_thr < 0.f ? 0.f : rescale_thr;
  if (fa_waves() == 8)
    return causal ? launch_fa(fa_fwd_kernel<true, 8>, a, 4 * kImg, st, 256, 512)
                  : launch_fa(fa_fwd_kernel<false, 8>, a, 4 * kImg, st, 256, 512);
  return causal ? launch_fa(fa_fwd_kernel<true>, a, 4 * kImg, st)
                : launch_fa(fa_fwd_kernel<false>, a, 4 * kImg, st);
}

hipError_t launch_flash_bwd(const void* q, const void* k, const void* v, const void* o,
                            const void* dout, const float* lse, float* dsum, void* dq, void* dk,
                            void* dv, int B, int H, int KV, int S, float scale, bool causal,
                            hipStream_t st) {
  if (!fa_shape_ok(B, H, KV, S)) return hipErrorInvalidValue;
  FaArgs a{};
  a.q = static_cast<const uint16_t*>(q);
  a.k = static_cast<const uint16_t*>(k);
  a.v = static_cast<const uint16_t*>(v);
  a.o = static_cast<const uint16_t*>(o);
  a.dout = static_cast<const uint16_t*>(dout);
  a.out = static_cast<uint16_t*>(dq);
  a.dk = static_cast<uint16_t*>(dk);
  a.dv = static_cast<uint16_t*>(dv);
  a.lse = const_cast<float*>(lse);
  a.dsum = dsum;
  a.B = B; a.H = H; a.KV = KV; a.S = S;
  a.scale = scale;
  a.c = scale * 1.4426950408889634f;
  // dQ first: it also writes D = rowsum(dO * O), which the dK / dV kernel reads
  hipError_t e;
  if (fa_waves() == 8)
    e = causal ? launch_fa(fa_dq_kernel<true, 8>, a, 4 * kImg, st, 256, 512)
               : launch_fa(fa_dq_kernel<false, 8>, a, 4 * kImg, st, 256, 512);
  else
    e = causal ? launch_fa(fa_dq_kernel<true>, a, 4 * kImg, st)
               : launch_fa(fa_dq_kernel<false>, a, 4 * kImg, st);
  if (e != hipSuccess) return e;
  constexpr int smem = kVImg + 2 * kKVBuf;
  return causal ? launch_fa(fa_dkdv_kernel<true>, a, smem, st, kKVKeys, kKVThreads)
                : launch_fa(fa_dkdv_kernel<false>, a, smem, st, kKVKeys, kKVThreads);
}

}  // namespace cml
