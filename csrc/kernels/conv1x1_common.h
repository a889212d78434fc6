// Device code shared by the fused 1x1-convolution kernels: conv1x1.hip (persistent, register-
// staged operands) and conv1x1g.hip (global_load_lds-staged 256-wide tiles). Operand LDS images,
// the argument block, and the per-wave epilogue (bf16 rounding, BN statistics / BN-backward sums,
// residual-link and BN + residual + ReLU epilogues, coalesced 16-B stores through LDS).
#pragma once
#include "common.h"

namespace cml {
namespace c1 {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBK = 64;          // K per step: one 128-B LDS row per output channel / pixel
constexpr int kThreads = 256;    // 4 waves

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// byte offset of 16-B chunk c (0..7) of row `row` in a [rows][128 B] image. Row parity picks the
// half of the 256-B bank row, and the XOR with row bits 1..3 spreads the 16 rows of each
// ds_read_b128 lane group ({0-3,12-15,20-27}, ...) over 16 distinct 16-B bank slots.
__device__ __forceinline__ int swz(int row, int c) { return row * 128 + 16 * (c ^ ((row >> 1) & 7)); }

// Prologue modes (f applied to x while staging) and statistics modes (epilogue sums).
enum { PM_NONE = 0, PM_BNRELU = 1, PM_BNBWD = 2, PM_CAT = 3 };
enum { SM_BN = 0, SM_BNBWD = 1, SM_OFF = 2, SM_BNRES = 3 };

struct C1Args {
  const uint16_t* x;      // [rows_in][K]
  const uint16_t* w;      // [N][K]
  uint16_t* y;            // [M][N]
  float* part;            // [ntn][wgpn * WM][2][BN] or null
  const float* pro_sc;    // PM_BNRELU: sc[K]; PM_BNBWD: a[K]
  const float* pro_bi;    // PM_BNRELU: bi[K]; PM_BNBWD: b[K]
  const float* pro_c;     // PM_BNBWD: c[K]
  const uint16_t* x2;     // PM_BNBWD: z [rows_in][K] (the BN input)
  const uint8_t* xm;      // PM_BNBWD: ReLU bit mask of the BN output [rows_in][K / 8]
  const uint16_t* link;   // EL: [M][N] added to the product where lm's bit is set
  const uint8_t* lm;      // EL: [M][N / 8]
  const uint16_t* sz;     // SM_BNBWD: z of the BN whose backward sums are taken [M][N]
  const uint8_t* sm;      // SM_BNBWD: its ReLU bit mask [M][N / 8]
  const float* shift;     // [N] or null (SM_BN: statistics shift; SM_BNBWD: the BN's mean)
  const float* ep_sc;     // SM_BNRES: y = max(v ep_sc + ep_bi + link, 0) per output channel [N]
  const float* ep_bi;
  uint8_t* ymask;         // SM_BNRES: bit mask of y > 0 [M][N / 8]
  // PM_CAT (two sources concatenated along K): the first source (x, K1 channels) is staged as
  // (mask xm ? x : 0) -- a BN + ReLU backward's affine a u + c is folded into w and `bias` by the
  // caller -- or, with cat_bnrelu, as max(x pro_sc + pro_bi, 0) (pro_sc / pro_bi [K1]); the second
  // (x2, K - K1 channels) as max(x2 pro_sc2 + pro_bi2, 0), or as x2 itself when pro_sc2 is null.
  const float* pro_sc2;
  const float* pro_bi2;
  const float* bias;      // PM_CAT: [N] added to the fp32 products before rounding, or null
  int K1;
  int cat_bnrelu;
  int M, K, N;
  int ntn, wgpn, mtiles;
  int H, W, OW, OHW;      // S2: input H, W; output W and H*W
  // EL with link_s2: link is [N][ceil(H/2)][ceil(W/2)][N channels] (a stride-2 conv's compact
  // data gradient), added at the even pixels of this [N][H][W] output (lm unused)
  int link_s2, lW, lHW, lOW, lOHW;
  // diagnostics only (bench/conv1x1g.py --ablate; 0 in production): quad-phase kernel skips
  // bit 0 the MFMAs, bit 1 the DMA issue, bit 2 the in-LDS prologue, bit 3 the epilogue
  int ablate;
};

__device__ __forceinline__ int64_t src_row(const C1Args& a, int m, bool s2) {
  m = m < a.M ? m : a.M - 1;                                    // clamped: loads stay in bounds
  if (s2) {
    const int img = m / a.OHW;
    const int rem = m - img * a.OHW;
    const int oh = rem / a.OW;
    const int ow = rem - oh * a.OW;
    return static_cast<int64_t>(img) * a.H * a.W + 2 * oh * a.W + 2 * ow;
  }
  return m;
}

// prologue coefficient table s_aff = {sc[K], bi[K]} in LDS. PM_CAT: the first K1 entries are the
// first source's BN affine (cat_bnrelu; 1 / 0 when it is masked), the rest the second source's
// (pro_sc2 / pro_bi2; 1 / 0 when it is staged as is).
__device__ __forceinline__ void fill_aff(const C1Args& a, bool cat, float* s_aff, int K, int tid,
                                         int nt) {
  for (int k = tid; k < K; k += nt) {
    float sc, bi;
    if (!cat) {
      sc = a.pro_sc[k];
      bi = a.pro_bi[k];
    } else if (k < a.K1) {
      sc = a.cat_bnrelu ? a.pro_sc[k] : 1.f;
      bi = a.cat_bnrelu ? a.pro_bi[k] : 0.f;
    } else {
      sc = a.pro_sc2 ? a.pro_sc2[k - a.K1] : 1.f;
      bi = a.pro_sc2 ? a.pro_bi2[k - a.K1] : 0.f;
    }
    s_aff[k] = sc;
    s_aff[K + k] = bi;
  }
}

__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const float4 u0 = reinterpret_cast<const float4*>(p)[0], u1 = reinterpret_cast<const float4*>(p)[1];
  v[0] = u0.x; v[1] = u0.y; v[2] = u0.z; v[3] = u0.w;
  v[4] = u1.x; v[5] = u1.y; v[6] = u1.z; v[7] = u1.w;
}

// Round the wave's 64 (n) x 64 (m) block to bf16 and store it, adding the stored values (minus the
// shift) to the statistics. The accumulator layout (lane = pixel, 4 consecutive channels per
// register group) would make every global store instruction touch 32 lines with 16 B each (the
// kernel then wrote at ~3 TB/s); instead the block goes through the wave's own 8 KB LDS image
// [pixel][128 B] (XOR-swizzled like the operand images) and comes back as 16-B pieces, 8 lanes per
// 128-B pixel row: every store instruction writes whole lines. The read-back also gives each lane
// a fixed group of 8 channels (lane & 7), so the statistics need 16 registers (sum and sum of
// squares of 8 channels) instead of 64. Only this wave touches its image: no workgroup barrier.
//
// EL: the stored value is bf16(bf16(acc) + (lm bit ? link : 0)) (a data gradient plus the masked
// residual gradient of the same tensor). SM_BNBWD: the sums are s = sum (sm bit ? v : 0) and
// q = sum (sm bit ? v : 0) (sz - shift) -- the backward reduction of the BN + ReLU whose output
// gradient v is (the consumer BN's mean in shift) -- instead of the BN statistics of v.
// DM (SM_BNBWD without a stored mask, PM_CAT data gradients of the recompute tails): the ReLU bit
// is recomputed from the BN input, sz * ep_sc + ep_bi > 0 (the BN's own affine, as its forward
// prologue applied it), so the BN + ReLU backward that follows needs no reduction pass of its own.
// mhi: global row of block rows 32..63 (default m0 + 32; the quad-phase kernel's waves own two
// separate 32-row groups).
// BIAS: bsrc[ncol0 + channel] (when bsrc is set: PM_CAT's folded affine, a.bias from the tile's
// first channel, or its LDS copy) is added to every product before rounding.
template <bool EL, int SM, int MT, bool DM = false, bool BIAS = false>
__device__ __forceinline__ void epilogue(const C1Args& a, f32x16 (&acc)[2][2], float (&ss)[8],
                                         float (&sq)[8], const float (&sh)[8], char* simg, int m0,
                                         int ncol0, int n0, int lane, int mhi = -1,
                                         const float* bsrc = nullptr) {
  const int h = lane >> 5, r32 = lane & 31;
  const int c = lane & 7;
  const int mh = mhi < 0 ? m0 + 32 : mhi;
  auto grow = [&](int p) { return p < 32 ? m0 + p : mh + (p - 32); };
  // EL / SM_BNBWD operands of the read-back rows are issued as one batch before they are needed
  // (a 1-2 k-step GEMM was otherwise bound by these dependent loads, one latency per row pair):
  // all 8 rows at once with one operand (EL), in batches of 4 with two, halved again at MT = 2
  // (more registers would spill). Rows past M re-read row M - 1 (a wave block of a partial tile
  // can start past M).
  constexpr bool LD = EL || SM == SM_BNBWD || SM == SM_BNRES;
  constexpr int RB = ((EL && SM == SM_BNBWD) ? 4 : 8) / MT /   // rows per batch
                     ((SM == SM_BNRES && MT == 2) ? 2 : 1);
  uint4 lv[RB], zv[RB];
  uint32_t lbv[RB], zbv[RB];
  if constexpr (!(EL && SM == SM_BNBWD)) {   // one operand: keep the row body's arguments defined
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      if constexpr (!EL) lbv[k] = 0u;
      if constexpr (!EL && SM != SM_BNRES) lv[k] = make_uint4(0u, 0u, 0u, 0u);
      if constexpr (SM != SM_BNBWD) { zv[k] = make_uint4(0u, 0u, 0u, 0u); zbv[k] = 0u; }
    }
  }
  // SM_BNRES / DM: the lane's 8 output channels' BN coefficients
  float esc[8], ebi[8];
  if constexpr (SM == SM_BNRES || DM) {
    ld8f(a.ep_sc + n0 + ncol0 + 8 * c, esc);
    ld8f(a.ep_bi + n0 + ncol0 + 8 * c, ebi);
  }
  auto issue = [&](int k0) {
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int p = 8 * (k0 + k) + (lane >> 3);
      const int gp = grow(p);
      const int64_t row = gp < a.M ? gp : a.M - 1;
      const int64_t e0 = row * a.N + n0 + ncol0 + 8 * c;
      if constexpr (EL) {
        if (a.link_s2) {   // compact stride-2 gradient: only the even pixels get an addend
          const int img = static_cast<int>(row / a.lHW);
          const int rem = static_cast<int>(row - static_cast<int64_t>(img) * a.lHW);
          const int hh = rem / a.lW, ww = rem - hh * a.lW;
          const bool ev = !((hh | ww) & 1);
          const int64_t lrow = ev ? static_cast<int64_t>(img) * a.lOHW + (hh >> 1) * a.lOW + (ww >> 1) : 0;
          lv[k] = *reinterpret_cast<const uint4*>(a.link + lrow * a.N + n0 + ncol0 + 8 * c);
          lbv[k] = ev ? 0xffu : 0u;
        } else {
          lv[k] = *reinterpret_cast<const uint4*>(a.link + e0);
          lbv[k] = a.lm ? a.lm[e0 >> 3] : 0xffu;   // no mask: a plain residual add
        }
      }
      if constexpr (SM == SM_BNRES)   // (no residual: link null)
        lv[k] = a.link ? *reinterpret_cast<const uint4*>(a.link + e0) : make_uint4(0u, 0u, 0u, 0u);
      if constexpr (SM == SM_BNBWD) {
        zv[k] = *reinterpret_cast<const uint4*>(a.sz + e0);
        zbv[k] = DM ? 0u : a.sm[e0 >> 3];
      }
    }
  };
  if constexpr (LD) issue(0);
  const bool bias = BIAS && bsrc != nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      // channels 32 i + 8 g + 4 h .. +3 = half h of 16-B chunk 4 i + g of the pixel row
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bias) bv = *reinterpret_cast<const float4*>(bsrc + ncol0 + 32 * i + 8 * g + 4 * h);
#pragma unroll
      for (int jm = 0; jm < 2; ++jm) {
        const int p = 32 * jm + r32;                   // pixel row of the wave block
        const f32x16& v = acc[i][jm];
        *reinterpret_cast<uint2*>(simg + swz(p, 4 * i + g) + 8 * h) =
            make_uint2(pk_bf16(v[4 * g + 0] + bv.x, v[4 * g + 1] + bv.y),
                       pk_bf16(v[4 * g + 2] + bv.z, v[4 * g + 3] + bv.w));
      }
    }
  }
  // the wave's own LDS writes complete before its reads
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  // one read-back row: 8 channels (lane & 7) of pixel 8 k + lane / 8
  auto row = [&](int k, const uint4& l, uint32_t lb, const uint4& z, uint32_t zb) {
    const int p = 8 * k + (lane >> 3);
    uint4 v = *reinterpret_cast<const uint4*>(simg + swz(p, c));
    const int gp = grow(p);
    if (gp >= a.M) return;
    const int64_t e0 = static_cast<int64_t>(gp) * a.N + n0 + ncol0 + 8 * c;
    if constexpr (EL) {
      const uint32_t l4[4] = {l.x, l.y, l.z, l.w};
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = __uint_as_float(w4[q] << 16) +
                         (((lb >> (2 * q)) & 1u) ? __uint_as_float(l4[q] << 16) : 0.f);
        const float hi = __uint_as_float(w4[q] & 0xffff0000u) +
                         (((lb >> (2 * q + 1)) & 1u) ? __uint_as_float(l4[q] & 0xffff0000u) : 0.f);
        w4[q] = pk_bf16(lo, hi);
      }
      v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    if constexpr (SM == SM_BNRES) {   // y = max(bn(v) + res, 0) and its bit mask; no statistics
      const uint32_t r4[4] = {l.x, l.y, l.z, l.w};
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      uint32_t bits = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = fmaf(__uint_as_float(w4[q] << 16), esc[2 * q], ebi[2 * q]) +
                         __uint_as_float(r4[q] << 16);
        const float hi = fmaf(__uint_as_float(w4[q] & 0xffff0000u), esc[2 * q + 1], ebi[2 * q + 1]) +
                         __uint_as_float(r4[q] & 0xffff0000u);
        bits |= (lo > 0.f ? 1u : 0u) << (2 * q);
        bits |= (hi > 0.f ? 1u : 0u) << (2 * q + 1);
        w4[q] = pk_bf16(fmaxf(lo, 0.f), fmaxf(hi, 0.f));
      }
      *reinterpret_cast<uint4*>(a.y + e0) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      a.ymask[e0 >> 3] = static_cast<uint8_t>(bits);
      return;
    }
    if (SM != SM_BN || a.y) *reinterpret_cast<uint4*>(a.y + e0) = v;   // SM_BN, y null: stats only
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    if constexpr (SM == SM_BN) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = __uint_as_float(w4[q] << 16) - sh[2 * q];
        const float hi = __uint_as_float(w4[q] & 0xffff0000u) - sh[2 * q + 1];
        ss[2 * q] += lo;
        ss[2 * q + 1] += hi;
        sq[2 * q] = fmaf(lo, lo, sq[2 * q]);
        sq[2 * q + 1] = fmaf(hi, hi, sq[2 * q + 1]);
      }
    } else if constexpr (SM == SM_BNBWD) {
      const uint32_t z4[4] = {z.x, z.y, z.z, z.w};
      if constexpr (DM) {
        zb = 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          zb |= (fmaf(__uint_as_float(z4[q] << 16), esc[2 * q], ebi[2 * q]) > 0.f ? 1u : 0u) << (2 * q);
          zb |= (fmaf(__uint_as_float(z4[q] & 0xffff0000u), esc[2 * q + 1], ebi[2 * q + 1]) > 0.f
                     ? 1u : 0u) << (2 * q + 1);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = ((zb >> (2 * q)) & 1u) ? __uint_as_float(w4[q] << 16) : 0.f;
        const float hi = ((zb >> (2 * q + 1)) & 1u) ? __uint_as_float(w4[q] & 0xffff0000u) : 0.f;
        ss[2 * q] += lo;
        ss[2 * q + 1] += hi;
        sq[2 * q] = fmaf(lo, __uint_as_float(z4[q] << 16) - sh[2 * q], sq[2 * q]);
        sq[2 * q + 1] = fmaf(hi, __uint_as_float(z4[q] & 0xffff0000u) - sh[2 * q + 1], sq[2 * q + 1]);
      }
    }
  };
  if constexpr (LD) {
#pragma unroll
    for (int kb = 0; kb < 8; kb += RB) {
      if (kb > 0) issue(kb);
#pragma unroll
      for (int k = 0; k < RB; ++k) row(kb + k, lv[k], lbv[k], zv[k], zbv[k]);
    }
  } else {
    const uint4 none = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll 2
    for (int k = 0; k < 8; ++k) row(k, none, 0u, none, 0u);
  }
  // the image is rewritten by the next tile's epilogue only after these reads have returned
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jm = 0; jm < 2; ++jm)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][jm][k] = 0.f;
}

}  // namespace c1

// conv1x1g.hip: the global_load_lds-staged kernel for the same (prologue, epilogue) modes.
// conv1x1g_pick: policy (CML_C1G = 0 / 1 / auto); part slabs: [ntn][R][2][BN] + fold area.
bool conv1x1g_eligible(int64_t M, int K, int N, int pm);
// bnres: the two-source GEMM with the BN + residual + ReLU epilogue (conv1x1_cat_bnres)
bool conv1x1g_pick(int64_t M, int K, int N, int pm, bool bnres = false);
size_t conv1x1g_part_floats(int64_t M, int K, int N, int pm);
hipError_t launch_conv1x1g(const c1::C1Args& a, int pm, int sm, bool el, hipStream_t st, int* R,
                           int* BN);

}  // namespace cml
