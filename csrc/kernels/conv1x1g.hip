// Fused 1x1 convolutions on the global_load_lds GEMM machinery of conv_gemm.hip: 256 x 256 (or
// 256 x 128) output tiles, 8 waves of 64 (m) x 128 (n) (or 64 x 64), both operands copied
// global -> LDS by the DMA path (global_load_lds_dwordx4, no VGPR staging) into two buffers, one
// vmcnt(0) + barrier per 64-deep k-step. Same products and epilogues as conv1x1.hip:
//
//   y[m][n] = sum_k W[n][k] f(x[m][k])
//   f = identity                                   (PM_NONE)
//     = max(x sc[k] + bi[k], 0)                     (PM_BNRELU: the producer's BN + ReLU)
//     = a[k] (mask ? x : 0) + c[k]  for k < K1      (PM_CAT: a BN + ReLU backward of the block
//       max(x2 sc[k] + bi[k], 0)    for k >= K1      output gradient | a recomputed BN + ReLU
//                                                    output, one GEMM over two K-concatenated
//                                                    sources)
//
// conv1x1.hip transforms x while staging it through registers, which is what keeps its operand
// pipeline shallow (0.4-0.6 PFLOP/s on the compute-bound shapes). Here the DMA lands raw bf16 in
// LDS (its image must be lane-linear, so no transform on the way) and the prologue runs on the MFMA
// B fragments after the ds_read: each lane's fragment is 8 consecutive channels of one pixel, so
// it needs 8 (sc, bi) pairs (two ds_read_b128 each from an fp32 coefficient table in LDS) and, for
// the masked source, one mask byte (staged per k-step by a 4-byte global_load_lds). The arithmetic
// is conv1x1.hip's (same fmaf, same bf16 rounding), so the operands -- and with the same k order
// the products -- are bit-identical. The VALU work (~3.5 instructions per element) issues beside
// the other wave's MFMAs (two waves per SIMD).
//
// Epilogue: conv1x1_common.h's per-wave 64 x 64 block epilogue, called for each 64-channel half of
// the wave's tile through its own 8 KB LDS image (the staging buffers are free by then); BN
// statistics / BN-backward sums go to one partial row per (m-tile, wave row) of a tall slab that
// launch_bn_stats_finalize / launch_bnbwd_sums_finalize fold (fixed order, deterministic).
// Tiles are mapped XCD-aware: the n-tiles of one m-tile are consecutive on one XCD.
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "conv1x1_common.h"
#include "kernels.h"

namespace cml {
namespace {
using namespace c1;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

// f of one B fragment (8 channels k0 .. k0 + 7 of one pixel); sc / bi: the channels' coefficients
// MASKED: a (bit ? x : 0) + c, else max(x sc + bi, 0)
template <bool MASKED>
__device__ __forceinline__ bf16x8_t prologue(bf16x8_t v, const float (&sc)[8], const float (&bi)[8],
                                             uint32_t bits) {
  uint4 u = *reinterpret_cast<const uint4*>(&v);
  uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float lo, hi;
    if constexpr (MASKED) {
      const float glo = ((bits >> (2 * i)) & 1u) ? __uint_as_float(w4[i] << 16) : 0.f;
      const float ghi = ((bits >> (2 * i + 1)) & 1u) ? __uint_as_float(w4[i] & 0xffff0000u) : 0.f;
      lo = fmaf(sc[2 * i], glo, bi[2 * i]);
      hi = fmaf(sc[2 * i + 1], ghi, bi[2 * i + 1]);
    } else {
      lo = fmaxf(fmaf(__uint_as_float(w4[i] << 16), sc[2 * i], bi[2 * i]), 0.f);
      hi = fmaxf(fmaf(__uint_as_float(w4[i] & 0xffff0000u), sc[2 * i + 1], bi[2 * i + 1]), 0.f);
    }
    w4[i] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
  }
  u = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  return *reinterpret_cast<const bf16x8_t*>(&u);
}

// BM x BN tile, waves of 64 (m) x WTN (n). PM: prologue; SM: statistics / epilogue mode; EL:
// masked residual-link epilogue (conv1x1_common.h).
// TL: the prologue is applied once per k-step to the staged x tile in LDS by all threads (then a
// barrier) instead of on every wave's B fragments (each x fragment is read by BN / WTN waves).
template <int BM, int BN, int WTN, int PM, int SM, bool EL, bool TL>
__global__ __launch_bounds__(BM * BN / WTN, 1) void conv1x1g_kernel(C1Args a) {
  constexpr int WN = BN / WTN, WM = BM / 64, NW = WN * WM, NT = NW * 64;
  constexpr int NI = WTN / 32;                                   // accumulator rows (n) per wave
  constexpr int QA = BM / (8 * NW), QB = BN / (8 * NW);          // glds per wave per k-step
  static_assert(QA * 8 * NW == BM && QB * 8 * NW == BN, "rows split evenly over the waves");
  static_assert(WTN % 64 == 0, "the epilogue works on 64-channel halves");
  constexpr bool CAT = PM == PM_CAT;
  static_assert(!CAT || BM / NW == 32, "one 4-byte glds per wave stages the k-step's mask bytes");
  constexpr int SX = BM * 128, SW = BN * 128, SMK = CAT ? BM * 8 : 0;
  constexpr int SB = SX + SW + SMK;                              // one staging buffer
  static_assert(NW * 8192 <= 2 * SB, "the epilogue images fit the staging area");
  constexpr bool DM = CAT && SM == SM_BNBWD;                     // ReLU bit recomputed from z
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_aff = reinterpret_cast<float*>(smem + 2 * SB);        // [2][K] prologue coefficients

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;
  const int h = lane >> 5, r32 = lane & 31;
  // bijective XCD remap: consecutive tile ids share an XCD
  const int G = a.ntn * a.mtiles, b = blockIdx.x, xcd = b & 7, q8 = G >> 3, r8 = G & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int mt = t / a.ntn, nt = t - mt * a.ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int K = a.K, KS = K / kBK;
  const int K1 = CAT ? a.K1 : K;

  if constexpr (PM != PM_NONE) {
    for (int k = tid; k < K; k += NT) {
      s_aff[k] = a.pro_sc[k];
      s_aff[K + k] = a.pro_bi[k];
    }
  }
  // this lane's staged rows (clamped: rows past M load row M - 1; their products are dropped)
  const int p = lane & 7, lrow = lane >> 3;
  int64_t xr[QA];
#pragma unroll
  for (int i = 0; i < QA; ++i) {
    const int m = m0 + wave * (BM / NW) + 8 * i + lrow;
    xr[i] = m < a.M ? m : a.M - 1;
  }
  const int64_t mrow = CAT ? ((m0 + wave * 32 + (lane >> 1)) < a.M ? m0 + wave * 32 + (lane >> 1)
                                                                   : a.M - 1)
                           : 0;

  auto issue = [&](int ks, int buf) {
    char* base = smem + buf * SB;
    const bool first = !CAT || ks * kBK < K1;
#pragma unroll
    for (int i = 0; i < QA; ++i) {
      const int row = wave * (BM / NW) + 8 * i + lrow;
      const int c = p ^ ((row >> 1) & 7);
      const uint16_t* src;
      if constexpr (CAT)
        src = first ? a.x + xr[i] * K1 + ks * kBK + 8 * c
                    : a.x2 + xr[i] * (K - K1) + (ks * kBK - K1) + 8 * c;
      else
        src = a.x + xr[i] * K + ks * kBK + 8 * c;
      __builtin_amdgcn_global_load_lds((g_void*)src,
                                       (lds_void*)(base + (wave * (BM / NW) + 8 * i) * 128), 16, 0,
                                       0);
    }
#pragma unroll
    for (int i = 0; i < QB; ++i) {
      const int row = wave * (BN / NW) + 8 * i + lrow;
      const int c = p ^ ((row >> 1) & 7);
      const uint16_t* src = a.w + static_cast<int64_t>(n0 + row) * K + ks * kBK + 8 * c;
      __builtin_amdgcn_global_load_lds((g_void*)src,
                                       (lds_void*)(base + SX + (wave * (BN / NW) + 8 * i) * 128),
                                       16, 0, 0);
    }
    // 8 mask bytes per pixel row (the second source's steps re-read step 0's); none when both
    // sources are BN + ReLU outputs (cat_bnrelu: no mask tensor)
    if (CAT && !a.cat_bnrelu) {
      const uint8_t* src = a.xm + mrow * (K1 / 8) + (first ? ks * 8 : 0) + 4 * (lane & 1);
      __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(base + SX + SW + wave * 256), 4,
                                       0, 0);
    }
  };

  f32x16 acc[NI][2];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      acc[i][0][k] = 0.f;
      acc[i][1][k] = 0.f;
    }

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                       // step 0 and the coefficient table visible
  for (int ks = 0; ks < KS; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < KS) issue(ks + 1, buf ^ 1);
    const char* sx = smem + buf * SB;
    const char* sw = sx + SX;
    const uint8_t* smk = reinterpret_cast<const uint8_t*>(sw + SW);
    const bool masked = CAT && ks * kBK < K1 && !a.cat_bnrelu;
    if constexpr (TL && PM != PM_NONE) {
      // thread: logical 16-B chunk tid & 7 (8 channels) of rows tid / 8 + NT / 8 * i, in place
      char* sxw = smem + buf * SB;
      const int c = tid & 7;
      float sc[8], bi[8];
      ld8f(s_aff + ks * kBK + 8 * c, sc);
      ld8f(s_aff + K + ks * kBK + 8 * c, bi);
#pragma unroll
      for (int i = 0; i < BM / (NT / 8); ++i) {
        const int row = (tid >> 3) + (NT / 8) * i;
        bf16x8_t* q = reinterpret_cast<bf16x8_t*>(sxw + swz(row, c));
        if (masked) *q = prologue<true>(*q, sc, bi, smk[row * 8 + c]);
        else *q = prologue<false>(*q, sc, bi, 0u);
      }
      // LDS writes visible to every wave; a raw barrier, so the DMA of step ks + 1 stays in
      // flight (__syncthreads would wait for it)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int kk = 0; kk < kBK / 16; ++kk) {
      bf16x8_t A[NI], B[2];
#pragma unroll
      for (int i = 0; i < NI; ++i)
        A[i] = *reinterpret_cast<const bf16x8_t*>(sw + swz(wn * WTN + 32 * i + r32, 2 * kk + h));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        B[j] = *reinterpret_cast<const bf16x8_t*>(sx + swz(wm * 64 + 32 * j + r32, 2 * kk + h));
      if constexpr (PM != PM_NONE && !TL) {
        const int k0 = ks * kBK + 16 * kk + 8 * h;   // this lane's 8 channels
        float sc[8], bi[8];
        ld8f(s_aff + k0, sc);
        ld8f(s_aff + K + k0, bi);
        if (masked) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            B[j] = prologue<true>(B[j], sc, bi, smk[(wm * 64 + 32 * j + r32) * 8 + 2 * kk + h]);
        } else {
#pragma unroll
          for (int j = 0; j < 2; ++j) B[j] = prologue<false>(B[j], sc, bi, 0u);
        }
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(A[i], B[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: the wave's 64 (m) x WTN (n) block, 64 channels at a time, through its own 8 KB image
  char* simg = smem + wave * 8192;
  constexpr bool STATS = SM == SM_BN || SM == SM_BNBWD;
  float ss[8], sq[8], sh[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    ss[q] = 0.f;
    sq[q] = 0.f;
    sh[q] = 0.f;
  }
#pragma unroll
  for (int sb = 0; sb < WTN / 64; ++sb) {
    const int ncol0 = wn * WTN + 64 * sb;
    if constexpr (STATS) {
      if (a.shift) {
#pragma unroll
        for (int q = 0; q < 8; ++q) sh[q] = a.shift[n0 + ncol0 + 8 * (lane & 7) + q];
      }
    }
    f32x16 blk[2][2] = {{acc[2 * sb][0], acc[2 * sb][1]}, {acc[2 * sb + 1][0], acc[2 * sb + 1][1]}};
    epilogue<EL, SM, 2, DM>(a, blk, ss, sq, sh, simg, m0 + wm * 64, ncol0, n0, lane);
    if (STATS && a.part) {   // (SM_BN without a slab: the conv only, no statistics)
      // fold the 8 lanes sharing a channel group (lane & 7): one partial row per (m-tile, wm)
      float* pp = a.part + (static_cast<int64_t>(nt) * a.mtiles * WM + mt * WM + wm) * 2 * BN;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float sv = ss[q], qv = sq[q];
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) {
          sv += __shfl_xor(sv, o, 64);
          qv += __shfl_xor(qv, o, 64);
        }
        if (lane < 8) {
          pp[ncol0 + 8 * lane + q] = sv;
          pp[BN + ncol0 + 8 * lane + q] = qv;
        }
        ss[q] = 0.f;
        sq[q] = 0.f;
      }
    }
  }
}

struct GPlan {
  int BM, BN, WTN, ntn, mtiles;
  size_t lds;
};

GPlan gplan(int64_t M, int K, int N, int pm) {
  GPlan p{};
  p.BM = 256;
  p.BN = N % 256 == 0 ? 256 : 128;
  p.WTN = p.BN == 256 ? 128 : 64;
  p.ntn = N / p.BN;
  p.mtiles = static_cast<int>((M + p.BM - 1) / p.BM);
  const size_t sb = static_cast<size_t>(p.BM + p.BN) * 128 + (pm == PM_CAT ? p.BM * 8 : 0);
  p.lds = 2 * sb + (pm != PM_NONE ? static_cast<size_t>(2) * K * 4 : 0);
  return p;
}

template <int BN, int WTN, int PM, int SM, bool EL>
hipError_t launch_k(const C1Args& a, const GPlan& p, hipStream_t st) {
  auto k = &conv1x1g_kernel<256, BN, WTN, PM, SM, EL, true>;
  if constexpr (PM != PM_NONE) {
    static const bool frag = [] {   // CML_C1G_FRAG=1: prologue on the B fragments (A/B)
      const char* e = getenv("CML_C1G_FRAG");
      return e && e[0] == '1';
    }();
    if (frag) k = &conv1x1g_kernel<256, BN, WTN, PM, SM, EL, false>;
  }
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(p.lds));
  k<<<p.ntn * p.mtiles, 256 * BN / WTN, p.lds, st>>>(a);
  return hipGetLastError();
}

template <int PM, int SM, bool EL>
hipError_t launch_m(const C1Args& a, const GPlan& p, hipStream_t st) {
  return p.BN == 256 ? launch_k<256, 128, PM, SM, EL>(a, p, st)
                     : launch_k<128, 64, PM, SM, EL>(a, p, st);
}

}  // namespace

namespace {
int g_mode = -1;   // 0 off, 1 wherever eligible, 2 auto (the shape policy below)
}  // namespace

int conv1x1g_mode() {
  if (g_mode < 0) {
    const char* e = getenv("CML_C1G");
    g_mode = (!e || !strcmp(e, "auto")) ? 2 : (atoi(e) ? 1 : 0);
  }
  return g_mode;
}

void set_conv1x1g_mode(int mode) { g_mode = mode; }

bool conv1x1g_eligible(int64_t M, int K, int N, int pm) {
  if (K % kBK || N % 128 || K < kBK || M < 1 || M >= (1ll << 31) || N > 4096) return false;
  const GPlan p = gplan(M, K, N, pm);
  return p.lds <= 160 * 1024 && static_cast<int64_t>(p.ntn) * p.mtiles < (1ll << 31);
}

bool conv1x1g_pick(int64_t M, int K, int N, int pm) {
  const int mode = conv1x1g_mode();
  if (mode == 0 || !conv1x1g_eligible(M, K, N, pm)) return false;
  if (mode == 1) return true;
  // auto: the GEMMs where conv1x1.hip's register-staged pipeline is compute-limited. The
  // persistent kernel keeps streaming while it runs epilogues, so it stays on the HBM-bound shapes
  // (few k-steps per tile).
  return K >= 256;
}

size_t conv1x1g_part_floats(int64_t M, int K, int N, int pm) {
  const GPlan p = gplan(M, K, N, pm);
  const int R = p.mtiles * (p.BM / 64);
  return static_cast<size_t>(p.ntn) * (static_cast<size_t>(R) + bn_part_fold_slices(R, p.ntn)) *
         2 * p.BN;
}

hipError_t launch_conv1x1g(const C1Args& a0, int pm, int sm, bool el, hipStream_t st, int* R,
                           int* BN) {
  const GPlan p = gplan(a0.M, a0.K, a0.N, pm);
  C1Args a = a0;
  a.ntn = p.ntn;
  a.mtiles = p.mtiles;
  a.wgpn = 0;
  *R = p.mtiles * (p.BM / 64);
  *BN = p.BN;
  if (pm == PM_NONE && sm == SM_BN && !el) return launch_m<PM_NONE, SM_BN, false>(a, p, st);
  if (pm == PM_BNRELU && sm == SM_BN && !el) return launch_m<PM_BNRELU, SM_BN, false>(a, p, st);
  if (pm == PM_BNRELU && sm == SM_BNRES && !el) return launch_m<PM_BNRELU, SM_BNRES, false>(a, p, st);
  if (pm == PM_NONE && sm == SM_OFF && el) return launch_m<PM_NONE, SM_OFF, true>(a, p, st);
  if (pm == PM_NONE && sm == SM_BNBWD && el) return launch_m<PM_NONE, SM_BNBWD, true>(a, p, st);
  if (pm == PM_CAT && sm == SM_OFF && !el) return launch_m<PM_CAT, SM_OFF, false>(a, p, st);
  if (pm == PM_CAT && sm == SM_BNRES && !el) return launch_m<PM_CAT, SM_BNRES, false>(a, p, st);
  if (pm == PM_CAT && sm == SM_BNBWD && !el) return launch_m<PM_CAT, SM_BNBWD, false>(a, p, st);
  return hipErrorInvalidValue;
}

}  // namespace cml
