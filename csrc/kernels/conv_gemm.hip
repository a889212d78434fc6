// Implicit-GEMM NHWC convolution, stride 1 or 2, 1x1 or 3x3 (padding 1), on MFMA with both operands
// staged by global_load_lds into two LDS buffers:
//
//   y[m][n] = sum_{tap, c} x[src(m, tap)][c] * w[n][tap * C + c]
//
// (a 3x3 data gradient is this with dy as x and the rotated, transposed weights). Design
// (gfx950): a workgroup of BM BN / 4096 waves owns a BM (pixels) x BN (channels) tile, every wave a 64 x 64
// block = 2 x 2 v_mfma_f32_32x32x16_bf16 accumulators; one k-step = 64 input channels of one
// tap. The k-step ks + 1 is copied global -> LDS by the DMA path (global_load_lds_dwordx4: 8 rows
// x 128 B per wave instruction, no VGPR staging) while step ks is multiplied, and retired by one
// vmcnt(0) + barrier per step. Rows are gathered per lane (the global source address is per
// lane): padded taps and rows past M read a zero row. The LDS image is lane-linear, so the bank
// swizzle lives in the SOURCE address: lane p of a row loads chunk p ^ ((row >> 1) & 7), and the
// fragment reads use the same involution (conv1x1.hip's swz). The fp32 accumulators go out through
// a per-wave LDS image as whole-line 16-B stores. Tiles are mapped XCD-aware (the n-tiles of one
// m-tile are consecutive on one XCD: x comes from HBM once and from that XCD's L2 after).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

constexpr int kBK = 64;

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int swz(int row, int c) { return row * 128 + 16 * (c ^ ((row >> 1) & 7)); }

struct GArgs {
  const uint16_t* x;      // [rows][C]
  const uint16_t* w;      // [N][TAPS * C]
  uint16_t* y;            // [M][N]
  const uint16_t* zero;   // >= 64 zero elements
  float* part;            // ST: [ntn][mtiles * WM][2][BN] shifted sums of the bf16 output
  const float* shift;     // ST: [N] statistics shift (the BN running mean) or null; BB: the BN's mean
  const uint16_t* sz;     // BB: input z [M][N] of the BN + ReLU whose output gradient y is
  const float* ep_sc;     // BB: that BN's affine [N] (ReLU bit: z ep_sc + ep_bi > 0)
  const float* ep_bi;
  int M, C, N, H, W, HW;   // H, W: output
  int S, IH, IW, IHW;     // stride; input height, width and pixels per image
  int KS;                 // TAPS * C / 64
  int ntn, tiles;
  // PAR (stride-2 3x3 data gradient, one output parity class per launch): the class (py, px), the
  // weight row stride (9 C), and this class's rows of the statistics slab (total rows per n-tile,
  // first row)
  int py, px, wld, prt, prb;
};

// NBUF = 2: the DMA of step ks + 1 overlaps step ks, retired by vmcnt(0) + barrier per step.
// NBUF = 3: steps ks + 1 and ks + 2 in flight; a counted vmcnt (this wave's instructions of one
// step) + a raw s_barrier retires only step ks + 1 (a __syncthreads() would drain the queue).
// WTN: output channels per wave (64: 2 x 2 accumulators; 128: 4 x 2, half the x-fragment reads
// per MFMA).
// ST: the epilogue also accumulates the BN statistics (sum, sum of squares of y_bf16 - shift) of
// the stored values per channel and writes one partial row per (m-tile, wave row).
// BB (with ST): instead the sums of the backward of the BN + ReLU whose output gradient y is (a
// data gradient): s = sum y', q = sum y' (z - mean) with y' = (z ep_sc + ep_bi > 0) ? y : 0, the
// ReLU bit recomputed from the BN input z -- that BN's backward then needs no reduction pass.
// PAR: the data gradient of a stride-2 / padding-1 3x3 conv with an even input, one output parity
// class (py, px) per launch. dx[2 m + py][2 l + px] gathers dy only through the taps of matching
// parity: along an axis, parity 0 takes ky = 1 from dy row m, parity 1 takes ky = 0 from row m + 1
// and ky = 2 from row m; so the classes run 1 / 2 / 2 / 4 taps (9 in total, no multiply by a
// structural zero). x = dy (C = its channels, output grid = dy's grid), w = the rotated,
// transposed layout wr [N][9 C] of the data gradient; output rows go to dx's pixels of the class.
template <int BM, int BN, int TAPS, int NBUF = 2, int WTN = 64, bool ST = false, bool BB = false,
          bool PAR = false>
__global__ __launch_bounds__(BM * BN / WTN, 1) void conv_gemm_kernel(GArgs a) {
  constexpr int WN = BN / WTN, WM = BM / 64, NW = WN * WM;
  constexpr int NI = WTN / 32;                  // accumulator rows (n) per wave
  constexpr int QA = BM / (8 * NW), QB = BN / (8 * NW);   // glds instructions per wave per step
  static_assert(QA * 8 * NW == BM && QB * 8 * NW == BN, "rows split evenly over the waves");
  constexpr int SB = (BM + BN) * 128;           // one LDS buffer: x tile then w tile
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;
  const int h = lane >> 5, r32 = lane & 31;
  // bijective XCD remap: consecutive tile ids share an XCD
  const int G = a.tiles, b = blockIdx.x, xcd = b & 7, q8 = G >> 3, r8 = G & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int mt = t / a.ntn, nt = t - mt * a.ntn;
  const int m0 = mt * BM, n0 = nt * BN;

  // this lane's staged rows: x rows wave * (BM / NW) + 8 i + lane / 8, w rows likewise
  const int p = lane & 7, lrow = lane >> 3;
  int pimg[QA], poh[QA], pow_[QA];
#pragma unroll
  for (int i = 0; i < QA; ++i) {
    const int m = m0 + wave * (BM / NW) + 8 * i + lrow;
    if (m < a.M) {
      const int img = m / a.HW, rem = m - img * a.HW;
      pimg[i] = img * a.IHW;
      poh[i] = rem / a.W;
      pow_[i] = rem - poh[i] * a.W;
    } else {
      pimg[i] = -1;
      poh[i] = 0;
      pow_[i] = 0;
    }
  }

  const int wld = PAR ? a.wld : a.KS * kBK;
  auto issue = [&](int ks, int buf) {
    const int CS = a.C >> 6;
    const int tap = TAPS == 1 ? 0 : ks / CS;
    const int cc = ks - tap * CS;
    int dy = TAPS == 1 ? 0 : tap / 3 - 1, dx = TAPS == 1 ? 0 : tap - 3 * (tap / 3) - 1;
    int wcol = ks * kBK;
    if constexpr (PAR) {
      const int tyi = a.px ? (tap >> 1) : tap, txi = a.px ? (tap & 1) : 0;
      const int ky = a.py ? (tyi ? 2 : 0) : 1, kx = a.px ? (txi ? 2 : 0) : 1;
      dy = (a.py && tyi == 0) ? 1 : 0;
      dx = (a.px && txi == 0) ? 1 : 0;
      wcol = (3 * (2 - ky) + (2 - kx)) * a.C + cc * kBK;   // wr's tap (2 - ky, 2 - kx)
    }
    char* base = smem + buf * SB;
#pragma unroll
    for (int i = 0; i < QA; ++i) {
      const int row = wave * (BM / NW) + 8 * i + lrow;
      const int ih = a.S * poh[i] + dy, iw = a.S * pow_[i] + dx;
      const bool ok = pimg[i] >= 0 && static_cast<unsigned>(ih) < static_cast<unsigned>(a.IH) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(a.IW);
      const int c = p ^ ((row >> 1) & 7);
      const uint16_t* src = ok ? a.x + (static_cast<int64_t>(pimg[i]) + ih * a.IW + iw) * a.C +
                                     cc * kBK + 8 * c
                               : a.zero;
      __builtin_amdgcn_global_load_lds((g_void*)src,
                                       (lds_void*)(base + (wave * (BM / NW) + 8 * i) * 128), 16, 0,
                                       0);
    }
    char* wb = base + BM * 128;
#pragma unroll
    for (int i = 0; i < QB; ++i) {
      const int row = wave * (BN / NW) + 8 * i + lrow;
      const int c = p ^ ((row >> 1) & 7);
      const uint16_t* src = a.w + static_cast<int64_t>(n0 + row) * wld + wcol + 8 * c;
      __builtin_amdgcn_global_load_lds((g_void*)src,
                                       (lds_void*)(wb + (wave * (BN / NW) + 8 * i) * 128), 16, 0, 0);
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
  if constexpr (NBUF == 3) {
    if (a.KS > 1) {
      issue(1, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QA + QB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int ks = 0; ks < a.KS; ++ks) {
    const int buf = NBUF == 3 ? ks % 3 : (ks & 1);
    if constexpr (NBUF == 3) {
      if (ks + 2 < a.KS) issue(ks + 2, (ks + 2) % 3);
    } else {
      if (ks + 1 < a.KS) issue(ks + 1, buf ^ 1);
    }
    const char* sx = smem + buf * SB;
    const char* sw = sx + BM * 128;
#pragma unroll
    for (int kk = 0; kk < kBK / 16; ++kk) {
      bf16x8_t A[NI], B[2];
#pragma unroll
      for (int i = 0; i < NI; ++i)
        A[i] = *reinterpret_cast<const bf16x8_t*>(sw + swz(wn * WTN + 32 * i + r32, 2 * kk + h));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        B[j] = *reinterpret_cast<const bf16x8_t*>(sx + swz(wm * 64 + 32 * j + r32, 2 * kk + h));
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(A[i], B[j], acc[i][j]);
    }
    if constexpr (NBUF == 3) {
      // retire step ks + 1 (this wave's loads of step ks + 2 may stay in flight); the barrier also
      // ends every wave's reads of buffer ks % 3 before step ks + 1 re-issues into it
      if (ks + 2 < a.KS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QA + QB) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // epilogue: the wave's WTN (n) x 64 (m) block, 64 channels at a time, via its own 8 KB LDS image
  // (the staging buffers are free now)
  char* simg = smem + wave * 8192;
  const int c = lane & 7;
  const int mb = m0 + wm * 64;
  // output row of GEMM row m (PAR: the class pixel of dx, a 2H x 2W image)
  auto orow = [&](int m) -> int64_t {
    if constexpr (PAR) {
      const int img = m / a.HW, rem = m - img * a.HW;
      const int oh = rem / a.W, ow = rem - oh * a.W;
      return static_cast<int64_t>(img) * 4 * a.HW + (2 * oh + a.py) * (2 * a.W) + 2 * ow + a.px;
    } else {
      return m;
    }
  };
#pragma unroll
  for (int sb = 0; sb < WTN / 64; ++sb) {
#pragma unroll
    for (int jm = 0; jm < 2; ++jm) {
      const int pr = 32 * jm + r32;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x16& v = acc[2 * sb + i][jm];
          const uint32_t b0 = f2bf(v[4 * g + 0]), b1 = f2bf(v[4 * g + 1]);
          const uint32_t b2 = f2bf(v[4 * g + 2]), b3 = f2bf(v[4 * g + 3]);
          *reinterpret_cast<uint2*>(simg + swz(pr, 4 * i + g) + 8 * h) =
              make_uint2(b0 | (b1 << 16), b2 | (b3 << 16));
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int cb = n0 + wn * WTN + 64 * sb + 8 * c;   // this lane's 8 channels
    float sh[8], ss[8], sq[8], esc[8], ebi[8];
    if constexpr (ST) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        sh[q] = a.shift ? a.shift[cb + q] : 0.f;
        ss[q] = 0.f;
        sq[q] = 0.f;
        if constexpr (BB) {
          esc[q] = a.ep_sc[cb + q];
          ebi[q] = a.ep_bi[cb + q];
        }
      }
    }
    // BB: the 8 rows' z chunks issued together (rows past M re-read row M - 1)
    uint4 zr[BB ? 8 : 1];
    if constexpr (BB) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int m = mb + 8 * k + (lane >> 3);
        zr[k] = *reinterpret_cast<const uint4*>(a.sz + orow(m < a.M ? m : a.M - 1) * a.N + cb);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int pr = 8 * k + (lane >> 3);
      const uint4 v = *reinterpret_cast<const uint4*>(simg + swz(pr, c));
      if (mb + pr < a.M) {
        *reinterpret_cast<uint4*>(a.y + orow(mb + pr) * a.N + cb) = v;
        if constexpr (BB) {
          const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
          const uint32_t z4[4] = {zr[k].x, zr[k].y, zr[k].z, zr[k].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float zlo = __uint_as_float(z4[q] << 16);
            const float zhi = __uint_as_float(z4[q] & 0xffff0000u);
            const float lo = fmaf(zlo, esc[2 * q], ebi[2 * q]) > 0.f ? __uint_as_float(w4[q] << 16) : 0.f;
            const float hi = fmaf(zhi, esc[2 * q + 1], ebi[2 * q + 1]) > 0.f
                                 ? __uint_as_float(w4[q] & 0xffff0000u) : 0.f;
            ss[2 * q] += lo;
            ss[2 * q + 1] += hi;
            sq[2 * q] = fmaf(lo, zlo - sh[2 * q], sq[2 * q]);
            sq[2 * q + 1] = fmaf(hi, zhi - sh[2 * q + 1], sq[2 * q + 1]);
          }
        } else if constexpr (ST) {
          const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = __uint_as_float(w4[q] << 16) - sh[2 * q];
            const float hi = __uint_as_float(w4[q] & 0xffff0000u) - sh[2 * q + 1];
            ss[2 * q] += lo;
            ss[2 * q + 1] += hi;
            sq[2 * q] = fmaf(lo, lo, sq[2 * q]);
            sq[2 * q + 1] = fmaf(hi, hi, sq[2 * q + 1]);
          }
        }
      }
    }
    if constexpr (ST) {
      // fold the 8 lanes sharing a channel group (lane & 7), one partial row per (m-tile, wm)
      const int prt = PAR ? a.prt : (a.tiles / a.ntn) * WM, prb = PAR ? a.prb : 0;
      float* pp = a.part + (static_cast<int64_t>(nt) * prt + prb + mt * WM + wm) * 2 * BN;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float sv = ss[q], qv = sq[q];
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) {
          sv += __shfl_xor(sv, o, 64);
          qv += __shfl_xor(qv, o, 64);
        }
        if (lane < 8) {
          const int col = wn * WTN + 64 * sb + 8 * lane + q;
          pp[col] = sv;
          pp[BN + col] = qv;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

template <int BM, int BN, int TAPS, int NBUF, int WTN = 64>
hipError_t launch_g(const GArgs& a, hipStream_t st) {
  auto k = !a.part ? &conv_gemm_kernel<BM, BN, TAPS, NBUF, WTN, false>
            : (a.sz ? &conv_gemm_kernel<BM, BN, TAPS, NBUF, WTN, true, true>
                    : &conv_gemm_kernel<BM, BN, TAPS, NBUF, WTN, true>);
  const size_t lds = NBUF * static_cast<size_t>(BM + BN) * 128;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  k<<<a.tiles, BM * BN / WTN, lds, st>>>(a);
  return hipGetLastError();
}

// CML_CONV_GEMM_VARIANT (A/B): 0 = 128 x 128, 2 buffers; 1 = 128 x 128, 3 buffers;
// 2 = 256 x 128 (8 waves), 2 buffers; 3 = 256 x 128, 3 buffers; 4 (default) = 256 x 256, 8 waves
// of 64 x 128 (N % 256 == 0, else 2). N % 128 != 0: 256 x 64.
// Measured on the ResNet-50 3x3 shapes at batch 2048 (bench/conv3x3.py, profiles/r02_conv_gemm24/,
// r02_conv_gemm30/): 2 beats 0, 1, 3 (the third buffer does not pay here); 4 is 13-17 % faster
// than 2 on the 256 / 512-channel layers (3x3 data gradient 0.52 ms vs MIOpen 0.71-0.74).
int gemm_variant() {
  static const int v = [] {
    const char* e = getenv("CML_CONV_GEMM_VARIANT");
    return e ? atoi(e) : 4;
  }();
  return v;
}

// CML_CONV_GEMM_NARROW (A/B, N % 128 != 0): 0 (default) = 256 x 64, 2 buffers; 1 = 256 x 64,
// 3 buffers; 2 = 128 x 64, 2 buffers; 3 = 128 x 64, 3 buffers
int narrow_variant() {
  static const int v = [] {
    const char* e = getenv("CML_CONV_GEMM_NARROW");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// Small-M shapes (the layer-3 / 4 convs at batch 256: 98-196 tiles of 256 x 256 for 256 CUs) take
// smaller tiles when the 256 x 256 grid has fewer than CML_CONV_GEMM_SMALLM tiles (default 512;
// 0 disables): variant CML_CONV_GEMM_SMALLV (default 0 = 128 x 128, 2 workgroups per CU).
int smallm_tiles() {
  static const int v = [] {
    const char* e = getenv("CML_CONV_GEMM_SMALLM");
    return e ? atoi(e) : 512;
  }();
  return v;
}
int smallm_variant() {
  static const int v = [] {
    const char* e = getenv("CML_CONV_GEMM_SMALLV");
    return e ? atoi(e) : 0;
  }();
  return v;
}

int pick_variant(int64_t M, int N, int* BM, int* BN);

// CML_CONV_GEMM2 (A/B, default 1; profiles/r04_12: 3x3 class 23.00 -> 22.60 ms per step):
// stride-1 3x3 convs whose 256 x 256 grid is used (variant 4)
// and whose pixel count is a multiple of 256 run on gemm.hip's schedule instead (launch_gemm_conv:
// 16x16x32 MFMAs, four staggered phases per k-tile with 4 DMA units in flight and counted vmcnt,
// no per-step drain) with the same epilogues
// The 128-channel convs (layer 2: variant 2's 256 x 128 tiles, 0.6-0.67 PFLOP/s) take gemm.hip's
// 512 x 128 tile when the grid has enough of them (gemm_conv_tm == 512).
// Returns the m-tile (256 / 512) or 0.
int use_gemm2(int64_t M, int N, int C, int taps, int stride) {
  static const bool on = [] {
    const char* e = getenv("CML_CONV_GEMM2");
    return !e || e[0] != '0';
  }();
  // CML_GEMM2_S2=0: the stride-2 forwards stay on conv_gemm.hip (A/B)
  static const bool s2 = [] {
    const char* e = getenv("CML_GEMM2_S2");
    return !e || e[0] != '0';
  }();
  if (!on || taps != 9 || (stride != 1 && !(stride == 2 && s2))) return 0;
  const int tm = gemm_conv_tm(M, N, C);
  if (tm == 512) return 512;
  // (stride 2 on the square tile measured no faster than conv_gemm.hip's 256 x 256: 529.7 vs
  // 528.4 us for the layer-3 / 4 forwards, profiles/r05_47/: the tall tile only)
  if (stride == 2) return 0;
  int BM = 0, BN = 0;
  return tm == 256 && pick_variant(M, N, &BM, &BN) == 4 ? 256 : 0;
}

// the variant and tile (BM, BN) for an M x N output
int pick_variant(int64_t M, int N, int* BM, int* BN) {
  const bool wide = N % 128 == 0;
  int v = wide ? gemm_variant() : 0;
  if (v == 4 && N % 256) v = 2;                   // 256 x 256 tiles need N % 256 == 0
  if (v == 4 && smallm_tiles() > 0 && (M + 255) / 256 * (N / 256) < smallm_tiles())
    v = smallm_variant();
  *BM = !wide ? (narrow_variant() >= 2 ? 128 : 256) : (v >= 2 ? 256 : 128);
  *BN = v == 4 ? 256 : (wide ? 128 : 64);
  return v;
}

template <int TAPS>
hipError_t launch_v(GArgs& a, int64_t M, hipStream_t st) {
  const bool wide = a.N % 128 == 0;
  int BM, BN;
  const int v = pick_variant(M, a.N, &BM, &BN);
  a.ntn = a.N / BN;
  const int64_t tiles = (M + BM - 1) / BM * a.ntn;
  if (tiles >= (1ll << 31)) return hipErrorInvalidValue;
  a.tiles = static_cast<int>(tiles);
  if (!wide) {
    switch (narrow_variant()) {
      case 1: return launch_g<256, 64, TAPS, 3>(a, st);
      case 2: return launch_g<128, 64, TAPS, 2>(a, st);
      case 3: return launch_g<128, 64, TAPS, 3>(a, st);
      default: return launch_g<256, 64, TAPS, 2>(a, st);
    }
  }
  switch (v) {
    case 1: return launch_g<128, 128, TAPS, 3>(a, st);
    case 2: return launch_g<256, 128, TAPS, 2>(a, st);
    case 3: return launch_g<256, 128, TAPS, 3>(a, st);
    case 4: return launch_g<256, 256, TAPS, 2, 128>(a, st);
    default: return launch_g<128, 128, TAPS, 2>(a, st);
  }
}

}  // namespace

namespace {
// the tile (BM, BN) launch_v picks for M x N
void tile_of(int64_t M, int N, int* BM, int* BN) { (void)pick_variant(M, N, BM, BN); }
}  // namespace

size_t conv_gemm_part_floats(int64_t M, int N) {
  int BM, BN;
  tile_of(M, N, &BM, &BN);
  const int64_t mtiles = (M + BM - 1) / BM;
  const int R = static_cast<int>(mtiles * (BM / 64));
  // the slab, then the fold area of launch_bn_stats_finalize
  size_t g = static_cast<size_t>(N / BN) *
             (static_cast<size_t>(R) + bn_part_fold_slices(R, N / BN)) * 2 * BN;
  // gemm.hip's slab when a 3x3 conv of this M x N runs there (use_gemm2)
  if (const int tm = M % 64 == 0 ? gemm_conv_tm(M, N, 64) : 0) {
    const int tn = 65536 / tm, R2 = static_cast<int>(M / tm) * (tm / 128);
    g = std::max(g, static_cast<size_t>(N / tn) *
                        (static_cast<size_t>(R2) + bn_part_fold_slices(R2, N / tn)) * 2 * tn);
  }
  return N == 64 && g < conv3x3p_part_floats() ? conv3x3p_part_floats() : g;
}

hipError_t launch_conv_gemm(const void* x, const void* w, void* y, const void* zero, int Nimg,
                            int H, int W, int C, int N, int taps, hipStream_t st, float* part,
                            const float* shift, float* mean, float* invstd, float* rmean,
                            float* rvar, float eps, float momentum, int stride,
                            const BnAffineOut* aff) {
  if (stride != 1 && stride != 2) return hipErrorInvalidValue;
  const int OH = (H - 1) / stride + 1, OW = (W - 1) / stride + 1;
  const int64_t M = static_cast<int64_t>(Nimg) * OH * OW;
  if (C % kBK || N % 64 || (taps != 1 && taps != 9) || M < 1 || M >= (1ll << 31) ||
      static_cast<int64_t>(Nimg) * H * W >= (1ll << 31) || static_cast<int64_t>(taps) * C > 65536)
    return hipErrorInvalidValue;
  GArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.w = reinterpret_cast<const uint16_t*>(w);
  a.y = reinterpret_cast<uint16_t*>(y);
  a.zero = reinterpret_cast<const uint16_t*>(zero);
  a.M = static_cast<int>(M);
  a.C = C;
  a.N = N;
  a.H = OH;
  a.W = OW;
  a.HW = OH * OW;
  a.S = stride;
  a.IH = H;
  a.IW = W;
  a.IHW = H * W;
  a.KS = taps * C / kBK;
  a.part = part;
  a.shift = shift;
  if (conv3x3p_eligible(Nimg, H, W, C, N, taps, stride)) {
    int R = 0;
    hipError_t e = launch_conv3x3p(x, w, y, zero, Nimg, H, part ? 1 : 0, part, shift, nullptr,
                                   nullptr, nullptr, st, &R);
    if (e != hipSuccess || !part || !mean) return e;
    return launch_bn_stats_finalize(part, R, 64, 64, M, shift, eps, momentum, mean, invstd, rmean,
                                    rvar, st, nullptr, aff);
  }
  if (const int tm = use_gemm2(M, N, C, taps, stride)) {
    GemmArgs g{};
    g.a = a.x;
    g.b = a.w;
    g.y = a.y;
    g.zero = a.zero;
    g.M = M;
    g.N = N;
    g.C = C;
    g.H = OH;
    g.W = OW;
    g.s2 = stride == 2 ? 1 : 0;
    g.IH = H;
    g.IW = W;
    g.part = part;
    g.shift = shift;
    hipError_t e = launch_gemm_conv(g, part ? EP_CONV_ST : EP_STORE, st);
    if (e != hipSuccess || !part || !mean) return e;
    const int tn = 65536 / tm, R = static_cast<int>(M / tm) * (tm / 128);
    return launch_bn_stats_finalize(part, R, tn, N, M, shift, eps, momentum, mean, invstd, rmean,
                                    rvar, st, part + static_cast<size_t>(N / tn) * R * 2 * tn, aff);
  }
  hipError_t e = taps == 1 ? launch_v<1>(a, M, st) : launch_v<9>(a, M, st);
  if (e != hipSuccess || !part || !mean) return e;
  int BM, BN;
  tile_of(M, N, &BM, &BN);
  const int R = static_cast<int>((M + BM - 1) / BM) * (BM / 64);
  return launch_bn_stats_finalize(part, R, BN, N, M, shift, eps, momentum, mean, invstd, rmean,
                                  rvar, st, part + static_cast<size_t>(N / BN) * R * 2 * BN, aff);
}

hipError_t launch_conv_gemm_bnsums(const void* x, const void* w, void* y, const void* zero,
                                   int Nimg, int H, int W, int C, int N, int taps, const void* z,
                                   const float* sc, const float* bi, const float* mean,
                                   const float* invstd, float* part, float* sdz, float* sdzx,
                                   hipStream_t st, void* dgamma, void* dbeta) {
  const int64_t M = static_cast<int64_t>(Nimg) * H * W;
  if (C % kBK || N % 64 || (taps != 1 && taps != 9) || M < 1 || M >= (1ll << 31) ||
      static_cast<int64_t>(taps) * C > 65536 || !z || !sc || !bi || !mean || !invstd || !part ||
      !sdz || !sdzx)
    return hipErrorInvalidValue;
  GArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.w = reinterpret_cast<const uint16_t*>(w);
  a.y = reinterpret_cast<uint16_t*>(y);
  a.zero = reinterpret_cast<const uint16_t*>(zero);
  a.M = static_cast<int>(M);
  a.C = C;
  a.N = N;
  a.H = H;
  a.W = W;
  a.HW = H * W;
  a.S = 1;
  a.IH = H;
  a.IW = W;
  a.IHW = H * W;
  a.KS = taps * C / kBK;
  a.part = part;
  a.shift = mean;
  a.sz = reinterpret_cast<const uint16_t*>(z);
  a.ep_sc = sc;
  a.ep_bi = bi;
  if (conv3x3p_eligible(Nimg, H, W, C, N, taps, 1)) {
    int R = 0;
    hipError_t e = launch_conv3x3p(x, w, y, zero, Nimg, H, 2, part, mean, z, sc, bi, st, &R);
    if (e != hipSuccess) return e;
    return launch_bnbwd_sums_finalize(part, R, 64, 64, invstd, sdz, sdzx, st, nullptr, dgamma,
                                      dbeta);
  }
  if (const int tm = use_gemm2(M, N, C, taps, 1)) {
    GemmArgs g{};
    g.a = a.x;
    g.b = a.w;
    g.y = a.y;
    g.zero = a.zero;
    g.M = M;
    g.N = N;
    g.C = C;
    g.H = H;
    g.W = W;
    g.part = part;
    g.shift = mean;
    g.sz = a.sz;
    g.ep_sc = sc;
    g.ep_bi = bi;
    hipError_t e = launch_gemm_conv(g, EP_CONV_BB, st);
    if (e != hipSuccess) return e;
    const int tn = 65536 / tm, R = static_cast<int>(M / tm) * (tm / 128);
    return launch_bnbwd_sums_finalize(part, R, tn, N, invstd, sdz, sdzx, st,
                                      part + static_cast<size_t>(N / tn) * R * 2 * tn, dgamma,
                                      dbeta);
  }
  hipError_t e = taps == 1 ? launch_v<1>(a, M, st) : launch_v<9>(a, M, st);
  if (e != hipSuccess) return e;
  int BM, BN;
  tile_of(M, N, &BM, &BN);
  const int R = static_cast<int>((M + BM - 1) / BM) * (BM / 64);
  return launch_bnbwd_sums_finalize(part, R, BN, N, invstd, sdz, sdzx, st,
                                    part + static_cast<size_t>(N / BN) * R * 2 * BN, dgamma, dbeta);
}

namespace {
// the tile of the stride-2 data gradient for N = Ci output channels
// (small grids -- fewer than smallm_tiles() 256 x 256 tiles per class, e.g. batch 256 -- take
// 128 x 128 tiles, two workgroups per CU)
void tile_par(int64_t Mc, int N, int* BM, int* BN, int* WTN) {
  *BM = 256;
  *BN = N % 256 == 0 ? 256 : (N % 128 == 0 ? 128 : 64);
  *WTN = *BN == 256 ? 128 : 64;
  if (*BN >= 128 && smallm_tiles() > 0 && (Mc + 255) / 256 * (N / 256 > 0 ? N / 256 : 1) <
                                               smallm_tiles()) {
    *BM = 128;
    *BN = 128;
    *WTN = 64;
  }
}

template <int BM, int BN, int WTN>
hipError_t launch_par(GArgs a, hipStream_t st) {
  auto k = a.sz ? &conv_gemm_kernel<BM, BN, 9, 2, WTN, true, true, true>
                : &conv_gemm_kernel<BM, BN, 9, 2, WTN, false, false, true>;
  const size_t lds = 2 * static_cast<size_t>(BM + BN) * 128;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  a.ntn = a.N / BN;
  const int64_t mt = (static_cast<int64_t>(a.M) + BM - 1) / BM;
  if (mt * a.ntn >= (1ll << 31)) return hipErrorInvalidValue;
  a.tiles = static_cast<int>(mt * a.ntn);
  a.prt = static_cast<int>(4 * mt * (BM / 64));
  // the 4-tap class first, the 1-tap class last (its short k loop fills the others' tails)
  static const int order[4][2] = {{1, 1}, {1, 0}, {0, 1}, {0, 0}};
  for (int i = 0; i < 4; ++i) {
    a.py = order[i][0];
    a.px = order[i][1];
    a.KS = (a.py + 1) * (a.px + 1) * (a.C / kBK);
    a.prb = static_cast<int>(i * mt * (BM / 64));
    k<<<a.tiles, BM * BN / WTN, lds, st>>>(a);
  }
  return hipGetLastError();
}
}  // namespace

size_t conv_gemm_s2dgrad_part_floats(int64_t Mc, int N) {
  int BM, BN, WTN;
  tile_par(Mc, N, &BM, &BN, &WTN);
  const int R = static_cast<int>(4 * ((Mc + BM - 1) / BM) * (BM / 64));
  const size_t g = static_cast<size_t>(N / BN) *
                   (static_cast<size_t>(R) + bn_part_fold_slices(R, N / BN)) * 2 * BN;
  return N == 64 && g < conv3x3p_part_floats() ? conv3x3p_part_floats() : g;
}

// dx [Nimg, 2 Ho, 2 Wo, Ci] of a stride-2 / padding-1 3x3 conv from dy [Nimg, Ho, Wo, Co] and
// the rotated, transposed weights wr [Ci][9 Co] (conv3x3_wlayouts), four parity-class launches
// that together write every pixel once. With z: also the sums of the BN + ReLU backward dx feeds
// (as launch_conv_gemm_bnsums).
hipError_t launch_conv_gemm_s2dgrad(const void* dy, const void* wr, void* dx, const void* zero,
                                    int Nimg, int Ho, int Wo, int Co, int Ci, const void* z,
                                    const float* sc, const float* bi, const float* mean,
                                    const float* invstd, float* part, float* sdz, float* sdzx,
                                    hipStream_t st, void* dgamma, void* dbeta) {
  const int64_t Mc = static_cast<int64_t>(Nimg) * Ho * Wo;
  if (Co % kBK || Ci % 64 || Mc < 1 || 4 * Mc >= (1ll << 31) || 9ll * Co > 65536 || !zero)
    return hipErrorInvalidValue;
  if (z && (!sc || !bi || !mean || !invstd || !part || !sdz || !sdzx)) return hipErrorInvalidValue;
  GArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(dy);
  a.w = reinterpret_cast<const uint16_t*>(wr);
  a.y = reinterpret_cast<uint16_t*>(dx);
  a.zero = reinterpret_cast<const uint16_t*>(zero);
  a.M = static_cast<int>(Mc);
  a.C = Co;
  a.N = Ci;
  a.H = Ho;
  a.W = Wo;
  a.HW = Ho * Wo;
  a.S = 1;
  a.IH = Ho;
  a.IW = Wo;
  a.IHW = Ho * Wo;
  a.wld = 9 * Co;
  if (z) {
    a.part = part;
    a.shift = mean;
    a.sz = reinterpret_cast<const uint16_t*>(z);
    a.ep_sc = sc;
    a.ep_bi = bi;
  }
  int BM, BN, WTN;
  tile_par(Mc, Ci, &BM, &BN, &WTN);
  hipError_t e;
  if (BM == 128) e = launch_par<128, 128, 64>(a, st);
  else if (BN == 256) e = launch_par<256, 256, 128>(a, st);
  else if (BN == 128) e = launch_par<256, 128, 64>(a, st);
  else e = launch_par<256, 64, 64>(a, st);
  if (e != hipSuccess || !z) return e;
  const int R = static_cast<int>(4 * ((Mc + BM - 1) / BM) * (BM / 64));
  return launch_bnbwd_sums_finalize(part, R, BN, Ci, invstd, sdz, sdzx, st,
                                    part + static_cast<size_t>(Ci / BN) * R * 2 * BN, dgamma,
                                    dbeta);
}

namespace {
// The two GEMM layouts of a 3x3 conv weight w[co][ci][ky][kx] (any strides, bf16) in one pass:
//   wf[co][(3 ky + kx) Ci + ci]        = w[co][ci][ky][kx]          (forward implicit GEMM)
//   wr[ci][(3 ky + kx) Co + co]        = w[co][ci][2 - ky][2 - kx]  (data gradient: rotated,
//                                                                     transposed)
// One thread per weight element (replaces a permute copy, a flip and a second permute copy).
__global__ __launch_bounds__(256) void conv3x3_wlayouts_kernel(const uint16_t* __restrict__ w,
                                                              int Co, int Ci, int64_t s0,
                                                              int64_t s1, int64_t s2, int64_t s3,
                                                              uint16_t* __restrict__ wf,
                                                              uint16_t* __restrict__ wr) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= static_cast<int64_t>(Co) * Ci * 9) return;
  // e enumerates (co, tap, ci) so the wf writes are contiguous
  const int ci = static_cast<int>(e % Ci);
  const int t = static_cast<int>((e / Ci) % 9);
  const int co = static_cast<int>(e / (static_cast<int64_t>(Ci) * 9));
  const int ky = t / 3, kx = t - 3 * (t / 3);
  const uint16_t v = w[co * s0 + ci * s1 + ky * s2 + kx * s3];
  if (wf) wf[e] = v;
  wr[(static_cast<int64_t>(ci) * 9 + (8 - t)) * Co + co] = v;
}

// Several weights' layouts in one launch (the 16 3x3 convs of a ResNet-50 forward and its 1x1
// transposes: one launch instead of 16 + 12 ~5-9 us ones): descriptors by value, workgroups
// [blk0[d], blk0[d + 1]) on weight d.
struct WlMulti {
  WlDesc d[kWlMax];
  int blk0[kWlMax + 1];
  int n;
};

__global__ __launch_bounds__(256) void conv3x3_wlayouts_multi_kernel(const WlMulti m) {
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < m.n && b >= m.blk0[i + 1]) ++i;
  const WlDesc& d = m.d[i];
  const int T = d.taps;   // 9 (3x3) or 1 (1x1: wr is the plain transpose)
  const int64_t e = static_cast<int64_t>(b - m.blk0[i]) * 256 + threadIdx.x;
  if (e >= static_cast<int64_t>(d.Co) * d.Ci * T) return;
  const int ci = static_cast<int>(e % d.Ci);
  const int t = static_cast<int>((e / d.Ci) % T);
  const int co = static_cast<int>(e / (static_cast<int64_t>(d.Ci) * T));
  const int ky = t / 3, kx = t - 3 * (t / 3);
  const uint16_t* w = reinterpret_cast<const uint16_t*>(d.w);
  const uint16_t v = w[co * d.s0 + ci * d.s1 + ky * d.s2 + kx * d.s3];
  if (d.wf) reinterpret_cast<uint16_t*>(d.wf)[e] = v;
  reinterpret_cast<uint16_t*>(d.wr)[(static_cast<int64_t>(ci) * T + (T - 1 - t)) * d.Co + co] = v;
}
}  // namespace

hipError_t launch_conv3x3_wlayouts_multi(const WlDesc* d, int n, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += kWlMax) {
    WlMulti m{};
    m.n = n - i0 < kWlMax ? n - i0 : kWlMax;
    int64_t blk = 0;
    for (int i = 0; i < m.n; ++i) {
      const WlDesc& x = d[i0 + i];
      if (x.Co < 1 || x.Ci < 1 || !x.w || !x.wr || (x.taps != 1 && x.taps != 9))
        return hipErrorInvalidValue;
      m.d[i] = x;
      m.blk0[i] = static_cast<int>(blk);
      blk += (static_cast<int64_t>(x.Co) * x.Ci * x.taps + 255) / 256;
      if (blk >= (1ll << 31)) return hipErrorInvalidValue;
    }
    m.blk0[m.n] = static_cast<int>(blk);
    conv3x3_wlayouts_multi_kernel<<<static_cast<unsigned>(blk), 256, 0, st>>>(m);
  }
  return hipGetLastError();
}

hipError_t launch_conv3x3_wlayouts(const void* w, int Co, int Ci, int64_t s0, int64_t s1,
                                   int64_t s2, int64_t s3, void* wf, void* wr, hipStream_t st) {
  if (Co < 1 || Ci < 1 || !wr) return hipErrorInvalidValue;
  const int64_t n = static_cast<int64_t>(Co) * Ci * 9;
  conv3x3_wlayouts_kernel<<<static_cast<unsigned>((n + 255) / 256), 256, 0, st>>>(
      reinterpret_cast<const uint16_t*>(w), Co, Ci, s0, s1, s2, s3,
      reinterpret_cast<uint16_t*>(wf), reinterpret_cast<uint16_t*>(wr));
  return hipGetLastError();
}

}  // namespace cml
