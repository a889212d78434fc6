// Weight gradient of a 3x3 / stride 2 / padding 1 convolution on NHWC bf16 tensors with an even
// input (the ResNet-50 downsample blocks' conv2: 56 -> 28, 28 -> 14, 14 -> 7), all nine taps in
// one workgroup:
//
//   dW[co][ky][kx][ci] = sum_o dy[o][co] x[2 o + (ky, kx) - 1][ci]     (o over output pixels)
//
// Round 3 left these on MIOpen (igemm_wrw ... "ex1": 0.62-0.86 ms per call at batch 2048,
// profiles/r04_14/kernels_b2048.md). Unlike the stride-1 kernel (wgrad3x3.hip, x unshifted and
// dy shifted per tap) the shifted operand here is x, and stride 2 makes its window four times the
// output chunk. Design (gfx950):
//
// * A chunk is R output rows of one image (R Wo <= 64 pixels, padded to whole 16-pixel k-steps
//   with zero dy rows; an image's last chunk may have fewer rows). LDS holds its dy rows
//   [pixel][64 CT co] (192 / 320-B rows) and the RAW x rows 2 oh0 - 1 .. 2 oh0 + 2 R - 1 with
//   one zero column on the left ([(2R + 1) (W + 1)][64 ci], 160-B rows), both copied global ->
//   LDS by the DMA path (global_load_lds_dwordx4; rows outside the image and the pad column from
//   a zero row). Tap (ky, kx) of output pixel (lr, ow) is x row (2 lr + ky) (W + 1) + 2 ow + kx:
//   a plain per-lane row address, no gather at read time.
// * Row pitches for conflict-free ds_read_b64_tr_b16 (the 4 pixel rows of a transposed read must
//   fall in 4 disjoint 64-B bank windows): dy rows are consecutive (192 / 320 B), x rows of
//   consecutive output pixels are 2 apart (160 B: 2 x 160 = 64 mod 256).
// * 12 waves = 3 tap rows (ky) x 2 co halves x 2 ci halves (the 64 CT x 64 tile); every wave
//   holds the three kx taps of its ky for 32 CT co: 3 CT v_mfma_f32_32x32x16_bf16 accumulators.
//   Per 16-pixel k-step: CT dy fragments (co, unshifted) and 3 x fragments (ci, shifted per kx).
// * Two buffers (<= 116 KB; the next chunk's DMA overlaps this chunk's MFMAs), one workgroup per
//   CU, 3 waves per SIMD; split-K over chunks, fp32 partials
//   [split][Co][9][Ci] folded in a fixed order (wgrad1x1_fold), so dW comes out in the
//   channels_last order of [Co, Ci, 3, 3].
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

constexpr int kNW = 12;             // waves per workgroup
constexpr int kMaxPx = 64;          // output pixels per chunk
constexpr int kMaxKS = kMaxPx / 16;
constexpr int kRX = 160;            // x LDS row: 64 ci + 32 B
constexpr int kMaxQ = 6;            // DMA instructions per wave and chunk (<= 72 KB of LDS)

__device__ __forceinline__ f32x16 mfma(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ s16x4 ld_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ bf16x8_t cat(s16x4 a, s16x4 b) {
  return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct S2Args {
  const uint16_t* dy;     // [B][Ho][Wo][Co]
  const uint16_t* x;      // [B][2 Ho][2 Wo][Ci]
  const uint16_t* zero;   // >= 8 zero bf16
  float* part;            // [S][Co][9][Ci]
  int Ho, Wo, Co, Ci;
  int R, npx, nks;        // output rows per chunk, real / padded-to-16 pixels per chunk
  int nch, cps;           // chunks, chunks per split
  int tiles_ci, tiles;    // ci tiles (64), co x ci tiles
  int rd, rx;             // LDS bytes of the dy and x regions (multiples of 1 KB)
  int nbuf;               // 2: the next chunk's DMA overlaps this chunk's MFMAs
};

// CT: 32-channel co blocks per wave (tile Co = 64 CT): the x window, 4.6x the chunk's pixels, is
// staged once per co tile, so CT = 2 halves its DMA bytes per MFMA
template <int CT>
__global__ __launch_bounds__(kNW * 64, 1) void wgrad3x3s2_kernel(S2Args a) {
  constexpr int kRD = 128 * CT + 64;          // dy LDS row: 64 CT co + 64 B (192 / 320)
  constexpr int SD = kRD / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ky = wave >> 2, cpart = wave & 1, ipart = (wave >> 1) & 1;
  const int h = lane >> 5, r32 = lane & 31, grp = lane >> 4, gi = lane & 15;
  const int q = gi >> 2, p = gi & 3;
  const int Gb = gridDim.x, b = blockIdx.x, xcd = b & 7, q8 = Gb >> 3, r8 = Gb & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int tile = t % a.tiles, split = t / a.tiles;
  const int tco = tile / a.tiles_ci, tci = tile - tco * a.tiles_ci;
  const int co0 = tco * 64 * CT, ci0 = tci * 64;
  const int Wo = a.Wo, W = 2 * a.Wo, H = 2 * a.Ho, W1 = W + 1;
  const int nqd = a.rd >> 10, nqx = a.rx >> 10;

  // chunk-invariant DMA plan of this lane: dy slot s is row s / 12, chunk s % 12 (so: element
  // offset, -1 zero; sr: the pixel row); x slot s is row s / 10 = (xr, xc) of the staged window,
  // chunk s % 10 (so: element offset in the x row, -1 zero; sr: xr)
  int so[kMaxQ], sr[kMaxQ];
#pragma unroll
  for (int i = 0; i < kMaxQ; ++i) {
    const int qi = wave + kNW * i;
    so[i] = -1;
    sr[i] = 0;
    if (qi < nqd) {
      const int s = qi * 64 + lane, row = s / SD, j = s - row * SD;
      if (row < a.npx && j < 8 * CT) {
        so[i] = row * a.Co + 8 * j;
        sr[i] = row;
      }
    } else if (qi < nqd + nqx) {
      const int s = (qi - nqd) * 64 + lane, row = s / 10, j = s - row * 10;
      const int xr = row / W1, xc = row - xr * W1;
      if (xr <= 2 * a.R && xc >= 1 && j < 8) {
        so[i] = (xc - 1) * a.Ci + 8 * j;
        sr[i] = xr;
      }
    }
  }
  // chunk c: output rows oh0 .. oh0 + R - 1 of image c / per (the last chunk of an image may be
  // shorter: its missing dy rows and the x rows past the image read the zero row)
  const int per = (a.Ho + a.R - 1) / a.R;
  auto issue = [&](int c, int buf) {
    char* base = smem + buf * (a.rd + a.rx);
    const int img = c / per, oh0 = (c - img * per) * a.R;
    const int npx_c = min(a.R, a.Ho - oh0) * Wo;
    const int64_t dbase = ((static_cast<int64_t>(img) * a.Ho + oh0) * Wo) * a.Co + co0;
    const int64_t xbase = static_cast<int64_t>(img) * H * W * a.Ci + ci0;
#pragma unroll
    for (int i = 0; i < kMaxQ; ++i) {
      const int qi = wave + kNW * i;
      if (qi < nqd + nqx) {
        const uint16_t* src = a.zero;
        if (qi < nqd) {
          if (so[i] >= 0 && sr[i] < npx_c) src = a.dy + dbase + so[i];
        } else {
          const int xrow = 2 * oh0 - 1 + sr[i];
          if (so[i] >= 0 && xrow >= 0 && xrow < H)
            src = a.x + xbase + static_cast<int64_t>(xrow) * W * a.Ci + so[i];
        }
        __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(base + qi * 1024), 16, 0, 0);
      }
    }
  };

  // fragment addresses (chunk-invariant). dy: pixel rows k = 16 ks + 8 h + q (+ 4), channels
  // cpart 32 + 16 (grp & 1) + 4 p. x: the pixel's tap-(ky, 0) row, + kx rows per tap; channels
  // 16 (grp & 1) + 4 p (+ 32 per ci block j).
  const int chd = 2 * (cpart * 32 * CT + 16 * (grp & 1) + 4 * p);
  const int chx = 2 * (ipart * 32 + 16 * (grp & 1) + 4 * p);
  int xa0[kMaxKS], xa1[kMaxKS];
#pragma unroll
  for (int ks = 0; ks < kMaxKS; ++ks) {
    int k0 = 16 * ks + 8 * h + q, k1 = k0 + 4;
    k0 = k0 < a.npx ? k0 : a.npx - 1;   // padded pixels: dy is zero there, any x row will do
    k1 = k1 < a.npx ? k1 : a.npx - 1;
    const int l0 = k0 / Wo, l1 = k1 / Wo;
    xa0[ks] = a.rd + ((2 * l0 + ky) * W1 + 2 * (k0 - l0 * Wo)) * kRX + chx;
    xa1[ks] = a.rd + ((2 * l1 + ky) * W1 + 2 * (k1 - l1 * Wo)) * kRX + chx;
  }
  const int da = (8 * h + q) * kRD + chd;

  f32x16 acc[3][CT];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int u = 0; u < CT; ++u)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][u][k] = 0.f;

  const int c_lo = split * a.cps;
  const int c_hi = min(a.nch, c_lo + a.cps);
  // one buffer: DMA, wait, MFMAs, barrier per chunk (other workgroups on the CU fill the gap);
  // two: chunk c + 1 is copied while chunk c is multiplied
  if (a.nbuf == 2 && c_lo < c_hi) issue(c_lo, 0);
  for (int c = c_lo; c < c_hi; ++c) {
    int buf = 0;
    if (a.nbuf == 2) {
      buf = (c - c_lo) & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (c + 1 < c_hi) issue(c + 1, buf ^ 1);
    } else {
      issue(c, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const char* sb = smem + buf * (a.rd + a.rx);
    for (int ks = 0; ks < a.nks; ++ks) {
      const char* pd = sb + da + 16 * ks * kRD;
      bf16x8_t A[CT];
#pragma unroll
      for (int u = 0; u < CT; ++u) A[u] = cat(ld_tr(pd + 64 * u), ld_tr(pd + 64 * u + 4 * kRD));
      bf16x8_t B[3];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
        B[kx] = cat(ld_tr(sb + xa0[ks] + kx * kRX), ld_tr(sb + xa1[ks] + kx * kRX));
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int u = 0; u < CT; ++u) acc[kx][u] = mfma(A[u], B[kx], acc[kx][u]);
    }
    if (a.nbuf == 1) __syncthreads();   // every wave is done with the buffer: next chunk's DMA
  }

  // partials [split][co][tap][ci]: lane r32 = ci column, register k = co row (k & 3) + 8 (k >> 2)
  // + 4 h; accumulator kx of wave ky is tap 3 ky + kx
  float* pw = a.part + static_cast<int64_t>(split) * a.Co * 9 * a.Ci;
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const int tap = 3 * ky + kx;
#pragma unroll
    for (int u = 0; u < CT; ++u)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int co = co0 + cpart * 32 * CT + 32 * u + (k & 3) + 8 * (k >> 2) + 4 * h;
        const int ci = ci0 + ipart * 32 + r32;
        pw[(static_cast<int64_t>(co) * 9 + tap) * a.Ci + ci] = acc[kx][u][k];
      }
  }
}

bool enabled() {
  static const bool v = [] {
    const char* e = getenv("CML_WGRAD3X3_S2");
    return !e || e[0] != '0';
  }();
  return v;
}

struct Plan {
  int R, npx, nks, nch, S, cps, rd, rx, nbuf, ct;
  size_t lds;
};

bool make_plan(int B, int Ho, int Wo, int Co, int Ci, Plan* pl) {
  if (B < 1 || Ho < 1 || Wo < 1 || Co % 64 || Ci % 64) return false;
  const int R = std::min(Ho, kMaxPx / Wo);   // the last chunk of an image may be shorter
  if (R < 1) return false;
  Plan p{};
  p.R = R;
  p.npx = R * Wo;
  p.nks = (p.npx + 15) / 16;
  p.ct = Co % 128 == 0 ? 2 : 1;
  p.rd = (p.nks * 16 * (128 * p.ct + 64) + 1023) / 1024 * 1024;
  p.rx = ((2 * R + 1) * (2 * Wo + 1) * kRX + 1023) / 1024 * 1024;
  if ((p.rd + p.rx) / 1024 > kNW * kMaxQ) return false;
  p.nbuf = 2 * (p.rd + p.rx) <= 160 * 1024 ? 2 : 1;
  p.lds = static_cast<size_t>(p.nbuf) * (p.rd + p.rx);
  const int64_t nch = static_cast<int64_t>(B) * ((Ho + R - 1) / R);
  if (nch >= (1ll << 30)) return false;
  p.nch = static_cast<int>(nch);
  const int tiles = (Co / (64 * p.ct)) * (Ci / 64);
  // ~2 workgroups per CU; splits bound the fp32 partials to ~96 MB
  int s = (512 + tiles - 1) / tiles;
  const int64_t smax = std::max<int64_t>(1, (96ll << 20) / (4ll * 9 * Co * Ci));
  s = static_cast<int>(std::min<int64_t>({static_cast<int64_t>(s), smax, nch}));
  s = std::max(s, 1);
  p.cps = (p.nch + s - 1) / s;
  p.S = (p.nch + p.cps - 1) / p.cps;
  *pl = p;
  return true;
}

}  // namespace

bool wgrad3x3_s2_plan(int B, int Ho, int Wo, int Co, int Ci, int* splits) {
  Plan p;
  if (!enabled() || !make_plan(B, Ho, Wo, Co, Ci, &p)) return false;
  *splits = p.S;
  return true;
}

hipError_t launch_wgrad3x3_s2(const void* dy, const void* x, const void* zero, float* part, void* dw,
                              bool dw_bf16, int B, int Ho, int Wo, int Co, int Ci, hipStream_t st) {
  Plan p;
  if (!make_plan(B, Ho, Wo, Co, Ci, &p)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) |
       reinterpret_cast<uintptr_t>(zero)) % 16)
    return hipErrorInvalidValue;
  S2Args a{};
  a.dy = reinterpret_cast<const uint16_t*>(dy);
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.zero = reinterpret_cast<const uint16_t*>(zero);
  a.part = part;
  a.Ho = Ho;
  a.Wo = Wo;
  a.Co = Co;
  a.Ci = Ci;
  a.R = p.R;
  a.npx = p.npx;
  a.nks = p.nks;
  a.nch = p.nch;
  a.cps = p.cps;
  a.tiles_ci = Ci / 64;
  a.tiles = (Co / (64 * p.ct)) * a.tiles_ci;
  a.rd = p.rd;
  a.rx = p.rx;
  a.nbuf = p.nbuf;
  auto kern = p.ct == 2 ? &wgrad3x3s2_kernel<2> : &wgrad3x3s2_kernel<1>;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(p.lds));
  kern<<<a.tiles * p.S, kNW * 64, p.lds, st>>>(a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_wgrad_fold(part, p.S, 9ll * Co * Ci, dw, dw_bf16, st);
}

}  // namespace cml
