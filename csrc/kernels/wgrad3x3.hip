// Weight gradient of a 3x3 / stride 1 / padding 1 convolution on NHWC bf16 tensors, all nine taps
// in one workgroup:
//
//   dW[co][tap][ci] = sum_i dy[i - s(tap)][co] x[i][ci]       (i over input pixels, s = (dh, dw),
//                                                              dy zero outside the image)
//
// i.e. nine GEMMs whose reduction runs over pixels and which share their x operand. MIOpen's
// weight-gradient kernels run these ResNet-50 shapes at 0.39-0.71 PFLOP/s (batch 2048,
// profiles/r02_conv3x3_wgrad26.jsonl); wgrad1x1.hip's TAP mode (one tap per grid z) re-reads x
// and dy per tap and is slower still. Design (gfx950):
//
// * A chunk is R rows of one image (or G whole small images): its x rows [pixel][TCI channels]
//   and the dy rows it needs -- the same rows plus one halo row above and below, with a zero
//   column on each side -- are copied global -> LDS by the DMA path (global_load_lds_dwordx4, no
//   VGPR staging), double buffered, one vmcnt(0) + barrier per chunk. Padding (halo rows outside
//   the image, the side columns, the pixels past the chunk) is loaded from a zero row, so every
//   tap's dy operand is a plain row offset into the padded image: row(i) - s = base(i) + (1 - dh)
//   (W + 2) + (1 - dw). No masks, no per-tap address arithmetic beyond an add.
// * LDS rows are padded to 64 B past a multiple of 256 B (192 / 320 B): the four consecutive rows
//   of a ds_read_b64_tr_b16 half-wave land on four disjoint 16-bank windows (conflict-free
//   without a swizzle, so the shifted reads need no per-row XOR).
// * 12 waves = 3 tap rows (dh) x 2 (co halves of 32) x 2 (ci parts of 32 NB); every wave holds
//   the three dw taps of its dh: 3 x NB v_mfma_f32_32x32x16_bf16 accumulators. Per 16-pixel k-step
//   a wave reads NB x fragments and 3 shifted dy fragments (transposed reads, k = pixel) for 3 NB
//   MFMAs. 3 waves per SIMD (<= 168 registers).
// * Split-K over chunks; fp32 partials [split][Co][9][Ci] folded in a fixed order
//   (wgrad1x1_fold), so dW comes out in the channels_last order of [Co, Ci, 3, 3].
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

constexpr int kKP = 112;          // pixels per chunk (7 k-steps of 16)
constexpr int kKS = kKP / 16;
constexpr int kNW = 12;           // waves per workgroup
constexpr int kRBD = 192;         // dy LDS row: 64 channels + 64 B
constexpr int kMaxDyRows = 232;
constexpr int kMaxIX = 3, kMaxID = 4;   // DMA instructions per wave and chunk (x, dy)

__device__ __forceinline__ f32x16 mfma(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ s16x4 ld_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ bf16x8_t cat(s16x4 a, s16x4 b) {
  return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct W3Args {
  const uint16_t* dy;     // [B][H][W][Co]
  const uint16_t* x;      // [B][H][W][Ci]
  const uint16_t* zero;   // >= 8 zero bf16
  float* part;            // [S][Co][9][Ci]
  int H, W, Co, Ci;
  int R, G;               // chunk = R rows of one image (G == 1) or G whole images (R == H)
  int npx;                // real pixels per chunk (G R W <= kKP)
  int nch, cps;           // chunks, chunks per split
  int tiles_ci, tiles;    // ci tiles, co x ci tiles
  int rx, rd;             // LDS bytes of the x and dy regions (multiples of 1 KB)
};

// pixel k of a chunk -> its row in the padded dy image, minus (W + 3) (the dh = dw = +1 shift)
__device__ __forceinline__ int base_row(int k, int W, int HW, int G) {
  const int r = k / W;
  int b = k + 2 * r;
  if (G > 1) b += (k / HW) * (2 * W + 4);
  return b;
}

template <int TCI>
__global__ __launch_bounds__(kNW * 64, 1) void wgrad3x3_kernel(W3Args a) {
  constexpr int NB = TCI / 64;                  // 32-channel ci blocks per wave
  constexpr int RBX = TCI * 2 + 64;             // x LDS row bytes
  constexpr int SX = RBX / 16, SD = kRBD / 16;  // 16-B slots per row
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int dhi = wave >> 2, sub = wave & 3;    // dh + 1; co half / ci part
  const int cpart = sub & 1, ipart = sub >> 1;
  const int h = lane >> 5, r32 = lane & 31, grp = lane >> 4, gi = lane & 15;
  const int q = gi >> 2, p = gi & 3;
  // bijective XCD remap: the tiles of one split are consecutive and share an XCD's L2
  const int Gb = gridDim.x, b = blockIdx.x, xcd = b & 7, q8 = Gb >> 3, r8 = Gb & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int tile = t % a.tiles, split = t / a.tiles;
  const int tco = tile / a.tiles_ci, tci = tile - tco * a.tiles_ci;
  const int co0 = tco * 64, ci0 = tci * TCI;
  const int W = a.W, HW = a.H * a.W, W2 = a.W + 2;
  const int PB = (a.G == 1 ? a.R + 2 : a.H + 2) * W2;   // padded rows per image block

  // chunk-invariant DMA plan of this lane: source offsets relative to the chunk origin (-1: zero)
  const int nqx = a.rx >> 10, nqd = a.rd >> 10;
  int xo[kMaxIX], dof[kMaxID];
  uint32_t dtop = 0u, dbot = 0u;
#pragma unroll
  for (int i = 0; i < kMaxIX; ++i) {
    const int s = (wave + kNW * i) * 64 + lane, row = s / SX, j = s - row * SX;
    xo[i] = (row < a.npx && j < TCI / 8) ? row * a.Ci + 8 * j : -1;
  }
#pragma unroll
  for (int i = 0; i < kMaxID; ++i) {
    const int s = (wave + kNW * i) * 64 + lane, row = s / SD, j = s - row * SD;
    const int g = row / PB, rem = row - g * PB, pr = rem / W2, pc = rem - pr * W2;
    bool ok = j < 8 && g < a.G && pc >= 1 && pc <= W;
    if (a.G > 1) ok = ok && pr >= 1 && pr <= a.H;
    dof[i] = ok ? ((g * a.H + pr) * W + pc) * a.Co + 8 * j : -1;
    if (a.G == 1 && pr == 0) dtop |= 1u << i;
    if (a.G == 1 && pr == a.R + 1) dbot |= 1u << i;
  }

  auto issue = [&](int c, int buf) {
    int64_t pix0;
    bool topok = true, botok = true;
    if (a.G == 1) {
      const int per = a.H / a.R, img = c / per, h0 = (c - img * per) * a.R;
      pix0 = (static_cast<int64_t>(img) * a.H + h0) * W;
      topok = h0 > 0;
      botok = h0 + a.R < a.H;
    } else {
      pix0 = static_cast<int64_t>(c) * a.G * HW;
    }
    const int64_t xbase = pix0 * a.Ci + ci0;
    const int64_t dbase = (pix0 - W - 1) * a.Co + co0;
    char* xb = smem + buf * (a.rx + a.rd);
    char* db = xb + a.rx;
#pragma unroll
    for (int i = 0; i < kMaxIX; ++i) {
      const int qi = wave + kNW * i;
      if (qi < nqx) {
        const uint16_t* src = xo[i] >= 0 ? a.x + xbase + xo[i] : a.zero;
        __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(xb + qi * 1024), 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < kMaxID; ++i) {
      const int qi = wave + kNW * i;
      if (qi < nqd) {
        const bool ok = dof[i] >= 0 && (topok || !((dtop >> i) & 1u)) &&
                        (botok || !((dbot >> i) & 1u));
        const uint16_t* src = ok ? a.dy + dbase + dof[i] : a.zero;
        __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(db + qi * 1024), 16, 0, 0);
      }
    }
  };

  // fragment addresses (chunk-invariant): x rows are the pixels, dy rows the shifted pixels
  const int chx = 2 * (ipart * 32 * NB + 16 * (grp & 1) + 4 * p);
  const int xa = (8 * h + q) * RBX + chx;
  const int chd = 2 * (cpart * 32 + 16 * (grp & 1) + 4 * p);
  int da0[kKS], da1[kKS];
#pragma unroll
  for (int ks = 0; ks < kKS; ++ks) {
    da0[ks] = base_row(16 * ks + 8 * h + q, W, HW, a.G) * kRBD + chd;
    da1[ks] = base_row(16 * ks + 8 * h + q + 4, W, HW, a.G) * kRBD + chd;
  }
  const int sdh = (2 - dhi) * W2 * kRBD;          // this wave's dh row shift

  f32x16 acc[3][NB];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;

  const int c_lo = split * a.cps;
  const int c_hi = min(a.nch, c_lo + a.cps);
  if (c_lo < c_hi) issue(c_lo, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int c = c_lo; c < c_hi; ++c) {
    const int buf = (c - c_lo) & 1;
    if (c + 1 < c_hi) issue(c + 1, buf ^ 1);
    const char* xb = smem + buf * (a.rx + a.rd);
    const char* db = xb + a.rx + sdh;
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) {
      bf16x8_t B[NB], A[3];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const char* px = xb + xa + 16 * ks * RBX + 64 * j;
        B[j] = cat(ld_tr(px), ld_tr(px + 4 * RBX));
      }
#pragma unroll
      for (int tt = 0; tt < 3; ++tt)
        A[tt] = cat(ld_tr(db + da0[ks] + tt * kRBD), ld_tr(db + da1[ks] + tt * kRBD));
#pragma unroll
      for (int tt = 0; tt < 3; ++tt)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[tt][j] = mfma(A[tt], B[j], acc[tt][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // partials [split][co][tap][ci]: lane r32 = ci column, register k = co row (k&3) + 8 (k>>2) + 4h;
  // accumulator tt holds dw = 1 - tt, so tap = 3 dhi + 2 - tt
  float* pw = a.part + static_cast<int64_t>(split) * a.Co * 9 * a.Ci;
#pragma unroll
  for (int tt = 0; tt < 3; ++tt) {
    const int tap = 3 * dhi + 2 - tt;
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int co = co0 + cpart * 32 + (k & 3) + 8 * (k >> 2) + 4 * h;
        const int ci = ci0 + ipart * 32 * NB + 32 * j + r32;
        pw[(static_cast<int64_t>(co) * 9 + tap) * a.Ci + ci] = acc[tt][j][k];
      }
  }
}

int direct_enabled() {
  static const int v = [] {
    const char* e = getenv("CML_WGRAD3X3_DIRECT");
    return e ? atoi(e) : 1;
  }();
  return v;
}

}  // namespace

bool wgrad3x3_direct_plan(int B, int H, int W, int Co, int Ci, int* splits, int* tci) {
  if (!direct_enabled() || B < 1 || H < 1 || W < 1 || Co % 64 || !(Ci == 64 || Ci % 128 == 0))
    return false;
  int R, G = 1;
  if (H * W <= kKP) {
    R = H;
    for (int g = kKP / (H * W); g >= 1; --g)
      if (B % g == 0) { G = g; break; }
  } else {
    R = 0;
    for (int r = kKP / W; r >= 1; --r)
      if (H % r == 0) { R = r; break; }
    if (R == 0) return false;
  }
  const int k = kKP - 1, HW = H * W;
  const int maxrow = k + 2 * (k / W) + (G > 1 ? (k / HW) * (2 * W + 4) : 0) + 2 * (W + 2) + 2;
  const int PB = (G == 1 ? R + 2 : H + 2) * (W + 2);
  const int dyr = std::max(G * PB, maxrow + 1);
  if (dyr > kMaxDyRows) return false;
  const int T = Ci % 128 == 0 ? 128 : 64;
  const int64_t nch = G == 1 ? static_cast<int64_t>(B) * (H / R) : B / G;
  if (nch >= (1ll << 30)) return false;
  const int tiles = (Co / 64) * (Ci / T);
  int s = (256 + tiles - 1) / tiles;
  s = s < 1 ? 1 : (s > nch ? static_cast<int>(nch) : s);
  const int cps = static_cast<int>((nch + s - 1) / s);
  *splits = static_cast<int>((nch + cps - 1) / cps);
  *tci = T;
  return true;
}

hipError_t launch_wgrad3x3_direct(const void* dy, const void* x, const void* zero, float* part,
                                  void* dw, bool dw_bf16, int B, int H, int W, int Co, int Ci,
                                  hipStream_t st) {
  int S, T;
  if (!wgrad3x3_direct_plan(B, H, W, Co, Ci, &S, &T)) return hipErrorInvalidValue;
  W3Args a{};
  a.dy = reinterpret_cast<const uint16_t*>(dy);
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.zero = reinterpret_cast<const uint16_t*>(zero);
  a.part = part;
  a.H = H;
  a.W = W;
  a.Co = Co;
  a.Ci = Ci;
  const int HW = H * W;
  if (HW <= kKP) {
    a.R = H;
    a.G = 1;
    for (int g = kKP / HW; g >= 1; --g)
      if (B % g == 0) { a.G = g; break; }
  } else {
    a.G = 1;
    for (int r = kKP / W; r >= 1; --r)
      if (H % r == 0) { a.R = r; break; }
  }
  a.npx = a.G * a.R * W;
  a.nch = a.G == 1 ? B * (H / a.R) : B / a.G;
  a.cps = (a.nch + S - 1) / S;
  a.tiles_ci = Ci / T;
  a.tiles = (Co / 64) * a.tiles_ci;
  const int k = kKP - 1;
  const int maxrow = k + 2 * (k / W) + (a.G > 1 ? (k / HW) * (2 * W + 4) : 0) + 2 * (W + 2) + 2;
  const int dyr = std::max(a.G * (a.G == 1 ? a.R + 2 : H + 2) * (W + 2), maxrow + 1);
  a.rx = (kKP * (T * 2 + 64) + 1023) / 1024 * 1024;
  a.rd = (dyr * kRBD + 1023) / 1024 * 1024;
  if ((a.rx >> 10) > kNW * kMaxIX || (a.rd >> 10) > kNW * kMaxID) return hipErrorInvalidValue;
  const size_t lds = 2 * static_cast<size_t>(a.rx + a.rd);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int grid = a.tiles * S;
  auto kern = T == 128 ? &wgrad3x3_kernel<128> : &wgrad3x3_kernel<64>;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  kern<<<grid, kNW * 64, lds, st>>>(a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_wgrad_fold(part, S, 9ll * Co * Ci, dw, dw_bf16, st);
}

}  // namespace cml
