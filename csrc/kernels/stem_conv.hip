// ResNet stem: 7x7 / stride 2 / pad 3 convolution (C_in <= 4 -> 64 channels) on MFMA, with the
// BatchNorm that follows it folded into the two passes.
//
// forward  stem_conv_fwd: implicit GEMM z[pix][co] = sum_k im2col[pix][k] W[co][k] on
//          v_mfma_f32_32x32x16_bf16. A band of kTY output rows is one tile: its input rows are
//          staged once in LDS (4 channels = 8 B per pixel, zero padding, C_in = 3 read directly, so
//          no channel-padding pass), the packed weights live in registers for the workgroup's
//          lifetime (persistent grid), and the epilogue stores z and accumulates the BatchNorm
//          statistics (per-channel sum and sum of squares) -> no separate statistics pass over the
//          822 MB stem output. K order: (ky 0..6)(kx 0..7, 7 = zero tap)(c 0..3) = 224, so every
//          MFMA k-step is one input row x 4 taps x 4 channels = two 16-B LDS reads per lane.
//
// backward stem_wgrad: the BatchNorm backward and the weight gradient in ONE pass over
//          (g, z, x), g = the max-pool gradient, already masked by the ReLU (the fused pool forward
//          marks windows whose max is <= 0 with argmax 255, so they route no gradient).
//          With xhat = (z - mean) invstd the BN backward is
//            dz = gamma invstd (g - mean(g) - xhat mean(g xhat)),
//          and dW = sum_p dz[p] (x) im2col[p] is linear in dz. mean(g) comes with g (the pool
//          backward sums its output per channel), so the kernel stages g - mean(g) and accumulates
//            G = sum_p (g - mean(g)) (x) im2col,  X = sum_p xhat (x) im2col,  s2 = sum_p g xhat
//          and stem_wgrad_finalize forms dW = gamma invstd (G - s2/M X), dgamma = s2,
//          dbeta = sum_p g. dz never exists: the BN backward reduce and apply passes
//          (2.5 GB of traffic at batch 512) and the library weight-gradient kernel become this
//          one pass. The products sum over pixels, so both MFMA operands come out of LDS through
//          ds_read_b64_tr_b16 (the gfx950 transpose read): the g / xhat chunk is stored
//          [pixel][channel] as loaded and the input tile is the same one the forward uses; no
//          im2col or transposed copy is materialised anywhere. 8 waves: (g, xhat) x (channel
//          blocks 0, 1) x (kernel rows 0-3 | 4-6), 7 accumulators per SIMD.
#include <math.h>

#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kCo = 64;                 // output channels
constexpr int kKP = 224;                // packed K
constexpr int kSteps = kKP / 16;        // 14 MFMA k-steps, step s = (ky = s / 2, kx = 4 (s & 1) ..)
constexpr int kTY = 8;                  // forward: output rows per tile
constexpr int kTYB = 16;                // backward: output rows per tile (fewer tile-load bubbles)
constexpr int kFT = 256;                // forward workgroup: 4 waves
constexpr int kBT = 512;                // backward workgroup: 8 waves
constexpr int kCh = 128;                // backward pixel chunk: 8 x 16 pixels, 8 MFMA k-steps
constexpr int kPartW = 2 * kCo * kKP + 2 * kCo;   // floats per backward partial: G, X, s2, s1
constexpr int kColaS = 8;               // input column sums: pixel slices (workgroups) per tap

__host__ __device__ constexpr int tile_cols(int OW) { return 2 * OW + 6; }   // ix = -3 .. 2 OW + 2
__host__ __device__ constexpr int tile_rows(int TY) { return 2 * TY + 5; }

__device__ __forceinline__ f32x16 mfma(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8_t ld_frag(const uint16_t* p) {   // 16-B aligned
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}
// transposed LDS read (T10): lane 4q + p of each 16-lane group gives the address of row q,
// columns 4p..4p+3 of a 4 x 16 block; lane i receives column i, row q in element q
__device__ __forceinline__ s16x4 ld_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ bf16x8_t cat(s16x4 a, s16x4 b) {
  return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
// exact row of pixel index p < 2^20 in a band of width OW (float reciprocal, no integer divide)
__device__ __forceinline__ int row_of(int p, float inv_ow) {
  return __float2int_rz((static_cast<float>(p) + 0.5f) * inv_ow);
}

// Input rows 2 oy0 - 3 .. 2 oy0 + 2 TY + 1 of image n -> LDS [tile_rows][WT] x 8 B (zero outside
// the image; channels C..3 zero). VEC (C = 3, W % 4 == 0, 8-B aligned rows): a thread moves 4
// pixels = 24 B as three 8-B loads, up to 4 groups in flight, so a tile costs about one memory
// round trip instead of one per input row.
template <int C, int TY, bool VEC>
__device__ __forceinline__ void stage_input(const uint16_t* __restrict__ x, uint2* __restrict__ tile,
                                            int n, int oy0, int H, int W, int WT, int tid,
                                            int nthr) {
  const int iy0 = 2 * oy0 - 3;
  if constexpr (VEC) {
    const int t0 = iy0 < 0 ? -iy0 : 0;                          // first in-image tile row
    const int t1 = min(tile_rows(TY), H - iy0);                 // one past the last
    // zero: rows outside the image and the pad columns (u < 3, u >= W + 3) of the others
    const int npad = WT - W;                                    // u < 3 and u >= W + 3
    for (int t = 0; t < tile_rows(TY); ++t) {
      if (t < t0 || t >= t1) {
        for (int u = tid; u < WT; u += nthr) tile[t * WT + u] = make_uint2(0u, 0u);
      } else if (tid < npad) {
        tile[t * WT + (tid < 3 ? tid : W + tid)] = make_uint2(0u, 0u);
      }
    }
    const int G = W / 4;
    const int total = (t1 > t0 ? t1 - t0 : 0) * G;
    const float inv_g = 1.f / static_cast<float>(G);
    const uint16_t* xb = x + (static_cast<int64_t>(n) * H + iy0) * W * 3;
    for (int e0 = tid; e0 < total; e0 += 4 * nthr) {
      uint2 v[4][3];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = e0 + k * nthr;
        const int ec = e < total ? e : 0;
        const int tr = __float2int_rz((static_cast<float>(ec) + 0.5f) * inv_g);
        const int g = ec - tr * G;
        const uint2* src = reinterpret_cast<const uint2*>(xb + (static_cast<int64_t>(t0 + tr) * W + 4 * g) * 3);
        v[k][0] = src[0];
        v[k][1] = src[1];
        v[k][2] = src[2];
      }
      // all loads in flight before the first LDS write: hipcc sinks each load into the guarded
      // write block that uses it (one memory round trip per item); the empty asm consumes them here
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(v[k][i].x), "+v"(v[k][i].y));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = e0 + k * nthr;
        if (e >= total) break;
        const int tr = __float2int_rz((static_cast<float>(e) + 0.5f) * inv_g);
        const int g = e - tr * G;
        // 12 bf16 = pixels 4g..4g+3 x channels 0..2 -> four 8-B LDS pixels (channel 3 = 0)
        const uint32_t w0 = v[k][0].x, w1 = v[k][0].y, w2 = v[k][1].x, w3 = v[k][1].y,
                       w4 = v[k][2].x, w5 = v[k][2].y;
        uint2* dst = tile + (t0 + tr) * WT + 3 + 4 * g;
        dst[0] = make_uint2(w0, w1 & 0xffffu);
        dst[1] = make_uint2((w1 >> 16) | (w2 << 16), w2 >> 16);
        dst[2] = make_uint2(w3, w4 & 0xffffu);
        dst[3] = make_uint2((w4 >> 16) | (w5 << 16), w5 >> 16);
      }
    }
  } else {
#pragma unroll 3
    for (int t = 0; t < tile_rows(TY); ++t) {
      const int iy = iy0 + t;
      const bool rok = iy >= 0 && iy < H;
      const uint16_t* xr = x + (static_cast<int64_t>(n) * H + (rok ? iy : 0)) * W * C;
      for (int u = tid; u < WT; u += nthr) {
        const int ix = u - 3;
        uint2 v = make_uint2(0u, 0u);
        if (rok && ix >= 0 && ix < W) {
          if constexpr (C == 4) {
            v = *reinterpret_cast<const uint2*>(xr + static_cast<int64_t>(ix) * 4);
          } else {
            const uint16_t* q = xr + static_cast<int64_t>(ix) * C;
            const uint32_t c0 = q[0];
            const uint32_t c1 = C > 1 ? q[1] : 0u;
            const uint32_t c2 = C > 2 ? q[2] : 0u;
            v = make_uint2(c0 | (c1 << 16), c2);
          }
        }
        tile[t * WT + u] = v;
      }
    }
  }
}

// ----------------------------------------------------------------------------------- forward
template <int C, bool VEC>
__global__ __launch_bounds__(kFT) void stem_conv_fwd_kernel(const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ wpk,
                                                           uint16_t* __restrict__ z,
                                                           float* __restrict__ part, int N,
                                                           int H, int W, int OH, int OW) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint2* tile = reinterpret_cast<uint2*>(smem);
  const int WT = tile_cols(OW);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const float inv_ow = 1.f / static_cast<float>(OW);
  // B operand of step s, channel block b: lane (r, h) holds W[32 b + r][16 s + 8 h .. + 7]
  bf16x8_t wf[kSteps][2];
#pragma unroll
  for (int s = 0; s < kSteps; ++s)
#pragma unroll
    for (int b = 0; b < 2; ++b) wf[s][b] = ld_frag(wpk + (32 * b + r) * kKP + 16 * s + 8 * h);
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  const int bands = (OH + kTY - 1) / kTY;
  const int ntiles = N * bands;
  const int nblk = (kTY * OW + 31) / 32;
  for (int tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
    const int n = tl / bands;
    const int oy0 = (tl - n * bands) * kTY;
    const int pv = min(kTY, OH - oy0) * OW;            // valid pixels of the band
    __syncthreads();                                   // previous tile's LDS readers are done
    stage_input<C, kTY, VEC>(x, tile, n, oy0, H, W, WT, threadIdx.x, kFT);
    __syncthreads();
    uint16_t* zt = z + ((static_cast<int64_t>(n) * OH + oy0) * OW) * kCo;
    for (int blk = wave; blk < nblk; blk += kFT / 64) {
      const int p = 32 * blk + r;
      const int pc = p < pv ? p : 0;                   // rows past the band: read pixel 0, drop
      const int oyl = row_of(pc, inv_ow);
      const int ox = pc - oyl * OW;
      // A operand: lane (r = pixel, h) holds taps kx0 + 2h, kx0 + 2h + 1 x 4 channels of row ky
      const uint16_t* a0 = reinterpret_cast<const uint16_t*>(tile + 2 * oyl * WT + 2 * ox + 2 * h);
      f32x16 acc0 = {}, acc1 = {};
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        const bf16x8_t a = ld_frag(a0 + 4 * ((s >> 1) * WT + 4 * (s & 1)));
        acc0 = mfma(a, wf[s][0], acc0);
        acc1 = mfma(a, wf[s][1], acc1);
      }
      // register i: pixel 32 blk + (i & 3) + 8 (i >> 2) + 4 h, channel 32 b + r. One cvt_pk per
      // channel pair (r, r + 32) of a pixel, stored as its low and high halves.
      uint16_t* zb = zt + static_cast<int64_t>(32 * blk + 4 * h) * kCo + r;
      if (32 * (blk + 1) <= pv) {                      // whole block inside the band
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v0 = acc0[i], v1 = acc1[i];
          const uint32_t pk = static_cast<uint32_t>(f2bf(v0)) | (static_cast<uint32_t>(f2bf(v1)) << 16);
          uint16_t* zo = zb + ((i & 3) + 8 * (i >> 2)) * kCo;
          zo[0] = static_cast<uint16_t>(pk);
          zo[32] = static_cast<uint16_t>(pk >> 16);
          s1[0] += v0;
          s2[0] = fmaf(v0, v0, s2[0]);
          s1[1] += v1;
          s2[1] = fmaf(v1, v1, s2[1]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int pp = 32 * blk + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (pp < pv) {
            const float v0 = acc0[i], v1 = acc1[i];
            uint16_t* zo = zb + ((i & 3) + 8 * (i >> 2)) * kCo;
            zo[0] = f2bf(v0);
            zo[32] = f2bf(v1);
            s1[0] += v0;
            s2[0] = fmaf(v0, v0, s2[0]);
            s1[1] += v1;
            s2[1] = fmaf(v1, v1, s2[1]);
          }
        }
      }
    }
  }
  // workgroup partial [2][64] in a fixed order: (wave, half) slots summed by 128 threads
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);         // [4 waves][2 h][2 stat][64]
  const int slot = wave * 2 + h;
  red[(slot * 2 + 0) * kCo + r] = s1[0];
  red[(slot * 2 + 0) * kCo + 32 + r] = s1[1];
  red[(slot * 2 + 1) * kCo + r] = s2[0];
  red[(slot * 2 + 1) * kCo + 32 + r] = s2[1];
  __syncthreads();
  if (threadIdx.x < 2 * kCo) {
    const int st = threadIdx.x / kCo, c = threadIdx.x % kCo;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 2 * (kFT / 64); ++k) acc += red[(k * 2 + st) * kCo + c];
    part[static_cast<int64_t>(blockIdx.x) * 2 * kCo + st * kCo + c] = acc;
  }
}

// mean / invstd from the [nb][2][64] sums (fp64 fold, 16 slices x 64 channels, fixed order);
// running statistics update with the unbiased variance.
__global__ __launch_bounds__(1024) void stem_stats_finalize_kernel(const float* __restrict__ part,
                                                                  int nb, double M, float eps,
                                                                  float momentum,
                                                                  float* __restrict__ mean,
                                                                  float* __restrict__ invstd,
                                                                  float* __restrict__ rmean,
                                                                  float* __restrict__ rvar) {
  __shared__ double ls[16][kCo], lq[16][kCo];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
  double S = 0.0, Q = 0.0;
  for (int b = sl; b < nb; b += 16) {
    S += part[static_cast<int64_t>(b) * 2 * kCo + c];
    Q += part[static_cast<int64_t>(b) * 2 * kCo + kCo + c];
  }
  ls[sl][c] = S;
  lq[sl][c] = Q;
  __syncthreads();
  if (sl != 0) return;
  S = 0.0;
  Q = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    S += ls[k][c];
    Q += lq[k][c];
  }
  const double mu = S / M;
  double var = Q / M - mu * mu;
  if (var < 0.0) var = 0.0;
  mean[c] = static_cast<float>(mu);
  invstd[c] = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
  if (rmean) {
    const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
    rmean[c] = static_cast<float>((1.0 - momentum) * rmean[c] + momentum * mu);
    rvar[c] = static_cast<float>((1.0 - momentum) * rvar[c] + momentum * unb);
  }
}

// ---------------------------------------------------------------------------------- backward
// byte offset of 16-B chunk ch (8 channels) of pixel row rho in a [64 pixels][64 channels] image:
// chunks 0-3 / 4-7 swap on rows with bit 1 set, so the 4 rows of a transposed read hit 4 distinct
// 16-bank groups (no conflicts with 128-B rows)
__device__ __forceinline__ int chunk_off(int rho, int ch) {
  return rho * 128 + ((ch ^ (((rho >> 1) & 1) << 2)) << 4);
}

// GATHER: g is the max-pool's OUTPUT gradient [N][PH][PW][64] with the forward's argmax bytes pidx
// (3x3 / stride 2 / pad 1, window (j, i) covers rows 2j - 1 .. 2j + 1, tap = 3 row + col inside
// it, 255 = ReLU-masked window), so the full-resolution pool gradient (4x the pooled size) is never
// written or read. A chunk's 8 x 16 pixels lie in the 6 x 10 pooled windows from (oyc / 2 - 1,
// oxc / 2 - 1): that tile (7.5 KB of gradient + 3.75 KB of argmax bytes, one 16-B + 8-B item per
// thread) is prefetched like z, put in LDS, and every pixel sums the (up to) 2 x 2 windows that
// route to it. (Per-pixel window loads straight to registers needed 4 x 24 B per pixel and spilled.)
constexpr int kPR = 6, kPC = 10;                      // pooled rows / cols of a chunk's windows
constexpr int kPoolLds = kPR * kPC * (kCo * 2 + kCo);  // gradient [60][64] bf16 + argmax [60][64] B
// CLS (GATHER only): staging pixels are dealt to waves by pooled-window parity class -- (row & 1,
// col & 1) of a wave's pixels is wave-uniform, so a wave visits only the 1, 2 or 4 windows that
// can route to them (the per-pixel form evaluates all 4 per pixel, masked by tap); the SIMD
// partners w, w + 4 take complementary classes: (even, even) + (odd, odd) = 1 + 4 windows,
// (even, odd) + (odd, even) = 2 + 2, instead of 4 + 4
template <int C, bool VEC, int OWC, bool GATHER, bool CLS = false>
__global__ __launch_bounds__(kBT) void stem_wgrad_kernel(const uint16_t* __restrict__ g,
                                                        const uint16_t* __restrict__ z,
                                                        const uint16_t* __restrict__ x,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ gsum,
                                                        float* __restrict__ part, int N, int H,
                                                        int W, int OH, int OW_,
                                                        const uint8_t* __restrict__ pidx, int PH,
                                                        int PW) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* gbuf = smem;                                   // [128 px][64 ch] bf16, swizzled
  char* xbuf = smem + kCh * 128;
  uint2* tile = reinterpret_cast<uint2*>(smem + 2 * kCh * 128);
  // GATHER: the chunk's pooled tile after the input tile
  char* pgbuf = smem + 2 * kCh * 128 + ((tile_rows(kTYB) * tile_cols(OWC > 0 ? OWC : OW_) * 8 + 15) & ~15);
  char* pibuf = pgbuf + kPR * kPC * 128;
  // OWC > 0: the width is a compile-time constant (the 224-px ResNet input) and every chunk is
  // full, so the transposed reads of a chunk use one base address and immediate offsets
  const int OW = OWC > 0 ? OWC : OW_;
  const int WT = tile_cols(OW);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // scalar: uniform branches below
  const int h = lane >> 5, r = lane & 31;
  const int gi = lane & 15, grp = lane >> 4;           // 16-lane group of the transposed reads
  const int q = gi >> 2, pq = gi & 3;
  // wave -> M block mb (0, 1: g channels 0-31 / 32-63; 2, 3: xhat) x kernel rows ky0 .. +nky-1;
  // waves w and w + 4 share a SIMD, so every SIMD owns 4 + 3 = 7 accumulators
  const int mb = wave & 3;
  const int ky0 = wave < 4 ? 0 : 4;
  const int nky = wave < 4 ? 4 : 3;
  const char* abuf = (mb < 2 ? gbuf : xbuf) + 8 * (pq & 1);
  const int chn0 = 4 * (mb & 1) + 2 * (grp & 1) + (pq >> 1);
  // a chunk is an 8 x 16 block of output pixels, pixel rho = 16 row + col: the pixel rows of
  // k-step ks's transposed reads, rho = 16 ks + 8 h + 4 e + q, are row ks, col 8 h + 4 e + q
  const int cc = tid & 7, srho = tid >> 3;             // staging: pixels srho, srho + 64
  // CLS: class (pr, pc) = (wave >> 2, pr ^ (wave >> 1 & 1)), pixel rows pr + 2 (wave & 1) + 4 j,
  // columns pc + 2 (lane >> 3)
  const int cpr = wave >> 2, cpc = cpr ^ ((wave >> 1) & 1);
  auto pix_of = [&](int j) {
    if constexpr (CLS) return (cpr + 2 * (wave & 1) + 4 * j) * 16 + cpc + 2 * (lane >> 3);
    else return srho + 64 * j;
  };
  // g is staged as it is and mean(g) enters the finalize through the column sums of the input
  // patches (colA): staging g - mean(g) rounded every unrouted pixel's 0 - mean(g) to the same
  // bf16 value, a per-channel bias whose share of dW grew with the batch (profiles/r03_26/)
  float mu[8], is[8], s2[8], s1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    is[k] = invstd[8 * cc + k];
    mu[k] = -mean[8 * cc + k] * is[k];                 // xhat = z * is + mu
    s2[k] = 0.f;
    s1[k] = 0.f;
  }
  (void)gsum;
  f32x16 acc[4] = {};
  const int bands = (OH + kTYB - 1) / kTYB;
  const int ntiles = N * bands;
  const int ncx = (OW + 15) / 16;
  const int nch = 2 * ncx;                             // chunks per tile (cy 0..1, cx)
  // one-chunk register prefetch of (g, z) across the flattened (tile, chunk) sequence. Loads are
  // unconditional (clamped address) and invalid pixels are zeroed at use: a branch around the
  // loads makes the compiler wait for them at the join, i.e. no prefetch at all
  uint4 gv[GATHER ? 1 : 2], zv[2];
  bool okv[2];
  // GATHER: this thread's item of the chunk's pooled tile (pixel e / 8 of the 6 x 10 windows,
  // channels 8 (e % 8) ..; items >= 480 idle) and whether it lies inside the pooled image
  uint4 pv;
  uint2 iv;
  bool pok;
  const int pe = tid >> 3;
  auto fetch = [&](int tl, int ch) {
    const int n = tl / bands;
    const int oy0 = (tl - n * bands) * kTYB;
    const int cy = ch >= ncx ? 1 : 0, cx = ch - cy * ncx;
    const int oyend = min(OH, oy0 + kTYB);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rho = pix_of(j);
      const int oy = oy0 + 8 * cy + (rho >> 4), ox = 16 * cx + (rho & 15);
      okv[j] = tl < ntiles && oy < oyend && ox < OW;
      const int pix = okv[j] ? (n * OH + oy) * OW + ox : 0;
      const int64_t o = static_cast<int64_t>(pix) * kCo + 8 * cc;
      if constexpr (!GATHER) gv[j] = *reinterpret_cast<const uint4*>(g + o);
      zv[j] = *reinterpret_cast<const uint4*>(z + o);
    }
    if constexpr (GATHER) {
      const int pj = (oy0 + 8 * cy) / 2 - 1 + pe / kPC, pi = 8 * cx - 1 + pe % kPC;
      pok = tl < ntiles && pe < kPR * kPC && pj >= 0 && pj < PH && pi >= 0 && pi < PW;
      const int64_t po =
          ((static_cast<int64_t>(pok ? n : 0) * PH + (pok ? pj : 0)) * PW + (pok ? pi : 0)) * kCo +
          8 * cc;
      pv = *reinterpret_cast<const uint4*>(g + po);
      iv = *reinterpret_cast<const uint2*>(pidx + po);
    }
  };
  fetch(blockIdx.x, 0);
  for (int tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
    const int n = tl / bands;
    const int oy0 = (tl - n * bands) * kTYB;
    const int rows = min(kTYB, OH - oy0);              // valid rows of the band
    for (int ch = 0; ch < nch; ++ch) {
      const int cy = ch >= ncx ? 1 : 0, cx = ch - cy * ncx;
      const int r0 = 8 * cy, c0 = 16 * cx;             // chunk origin inside the band
      __syncthreads();                                 // previous chunk's / tile's readers done
      if (ch == 0) stage_input<C, kTYB, VEC>(x, tile, n, oy0, H, W, WT, tid, kBT);
      if constexpr (GATHER) {
        if (pe < kPR * kPC) {   // windows outside the pooled image route nothing (argmax 0xff)
          *reinterpret_cast<uint4*>(pgbuf + pe * 128 + 16 * cc) = pok ? pv : make_uint4(0u, 0u, 0u, 0u);
          *reinterpret_cast<uint2*>(pibuf + pe * 64 + 8 * cc) =
              pok ? iv : make_uint2(0xffffffffu, 0xffffffffu);
        }
        __syncthreads();
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        // ---- g / xhat of the prefetched pixels -> LDS; BN-backward sums
        const bool ok = OWC > 0 || okv[j];             // fixed-width instance: always valid
        float gf[8];
        if constexpr (GATHER) {
          // pixel (r, c) of the chunk (oyc, oxc even): windows (r + 1) / 2 + 1 - a, (c + 1) / 2 +
          // 1 - b of the tile, tap (ta + 2a, tb + 2b) with ta = (r + 1) & 1, tb = (c + 1) & 1
          const int rr = pix_of(j) >> 4, rc = pix_of(j) & 15;
          const int lr = ((rr + 1) >> 1) + 1, lc = ((rc + 1) >> 1) + 1;
          // CLS: the parities come from the (scalar) wave index, so the skips below are uniform
          const int ta = CLS ? 1 - cpr : (rr + 1) & 1, tb = CLS ? 1 - cpc : (rc + 1) & 1;
#pragma unroll
          for (int k = 0; k < 8; ++k) gf[k] = 0.f;
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              if (CLS && ((a == 1 && ta == 1) || (b == 1 && tb == 1))) continue;   // tap 3: none
              const int tta = ta + 2 * a, ttb = tb + 2 * b;
              const uint32_t me = tta <= 2 && ttb <= 2 ? static_cast<uint32_t>(3 * tta + ttb) : 0x100u;
              const int w = (lr - a) * kPC + (lc - b);
              const uint4 pw = *reinterpret_cast<const uint4*>(pgbuf + w * 128 + 16 * cc);
              const uint2 iw = *reinterpret_cast<const uint2*>(pibuf + w * 64 + 8 * cc);
              const uint32_t pw4[4] = {pw.x, pw.y, pw.z, pw.w};
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                const uint32_t byte = ((k < 4 ? iw.x : iw.y) >> (8 * (k & 3))) & 0xffu;
                const float d = (k & 1) ? __uint_as_float(pw4[k >> 1] & 0xffff0000u)
                                        : __uint_as_float(pw4[k >> 1] << 16);
                gf[k] += byte == me ? d : 0.f;
              }
            }
        } else {
          const uint32_t gw[4] = {gv[j].x, gv[j].y, gv[j].z, gv[j].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            gf[2 * k] = __uint_as_float(gw[k] << 16);
            gf[2 * k + 1] = __uint_as_float(gw[k] & 0xffff0000u);
          }
        }
        const uint32_t zw[4] = {zv[j].x, zv[j].y, zv[j].z, zv[j].w};
        uint32_t xw[4], cw[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float g0 = gf[2 * k], g1 = gf[2 * k + 1];
          float x0 = fmaf(__uint_as_float(zw[k] << 16), is[2 * k], mu[2 * k]);
          float x1 = fmaf(__uint_as_float(zw[k] & 0xffff0000u), is[2 * k + 1], mu[2 * k + 1]);
          float c0 = g0, c1 = g1;
          x0 = ok ? x0 : 0.f;
          x1 = ok ? x1 : 0.f;
          c0 = ok ? c0 : 0.f;
          c1 = ok ? c1 : 0.f;
          s2[2 * k] = fmaf(g0, x0, s2[2 * k]);
          s2[2 * k + 1] = fmaf(g1, x1, s2[2 * k + 1]);
          if constexpr (GATHER) {   // dbeta = sum g (fp32 gathered values, before rounding)
            s1[2 * k] += ok ? g0 : 0.f;
            s1[2 * k + 1] += ok ? g1 : 0.f;
          }
          xw[k] = static_cast<uint32_t>(f2bf(x0)) | (static_cast<uint32_t>(f2bf(x1)) << 16);
          cw[k] = static_cast<uint32_t>(f2bf(c0)) | (static_cast<uint32_t>(f2bf(c1)) << 16);
        }
        const int rho = pix_of(j);
        *reinterpret_cast<uint4*>(gbuf + chunk_off(rho, cc)) = make_uint4(cw[0], cw[1], cw[2], cw[3]);
        *reinterpret_cast<uint4*>(xbuf + chunk_off(rho, cc)) = make_uint4(xw[0], xw[1], xw[2], xw[3]);
      }
      if (ch + 1 < nch) fetch(tl, ch + 1);
      else fetch(tl + gridDim.x, 0);
      __syncthreads();
      if (r0 >= rows) continue;                        // chunk row entirely past the band
      auto run = [&](auto full_c) {
        constexpr bool FULL = decltype(full_c)::value;
        // B (input tile) address of k-step ks, half e: pixel (r0 + ks, c0 + 8 h + 4 e + q).
        // Partial chunks clamp the pixel into the band / image so every lane reads inside the
        // tile (invalid pixels have zero g / xhat rows); full chunks are one base + constant
        // offsets.
        auto baddr = [&](int ks, int e) {
          if constexpr (FULL) {
            return (2 * r0 + ky0) * WT + 2 * (c0 + 8 * h + q) + 4 * (grp & 1) + pq +
                   2 * ks * WT + 8 * e;
          } else {
            const int oyl = min(r0 + ks, rows - 1);
            const int oxl = min(c0 + 8 * h + 4 * e + q, OW - 1);
            return (2 * oyl + ky0) * WT + 2 * oxl + 4 * (grp & 1) + pq;
          }
        };
        // software pipeline: the fragments of k-step ks + 1 are read while ks's MFMAs run
        s16x4 fa[2][2], fb[2][4][2];
        auto load = [&](int ks, int buf) {
          const int rho0 = 16 * ks + 8 * h + q;
          fa[buf][0] = ld_tr(abuf + chunk_off(rho0, chn0));
          fa[buf][1] = ld_tr(abuf + chunk_off(rho0 + 4, chn0));
          const int b0 = baddr(ks, 0), b1 = baddr(ks, 1);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            if (kk < nky) {
              fb[buf][kk][0] = ld_tr(reinterpret_cast<const char*>(tile + b0 + kk * WT));
              fb[buf][kk][1] = ld_tr(reinterpret_cast<const char*>(tile + b1 + kk * WT));
            }
          }
        };
        auto step = [&](int ks, int buf) {
          (void)ks;
          const bf16x8_t A = cat(fa[buf][0], fa[buf][1]);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            if (kk < nky) acc[kk] = mfma(A, cat(fb[buf][kk][0], fb[buf][kk][1]), acc[kk]);
        };
        if constexpr (FULL) {
          // software pipeline over k-step pairs (rolled, so the scheduler cannot hoist every
          // fragment read of the chunk): k-step ks + 1's fragments load while ks's MFMAs run
          load(0, 0);
#pragma unroll 1
          for (int ks = 0; ks < kCh / 16; ks += 2) {
            load(ks + 1, 1);
            step(ks, 0);
            if (ks + 2 < kCh / 16) load(ks + 2, 0);
            step(ks + 1, 1);
          }
        } else {
#pragma unroll 1
          for (int ks = 0; ks < kCh / 16; ++ks) {
            load(ks, 0);
            step(ks, 0);
          }
        }
      };
      if constexpr (OWC > 0) {
        run(std::true_type{});                         // host guarantees OW == OWC, OH % kTYB == 0
      } else {
        run(std::false_type{});                        // generic shapes: clamped + masked path
      }
    }
  }
  // ---- partials: G [64][224], X [64][224], colA [224], s1 [64], s2 [64]
  float* pw = part + static_cast<int64_t>(blockIdx.x) * kPartW;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    if (kk < nky) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int co = 32 * (mb & 1) + (i & 3) + 8 * (i >> 2) + 4 * h;
        pw[(mb >> 1) * kCo * kKP + co * kKP + (ky0 + kk) * 32 + r] = acc[kk][i];
      }
    }
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);         // [64 staging rows][64]
#pragma unroll
  for (int k = 0; k < 8; ++k) red[srho * kCo + 8 * cc + k] = s2[k];
  __syncthreads();
  if (tid < kCo) {
    float s = 0.f;
    for (int k = 0; k < kBT / 8; ++k) s += red[k * kCo + tid];
    pw[2 * kCo * kKP + tid] = s;
  }
  if constexpr (GATHER) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) red[srho * kCo + 8 * cc + k] = s1[k];
    __syncthreads();
    if (tid < kCo) {
      float s = 0.f;
      for (int k = 0; k < kBT / 8; ++k) s += red[k * kCo + tid];
      pw[2 * kCo * kKP + kCo + tid] = s;
    }
  }
}

// ------------------------------------------------------- backward, producer / consumer form
// stem_wgrad_kernel<3, true, OWC, true> (the pool-gradient gather at a fixed width, OH % 16 == 0)
// with the two halves of the workgroup in fixed roles instead of alternating phases: waves 0-3
// (producers) stage chunk s -- pooled-gradient gather, BN terms, the bf16 g / xhat images -- while
// waves 4-7 (consumers) run chunk s - 1's MFMAs; one barrier per chunk. Each SIMD holds one wave
// of each role (w, w + 4), so its vector ALU (staging) and matrix pipe (products) work side by
// side; the alternating form ran them one after the other (rocprofv3 at batch 2560: MFMA busy
// 23 %, 42 % of wave time waiting, profiles/r06_19/). Chunk images and pooled tiles have two
// buffers each (pooled tile s + 1 is written during chunk s, so the one barrier orders it); the
// single input tile is restaged by all waves at a band change, between two barriers. A producer
// thread stages 4 pixels, one per pooled-window parity class (row & 1, col & 1) -- a compile-time
// constant per item, so each item visits exactly its 1, 2 or 4 windows. A consumer owns one M
// block (g or xhat x channel half) over all 7 kernel rows. Same partial layout and the same
// summation order per accumulator as the alternating kernel; the BN sums (s1, s2) are per-thread
// in a different pixel order.
constexpr int kPoolBuf = kPR * kPC * (kCo * 2 + kCo);      // one pooled tile: gradient + argmax
constexpr int kChunkBuf = 2 * kCh * 128;                   // one chunk's g and xhat images
template <int OWC>
constexpr int pc_tile_bytes() { return (tile_rows(kTYB) * tile_cols(OWC) * 8 + 15) & ~15; }
template <int OWC>
constexpr int pc_lds() { return 2 * kChunkBuf + pc_tile_bytes<OWC>() + 2 * kPoolBuf; }

template <int OWC>
__global__ __launch_bounds__(kBT) void stem_wgrad_pc_kernel(const uint16_t* __restrict__ g,
                                                           const uint16_t* __restrict__ z,
                                                           const uint16_t* __restrict__ x,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           float* __restrict__ part, int N, int H,
                                                           int W, int OH,
                                                           const uint8_t* __restrict__ pidx, int PH,
                                                           int PW, int abl) {
  static_assert(OWC % 16 == 0 && pc_lds<OWC>() <= 160 * 1024, "stem_wgrad_pc shape");
  constexpr int OW = OWC, WT = tile_cols(OWC);
  constexpr int ncx = OWC / 16, nch = 2 * ncx;          // chunks per band (cy 0..1, cx)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* cbuf = smem;                                     // [2][g | xhat] chunk images
  uint2* tile = reinterpret_cast<uint2*>(smem + 2 * kChunkBuf);
  char* pbuf = smem + 2 * kChunkBuf + pc_tile_bytes<OWC>();   // [2] pooled tiles
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool prod = wave < 4;
  const int bands = OH / kTYB;
  const int ntiles = N * bands;
  const int mytiles =
      static_cast<int>(blockIdx.x) < ntiles ? (ntiles - 1 - static_cast<int>(blockIdx.x)) / gridDim.x + 1 : 0;
  const int S = mytiles * nch;
  // chunk s of this workgroup -> image, band origin, chunk (cy, cx); false (clamped) past the end
  auto chunk_pos = [&](int s, int& n, int& oy0, int& cy, int& cx) {
    const int k = s / nch, ch = s - k * nch;
    const bool ok = s < S;
    const int tl = ok ? static_cast<int>(blockIdx.x) + k * static_cast<int>(gridDim.x)
                      : static_cast<int>(blockIdx.x) % (ntiles > 0 ? ntiles : 1);
    n = tl / bands;
    oy0 = (tl - n * bands) * kTYB;
    cy = ch >= ncx ? 1 : 0;
    cx = ch - cy * ncx;
    return ok;
  };

  // ---- producer state: channel group cc, column pair pk, row pair pw (pixel row pr + 2 pw,
  // column pc + 2 pk of class j = 2 pr + pc)
  const int cc = tid & 7, pk = (tid >> 3) & 7, pwv = wave & 3;
  float mu[8], is[8], s2[8], s1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    is[k] = invstd[8 * cc + k];
    mu[k] = -mean[8 * cc + k] * is[k];
    s2[k] = 0.f;
    s1[k] = 0.f;
  }
  // register sets of even / odd chunks (A / B): z of chunk s is loaded two iterations ahead, the
  // pooled tile of chunk s three ahead (it is written to LDS one iteration before it is read)
  uint4 zA[4], zB[4];
  struct PoolRegs {
    uint4 v[2];
    uint2 i[2];
    bool ok[2];
  } pA, pB;
  auto fetch_z = [&](uint4 (&zv)[4], int s) {
    int n, oy0, cy, cx;
    const bool ok = chunk_pos(s, n, oy0, cy, cx);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = (j >> 1) + 2 * pwv, col = (j & 1) + 2 * pk;
      const int pix = ok ? (n * OH + oy0 + 8 * cy + row) * OW + 16 * cx + col : 0;
      zv[j] = *reinterpret_cast<const uint4*>(z + static_cast<int64_t>(pix) * kCo + 8 * cc);
    }
  };
  // pooled tile items: window e = tid / 8 + 32 u (60 of 64 used), channels 8 cc ..
  auto fetch_pool = [&](PoolRegs& pr, int s) {
    int n, oy0, cy, cx;
    const bool ok = chunk_pos(s, n, oy0, cy, cx);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = (tid >> 3) + 32 * u;
      const int pj = (oy0 + 8 * cy) / 2 - 1 + e / kPC, pi = 8 * cx - 1 + e % kPC;
      const bool pok = ok && e < kPR * kPC && pj >= 0 && pj < PH && pi >= 0 && pi < PW;
      pr.ok[u] = pok;
      const int64_t po =
          ((static_cast<int64_t>(pok ? n : 0) * PH + (pok ? pj : 0)) * PW + (pok ? pi : 0)) * kCo +
          8 * cc;
      pr.v[u] = *reinterpret_cast<const uint4*>(g + po);
      pr.i[u] = *reinterpret_cast<const uint2*>(pidx + po);
    }
  };
  // the buffer parity of chunk s is a compile-time constant at every call (PAR = s & 1): the two
  // halves of the unrolled producer loop then differ in their LDS offsets, so they are not merged
  // back into one body (hipcc did, rotating the A / B sets through copies that waited on the loads)
  auto put_pool = [&](const PoolRegs& pr, auto par_c) {   // a chunk's tile -> pooled buffer PAR
    constexpr int PAR = decltype(par_c)::value;
    char* pg = pbuf + PAR * kPoolBuf;
    char* pi = pg + kPR * kPC * 128;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = (tid >> 3) + 32 * u;
      if (e < kPR * kPC) {   // windows outside the pooled image route nothing (argmax 0xff)
        *reinterpret_cast<uint4*>(pg + e * 128 + 16 * cc) =
            pr.ok[u] ? pr.v[u] : make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint2*>(pi + e * 64 + 8 * cc) =
            pr.ok[u] ? pr.i[u] : make_uint2(0xffffffffu, 0xffffffffu);
      }
    }
  };
  auto produce = [&](const uint4 (&zv)[4], auto par_c) {    // a chunk -> chunk buffer PAR
    constexpr int PAR = decltype(par_c)::value;
    const char* pg = pbuf + PAR * kPoolBuf;
    const char* pi = pg + kPR * kPC * 128;
    char* gb = cbuf + PAR * kChunkBuf;
    char* xb = gb + kCh * 128;
    auto item = [&](auto j_c) {
      constexpr int j = decltype(j_c)::value;
      constexpr int pr = j >> 1, pc = j & 1, ta = 1 - pr, tb = 1 - pc;
      const int row = pr + 2 * pwv, col = pc + 2 * pk;
      const int lr = ((row + 1) >> 1) + 1, lc = ((col + 1) >> 1) + 1;
      float gf[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) gf[k] = 0.f;
#pragma unroll
      for (int a = 0; a <= pr; ++a)
#pragma unroll
        for (int b = 0; b <= pc; ++b) {   // taps (ta + 2 a, tb + 2 b) <= 2: the routing windows
          const uint32_t me = static_cast<uint32_t>(3 * (ta + 2 * a) + tb + 2 * b);
          const int w = (lr - a) * kPC + (lc - b);
          const uint4 pw4v = *reinterpret_cast<const uint4*>(pg + w * 128 + 16 * cc);
          const uint2 iw = *reinterpret_cast<const uint2*>(pi + w * 64 + 8 * cc);
          const uint32_t pw4[4] = {pw4v.x, pw4v.y, pw4v.z, pw4v.w};
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t byte = ((k < 4 ? iw.x : iw.y) >> (8 * (k & 3))) & 0xffu;
            const float d = (k & 1) ? __uint_as_float(pw4[k >> 1] & 0xffff0000u)
                                    : __uint_as_float(pw4[k >> 1] << 16);
            gf[k] += byte == me ? d : 0.f;
          }
        }
      const uint32_t zw[4] = {zv[j].x, zv[j].y, zv[j].z, zv[j].w};
      uint32_t xw[4], cw[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float g0 = gf[2 * k], g1 = gf[2 * k + 1];
        const float x0 = fmaf(__uint_as_float(zw[k] << 16), is[2 * k], mu[2 * k]);
        const float x1 = fmaf(__uint_as_float(zw[k] & 0xffff0000u), is[2 * k + 1], mu[2 * k + 1]);
        s2[2 * k] = fmaf(g0, x0, s2[2 * k]);
        s2[2 * k + 1] = fmaf(g1, x1, s2[2 * k + 1]);
        s1[2 * k] += g0;
        s1[2 * k + 1] += g1;
        xw[k] = pk_bf16(x0, x1);
        cw[k] = pk_bf16(g0, g1);
      }
      const int rho = row * 16 + col;
      *reinterpret_cast<uint4*>(gb + chunk_off(rho, cc)) = make_uint4(cw[0], cw[1], cw[2], cw[3]);
      *reinterpret_cast<uint4*>(xb + chunk_off(rho, cc)) = make_uint4(xw[0], xw[1], xw[2], xw[3]);
    };
    item(std::integral_constant<int, 0>{});
    item(std::integral_constant<int, 1>{});
    item(std::integral_constant<int, 2>{});
    item(std::integral_constant<int, 3>{});
  };

  // ---- consumer state: M block mb (0, 1: g channels 0-31 / 32-63; 2, 3: xhat), kernel rows 0-6
  const int mb = wave & 3;
  const int h = lane >> 5, r = lane & 31;
  const int gi = lane & 15, grp = lane >> 4;
  const int q = gi >> 2, pq = gi & 3;
  const int chn0 = 4 * (mb & 1) + 2 * (grp & 1) + (pq >> 1);
  f32x16 acc[7] = {};
  auto consume = [&](int s) {
    int n, oy0, cy, cx;
    chunk_pos(s, n, oy0, cy, cx);
    const int r0 = 8 * cy, c0 = 16 * cx;
    const char* abuf = cbuf + (s & 1) * kChunkBuf + (mb < 2 ? 0 : kCh * 128) + 8 * (pq & 1);
    // B (input tile) address of k-step ks, half e: pixel (r0 + ks, c0 + 8 h + 4 e + q), row ky 0
    const int bbase = 2 * r0 * WT + 2 * (c0 + 8 * h + q) + 4 * (grp & 1) + pq;
    s16x4 fa[2][2], fb[2][7][2];
    auto load = [&](int ks, int buf) {
      const int rho0 = 16 * ks + 8 * h + q;
      fa[buf][0] = ld_tr(abuf + chunk_off(rho0, chn0));
      fa[buf][1] = ld_tr(abuf + chunk_off(rho0 + 4, chn0));
      const int b0 = bbase + 2 * ks * WT;
#pragma unroll
      for (int kk = 0; kk < 7; ++kk) {
        fb[buf][kk][0] = ld_tr(reinterpret_cast<const char*>(tile + b0 + kk * WT));
        fb[buf][kk][1] = ld_tr(reinterpret_cast<const char*>(tile + b0 + kk * WT + 8));
      }
    };
    auto step = [&](int buf) {
      const bf16x8_t A = cat(fa[buf][0], fa[buf][1]);
#pragma unroll
      for (int kk = 0; kk < 7; ++kk) acc[kk] = mfma(A, cat(fb[buf][kk][0], fb[buf][kk][1]), acc[kk]);
    };
    load(0, 0);
#pragma unroll 1
    for (int ks = 0; ks < kCh / 16; ks += 2) {
      load(ks + 1, 1);
      step(0);
      if (ks + 2 < kCh / 16) load(ks + 2, 0);
      step(1);
    }
  };

  // ---- pipeline: iteration s = producers stage chunk s, consumers multiply chunk s - 1. The two
  // roles run separate loops with the same barrier sequence (wave-uniform roles), so neither
  // role's registers are live in the other's loop.
  // abl (timing ablations, CML_STEM_PC_ABL; results are wrong when set): 1 no staging compute,
  // 2 no products, 4 no input-tile restage
  auto band_change = [&](int s) {   // consumers enter a new band at chunk s - 1: restage the tile
    if (s >= 1 && (s - 1) % nch == 0) {
      int n, oy0, cy, cx;
      chunk_pos(s - 1, n, oy0, cy, cx);
      if (!(abl & 4)) stage_input<3, kTYB, true>(x, tile, n, oy0, H, W, WT, tid, kBT);
      __syncthreads();
    }
  };
  float* pw = part + static_cast<int64_t>(blockIdx.x) * kPartW;
  if (prod) {
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    fetch_pool(pA, 0);
    put_pool(pA, P0{});
    fetch_pool(pB, 1);
    fetch_pool(pA, 2);
    fetch_z(zA, 0);
    fetch_z(zB, 1);
    __syncthreads();
    // unrolled by two so the A / B register sets are named statically
    for (int s = 0; s <= S; s += 2) {
      band_change(s);
      if (s < S) {
        if (!(abl & 1)) produce(zA, P0{});
        put_pool(pB, P1{});
      }
      // loads unconditional (clamped past the end): a path without them would make the compiler's
      // in-order vmcnt accounting wait for the newest loads at the next use
      fetch_pool(pB, s + 3);
      fetch_z(zA, s + 2);
      __syncthreads();
      if (s + 1 > S) break;
      band_change(s + 1);
      if (s + 1 < S) {
        if (!(abl & 1)) produce(zB, P1{});
        put_pool(pA, P0{});
      }
      fetch_pool(pA, s + 4);
      fetch_z(zB, s + 3);
      __syncthreads();
    }
  } else {
    __syncthreads();
    for (int s = 0; s <= S; ++s) {
      band_change(s);
      if (s >= 1 && !(abl & 2)) consume(s - 1);
      __syncthreads();
    }
    // G [64][224], X [64][224]
#pragma unroll
    for (int kk = 0; kk < 7; ++kk)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int co = 32 * (mb & 1) + (i & 3) + 8 * (i >> 2) + 4 * h;
        pw[(mb >> 1) * kCo * kKP + co * kKP + kk * 32 + r] = acc[kk][i];
      }
  }

  // ---- s2 [64], s1 [64] from the producers' per-thread sums
  float* red = reinterpret_cast<float*>(smem);           // [32 producer rows][64]
  const int prow = tid >> 3;
  if (prod) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[prow * kCo + 8 * cc + k] = s2[k];
  }
  __syncthreads();
  if (tid < kCo) {
    float sum = 0.f;
    for (int k = 0; k < 32; ++k) sum += red[k * kCo + tid];
    pw[2 * kCo * kKP + tid] = sum;
  }
  __syncthreads();
  if (prod) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[prow * kCo + 8 * cc + k] = s1[k];
  }
  __syncthreads();
  if (tid < kCo) {
    float sum = 0.f;
    for (int k = 0; k < 32; ++k) sum += red[k * kCo + tid];
    pw[2 * kCo * kKP + kCo + tid] = sum;
  }
}

// fold the [nb][kPartW] partials (fp64, fixed order; 4 in flight per thread)
__global__ __launch_bounds__(256) void stem_wgrad_fold_kernel(const float* __restrict__ part, int nb,
                                                             double* __restrict__ tot) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= kPartW) return;
  double S = 0.0;
  int b = 0;
  for (; b + 3 < nb; b += 4) {
    const float v0 = part[static_cast<int64_t>(b) * kPartW + e];
    const float v1 = part[static_cast<int64_t>(b + 1) * kPartW + e];
    const float v2 = part[static_cast<int64_t>(b + 2) * kPartW + e];
    const float v3 = part[static_cast<int64_t>(b + 3) * kPartW + e];
    S += v0;
    S += v1;
    S += v2;
    S += v3;
  }
  for (; b < nb; ++b) S += part[static_cast<int64_t>(b) * kPartW + e];
  tot[e] = S;
}

// dW[co][c][ky][kx] = gamma invstd (G - s1/M colA - s2/M X) with G = sum g (x) im2col,
// X = sum xhat (x) im2col, colA[k] = sum over pixels of im2col[.][k] (stem_cola); dgamma = s2,
// dbeta = s1 = sum g: the channel sums of the pool backward (gsum) or, without them (GATHER), the
// kernel's own partials.
// BF: the three outputs in bf16 (RNE of the fp32 values: the parameters' dtype, no cast launches)
// (the empty asm keeps the fp32 rounding step: without it the fp64 -> fp32 -> bf16 conversion chain
// may be folded into one fp64 -> bf16 rounding, which differs from casting the fp32 output where
// the fp32 value is a bf16 tie)
template <bool BF>
__device__ __forceinline__ void stem_out(void* p, int i, float v) {
  if constexpr (BF) {
    asm volatile("" : "+v"(v));
    reinterpret_cast<uint16_t*>(p)[i] = f2bf(v);
  } else {
    reinterpret_cast<float*>(p)[i] = v;
  }
}

template <bool BF>
__global__ __launch_bounds__(256) void stem_wgrad_final_kernel(const double* __restrict__ tot,
                                                              const uint16_t* __restrict__ gamma,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ gsum,
                                                              const double* __restrict__ cola,
                                                              double M, int C,
                                                              void* __restrict__ dw,
                                                              void* __restrict__ dgamma,
                                                              void* __restrict__ dbeta) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const double* G = tot;
  const double* X = tot + kCo * kKP;
  const double* S2 = tot + 2 * kCo * kKP;
  const double* S1 = S2 + kCo;
  if (e < kCo * C * 49) {
    const int co = e / (C * 49);
    const int rem = e - co * C * 49;
    const int c = rem / 49, t = rem - (rem / 49) * 49;
    const int ky = t / 7, kx = t - ky * 7;
    const int kc = (ky * 8 + kx) * 4 + c;
    const double a = static_cast<double>(bf2f(gamma[co])) * invstd[co];
    const double s1 = gsum ? static_cast<double>(gsum[co]) : S1[co];
    double ca = 0.0;
    for (int sl = 0; sl < kColaS; ++sl) ca += cola[sl * kKP + kc];
    stem_out<BF>(dw, e, static_cast<float>(
        a * (G[co * kKP + kc] - s1 / M * ca - S2[co] / M * X[co * kKP + kc])));
  }
  if (e < kCo) {
    stem_out<BF>(dgamma, e, static_cast<float>(S2[e]));
    stem_out<BF>(dbeta, e, gsum ? gsum[e] : static_cast<float>(S1[e]));
  }
}

// colA[k], k = (ky * 8 + kx) * 4 + c: the sum over every output pixel (n, oy, ox) of the input
// patch value x[n][2 oy + ky - 3][2 ox + kx - 3][c] (0 outside the image). Pass 1 sums x over
// chunks of kColaChunk images per input pixel (grid = input rows x image chunks, a thread per
// (column, channel), images in order, 8 loads in flight) into fp32 partials [chunk][H][W][C];
// pass 2 (kColaS workgroups per tap) adds, in fp64 and a fixed order, the partials of the pixels
// that tap (ky, kx) reaches: rows ky - 3 + 2 oy and columns kx - 3 + 2 ox inside the image.
constexpr int kColaChunk = 128;   // images per partial
// V: 16-B loads (W C a multiple of 8): thread = 8 consecutive (column, channel) values of the row
// x one of 256 / (W C / 8) image slices (fixed-order LDS combine of the slices)
template <bool V>
__global__ __launch_bounds__(256) void stem_cola_rows_kernel(const uint16_t* __restrict__ x, int N,
                                                            int H, int W, int C,
                                                            float* __restrict__ part) {
  const int iy = blockIdx.x;
  const int n0 = blockIdx.y * kColaChunk, n1 = min(N, n0 + kColaChunk);
  const int64_t img = static_cast<int64_t>(H) * W * C;
  const int WC = W * C;
  float* out = part + (static_cast<int64_t>(blockIdx.y) * H + iy) * WC;
  if constexpr (V) {
    __shared__ float red[256][9];
    const int G8 = WC / 8;
    const int nsl = G8 >= 256 ? 1 : 256 / G8;
    for (int gb = 0; gb < G8; gb += 256 / nsl) {
      const int grp = gb + threadIdx.x % (256 / nsl), sl = threadIdx.x / (256 / nsl);
      float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (grp < G8 && sl < nsl) {
        const uint16_t* px = x + static_cast<int64_t>(iy) * WC + 8 * grp;
        int n = n0 + sl;
        for (; n + 3 * nsl < n1; n += 4 * nsl) {
          float v[4][8];
#pragma unroll
          for (int u = 0; u < 4; ++u) load_vec<bf16, 8>(reinterpret_cast<const bf16*>(px + (n + u * nsl) * img), v[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] += v[u][k];
        }
        for (; n < n1; n += nsl) {
          float v[8];
          load_vec<bf16, 8>(reinterpret_cast<const bf16*>(px + n * img), v);
#pragma unroll
          for (int k = 0; k < 8; ++k) a[k] += v[k];
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) red[threadIdx.x][k] = a[k];
      __syncthreads();
      const int per = 256 / nsl;
      if (threadIdx.x < per && gb + threadIdx.x < G8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float s = 0.f;
          for (int q = 0; q < nsl; ++q) s += red[q * per + threadIdx.x][k];
          out[8 * (gb + threadIdx.x) + k] = s;
        }
      }
    }
  } else {
    for (int e = threadIdx.x; e < WC; e += 256) {
      const uint16_t* px = x + static_cast<int64_t>(iy) * WC + e;
      float a = 0.f;
      int n = n0;
      for (; n + 8 <= n1; n += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = bf2f(px[(n + u) * img]);
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u];
      }
      for (; n < n1; ++n) a += bf2f(px[n * img]);
      out[e] = a;
    }
  }
}

// kColaS 1024-thread workgroups per tap, each over every kColaS-th block of kColaT output pixels;
// a thread issues the kColaU chunk partials of a pixel (x C channels) as independent loads before
// adding them (one workgroup per tap with a serial chain of dependent loads per pixel made this
// pass latency bound: 423 us at batch 2048, profiles/r04_26/), then a fixed-order wave shuffle +
// LDS combine into cola[slice][tap][4]; stem_wgrad_final adds the slices in order (deterministic)
constexpr int kColaT = 1024, kColaU = 8;
__global__ __launch_bounds__(kColaT) void stem_cola_kernel(const float* __restrict__ part, int nchunk,
                                                          int H, int W, int C, int OH, int OW,
                                                          double* __restrict__ cola) {
  __shared__ double red[kColaT / 64][4];
  const int t = blockIdx.x;                 // tap ky * 8 + kx (kx = 7: the zero tap)
  const int ky = t / 8, kx = t - 8 * (t / 8);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  if (kx < 7) {
    const int64_t plane = static_cast<int64_t>(H) * W * C;
    for (int q = blockIdx.y * kColaT + threadIdx.x; q < OH * OW; q += kColaS * kColaT) {
      const int oy = q / OW, ox = q - oy * OW;
      const int iy = ky - 3 + 2 * oy, ix = kx - 3 + 2 * ox;
      if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
      const float* d = part + (static_cast<int64_t>(iy) * W + ix) * C;
      int k = 0;
      for (; k + kColaU <= nchunk; k += kColaU) {
        float v[kColaU][4];
#pragma unroll
        for (int u = 0; u < kColaU; ++u)
#pragma unroll
          for (int c = 0; c < 4; ++c) {   // channel C..3 reads clamp to C - 1 and count 0
            const float e = d[(k + u) * plane + (c < C ? c : C - 1)];
            v[u][c] = c < C ? e : 0.f;
          }
#pragma unroll
        for (int u = 0; u < kColaU; ++u)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[c] += v[u][c];
      }
      for (; k < nchunk; ++k)
        for (int c = 0; c < C; ++c) acc[c] += d[k * plane + c];
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc[c] += __shfl_xor(acc[c], o);
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c) red[wave][c] = acc[c];
  __syncthreads();
  if (threadIdx.x < 4) {
    double s = 0.0;
    for (int k = 0; k < kColaT / 64; ++k) s += red[k][threadIdx.x];
    cola[blockIdx.y * kKP + t * 4 + threadIdx.x] = threadIdx.x < C ? s : 0.0;
  }
}

size_t fwd_lds(int OW) {   // input tile; the final reduction reuses it
  const size_t need = static_cast<size_t>(tile_rows(kTY)) * tile_cols(OW) * 8;
  const size_t red = static_cast<size_t>(kFT / 64) * 2 * 2 * kCo * sizeof(float);
  return need > red ? need : red;
}
size_t bwd_lds(int OW, bool gather = true) {   // chunk images + input tile (+ pooled tile); the
                                                 // final reduction reuses it
  const size_t need = 2 * kCh * 128 +
                      ((static_cast<size_t>(tile_rows(kTYB)) * tile_cols(OW) * 8 + 15) & ~static_cast<size_t>(15)) +
                      (gather ? kPoolLds : 0);
  const size_t red = static_cast<size_t>(kBT / 8) * kCo * sizeof(float);
  return need > red ? need : red;
}

int persistent_grid(const void* fn, int threads, size_t lds, int ntiles) {
  int dev = 0, cus = 256, occ = 1;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, lds) != hipSuccess || occ < 1) occ = 1;
  const int g = cus * occ;
  return g < ntiles ? g : ntiles;
}

// the backward tile needs > 64 KiB of dynamic LDS: opt in once per kernel instance
void wgrad_lds_optin() {
  static const bool done = [] {
    const void* fns[9] = {reinterpret_cast<const void*>(&stem_wgrad_kernel<3, true, 112, true, true>),
                          reinterpret_cast<const void*>(&stem_wgrad_kernel<3, true, 112, false>),
                          reinterpret_cast<const void*>(&stem_wgrad_kernel<3, true, 0, false>),
                          reinterpret_cast<const void*>(&stem_wgrad_kernel<3, false, 0, false>),
                          reinterpret_cast<const void*>(&stem_wgrad_kernel<4, false, 0, false>),
                          reinterpret_cast<const void*>(&stem_wgrad_kernel<3, true, 112, true>),
                          reinterpret_cast<const void*>(&stem_wgrad_kernel<3, true, 0, true>),
                          reinterpret_cast<const void*>(&stem_wgrad_kernel<3, false, 0, true>),
                          reinterpret_cast<const void*>(&stem_wgrad_kernel<4, false, 0, true>)};
    for (const void* f : fns)
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_wgrad_pc_kernel<112>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, pc_lds<112>());
    return true;
  }();
  (void)done;
}

}  // namespace

int stem_fwd_grid(int N, int OH, int OW, int C) {
  const int ntiles = N * ((OH + kTY - 1) / kTY);
  const void* fn = C == 4 ? reinterpret_cast<const void*>(&stem_conv_fwd_kernel<4, false>)
                          : reinterpret_cast<const void*>(&stem_conv_fwd_kernel<3, true>);
  return persistent_grid(fn, kFT, fwd_lds(OW), ntiles);
}

int stem_bwd_grid(int N, int OH, int OW, int C) {
  wgrad_lds_optin();
  const int ntiles = N * ((OH + kTYB - 1) / kTYB);
  const void* fn = C == 4 ? reinterpret_cast<const void*>(&stem_wgrad_kernel<4, false, 0, true>)
                          : reinterpret_cast<const void*>(&stem_wgrad_kernel<3, true, 112, true>);
  return persistent_grid(fn, kBT, bwd_lds(OW), ntiles);
}

size_t stem_wgrad_part_floats() { return kPartW; }
size_t stem_wgrad_tot_doubles() { return kPartW + kColaS * kKP; }   // partial totals + colA slices
size_t stem_cola_work_floats(int N, int H, int W, int C) {
  return static_cast<size_t>((N + kColaChunk - 1) / kColaChunk) * H * W * C;
}

hipError_t launch_stem_conv_fwd(const void* x, const void* wpk, void* z, float* part, int grid,
                                float* mean, float* invstd, float* rmean, float* rvar, float eps,
                                float momentum, int N, int H, int W, int C, int OH, int OW,
                                hipStream_t st) {
  if ((C != 3 && C != 4) || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1 || N < 1 || grid < 1)
    return hipErrorInvalidValue;
  if (fwd_lds(OW) > 64 * 1024 || OH * OW >= (1 << 20)) return hipErrorInvalidValue;
  const size_t lds = fwd_lds(OW);
  const auto* xp = reinterpret_cast<const uint16_t*>(x);
  const auto* wp = reinterpret_cast<const uint16_t*>(wpk);
  auto* zp = reinterpret_cast<uint16_t*>(z);
  const bool vec = C == 3 && W % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0;
  if (C == 4) stem_conv_fwd_kernel<4, false><<<grid, kFT, lds, st>>>(xp, wp, zp, part, N, H, W, OH, OW);
  else if (vec) stem_conv_fwd_kernel<3, true><<<grid, kFT, lds, st>>>(xp, wp, zp, part, N, H, W, OH, OW);
  else stem_conv_fwd_kernel<3, false><<<grid, kFT, lds, st>>>(xp, wp, zp, part, N, H, W, OH, OW);
  if (mean != nullptr)
    stem_stats_finalize_kernel<<<1, 1024, 0, st>>>(part, grid, static_cast<double>(N) * OH * OW,
                                                   eps, momentum, mean, invstd, rmean, rvar);
  return hipGetLastError();
}

hipError_t launch_stem_wgrad(const void* g, const void* z, const void* x, const float* mean,
                             const float* invstd, const void* gamma, const float* gsum,
                             float* part, int grid, double* tot, void* dw, void* dgamma,
                             void* dbeta, int N, int H, int W, int C, int OH, int OW,
                             hipStream_t st, const uint8_t* pidx, float* cola_work,
                             bool out_bf16) {
  if (!cola_work || (!pidx && !gsum)) return hipErrorInvalidValue;
  if ((C != 3 && C != 4) || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1 || N < 1 || grid < 1)
    return hipErrorInvalidValue;
  if (bwd_lds(OW, pidx != nullptr) > 120 * 1024 ||
      static_cast<int64_t>(N) * OH * OW >= (1ll << 31) / kCo)
    return hipErrorInvalidValue;
  const size_t lds = bwd_lds(OW, pidx != nullptr);
  wgrad_lds_optin();
  const auto* gp = reinterpret_cast<const uint16_t*>(g);
  const auto* zp = reinterpret_cast<const uint16_t*>(z);
  const auto* xp = reinterpret_cast<const uint16_t*>(x);
  const int PH = (OH - 1) / 2 + 1, PW = (OW - 1) / 2 + 1;   // the 3x3 / s2 / p1 pool's output
  const bool vec = C == 3 && W % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0;
#define CML_WG(CC, V, OWC, G) stem_wgrad_kernel<CC, V, OWC, G><<<grid, kBT, lds, st>>>(gp, zp, xp, mean, invstd, gsum, part, N, H, W, OH, OW, pidx, PH, PW)
  // CML_STEM_CLS=0: the per-pixel window form of the bench-shape gather instance (A/B)
  const char* cls_env = std::getenv("CML_STEM_CLS");
  const bool cls = !(cls_env && cls_env[0] == '0');
#define CML_WG_ALL(G)                                       \
  if (C == 4) CML_WG(4, false, 0, G);                        \
  else if (G && cls && vec && OW == 112 && OH % kTYB == 0)   \
    stem_wgrad_kernel<3, true, 112, true, true><<<grid, kBT, lds, st>>>(gp, zp, xp, mean, invstd, gsum, part, N, H, W, OH, OW, pidx, PH, PW); \
  else if (vec && OW == 112 && OH % kTYB == 0) CML_WG(3, true, 112, G); \
  else if (vec) CML_WG(3, true, 0, G);                       \
  else CML_WG(3, false, 0, G);
  // CML_STEM_PC=0: the alternating kernel at the bench shape too (A/B)
  const char* pc_env = std::getenv("CML_STEM_PC");
  const bool pc = !(pc_env && pc_env[0] == '0');
  if (pidx && pc && C == 3 && vec && OW == 112 && OH % kTYB == 0) {
    const char* abl_env = std::getenv("CML_STEM_PC_ABL");
    const int abl = abl_env ? std::atoi(abl_env) : 0;
    stem_wgrad_pc_kernel<112><<<grid, kBT, pc_lds<112>(), st>>>(gp, zp, xp, mean, invstd, part, N,
                                                               H, W, OH, pidx, PH, PW, abl);
  } else if (pidx) {
    CML_WG_ALL(true)
  } else {
    CML_WG_ALL(false)
  }
#undef CML_WG_ALL
#undef CML_WG
  stem_wgrad_fold_kernel<<<(kPartW + 255) / 256, 256, 0, st>>>(part, grid, tot);
  double* cola = tot + kPartW;   // tot has room for the column sums after the partial totals
  const int nchunk = (N + kColaChunk - 1) / kColaChunk;
  const bool v16 = (W * C) % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (v16) stem_cola_rows_kernel<true><<<dim3(H, nchunk), 256, 0, st>>>(xp, N, H, W, C, cola_work);
  else stem_cola_rows_kernel<false><<<dim3(H, nchunk), 256, 0, st>>>(xp, N, H, W, C, cola_work);
  stem_cola_kernel<<<dim3(kKP / 4, kColaS), kColaT, 0, st>>>(cola_work, nchunk, H, W, C, OH, OW, cola);
  if (out_bf16)
    stem_wgrad_final_kernel<true><<<(kCo * C * 49 + 255) / 256, 256, 0, st>>>(
        tot, reinterpret_cast<const uint16_t*>(gamma), invstd, pidx ? nullptr : gsum, cola,
        static_cast<double>(N) * OH * OW, C, dw, dgamma, dbeta);
  else
    stem_wgrad_final_kernel<false><<<(kCo * C * 49 + 255) / 256, 256, 0, st>>>(
        tot, reinterpret_cast<const uint16_t*>(gamma), invstd, pidx ? nullptr : gsum, cola,
        static_cast<double>(N) * OH * OW, C, dw, dgamma, dbeta);
  return hipGetLastError();
}

}  // namespace cml
