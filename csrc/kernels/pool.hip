// NHWC bf16 max-pool (k x k, stride s, padding p) forward + backward for the ResNet stem.
//
// PyTorch's channels_last max-pool backward scatters with int64 indices (the stem's index tensor
// alone is as large as the input). Here the forward stores the window position of the max as one
// byte per output element, and the backward is a GATHER: each input pixel visits the <= ceil(k/s)^2
// windows that cover it and sums the gradients whose argmax is that pixel — no atomics, bitwise
// deterministic, every access a 16-byte vector of 8 channels.
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kPB = 256;

// Grid: x covers the (w, channel-group) positions of one row, y strides over the N*H rows, so a
// thread needs one 32-bit division (w, g from its row offset) instead of three 64-bit div/mods
// (64-bit integer division is a long emulated sequence on CDNA and made the first version of the
// backward VALU-bound at 2.2 TB/s).
// Forward. KK = compile-time window size (3 for the stem; 0 = runtime k): with KK fixed the
// KK*KK 16-byte loads of a window are all in flight before the max (out-of-image taps load a
// clamped in-image address and are masked).
// AFF: the input is a pre-BatchNorm tensor; every tap is mapped through the BN affine
// (x * sc + bi, sc = gamma * invstd, bi = beta - mean * sc), the max taken, then the ReLU
// (max(relu(u)) = relu(max(u))), so the stem's BN+ReLU output never exists in memory. A window
// whose max is <= 0 gets argmax 255: its gradient is the ReLU's zero, and the backward gather
// routes it nowhere, i.e. the pool gradient comes out already masked by the ReLU.
template <int KK, bool AFF>
__global__ __launch_bounds__(kPB) void maxpool_fwd_kernel(const bf16* __restrict__ x,
                                                         bf16* __restrict__ y,
                                                         uint8_t* __restrict__ idx, int N, int H,
                                                         int W, int C, int OH, int OW, int k_rt,
                                                         int s, int p,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const bf16* __restrict__ gamma,
                                                         const bf16* __restrict__ beta) {
  const int k = KK > 0 ? KK : k_rt;
  const int cg = C / 8;
  const int i = blockIdx.x * kPB + threadIdx.x;
  if (i >= OW * cg) return;
  const int ow = i / cg;
  const int g = i - ow * cg;
  float sc[8], bi[8];
  if constexpr (AFF) {
    float ga[8], be[8];
    load_vec<bf16, 8>(gamma + 8 * g, ga);
    load_vec<bf16, 8>(beta + 8 * g, be);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      sc[v] = invstd[8 * g + v] * ga[v];
      bi[v] = be[v] - mean[8 * g + v] * sc[v];
    }
  }
  for (int row = blockIdx.y; row < N * OH; row += gridDim.y) {
    const int n = row / OH;
    const int oh = row - n * OH;
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      best[v] = -__builtin_inff();
      arg[v] = 0;
    }
    if constexpr (KK > 0) {
      float t[KK][KK][8];
      bool in[KK][KK];
#pragma unroll
      for (int a = 0; a < KK; ++a)
#pragma unroll
        for (int b = 0; b < KK; ++b) {
          const int h = oh * s - p + a, w = ow * s - p + b;
          in[a][b] = h >= 0 && h < H && w >= 0 && w < W;
          const int hh = in[a][b] ? h : 0, ww = in[a][b] ? w : 0;
          load_vec<bf16, 8>(x + ((static_cast<int64_t>(n) * H + hh) * W + ww) * C + 8 * g, t[a][b]);
          if constexpr (AFF) {
#pragma unroll
            for (int v = 0; v < 8; ++v) t[a][b][v] = fmaf(t[a][b][v], sc[v], bi[v]);
          }
        }
#pragma unroll
      for (int a = 0; a < KK; ++a)
#pragma unroll
        for (int b = 0; b < KK; ++b)
#pragma unroll
          for (int v = 0; v < 8; ++v) {
            const float val = t[a][b][v];
            const bool take = in[a][b] && (val > best[v] || (val != val));   // NaN propagates
            best[v] = take ? val : best[v];
            arg[v] = take ? static_cast<uint8_t>(a * KK + b) : arg[v];
          }
    } else {
      for (int a = 0; a < k; ++a) {
        const int h = oh * s - p + a;
        if (h < 0 || h >= H) continue;
        const bf16* xrow = x + (static_cast<int64_t>(n) * H + h) * W * C + 8 * g;
        for (int b = 0; b < k; ++b) {
          const int w = ow * s - p + b;
          if (w < 0 || w >= W) continue;
          float v8[8];
          load_vec<bf16, 8>(xrow + static_cast<int64_t>(w) * C, v8);
          if constexpr (AFF) {
#pragma unroll
            for (int v = 0; v < 8; ++v) v8[v] = fmaf(v8[v], sc[v], bi[v]);
          }
#pragma unroll
          for (int v = 0; v < 8; ++v) {
            const bool take = v8[v] > best[v] || (v8[v] != v8[v]);
            best[v] = take ? v8[v] : best[v];
            arg[v] = take ? static_cast<uint8_t>(a * k + b) : arg[v];
          }
        }
      }
    }
    if constexpr (AFF) {
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        arg[v] = best[v] > 0.f || best[v] != best[v] ? arg[v] : static_cast<uint8_t>(255);
        best[v] = best[v] > 0.f || best[v] != best[v] ? best[v] : 0.f;
      }
    }
    const int64_t o = (static_cast<int64_t>(row) * OW + ow) * C + 8 * g;
    store_bf16<8>(y + o, best);
    uint2 m;
    m.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (static_cast<uint32_t>(arg[3]) << 24);
    m.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (static_cast<uint32_t>(arg[7]) << 24);
    *reinterpret_cast<uint2*>(idx + o) = m;
  }
}

// Stem forward (k = 3, s = 2, p = 1, BN affine): one thread owns a 2 x 2 block of outputs x 8
// channels, whose windows cover a 5 x 5 block of input taps. The taps are loaded one input row at
// a time (5 x 16 B in flight), mapped through the affine once, and fed to every output window
// that contains them: 25 loads + 25 affine FMAs per 4 outputs instead of 36 + 36. Tie and NaN
// rules as maxpool_fwd_kernel (first max in window order, NaN propagates; max <= 0 -> argmax 255).
__global__ __launch_bounds__(kPB) void maxpool_fwd_k3s2_aff_kernel(
    const bf16* __restrict__ x, bf16* __restrict__ y, uint8_t* __restrict__ idx, int N, int H,
    int W, int C, int OH, int OW, const float* __restrict__ mean,
    const float* __restrict__ invstd, const bf16* __restrict__ gamma,
    const bf16* __restrict__ beta) {
  const int cg = C / 8;
  const int OWB = (OW + 1) / 2, OHB = (OH + 1) / 2;
  const int t = blockIdx.x * kPB + threadIdx.x;
  if (t >= OWB * cg) return;
  const int i = t / cg;
  const int g = t - i * cg;
  float sc[8], bi[8];
  {
    float ga[8], be[8];
    load_vec<bf16, 8>(gamma + 8 * g, ga);
    load_vec<bf16, 8>(beta + 8 * g, be);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      sc[v] = invstd[8 * g + v] * ga[v];
      bi[v] = be[v] - mean[8 * g + v] * sc[v];
    }
  }
  for (int band = blockIdx.y; band < N * OHB; band += gridDim.y) {
    const int n = band / OHB;
    const int j = band - n * OHB;
    float best[2][2][8];
    uint8_t arg[2][2][8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          best[a][b][v] = -__builtin_inff();
          arg[a][b][v] = 0;
        }
#pragma unroll
    for (int tr = 0; tr < 5; ++tr) {                  // input row 4j - 1 + tr
      const int h = 4 * j - 1 + tr;
      const bool hok = h >= 0 && h < H;
      float tap[5][8];
      bool wok[5];
#pragma unroll
      for (int u = 0; u < 5; ++u) {
        const int w = 4 * i - 1 + u;
        wok[u] = hok && w >= 0 && w < W;
        const int hh = wok[u] ? h : 0, ww = wok[u] ? w : 0;
        load_vec<bf16, 8>(x + ((static_cast<int64_t>(n) * H + hh) * W + ww) * C + 8 * g, tap[u]);
      }
#pragma unroll
      for (int u = 0; u < 5; ++u)
#pragma unroll
        for (int v = 0; v < 8; ++v) tap[u][v] = fmaf(tap[u][v], sc[v], bi[v]);
      // output (a, b) window row = tr - 2a, column = u - 2b, both in 0..2; taps in window order
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int wr = tr - 2 * a;
        if (wr < 0 || wr > 2) continue;               // compile-time after unrolling
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int wc = 0; wc < 3; ++wc) {
            const int u = wc + 2 * b;
#pragma unroll
            for (int v = 0; v < 8; ++v) {
              const float val = tap[u][v];
              const bool take = wok[u] && (val > best[a][b][v] || (val != val));
              best[a][b][v] = take ? val : best[a][b][v];
              arg[a][b][v] = take ? static_cast<uint8_t>(wr * 3 + wc) : arg[a][b][v];
            }
          }
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = 2 * j + a, ow = 2 * i + b;
        if (oh >= OH || ow >= OW) continue;
        float o[8];
        uint8_t m[8];
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          const float bv = best[a][b][v];
          const bool pos = bv > 0.f || bv != bv;
          o[v] = pos ? bv : 0.f;
          m[v] = pos ? arg[a][b][v] : static_cast<uint8_t>(255);
        }
        const int64_t off = ((static_cast<int64_t>(n) * OH + oh) * OW + ow) * C + 8 * g;
        store_bf16<8>(y + off, o);
        uint2 mm;
        mm.x = m[0] | (m[1] << 8) | (m[2] << 16) | (static_cast<uint32_t>(m[3]) << 24);
        mm.y = m[4] | (m[5] << 8) | (m[6] << 16) | (static_cast<uint32_t>(m[7]) << 24);
        *reinterpret_cast<uint2*>(idx + off) = mm;
      }
  }
}

// Backward. KS = ceil(k / s) candidate windows per dimension (2 for the 3x3/s2 stem): with KS a
// compile-time constant all KS*KS (idx, dy) loads of a pixel are issued before any is consumed
// (invalid windows load a clamped valid address and contribute zero), instead of a
// load-wait-accumulate loop per window.
template <int KS>
__global__ __launch_bounds__(kPB) void maxpool_bwd_kernel(const bf16* __restrict__ dy,
                                                         const uint8_t* __restrict__ idx,
                                                         bf16* __restrict__ dx, int N, int H, int W,
                                                         int C, int OH, int OW, int k, int s,
                                                         int p) {
  const int cg = C / 8;
  const int i0 = blockIdx.x * kPB + threadIdx.x;
  if (i0 >= W * cg) return;
  const int w = i0 / cg;
  const int g = i0 - w * cg;
  // windows ow with ow*s - p <= w <= ow*s - p + k - 1, i.e. ow in [ow0, ow1], ow1 - ow0 < KS
  const int ow1 = min(OW - 1, (w + p) / s);
  for (int row = blockIdx.y; row < N * H; row += gridDim.y) {
    const int n = row / H;
    const int h = row - n * H;
    const int oh1 = min(OH - 1, (h + p) / s);
    uint2 m[KS][KS];
    float d[KS][KS][8];
    bool ok[KS][KS];
#pragma unroll
    for (int a = 0; a < KS; ++a) {
      const int oh = oh1 - a;
      const int ia = h - (oh * s - p);
      const bool oka = oh >= 0 && ia >= 0 && ia < k;
#pragma unroll
      for (int b = 0; b < KS; ++b) {
        const int ow = ow1 - b;
        const int ib = w - (ow * s - p);
        ok[a][b] = oka && ow >= 0 && ib >= 0 && ib < k;
        const int64_t o = ((static_cast<int64_t>(n) * OH + (ok[a][b] ? oh : 0)) * OW +
                           (ok[a][b] ? ow : 0)) * C + 8 * g;
        m[a][b] = *reinterpret_cast<const uint2*>(idx + o);
        load_vec<bf16, 8>(dy + o, d[a][b]);
      }
    }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < KS; ++a)
#pragma unroll
      for (int b = 0; b < KS; ++b) {
        const int ia = h - ((oh1 - a) * s - p), ib = w - ((ow1 - b) * s - p);
        const uint32_t me = ok[a][b] ? static_cast<uint32_t>(ia * k + ib) : 0xffffffffu;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          acc[v] += (((m[a][b].x >> (8 * v)) & 0xff) == me) ? d[a][b][v] : 0.f;
          acc[v + 4] += (((m[a][b].y >> (8 * v)) & 0xff) == me) ? d[a][b][v + 4] : 0.f;
        }
      }
    store_bf16<8>(dx + (static_cast<int64_t>(row) * W + w) * C + 8 * g, acc);
  }
}

// Backward specialised for the ResNet stem (k = 3, s = 2, p = 1): one thread owns a 2x2 block of
// input pixels (h = 2j + dh, w = 2i + dw) x 8 channels. Exactly the 4 windows (oh, ow) in
// {j, j+1} x {i, i+1} can cover that block, so each window's (argmax, dy) is read once per 4
// pixels instead of once per pixel: the generic gather above moves ~6 bytes through L2 per byte of
// dx it writes, this one ~1.5.
// part (optional): per-workgroup channel sums of dx, [gridDim.y * gridDim.x][C] (the stem's
// BatchNorm dbeta, so its backward needs no separate reduction pass).
// dy2 (optional): a second gradient of the pool output, summed on load (ResNet layer1.0's
// downsample conv reads the pool output too; its data gradient arrives here instead of through
// an elementwise add pass).
__global__ __launch_bounds__(kPB) void maxpool_bwd_k3s2_kernel(const bf16* __restrict__ dy,
                                                              const bf16* __restrict__ dy2,
                                                              const uint8_t* __restrict__ idx,
                                                              bf16* __restrict__ dx, int N, int H,
                                                              int W, int C, int OH, int OW,
                                                              float* __restrict__ part) {
  const int cg = C / 8;
  const int HB = (H + 1) / 2, WB = (W + 1) / 2;
  const int t = blockIdx.x * kPB + threadIdx.x;
  const bool active = t < WB * cg;
  const int i = active ? t / cg : 0;
  const int g = t - (t / cg) * cg;
  float tsum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int band = active ? blockIdx.y : N * HB; band < N * HB; band += gridDim.y) {
    const int n = band / HB;
    const int j = band - n * HB;
    uint2 m[2][2];
    float d[2][2][8];
    bool ok[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = j + a, ow = i + b;
        ok[a][b] = oh < OH && ow < OW;
        const int64_t o = ((static_cast<int64_t>(n) * OH + (ok[a][b] ? oh : 0)) * OW +
                           (ok[a][b] ? ow : 0)) * C + 8 * g;
        m[a][b] = *reinterpret_cast<const uint2*>(idx + o);
        load_vec<bf16, 8>(dy + o, d[a][b]);
        if (dy2) {
          float e[8];
          load_vec<bf16, 8>(dy2 + o, e);
#pragma unroll
          for (int v = 0; v < 8; ++v) d[a][b][v] += e[v];
        }
      }
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const int h = 2 * j + dh;
      if (h >= H) break;
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int w = 2 * i + dw;
        if (w >= W) break;
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            // tap of (h, w) inside window (j + a, i + b): row h - (2(j+a) - 1), col likewise
            const int ta = dh + 1 - 2 * a, tb = dw + 1 - 2 * b;
            if (ta < 0 || tb < 0) continue;          // compile-time after unrolling
            const uint32_t me = ok[a][b] ? static_cast<uint32_t>(ta * 3 + tb) : 0xffffffffu;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              acc[v] += (((m[a][b].x >> (8 * v)) & 0xff) == me) ? d[a][b][v] : 0.f;
              acc[v + 4] += (((m[a][b].y >> (8 * v)) & 0xff) == me) ? d[a][b][v + 4] : 0.f;
            }
          }
        store_bf16<8>(dx + ((static_cast<int64_t>(n) * H + h) * W + w) * C + 8 * g, acc);
        if (part) {
#pragma unroll
          for (int v = 0; v < 8; ++v) tsum[v] += acc[v];
        }
      }
    }
  }
  if (part == nullptr) return;
  // fixed-order workgroup reduction: channel group g's threads are t = g, g + cg, ...
  __shared__ float red[kPB][9];
#pragma unroll
  for (int v = 0; v < 8; ++v) red[threadIdx.x][v] = tsum[v];
  __syncthreads();
  float* pb = part + (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * C;
  for (int c = threadIdx.x; c < C; c += kPB) {
    const int gc = c >> 3, v = c & 7;
    // thread-index offset of this block's first thread with channel group gc
    const int first = (gc - (blockIdx.x * kPB) % cg + cg) % cg;
    float acc = 0.f;
    for (int k = first; k < kPB; k += cg) acc += red[k][v];
    pb[c] = acc;
  }
}

// first fold level: workgroup b sums rows [b nb / G, (b + 1) nb / G) of [nb][C] into out[b][C]
// (kPB / C slices per channel, fixed order)
__global__ __launch_bounds__(kPB) void colsum_fold_rows_kernel(const float* __restrict__ part,
                                                               int nb, int C,
                                                               float* __restrict__ out) {
  __shared__ float ls[kPB];
  const int G = gridDim.x;
  const int lo = static_cast<int>(static_cast<int64_t>(blockIdx.x) * nb / G);
  const int hi = static_cast<int>(static_cast<int64_t>(blockIdx.x + 1) * nb / G);
  const int nsl = kPB / C;
  const int c = threadIdx.x % C, sl = threadIdx.x / C;
  float acc = 0.f;
  if (sl < nsl) {
    int b = lo + sl;
    for (; b + 3 * nsl < hi; b += 4 * nsl) {
      const float v0 = part[static_cast<int64_t>(b) * C + c];
      const float v1 = part[static_cast<int64_t>(b + nsl) * C + c];
      const float v2 = part[static_cast<int64_t>(b + 2 * nsl) * C + c];
      const float v3 = part[static_cast<int64_t>(b + 3 * nsl) * C + c];
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; b < hi; b += nsl) acc += part[static_cast<int64_t>(b) * C + c];
  }
  ls[threadIdx.x] = acc;
  __syncthreads();
  for (int cc = threadIdx.x; cc < C; cc += kPB) {
    float s = 0.f;
    for (int k = 0; k < nsl; ++k) s += ls[k * C + cc];
    out[static_cast<int64_t>(blockIdx.x) * C + cc] = s;
  }
}

// out[c] = sum over nb partial rows [nb][C] (fp64, 1024 threads = slices x channels, fixed order)
__global__ __launch_bounds__(1024) void colsum_fold_kernel(const float* __restrict__ part, int nb,
                                                           int C, float* __restrict__ out) {
  __shared__ double ls[1024];
  const int nsl = 1024 / C;
  const int c = threadIdx.x % C, sl = threadIdx.x / C;
  double acc = 0.0;
  if (sl < nsl)
    for (int b = sl; b < nb; b += nsl) acc += part[static_cast<int64_t>(b) * C + c];
  ls[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < C) {
    double s = 0.0;
    for (int k = 0; k < nsl; ++k) s += ls[k * C + threadIdx.x];
    out[threadIdx.x] = static_cast<float>(s);
  }
}

// Routed channel sums of a max-pool output gradient (the stem backward's dbeta and mean(g) when
// stem_wgrad gathers the pool's input gradient itself): a window whose argmax byte is 255 (max <= 0,
// ReLU-masked) routes nothing, every other window routes its gradient to exactly one input pixel.
// Thread = 8 channels of one pooled pixel row per iteration (4 rows in flight), per-workgroup
// partials [nb][C] in a fixed order. DY2: dsum = bf16(dy + dy2) for the gather.
template <bool DY2>
__global__ __launch_bounds__(kPB) void pool_gsum_kernel(const bf16* __restrict__ dy,
                                                       const bf16* __restrict__ dy2,
                                                       const uint8_t* __restrict__ idx,
                                                       bf16* __restrict__ dsum, int64_t P, int C,
                                                       int64_t ppb, float* __restrict__ part) {
  const int cg = C / 8, rpi = kPB / cg;
  const int g = threadIdx.x % cg;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * ppb;
  const int64_t hi = lo + ppb < P ? lo + ppb : P;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r0 = lo + threadIdx.x / cg; r0 < hi; r0 += 4 * rpi) {
    float d[4][8];
    uint2 m[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // clamped unconditional loads, zeroed past the range
      const int64_t r = r0 + u * rpi < hi ? r0 + u * rpi : hi - 1;
      load_vec<bf16, 8>(dy + r * C + 8 * g, d[u]);
      m[u] = *reinterpret_cast<const uint2*>(idx + r * C + 8 * g);
      if constexpr (DY2) {
        float e[8];
        load_vec<bf16, 8>(dy2 + r * C + 8 * g, e);
#pragma unroll
        for (int v = 0; v < 8; ++v) d[u][v] += e[v];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t r = r0 + u * rpi;
      if (r >= hi) break;
      if constexpr (DY2) store_bf16<8>(dsum + r * C + 8 * g, d[u]);
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const uint32_t b = ((v < 4 ? m[u].x : m[u].y) >> (8 * (v & 3))) & 0xffu;
        s[v] += b != 0xffu ? d[u][v] : 0.f;
      }
    }
  }
  __shared__ float red[kPB][9];
#pragma unroll
  for (int v = 0; v < 8; ++v) red[threadIdx.x][v] = s[v];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kPB) {
    const int gc = c >> 3, v = c & 7;
    float acc = 0.f;
    for (int k = gc; k < kPB; k += cg) acc += red[k][v];
    part[static_cast<int64_t>(blockIdx.x) * C + c] = acc;
  }
}

dim3 pgrid(int inner, int rows) {
  return dim3((inner + kPB - 1) / kPB, rows < 65535 ? rows : 65535);
}


// Channel zero-padding of NHWC bf16 images, C -> 4 (the ResNet stem: MIOpen's vectorised NHWC
// 7x7 kernels need Cin % 4 == 0; Cin = 3 falls back to a scalar path that is 1.4x slower for the
// forward and weight gradient, bench/stem_pad.py). One lane per pixel: C loads, one 8-B store.
__global__ __launch_bounds__(256) void pad_c4_kernel(const uint16_t* __restrict__ x,
                                                    uint2* __restrict__ y, int64_t npix, int C) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; p < npix; p += stride) {
    uint16_t v[4] = {0, 0, 0, 0};
    for (int c = 0; c < C; ++c) v[c] = x[p * C + c];
    y[p] = make_uint2(v[0] | (uint32_t(v[1]) << 16), v[2] | (uint32_t(v[3]) << 16));
  }
}

// Stride-2 pixel subsampling of NHWC bf16 (what a 1x1 stride-2 conv reads), and its backward: a
// full-resolution gradient with g at the even pixels and zeros elsewhere, written in one pass.
// 16-B vectors; C % 8 == 0.
__global__ __launch_bounds__(256) void subsample2_kernel(const uint4* __restrict__ x,
                                                         uint4* __restrict__ y, int64_t total,
                                                         int C8, int OH, int OW, int H, int W) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= total) return;
  const int64_t pix = e / C8;
  const int c = static_cast<int>(e - pix * C8);
  const int64_t n = pix / (static_cast<int64_t>(OH) * OW);
  const int rem = static_cast<int>(pix - n * OH * OW);
  const int oh = rem / OW, ow = rem - oh * OW;
  y[e] = x[((n * H + 2 * oh) * W + 2 * ow) * C8 + c];
}

__global__ __launch_bounds__(256) void upsample2_scatter_kernel(const uint4* __restrict__ g,
                                                                uint4* __restrict__ dx,
                                                                int64_t total, int C8, int OH,
                                                                int OW, int H, int W) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= total) return;
  const int64_t pix = e / C8;
  const int c = static_cast<int>(e - pix * C8);
  const int64_t n = pix / (static_cast<int64_t>(H) * W);
  const int rem = static_cast<int>(pix - n * H * W);
  const int h = rem / W, w = rem - h * W;
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (!(h & 1) && !(w & 1)) v = g[((n * OH + (h >> 1)) * OW + (w >> 1)) * C8 + c];
  dx[e] = v;
}

// Global-average-pool backward into NHWC: dx[n][p][c] = bf16(float(g[n][c]) / HW) for every pixel
// p (one write-only pass; 8 channels per thread, the same fp32 division as g.float() / HW).
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const uint4* __restrict__ g,
                                                          uint4* __restrict__ dx, int64_t total,
                                                          int C8, int HW, float hw) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= total) return;
  const int64_t pix = e / C8;
  const int c = static_cast<int>(e - pix * C8);
  const int64_t n = pix / HW;
  const uint4 u = g[n * C8 + c];
  const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    o[q] = pk_bf16(__uint_as_float(w4[q] << 16) / hw, __uint_as_float(w4[q] & 0xffff0000u) / hw);
  dx[e] = make_uint4(o[0], o[1], o[2], o[3]);
}

}  // namespace

hipError_t launch_avgpool_bwd(const void* g, void* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8 || N < 1 || HW < 1) return hipErrorInvalidValue;
  const int C8 = C / 8;
  const int64_t total = static_cast<int64_t>(N) * HW * C8;
  avgpool_bwd_kernel<<<static_cast<unsigned>((total + 255) / 256), 256, 0, st>>>(
      reinterpret_cast<const uint4*>(g), reinterpret_cast<uint4*>(dx), total, C8, HW,
      static_cast<float>(HW));
  return hipGetLastError();
}

// CML_POOL_BLOCKS=0 selects the one-output-per-thread forward for the stem (A/B)
static bool k3s2_blocks() {
  static const bool on = [] {
    const char* e = getenv("CML_POOL_BLOCKS");
    return !(e && e[0] == '0');
  }();
  return on;
}

hipError_t launch_subsample2(const void* x, void* y, int N, int H, int W, int C, hipStream_t st) {
  if (C % 8 || N < 1 || H < 1 || W < 1) return hipErrorInvalidValue;
  const int OH = (H + 1) / 2, OW = (W + 1) / 2, C8 = C / 8;
  const int64_t total = static_cast<int64_t>(N) * OH * OW * C8;
  subsample2_kernel<<<static_cast<unsigned>((total + 255) / 256), 256, 0, st>>>(
      reinterpret_cast<const uint4*>(x), reinterpret_cast<uint4*>(y), total, C8, OH, OW, H, W);
  return hipGetLastError();
}

hipError_t launch_upsample2_scatter(const void* g, void* dx, int N, int H, int W, int C,
                                    hipStream_t st) {
  if (C % 8 || N < 1 || H < 1 || W < 1) return hipErrorInvalidValue;
  const int OH = (H + 1) / 2, OW = (W + 1) / 2, C8 = C / 8;
  const int64_t total = static_cast<int64_t>(N) * H * W * C8;
  upsample2_scatter_kernel<<<static_cast<unsigned>((total + 255) / 256), 256, 0, st>>>(
      reinterpret_cast<const uint4*>(g), reinterpret_cast<uint4*>(dx), total, C8, OH, OW, H, W);
  return hipGetLastError();
}

hipError_t launch_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C,
                              int OH, int OW, int k, int s, int p, hipStream_t st) {
  return launch_bn_relu_maxpool_fwd(x, nullptr, nullptr, nullptr, nullptr, y, idx, N, H, W, C, OH,
                                    OW, k, s, p, st);
}

hipError_t launch_bn_relu_maxpool_fwd(const void* x, const float* mean, const float* invstd,
                                      const void* gamma, const void* beta, void* y, void* idx,
                                      int N, int H, int W, int C, int OH, int OW, int k, int s,
                                      int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return hipErrorInvalidValue;
  if (N * OH < 1) return hipErrorInvalidValue;
  const dim3 grid = pgrid(OW * (C / 8), N * OH);
  const bf16* xp = reinterpret_cast<const bf16*>(x);
  bf16* yp = reinterpret_cast<bf16*>(y);
  uint8_t* ip = reinterpret_cast<uint8_t*>(idx);
  const bf16* gp = reinterpret_cast<const bf16*>(gamma);
  const bf16* bp = reinterpret_cast<const bf16*>(beta);
  const bool aff = mean != nullptr;
#define CML_MP(KK, A) maxpool_fwd_kernel<KK, A><<<grid, kPB, 0, st>>>(xp, yp, ip, N, H, W, C, OH, OW, k, s, p, mean, invstd, gp, bp)
  if (k == 3 && s == 2 && p == 1 && aff && k3s2_blocks()) {
    maxpool_fwd_k3s2_aff_kernel<<<pgrid(((OW + 1) / 2) * (C / 8), N * ((OH + 1) / 2)), kPB, 0, st>>>(
        xp, yp, ip, N, H, W, C, OH, OW, mean, invstd, gp, bp);
  } else if (k == 3 && aff) CML_MP(3, true);
  else if (k == 3) CML_MP(3, false);
  else if (aff) CML_MP(0, true);
  else CML_MP(0, false);
#undef CML_MP
  return hipGetLastError();
}

hipError_t launch_maxpool_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W,
                              int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return hipErrorInvalidValue;
  if (N * H < 1) return hipErrorInvalidValue;
  if (k == 3 && s == 2 && p == 1) {
    maxpool_bwd_k3s2_kernel<<<pgrid(((W + 1) / 2) * (C / 8), N * ((H + 1) / 2)), kPB, 0, st>>>(
        reinterpret_cast<const bf16*>(dy), nullptr, reinterpret_cast<const uint8_t*>(idx),
        reinterpret_cast<bf16*>(dx), N, H, W, C, OH, OW, nullptr);
    return hipGetLastError();
  }
  const int ks = (k + s - 1) / s;
  const dim3 grid = pgrid(W * (C / 8), N * H);
  const bf16* dyp = reinterpret_cast<const bf16*>(dy);
  const uint8_t* ip = reinterpret_cast<const uint8_t*>(idx);
  bf16* dxp = reinterpret_cast<bf16*>(dx);
  switch (ks) {
    case 1: maxpool_bwd_kernel<1><<<grid, kPB, 0, st>>>(dyp, ip, dxp, N, H, W, C, OH, OW, k, s, p); break;
    case 2: maxpool_bwd_kernel<2><<<grid, kPB, 0, st>>>(dyp, ip, dxp, N, H, W, C, OH, OW, k, s, p); break;
    case 3: maxpool_bwd_kernel<3><<<grid, kPB, 0, st>>>(dyp, ip, dxp, N, H, W, C, OH, OW, k, s, p); break;
    default: return hipErrorInvalidValue;   // caller falls back to PyTorch
  }
  return hipGetLastError();
}

hipError_t launch_pad_c4(const void* x, void* y, int64_t npix, int C, hipStream_t st) {
  if (C < 1 || C > 4 || npix < 1 || (reinterpret_cast<uintptr_t>(y) & 7)) return hipErrorInvalidValue;
  int64_t b = (npix + 255) / 256;
  if (b > 16384) b = 16384;
  pad_c4_kernel<<<static_cast<unsigned>(b), 256, 0, st>>>(reinterpret_cast<const uint16_t*>(x),
                                                          reinterpret_cast<uint2*>(y), npix, C);
  return hipGetLastError();
}

// grid.y of the summing backward: one band per workgroup row like the plain kernel (a capped grid
// that loops over bands is latency-bound: +35 % time), the partial rows folded in two levels
constexpr int kSumRows = 65535;
constexpr int kFold1 = 256;

size_t maxpool_bwd_sum_workspace_bytes(int N, int H, int W, int C) {
  const int gx = ((((W + 1) / 2) * (C / 8)) + kPB - 1) / kPB;
  const int rows = N * ((H + 1) / 2);
  const int gy = rows < kSumRows ? rows : kSumRows;
  return (static_cast<size_t>(gx) * gy + kFold1) * C * sizeof(float);
}

hipError_t launch_maxpool_bwd_sum(const void* dy, const void* dy2, const void* idx, void* dx,
                                  float* sums, void* work, int N, int H, int W, int C, int OH,
                                  int OW, hipStream_t st) {
  if (C % 8 || C > kPB || kPB % C || N * H < 1) return hipErrorInvalidValue;
  const int gx = ((((W + 1) / 2) * (C / 8)) + kPB - 1) / kPB;
  const int rows = N * ((H + 1) / 2);
  const int gy = rows < kSumRows ? rows : kSumRows;
  float* part = reinterpret_cast<float*>(work);
  maxpool_bwd_k3s2_kernel<<<dim3(gx, gy), kPB, 0, st>>>(
      reinterpret_cast<const bf16*>(dy), reinterpret_cast<const bf16*>(dy2),
      reinterpret_cast<const uint8_t*>(idx),
      reinterpret_cast<bf16*>(dx), N, H, W, C, OH, OW, part);
  float* part2 = part + static_cast<int64_t>(gx) * gy * C;
  colsum_fold_rows_kernel<<<kFold1, kPB, 0, st>>>(part, gx * gy, C, part2);
  colsum_fold_kernel<<<1, 1024, 0, st>>>(part2, kFold1, C, sums);
  return hipGetLastError();
}

constexpr int kGsumBlocks = 1024;

size_t pool_gsum_workspace_floats(int64_t, int C) { return static_cast<size_t>(kGsumBlocks) * C; }

hipError_t launch_pool_gsum(const void* dy, const void* dy2, const void* idx, void* dsum,
                            float* sums, float* work, int64_t P, int C, hipStream_t st) {
  if (C % 8 || C > kPB || kPB % C || P < 1 || (dy2 && !dsum)) return hipErrorInvalidValue;
  const int rpi = kPB / (C / 8);
  int64_t nb = (P + 16 * rpi - 1) / (16 * rpi);   // >= 16 row iterations per workgroup
  if (nb > kGsumBlocks) nb = kGsumBlocks;
  const int64_t ppb = ((P + nb - 1) / nb + rpi - 1) / rpi * rpi;
  nb = (P + ppb - 1) / ppb;
  const auto* d = reinterpret_cast<const bf16*>(dy);
  const auto* d2 = reinterpret_cast<const bf16*>(dy2);
  const auto* ix = reinterpret_cast<const uint8_t*>(idx);
  auto* ds = reinterpret_cast<bf16*>(dsum);
  if (dy2) pool_gsum_kernel<true><<<static_cast<unsigned>(nb), kPB, 0, st>>>(d, d2, ix, ds, P, C, ppb, work);
  else pool_gsum_kernel<false><<<static_cast<unsigned>(nb), kPB, 0, st>>>(d, d2, ix, ds, P, C, ppb, work);
  colsum_fold_kernel<<<1, 1024, 0, st>>>(work, static_cast<int>(nb), C, sums);
  return hipGetLastError();
}

}  // namespace cml
