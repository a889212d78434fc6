// NHWC bf16 max-pool (k x k, stride s, padding p) forward + backward for the ResNet stem.
//
// PyTorch's channels_last max-pool backward scatters with int64 indices (the stem's index tensor
// alone is as large as the input). Here the forward stores the window position of the max as one
// byte per output element, and the backward is a GATHER: each input pixel visits the <= ceil(k/s)^2
// windows that cover it and sums the gradients whose argmax is that pixel — no atomics, bitwise
// deterministic, every access a 16-byte vector of 8 channels.
#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kPB = 256;

// Grid: x covers the (w, channel-group) positions of one row, y strides over the N*H rows, so a
// thread needs one 32-bit division (w, g from its row offset) instead of three 64-bit div/mods
// (64-bit integer division is a long emulated sequence on CDNA and made the first version of the
// backward VALU-bound at 2.2 TB/s).
__global__ __launch_bounds__(kPB) void maxpool_fwd_kernel(const bf16* __restrict__ x,
                                                         bf16* __restrict__ y,
                                                         uint8_t* __restrict__ idx, int N, int H,
                                                         int W, int C, int OH, int OW, int k, int s,
                                                         int p) {
  const int cg = C / 8;
  const int i = blockIdx.x * kPB + threadIdx.x;
  if (i >= OW * cg) return;
  const int ow = i / cg;
  const int g = i - ow * cg;
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
    for (int a = 0; a < k; ++a) {
      const int h = oh * s - p + a;
      if (h < 0 || h >= H) continue;
      const bf16* xrow = x + (static_cast<int64_t>(n) * H + h) * W * C + 8 * g;
      for (int b = 0; b < k; ++b) {
        const int w = ow * s - p + b;
        if (w < 0 || w >= W) continue;
        float v8[8];
        load_vec<bf16, 8>(xrow + static_cast<int64_t>(w) * C, v8);
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          const bool take = v8[v] > best[v] || (v8[v] != v8[v]);   // NaN propagates
          best[v] = take ? v8[v] : best[v];
          arg[v] = take ? static_cast<uint8_t>(a * k + b) : arg[v];
        }
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
  // windows ow with ow*s - p <= w <= ow*s - p + k - 1
  const int ow0 = max(0, (w + p - k + s) / s), ow1 = min(OW - 1, (w + p) / s);
  for (int row = blockIdx.y; row < N * H; row += gridDim.y) {
    const int n = row / H;
    const int h = row - n * H;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int oh0 = max(0, (h + p - k + s) / s), oh1 = min(OH - 1, (h + p) / s);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int a = h - (oh * s - p);
      if (a < 0 || a >= k) continue;
      const int64_t orow = (static_cast<int64_t>(n) * OH + oh) * OW;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int b = w - (ow * s - p);
        if (b < 0 || b >= k) continue;
        const uint32_t me = static_cast<uint32_t>(a * k + b);
        const int64_t o = (orow + ow) * C + 8 * g;
        const uint2 m = *reinterpret_cast<const uint2*>(idx + o);
        float d8[8];
        load_vec<bf16, 8>(dy + o, d8);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          acc[v] += (((m.x >> (8 * v)) & 0xff) == me) ? d8[v] : 0.f;
          acc[v + 4] += (((m.y >> (8 * v)) & 0xff) == me) ? d8[v + 4] : 0.f;
        }
      }
    }
    store_bf16<8>(dx + (static_cast<int64_t>(row) * W + w) * C + 8 * g, acc);
  }
}

dim3 pgrid(int inner, int rows) {
  return dim3((inner + kPB - 1) / kPB, rows < 65535 ? rows : 65535);
}

}  // namespace

hipError_t launch_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C,
                              int OH, int OW, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return hipErrorInvalidValue;
  if (N * OH < 1) return hipErrorInvalidValue;
  maxpool_fwd_kernel<<<pgrid(OW * (C / 8), N * OH), kPB, 0, st>>>(
      reinterpret_cast<const bf16*>(x), reinterpret_cast<bf16*>(y),
      reinterpret_cast<uint8_t*>(idx), N, H, W, C, OH, OW, k, s, p);
  return hipGetLastError();
}

hipError_t launch_maxpool_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W,
                              int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return hipErrorInvalidValue;
  if (N * H < 1) return hipErrorInvalidValue;
  maxpool_bwd_kernel<<<pgrid(W * (C / 8), N * H), kPB, 0, st>>>(
      reinterpret_cast<const bf16*>(dy), reinterpret_cast<const uint8_t*>(idx),
      reinterpret_cast<bf16*>(dx), N, H, W, C, OH, OW, k, s, p);
  return hipGetLastError();
}

}  // namespace cml
