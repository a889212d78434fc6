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

__global__ __launch_bounds__(kPB) void maxpool_fwd_kernel(const bf16* __restrict__ x,
                                                         bf16* __restrict__ y,
                                                         uint8_t* __restrict__ idx, int N, int H,
                                                         int W, int C, int OH, int OW, int k, int s,
                                                         int p) {
  const int cg = C / 8;
  const int64_t total = static_cast<int64_t>(N) * OH * OW * cg;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kPB + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kPB) {
    const int g = static_cast<int>(t % cg);
    int64_t r = t / cg;
    const int ow = static_cast<int>(r % OW);
    r /= OW;
    const int oh = static_cast<int>(r % OH);
    const int n = static_cast<int>(r / OH);
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      best[v] = -__builtin_inff();
      arg[v] = 0;
    }
    for (int i = 0; i < k; ++i) {
      const int h = oh * s - p + i;
      if (h < 0 || h >= H) continue;
      for (int j = 0; j < k; ++j) {
        const int w = ow * s - p + j;
        if (w < 0 || w >= W) continue;
        float v8[8];
        load_vec<bf16, 8>(x + ((static_cast<int64_t>(n) * H + h) * W + w) * C + 8 * g, v8);
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          const bool take = v8[v] > best[v] || (v8[v] != v8[v]);   // NaN propagates
          best[v] = take ? v8[v] : best[v];
          arg[v] = take ? static_cast<uint8_t>(i * k + j) : arg[v];
        }
      }
    }
    const int64_t o = ((static_cast<int64_t>(n) * OH + oh) * OW + ow) * C + 8 * g;
    store_bf16<8>(y + o, best);
    uint2 a;
    a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (static_cast<uint32_t>(arg[3]) << 24);
    a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (static_cast<uint32_t>(arg[7]) << 24);
    *reinterpret_cast<uint2*>(idx + o) = a;
  }
}

__global__ __launch_bounds__(kPB) void maxpool_bwd_kernel(const bf16* __restrict__ dy,
                                                         const uint8_t* __restrict__ idx,
                                                         bf16* __restrict__ dx, int N, int H, int W,
                                                         int C, int OH, int OW, int k, int s,
                                                         int p) {
  const int cg = C / 8;
  const int64_t total = static_cast<int64_t>(N) * H * W * cg;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kPB + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kPB) {
    const int g = static_cast<int>(t % cg);
    int64_t r = t / cg;
    const int w = static_cast<int>(r % W);
    r /= W;
    const int h = static_cast<int>(r % H);
    const int n = static_cast<int>(r / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // windows oh with oh*s - p <= h <= oh*s - p + k - 1
    const int oh0 = max(0, (h + p - k + s) / s), oh1 = min(OH - 1, (h + p) / s);
    const int ow0 = max(0, (w + p - k + s) / s), ow1 = min(OW - 1, (w + p) / s);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int i = h - (oh * s - p);
      if (i < 0 || i >= k) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int j = w - (ow * s - p);
        if (j < 0 || j >= k) continue;
        const uint8_t me = static_cast<uint8_t>(i * k + j);
        const int64_t o = ((static_cast<int64_t>(n) * OH + oh) * OW + ow) * C + 8 * g;
        const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
        float d8[8];
        load_vec<bf16, 8>(dy + o, d8);
        const uint32_t lo = a.x, hi = a.y;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          acc[v] += (((lo >> (8 * v)) & 0xff) == me) ? d8[v] : 0.f;
          acc[v + 4] += (((hi >> (8 * v)) & 0xff) == me) ? d8[v + 4] : 0.f;
        }
      }
    }
    store_bf16<8>(dx + ((static_cast<int64_t>(n) * H + h) * W + w) * C + 8 * g, acc);
  }
}

int pgrid(int64_t work) {
  int64_t b = (work + kPB - 1) / kPB;
  if (b > 4096) b = 4096;
  return static_cast<int>(b < 1 ? 1 : b);
}

}  // namespace

hipError_t launch_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C,
                              int OH, int OW, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return hipErrorInvalidValue;
  maxpool_fwd_kernel<<<pgrid(static_cast<int64_t>(N) * OH * OW * (C / 8)), kPB, 0, st>>>(
      reinterpret_cast<const bf16*>(x), reinterpret_cast<bf16*>(y),
      reinterpret_cast<uint8_t*>(idx), N, H, W, C, OH, OW, k, s, p);
  return hipGetLastError();
}

hipError_t launch_maxpool_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W,
                              int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return hipErrorInvalidValue;
  maxpool_bwd_kernel<<<pgrid(static_cast<int64_t>(N) * H * W * (C / 8)), kPB, 0, st>>>(
      reinterpret_cast<const bf16*>(dy), reinterpret_cast<const uint8_t*>(idx),
      reinterpret_cast<bf16*>(dx), N, H, W, C, OH, OW, k, s, p);
  return hipGetLastError();
}

}  // namespace cml
