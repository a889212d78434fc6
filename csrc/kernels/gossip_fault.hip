// Decentralized gossip mixing (N09) and Byzantine fault injection (N10).
//
// Gossip: after the local step each rank holds its own fp32 master x and has received its ring
// neighbours' bf16 parameters (RCCL send/recv, both directions at once). The mix
//   x <- (w0 + w1 + w2) x + w1 * c_l (left - x) + w2 * c_r (right - x)
// with c = min(1, clip / ||neighbour - x||) (robust gossip: a Byzantine neighbour moves us by at
// most `clip`) is one streaming pass; the two distances need one reduction pass first. Partial
// sums go to a per-workgroup slab and the mix kernel's workgroups each fold the slab (<= 2048
// values, L2-resident) in a fixed order, so the result is deterministic and needs no extra
// launch or host sync.
#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kBlk = 256;
constexpr int kMaxBlk = 1024;

template <typename T>
__device__ __forceinline__ float ld1(const T* p, int64_t e) {
  if constexpr (sizeof(T) == 2) return bf2f(reinterpret_cast<const uint16_t*>(p)[e]);
  else return p[e];
}

template <typename T>
__global__ __launch_bounds__(kBlk) void pair_sqdist_kernel(const float* __restrict__ x,
                                                          const T* __restrict__ l,
                                                          const T* __restrict__ r, int64_t D,
                                                          float* __restrict__ part) {
  float sl = 0.f, sr = 0.f;
  const int64_t nv = D / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlk;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kBlk + threadIdx.x; t < nv; t += stride) {
    float xv[8], lv[8], rv[8];
    load_vec<float, 8>(x + t * 8, xv);
    load_vec<T, 8>(l + t * 8, lv);
    load_vec<T, 8>(r + t * 8, rv);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const float a = lv[v] - xv[v], b = rv[v] - xv[v];
      sl = fmaf(a, a, sl);
      sr = fmaf(b, b, sr);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t e = nv * 8 + threadIdx.x; e < D; e += kBlk) {
      const float a = ld1(l, e) - x[e];
      const float b = ld1(r, e) - x[e];
      sl = fmaf(a, a, sl);
      sr = fmaf(b, b, sr);
    }
  }
  __shared__ float red[2][kBlk / kWave];
  sl = wave_sum(sl);
  sr = wave_sum(sr);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = sl;
    red[1][wv] = sr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < kBlk / kWave; ++k) {
      a += red[0][k];
      b += red[1][k];
    }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

template <typename T>
__global__ __launch_bounds__(kBlk) void gossip_mix_kernel(float* __restrict__ x,
                                                         T* __restrict__ p,
                                                         const T* __restrict__ l,
                                                         const T* __restrict__ r, int64_t D,
                                                         float w0, float w1, float w2, float clip,
                                                         const float* __restrict__ part, int nblk) {
  __shared__ float scl[2];
  if (threadIdx.x < 64) {
    double a = 0.0, b = 0.0;
    if (clip > 0.f) {
      for (int k = threadIdx.x; k < nblk; k += 64) {
        a += part[2 * k];
        b += part[2 * k + 1];
      }
      a = wave_sum(a);
      b = wave_sum(b);
    }
    if (threadIdx.x == 0) {
      scl[0] = clip > 0.f ? fminf(1.f, clip / fmaxf(sqrtf(static_cast<float>(a)), 1e-30f)) : 1.f;
      scl[1] = clip > 0.f ? fminf(1.f, clip / fmaxf(sqrtf(static_cast<float>(b)), 1e-30f)) : 1.f;
    }
  }
  __syncthreads();
  const float cl = w1 * scl[0], cr = w2 * scl[1], cs = w0 + w1 + w2;
  const int64_t nv = D / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlk;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kBlk + threadIdx.x; t < nv; t += stride) {
    float xv[8], lv[8], rv[8];
    load_vec<float, 8>(x + t * 8, xv);
    load_vec<T, 8>(l + t * 8, lv);
    load_vec<T, 8>(r + t * 8, rv);
#pragma unroll
    for (int v = 0; v < 8; ++v) xv[v] = fmaf(cs, xv[v], fmaf(cl, lv[v] - xv[v], cr * (rv[v] - xv[v])));
    store_f32<8>(x + t * 8, xv);
    if (p) {
      if constexpr (sizeof(T) == 2) store_bf16<8>(p + t * 8, xv);
      else store_f32<8>(p + t * 8, xv);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t e = nv * 8 + threadIdx.x; e < D; e += kBlk) {
      const float xe = x[e];
      const float v = fmaf(cs, xe, fmaf(cl, ld1(l, e) - xe, cr * (ld1(r, e) - xe)));
      x[e] = v;
      if (p) {
        if constexpr (sizeof(T) == 2) reinterpret_cast<uint16_t*>(p)[e] = f2bf(v);
        else p[e] = v;
      }
    }
  }
}

// ---------------------------------------------------------------- fault injection
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float gauss(uint64_t seed, int64_t i) {
  const uint64_t h = mix64(seed ^ mix64(static_cast<uint64_t>(i)));
  const float u1 = (static_cast<float>(h >> 40) + 1.0f) * (1.0f / 16777217.0f);
  const float u2 = static_cast<float>((h >> 16) & 0xffffff) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530718f * u2);
}

template <typename T>
__global__ __launch_bounds__(kBlk) void fault_kernel(T* g, int64_t D, int kind, float scale,
                                                    float sigma, uint64_t seed) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlk;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlk + threadIdx.x; i < D; i += stride) {
    float v;
    if constexpr (sizeof(T) == 2) v = bf2f(reinterpret_cast<uint16_t*>(g)[i]);
    else v = g[i];
    switch (kind) {
      case 1: v = -scale * v; break;                      // sign flip
      case 2: v = sigma * gauss(seed, i); break;          // gaussian
      case 3: v = scale * v; break;                       // scaled
      case 4: v = 0.f; break;                             // zero
      case 5: v = __builtin_nanf(""); break;              // nan
      default: break;
    }
    if constexpr (sizeof(T) == 2) reinterpret_cast<uint16_t*>(g)[i] = f2bf(v);
    else g[i] = v;
  }
}

int nblocks(int64_t work, int cap) {
  int64_t b = (work + kBlk - 1) / kBlk;
  if (b > cap) b = cap;
  return static_cast<int>(b < 1 ? 1 : b);
}

}  // namespace

size_t gossip_workspace_bytes(int64_t) { return 2 * kMaxBlk * sizeof(float); }

template <typename T>
void gossip_t(float* master, void* param_out, const void* left, const void* right, int64_t D,
              float w0, float w1, float w2, float clip, void* work, hipStream_t stream) {
  float* part = reinterpret_cast<float*>(work);
  const int nb = nblocks(D / 8, kMaxBlk);
  if (clip > 0.f)
    pair_sqdist_kernel<T><<<nb, kBlk, 0, stream>>>(master, reinterpret_cast<const T*>(left),
                                                   reinterpret_cast<const T*>(right), D, part);
  gossip_mix_kernel<T><<<nblocks(D / 8, 2048), kBlk, 0, stream>>>(
      master, reinterpret_cast<T*>(param_out), reinterpret_cast<const T*>(left),
      reinterpret_cast<const T*>(right), D, w0, w1, w2, clip, part, nb);
}

hipError_t launch_gossip_mix(int dtype, float* master, void* param_out, const void* left,
                             const void* right, int64_t D, float w0, float w1, float w2,
                             float clip, void* work, hipStream_t stream) {
  if ((reinterpret_cast<uintptr_t>(master) | reinterpret_cast<uintptr_t>(left) |
       reinterpret_cast<uintptr_t>(right) | reinterpret_cast<uintptr_t>(param_out)) % 16)
    return hipErrorInvalidValue;
  if (dtype == DT_BF16) gossip_t<bf16>(master, param_out, left, right, D, w0, w1, w2, clip, work, stream);
  else gossip_t<float>(master, param_out, left, right, D, w0, w1, w2, clip, work, stream);
  return hipGetLastError();
}

hipError_t launch_fault(int dtype, void* g, int64_t D, int kind, float scale, float sigma,
                        uint64_t seed, hipStream_t stream) {
  const int nb = nblocks(D, 2048);
  if (dtype == DT_BF16)
    fault_kernel<bf16><<<nb, kBlk, 0, stream>>>(reinterpret_cast<bf16*>(g), D, kind, scale, sigma, seed);
  else
    fault_kernel<float><<<nb, kBlk, 0, stream>>>(reinterpret_cast<float*>(g), D, kind, scale, sigma, seed);
  return hipGetLastError();
}

}  // namespace cml
