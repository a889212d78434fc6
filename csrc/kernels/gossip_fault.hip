// Decentralized gossip mixing (N09) and Byzantine fault injection (N10).
//
// Gossip: after the local step each rank holds its own fp32 master x and has received the bf16
// parameters of its k neighbours in this step's communication graph (ring: r - 1 and r + 1;
// exponential graphs: r +- 2^i, RCCL send/recv, all directions at once). The mix
//   x <- (w0 + sum_k w_k) x + sum_k w_k c_k (nb_k - x)
// with c_k = min(1, clip / ||nb_k - x||) (robust gossip: a Byzantine neighbour moves us by at
// most `clip`) is one streaming pass; the k distances need one reduction pass first. Partial
// sums go to a per-workgroup slab and the mix kernel's workgroups each fold the slab (<= 2048
// values, L2-resident) in a fixed order, so the result is deterministic and needs no extra
// launch or host sync.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kBlk = 256;
constexpr int kMaxBlk = 1024;
constexpr int kMaxNbrs = 8;     // neighbours of one gossip mix (the 7 xGMI peers of an 8-GPU node)

template <typename T>
__device__ __forceinline__ float ld1(const T* p, int64_t e) {
  if constexpr (sizeof(T) == 2) return bf2f(reinterpret_cast<const uint16_t*>(p)[e]);
  else return p[e];
}

// Neighbour pointers and mixing weights of one gossip step (by value: one kernel argument).
template <typename T>
struct Nbrs {
  const T* p[kMaxNbrs];
  float w[kMaxNbrs];
};

// per-workgroup partial ||nb_k - x||^2 for every neighbour k: part[k * nblk + block]
template <typename T, int K>
__global__ __launch_bounds__(kBlk) void nbr_sqdist_kernel(const float* __restrict__ x, Nbrs<T> nb,
                                                         int64_t D, float* __restrict__ part) {
  float s[K];
#pragma unroll
  for (int k = 0; k < K; ++k) s[k] = 0.f;
  const int64_t nv = D / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlk;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kBlk + threadIdx.x; t < nv; t += stride) {
    float xv[8];
    load_vec<float, 8>(x + t * 8, xv);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float v[8];
      load_vec<T, 8>(nb.p[k] + t * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[e] - xv[e];
        s[k] = fmaf(d, d, s[k]);
      }
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t e = nv * 8 + threadIdx.x; e < D; e += kBlk) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float d = ld1(nb.p[k], e) - x[e];
        s[k] = fmaf(d, d, s[k]);
      }
    }
  }
  __shared__ float red[K][kBlk / kWave];
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float v = wave_sum(s[k]);
    if ((threadIdx.x & 63) == 0) red[k][wv] = v;
  }
  __syncthreads();
  if (threadIdx.x < K) {
    float a = 0.f;
    for (int w = 0; w < kBlk / kWave; ++w) a += red[threadIdx.x][w];
    part[static_cast<int64_t>(threadIdx.x) * gridDim.x + blockIdx.x] = a;
  }
}

// x <- (w0 + sum_k w_k) x + sum_k w_k c_k (nb_k - x), c_k = min(1, clip / ||nb_k - x||); the
// sum is formed from the last neighbour down (for K = 2: fmaf(c0, l - x, c1 (r - x)), the ring
// kernel's expression). Each workgroup folds the distance slab itself (fixed order).
template <typename T, int K>
__global__ __launch_bounds__(kBlk) void gossip_mix_kernel(float* __restrict__ x, T* __restrict__ p,
                                                         T* __restrict__ p2,
                                                         Nbrs<T> nb, int64_t D, float w0,
                                                         float clip, const float* __restrict__ part,
                                                         int nblk) {
  __shared__ float scl[K];
  if (threadIdx.x < 64) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double a = 0.0;
      if (clip > 0.f) {
        for (int b = threadIdx.x; b < nblk; b += 64) a += part[static_cast<int64_t>(k) * nblk + b];
        a = wave_sum(a);
      }
      if (threadIdx.x == 0)
        scl[k] = clip > 0.f ? fminf(1.f, clip / fmaxf(sqrtf(static_cast<float>(a)), 1e-30f)) : 1.f;
    }
  }
  __syncthreads();
  float c[K];
  float cs = w0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    c[k] = nb.w[k] * scl[k];
    cs += nb.w[k];
  }
  const int64_t nv = D / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlk;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kBlk + threadIdx.x; t < nv; t += stride) {
    float xv[8], acc[8];
    load_vec<float, 8>(x + t * 8, xv);
    {
      float v[8];
      load_vec<T, 8>(nb.p[K - 1] + t * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = c[K - 1] * (v[e] - xv[e]);
    }
#pragma unroll
    for (int k = K - 2; k >= 0; --k) {
      float v[8];
      load_vec<T, 8>(nb.p[k] + t * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(c[k], v[e] - xv[e], acc[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = fmaf(cs, xv[e], acc[e]);
    store_f32<8>(x + t * 8, xv);
    if (p) {
      if constexpr (sizeof(T) == 2) store_bf16<8>(p + t * 8, xv);
      else store_f32<8>(p + t * 8, xv);
    }
    if (p2) {   // the delayed-gossip send buffer: written here instead of copied from p
      if constexpr (sizeof(T) == 2) store_bf16<8>(p2 + t * 8, xv);
      else store_f32<8>(p2 + t * 8, xv);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t e = nv * 8 + threadIdx.x; e < D; e += kBlk) {
      const float xe = x[e];
      float acc = c[K - 1] * (ld1(nb.p[K - 1], e) - xe);
#pragma unroll
      for (int k = K - 2; k >= 0; --k) acc = fmaf(c[k], ld1(nb.p[k], e) - xe, acc);
      const float v = fmaf(cs, xe, acc);
      x[e] = v;
      if (p) {
        if constexpr (sizeof(T) == 2) reinterpret_cast<uint16_t*>(p)[e] = f2bf(v);
        else p[e] = v;
      }
      if (p2) {
        if constexpr (sizeof(T) == 2) reinterpret_cast<uint16_t*>(p2)[e] = f2bf(v);
        else p2[e] = v;
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

size_t gossip_workspace_bytes(int64_t) { return kMaxNbrs * kMaxBlk * sizeof(float); }

namespace {
template <typename T, int K>
void gossip_k(float* master, void* param_out, void* param_out2, const Nbrs<T>& nb, int64_t D,
              float w0, float clip, void* work, hipStream_t stream) {
  float* part = reinterpret_cast<float*>(work);
  const int nb_blocks = nblocks(D / 8, kMaxBlk);
  if (clip > 0.f) nbr_sqdist_kernel<T, K><<<nb_blocks, kBlk, 0, stream>>>(master, nb, D, part);
  static const int cap = [] {   // CML_GOSSIP_GRID_CAP (default 0: one vector per thread, the
    const char* e = getenv("CML_GOSSIP_GRID_CAP");   // fastest streaming form; 2048: the former
    return e ? atoi(e) : 0;                          // grid-stride launch)
  }();
  gossip_mix_kernel<T, K><<<nblocks(D / 8, cap > 0 ? cap : (1 << 30)), kBlk, 0, stream>>>(
      master, reinterpret_cast<T*>(param_out), reinterpret_cast<T*>(param_out2), nb, D, w0, clip,
      part, nb_blocks);
}

template <typename T>
hipError_t gossip_t(float* master, void* param_out, void* param_out2, const void* const* nbrs,
                    const float* w, int k, int64_t D, float w0, float clip, void* work,
                    hipStream_t stream) {
  Nbrs<T> nb{};
  for (int i = 0; i < k; ++i) {
    nb.p[i] = reinterpret_cast<const T*>(nbrs[i]);
    nb.w[i] = w[i];
  }
  switch (k) {
    case 1: gossip_k<T, 1>(master, param_out, param_out2, nb, D, w0, clip, work, stream); break;
    case 2: gossip_k<T, 2>(master, param_out, param_out2, nb, D, w0, clip, work, stream); break;
    case 3: gossip_k<T, 3>(master, param_out, param_out2, nb, D, w0, clip, work, stream); break;
    case 4: gossip_k<T, 4>(master, param_out, param_out2, nb, D, w0, clip, work, stream); break;
    case 5: gossip_k<T, 5>(master, param_out, param_out2, nb, D, w0, clip, work, stream); break;
    case 6: gossip_k<T, 6>(master, param_out, param_out2, nb, D, w0, clip, work, stream); break;
    case 7: gossip_k<T, 7>(master, param_out, param_out2, nb, D, w0, clip, work, stream); break;
    case 8: gossip_k<T, 8>(master, param_out, param_out2, nb, D, w0, clip, work, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
}  // namespace

hipError_t launch_gossip_mix_k(int dtype, float* master, void* param_out, const void* const* nbrs,
                               const float* w, int k, int64_t D, float w0, float clip, void* work,
                               hipStream_t stream, void* param_out2) {
  if (k < 1 || k > kMaxNbrs) return hipErrorInvalidValue;
  uintptr_t a = reinterpret_cast<uintptr_t>(master) | reinterpret_cast<uintptr_t>(param_out) |
                reinterpret_cast<uintptr_t>(param_out2);
  for (int i = 0; i < k; ++i) a |= reinterpret_cast<uintptr_t>(nbrs[i]);
  if (a % 16) return hipErrorInvalidValue;
  return dtype == DT_BF16
             ? gossip_t<bf16>(master, param_out, param_out2, nbrs, w, k, D, w0, clip, work, stream)
             : gossip_t<float>(master, param_out, param_out2, nbrs, w, k, D, w0, clip, work, stream);
}

hipError_t launch_gossip_mix(int dtype, float* master, void* param_out, const void* left,
                             const void* right, int64_t D, float w0, float w1, float w2,
                             float clip, void* work, hipStream_t stream) {
  const void* nb[2] = {left, right};
  const float w[2] = {w1, w2};
  return launch_gossip_mix_k(dtype, master, param_out, nb, w, 2, D, w0, clip, work, stream);
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
