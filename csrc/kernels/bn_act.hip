// Fused training BatchNorm + (residual add) + ReLU for NHWC (channels_last) bf16 activations.
//
// The ResNet-50 profile (profiles/r01_*) spends ~62 % of GPU time in PyTorch's channels_last BN
// kernels (stats collection and backward reduce at ~5 % of HBM bandwidth) plus separate ReLU /
// threshold-backward / residual passes. Here each BN-ReLU is:
//   forward : stats (read x) -> finalize (per-channel, tiny) -> apply (read x [+res], write y)
//   backward: reduce (read dy, x [+res]) -> finalize -> apply (read dy, x [+res], write dx [+dres])
// = 3 + 5 activation passes, the ReLU mask recomputed from x (z = x*scale + bias + res > 0) so y is
// never re-read. Every thread owns 8 consecutive channels (one 16-B load per row); a 256-thread
// workgroup covers 256/(C/8) rows per iteration and walks a contiguous row range, so every load
// instruction is a dense 1-KiB wave access. Per-workgroup partial sums go to a [nb][2][C] slab
// that a per-channel finalize kernel folds in fp64 in block order (deterministic). Variance uses
// sums shifted by the first row's value (cancellation-safe for post-conv activations).
#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kBT = 256;

struct BNGeom {
  int tpr;     // threads per row = C / 8
  int rpi;     // rows per workgroup iteration = 256 / tpr
  int nb;      // workgroups
  int64_t rpb; // rows per workgroup
};

BNGeom geom(int64_t M, int C) {
  BNGeom g;
  g.tpr = C / 8;
  g.rpi = kBT / g.tpr;
  const int64_t iters = (M + g.rpi - 1) / g.rpi;
  int64_t nb = (iters + 15) / 16;          // >= 16 row-iterations per workgroup
  if (nb > 1024) nb = 1024;
  if (nb < 1) nb = 1;
  g.rpb = ((M + nb - 1) / nb + g.rpi - 1) / g.rpi * g.rpi;
  g.nb = static_cast<int>((M + g.rpb - 1) / g.rpb);
  return g;
}

__device__ __forceinline__ void ld8(const bf16* p, float (&o)[8]) { load_vec<bf16, 8>(p, o); }

// Fold per-thread accumulators [8] x 2 across the rows of a workgroup (same channel group) and
// write one [2][C] partial per workgroup.
__device__ __forceinline__ void block_partial(float (&a)[8], float (&b)[8], int tpr, int C,
                                              float* __restrict__ part) {
  __shared__ float sa[kBT * 8];
  __shared__ float sb[kBT * 8];
  const int t = threadIdx.x;
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    sa[t * 8 + v] = a[v];
    sb[t * 8 + v] = b[v];
  }
  __syncthreads();
  const int rpi = kBT / tpr;
  float* pa = part + static_cast<int64_t>(blockIdx.x) * 2 * C;
  float* pb = pa + C;
  for (int c = t; c < C; c += kBT) {
    const int g = c >> 3, v = c & 7;
    float x = 0.f, y = 0.f;
    for (int r = 0; r < rpi; ++r) {
      x += sa[(r * tpr + g) * 8 + v];
      y += sb[(r * tpr + g) * 8 + v];
    }
    pa[c] = x;
    pb[c] = y;
  }
}

// ----------------------------------------------------------------------------- forward
__global__ __launch_bounds__(kBT) void bn_stats_kernel(const bf16* __restrict__ x, int64_t M, int C,
                                                      int64_t rpb, float* __restrict__ part) {
  const int tpr = C / 8;
  const int rpi = kBT / tpr;
  const int g = threadIdx.x % tpr;
  const int r0 = threadIdx.x / tpr;
  float sh[8];
  ld8(x + 8 * g, sh);   // shift = row 0
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * rpb;
  const int64_t hi = lo + rpb < M ? lo + rpb : M;
  for (int64_t r = lo + r0; r < hi; r += rpi) {
    float v[8];
    ld8(x + r * C + 8 * g, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = v[k] - sh[k];
      s[k] += d;
      q[k] = fmaf(d, d, q[k]);
    }
  }
  block_partial(s, q, tpr, C, part);
}

// Fold the [nb][2][C] slab for 32 channels per workgroup: 8 slices of the partial blocks per
// channel, 4 independent fp64 accumulators per thread (loads stay in flight), then a fixed-order
// LDS combine -> deterministic (s, q) per channel in the first 32 threads.
constexpr int kFC = 32;               // channels per finalize workgroup
constexpr int kFS = kBT / kFC;        // partial-block slices
__device__ __forceinline__ bool fold_partials(const float* __restrict__ part, int nb, int C,
                                              double& s_out, double& q_out, int& c_out) {
  __shared__ double ls[kFS][kFC], lq[kFS][kFC];
  const int cl = threadIdx.x % kFC, sl = threadIdx.x / kFC;
  const int c = blockIdx.x * kFC + cl;
  double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
  if (c < C) {
    int b = sl;
    for (; b + 3 * kFS < nb; b += 4 * kFS) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* p = part + static_cast<int64_t>(b + u * kFS) * 2 * C;
        s[u] += p[c];
        q[u] += p[C + c];
      }
    }
    for (; b < nb; b += kFS) {
      const float* p = part + static_cast<int64_t>(b) * 2 * C;
      s[0] += p[c];
      q[0] += p[C + c];
    }
  }
  ls[sl][cl] = (s[0] + s[1]) + (s[2] + s[3]);
  lq[sl][cl] = (q[0] + q[1]) + (q[2] + q[3]);
  __syncthreads();
  if (sl != 0 || c >= C) return false;
  double S = 0.0, Q = 0.0;
#pragma unroll
  for (int k = 0; k < kFS; ++k) {
    S += ls[k][cl];
    Q += lq[k][cl];
  }
  s_out = S;
  q_out = Q;
  c_out = c;
  return true;
}

// mean / invstd (fp32 [C]) from the partial slab; running stats update (unbiased variance).
__global__ __launch_bounds__(kBT) void bn_finalize_kernel(const float* __restrict__ part, int nb,
                                                         const bf16* __restrict__ x, int64_t M,
                                                         int C, float eps, float momentum,
                                                         float* __restrict__ mean,
                                                         float* __restrict__ invstd,
                                                         float* __restrict__ rmean,
                                                         float* __restrict__ rvar) {
  double s, q;
  int c;
  if (!fold_partials(part, nb, C, s, q, c)) return;
  const double ms = s / static_cast<double>(M);
  double var = q / static_cast<double>(M) - ms * ms;
  if (var < 0.0) var = 0.0;
  const double mu = static_cast<double>(bf2f(reinterpret_cast<const uint16_t*>(x)[c])) + ms;
  mean[c] = static_cast<float>(mu);
  invstd[c] = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
  if (rmean) {
    const double unb = M > 1 ? var * static_cast<double>(M) / static_cast<double>(M - 1) : var;
    rmean[c] = static_cast<float>((1.0 - momentum) * rmean[c] + momentum * mu);
    rvar[c] = static_cast<float>((1.0 - momentum) * rvar[c] + momentum * unb);
  }
}

__device__ __forceinline__ void chan_affine(int g, const float* mean, const float* invstd,
                                            const bf16* gamma, const bf16* beta, float (&sc)[8],
                                            float (&bi)[8]) {
  float ga[8], be[8];
  ld8(gamma + 8 * g, ga);
  ld8(beta + 8 * g, be);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = invstd[8 * g + k] * ga[k];
    bi[k] = be[k] - mean[8 * g + k] * sc[k];
  }
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(kBT) void bn_apply_kernel(const bf16* __restrict__ x,
                                                      const bf16* __restrict__ res,
                                                      bf16* __restrict__ y, int64_t M, int C,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ invstd,
                                                      const bf16* __restrict__ gamma,
                                                      const bf16* __restrict__ beta) {
  const int tpr = C / 8;
  const int g = threadIdx.x % tpr;
  float sc[8], bi[8];
  chan_affine(g, mean, invstd, gamma, beta, sc, bi);
  const int64_t rstride = static_cast<int64_t>(gridDim.x) * (kBT / tpr);
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kBT / tpr) + threadIdx.x / tpr; r < M; r += rstride) {
    float v[8];
    ld8(x + r * C + 8 * g, v);
    float rv[8];
    if constexpr (RES) ld8(res + r * C + 8 * g, rv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float z = fmaf(v[k], sc[k], bi[k]);
      if constexpr (RES) z += rv[k];
      if constexpr (RELU) z = fmaxf(z, 0.f);
      v[k] = z;
    }
    store_bf16<8>(y + r * C + 8 * g, v);
  }
}

// ----------------------------------------------------------------------------- backward
template <bool RES, bool RELU>
__global__ __launch_bounds__(kBT) void bn_bwd_reduce_kernel(const bf16* __restrict__ dy,
                                                           const bf16* __restrict__ x,
                                                           const bf16* __restrict__ res, int64_t M,
                                                           int C, int64_t rpb,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const bf16* __restrict__ gamma,
                                                           const bf16* __restrict__ beta,
                                                           float* __restrict__ part) {
  const int tpr = C / 8;
  const int rpi = kBT / tpr;
  const int g = threadIdx.x % tpr;
  float sc[8], bi[8], mu[8], is[8];
  chan_affine(g, mean, invstd, gamma, beta, sc, bi);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = mean[8 * g + k];
    is[k] = invstd[8 * g + k];
  }
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * rpb;
  const int64_t hi = lo + rpb < M ? lo + rpb : M;
  for (int64_t r = lo + threadIdx.x / tpr; r < hi; r += rpi) {
    float d[8], v[8], rv[8];
    ld8(dy + r * C + 8 * g, d);
    ld8(x + r * C + 8 * g, v);
    if constexpr (RES && RELU) ld8(res + r * C + 8 * g, rv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float dz = d[k];
      if constexpr (RELU) {
        float z = fmaf(v[k], sc[k], bi[k]);
        if constexpr (RES) z += rv[k];
        dz = z > 0.f ? dz : 0.f;
      }
      s[k] += dz;
      q[k] = fmaf(dz, (v[k] - mu[k]) * is[k], q[k]);
    }
  }
  block_partial(s, q, tpr, C, part);
}

__global__ __launch_bounds__(kBT) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nb,
                                                             int C, float* __restrict__ sdz,
                                                             float* __restrict__ sdzx,
                                                             bf16* __restrict__ dgamma,
                                                             bf16* __restrict__ dbeta) {
  double s, q;
  int c;
  if (!fold_partials(part, nb, C, s, q, c)) return;
  sdz[c] = static_cast<float>(s);
  sdzx[c] = static_cast<float>(q);
  reinterpret_cast<uint16_t*>(dbeta)[c] = f2bf(static_cast<float>(s));
  reinterpret_cast<uint16_t*>(dgamma)[c] = f2bf(static_cast<float>(q));
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(kBT) void bn_bwd_apply_kernel(const bf16* __restrict__ dy,
                                                          const bf16* __restrict__ x,
                                                          const bf16* __restrict__ res,
                                                          bf16* __restrict__ dx,
                                                          bf16* __restrict__ dres, int64_t M, int C,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const bf16* __restrict__ gamma,
                                                          const bf16* __restrict__ beta,
                                                          const float* __restrict__ sdz,
                                                          const float* __restrict__ sdzx) {
  const int tpr = C / 8;
  const int g = threadIdx.x % tpr;
  float sc[8], bi[8], mu[8], is[8], a[8], b[8];
  chan_affine(g, mean, invstd, gamma, beta, sc, bi);
  const float invM = 1.0f / static_cast<float>(M);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = mean[8 * g + k];
    is[k] = invstd[8 * g + k];
    a[k] = sdz[8 * g + k] * invM;
    b[k] = sdzx[8 * g + k] * invM;
  }
  const int64_t rstride = static_cast<int64_t>(gridDim.x) * (kBT / tpr);
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kBT / tpr) + threadIdx.x / tpr; r < M; r += rstride) {
    float d[8], v[8], rv[8], o[8];
    ld8(dy + r * C + 8 * g, d);
    ld8(x + r * C + 8 * g, v);
    if constexpr (RES && RELU) ld8(res + r * C + 8 * g, rv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float dz = d[k];
      if constexpr (RELU) {
        float z = fmaf(v[k], sc[k], bi[k]);
        if constexpr (RES) z += rv[k];
        dz = z > 0.f ? dz : 0.f;
      }
      d[k] = dz;
      const float xh = (v[k] - mu[k]) * is[k];
      o[k] = sc[k] * (dz - a[k] - xh * b[k]);
    }
    store_bf16<8>(dx + r * C + 8 * g, o);
    if constexpr (RES) store_bf16<8>(dres + r * C + 8 * g, d);
  }
}

int apply_grid(int64_t M, int C) {
  const int rpi = kBT / (C / 8);
  int64_t b = (M + rpi - 1) / rpi;
  if (b > 2048) b = 2048;
  return static_cast<int>(b < 1 ? 1 : b);
}

}  // namespace

size_t bn_workspace_bytes(int64_t M, int C) {
  const BNGeom g = geom(M, C);
  return static_cast<size_t>(g.nb) * 2 * C * sizeof(float);
}

hipError_t launch_bn_fwd(const void* x, const void* res, void* y, int64_t M, int C,
                         const void* gamma, const void* beta, float* mean, float* invstd,
                         float* rmean, float* rvar, float eps, float momentum, int relu,
                         int training, void* work, hipStream_t st) {
  if (C % 8 != 0 || C / 8 > kBT || (kBT % (C / 8)) != 0 || M < 1) return hipErrorInvalidValue;
  const bf16* xb = reinterpret_cast<const bf16*>(x);
  if (training) {
    const BNGeom g = geom(M, C);
    float* part = reinterpret_cast<float*>(work);
    bn_stats_kernel<<<g.nb, kBT, 0, st>>>(xb, M, C, g.rpb, part);
    bn_finalize_kernel<<<(C + kFC - 1) / kFC, kBT, 0, st>>>(part, g.nb, xb, M, C, eps, momentum,
                                                            mean, invstd, rmean, rvar);
  }
  const int ga = apply_grid(M, C);
  const bf16* rb = reinterpret_cast<const bf16*>(res);
  bf16* yb = reinterpret_cast<bf16*>(y);
  const bf16* gm = reinterpret_cast<const bf16*>(gamma);
  const bf16* bt = reinterpret_cast<const bf16*>(beta);
  if (res && relu) bn_apply_kernel<true, true><<<ga, kBT, 0, st>>>(xb, rb, yb, M, C, mean, invstd, gm, bt);
  else if (res) bn_apply_kernel<true, false><<<ga, kBT, 0, st>>>(xb, rb, yb, M, C, mean, invstd, gm, bt);
  else if (relu) bn_apply_kernel<false, true><<<ga, kBT, 0, st>>>(xb, rb, yb, M, C, mean, invstd, gm, bt);
  else bn_apply_kernel<false, false><<<ga, kBT, 0, st>>>(xb, rb, yb, M, C, mean, invstd, gm, bt);
  return hipGetLastError();
}

hipError_t launch_bn_bwd(const void* dy, const void* x, const void* res, void* dx, void* dres,
                         int64_t M, int C, const void* gamma, const void* beta, const float* mean,
                         const float* invstd, void* dgamma, void* dbeta, float* sdz, float* sdzx,
                         int relu, void* work, hipStream_t st) {
  if (C % 8 != 0 || C / 8 > kBT || (kBT % (C / 8)) != 0 || M < 1) return hipErrorInvalidValue;
  const BNGeom g = geom(M, C);
  float* part = reinterpret_cast<float*>(work);
  const bf16* d = reinterpret_cast<const bf16*>(dy);
  const bf16* xb = reinterpret_cast<const bf16*>(x);
  const bf16* rb = reinterpret_cast<const bf16*>(res);
  const bf16* gm = reinterpret_cast<const bf16*>(gamma);
  const bf16* bt = reinterpret_cast<const bf16*>(beta);
  if (res && relu) bn_bwd_reduce_kernel<true, true><<<g.nb, kBT, 0, st>>>(d, xb, rb, M, C, g.rpb, mean, invstd, gm, bt, part);
  else if (relu) bn_bwd_reduce_kernel<false, true><<<g.nb, kBT, 0, st>>>(d, xb, rb, M, C, g.rpb, mean, invstd, gm, bt, part);
  else bn_bwd_reduce_kernel<false, false><<<g.nb, kBT, 0, st>>>(d, xb, rb, M, C, g.rpb, mean, invstd, gm, bt, part);
  bn_bwd_finalize_kernel<<<(C + kFC - 1) / kFC, kBT, 0, st>>>(part, g.nb, C, sdz, sdzx,
                                                              reinterpret_cast<bf16*>(dgamma),
                                                              reinterpret_cast<bf16*>(dbeta));
  const int ga = apply_grid(M, C);
  bf16* dxb = reinterpret_cast<bf16*>(dx);
  bf16* drb = reinterpret_cast<bf16*>(dres);
  if (res && relu) bn_bwd_apply_kernel<true, true><<<ga, kBT, 0, st>>>(d, xb, rb, dxb, drb, M, C, mean, invstd, gm, bt, sdz, sdzx);
  else if (res) bn_bwd_apply_kernel<true, false><<<ga, kBT, 0, st>>>(d, xb, rb, dxb, drb, M, C, mean, invstd, gm, bt, sdz, sdzx);
  else if (relu) bn_bwd_apply_kernel<false, true><<<ga, kBT, 0, st>>>(d, xb, rb, dxb, drb, M, C, mean, invstd, gm, bt, sdz, sdzx);
  else bn_bwd_apply_kernel<false, false><<<ga, kBT, 0, st>>>(d, xb, rb, dxb, drb, M, C, mean, invstd, gm, bt, sdz, sdzx);
  return hipGetLastError();
}

}  // namespace cml
