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
#include <cstdlib>

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

// Every activation the BN passes read is read once per pass: CML_BN_NT = 1 makes those loads
// nontemporal (A/B switch, a device flag set once per process before the first BN launch)
__device__ int g_bn_nt = 0;
typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ld8(const bf16* p, float (&o)[8]) {
  if (g_bn_nt) {
    const v4u_t t = __builtin_nontemporal_load(reinterpret_cast<const v4u_t*>(p));
    const uint32_t w[4] = {t[0], t[1], t[2], t[3]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = __uint_as_float(w[i] << 16);
      o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    load_vec<bf16, 8>(p, o);
  }
}
void bn_nt_init() {
  static const bool done = [] {
    const char* e = getenv("CML_BN_NT");
    const int v = e ? atoi(e) : 0;
    if (v) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bn_nt), &v, sizeof(int));
    return true;
  }();
  (void)done;
}

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
  // 4 rows (4 x 16-B loads) in flight per lane: one load per iteration left the stats pass
  // latency-bound at ~4.3 TB/s (profiles/r01_prof17_*)
  int64_t r = lo + r0;
  for (; r + 3 * rpi < hi; r += 4 * rpi) {
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) ld8(x + (r + u * rpi) * C + 8 * g, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[u][k] - sh[k];
        s[k] += d;
        q[k] = fmaf(d, d, q[k]);
      }
  }
  for (; r < hi; r += rpi) {
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

// Fold the [nb][2][C] slab for 8 channels per workgroup: 32 slices of the partial blocks per
// channel, 8 partials (16 loads) in flight per thread, fp64 accumulation, then a fixed-order LDS
// combine -> deterministic (s, q) per channel in the first 8 threads. The fold is latency-bound
// (nb <= 1024 partials, L2-resident), so the slices keep every thread's chain of dependent load
// rounds at nb / 256 (4 for nb = 1024); 32 channels x 8 slices took ~13 us per BN layer.
constexpr int kFC = 8;                // channels per finalize workgroup
constexpr int kFS = kBT / kFC;        // partial-block slices
__device__ __forceinline__ bool fold_partials(const float* __restrict__ part, int nb, int C,
                                              double& s_out, double& q_out, int& c_out) {
  __shared__ double ls[kFS][kFC], lq[kFS][kFC];
  const int cl = threadIdx.x % kFC, sl = threadIdx.x / kFC;
  const int c = blockIdx.x * kFC + cl;
  double S = 0.0, Q = 0.0;
  if (c < C) {
    int b = sl;
    for (; b + 7 * kFS < nb; b += 8 * kFS) {
      float s[8], q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float* p = part + static_cast<int64_t>(b + u * kFS) * 2 * C;
        s[u] = p[c];
        q[u] = p[C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        S += s[u];
        Q += q[u];
      }
    }
    for (; b < nb; b += kFS) {
      const float* p = part + static_cast<int64_t>(b) * 2 * C;
      S += p[c];
      Q += p[C + c];
    }
  }
  ls[sl][cl] = S;
  lq[sl][cl] = Q;
  __syncthreads();
  if (sl != 0 || c >= C) return false;
  S = 0.0;
  Q = 0.0;
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

// MASK (RES + RELU blocks): also write the ReLU mask as one bit per element ([M, C/8] bytes), so
// the backward never reads the residual again (2 B/elem per backward pass -> 1/8 B).
template <bool RES, bool RELU, bool MASK>
__global__ __launch_bounds__(kBT) void bn_apply_kernel(const bf16* __restrict__ x,
                                                      const bf16* __restrict__ res,
                                                      bf16* __restrict__ y,
                                                      uint8_t* __restrict__ mask, int64_t M, int C,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ invstd,
                                                      const bf16* __restrict__ gamma,
                                                      const bf16* __restrict__ beta) {
  const int tpr = C / 8;
  const int g = threadIdx.x % tpr;
  float sc[8], bi[8];
  chan_affine(g, mean, invstd, gamma, beta, sc, bi);
  const int64_t rstride = static_cast<int64_t>(gridDim.x) * (kBT / tpr);
  // two rows per iteration: both rows' loads are issued before either is used
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kBT / tpr) + threadIdx.x / tpr; r < M;
       r += 2 * rstride) {
    const bool two = r + rstride < M;
    float v[2][8], rv[2][8];
    ld8(x + r * C + 8 * g, v[0]);
    if constexpr (RES) ld8(res + r * C + 8 * g, rv[0]);
    if (two) {
      ld8(x + (r + rstride) * C + 8 * g, v[1]);
      if constexpr (RES) ld8(res + (r + rstride) * C + 8 * g, rv[1]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      const int64_t ru = r + u * rstride;
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float z = fmaf(v[u][k], sc[k], bi[k]);
        if constexpr (RES) z += rv[u][k];
        if constexpr (MASK) bits |= (z > 0.f ? 1u : 0u) << k;
        if constexpr (RELU) z = fmaxf(z, 0.f);
        v[u][k] = z;
      }
      store_bf16<8>(y + ru * C + 8 * g, v[u]);
      if constexpr (MASK) mask[ru * tpr + g] = static_cast<uint8_t>(bits);
    }
  }
}

// ----------------------------------------------------------------------------- backward
// ReLU handling in the backward: RM_NONE (no ReLU), RM_RECOMP (mask recomputed from x: BN-ReLU
// without residual), RM_MASK (bit mask written by the forward: BN + residual + ReLU).
// DY2: the output gradient arrives in two parts (dy + dy2, see ops.bn.ResidualLink) and is summed
// on load, replacing a separate elementwise add pass.
enum { RM_NONE = 0, RM_RECOMP = 1, RM_MASK = 2 };

template <int RM, bool DY2>
__device__ __forceinline__ void load_dz(const bf16* __restrict__ dy, const bf16* __restrict__ dy2,
                                        const uint8_t* __restrict__ mask, int64_t r, int C, int g,
                                        const float (&v)[8], const float (&sc)[8],
                                        const float (&bi)[8], float (&dz)[8]) {
  ld8(dy + r * C + 8 * g, dz);
  if constexpr (DY2) {
    float d2[8];
    ld8(dy2 + r * C + 8 * g, d2);
#pragma unroll
    for (int k = 0; k < 8; ++k) dz[k] += d2[k];
  }
  if constexpr (RM == RM_MASK) {
    const uint32_t bits = mask[r * (C / 8) + g];
#pragma unroll
    for (int k = 0; k < 8; ++k) dz[k] = ((bits >> k) & 1u) ? dz[k] : 0.f;
  } else if constexpr (RM == RM_RECOMP) {
#pragma unroll
    for (int k = 0; k < 8; ++k) dz[k] = fmaf(v[k], sc[k], bi[k]) > 0.f ? dz[k] : 0.f;
  }
}

template <int RM, bool DY2>
__global__ __launch_bounds__(kBT) void bn_bwd_reduce_kernel(const bf16* __restrict__ dy,
                                                           const bf16* __restrict__ dy2,
                                                           const bf16* __restrict__ x,
                                                           const uint8_t* __restrict__ mask,
                                                           int64_t M, int C, int64_t rpb,
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
  int64_t r = lo + threadIdx.x / tpr;
  for (; r + rpi < hi; r += 2 * rpi) {   // two rows' loads in flight
    float v[2][8], dz[2][8];
    ld8(x + r * C + 8 * g, v[0]);
    ld8(x + (r + rpi) * C + 8 * g, v[1]);
    load_dz<RM, DY2>(dy, dy2, mask, r, C, g, v[0], sc, bi, dz[0]);
    load_dz<RM, DY2>(dy, dy2, mask, r + rpi, C, g, v[1], sc, bi, dz[1]);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += dz[u][k];
        q[k] = fmaf(dz[u][k], (v[u][k] - mu[k]) * is[k], q[k]);
      }
  }
  for (; r < hi; r += rpi) {
    float v[8], dz[8];
    ld8(x + r * C + 8 * g, v);
    load_dz<RM, DY2>(dy, dy2, mask, r, C, g, v, sc, bi, dz);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[k] += dz[k];
      q[k] = fmaf(dz[k], (v[k] - mu[k]) * is[k], q[k]);
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

// DRES: also write the gradient of the residual input (= the masked output gradient).
template <int RM, bool DRES, bool DY2>
__global__ __launch_bounds__(kBT) void bn_bwd_apply_kernel(const bf16* __restrict__ dy,
                                                          const bf16* __restrict__ dy2,
                                                          const bf16* __restrict__ x,
                                                          const uint8_t* __restrict__ mask,
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
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kBT / tpr) + threadIdx.x / tpr; r < M;
       r += 2 * rstride) {   // two rows' loads in flight
    const bool two = r + rstride < M;
    float v[2][8], dz[2][8];
    ld8(x + r * C + 8 * g, v[0]);
    if (two) ld8(x + (r + rstride) * C + 8 * g, v[1]);
    load_dz<RM, DY2>(dy, dy2, mask, r, C, g, v[0], sc, bi, dz[0]);
    if (two) load_dz<RM, DY2>(dy, dy2, mask, r + rstride, C, g, v[1], sc, bi, dz[1]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      const int64_t ru = r + u * rstride;
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (v[u][k] - mu[k]) * is[k];
        o[k] = sc[k] * (dz[u][k] - a[k] - xh * b[k]);
      }
      store_bf16<8>(dx + ru * C + 8 * g, o);
      if constexpr (DRES) store_bf16<8>(dres + ru * C + 8 * g, dz[u]);
    }
  }
}

// ----------------------------------------------------------------------------- two BNs, one sum
// Downsample-block tail: y = relu(bn3(x1) + bn_d(x2)). The shortcut BN's output is never
// materialised: its affine is applied on the fly in the apply pass, and the backward computes both
// BNs' reductions in one pass over (dy [+ dy2], mask, x1, x2) and both input gradients in one more,
// with no residual-gradient tensor in between (per element 10.1 B forward / 16.25 B backward vs
// 14.1 / 22.25 B for BN + BN + add).
template <bool MASK>
__global__ __launch_bounds__(kBT) void bn_apply2_kernel(const bf16* __restrict__ x1,
                                                       const bf16* __restrict__ x2,
                                                       bf16* __restrict__ y,
                                                       uint8_t* __restrict__ mask, int64_t M, int C,
                                                       const float* __restrict__ mean1,
                                                       const float* __restrict__ invstd1,
                                                       const bf16* __restrict__ gamma1,
                                                       const bf16* __restrict__ beta1,
                                                       const float* __restrict__ mean2,
                                                       const float* __restrict__ invstd2,
                                                       const bf16* __restrict__ gamma2,
                                                       const bf16* __restrict__ beta2) {
  const int tpr = C / 8;
  const int g = threadIdx.x % tpr;
  float sc1[8], bi1[8], sc2[8], bi2[8];
  chan_affine(g, mean1, invstd1, gamma1, beta1, sc1, bi1);
  chan_affine(g, mean2, invstd2, gamma2, beta2, sc2, bi2);
#pragma unroll
  for (int k = 0; k < 8; ++k) bi1[k] += bi2[k];
  const int64_t rstride = static_cast<int64_t>(gridDim.x) * (kBT / tpr);
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kBT / tpr) + threadIdx.x / tpr; r < M;
       r += 2 * rstride) {
    const bool two = r + rstride < M;
    float a[2][8], b[2][8];
    ld8(x1 + r * C + 8 * g, a[0]);
    ld8(x2 + r * C + 8 * g, b[0]);
    if (two) {
      ld8(x1 + (r + rstride) * C + 8 * g, a[1]);
      ld8(x2 + (r + rstride) * C + 8 * g, b[1]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      const int64_t ru = r + u * rstride;
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float z = fmaf(a[u][k], sc1[k], fmaf(b[u][k], sc2[k], bi1[k]));
        if constexpr (MASK) bits |= (z > 0.f ? 1u : 0u) << k;
        a[u][k] = fmaxf(z, 0.f);
      }
      store_bf16<8>(y + ru * C + 8 * g, a[u]);
      if constexpr (MASK) mask[ru * tpr + g] = static_cast<uint8_t>(bits);
    }
  }
}

// one pass: s = sum dz, q1 = sum dz xh1, q2 = sum dz xh2 -> part1 [nb][2][C] (s, q1),
// part2 [nb][2][C] (s, q2)
template <bool DY2>
__global__ __launch_bounds__(kBT) void bn_bwd_reduce2_kernel(const bf16* __restrict__ dy,
                                                            const bf16* __restrict__ dy2,
                                                            const bf16* __restrict__ x1,
                                                            const bf16* __restrict__ x2,
                                                            const uint8_t* __restrict__ mask,
                                                            int64_t M, int C, int64_t rpb,
                                                            const float* __restrict__ mean1,
                                                            const float* __restrict__ invstd1,
                                                            const float* __restrict__ mean2,
                                                            const float* __restrict__ invstd2,
                                                            float* __restrict__ part1,
                                                            float* __restrict__ part2) {
  const int tpr = C / 8;
  const int rpi = kBT / tpr;
  const int g = threadIdx.x % tpr;
  float mu1[8], is1[8], mu2[8], is2[8], dummy[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu1[k] = mean1[8 * g + k];
    is1[k] = invstd1[8 * g + k];
    mu2[k] = mean2[8 * g + k];
    is2[k] = invstd2[8 * g + k];
    dummy[k] = 0.f;
  }
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float q2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * rpb;
  const int64_t hi = lo + rpb < M ? lo + rpb : M;
  for (int64_t r = lo + threadIdx.x / tpr; r < hi; r += rpi) {
    float a[8], b[8], dz[8];
    ld8(x1 + r * C + 8 * g, a);
    ld8(x2 + r * C + 8 * g, b);
    load_dz<RM_MASK, DY2>(dy, dy2, mask, r, C, g, a, dummy, dummy, dz);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[k] += dz[k];
      q1[k] = fmaf(dz[k], (a[k] - mu1[k]) * is1[k], q1[k]);
      q2[k] = fmaf(dz[k], (b[k] - mu2[k]) * is2[k], q2[k]);
    }
  }
  block_partial(s, q1, tpr, C, part1);
  __syncthreads();   // block_partial's LDS is reused
  block_partial(s, q2, tpr, C, part2);
}

template <bool DY2>
__global__ __launch_bounds__(kBT) void bn_bwd_apply2_kernel(const bf16* __restrict__ dy,
                                                           const bf16* __restrict__ dy2,
                                                           const bf16* __restrict__ x1,
                                                           const bf16* __restrict__ x2,
                                                           const uint8_t* __restrict__ mask,
                                                           bf16* __restrict__ dx1,
                                                           bf16* __restrict__ dx2, int64_t M, int C,
                                                           const float* __restrict__ mean1,
                                                           const float* __restrict__ invstd1,
                                                           const bf16* __restrict__ gamma1,
                                                           const float* __restrict__ mean2,
                                                           const float* __restrict__ invstd2,
                                                           const bf16* __restrict__ gamma2,
                                                           const float* __restrict__ sdz,
                                                           const float* __restrict__ sdzx1,
                                                           const float* __restrict__ sdzx2) {
  const int tpr = C / 8;
  const int g = threadIdx.x % tpr;
  const float invM = 1.0f / static_cast<float>(M);
  float g1[8], g2[8], mu1[8], is1[8], mu2[8], is2[8], c1[8], c2[8], av[8], b1[8], b2[8], dummy[8];
  ld8(gamma1 + 8 * g, g1);
  ld8(gamma2 + 8 * g, g2);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu1[k] = mean1[8 * g + k];
    is1[k] = invstd1[8 * g + k];
    mu2[k] = mean2[8 * g + k];
    is2[k] = invstd2[8 * g + k];
    c1[k] = g1[k] * is1[k];
    c2[k] = g2[k] * is2[k];
    av[k] = sdz[8 * g + k] * invM;
    b1[k] = sdzx1[8 * g + k] * invM;
    b2[k] = sdzx2[8 * g + k] * invM;
    dummy[k] = 0.f;
  }
  const int64_t rstride = static_cast<int64_t>(gridDim.x) * (kBT / tpr);
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kBT / tpr) + threadIdx.x / tpr; r < M;
       r += rstride) {
    float a[8], b[8], dz[8], o1[8], o2[8];
    ld8(x1 + r * C + 8 * g, a);
    ld8(x2 + r * C + 8 * g, b);
    load_dz<RM_MASK, DY2>(dy, dy2, mask, r, C, g, a, dummy, dummy, dz);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d0 = dz[k] - av[k];
      o1[k] = c1[k] * (d0 - (a[k] - mu1[k]) * is1[k] * b1[k]);
      o2[k] = c2[k] * (d0 - (b[k] - mu2[k]) * is2[k] * b2[k]);
    }
    store_bf16<8>(dx1 + r * C + 8 * g, o1);
    store_bf16<8>(dx2 + r * C + 8 * g, o2);
  }
}

// CML_BN_GRID_CAP: the most workgroups an apply pass launches (default 2048: grid-stride loops
// with two rows in flight; 0 = no cap, one row iteration per workgroup). A/B switch.
int apply_cap() {
  static const int v = [] {
    const char* e = getenv("CML_BN_GRID_CAP");
    return e ? atoi(e) : 2048;
  }();
  return v;
}

int apply_grid(int64_t M, int C) {
  const int rpi = kBT / (C / 8);
  int64_t b = (M + rpi - 1) / rpi;
  const int cap = apply_cap();
  if (cap > 0 && b > cap) b = cap;
  if (b > (1LL << 30)) b = 1LL << 30;
  return static_cast<int>(b < 1 ? 1 : b);
}

}  // namespace

size_t bn_workspace_bytes(int64_t M, int C) {
  const BNGeom g = geom(M, C);
  return static_cast<size_t>(g.nb) * 2 * C * sizeof(float);
}

hipError_t launch_bn_fwd(const void* x, const void* res, void* y, void* mask, int64_t M, int C,
                         const void* gamma, const void* beta, float* mean, float* invstd,
                         float* rmean, float* rvar, float eps, float momentum, int relu,
                         int training, void* work, hipStream_t st) {
  bn_nt_init();
  if (C % 8 != 0 || C / 8 > kBT || (kBT % (C / 8)) != 0 || M < 1) return hipErrorInvalidValue;
  if (mask && !(res && relu)) return hipErrorInvalidValue;
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
  uint8_t* mk = reinterpret_cast<uint8_t*>(mask);
  const bf16* gm = reinterpret_cast<const bf16*>(gamma);
  const bf16* bt = reinterpret_cast<const bf16*>(beta);
  if (mask) bn_apply_kernel<true, true, true><<<ga, kBT, 0, st>>>(xb, rb, yb, mk, M, C, mean, invstd, gm, bt);
  else if (res && relu) bn_apply_kernel<true, true, false><<<ga, kBT, 0, st>>>(xb, rb, yb, mk, M, C, mean, invstd, gm, bt);
  else if (res) bn_apply_kernel<true, false, false><<<ga, kBT, 0, st>>>(xb, rb, yb, mk, M, C, mean, invstd, gm, bt);
  else if (relu) bn_apply_kernel<false, true, false><<<ga, kBT, 0, st>>>(xb, rb, yb, mk, M, C, mean, invstd, gm, bt);
  else bn_apply_kernel<false, false, false><<<ga, kBT, 0, st>>>(xb, rb, yb, mk, M, C, mean, invstd, gm, bt);
  return hipGetLastError();
}

namespace {
template <int RM, bool DRES, bool DY2>
void bwd_t(const bf16* d, const bf16* d2, const bf16* xb, const uint8_t* mk, bf16* dxb, bf16* drb,
           int64_t M, int C, const bf16* gm, const bf16* bt, const float* mean, const float* invstd,
           bf16* dgamma, bf16* dbeta, float* sdz, float* sdzx, float* part, hipStream_t st) {
  const BNGeom g = geom(M, C);
  bn_bwd_reduce_kernel<RM, DY2><<<g.nb, kBT, 0, st>>>(d, d2, xb, mk, M, C, g.rpb, mean, invstd, gm,
                                                       bt, part);
  bn_bwd_finalize_kernel<<<(C + kFC - 1) / kFC, kBT, 0, st>>>(part, g.nb, C, sdz, sdzx, dgamma,
                                                              dbeta);
  if (dxb == nullptr) return;          // sums only (the consumer applies the backward itself)
  bn_bwd_apply_kernel<RM, DRES, DY2><<<apply_grid(M, C), kBT, 0, st>>>(
      d, d2, xb, mk, dxb, drb, M, C, mean, invstd, gm, bt, sdz, sdzx);
}

template <bool DY2>
hipError_t bwd_dispatch(int rm, bool dres, const bf16* d, const bf16* d2, const bf16* xb,
                        const uint8_t* mk, bf16* dxb, bf16* drb, int64_t M, int C, const bf16* gm,
                        const bf16* bt, const float* mean, const float* invstd, bf16* dg, bf16* db,
                        float* sdz, float* sdzx, float* part, hipStream_t st) {
#define CML_BWD(RMV, DR) bwd_t<RMV, DR, DY2>(d, d2, xb, mk, dxb, drb, M, C, gm, bt, mean, invstd, dg, db, sdz, sdzx, part, st)
  if (rm == RM_MASK && dres) CML_BWD(RM_MASK, true);
  else if (rm == RM_MASK) CML_BWD(RM_MASK, false);
  else if (rm == RM_RECOMP && !dres) CML_BWD(RM_RECOMP, false);
  else if (rm == RM_NONE && dres) CML_BWD(RM_NONE, true);
  else if (rm == RM_NONE) CML_BWD(RM_NONE, false);
  else return hipErrorInvalidValue;   // ReLU with a residual needs the forward's mask
#undef CML_BWD
  return hipSuccess;
}
}  // namespace

hipError_t launch_bn_bwd(const void* dy, const void* dy2, const void* x, const void* mask,
                         void* dx, void* dres, int64_t M, int C, const void* gamma,
                         const void* beta, const float* mean, const float* invstd, void* dgamma,
                         void* dbeta, float* sdz, float* sdzx, int relu, void* work,
                         hipStream_t st) {
  bn_nt_init();
  if (C % 8 != 0 || C / 8 > kBT || (kBT % (C / 8)) != 0 || M < 1) return hipErrorInvalidValue;
  const int rm = !relu ? RM_NONE : (mask ? RM_MASK : RM_RECOMP);
  const bf16* d = reinterpret_cast<const bf16*>(dy);
  const bf16* d2 = reinterpret_cast<const bf16*>(dy2);
  const bf16* xb = reinterpret_cast<const bf16*>(x);
  const uint8_t* mk = reinterpret_cast<const uint8_t*>(mask);
  const bf16* gm = reinterpret_cast<const bf16*>(gamma);
  const bf16* bt = reinterpret_cast<const bf16*>(beta);
  bf16* dxb = reinterpret_cast<bf16*>(dx);
  bf16* drb = reinterpret_cast<bf16*>(dres);
  float* part = reinterpret_cast<float*>(work);
  hipError_t e = dy2 ? bwd_dispatch<true>(rm, drb != nullptr, d, d2, xb, mk, dxb, drb, M, C, gm, bt,
                                           mean, invstd, reinterpret_cast<bf16*>(dgamma),
                                           reinterpret_cast<bf16*>(dbeta), sdz, sdzx, part, st)
                     : bwd_dispatch<false>(rm, drb != nullptr, d, d2, xb, mk, dxb, drb, M, C, gm, bt,
                                           mean, invstd, reinterpret_cast<bf16*>(dgamma),
                                           reinterpret_cast<bf16*>(dbeta), sdz, sdzx, part, st);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

namespace {
// sc = gamma invstd, bi = beta - mean sc per channel: the BN affine the fused conv prologues /
// epilogues take (one launch instead of PyTorch's five small ones; rounded exactly as those:
// separate fp32 multiply and subtract, no contraction)
__global__ __launch_bounds__(256) void bn_affine_kernel(const uint16_t* __restrict__ gamma,
                                                        const uint16_t* __restrict__ beta,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, int C,
                                                        float* __restrict__ sc,
                                                        float* __restrict__ bi) {
#pragma clang fp contract(off)
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  // (plain operators under contract(off): the __f*_rn helpers are inlined with contraction on)
  const float s = __uint_as_float(static_cast<uint32_t>(gamma[c]) << 16) * invstd[c];
  sc[c] = s;
  const float ms = mean[c] * s;
  bi[c] = __uint_as_float(static_cast<uint32_t>(beta[c]) << 16) - ms;
}
}  // namespace

hipError_t launch_bn_affine(const void* gamma, const void* beta, const float* mean,
                            const float* invstd, int C, float* sc, float* bi, hipStream_t st) {
  bn_nt_init();
  if (C < 1) return hipErrorInvalidValue;
  bn_affine_kernel<<<(C + 255) / 256, 256, 0, st>>>(reinterpret_cast<const uint16_t*>(gamma),
                                                   reinterpret_cast<const uint16_t*>(beta), mean,
                                                   invstd, C, sc, bi);
  return hipGetLastError();
}

hipError_t launch_bn_bwd_apply(const void* dy, const void* x, void* dx, int64_t M, int C,
                               const void* gamma, const void* beta, const float* mean,
                               const float* invstd, const float* sdz, const float* sdzx,
                               hipStream_t st) {
  bn_nt_init();
  if (C % 8 != 0 || C / 8 > kBT || (kBT % (C / 8)) != 0 || M < 1) return hipErrorInvalidValue;
  bn_bwd_apply_kernel<RM_RECOMP, false, false><<<apply_grid(M, C), kBT, 0, st>>>(
      reinterpret_cast<const bf16*>(dy), nullptr, reinterpret_cast<const bf16*>(x), nullptr,
      reinterpret_cast<bf16*>(dx), nullptr, M, C, mean, invstd,
      reinterpret_cast<const bf16*>(gamma), reinterpret_cast<const bf16*>(beta), sdz, sdzx);
  return hipGetLastError();
}

hipError_t launch_bn_fwd2(const void* x1, const void* x2, void* y, void* mask, int64_t M, int C,
                          const void* gamma1, const void* beta1, const void* gamma2,
                          const void* beta2, float* mean1, float* invstd1, float* mean2,
                          float* invstd2, float* rmean1, float* rvar1, float* rmean2,
                          float* rvar2, float eps, float momentum, int training, void* work,
                          hipStream_t st) {
  bn_nt_init();
  if (C % 8 != 0 || C / 8 > kBT || (kBT % (C / 8)) != 0 || M < 1) return hipErrorInvalidValue;
  const bf16* a = reinterpret_cast<const bf16*>(x1);
  const bf16* b = reinterpret_cast<const bf16*>(x2);
  if (training) {
    const BNGeom g = geom(M, C);
    float* part = reinterpret_cast<float*>(work);
    bn_stats_kernel<<<g.nb, kBT, 0, st>>>(a, M, C, g.rpb, part);
    bn_finalize_kernel<<<(C + kFC - 1) / kFC, kBT, 0, st>>>(part, g.nb, a, M, C, eps, momentum,
                                                            mean1, invstd1, rmean1, rvar1);
    bn_stats_kernel<<<g.nb, kBT, 0, st>>>(b, M, C, g.rpb, part);
    bn_finalize_kernel<<<(C + kFC - 1) / kFC, kBT, 0, st>>>(part, g.nb, b, M, C, eps, momentum,
                                                            mean2, invstd2, rmean2, rvar2);
  }
  const int ga = apply_grid(M, C);
  auto* yb = reinterpret_cast<bf16*>(y);
  auto* mk = reinterpret_cast<uint8_t*>(mask);
  auto* g1 = reinterpret_cast<const bf16*>(gamma1);
  auto* b1 = reinterpret_cast<const bf16*>(beta1);
  auto* g2 = reinterpret_cast<const bf16*>(gamma2);
  auto* b2 = reinterpret_cast<const bf16*>(beta2);
  if (mask) bn_apply2_kernel<true><<<ga, kBT, 0, st>>>(a, b, yb, mk, M, C, mean1, invstd1, g1, b1, mean2, invstd2, g2, b2);
  else bn_apply2_kernel<false><<<ga, kBT, 0, st>>>(a, b, yb, mk, M, C, mean1, invstd1, g1, b1, mean2, invstd2, g2, b2);
  return hipGetLastError();
}

size_t bn2_workspace_bytes(int64_t M, int C) { return 2 * bn_workspace_bytes(M, C); }

hipError_t launch_bn_bwd2(const void* dy, const void* dy2, const void* x1, const void* x2,
                          const void* mask, void* dx1, void* dx2, int64_t M, int C,
                          const void* gamma1, const void* gamma2, const float* mean1,
                          const float* invstd1, const float* mean2, const float* invstd2,
                          void* dgamma1, void* dbeta1, void* dgamma2, void* dbeta2, float* sdz,
                          float* sdzx1, float* sdz_b, float* sdzx2, void* work, hipStream_t st) {
  bn_nt_init();
  if (C % 8 != 0 || C / 8 > kBT || (kBT % (C / 8)) != 0 || M < 1 || !mask) return hipErrorInvalidValue;
  const BNGeom g = geom(M, C);
  float* part1 = reinterpret_cast<float*>(work);
  float* part2 = part1 + static_cast<int64_t>(g.nb) * 2 * C;
  auto* d = reinterpret_cast<const bf16*>(dy);
  auto* d2 = reinterpret_cast<const bf16*>(dy2);
  auto* a = reinterpret_cast<const bf16*>(x1);
  auto* b = reinterpret_cast<const bf16*>(x2);
  auto* mk = reinterpret_cast<const uint8_t*>(mask);
  if (dy2) bn_bwd_reduce2_kernel<true><<<g.nb, kBT, 0, st>>>(d, d2, a, b, mk, M, C, g.rpb, mean1, invstd1, mean2, invstd2, part1, part2);
  else bn_bwd_reduce2_kernel<false><<<g.nb, kBT, 0, st>>>(d, d2, a, b, mk, M, C, g.rpb, mean1, invstd1, mean2, invstd2, part1, part2);
  bn_bwd_finalize_kernel<<<(C + kFC - 1) / kFC, kBT, 0, st>>>(part1, g.nb, C, sdz, sdzx1,
                                                              reinterpret_cast<bf16*>(dgamma1),
                                                              reinterpret_cast<bf16*>(dbeta1));
  bn_bwd_finalize_kernel<<<(C + kFC - 1) / kFC, kBT, 0, st>>>(part2, g.nb, C, sdz_b, sdzx2,
                                                              reinterpret_cast<bf16*>(dgamma2),
                                                              reinterpret_cast<bf16*>(dbeta2));
  auto* o1 = reinterpret_cast<bf16*>(dx1);
  auto* o2 = reinterpret_cast<bf16*>(dx2);
  auto* g1 = reinterpret_cast<const bf16*>(gamma1);
  auto* g2 = reinterpret_cast<const bf16*>(gamma2);
  const int ga = apply_grid(M, C);
  if (dy2) bn_bwd_apply2_kernel<true><<<ga, kBT, 0, st>>>(d, d2, a, b, mk, o1, o2, M, C, mean1, invstd1, g1, mean2, invstd2, g2, sdz, sdzx1, sdzx2);
  else bn_bwd_apply2_kernel<false><<<ga, kBT, 0, st>>>(d, d2, a, b, mk, o1, o2, M, C, mean1, invstd1, g1, mean2, invstd2, g2, sdz, sdzx1, sdzx2);
  return hipGetLastError();
}

// Training statistics only (stats + finalize), for consumers that apply the affine themselves.
hipError_t launch_bn_stats(const void* x, int64_t M, int C, float* mean, float* invstd,
                           float* rmean, float* rvar, float eps, float momentum, void* work,
                           hipStream_t st) {
  bn_nt_init();
  if (C % 8 != 0 || C / 8 > kBT || (kBT % (C / 8)) != 0 || M < 1) return hipErrorInvalidValue;
  const bf16* xb = reinterpret_cast<const bf16*>(x);
  const BNGeom g = geom(M, C);
  float* part = reinterpret_cast<float*>(work);
  bn_stats_kernel<<<g.nb, kBT, 0, st>>>(xb, M, C, g.rpb, part);
  bn_finalize_kernel<<<(C + kFC - 1) / kFC, kBT, 0, st>>>(part, g.nb, xb, M, C, eps, momentum,
                                                          mean, invstd, rmean, rvar);
  return hipGetLastError();
}

}  // namespace cml
