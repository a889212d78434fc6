// Small-matrix algebra of the recompute tails' backward (ops/conv.py _RecomputeTailFn /
// _RecomputeDownTailFn) in two launches instead of ~17 PyTorch kernels per tail.
//
// With u = m * g (the block-output gradient through bn3's ReLU mask), the conv3 weights
// W [Co][p] and the tail input y2 (p channels):
//   P = u^T y2 [Co][p], s = sum u [Co]        (wgrad1x1_ex, given)
//   Gram = y2^T y2 [p][p], cy = sum y2 [p]     (given)
//   q = invstd (rowsum(W * P) - mean s)         bn3's second backward sum
//   a, b, c: bn3's backward coefficients        dz3 = a u + b z3 + c  (bn_bwd_coeffs' formulas)
//   dW = diag(a) P + diag(b) W Gram + c cy^T    conv3's weight gradient (bf16)
//   G = W^T diag(b) W [p][p]                    (symmetric)
//   w_cat = [W^T diag(a) | G] (bf16 [p][Co + p]), bias = W^T c [p]
//        so that dy2 = [(m ? g : 0) | y2] w_cat^T + bias  (conv1x1_cat with the folded affine)
//
// Three launches: tail_coeffs_kernel (one wave per channel: q needs a row reduction, then the
// coefficients), tail_mats_kernel (dW tiles, split-K partials of G, w_cat's transposed first part
// and bias partials; fp32 FMA from LDS -- the products are 1-70 MFLOP, far below what an MFMA tile
// pipeline needs to pay for, so the work is spread over many small workgroups instead), and
// tail_fin_kernel (sums the partials into w_cat's second part and bias).
#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

__global__ __launch_bounds__(256) void tail_coeffs_kernel(
    const uint16_t* __restrict__ W, const float* __restrict__ P, const float* __restrict__ s,
    const uint16_t* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ invstd, int Co, int p, float invM, float* __restrict__ coef,
    uint16_t* __restrict__ dgamma, uint16_t* __restrict__ dbeta) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= Co) return;
  float acc = 0.f;
  for (int k = lane; k < p; k += 64)
    acc = fmaf(bf2f(W[static_cast<int64_t>(c) * p + k]), P[static_cast<int64_t>(c) * p + k], acc);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane != 0) return;
  const float is = invstd[c], mu = mean[c], sd = s[c];
  const float q = (acc - mu * sd) * is;
  const float sc = is * bf2f(gamma[c]);
  const float b = -sc * is * q * invM;
  coef[c] = sc;                          // a
  coef[Co + c] = b;                      // b
  coef[2 * Co + c] = -sc * sd * invM - b * mu;   // c
  dgamma[c] = f2bf(q);
  dbeta[c] = f2bf(sd);
}

// roles by blockIdx.x (every operand tile staged through LDS by coalesced loads that are all in
// flight together; round 3's first version read them straight from L2 in long dependent loops,
// ~55 us per tail):
//   [0, nD)            dW tiles of 32 (c) x 64 (k), the j = 0 .. p reduction in chunks of 64
//   [nD, nD + nG)      G partials: 32 (k) x 64 (i) tiles x KS = Co / 64 slices of c -> gp slab
//   [nD + nG, ...)     64 (k) x 64 (c) tiles of w_cat's first part, W^T diag(a) (transposed through
//                      LDS: coalesced reads and writes), and bias partials over the tile's c -> bp
// Thread layout of a 32 x 64 tile: row tid / 8, 8 consecutive columns 8 (tid % 8).
__global__ __launch_bounds__(256) void tail_mats_kernel(
    const uint16_t* __restrict__ W, const float* __restrict__ P, const float* __restrict__ gram,
    const float* __restrict__ cy, const float* __restrict__ coef, int Co, int p, int nD, int nG,
    uint16_t* __restrict__ dW, uint16_t* __restrict__ wcat, float* __restrict__ gp,
    float* __restrict__ bp) {
  __shared__ float sa[64 * 65];   // dW: W chunk [32][65]; G: b W [64 c][32 k]; T: W tile [64][65]
  __shared__ float sb[64 * 64];   // dW: Gram chunk [64 j][64 k]; G: W [64 c][64 i]
  const int tid = threadIdx.x, b = blockIdx.x;
  const float* ca = coef;
  const float* cb = coef + Co;
  const float* cc = coef + 2 * Co;
  const int tk = p / 64;
  const int r = tid >> 3, c8 = 8 * (tid & 7);
  auto unpack8 = [](uint4 u, float* d) {
    const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      d[2 * q] = __uint_as_float(w4[q] << 16);
      d[2 * q + 1] = __uint_as_float(w4[q] & 0xffff0000u);
    }
  };
  if (b < nD) {
    // dW[c][k] = a_c P[c][k] + b_c sum_j W[c][j] Gram[j][k] + c_c cy[k]
    const int c0 = (b / tk) * 32, k0 = (b % tk) * 64;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int jc = 0; jc < p; jc += 64) {
      {   // W[c0 + r][jc + c8 .. + 8] and Gram rows jc + tid / 4 .. (4 float4 per thread)
        float d[8];
        unpack8(*reinterpret_cast<const uint4*>(W + static_cast<int64_t>(c0 + r) * p + jc + c8), d);
#pragma unroll
        for (int e = 0; e < 8; ++e) sa[r * 65 + c8 + e] = d[e];
        float4 g[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int idx = tid + 256 * e, row = idx >> 4, col = 4 * (idx & 15);
          g[e] = *reinterpret_cast<const float4*>(gram + static_cast<int64_t>(jc + row) * p + k0 + col);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int idx = tid + 256 * e, row = idx >> 4, col = 4 * (idx & 15);
          *reinterpret_cast<float4*>(sb + row * 64 + col) = g[e];
        }
      }
      __syncthreads();
#pragma unroll 8
      for (int jj = 0; jj < 64; ++jj) {
        const float wj = sa[r * 65 + jj];
        const float4 g0 = *reinterpret_cast<const float4*>(sb + jj * 64 + c8);
        const float4 g1 = *reinterpret_cast<const float4*>(sb + jj * 64 + c8 + 4);
        acc[0] = fmaf(wj, g0.x, acc[0]); acc[1] = fmaf(wj, g0.y, acc[1]);
        acc[2] = fmaf(wj, g0.z, acc[2]); acc[3] = fmaf(wj, g0.w, acc[3]);
        acc[4] = fmaf(wj, g1.x, acc[4]); acc[5] = fmaf(wj, g1.y, acc[5]);
        acc[6] = fmaf(wj, g1.z, acc[6]); acc[7] = fmaf(wj, g1.w, acc[7]);
      }
      __syncthreads();
    }
    const int c = c0 + r, k = k0 + c8;
    const float a = ca[c], bc = cb[c], cv = cc[c];
    const float* pr = P + static_cast<int64_t>(c) * p + k;
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaf(cv, cy[k + i], fmaf(bc, acc[i], a * pr[i]));
    *reinterpret_cast<uint4*>(dW + static_cast<int64_t>(c) * p + k) =
        make_uint4(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7]));
    return;
  }
  if (b < nD + nG) {
    // partial G[k][i] = sum_{c in slice} (b_c W[c][k]) W[c][i]
    const int KS = Co / 64, bb = b - nD, t = bb / KS, ks = bb - t * KS;
    const int k0 = (t / tk) * 32, i0 = (t % tk) * 64, cs = ks * 64;
    {   // sa[c][k] = b_c W[cs + c][k0 + k]: 64 rows x 32 -> one uint4 per thread
      const int row = tid >> 2, col = 8 * (tid & 3);
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(W + static_cast<int64_t>(cs + row) * p + k0 + col), d);
      const float bv = cb[cs + row];
#pragma unroll
      for (int e = 0; e < 8; ++e) sa[row * 32 + col + e] = d[e] * bv;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // sb[c][i] = W[cs + c][i0 + i]: 64 x 64, two uint4 per thread
      const int idx = tid + 256 * h, row = idx >> 3, col = 8 * (idx & 7);
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(W + static_cast<int64_t>(cs + row) * p + i0 + col), d);
#pragma unroll
      for (int e = 0; e < 8; ++e) sb[row * 64 + col + e] = d[e];
    }
    __syncthreads();
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int c = 0; c < 64; ++c) {
      const float a = sa[c * 32 + r];
      const float4 w0 = *reinterpret_cast<const float4*>(sb + c * 64 + c8);
      const float4 w1 = *reinterpret_cast<const float4*>(sb + c * 64 + c8 + 4);
      acc[0] = fmaf(a, w0.x, acc[0]); acc[1] = fmaf(a, w0.y, acc[1]);
      acc[2] = fmaf(a, w0.z, acc[2]); acc[3] = fmaf(a, w0.w, acc[3]);
      acc[4] = fmaf(a, w1.x, acc[4]); acc[5] = fmaf(a, w1.y, acc[5]);
      acc[6] = fmaf(a, w1.z, acc[6]); acc[7] = fmaf(a, w1.w, acc[7]);
    }
    float* o = gp + (static_cast<int64_t>(ks) * p + k0 + r) * p + i0 + c8;
    *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    return;
  }
  // w_cat[k][c] = W[c][k] a_c over a 64 (k) x 64 (c) tile, and bp[c-tile][k] = sum_c W[c][k] c_c
  const int t = b - nD - nG, k0 = (t % tk) * 64, ct = t / tk, c0 = ct * 64;
  const int64_t ldc = static_cast<int64_t>(Co) + p;   // w_cat row length
#pragma unroll
  for (int h = 0; h < 2; ++h) {   // sa[c][k] = W[c0 + c][k0 + k] (row stride 65)
    const int idx = tid + 256 * h, row = idx >> 3, col = 8 * (idx & 7);
    float d[8];
    unpack8(*reinterpret_cast<const uint4*>(W + static_cast<int64_t>(c0 + row) * p + k0 + col), d);
#pragma unroll
    for (int e = 0; e < 8; ++e) sa[row * 65 + col + e] = d[e];
  }
  __syncthreads();
  const int c = tid & 63;
  const float av = ca[c0 + c];
#pragma unroll 4
  for (int kk = tid >> 6; kk < 64; kk += 4)
    wcat[(k0 + kk) * ldc + c0 + c] = f2bf(sa[c * 65 + kk] * av);
  if (tid < 64) {
    float s = 0.f;
#pragma unroll 8
    for (int cc2 = 0; cc2 < 64; ++cc2) s = fmaf(sa[cc2 * 65 + tid], cc[c0 + cc2], s);
    bp[static_cast<int64_t>(ct) * p + k0 + tid] = s;
  }
}

// G = sum of the KS partial slabs -> w_cat[k][Co + i] (bf16), bias[k] = sum of the Co / 64 partials
__global__ __launch_bounds__(256) void tail_fin_kernel(const float* __restrict__ gp,
                                                       const float* __restrict__ bp, int Co, int p,
                                                       uint16_t* __restrict__ wcat,
                                                       float* __restrict__ bias) {
  const int KS = Co / 64;
  const int64_t e = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;   // 4 of p * p
  const int64_t pp = static_cast<int64_t>(p) * p;
  if (e < pp) {
    float4 s = *reinterpret_cast<const float4*>(gp + e);
    for (int ks = 1; ks < KS; ++ks) {
      const float4 v = *reinterpret_cast<const float4*>(gp + ks * pp + e);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const int k = static_cast<int>(e / p), i = static_cast<int>(e - static_cast<int64_t>(k) * p);
    *reinterpret_cast<uint2*>(wcat + static_cast<int64_t>(k) * (Co + p) + Co + i) =
        make_uint2(pk_bf16(s.x, s.y), pk_bf16(s.z, s.w));
  }
  if (blockIdx.x == 0) {
    for (int k = threadIdx.x; k < p; k += 256) {
      float s = 0.f;
      for (int ct = 0; ct < KS; ++ct) s += bp[static_cast<int64_t>(ct) * p + k];
      bias[k] = s;
    }
  }
}

// 8 consecutive outputs of a row per thread (k1, k2 multiples of 8)
__global__ __launch_bounds__(256) void scaled_cat_bias_kernel(
    const uint16_t* __restrict__ w1, const float* __restrict__ s1, int k1,
    const uint16_t* __restrict__ w2, const float* __restrict__ s2, int k2,
    const float* __restrict__ b1, const float* __restrict__ b2, int Co,
    uint16_t* __restrict__ out, float* __restrict__ bias) {
  const int cpr = (k1 + k2) / 8;
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= static_cast<int64_t>(Co) * cpr) return;
  const int r = static_cast<int>(e / cpr), c = static_cast<int>(e - static_cast<int64_t>(r) * cpr) * 8;
  const bool first = c < k1;
  const uint4 u = first ? *reinterpret_cast<const uint4*>(w1 + static_cast<int64_t>(r) * k1 + c)
                        : *reinterpret_cast<const uint4*>(w2 + static_cast<int64_t>(r) * k2 + c - k1);
  const float sv = first ? s1[r] : s2[r];
  const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    o[q] = pk_bf16(__uint_as_float(w4[q] << 16) * sv, __uint_as_float(w4[q] & 0xffff0000u) * sv);
  *reinterpret_cast<uint4*>(out + static_cast<int64_t>(r) * (k1 + k2) + c) =
      make_uint4(o[0], o[1], o[2], o[3]);
  if (c == 0) bias[r] = b1[r] + b2[r];
}
}  // namespace

hipError_t launch_scaled_cat_bias(const void* w1, const float* s1, int k1, const void* w2,
                                  const float* s2, int k2, const float* b1, const float* b2,
                                  int Co, void* out, float* bias, hipStream_t st) {
  if (Co < 1 || k1 < 8 || k2 < 8 || k1 % 8 || k2 % 8) return hipErrorInvalidValue;
  const int64_t n = static_cast<int64_t>(Co) * ((k1 + k2) / 8);
  scaled_cat_bias_kernel<<<static_cast<unsigned>((n + 255) / 256), 256, 0, st>>>(
      reinterpret_cast<const uint16_t*>(w1), s1, k1, reinterpret_cast<const uint16_t*>(w2), s2,
      k2, b1, b2, Co, reinterpret_cast<uint16_t*>(out), bias);
  return hipGetLastError();
}

hipError_t launch_tail_bwd_prep(const void* W, const float* P, const float* s, const float* gram,
                                const float* cy, const void* gamma, const float* mean,
                                const float* invstd, int Co, int p, int64_t M, float* work,
                                void* dW, void* wcat, float* bias, void* dgamma, void* dbeta,
                                hipStream_t st) {
  if (Co < 64 || Co % 64 || p < 64 || p % 64 || M < 1) return hipErrorInvalidValue;
  const uint16_t* w = reinterpret_cast<const uint16_t*>(W);
  float* coef = work;                                            // [3][Co]
  float* gp = work + 3 * Co;                                     // [Co / 64][p][p]
  float* bp = gp + static_cast<size_t>(Co / 64) * p * p;         // [Co / 64][p]
  tail_coeffs_kernel<<<(Co + 3) / 4, 256, 0, st>>>(
      w, P, s, reinterpret_cast<const uint16_t*>(gamma), mean, invstd, Co, p,
      1.0f / static_cast<float>(M), coef, reinterpret_cast<uint16_t*>(dgamma),
      reinterpret_cast<uint16_t*>(dbeta));
  const int tk = p / 64;
  const int nD = dW ? (Co / 32) * tk : 0;
  const int nG = (p / 32) * tk * (Co / 64);
  tail_mats_kernel<<<nD + nG + tk * (Co / 64), 256, 0, st>>>(
      w, P, gram, cy, coef, Co, p, nD, nG, reinterpret_cast<uint16_t*>(dW),
      reinterpret_cast<uint16_t*>(wcat), gp, bp);
  const int64_t pp = static_cast<int64_t>(p) * p;
  tail_fin_kernel<<<static_cast<int>((pp / 4 + 255) / 256), 256, 0, st>>>(
      gp, bp, Co, p, reinterpret_cast<uint16_t*>(wcat), bias);
  return hipGetLastError();
}

size_t tail_bwd_prep_work_floats(int Co, int p) {
  return 3 * static_cast<size_t>(Co) + static_cast<size_t>(Co / 64) * p * (p + 1);
}

}  // namespace cml
