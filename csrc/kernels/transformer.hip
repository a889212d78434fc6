// Transformer hot ops for gfx950 (wave64): fused cross-entropy over bf16 logits, RMSNorm,
// LayerNorm (+ residual add), QKV split + RoPE into the SDPA head-major layout, SwiGLU.
//
// All of these are HBM-bound, so every kernel moves each byte once per pass with 16-B vector
// accesses (8 bf16 per lane) and keeps the row in VGPRs between its reduction and its use:
//   * cross-entropy: forward = ONE read of the bf16 logits (online max / sum-exp per lane, then a
//     block combine) -> per-row logsumexp (4 B/row); backward = one read + one bf16 write of the
//     gradient, scaled by a device-resident grad_output / n_valid (no host sync). PyTorch's path
//     (logits.float() -> log_softmax -> nll, then their backwards) moves ~10 fp32 passes.
//   * RMSNorm / LayerNorm: one wave (D <= 1024) or four waves per row, the whole row held in
//     registers between its reductions (wave shuffles, + one LDS exchange for 4-wave rows) and
//     its use; the backward's dweight / dbias are per-row-group partial rows folded by a
//     fixed-order column kernel (deterministic, no atomics).
//   * RoPE: reads the fused [B, S, (H + 2 KV) hd] projection once and writes q / k rotated and v,
//     each already [B, heads, S, hd] contiguous (the transpose copy is fused away); the backward
//     writes the fused projection gradient in one pass (inverse rotation, v copied).
//   * SwiGLU: silu(a) * b over the fused [M, 2F] gate|up projection, backward in one pass.
#include <math.h>

#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kTB = 256;
constexpr int kWPB = kTB / kWave;   // waves (rows) per workgroup for the row kernels

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

__device__ __forceinline__ void ld8(const bf16* p, float (&o)[8]) { load_vec<bf16, 8>(p, o); }

__device__ __forceinline__ float ldbf(const bf16* p, int64_t i) {
  return bf2f(reinterpret_cast<const uint16_t*>(p)[i]);
}
__device__ __forceinline__ void stbf(bf16* p, int64_t i, float v) {
  reinterpret_cast<uint16_t*>(p)[i] = f2bf(v);
}

// ============================================================================ cross-entropy
// One workgroup per row. The row [e0, e0 + V) of a contiguous [R, V] matrix need not be 16-B
// aligned (V = 30522 for BERT): the aligned interior [ci0, ci1) is read with 16-B loads, the <= 7
// leading / trailing elements with scalar loads, so nothing outside the row is touched.
__device__ __forceinline__ void online_add(float& m, float& s, float v) {
  if (v > m) {
    s = s * __expf(m - v) + 1.f;
    m = v;
  } else {
    s += __expf(v - m);
  }
}

__global__ __launch_bounds__(kTB) void ce_fwd_kernel(const bf16* __restrict__ x, int V,
                                                    int64_t ld,
                                                    const int64_t* __restrict__ labels,
                                                    int64_t ignore, float* __restrict__ lse,
                                                    float* __restrict__ loss) {
  const int64_t r = blockIdx.x;
  const int t = threadIdx.x;
  const int64_t e0 = r * ld;   // row stride ld >= V (a padded logits buffer: ld % 8 == 0)
  const int64_t end = e0 + V;
  int64_t ci0 = (e0 + 7) & ~int64_t(7);
  int64_t ci1 = end & ~int64_t(7);
  if (ci0 > ci1) ci0 = ci1 = end;   // row shorter than one aligned chunk: all scalar
  float m = -INFINITY, s = 0.f;
  // edges (scalar)
  const int nhead = static_cast<int>(ci0 - e0), ntail = static_cast<int>(end - ci1);
  if (t < nhead) online_add(m, s, ldbf(x, e0 + t));
  if (t >= 64 && t - 64 < ntail) online_add(m, s, ldbf(x, ci1 + (t - 64)));
  // interior: 4 chunks of 8 in flight per lane
  constexpr int64_t kStep = static_cast<int64_t>(kTB) * 8;
  for (int64_t c = ci0 + static_cast<int64_t>(t) * 8; c < ci1; c += 4 * kStep) {
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (c + u * kStep < ci1) ld8(x + c + u * kStep, v[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (c + u * kStep < ci1) {
        float cm = v[u][0];
#pragma unroll
        for (int k = 1; k < 8; ++k) cm = fmaxf(cm, v[u][k]);
        if (cm > m) {
          s *= __expf(m - cm);
          m = cm;
        }
        if (m != -INFINITY) {
#pragma unroll
          for (int k = 0; k < 8; ++k) s += __expf(v[u][k] - m);
        }
      }
    }
  }
  // block combine of (m, s)
  __shared__ float sm[kWPB], ss[kWPB];
  const float wm = wave_max(m);
  float sc = (m == -INFINITY) ? 0.f : s * __expf(m - wm);
  sc = wave_sum(sc);
  const int w = t >> 6;
  if ((t & 63) == 0) {
    sm[w] = wm;
    ss[w] = sc;
  }
  __syncthreads();
  if (t == 0) {
    float M = sm[0];
#pragma unroll
    for (int k = 1; k < kWPB; ++k) M = fmaxf(M, sm[k]);
    float S = 0.f;
#pragma unroll
    for (int k = 0; k < kWPB; ++k) S += (sm[k] == -INFINITY) ? 0.f : ss[k] * __expf(sm[k] - M);
    const float L = M + __logf(S);
    lse[r] = L;
    const int64_t lab = labels[r];
    float l = 0.f;
    if (lab != ignore && lab >= 0 && lab < V) l = L - ldbf(x, e0 + lab);
    loss[r] = l;
  }
}

// grad = scale * (softmax(x) - onehot(label)); scale = *scale_ptr (grad_output / n_valid) for
// valid rows, 0 for ignored rows.
__global__ __launch_bounds__(kTB) void ce_bwd_kernel(const bf16* __restrict__ x, int V,
                                                    const int64_t* __restrict__ labels,
                                                    int64_t ignore, const float* __restrict__ lse,
                                                    const float* __restrict__ scale_ptr,
                                                    bf16* __restrict__ g,
                                                    const float* __restrict__ div_ptr) {
  const int64_t r = blockIdx.x;
  const int t = threadIdx.x;
  const int64_t e0 = r * static_cast<int64_t>(V);
  const int64_t end = e0 + V;
  int64_t ci0 = (e0 + 7) & ~int64_t(7);
  int64_t ci1 = end & ~int64_t(7);
  if (ci0 > ci1) ci0 = ci1 = end;
  const int64_t lab = labels[r];
  const bool valid = lab != ignore && lab >= 0 && lab < V;
  const float sc = valid ? (div_ptr ? *scale_ptr / *div_ptr : *scale_ptr) : 0.f;
  const float L = lse[r];
  const int64_t le = valid ? e0 + lab : -1;
  auto one = [&](int64_t e, float v) { return sc * __expf(v - L) - (e == le ? sc : 0.f); };
  const int nhead = static_cast<int>(ci0 - e0), ntail = static_cast<int>(end - ci1);
  if (t < nhead) stbf(g, e0 + t, one(e0 + t, ldbf(x, e0 + t)));
  if (t >= 64 && t - 64 < ntail) {
    const int64_t e = ci1 + (t - 64);
    stbf(g, e, one(e, ldbf(x, e)));
  }
  constexpr int64_t kStep = static_cast<int64_t>(kTB) * 8;
  for (int64_t c = ci0 + static_cast<int64_t>(t) * 8; c < ci1; c += 2 * kStep) {
    float v[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (c + u * kStep < ci1) ld8(x + c + u * kStep, v[u]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t cu = c + u * kStep;
      if (cu < ci1) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = one(cu + k, v[u][k]);
        store_bf16<8>(g + cu, o);
      }
    }
  }
}

// Backward over row-strided logits (ld % 8 == 0, so every row is 16-B aligned) into a gradient
// buffer of the same stride, plus the column sums of the gradient (the logits bias gradient, no
// second read of the R x V gradient): workgroup b owns rows [64 b, 64 b + 64) and sweeps the row
// block column chunk by column chunk (lane: 8 columns), 8 rows of loads in flight, so its 8 column
// sums per chunk accumulate in registers; part[b][c] = sum over its 64 rows (fixed order). Columns
// in [V, ld) of the gradient are written as 0 and contribute 0.
constexpr int kCeRows = 64;
__global__ __launch_bounds__(kTB) void ce_bwd_cs_kernel(const bf16* __restrict__ x, int V, int64_t ld,
                                                       const int64_t* __restrict__ labels,
                                                       int64_t ignore, const float* __restrict__ lse,
                                                       const float* __restrict__ scale_ptr,
                                                       bf16* __restrict__ g, float* __restrict__ part,
                                                       const float* __restrict__ div_ptr) {
  __shared__ float sL[kCeRows], sS[kCeRows];
  __shared__ int sLab[kCeRows];
  const int t = threadIdx.x;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kCeRows;
  if (t < kCeRows) {
    const int64_t lab = labels[r0 + t];
    const bool valid = lab != ignore && lab >= 0 && lab < V;
    sL[t] = lse[r0 + t];
    sS[t] = valid ? (div_ptr ? *scale_ptr / *div_ptr : *scale_ptr) : 0.f;
    sLab[t] = valid ? static_cast<int>(lab) : -1;
  }
  __syncthreads();
  const uint16_t* xr = reinterpret_cast<const uint16_t*>(x) + r0 * ld;
  uint16_t* gr = reinterpret_cast<uint16_t*>(g) + r0 * ld;
  for (int c = 8 * t; c < V; c += 8 * kTB) {
    float cs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cs[k] = 0.f;
    const int nv = V - c < 8 ? V - c : 8;   // valid columns of this chunk
    for (int rb = 0; rb < kCeRows; rb += 8) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const uint4*>(xr + (rb + u) * ld + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rr = rb + u;
        const float L = sL[rr], sc = sS[rr];
        const int lc = sLab[rr] - c;   // label column within the chunk (0..7) or outside
        const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        uint32_t o4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float lo = sc * __expf(__uint_as_float(w4[q] << 16) - L) - (lc == 2 * q ? sc : 0.f);
          float hi = sc * __expf(__uint_as_float(w4[q] & 0xffff0000u) - L) - (lc == 2 * q + 1 ? sc : 0.f);
          if (2 * q >= nv) lo = 0.f;
          if (2 * q + 1 >= nv) hi = 0.f;
          o4[q] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
          cs[2 * q] += __uint_as_float(o4[q] << 16);   // the stored (bf16) values are summed
          cs[2 * q + 1] += __uint_as_float(o4[q] & 0xffff0000u);
        }
        *reinterpret_cast<uint4*>(gr + (rb + u) * ld + c) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
      }
    }
    float* pp = part + static_cast<int64_t>(blockIdx.x) * ld + c;
    reinterpret_cast<float4*>(pp)[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
    reinterpret_cast<float4*>(pp)[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
  }
}

// dh = bf16(da * gelu'(h)) over n elements (n % 8 == 0): the backward of a GELU applied in a GEMM
// epilogue (gemm.hip EP_GELU) whose consumer is not a GEMM (BERT's MLM-head transform -> LayerNorm)
__global__ __launch_bounds__(kTB) void gelu_bwd_kernel(const bf16* __restrict__ da,
                                                      const bf16* __restrict__ h,
                                                      bf16* __restrict__ dh, int64_t n8) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kTB + threadIdx.x; i < n8;
       i += static_cast<int64_t>(gridDim.x) * kTB) {
    const uint4 av = reinterpret_cast<const uint4*>(da)[i];
    const uint4 hv = reinterpret_cast<const uint4*>(h)[i];
    const uint32_t a4[4] = {av.x, av.y, av.z, av.w}, h4[4] = {hv.x, hv.y, hv.z, hv.w};
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float lo = __uint_as_float(a4[q] << 16) * dgelu_f(__uint_as_float(h4[q] << 16));
      const float hi = __uint_as_float(a4[q] & 0xffff0000u) * dgelu_f(__uint_as_float(h4[q] & 0xffff0000u));
      o[q] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
    }
    reinterpret_cast<uint4*>(dh)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// out[s][c] = sum over the nb partial rows of segment s (in order) of part[.][c], c < V
__global__ __launch_bounds__(kTB) void ce_part_fold_kernel(const float* __restrict__ part, int nb,
                                                          int V, int64_t ld, void* __restrict__ out,
                                                          int64_t ldo, int out_f32) {
  const int c = blockIdx.x * kTB + threadIdx.x;
  const int s = blockIdx.y;
  if (c >= V) return;
  const float* p = part + static_cast<int64_t>(s) * nb * ld + c;
  float v = 0.f;
  for (int b = 0; b < nb; ++b) v += p[static_cast<int64_t>(b) * ld];
  if (out_f32) reinterpret_cast<float*>(out)[static_cast<int64_t>(s) * ldo + c] = v;
  else reinterpret_cast<uint16_t*>(out)[static_cast<int64_t>(s) * ldo + c] = f2bf(v);
}

// ============================================================================ RMSNorm / LayerNorm
// WPR waves per row (1 for D <= 1024, 4 above), kWPB / WPR rows per workgroup. Lane l of
// sub-wave u owns the 16-B chunks c = ((i * WPR + u) * 64 + l) * 8, i < NV, so the row sits in
// registers (NV * 8 floats per lane) between its reductions and its use; row reductions are wave
// shuffles plus, for WPR > 1, one LDS exchange.
template <int NV, int WPR>
__device__ __forceinline__ int chunk_col(int i, int sub, int lane) {
  return ((i * WPR + sub) * kWave + lane) * 8;
}

template <int NV, int WPR>
__device__ __forceinline__ void row_load(const bf16* __restrict__ p, int D, int sub, int lane,
                                         float (&v)[NV][8]) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = chunk_col<NV, WPR>(i, sub, lane);
    if (c < D) {
      ld8(p + c, v[i]);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[i][k] = 0.f;
    }
  }
}

template <int NV, int WPR>
__device__ __forceinline__ void row_store(bf16* __restrict__ p, int D, int sub, int lane,
                                          const float (&v)[NV][8]) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = chunk_col<NV, WPR>(i, sub, lane);
    if (c < D) store_bf16<8>(p + c, v[i]);
  }
}

// Sum of (a, b) over the WPR waves of a row (every lane gets the result). `red` holds
// [2 parities][kWPB][2]; the parity alternates per call so one barrier per call suffices.
template <int WPR>
__device__ __forceinline__ void row_sum2(float& a, float& b, float* red, int& parity) {
  a = wave_sum(a);
  b = wave_sum(b);
  if constexpr (WPR > 1) {
    const int w = threadIdx.x >> 6;
    float* r = red + parity * kWPB * 2;
    if ((threadIdx.x & 63) == 0) {
      r[w * 2] = a;
      r[w * 2 + 1] = b;
    }
    __syncthreads();
    const int w0 = w - w % WPR;
    a = 0.f;
    b = 0.f;
#pragma unroll
    for (int k = 0; k < WPR; ++k) {
      a += r[(w0 + k) * 2];
      b += r[(w0 + k) * 2 + 1];
    }
    parity ^= 1;
  }
}

// LN (layer norm, with beta) or RMS (no mean, no beta). RES: y = norm(x + res), and the bf16 sum is
// written to `sum` (the backward's input).
template <int NV, int WPR, bool LN, bool RES>
__global__ __launch_bounds__(kTB) void norm_fwd_kernel(const bf16* __restrict__ x,
                                                      const bf16* __restrict__ res,
                                                      const bf16* __restrict__ w,
                                                      const bf16* __restrict__ b,
                                                      bf16* __restrict__ y, bf16* __restrict__ sum,
                                                      float* __restrict__ mean_out,
                                                      float* __restrict__ rstd_out, int64_t M,
                                                      int D, float eps) {
  __shared__ float red[2 * kWPB * 2];
  int parity = 0;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int sub = wv % WPR;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * (kWPB / WPR) + wv / WPR;
  const bool live = r < M;   // (WPR > 1: whole workgroups agree, the grid is exact)
  if (WPR == 1 && !live) return;
  float v[NV][8];
  row_load<NV, WPR>(x + r * D, D, sub, lane, v);
  if constexpr (RES) {
    float a[NV][8];
    row_load<NV, WPR>(res + r * D, D, sub, lane, a);
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[i][k] = bf2f(f2bf(v[i][k] + a[i][k]));   // the stored sum
    row_store<NV, WPR>(sum + r * D, D, sub, lane, v);
  }
  const float invD = 1.f / static_cast<float>(D);
  float mu = 0.f;
  if constexpr (LN) {
    float s = 0.f, dummy = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[i][k];
    row_sum2<WPR>(s, dummy, red, parity);
    mu = s * invD;
  }
  float q = 0.f, dummy2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (chunk_col<NV, WPR>(i, sub, lane) < D) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[i][k] - mu;
        q = fmaf(d, d, q);
      }
    }
  }
  row_sum2<WPR>(q, dummy2, red, parity);
  const float rs = rsqrtf(q * invD + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = chunk_col<NV, WPR>(i, sub, lane);
    if (c < D) {
      float wt[8], bv[8];
      ld8(w + c, wt);
      if constexpr (LN) ld8(b + c, bv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float o = (v[i][k] - mu) * rs * wt[k];
        if constexpr (LN) o += bv[k];
        v[i][k] = o;
      }
    }
  }
  row_store<NV, WPR>(y + r * D, D, sub, lane, v);
  if (lane == 0 && sub == 0) {
    if constexpr (LN) mean_out[r] = mu;
    rstd_out[r] = rs;
  }
}

// Backward: xh = (x - mu) * rstd, g = dy * w;
//   RMS: dx = rstd * (g - xh * mean(g xh))
//   LN : dx = rstd * (g - mean(g) - xh * mean(g xh))
// Workgroup row groups walk rows r = g, g + ngroups, ... and accumulate dw (and db) partials over
// their rows; partial rows go to part[group][2][D] for the fixed-order column fold.
// DR: a second gradient of the normalised input (the residual stream's own gradient, see
// ops.transformer.add_norm) is added on the way out, replacing an elementwise add pass.
// Segments (batched virtual workers): the M rows are nseg consecutive segments of Ms rows and
// every workgroup works inside one segment (nbs workgroups per segment), so the partial rows of
// segment s are part[s nbs .. (s + 1) nbs) and fold to that worker's own dgamma / dbeta.
template <int NV, int WPR, bool LN, bool DR>
__global__ __launch_bounds__(kTB) void norm_bwd_kernel(const bf16* __restrict__ dy,
                                                      const bf16* __restrict__ dres,
                                                      const bf16* __restrict__ x,
                                                      const bf16* __restrict__ w,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ rstd,
                                                      bf16* __restrict__ dx, int64_t Mtot, int D,
                                                      float* __restrict__ part, int64_t Ms,
                                                      int nbs) {
  __shared__ float red[2 * kWPB * 2];
  int parity = 0;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int sub = wv % WPR;
  constexpr int kRPB = kWPB / WPR;
  const int seg = blockIdx.x / nbs;
  const int64_t r0 = static_cast<int64_t>(seg) * Ms;
  const int64_t M = r0 + Ms < Mtot ? r0 + Ms : Mtot;          // end of this segment's rows
  const int64_t grp = r0 + static_cast<int64_t>(blockIdx.x - seg * nbs) * kRPB + wv / WPR;
  const int ngrp = nbs * kRPB;
  float wt[NV][8];
  row_load<NV, WPR>(w, D, sub, lane, wt);
  float aw[NV][8], ab[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) aw[i][k] = ab[i][k] = 0.f;
  const float invD = 1.f / static_cast<float>(D);
  // rows r = grp, grp + ngrp, ... (WPR > 1: one row per workgroup, uniform trip counts); the next
  // row's x / dy loads are issued before the current row's reductions
  float xv[NV][8], dv[NV][8], ev[NV][8];
  if (grp < M) {
    row_load<NV, WPR>(x + grp * D, D, sub, lane, xv);
    row_load<NV, WPR>(dy + grp * D, D, sub, lane, dv);
    if constexpr (DR) row_load<NV, WPR>(dres + grp * D, D, sub, lane, ev);
  }
  for (int64_t r = grp; r < M; r += ngrp) {
    float xn[NV][8], dn[NV][8], en[NV][8];
    const int64_t rn = r + ngrp;
    if (rn < M) {
      row_load<NV, WPR>(x + rn * D, D, sub, lane, xn);
      row_load<NV, WPR>(dy + rn * D, D, sub, lane, dn);
      if constexpr (DR) row_load<NV, WPR>(dres + rn * D, D, sub, lane, en);
    }
    const float rs = rstd[r];
    const float mu = LN ? mean[r] : 0.f;
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[i][k] - mu) * rs;   // padded slots: x = dy = 0 -> contribute 0
        xv[i][k] = xh;
        const float g = dv[i][k] * wt[i][k];
        sg += g;
        sgx = fmaf(g, xh, sgx);
        aw[i][k] = fmaf(dv[i][k], xh, aw[i][k]);
        if constexpr (LN) ab[i][k] += dv[i][k];
      }
    row_sum2<WPR>(sg, sgx, red, parity);
    const float mgx = sgx * invD;
    const float mg = LN ? sg * invD : 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) dv[i][k] = rs * (dv[i][k] * wt[i][k] - mg - xv[i][k] * mgx);
    if constexpr (DR) {
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) dv[i][k] += ev[i][k];
    }
    row_store<NV, WPR>(dx + r * D, D, sub, lane, dv);
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        xv[i][k] = xn[i][k];
        dv[i][k] = dn[i][k];
        if constexpr (DR) ev[i][k] = en[i][k];
      }
  }
  // one partial row pair per workgroup: part[blockIdx.x][2][D]
  float* pw = part + static_cast<int64_t>(blockIdx.x) * 2 * D;
  if constexpr (WPR == 1) {
    // fold the 4 waves' partials through LDS in a fixed order (D <= 1024 here)
    __shared__ float lw[kWPB][2][1024];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = chunk_col<NV, WPR>(i, sub, lane);
      if (c < D) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          lw[wv][0][c + k] = aw[i][k];
          lw[wv][1][c + k] = ab[i][k];
        }
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += kTB) {
      pw[c] = (lw[0][0][c] + lw[1][0][c]) + (lw[2][0][c] + lw[3][0][c]);
      if constexpr (LN) pw[D + c] = (lw[0][1][c] + lw[1][1][c]) + (lw[2][1][c] + lw[3][1][c]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = chunk_col<NV, WPR>(i, sub, lane);
      if (c < D) {
        store_f32<8>(pw + c, aw[i]);
        if constexpr (LN) store_f32<8>(pw + D + c, ab[i]);
      }
    }
  }
}

// out_h[c] = sum_p part[p * pstride + h * D + c] (h = blockIdx.y), fixed order. A workgroup owns
// 16 columns x 16 partial slices (every lane has <= ceil(np / 16) loads, 4 in flight); the 16
// slice sums are combined through LDS in slice order. Latency, not bandwidth, bounds these folds,
// so they are spread over D / 16 workgroups instead of one thread per column.
// Segments (blockIdx.z): slices [z np, (z + 1) np) fold into out0 / out1 + z ostride.
__global__ __launch_bounds__(kTB) void fold_kernel(const float* __restrict__ part, int np,
                                                  int64_t pstride, int D, bf16* __restrict__ out0,
                                                  bf16* __restrict__ out1, int64_t ostride = 0) {
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  const int h = blockIdx.y;
  const int64_t zs = blockIdx.z;
  const float* src = part + zs * np * pstride + static_cast<int64_t>(h) * D + c;
  const int per = (np + 15) / 16;
  const int p0 = sl * per;
  const int p1 = p0 + per < np ? p0 + per : np;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    int p = p0;
    for (; p + 3 < p1; p += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = src[static_cast<int64_t>(p + u) * pstride];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += v[u];
    }
    for (; p < p1; ++p) a[0] += src[static_cast<int64_t>(p) * pstride];
  }
  __shared__ float red[16][17];
  red[sl][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (threadIdx.x < 16) {
    const int cc = blockIdx.x * 16 + threadIdx.x;
    if (cc < D) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) t += red[k][threadIdx.x];
      stbf((h == 0 ? out0 : out1) + zs * ostride, cc, t);
    }
  }
}

// Row-group geometry: D <= 1024 -> one wave per row (NV = 1 or 2); else 4 waves (NV = 1 or 2).
struct NormGeom {
  int nv, wpr;
};
NormGeom norm_geom(int D) {
  const int ch = D / 8;   // 16-B chunks per row
  if (ch <= kWave) return {1, 1};
  if (ch <= 2 * kWave) return {2, 1};
  if (ch <= 4 * kWave) return {1, 4};
  if (ch <= 8 * kWave) return {2, 4};
  return {0, 0};
}

// backward workgroups (= partial rows): up to 256, i.e. 1024 one-wave or 256 four-wave row groups
int norm_bwd_blocks(int64_t M, int wpr) {
  const int rpb = kWPB / wpr;
  int64_t g = (M + rpb - 1) / rpb;
  if (g > 256) g = 256;
  return static_cast<int>(g < 1 ? 1 : g);
}

// ============================================================================ RoPE + QKV split
// qkv: [B, S, (H + 2 KV) * hd] -> q [B, H, S, hd], k / v [B, KV, S, hd]. Interleaved pairs
// (x[2i], x[2i+1]) rotate by angle (cos, sin)[s, i] (fp32 tables [S, hd/2]); cos == null: no
// rotation (plain split + transpose). One lane per 8 elements (4 pairs) of one head vector.
__global__ __launch_bounds__(kTB) void rope_fwd_kernel(const bf16* __restrict__ qkv,
                                                      const float* __restrict__ cosb,
                                                      const float* __restrict__ sinb,
                                                      bf16* __restrict__ q, bf16* __restrict__ k,
                                                      bf16* __restrict__ v, int B, int S, int H,
                                                      int KV, int hd) {
  const int cph = hd / 8;   // chunks per head vector
  const int heads = H + 2 * KV;
  const int64_t total = static_cast<int64_t>(B) * S * heads * cph;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kTB;
  for (int64_t id = static_cast<int64_t>(blockIdx.x) * kTB + threadIdx.x; id < total; id += stride) {
    const int j = static_cast<int>(id % cph);
    const int64_t t1 = id / cph;
    const int hh = static_cast<int>(t1 % heads);
    const int64_t bs = t1 / heads;   // b * S + s
    const int s = static_cast<int>(bs % S);
    const int b = static_cast<int>(bs / S);
    float e[8];
    ld8(qkv + id * 8, e);
    bf16* dst;
    if (hh < H) {
      dst = q + ((static_cast<int64_t>(b) * H + hh) * S + s) * hd + j * 8;
    } else if (hh < H + KV) {
      dst = k + ((static_cast<int64_t>(b) * KV + (hh - H)) * S + s) * hd + j * 8;
    } else {
      dst = v + ((static_cast<int64_t>(b) * KV + (hh - H - KV)) * S + s) * hd + j * 8;
    }
    if (cosb != nullptr && hh < H + KV) {
      const float* cr = cosb + static_cast<int64_t>(s) * (hd / 2) + j * 4;
      const float* sr = sinb + static_cast<int64_t>(s) * (hd / 2) + j * 4;
      float cv[4], sv[4];
      load_vec<float, 4>(cr, cv);
      load_vec<float, 4>(sr, sv);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float x1 = e[2 * p], x2 = e[2 * p + 1];
        e[2 * p] = x1 * cv[p] - x2 * sv[p];
        e[2 * p + 1] = x1 * sv[p] + x2 * cv[p];
      }
    }
    store_bf16<8>(dst, e);
  }
}

// Inverse: dqkv[b, s, head, :] = R(-theta) dq / dk, dv copied.
__global__ __launch_bounds__(kTB) void rope_bwd_kernel(const bf16* __restrict__ dq,
                                                      const bf16* __restrict__ dk,
                                                      const bf16* __restrict__ dv,
                                                      const float* __restrict__ cosb,
                                                      const float* __restrict__ sinb,
                                                      bf16* __restrict__ dqkv, int B, int S,
                                                      int H, int KV, int hd, int grp) {
  const int cph = hd / 8;
  const int heads = H + 2 * KV;
  const int64_t total = static_cast<int64_t>(B) * S * heads * cph;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kTB;
  for (int64_t id = static_cast<int64_t>(blockIdx.x) * kTB + threadIdx.x; id < total; id += stride) {
    const int j = static_cast<int>(id % cph);
    const int64_t t1 = id / cph;
    const int hh = static_cast<int>(t1 % heads);
    const int64_t bs = t1 / heads;
    const int s = static_cast<int>(bs % S);
    const int b = static_cast<int>(bs / S);
    float e[8];
    if (hh < H) {
      ld8(dq + ((static_cast<int64_t>(b) * H + hh) * S + s) * hd + j * 8, e);
    } else {
      // dk / dv per query head ([B, KV grp, S, hd], grp > 1: the flash-attention backward's
      // per-head gradients): the grp heads of kv head g sum here, in fp32
      const bool isk = hh < H + KV;
      const int g = isk ? hh - H : hh - H - KV;
      const bf16* base = (isk ? dk : dv) +
                         ((static_cast<int64_t>(b) * KV + g) * grp * S + s) * hd + j * 8;
      ld8(base, e);
      for (int x = 1; x < grp; ++x) {
        float f[8];
        ld8(base + static_cast<int64_t>(x) * S * hd, f);
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] += f[i];
      }
    }
    if (cosb != nullptr && hh < H + KV) {
      const float* cr = cosb + static_cast<int64_t>(s) * (hd / 2) + j * 4;
      const float* sr = sinb + static_cast<int64_t>(s) * (hd / 2) + j * 4;
      float cv[4], sv[4];
      load_vec<float, 4>(cr, cv);
      load_vec<float, 4>(sr, sv);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float y1 = e[2 * p], y2 = e[2 * p + 1];
        e[2 * p] = y1 * cv[p] + y2 * sv[p];
        e[2 * p + 1] = -y1 * sv[p] + y2 * cv[p];
      }
    }
    store_bf16<8>(dqkv + id * 8, e);
  }
}

// ============================================================================ SwiGLU
// h: [M, 2F] = [a | b] (gate | up); y = silu(a) * b : [M, F].
__device__ __forceinline__ float sigm(float a) { return 1.f / (1.f + __expf(-a)); }

__global__ __launch_bounds__(kTB) void swiglu_fwd_kernel(const bf16* __restrict__ h,
                                                        bf16* __restrict__ y, int64_t M, int F) {
  const int cpr = F / 8;
  const int64_t total = M * cpr;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kTB;
  for (int64_t id = static_cast<int64_t>(blockIdx.x) * kTB + threadIdx.x; id < total; id += stride) {
    const int64_t r = id / cpr;
    const int c = static_cast<int>(id % cpr) * 8;
    float a[8], b[8];
    ld8(h + r * 2 * F + c, a);
    ld8(h + r * 2 * F + F + c, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = a[k] * sigm(a[k]) * b[k];
    store_bf16<8>(y + r * F + c, a);
  }
}

__global__ __launch_bounds__(kTB) void swiglu_bwd_kernel(const bf16* __restrict__ dy,
                                                        const bf16* __restrict__ h,
                                                        bf16* __restrict__ dh, int64_t M, int F) {
  const int cpr = F / 8;
  const int64_t total = M * cpr;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kTB;
  for (int64_t id = static_cast<int64_t>(blockIdx.x) * kTB + threadIdx.x; id < total; id += stride) {
    const int64_t r = id / cpr;
    const int c = static_cast<int>(id % cpr) * 8;
    float a[8], b[8], d[8];
    ld8(h + r * 2 * F + c, a);
    ld8(h + r * 2 * F + F + c, b);
    ld8(dy + r * F + c, d);
    float da[8], db[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float sg = sigm(a[k]);
      const float si = a[k] * sg;
      db[k] = d[k] * si;
      da[k] = d[k] * b[k] * (sg + si * (1.f - sg));
    }
    store_bf16<8>(dh + r * 2 * F + c, da);
    store_bf16<8>(dh + r * 2 * F + F + c, db);
  }
}

// ============================================================================ bias gradient
// db[c] = sum_r dy[r, c] over a bf16 [M, N] matrix (N % 8 == 0). PyTorch's generic column
// reduction runs these at ~0.4 TB/s; here workgroup (gx, gy) covers 512 columns (one 16-B chunk
// per lane, every row access a dense 1-KiB wave load) of a 16-row slice per wave, the 4 waves are
// combined through LDS, and fold_kernel adds the slices in a fixed order (deterministic).
constexpr int kCSRows = 32;   // rows per workgroup slice (8 per wave)

__global__ __launch_bounds__(kTB) void colsum_partial_kernel(const bf16* __restrict__ dy,
                                                            int64_t M, int N,
                                                            float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.x * kWave + lane) * 8;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kCSRows;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < N) {
    for (int64_t r = r0 + w; r < r0 + kCSRows && r < M; r += kWPB) {
      float v[8];
      ld8(dy + r * N + c, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += v[k];
    }
  }
  __shared__ float red[kWPB][kWave * 8];
#pragma unroll
  for (int k = 0; k < 8; ++k) red[w][lane * 8 + k] = a[k];
  __syncthreads();
  for (int i = threadIdx.x; i < kWave * 8; i += kTB) {
    const int col = blockIdx.x * kWave * 8 + i;
    if (col < N)
      part[static_cast<int64_t>(blockIdx.y) * N + col] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// CML_STREAM_GRID_CAP: the most workgroups of an elementwise launch (default 8192; 0 = no cap)
int stream_grid(int64_t work_items) {
  static const int cap = [] {
    const char* e = getenv("CML_STREAM_GRID_CAP");
    return e ? atoi(e) : 8192;
  }();
  int64_t b = (work_items + kTB - 1) / kTB;
  if (cap > 0 && b > cap) b = cap;
  if (b > (1LL << 30)) b = 1LL << 30;
  return static_cast<int>(b < 1 ? 1 : b);
}

}  // namespace

// ---------------------------------------------------------------------------- host launchers
hipError_t launch_ce_fwd(const void* logits, int64_t R, int V, int64_t ld, const int64_t* labels,
                         int64_t ignore, float* lse, float* loss, hipStream_t st) {
  if (R < 1 || V < 1 || ld < V || (reinterpret_cast<uintptr_t>(logits) & 15)) return hipErrorInvalidValue;
  ce_fwd_kernel<<<static_cast<unsigned>(R), kTB, 0, st>>>(reinterpret_cast<const bf16*>(logits), V,
                                                          ld, labels, ignore, lse, loss);
  return hipGetLastError();
}

hipError_t launch_ce_bwd(const void* logits, int64_t R, int V, const int64_t* labels,
                         int64_t ignore, const float* lse, const float* scale, void* grad,
                         hipStream_t st, const float* div) {
  if (R < 1 || V < 1 || (reinterpret_cast<uintptr_t>(logits) & 15) ||
      (reinterpret_cast<uintptr_t>(grad) & 15))
    return hipErrorInvalidValue;
  ce_bwd_kernel<<<static_cast<unsigned>(R), kTB, 0, st>>>(reinterpret_cast<const bf16*>(logits), V,
                                                          labels, ignore, lse, scale,
                                                          reinterpret_cast<bf16*>(grad), div);
  return hipGetLastError();
}

namespace {
__global__ __launch_bounds__(1024) void ce_mean_kernel(const float* __restrict__ loss,
                                                      const int64_t* __restrict__ labels,
                                                      int64_t R, int64_t ignore,
                                                      float* __restrict__ out,
                                                      float* __restrict__ cnt) {
  __shared__ double ss[1024];
  __shared__ long long sc[1024];
  const int t = threadIdx.x;
  double s = 0.0;
  long long c = 0;
  for (int64_t r = t; r < R; r += 1024) {
    s += static_cast<double>(loss[r]);
    c += labels[r] != ignore ? 1 : 0;
  }
  ss[t] = s;
  sc[t] = c;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (t < o) {
      ss[t] += ss[t + o];
      sc[t] += sc[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    const float n = static_cast<float>(sc[0] > 0 ? sc[0] : 1);
    out[0] = static_cast<float>(ss[0]) / n;
    cnt[0] = n;
  }
}
}  // namespace

hipError_t launch_ce_mean(const float* loss, const int64_t* labels, int64_t R, int64_t ignore,
                          float* out, float* count, hipStream_t st) {
  if (R < 1) return hipErrorInvalidValue;
  ce_mean_kernel<<<1, 1024, 0, st>>>(loss, labels, R, ignore, out, count);
  return hipGetLastError();
}

hipError_t launch_ce_bwd_cs(const void* logits, int64_t R, int V, int64_t ld,
                            const int64_t* labels, int64_t ignore, const float* lse,
                            const float* scale, void* grad, float* part, hipStream_t st,
                            const float* div) {
  if (R < kCeRows || R % kCeRows || V < 1 || ld < V || ld % 8 ||
      ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(grad) |
        reinterpret_cast<uintptr_t>(part)) & 15))
    return hipErrorInvalidValue;
  ce_bwd_cs_kernel<<<static_cast<unsigned>(R / kCeRows), kTB, 0, st>>>(
      reinterpret_cast<const bf16*>(logits), V, ld, labels, ignore, lse, scale,
      reinterpret_cast<bf16*>(grad), part, div);
  return hipGetLastError();
}

hipError_t launch_gelu_bwd(const void* da, const void* h, void* dh, int64_t n, hipStream_t st) {
  if (n < 1 || n % 8 || ((reinterpret_cast<uintptr_t>(da) | reinterpret_cast<uintptr_t>(h) |
                          reinterpret_cast<uintptr_t>(dh)) & 15))
    return hipErrorInvalidValue;
  gelu_bwd_kernel<<<stream_grid(n / 8), kTB, 0, st>>>(reinterpret_cast<const bf16*>(da),
                                                      reinterpret_cast<const bf16*>(h),
                                                      reinterpret_cast<bf16*>(dh), n / 8);
  return hipGetLastError();
}

hipError_t launch_ce_part_fold(const float* part, int64_t R, int V, int64_t ld, int nseg, void* out,
                               int64_t ldo, int out_f32, hipStream_t st) {
  if (nseg < 1 || R % (static_cast<int64_t>(kCeRows) * nseg) || V < 1 || ld < V) return hipErrorInvalidValue;
  const dim3 grid((V + kTB - 1) / kTB, nseg);
  ce_part_fold_kernel<<<grid, kTB, 0, st>>>(part, static_cast<int>(R / kCeRows / nseg), V, ld, out,
                                            ldo, out_f32);
  return hipGetLastError();
}

namespace {
template <int NV, int WPR>
void norm_fwd_t(bool ln, bool resid, const bf16* x, const bf16* res, const bf16* w, const bf16* b,
                bf16* y, bf16* sum, float* mean, float* rstd, int64_t M, int D, float eps,
                hipStream_t st) {
  constexpr int kRPB = kWPB / WPR;
  const unsigned g = static_cast<unsigned>((M + kRPB - 1) / kRPB);
#define CML_NF(L, R) norm_fwd_kernel<NV, WPR, L, R><<<g, kTB, 0, st>>>(x, res, w, b, y, sum, mean, rstd, M, D, eps)
  if (ln && resid) CML_NF(true, true);
  else if (ln) CML_NF(true, false);
  else if (resid) CML_NF(false, true);
  else CML_NF(false, false);
#undef CML_NF
}

template <int NV, int WPR>
void norm_bwd_t(bool ln, const bf16* dy, const bf16* dr, const bf16* x, const bf16* w,
                const float* mean, const float* rstd, bf16* dx, int64_t M, int D, float* part,
                int nblk, hipStream_t st, int64_t Ms, int nseg) {
  const unsigned g = static_cast<unsigned>(nblk) * nseg;
#define CML_NB(L, R) norm_bwd_kernel<NV, WPR, L, R><<<g, kTB, 0, st>>>(dy, dr, x, w, mean, rstd, dx, M, D, part, Ms, nblk)
  if (ln && dr) CML_NB(true, true);
  else if (ln) CML_NB(true, false);
  else if (dr) CML_NB(false, true);
  else CML_NB(false, false);
#undef CML_NB
}
}  // namespace

size_t norm_workspace_bytes(int64_t M, int D) {
  const NormGeom g = norm_geom(D);
  return static_cast<size_t>(norm_bwd_blocks(M, g.wpr < 1 ? 1 : g.wpr)) * 2 * D * sizeof(float);
}

hipError_t launch_norm_fwd(int ln, const void* x, const void* res, const void* w, const void* b,
                           void* y, void* sum, float* mean, float* rstd, int64_t M, int D,
                           float eps, hipStream_t st) {
  const NormGeom g = norm_geom(D);
  if (M < 1 || D % 8 || g.nv == 0 || (ln && (!b || !mean)) || (res && !sum)) return hipErrorInvalidValue;
  auto* xb = reinterpret_cast<const bf16*>(x);
  auto* rb = reinterpret_cast<const bf16*>(res);
  auto* wb = reinterpret_cast<const bf16*>(w);
  auto* bb = reinterpret_cast<const bf16*>(b);
  auto* yb = reinterpret_cast<bf16*>(y);
  auto* sb = reinterpret_cast<bf16*>(sum);
  const bool r = res != nullptr;
  if (g.wpr == 1 && g.nv == 1) norm_fwd_t<1, 1>(ln, r, xb, rb, wb, bb, yb, sb, mean, rstd, M, D, eps, st);
  else if (g.wpr == 1) norm_fwd_t<2, 1>(ln, r, xb, rb, wb, bb, yb, sb, mean, rstd, M, D, eps, st);
  else if (g.nv == 1) norm_fwd_t<1, 4>(ln, r, xb, rb, wb, bb, yb, sb, mean, rstd, M, D, eps, st);
  else norm_fwd_t<2, 4>(ln, r, xb, rb, wb, bb, yb, sb, mean, rstd, M, D, eps, st);
  return hipGetLastError();
}

size_t norm_workspace_bytes_seg(int64_t M, int D, int nseg) {
  const NormGeom g = norm_geom(D);
  return static_cast<size_t>(nseg) * norm_bwd_blocks(M / nseg, g.wpr < 1 ? 1 : g.wpr) * 2 * D *
         sizeof(float);
}

hipError_t launch_norm_bwd_seg(int ln, const void* dy, const void* dres, const void* x,
                               const void* w, const float* mean, const float* rstd, void* dx,
                               void* dw, void* db, int64_t M, int D, int nseg, int64_t ostride,
                               void* work, hipStream_t st) {
  const NormGeom g = norm_geom(D);
  if (M < 1 || D % 8 || g.nv == 0 || (ln && (!db || !mean)) || nseg < 1 || M % nseg ||
      nseg > 65535)
    return hipErrorInvalidValue;
  const int64_t Ms = M / nseg;
  const int ngrp = norm_bwd_blocks(Ms, g.wpr);
  auto* part = reinterpret_cast<float*>(work);
  auto* dyb = reinterpret_cast<const bf16*>(dy);
  auto* drb = reinterpret_cast<const bf16*>(dres);
  auto* xb = reinterpret_cast<const bf16*>(x);
  auto* wb = reinterpret_cast<const bf16*>(w);
  auto* dxb = reinterpret_cast<bf16*>(dx);
  if (g.wpr == 1 && g.nv == 1) norm_bwd_t<1, 1>(ln, dyb, drb, xb, wb, mean, rstd, dxb, M, D, part, ngrp, st, Ms, nseg);
  else if (g.wpr == 1) norm_bwd_t<2, 1>(ln, dyb, drb, xb, wb, mean, rstd, dxb, M, D, part, ngrp, st, Ms, nseg);
  else if (g.nv == 1) norm_bwd_t<1, 4>(ln, dyb, drb, xb, wb, mean, rstd, dxb, M, D, part, ngrp, st, Ms, nseg);
  else norm_bwd_t<2, 4>(ln, dyb, drb, xb, wb, mean, rstd, dxb, M, D, part, ngrp, st, Ms, nseg);
  fold_kernel<<<dim3((D + 15) / 16, ln ? 2 : 1, nseg), kTB, 0, st>>>(
      part, ngrp, 2 * static_cast<int64_t>(D), D, reinterpret_cast<bf16*>(dw),
      reinterpret_cast<bf16*>(db), ostride);
  return hipGetLastError();
}

hipError_t launch_norm_bwd(int ln, const void* dy, const void* dres, const void* x,
                           const void* w, const float* mean, const float* rstd, void* dx,
                           void* dw, void* db, int64_t M, int D, void* work, hipStream_t st) {
  return launch_norm_bwd_seg(ln, dy, dres, x, w, mean, rstd, dx, dw, db, M, D, 1, 0, work, st);
}

hipError_t launch_rope_fwd(const void* qkv, const float* cosb, const float* sinb, void* q, void* k,
                           void* v, int B, int S, int H, int KV, int hd, hipStream_t st) {
  if (hd % 8 || B < 1 || S < 1 || H < 1 || KV < 1) return hipErrorInvalidValue;
  const int64_t total = static_cast<int64_t>(B) * S * (H + 2 * KV) * (hd / 8);
  rope_fwd_kernel<<<stream_grid(total), kTB, 0, st>>>(
      reinterpret_cast<const bf16*>(qkv), cosb, sinb, reinterpret_cast<bf16*>(q),
      reinterpret_cast<bf16*>(k), reinterpret_cast<bf16*>(v), B, S, H, KV, hd);
  return hipGetLastError();
}

hipError_t launch_rope_bwd(const void* dq, const void* dk, const void* dv, const float* cosb,
                           const float* sinb, void* dqkv, int B, int S, int H, int KV, int hd,
                           hipStream_t st, int grp) {
  if (hd % 8 || B < 1 || S < 1 || H < 1 || KV < 1 || grp < 1) return hipErrorInvalidValue;
  const int64_t total = static_cast<int64_t>(B) * S * (H + 2 * KV) * (hd / 8);
  rope_bwd_kernel<<<stream_grid(total), kTB, 0, st>>>(
      reinterpret_cast<const bf16*>(dq), reinterpret_cast<const bf16*>(dk),
      reinterpret_cast<const bf16*>(dv), cosb, sinb, reinterpret_cast<bf16*>(dqkv), B, S, H, KV,
      hd, grp);
  return hipGetLastError();
}

hipError_t launch_swiglu_fwd(const void* h, void* y, int64_t M, int F, hipStream_t st) {
  if (M < 1 || F % 8) return hipErrorInvalidValue;
  swiglu_fwd_kernel<<<stream_grid(M * (F / 8)), kTB, 0, st>>>(reinterpret_cast<const bf16*>(h),
                                                              reinterpret_cast<bf16*>(y), M, F);
  return hipGetLastError();
}

hipError_t launch_swiglu_bwd(const void* dy, const void* h, void* dh, int64_t M, int F,
                             hipStream_t st) {
  if (M < 1 || F % 8) return hipErrorInvalidValue;
  swiglu_bwd_kernel<<<stream_grid(M * (F / 8)), kTB, 0, st>>>(
      reinterpret_cast<const bf16*>(dy), reinterpret_cast<const bf16*>(h),
      reinterpret_cast<bf16*>(dh), M, F);
  return hipGetLastError();
}

size_t colsum_workspace_bytes(int64_t M, int N) {
  return static_cast<size_t>((M + kCSRows - 1) / kCSRows) * N * sizeof(float);
}

// Column sums of nseg row segments of M / nseg rows each (segment z -> out + z ostride); the
// 32-row slices never straddle segments when M / nseg is a multiple of 32 (else -> invalid).
hipError_t launch_colsum_seg(const void* x, int64_t M, int N, int nseg, void* out,
                             int64_t ostride, void* work, hipStream_t st) {
  if (M < 1 || N < 8 || N % 8 || (reinterpret_cast<uintptr_t>(x) & 15) || nseg < 1 ||
      M % nseg || (M / nseg) % kCSRows || nseg > 65535)
    return hipErrorInvalidValue;
  const int64_t slices = (M + kCSRows - 1) / kCSRows;
  if (slices > 65535) return hipErrorInvalidValue;
  dim3 grid((N / 8 + kWave - 1) / kWave, static_cast<unsigned>(slices));
  colsum_partial_kernel<<<grid, kTB, 0, st>>>(reinterpret_cast<const bf16*>(x), M, N,
                                              reinterpret_cast<float*>(work));
  fold_kernel<<<dim3((N + 15) / 16, 1, nseg), kTB, 0, st>>>(
      reinterpret_cast<const float*>(work), static_cast<int>(slices / nseg), N, N,
      reinterpret_cast<bf16*>(out), nullptr, ostride);
  return hipGetLastError();
}

hipError_t launch_colsum(const void* x, int64_t M, int N, void* out, void* work, hipStream_t st) {
  if (M < 1 || N < 8 || N % 8 || (reinterpret_cast<uintptr_t>(x) & 15)) return hipErrorInvalidValue;
  const int64_t slices = (M + kCSRows - 1) / kCSRows;
  if (slices > 65535) return hipErrorInvalidValue;
  dim3 grid((N / 8 + kWave - 1) / kWave, static_cast<unsigned>(slices));
  colsum_partial_kernel<<<grid, kTB, 0, st>>>(reinterpret_cast<const bf16*>(x), M, N,
                                              reinterpret_cast<float*>(work));
  fold_kernel<<<dim3((N + 15) / 16, 1), kTB, 0, st>>>(reinterpret_cast<const float*>(work),
                                                      static_cast<int>(slices), N, N,
                                                      reinterpret_cast<bf16*>(out), nullptr);
  return hipGetLastError();
}

}  // namespace cml
