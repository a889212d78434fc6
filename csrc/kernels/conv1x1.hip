// Fused 1x1 convolution forward for NHWC bf16 activations, with the BatchNorm statistics of its
// output in the epilogue and (optionally) the producer's BatchNorm + ReLU in its prologue.
//
//   y[m][n] = sum_k W[n][k] * f(x[src(m)][k])         m = output pixel, n = output channel
//   f(v)    = v                                     (plain)
//           = max(v * sc[k] + bi[k], 0)             (PM_BNRELU: the previous BN + ReLU, applied on load)
//           = a (mask ? v : 0) + b z + c            (PM_BNBWD: a BN + ReLU backward on load; data
//                                                    gradient of a conv whose output fed that BN)
//   src(m)  = m, or the stride-2 input pixel of m   (S2: ResNet downsample convs)
//   part    = per-workgroup (sum, sum of squares) of (y_bf16 - shift[n]) for the BN finalize
//
// Why: in ResNet-50 every 1x1 conv feeds a training BatchNorm, whose statistics pass re-reads the
// whole conv output (~2 B/elem, 8 ms of a 166 ms batch-2048 step over all BNs), and the 3x3
// conv's BN-ReLU output y2 is written only to be read back by conv3 (4 B/elem). Here conv3 reads
// z2 and applies bn2 + ReLU while staging, and every 1x1 conv emits its BN sums while its output
// is still in registers; the apply pass then needs no statistics pass of its own.
//
// Tiling (gfx950, wave64): a 256-thread workgroup = WN x WM waves, each wave a 64 (n) x 64 (m)
// output block = 2 x 2 v_mfma_f32_32x32x16_bf16 accumulators. The products are C^T = W * X^T so
// the accumulator's lane index is the pixel and its 16 registers are output channels: the store is
// four 8-B chunks per lane, and the per-channel statistics accumulate in registers across every
// tile the workgroup visits (one cross-lane reduction per workgroup at the end). K runs in 64-wide
// steps through 128-B LDS rows (XOR-swizzled: every ds_read_b128 lane group hits 16 distinct bank
// slots); the next step is prefetched into registers while the current one is multiplied. W is
// kept resident in LDS for the whole launch when it fits (its n-tile is fixed per workgroup).
//
// Work split: workgroups are persistent; each owns one n-tile and every wgpn-th m-tile. The
// workgroups that share an m-tile (one per n-tile) get equal blockIdx % 8, i.e. run on one XCD
// under round-robin placement, so x is read from HBM once and re-read from that XCD's L2 (speed
// only: any placement is correct).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "conv1x1_common.h"
#include "kernels.h"

namespace cml {
namespace {
using namespace c1;

// W k-step ks of rows [n0, n0 + 32 CA) into LDS block `dst`. W is small and L2-resident, so it is
// loaded at staging time rather than prefetched across the MFMA phase.
template <int CA>
__device__ __forceinline__ void stage_w(const C1Args& a, char* dst, int n0, int srow, int ch, int ks) {
  uint4 tw[CA];
#pragma unroll
  for (int j = 0; j < CA; ++j)
    tw[j] = *reinterpret_cast<const uint4*>(a.w + static_cast<int64_t>(n0 + srow + 32 * j) * a.K + ks * kBK + 8 * ch);
#pragma unroll
  for (int j = 0; j < CA; ++j) *reinterpret_cast<uint4*>(dst + swz(srow + 32 * j, ch)) = tw[j];
}

// x step ks (and, for PM_BNBWD, the matching z chunks and mask bytes) into prefetch registers
template <int CB, int BM, bool S2, int PM>
__device__ __forceinline__ void load_x(const C1Args& a, uint4 (&pb)[CB], uint4 (&pz)[CB],
                                       uint32_t (&pm)[CB], int t, int ks, int srow, int ch) {
  if constexpr (PM == PM_CAT) {
    // the source is picked per k-step by address, and every row loads a mask byte (a valid dummy
    // when the step needs none): hipcc turns per-row conditional loads into branches that wait
    // vmcnt(0) before re-targeting a register with a load still in flight
    const int k0 = ks * kBK;
    const bool first = k0 < a.K1;
    const uint16_t* base = first ? a.x : a.x2;
    const int ld = first ? a.K1 : a.K - a.K1;
    const int ko = (first ? k0 : k0 - a.K1) + 8 * ch;
    const bool mk = first && !a.cat_bnrelu;
    const uint8_t* mb = a.cat_bnrelu ? reinterpret_cast<const uint8_t*>(a.x) : a.xm;
    const int mld = a.cat_bnrelu ? 0 : a.K1 / 8;
    const int mo = mk ? k0 / 8 + ch : 0;
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const int64_t r = src_row(a, t * BM + srow + 32 * j, false);
      pb[j] = *reinterpret_cast<const uint4*>(base + r * ld + ko);
      pm[j] = mb[r * mld + mo];
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    const int64_t r = src_row(a, t * BM + srow + 32 * j, S2);
    pb[j] = *reinterpret_cast<const uint4*>(a.x + r * a.K + ks * kBK + 8 * ch);
    if constexpr (PM == PM_BNBWD) {
      pz[j] = *reinterpret_cast<const uint4*>(a.x2 + r * a.K + ks * kBK + 8 * ch);
      pm[j] = a.xm[r * (a.K / 8) + ks * (kBK / 8) + ch];
    }
  }
}


// f(x) into the LDS image (packed VALU, common.h):
//   PM_BNRELU  max(x sc + bi, 0)                        (the producer's BN + ReLU)
//   PM_BNBWD   a (mask ? x : 0) + b z + c               (a BN + ReLU backward: x = dL/d(output),
//              z = the BN input; a = gamma invstd, b = -gamma invstd^2 q / M,
//              c = -gamma invstd s / M - b mean, with s, q the BN's backward sums)
//   PM_CAT     (mask ? x : 0)        for k < K1 (x = a BN + ReLU output gradient; the BN backward's
//                                    affine is folded into w and the epilogue bias), or
//              max(x sc + bi, 0)     for k < K1 with cat_bnrelu;
//              max(x2 sc + bi, 0)    for k >= K1 (a BN + ReLU output, recomputed), or x2 itself
//                                    (id2: a ReLU output that needs no BN): one GEMM over two
//                                    sources concatenated along K
// kofs: first input channel of this k-step (ks * 64); KA: entries per coefficient row of s_aff.
// The mode is uniform per k-step, so each is one straight loop over the thread's chunks.
template <int CB, int PM>
__device__ __forceinline__ void store_x(const uint4 (&pb)[CB], const uint4 (&pz)[CB],
                                        const uint32_t (&pm)[CB], char* sx, const float* s_aff,
                                        int KA, int kofs, int srow, int ch, int K1 = 0,
                                        int cat_bnrelu = 0, bool id2 = false) {
  auto put = [&](int j, uint4 v) { *reinterpret_cast<uint4*>(sx + swz(srow + 32 * j, ch)) = v; };
  // 0: as is, 1: BN + ReLU, 2: mask only
  const int mode = PM == PM_NONE ? 0
                 : PM == PM_CAT  ? (kofs < K1 ? (cat_bnrelu ? 1 : 2) : (id2 ? 0 : 1))
                                 : 1;
  if constexpr (PM == PM_BNBWD) {
    float sc[8], bi[8], cc[8];
    ld8f(s_aff + kofs + 8 * ch, sc);
    ld8f(s_aff + KA + kofs + 8 * ch, bi);
    ld8f(s_aff + 2 * KA + kofs + 8 * ch, cc);
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const uint32_t bits = pm[j];
      const uint4 g = make_uint4(mask_pk<0>(pb[j].x, bits), mask_pk<1>(pb[j].y, bits),
                                 mask_pk<2>(pb[j].z, bits), mask_pk<3>(pb[j].w, bits));
      const uint32_t g4[4] = {g.x, g.y, g.z, g.w};
      const uint32_t z4[4] = {pz[j].x, pz[j].y, pz[j].z, pz[j].w};
      uint32_t w4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2 gv = {__uint_as_float(g4[i] << 16), __uint_as_float(g4[i] & 0xffff0000u)};
        const f32x2 zv = {__uint_as_float(z4[i] << 16), __uint_as_float(z4[i] & 0xffff0000u)};
        const f32x2 t = __builtin_elementwise_fma(f32x2{bi[2 * i], bi[2 * i + 1]}, zv,
                                                  f32x2{cc[2 * i], cc[2 * i + 1]});
        const f32x2 r = __builtin_elementwise_fma(f32x2{sc[2 * i], sc[2 * i + 1]}, gv, t);
        w4[i] = pk_bf16(r.x, r.y);
      }
      put(j, make_uint4(w4[0], w4[1], w4[2], w4[3]));
    }
    return;
  }
  if (mode == 1) {
    float sc[8], bi[8];
    ld8f(s_aff + kofs + 8 * ch, sc);
    ld8f(s_aff + KA + kofs + 8 * ch, bi);
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const uint4 v = pb[j];
      put(j, make_uint4(bnrelu_pk(v.x, f32x2{sc[0], sc[1]}, f32x2{bi[0], bi[1]}),
                        bnrelu_pk(v.y, f32x2{sc[2], sc[3]}, f32x2{bi[2], bi[3]}),
                        bnrelu_pk(v.z, f32x2{sc[4], sc[5]}, f32x2{bi[4], bi[5]}),
                        bnrelu_pk(v.w, f32x2{sc[6], sc[7]}, f32x2{bi[6], bi[7]})));
    }
  } else if (mode == 2) {
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const uint4 v = pb[j];
      const uint32_t bits = pm[j];
      put(j, make_uint4(mask_pk<0>(v.x, bits), mask_pk<1>(v.y, bits), mask_pk<2>(v.z, bits),
                        mask_pk<3>(v.w, bits)));
    }
  } else {
#pragma unroll
    for (int j = 0; j < CB; ++j) put(j, pb[j]);
  }
}

// MT: 64-pixel sub-blocks per wave (wave tile 64 (n) x 64 MT (m)). MT = 2 halves the LDS operand
// reads per MFMA (2 A + 4 B fragments feed 8 MFMAs instead of 2 + 2 for 4) and the W re-staging
// per output pixel; its epilogue images then alias the x staging buffer (BM = 256 rows = 32 KB,
// behind one extra barrier per tile) to stay inside 80 KB of LDS.
template <int WN, int WM, int PM, bool WRES, bool S2, bool EL, int SM, int MT = 1>
__global__ __launch_bounds__(kThreads, 2) void conv1x1_bn_fwd_kernel(C1Args a) {
  constexpr int NAFF = PM == PM_BNBWD ? 3 : ((PM == PM_BNRELU || PM == PM_CAT) ? 2 : 0);
  const int KA = a.K;                                           // prologue coefficients per row
  constexpr int BN = 64 * WN, BM = 64 * WM * MT;
  constexpr int CA = BN / 32, CB = BM / 32;     // 16-B staging chunks per thread and step
  constexpr bool ALIAS = MT > 1;
  static_assert(!ALIAS || BM * 128 == 4 * 8192, "aliased epilogue images need a 32 KB x buffer");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KS = a.K / kBK;
  char* sw = smem;                                              // W: (WRES ? KS : 1) x [BN][128 B]
  char* sx = smem + (WRES ? KS : 1) * BN * 128;                 // x: [BM][128 B]
  float* s_aff = reinterpret_cast<float*>(sx + BM * 128);       // prologue coefficients [NAFF][K]
  float* s_sh = s_aff + NAFF * KA;                              // statistics shift [BN]
  float* s_bias = s_sh + BN;                                    // PM_CAT: epilogue bias [BN]
  char* s_img = ALIAS ? sx : reinterpret_cast<char*>(s_bias + BN);   // epilogue images: 4 x 8 KB

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;
  const int h = lane >> 5, r32 = lane & 31;
  const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
  const int nt = slot % a.ntn;
  const int j0 = (slot / a.ntn) * 8 + xcd;                     // first m-tile of this workgroup
  const int n0 = nt * BN;
  const int ch = tid & 7;                                       // 16-B chunk of every staged row
  const int srow = tid >> 3;                                    // first staged row (+32 per item)

  for (int c = tid; c < BN; c += kThreads) s_sh[c] = a.shift ? a.shift[n0 + c] : 0.f;
  if constexpr (PM == PM_CAT) {   // the bias of the workgroup's n-tile, read by every tile's epilogue
    for (int c = tid; c < BN; c += kThreads) s_bias[c] = a.bias ? a.bias[n0 + c] : 0.f;
  }
  if constexpr (NAFF > 0) fill_aff(a, PM == PM_CAT, s_aff, KA, tid, kThreads);
  if constexpr (NAFF > 2) {
    for (int k = tid; k < KA; k += kThreads) s_aff[2 * KA + k] = a.pro_c[k];
  }
  const bool id2 = PM == PM_CAT && a.pro_sc2 == nullptr;
  // first input channel of k-step ks
  auto kofs = [&](int ks_) { return ks_ * kBK; };
  if constexpr (WRES) {   // the whole W slice of this n-tile, once
    for (int ks = 0; ks < KS; ++ks) stage_w<CA>(a, sw + ks * BN * 128, n0, srow, ch, ks);
  }

  f32x16 acc[MT][2][2];
#pragma unroll
  for (int u = 0; u < MT; ++u)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        acc[u][i][0][k] = 0.f;
        acc[u][i][1][k] = 0.f;
      }
  // statistics: lane owns channels n0 + wn*64 + 8 (lane & 7) + q, q < 8 (see epilogue)
  float ss[8], sq[8], sh[8];

  uint4 pb[CB], pz[CB];
  uint32_t pm[CB];
  int t = j0, ks = 0;
  if (t < a.mtiles) {
    load_x<CB, BM, S2, PM>(a, pb, pz, pm, t, 0, srow, ch);
    __syncthreads();                 // s_aff / s_sh / resident W visible
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sh[q] = s_sh[wn * 64 + 8 * (lane & 7) + q];
      ss[q] = 0.f;
      sq[q] = 0.f;
    }
    store_x<CB, PM>(pb, pz, pm, sx, s_aff, KA, 0, srow, ch, a.K1, a.cat_bnrelu, id2);
    if constexpr (!WRES) stage_w<CA>(a, sw, n0, srow, ch, 0);
    __syncthreads();
    for (;;) {
      int tn = t, ksn = ks + 1;
      if (ksn == KS) {
        ksn = 0;
        tn = t + a.wgpn;
      }
      const bool more = tn < a.mtiles;
      // prefetch the next step's x into registers; past the end, reload the current (valid) step
      // instead of branching around the loads (hipcc would wait for them at the join)
      load_x<CB, BM, S2, PM>(a, pb, pz, pm, more ? tn : t, more ? ksn : ks, srow, ch);
      const char* wa = sw + (WRES ? ks : 0) * BN * 128;
#pragma unroll
      for (int kk = 0; kk < kBK / 16; ++kk) {
        bf16x8_t A[2], B[MT][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          A[i] = *reinterpret_cast<const bf16x8_t*>(wa + swz(wn * 64 + 32 * i + r32, 2 * kk + h));
#pragma unroll
        for (int u = 0; u < MT; ++u)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            B[u][j] = *reinterpret_cast<const bf16x8_t*>(
                sx + swz(wm * 64 * MT + 64 * u + 32 * j + r32, 2 * kk + h));
#pragma unroll
        for (int u = 0; u < MT; ++u)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[u][i][j] = mfma32(A[i], B[u][j], acc[u][i][j]);
      }
      if (ks == KS - 1) {
        if constexpr (ALIAS) __syncthreads();   // every wave is done reading x before the images
#pragma unroll
        for (int u = 0; u < MT; ++u)
          epilogue<EL, SM, MT, PM == PM_CAT && SM == SM_BNBWD,
                   PM == PM_CAT && SM != SM_BNRES>(a, acc[u], ss, sq, sh,
                                                               s_img + wave * 8192,
                           t * BM + wm * 64 * MT + 64 * u, wn * 64, n0, lane, -1,
                           a.bias ? s_bias : nullptr);
      }
      if (!more) break;
      __syncthreads();               // every wave is done reading this step's LDS
      store_x<CB, PM>(pb, pz, pm, sx, s_aff, KA, kofs(ksn), srow, ch, a.K1, a.cat_bnrelu, id2);
      if constexpr (!WRES) stage_w<CA>(a, sw, n0, srow, ch, ksn);
      __syncthreads();
      t = tn;
      ks = ksn;
    }
  }
  if (SM == SM_OFF || !a.part) return;
  if (t >= a.mtiles) {   // no tile: zero partials
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      ss[q] = 0.f;
      sq[q] = 0.f;
    }
  }
  // per-wave channel totals: reduce over the 8 lanes that share a channel group (lane >> 3)
  float* pp = a.part + (static_cast<int64_t>(nt) * a.wgpn * WM + j0 * WM + wm) * 2 * BN;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float s = ss[q], v = sq[q];
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      s += __shfl_xor(s, o, 64);
      v += __shfl_xor(v, o, 64);
    }
    if (lane < 8) {
      const int c = wn * 64 + 8 * lane + q;
      pp[c] = s;
      pp[BN + c] = v;
    }
  }
}

// BN statistics from the conv's partial slab: 8 channels per workgroup, 32 row slices each, fp64,
// fixed fold order (deterministic). mean = shift + S / M, var = Q / M - (S / M)^2.
__global__ __launch_bounds__(256) void conv1x1_bn_finalize_kernel(
    const float* __restrict__ part, int R, int BN, int N, int64_t M, const float* shift,
    float eps, float momentum, float* __restrict__ mean, float* __restrict__ invstd,
    float* __restrict__ rmean, float* __restrict__ rvar, const uint16_t* __restrict__ gamma,
    const uint16_t* __restrict__ beta, float* __restrict__ sc, float* __restrict__ bi) {
  __shared__ double ls[32][8], lq[32][8];
  const int cl = threadIdx.x & 7, sl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  double S = 0.0, Q = 0.0;
  if (c < N) {
    const int nt = c / BN, cc = c - nt * BN;
    const float* base = part + static_cast<int64_t>(nt) * R * 2 * BN + cc;
    int r = sl;
    for (; r + 3 * 32 < R; r += 4 * 32) {
      float s[4], q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s[u] = base[static_cast<int64_t>(r + 32 * u) * 2 * BN];
        q[u] = base[static_cast<int64_t>(r + 32 * u) * 2 * BN + BN];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        S += s[u];
        Q += q[u];
      }
    }
    for (; r < R; r += 32) {
      S += base[static_cast<int64_t>(r) * 2 * BN];
      Q += base[static_cast<int64_t>(r) * 2 * BN + BN];
    }
  }
  ls[sl][cl] = S;
  lq[sl][cl] = Q;
  __syncthreads();
  if (sl != 0 || c >= N) return;
  S = 0.0;
  Q = 0.0;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    S += ls[k][cl];
    Q += lq[k][cl];
  }
  const double ms = S / static_cast<double>(M);
  double var = Q / static_cast<double>(M) - ms * ms;
  if (var < 0.0) var = 0.0;
  const double mu = (shift ? static_cast<double>(shift[c]) : 0.0) + ms;
  const float mf = static_cast<float>(mu), isf = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
  mean[c] = mf;
  invstd[c] = isf;
  if (sc) {   // the BN affine as bn_affine computes it from the stored fp32 mean / invstd
#pragma clang fp contract(off)
    const float s = __uint_as_float(static_cast<uint32_t>(gamma[c]) << 16) * isf;
    sc[c] = s;
    const float mfs = mf * s;
    bi[c] = __uint_as_float(static_cast<uint32_t>(beta[c]) << 16) - mfs;
  }
  if (rmean) {
    const double unb = M > 1 ? var * static_cast<double>(M) / static_cast<double>(M - 1) : var;
    rmean[c] = static_cast<float>((1.0 - momentum) * rmean[c] + momentum * mu);
    rvar[c] = static_cast<float>((1.0 - momentum) * rvar[c] + momentum * unb);
  }
}

// First level of a two-level fold of a tall [ntn][R][2][BN] partial slab (one row per output tile
// of a non-persistent GEMM): block (s, nt) sums rows [s rp, (s + 1) rp) into out row s of
// [ntn][S][2][BN], so the per-channel finalize reads S << R rows (fixed order: deterministic).
__global__ __launch_bounds__(256) void part_fold_kernel(const float* __restrict__ part, int R,
                                                        int BN, int rp, int S,
                                                        float* __restrict__ out) {
  __shared__ float red[256];
  const int cols = 2 * BN, nt = blockIdx.y, s = blockIdx.x;
  const int RL = cols >= 256 ? 1 : 256 / cols;
  const int t = threadIdx.x, rl = t / (cols >= 256 ? 256 : cols);
  const int r0 = s * rp, r1 = min(R, r0 + rp);
  const float* base = part + static_cast<int64_t>(nt) * R * cols;
  float* ob = out + (static_cast<int64_t>(nt) * S + s) * cols;
  if (RL == 1) {
    for (int col = t; col < cols; col += 256) {
      float acc = 0.f;
      for (int r = r0; r < r1; ++r) acc += base[static_cast<int64_t>(r) * cols + col];
      ob[col] = acc;
    }
    return;
  }
  const int col = t - rl * cols;
  float acc = 0.f;
  for (int r = r0 + rl; r < r1; r += RL) acc += base[static_cast<int64_t>(r) * cols + col];
  red[t] = acc;
  __syncthreads();
  if (rl == 0) {
    for (int k = 1; k < RL; ++k) acc += red[k * cols + col];
    ob[col] = acc;
  }
}

// BN-backward sums from the partial slab (SM_BNBWD): sdz = S, sdzx = Q * invstd (same fixed fold
// order as the statistics finalize).
__global__ __launch_bounds__(256) void conv1x1_bnbwd_finalize_kernel(
    const float* __restrict__ part, int R, int BN, int N, const float* __restrict__ invstd,
    float* __restrict__ sdz, float* __restrict__ sdzx, uint16_t* __restrict__ dgamma,
    uint16_t* __restrict__ dbeta) {
  __shared__ double ls[32][8], lq[32][8];
  const int cl = threadIdx.x & 7, sl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  double S = 0.0, Q = 0.0;
  if (c < N) {
    const int nt = c / BN, cc = c - nt * BN;
    const float* base = part + static_cast<int64_t>(nt) * R * 2 * BN + cc;
    for (int r = sl; r < R; r += 32) {
      S += base[static_cast<int64_t>(r) * 2 * BN];
      Q += base[static_cast<int64_t>(r) * 2 * BN + BN];
    }
  }
  ls[sl][cl] = S;
  lq[sl][cl] = Q;
  __syncthreads();
  if (sl != 0 || c >= N) return;
  S = 0.0;
  Q = 0.0;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    S += ls[k][cl];
    Q += lq[k][cl];
  }
  const float fs = static_cast<float>(S), fq = static_cast<float>(Q * static_cast<double>(invstd[c]));
  sdz[c] = fs;
  sdzx[c] = fq;
  if (dgamma) {   // the BN's parameter gradients, as bn_bwd_coeffs_kernel rounds them
    dgamma[c] = f2bf(fq);
    dbeta[c] = f2bf(fs);
  }
}

// BN training statistics of z = y W^T (W [Co][P] bf16: the 1x1 conv's weights) from the Gram matrix
// G = y^T y [P][P] and the column sums cy of y over M rows (fp32: wgrad1x1_ex's products of the
// same bf16 y the conv multiplies): mean = W cy / M, var = w^T G w / M - mean^2, partial inner
// products (G w)_i in fp32 and everything after in fp64. These are the statistics of the
// fp32-accumulated products; the statistics-only conv pass they replace saw the same products
// rounded to bf16.
// Two launches. bn_stats_gram_kernel: workgroup (channel block of kGramNC, 64-row chunk jc of G)
// computes q_part = sum_i w_i sum_{j in jc} G[j][i] w_j (each thread 4 consecutive i, one float4
// of a G row per step) into an fp64 slab [P / 64][Co]; bn_stats_gram_fin_kernel (one wave per
// channel) sums the chunks in a fixed order (deterministic), adds S = w . cy and writes the
// statistics. ~0.7 TFLOP-equivalent of fp32 FMA per ResNet-50 step spread over (Co / 8) x (P / 64)
// workgroups (round 2's kernel read all of G in one workgroup per 16 channels with one float per
// load: ~45 us per call at any batch, 0.75 ms per step).
constexpr int kGramNC = 8;

__global__ __launch_bounds__(256) void bn_stats_gram_kernel(
    const float* __restrict__ G, const uint16_t* __restrict__ W, int P, int Co,
    double* __restrict__ part) {
  constexpr int NC = kGramNC;
  extern __shared__ float ws[];            // [P][NC] weights of this workgroup's channels
  __shared__ double red[4][NC];
  const int n0 = blockIdx.x * NC, jc = blockIdx.y * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int Q4 = P / 4;                              // float4 columns of a G row
  const int TG = Q4 < 256 ? Q4 : 256;                // threads per row subgroup
  const int JP = 256 / TG, JL = 64 / JP;             // row subgroups, rows per subgroup
  const int jp = tid / TG, q0 = tid - jp * TG;
  for (int e = tid; e < NC * P; e += 256) {
    const int c = e / P, j = e - c * P;
    ws[j * NC + c] = n0 + c < Co ? bf2f(W[static_cast<int64_t>(n0 + c) * P + j]) : 0.f;
  }
  __syncthreads();
  double q[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) q[c] = 0.0;
  const int j0 = jc + jp * JL;
  // G is symmetric: (G w)_i = sum_j G[j][i] w_j, the lanes reading consecutive float4 of row j
  for (int qi = q0; qi < Q4; qi += TG) {
    const int i = 4 * qi;
    float t[NC][4];
#pragma unroll
    for (int c = 0; c < NC; ++c) t[c][0] = t[c][1] = t[c][2] = t[c][3] = 0.f;
    const float* gp = G + static_cast<int64_t>(j0) * P + i;
#pragma unroll 8
    for (int j = 0; j < JL; ++j) {
      const float4 g = *reinterpret_cast<const float4*>(gp + static_cast<int64_t>(j) * P);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float w = ws[(j0 + j) * NC + c];
        t[c][0] = fmaf(g.x, w, t[c][0]);
        t[c][1] = fmaf(g.y, w, t[c][1]);
        t[c][2] = fmaf(g.z, w, t[c][2]);
        t[c][3] = fmaf(g.w, w, t[c][3]);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < NC; ++c)
        q[c] = fma(static_cast<double>(ws[(i + k) * NC + c]), static_cast<double>(t[c][k]), q[c]);
  }
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) q[c] += __shfl_xor(q[c], o, 64);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < NC; ++c) red[wv][c] = q[c];
  }
  __syncthreads();
  if (tid < NC && n0 + tid < Co)
    part[static_cast<int64_t>(blockIdx.y) * Co + n0 + tid] =
        red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
}

__global__ __launch_bounds__(256) void bn_stats_gram_fin_kernel(
    const double* __restrict__ part, const float* __restrict__ cy, const uint16_t* __restrict__ W,
    int P, int Co, int64_t M, float eps, float momentum, float* __restrict__ mean,
    float* __restrict__ invstd, float* __restrict__ rmean, float* __restrict__ rvar,
    const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ beta, float* __restrict__ sc,
    float* __restrict__ bi) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= Co) return;
  double S = 0.0;
  for (int i = lane; i < P; i += 64)
    S = fma(static_cast<double>(bf2f(W[static_cast<int64_t>(n) * P + i])), static_cast<double>(cy[i]), S);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) S += __shfl_xor(S, o, 64);
  if (lane != 0) return;
  double Q = 0.0;
  for (int c = 0; c < P / 64; ++c) Q += part[static_cast<int64_t>(c) * Co + n];
  const double mu = S / static_cast<double>(M);
  double var = Q / static_cast<double>(M) - mu * mu;
  if (var < 0.0) var = 0.0;
  const float mf = static_cast<float>(mu), isf = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
  mean[n] = mf;
  invstd[n] = isf;
  if (sc) {   // the BN affine (sc, bi) as bn_affine computes it from the stored fp32 mean / invstd
#pragma clang fp contract(off)
    const float s = __uint_as_float(static_cast<uint32_t>(gamma[n]) << 16) * isf;
    sc[n] = s;
    const float ms = mf * s;
    bi[n] = __uint_as_float(static_cast<uint32_t>(beta[n]) << 16) - ms;
  }
  if (rmean) {
    const double unb = M > 1 ? var * static_cast<double>(M) / static_cast<double>(M - 1) : var;
    rmean[n] = static_cast<float>((1.0 - momentum) * rmean[n] + momentum * mu);
    rvar[n] = static_cast<float>((1.0 - momentum) * rvar[n] + momentum * unb);
  }
}

// Per-channel coefficients of a training BN + ReLU backward, dz = a (mask ? dy : 0) + b z + c,
// from its sums s = sum dy', q = sum dy' xhat (dy' = masked dy); also dgamma = q, dbeta = s.
__global__ __launch_bounds__(256) void bn_bwd_coeffs_kernel(
    const float* __restrict__ sdz, const float* __restrict__ sdzx, const uint16_t* __restrict__ gamma,
    const float* __restrict__ mean, const float* __restrict__ invstd, int C, float invM,
    float* __restrict__ ca, float* __restrict__ cb, float* __restrict__ cc,
    uint16_t* __restrict__ dgamma, uint16_t* __restrict__ dbeta) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float is = invstd[c];
  const float sc = is * __uint_as_float(static_cast<uint32_t>(gamma[c]) << 16);
  const float b = -sc * is * sdzx[c] * invM;
  ca[c] = sc;
  cb[c] = b;
  cc[c] = -sc * sdz[c] * invM - b * mean[c];
  dgamma[c] = f2bf(sdzx[c]);
  dbeta[c] = f2bf(sdz[c]);
}

struct Plan {
  int WN, WM, MT, BN, BM, ntn, wgpn, mtiles, G;
  bool wres;
  size_t lds;
};

Plan plan_for(int WN, int64_t M, int K, int N, int naff, int mt = 1, int kaff = -1) {
  if (kaff < 0) kaff = K;
  Plan p{};
  p.WN = WN;
  p.WM = 4 / p.WN;
  p.MT = mt;
  p.BN = 64 * p.WN;
  p.BM = 64 * p.WM * mt;
  p.ntn = N / p.BN;
  p.mtiles = static_cast<int>((M + p.BM - 1) / p.BM);
  const int target = 512;                                     // 2 workgroups per CU
  int w = (target + p.ntn - 1) / p.ntn;
  const int mt8 = (p.mtiles + 7) / 8 * 8;
  w = (w + 7) / 8 * 8;
  p.wgpn = w < mt8 ? w : mt8;
  p.G = p.ntn * p.wgpn;
  const size_t wbytes = static_cast<size_t>(K) * p.BN * 2;
  const size_t xbytes = static_cast<size_t>(p.BM) * 128;
  const size_t aff = static_cast<size_t>(naff) * kaff * 4 + static_cast<size_t>(p.BN) * 8 +
                     (mt > 1 ? 0 : 4 * 8192);   // + the per-wave epilogue images (aliased at MT 2)
  p.wres = wbytes + xbytes + aff <= 80 * 1024;
  p.lds = (p.wres ? wbytes : static_cast<size_t>(p.BN) * 128) + xbytes + aff;
  return p;
}

// Widest n-tile that covers N, except that a 256-channel tile whose W slice cannot stay resident
// (K > 64) re-stages 32 KB of W per 64 pixels: there 128 x 128 tiles are ~2x faster
// (bench/conv1x1_fused.py, profiles/r02_conv1x1_*.jsonl).
// CML_C1_MT2=0 disables the MT = 2 tiles (A/B)
bool mt2_enabled() {
  static const bool on = [] {
    const char* e = getenv("CML_C1_MT2");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Also take the MT = 2 tile when it lets W stay resident (without the per-wave epilogue images
// the MT = 1 plan needs, W fits): the layer-2 recompute apply GEMM (K 128, N 512); step 133.5 ->
// 133.1 ms (profiles/r02_c1_mt2_wres47.txt). CML_C1_MT2_WRES=0 disables it (A/B).
bool mt2_wres_enabled() {
  static const bool on = [] {
    const char* e = getenv("CML_C1_MT2_WRES");
    return !(e && e[0] == '0');
  }();
  return on;
}

Plan make_plan(int64_t M, int K, int N, int naff, int kaff = -1, bool mt2_ok = true) {
  const int WN = N % 256 == 0 ? 4 : (N % 128 == 0 ? 2 : 1);
  Plan p = plan_for(WN, M, K, N, naff, 1, kaff);
  if (WN == 4 && !p.wres) p = plan_for(2, M, K, N, naff, 1, kaff);
  // non-resident 128 x 128 tiles: two 64-pixel sub-blocks per wave (see the kernel)
  // (not with the BN-backward prologue: its extra z / mask prefetch registers would spill)
  if (p.WN == 2 && !p.wres && naff < 3 && mt2_ok && mt2_enabled()) {
    const Plan q = plan_for(2, M, K, N, naff, 2, kaff);
    if ((!q.wres || mt2_wres_enabled()) && q.lds <= 80 * 1024) p = q;
  }
  return p;
}

template <int WN, int WM, int PM, bool WRES, bool S2, bool EL = false, int SM = SM_BN>
hipError_t launch_t(const C1Args& a, const Plan& p, hipStream_t st) {
  auto k = &conv1x1_bn_fwd_kernel<WN, WM, PM, WRES, S2, EL, SM, 1>;
  if constexpr (WN == 2 && PM != PM_BNBWD && SM != SM_BNBWD && !(PM == PM_CAT && SM == SM_BNRES)) {
    if (p.MT == 2) k = &conv1x1_bn_fwd_kernel<WN, WM, PM, WRES, S2, EL, SM, 2>;
  }
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  k<<<p.G, kThreads, p.lds, st>>>(a);
  return hipGetLastError();
}

template <int WN, int WM>
hipError_t launch_w(const C1Args& a, const Plan& p, bool pro, bool s2, hipStream_t st) {
  if (s2) {
    if (pro) return hipErrorInvalidValue;   // strided convs read a materialised block input
    return p.wres ? launch_t<WN, WM, PM_NONE, true, true>(a, p, st)
                  : launch_t<WN, WM, PM_NONE, false, true>(a, p, st);
  }
  if (pro)
    return p.wres ? launch_t<WN, WM, PM_BNRELU, true, false>(a, p, st)
                  : launch_t<WN, WM, PM_BNRELU, false, false>(a, p, st);
  return p.wres ? launch_t<WN, WM, PM_NONE, true, false>(a, p, st)
                : launch_t<WN, WM, PM_NONE, false, false>(a, p, st);
}

// backward variants (stride 1): mode 0 = BN-backward prologue, no statistics; 1 = masked link
// epilogue; 2 = masked link epilogue + BN-backward sums
template <int WN, int WM>
hipError_t launch_bwd_w(const C1Args& a, const Plan& p, int mode, hipStream_t st) {
  if (mode == 0)
    return p.wres ? launch_t<WN, WM, PM_BNBWD, true, false, false, SM_OFF>(a, p, st)
                  : launch_t<WN, WM, PM_BNBWD, false, false, false, SM_OFF>(a, p, st);
  if (mode == 1)
    return p.wres ? launch_t<WN, WM, PM_NONE, true, false, true, SM_OFF>(a, p, st)
                  : launch_t<WN, WM, PM_NONE, false, false, true, SM_OFF>(a, p, st);
  return p.wres ? launch_t<WN, WM, PM_NONE, true, false, true, SM_BNBWD>(a, p, st)
                : launch_t<WN, WM, PM_NONE, false, false, true, SM_BNBWD>(a, p, st);
}

hipError_t launch_bwd(const C1Args& a, const Plan& p, int mode, hipStream_t st) {
  if (p.WN == 4) return launch_bwd_w<4, 1>(a, p, mode, st);
  if (p.WN == 2) return launch_bwd_w<2, 2>(a, p, mode, st);
  return launch_bwd_w<1, 4>(a, p, mode, st);
}

// recompute tail (fused BN + residual + ReLU epilogue) and two-source (PM_CAT) data gradient
template <int WN, int WM>
hipError_t launch_tail_w(const C1Args& a, const Plan& p, bool cat, hipStream_t st) {
  if (cat && a.ymask)
    return p.wres ? launch_t<WN, WM, PM_CAT, true, false, false, SM_BNRES>(a, p, st)
                  : launch_t<WN, WM, PM_CAT, false, false, false, SM_BNRES>(a, p, st);
  if (cat && a.part)   // + the BN + ReLU backward sums of the output (mask recomputed, DM)
    return p.wres ? launch_t<WN, WM, PM_CAT, true, false, false, SM_BNBWD>(a, p, st)
                  : launch_t<WN, WM, PM_CAT, false, false, false, SM_BNBWD>(a, p, st);
  if (cat)
    return p.wres ? launch_t<WN, WM, PM_CAT, true, false, false, SM_OFF>(a, p, st)
                  : launch_t<WN, WM, PM_CAT, false, false, false, SM_OFF>(a, p, st);
  return p.wres ? launch_t<WN, WM, PM_BNRELU, true, false, false, SM_BNRES>(a, p, st)
                : launch_t<WN, WM, PM_BNRELU, false, false, false, SM_BNRES>(a, p, st);
}

hipError_t launch_tail(const C1Args& a, const Plan& p, bool cat, hipStream_t st) {
  if (p.WN == 4) return launch_tail_w<4, 1>(a, p, cat, st);
  if (p.WN == 2) return launch_tail_w<2, 2>(a, p, cat, st);
  return launch_tail_w<1, 4>(a, p, cat, st);
}

C1Args base_args(const void* x, const void* w, void* y, int64_t M, int K, int N, const Plan& p) {
  C1Args a{};
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.w = reinterpret_cast<const uint16_t*>(w);
  a.y = reinterpret_cast<uint16_t*>(y);
  a.M = static_cast<int>(M);
  a.K = K;
  a.N = N;
  a.ntn = p.ntn;
  a.wgpn = p.wgpn;
  a.mtiles = p.mtiles;
  return a;
}

bool bad_shape(int64_t M, int K, int N) {
  return K % kBK || N % 64 || M < 1 || M >= (1ll << 31) || K > 4096 || N > 4096;
}

}  // namespace

size_t conv1x1_bn_part_floats(int64_t M, int K, int N, bool pro) {
  const Plan p = make_plan(M, K, N, pro ? 2 : 0);
  const size_t g = conv1x1g_pick(M, K, N, pro ? PM_BNRELU : PM_NONE)
                       ? conv1x1g_part_floats(M, K, N, pro ? PM_BNRELU : PM_NONE) : 0;
  return std::max(static_cast<size_t>(p.G) * p.WM * 2 * p.BN, g);
}

int bn_part_fold_slices(int R, int ntn) {
  if (R <= 256) return 0;
  const int want = std::max(256, (2048 + ntn - 1) / ntn);
  return std::min((R + 15) / 16, want);
}

hipError_t launch_bn_stats_finalize(const float* part, int R, int BN, int N, int64_t M,
                                   const float* shift, float eps, float momentum, float* mean,
                                   float* invstd, float* rmean, float* rvar, hipStream_t st,
                                   float* fold, const BnAffineOut* aff) {
  if (aff && (!aff->gamma || !aff->beta || !aff->sc || !aff->bi)) return hipErrorInvalidValue;
  const int S = fold ? bn_part_fold_slices(R, N / BN) : 0;
  if (S > 0) {
    const int rp = (R + S - 1) / S;
    const int S2 = (R + rp - 1) / rp;
    part_fold_kernel<<<dim3(S2, N / BN), 256, 0, st>>>(part, R, BN, rp, S2, fold);
    part = fold;
    R = S2;
  }
  conv1x1_bn_finalize_kernel<<<(N + 7) / 8, 256, 0, st>>>(
      part, R, BN, N, M, shift, eps, momentum, mean, invstd, rmean, rvar,
      aff ? reinterpret_cast<const uint16_t*>(aff->gamma) : nullptr,
      aff ? reinterpret_cast<const uint16_t*>(aff->beta) : nullptr, aff ? aff->sc : nullptr,
      aff ? aff->bi : nullptr);
  return hipGetLastError();
}

// BN + ReLU backward sums {sdz, sdzx} from a GEMM's partial slab [ntn][R][2][BN] (tall slabs folded
// first, as launch_bn_stats_finalize does)
hipError_t launch_bnbwd_sums_finalize(const float* part, int R, int BN, int N, const float* invstd,
                                      float* sdz, float* sdzx, hipStream_t st, float* fold,
                                      void* dgamma, void* dbeta) {
  if ((dgamma == nullptr) != (dbeta == nullptr)) return hipErrorInvalidValue;
  const int S = fold ? bn_part_fold_slices(R, N / BN) : 0;
  if (S > 0) {
    const int rp = (R + S - 1) / S;
    const int S2 = (R + rp - 1) / rp;
    part_fold_kernel<<<dim3(S2, N / BN), 256, 0, st>>>(part, R, BN, rp, S2, fold);
    part = fold;
    R = S2;
  }
  conv1x1_bnbwd_finalize_kernel<<<(N + 7) / 8, 256, 0, st>>>(
      part, R, BN, N, invstd, sdz, sdzx, reinterpret_cast<uint16_t*>(dgamma),
      reinterpret_cast<uint16_t*>(dbeta));
  return hipGetLastError();
}

// the link + BN-backward-sums kernel runs MT = 1 tiles (at MT = 2 its epilogue operands spill)
size_t conv1x1_link_part_floats(int64_t M, int K, int N) {
  const Plan p = make_plan(M, K, N, 0, -1, false);
  const size_t g = conv1x1g_pick(M, K, N, PM_NONE) ? conv1x1g_part_floats(M, K, N, PM_NONE) : 0;
  return std::max(static_cast<size_t>(p.G) * p.WM * 2 * p.BN, g);
}

hipError_t launch_conv1x1_bnbwd(const void* g, const void* z, const uint8_t* mask, const float* ca,
                                const float* cb, const float* cc, const void* w, void* y,
                                int64_t M, int K, int N, hipStream_t st) {
  if (bad_shape(M, K, N)) return hipErrorInvalidValue;
  const Plan p = make_plan(M, K, N, 3);
  C1Args a = base_args(g, w, y, M, K, N, p);
  a.x2 = reinterpret_cast<const uint16_t*>(z);
  a.xm = mask;
  a.pro_sc = ca;
  a.pro_bi = cb;
  a.pro_c = cc;
  return launch_bwd(a, p, 0, st);
}

hipError_t launch_conv1x1_link(const void* x, const void* w, void* y, const void* link,
                               const uint8_t* lm, const void* sz, const uint8_t* sm,
                               const float* mean, const float* invstd, float* part, float* sdz,
                               float* sdzx, int64_t M, int K, int N, hipStream_t st) {
  if (bad_shape(M, K, N)) return hipErrorInvalidValue;
  const bool sums = sz != nullptr;
  if (sums && (!sm || !mean || !invstd || !part || !sdz || !sdzx)) return hipErrorInvalidValue;
  const Plan p = make_plan(M, K, N, 0, -1, !sums);
  C1Args a = base_args(x, w, y, M, K, N, p);
  a.link = reinterpret_cast<const uint16_t*>(link);
  a.lm = lm;
  if (sums) {
    a.sz = reinterpret_cast<const uint16_t*>(sz);
    a.sm = sm;
    a.shift = mean;
    a.part = part;
  }
  if (conv1x1g_pick(M, K, N, PM_NONE)) {
    int R, BN;
    hipError_t e = launch_conv1x1g(a, PM_NONE, sums ? SM_BNBWD : SM_OFF, true, st, &R, &BN);
    if (e != hipSuccess || !sums) return e;
    return launch_bnbwd_sums_finalize(part, R, BN, N, invstd, sdz, sdzx, st,
                                      part + static_cast<size_t>(N / BN) * R * 2 * BN);
  }
  hipError_t e = launch_bwd(a, p, sums ? 2 : 1, st);
  if (e != hipSuccess || !sums) return e;
  conv1x1_bnbwd_finalize_kernel<<<(N + 7) / 8, 256, 0, st>>>(part, p.wgpn * p.WM, p.BN, N,
                                                             invstd, sdz, sdzx, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_conv1x1_link_s2(const void* x, const void* w, void* y, const void* link,
                                  int Nimg, int H, int W, int K, int N, hipStream_t st) {
  const int64_t M = static_cast<int64_t>(Nimg) * H * W;
  if (bad_shape(M, K, N)) return hipErrorInvalidValue;
  const Plan p = make_plan(M, K, N, 0, -1, true);
  C1Args a = base_args(x, w, y, M, K, N, p);
  a.link = reinterpret_cast<const uint16_t*>(link);
  a.link_s2 = 1;
  a.lW = W;
  a.lHW = H * W;
  a.lOW = (W + 1) / 2;
  a.lOHW = ((H + 1) / 2) * a.lOW;
  if (conv1x1g_pick(M, K, N, PM_NONE)) {
    int R, BN;
    return launch_conv1x1g(a, PM_NONE, SM_OFF, true, st, &R, &BN);
  }
  return launch_bwd(a, p, 1, st);
}

hipError_t launch_bn_stats_gram(const float* G, const float* cy, const void* w, int P, int Co,
                                int64_t M, float eps, float momentum, float* mean, float* invstd,
                                float* rmean, float* rvar, double* part, hipStream_t st,
                                const void* gamma, const void* beta, float* sc, float* bi) {
  if (P < 64 || P % 64 || P > 2048 || Co < 1 || M < 1 || !part) return hipErrorInvalidValue;
  if (sc && (!gamma || !beta || !bi)) return hipErrorInvalidValue;
  const size_t lds = static_cast<size_t>(kGramNC) * P * sizeof(float);
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bn_stats_gram_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  const uint16_t* W = reinterpret_cast<const uint16_t*>(w);
  bn_stats_gram_kernel<<<dim3((Co + kGramNC - 1) / kGramNC, P / 64), 256, lds, st>>>(G, W, P, Co,
                                                                                     part);
  bn_stats_gram_fin_kernel<<<(Co + 3) / 4, 256, 0, st>>>(
      part, cy, W, P, Co, M, eps, momentum, mean, invstd, rmean, rvar,
      reinterpret_cast<const uint16_t*>(gamma), reinterpret_cast<const uint16_t*>(beta), sc, bi);
  return hipGetLastError();
}

hipError_t launch_bn_bwd_coeffs(const float* sdz, const float* sdzx, const void* gamma,
                                const float* mean, const float* invstd, int C, int64_t M,
                                float* ca, float* cb, float* cc, void* dgamma, void* dbeta,
                                hipStream_t st) {
  bn_bwd_coeffs_kernel<<<(C + 255) / 256, 256, 0, st>>>(
      sdz, sdzx, reinterpret_cast<const uint16_t*>(gamma), mean, invstd, C,
      1.0f / static_cast<float>(M), ca, cb, cc, reinterpret_cast<uint16_t*>(dgamma),
      reinterpret_cast<uint16_t*>(dbeta));
  return hipGetLastError();
}

hipError_t launch_conv1x1_bnres(const void* x, const void* w, void* y, uint8_t* ymask,
                                const float* pro_sc, const float* pro_bi, const float* ep_sc,
                                const float* ep_bi, const void* res, int64_t M, int K, int N,
                                hipStream_t st) {
  if (bad_shape(M, K, N) || !pro_sc || !pro_bi || !ep_sc || !ep_bi || !res || !ymask)
    return hipErrorInvalidValue;
  const Plan p = make_plan(M, K, N, 2);   // the plan of the statistics pass (same z rounding)
  C1Args a = base_args(x, w, y, M, K, N, p);
  a.pro_sc = pro_sc;
  a.pro_bi = pro_bi;
  a.ep_sc = ep_sc;
  a.ep_bi = ep_bi;
  a.link = reinterpret_cast<const uint16_t*>(res);
  a.ymask = ymask;
  if (conv1x1g_pick(M, K, N, PM_BNRELU)) {
    int R, BN;
    return launch_conv1x1g(a, PM_BNRELU, SM_BNRES, false, st, &R, &BN);
  }
  return launch_tail(a, p, false, st);
}

hipError_t launch_conv1x1_cat(const void* g, const uint8_t* mask, const void* x2, const float* sc2,
                              const float* bi2, const float* bias, const void* w, void* y,
                              int64_t M, int K1, int K, int N, hipStream_t st, const float* mean,
                              const float* invstd, float* part, float* sdz, float* sdzx,
                              void* dgamma, void* dbeta) {
  if ((dgamma == nullptr) != (dbeta == nullptr) || (dgamma && !mean)) return hipErrorInvalidValue;
  if (bad_shape(M, K, N) || K1 % kBK || K1 <= 0 || K1 >= K || !mask || (!sc2 != !bi2))
    return hipErrorInvalidValue;
  const bool sums = mean != nullptr;
  // sums: the output is the gradient of the BN + ReLU whose input is x2 itself (N = K - K1)
  if (sums && (!invstd || !part || !sdz || !sdzx || N != K - K1 || !sc2)) return hipErrorInvalidValue;
  const Plan p = make_plan(M, K, N, 2, -1, !sums);   // (the sums' MT = 2 tile spills)
  C1Args a = base_args(g, w, y, M, K, N, p);
  a.xm = mask;
  a.x2 = reinterpret_cast<const uint16_t*>(x2);
  a.pro_sc2 = sc2;
  a.pro_bi2 = bi2;
  a.bias = bias;
  a.K1 = K1;
  if (sums) {
    a.sz = a.x2;
    a.ep_sc = sc2;   // the BN's own affine: the second source's prologue coefficients
    a.ep_bi = bi2;
    a.shift = mean;
    a.part = part;
  }
  if (conv1x1g_pick(M, K, N, PM_CAT)) {
    int R, BN;
    hipError_t e = launch_conv1x1g(a, PM_CAT, sums ? SM_BNBWD : SM_OFF, false, st, &R, &BN);
    if (e != hipSuccess || !sums) return e;
    return launch_bnbwd_sums_finalize(part, R, BN, N, invstd, sdz, sdzx, st,
                                      part + static_cast<size_t>(N / BN) * R * 2 * BN, dgamma,
                                      dbeta);
  }
  hipError_t e = launch_tail(a, p, true, st);
  if (e != hipSuccess || !sums) return e;
  conv1x1_bnbwd_finalize_kernel<<<(N + 7) / 8, 256, 0, st>>>(
      part, p.wgpn * p.WM, p.BN, N, invstd, sdz, sdzx, reinterpret_cast<uint16_t*>(dgamma),
      reinterpret_cast<uint16_t*>(dbeta));
  return hipGetLastError();
}

size_t conv1x1_cat_part_floats(int64_t M, int K, int N) {
  const Plan p = make_plan(M, K, N, 2, -1, false);
  const size_t g = conv1x1g_pick(M, K, N, PM_CAT) ? conv1x1g_part_floats(M, K, N, PM_CAT) : 0;
  return std::max(static_cast<size_t>(p.G) * p.WM * 2 * p.BN, g);
}

hipError_t launch_conv1x1_cat_bnres(const void* x1, const void* x2, const float* sc1,
                                    const float* bi1, const float* sc2, const float* bi2,
                                    const void* w, const float* ep_sc, const float* ep_bi,
                                    const void* res, void* y, uint8_t* ymask, int64_t M, int K1,
                                    int K, int N, hipStream_t st) {
  if (bad_shape(M, K, N) || K1 % kBK || K1 <= 0 || K1 >= K || !sc1 || !bi1 || (!sc2 != !bi2) ||
      !ep_sc || !ep_bi || !ymask)
    return hipErrorInvalidValue;
  const Plan p = make_plan(M, K, N, 2, -1, false);   // (its MT = 2 tile spills)
  C1Args a = base_args(x1, w, y, M, K, N, p);
  a.x2 = reinterpret_cast<const uint16_t*>(x2);
  a.pro_sc = sc1;
  a.pro_bi = bi1;
  a.pro_sc2 = sc2;
  a.pro_bi2 = bi2;
  a.K1 = K1;
  a.cat_bnrelu = 1;
  a.ep_sc = ep_sc;
  a.ep_bi = ep_bi;
  a.link = reinterpret_cast<const uint16_t*>(res);
  a.ymask = ymask;
  if (conv1x1g_pick(M, K, N, PM_CAT, true)) {
    int R, BN;
    return launch_conv1x1g(a, PM_CAT, SM_BNRES, false, st, &R, &BN);
  }
  return launch_tail(a, p, true, st);
}

hipError_t launch_conv1x1_bn_fwd(const void* x, const void* w, void* y, float* part,
                                 const float* pro_sc, const float* pro_bi, const float* shift,
                                 int64_t M, int K, int N, int stride, int H, int W, float* mean,
                                 float* invstd, float* rmean, float* rvar, float eps,
                                 float momentum, hipStream_t st, const BnAffineOut* aff) {
  if (K % kBK || N % 64 || M < 1 || M >= (1ll << 31) || K > 4096 || N > 4096)
    return hipErrorInvalidValue;
  if (stride != 1 && stride != 2) return hipErrorInvalidValue;
  const bool pro = pro_sc != nullptr;
  const Plan p = make_plan(M, K, N, pro ? 2 : 0);
  C1Args a{};
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.w = reinterpret_cast<const uint16_t*>(w);
  a.y = reinterpret_cast<uint16_t*>(y);
  a.part = part;
  a.pro_sc = pro_sc;
  a.pro_bi = pro_bi;
  a.shift = shift;
  a.M = static_cast<int>(M);
  a.K = K;
  a.N = N;
  a.ntn = p.ntn;
  a.wgpn = p.wgpn;
  a.mtiles = p.mtiles;
  if (stride == 2) {
    if (H % 2 || W % 2) return hipErrorInvalidValue;
    a.H = H;
    a.W = W;
    a.OW = W / 2;
    a.OHW = (H / 2) * (W / 2);
  }
  const bool s2 = stride == 2;
  if (!s2 && conv1x1g_pick(M, K, N, pro ? PM_BNRELU : PM_NONE)) {
    int R, BN;
    hipError_t e = launch_conv1x1g(a, pro ? PM_BNRELU : PM_NONE, SM_BN, false, st, &R, &BN);
    if (e != hipSuccess || !part || !mean) return e;
    return launch_bn_stats_finalize(part, R, BN, N, M, shift, eps, momentum, mean, invstd, rmean,
                                    rvar, st, part + static_cast<size_t>(N / BN) * R * 2 * BN, aff);
  }
  hipError_t e;
  if (p.WN == 4) e = launch_w<4, 1>(a, p, pro, s2, st);
  else if (p.WN == 2) e = launch_w<2, 2>(a, p, pro, s2, st);
  else e = launch_w<1, 4>(a, p, pro, s2, st);
  if (e != hipSuccess || !part || !mean) return e;
  return launch_bn_stats_finalize(part, p.wgpn * p.WM, p.BN, N, M, shift, eps, momentum, mean,
                                  invstd, rmean, rvar, st, nullptr, aff);
}

}  // namespace cml
