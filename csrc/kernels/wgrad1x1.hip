// Weight gradient of a stride-1 1x1 convolution on NHWC bf16 activations:
//   dW[co][ci] = sum_p dy[p][co] x[p][ci]      (p over N*H*W pixels)
// i.e. a GEMM whose reduction runs over the pixel dimension, which both operands store
// contiguously per pixel. ResNet-50's deeper 1x1 convs (128..2048 channels, 25k..800k pixels at
// batch 1024) are where MIOpen's weight-gradient kernels run at 1.4-3.7 TB/s and 0.5-0.6
// PFLOP/s (tools/diag/wgrad1x1_bench.py).
//
// Layout: a workgroup owns a 128 (co) x 128 (ci) tile of dW over a contiguous range of pixels
// (split-K; fp32 partials folded in a fixed order by wgrad1x1_fold_kernel). Per 64-pixel chunk
// (two LDS stages, one barrier per chunk)
// the dy and x slices are staged as [pixel][channel] 256-B rows (XOR-swizzled so the transposed
// reads are bank-conflict free) and both MFMA operands come out through ds_read_b64_tr_b16 (the
// gfx950 transpose read: k = pixel runs down the rows). 4 waves = 2 (co) x 2 (ci) halves of
// 64 x 64, four v_mfma_f32_32x32x16_bf16 accumulators each. The next chunk is prefetched into
// registers with unconditional (clamped) loads while the current one is multiplied.
#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;


__device__ __forceinline__ f32x16 mfma(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ s16x4 ld_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ bf16x8_t cat(s16x4 a, s16x4 b) {
  return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
// component-wise select: a select of whole uint4 values becomes a select of their addresses and
// pushes the prefetch registers into scratch memory
__device__ __forceinline__ uint4 keep_if(bool ok, uint4 v) {
  return make_uint4(ok ? v.x : 0u, ok ? v.y : 0u, ok ? v.z : 0u, ok ? v.w : 0u);
}
// byte offset of 16-B chunk ch of row `row` in a [rows][ROWB] image; the XOR spreads the 4 rows x
// 64 B of each transposed read over all 64 banks. 256-B (and 512-B) rows: every row starts on the
// same bank, so chunk bits 0..3 are permuted by the row. 128-B rows (64 channels): row parity
// already selects the bank half, and rows 2-3 of each group of 4 take the other 64 B of it.
template <int ROWB>
__device__ __forceinline__ int img_off(int row, int ch) {
  if constexpr (ROWB == 128) return ROWB * row + 16 * (ch ^ (((row >> 1) & 1) << 2));
  return ROWB * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// TM (co) x TN (ci) tile, (TM / 64) x (TN / 64) waves of 64 x 64 (four 32 x 32 accumulators).
// PRO: x is the pre-BN activation z of a BN + ReLU whose output the conv consumed; the staging
// applies max(z * sc[ci] + bi[ci], 0) (bf16-rounded, as the forward's prologue did), so the
// BN-ReLU output is never materialised (conv1x1.hip's prologue is the forward counterpart).
//
// DPRO: dy is the output gradient g of a BN + ReLU that consumed the conv's output z; the staging
// forms the conv's output gradient dz = da (mask ? g : 0) + db z + dc per output channel
// (conv1x1.hip's PM_BNBWD), so dz is never materialised either.
//   DP_MASK   dz = da (mask ? g : 0) + dc   (no z term: the tail recompute path supplies it
//             algebraically, ops.conv._RecomputeTailFn)
//   DP_BNRELU dz = max(g da + db, 0)        (dy is itself the input of a BN + ReLU: Gram matrices
//             of a BN-ReLU output that is never stored)
// CS (runtime, cs_part non-null): per-split column sums of the staged dz over the pixels
// (bf16 values as multiplied), taken by the workgroups of the first ci tile.
enum { DP_NONE = 0, DP_FULL = 1, DP_MASK = 2, DP_BNRELU = 3 };
struct DPro {
  const uint16_t* z;      // [P][Co]   (DP_FULL)
  const uint8_t* mask;    // [P][Co / 8] (DP_FULL, DP_MASK)
  const float* a;         // [Co]
  const float* b;         //           (DP_FULL, DP_BNRELU)
  const float* c;         //           (DP_FULL, DP_MASK)
};

template <int TM, int TN, int KC, bool PRO, int DPRO>
__global__ __launch_bounds__((TM / 64) * (TN / 64) * 64) void wgrad1x1_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, float* __restrict__ part,
    int P, int Co, int Ci, int tiles_n, int cps, const float* __restrict__ pro_sc,
    const float* __restrict__ pro_bi, DPro dp, float* __restrict__ cs_part) {
  constexpr int kKC = KC;                              // pixels per chunk
  constexpr int NT = (TM / 64) * (TN / 64) * 64;
  constexpr int CA = TM / 8, CB = TN / 8;            // 16-B chunks per staged row
  constexpr int IA = kKC * CA / NT, IB = kKC * CB / NT;   // staged items per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];   // 2 x {dy [KC][TM], x [KC][TN]}
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / (TN / 64), wn = wave % (TN / 64);
  const int h = lane >> 5, r = lane & 31;
  const int gi = lane & 15, grp = lane >> 4, q = gi >> 2, pq = gi & 3;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int co0 = tm * TM, ci0 = tn * TN;
  const int nchunk = (P + kKC - 1) / kKC;
  const int c_lo = blockIdx.y * cps;
  const int c_hi = min(nchunk, c_lo + cps);
  // every staged x item of this thread covers the same 8 channels (NT is a multiple of CB)
  float psc[8], pbi[8];
  if constexpr (PRO) {
    const int cb = ci0 + 8 * (tid % CB);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      psc[q] = pro_sc[cb + q];
      pbi[q] = pro_bi[cb + q];
    }
  }
  // likewise every staged dy item covers the same 8 output channels (NT is a multiple of CA)
  float da[8], db[8], dc[8];
  if constexpr (DPRO != DP_NONE) {
    const int cb = co0 + 8 * (tid % CA);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      da[q] = dp.a[cb + q];
      db[q] = DPRO == DP_MASK ? 0.f : dp.b[cb + q];
      dc[q] = DPRO == DP_BNRELU ? 0.f : dp.c[cb + q];
    }
  }
  auto dpro = [&](uint4 v, uint4 zv, uint32_t bits) {
    if constexpr (DPRO == DP_MASK || DPRO == DP_BNRELU) {
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float lo, hi;
        if constexpr (DPRO == DP_MASK) {
          const float glo = ((bits >> (2 * i)) & 1u) ? __uint_as_float(w4[i] << 16) : 0.f;
          const float ghi = ((bits >> (2 * i + 1)) & 1u) ? __uint_as_float(w4[i] & 0xffff0000u) : 0.f;
          lo = fmaf(da[2 * i], glo, dc[2 * i]);
          hi = fmaf(da[2 * i + 1], ghi, dc[2 * i + 1]);
        } else {
          lo = fmaxf(fmaf(__uint_as_float(w4[i] << 16), da[2 * i], db[2 * i]), 0.f);
          hi = fmaxf(fmaf(__uint_as_float(w4[i] & 0xffff0000u), da[2 * i + 1], db[2 * i + 1]), 0.f);
        }
        w4[i] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
      }
      return make_uint4(w4[0], w4[1], w4[2], w4[3]);
    } else if constexpr (DPRO == DP_FULL) {
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      const uint32_t z4[4] = {zv.x, zv.y, zv.z, zv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float glo = ((bits >> (2 * i)) & 1u) ? __uint_as_float(w4[i] << 16) : 0.f;
        const float ghi = ((bits >> (2 * i + 1)) & 1u) ? __uint_as_float(w4[i] & 0xffff0000u) : 0.f;
        const float lo = fmaf(da[2 * i], glo, fmaf(db[2 * i], __uint_as_float(z4[i] << 16), dc[2 * i]));
        const float hi = fmaf(da[2 * i + 1], ghi,
                              fmaf(db[2 * i + 1], __uint_as_float(z4[i] & 0xffff0000u), dc[2 * i + 1]));
        w4[i] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
      }
      return make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    return v;
  };
  auto pro = [&](uint4 v) {
    if constexpr (PRO) {
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float lo = fmaxf(fmaf(__uint_as_float(w4[i] << 16), psc[2 * i], pbi[2 * i]), 0.f);
        const float hi = fmaxf(fmaf(__uint_as_float(w4[i] & 0xffff0000u), psc[2 * i + 1], pbi[2 * i + 1]), 0.f);
        w4[i] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
      }
      return make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    return v;
  };
  // prefetch registers; loads are unconditional (clamped pixel, zeroed at use) and selects are
  // component-wise: a branch around the loads makes hipcc wait at the join, and a select of
  // whole uint4 values became a select of addresses that put these registers in scratch
  constexpr bool HZ = DPRO == DP_FULL, HM = DPRO == DP_FULL || DPRO == DP_MASK;
  uint4 av[IA], bv[IB], zv[HZ ? IA : 1];
  uint32_t mv[HM ? IA : 1];
  if constexpr (!HZ) zv[0] = make_uint4(0u, 0u, 0u, 0u);
  if constexpr (!HM) mv[0] = 0u;
  auto fetch = [&](int c) {
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int e = tid + NT * j, row = e / CA, ch = e % CA;
      const int p = min(c * kKC + row, P - 1);
      av[j] = *reinterpret_cast<const uint4*>(dy + static_cast<int64_t>(p) * Co + co0 + 8 * ch);
      if constexpr (HZ)
        zv[j] = *reinterpret_cast<const uint4*>(dp.z + static_cast<int64_t>(p) * Co + co0 + 8 * ch);
      if constexpr (HM) mv[j] = dp.mask[static_cast<int64_t>(p) * (Co / 8) + co0 / 8 + ch];
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int e = tid + NT * j, row = e / CB, ch = e % CB;
      const int p = min(c * kKC + row, P - 1);
      bv[j] = *reinterpret_cast<const uint4*>(x + static_cast<int64_t>(p) * Ci + ci0 + 8 * ch);
    }
  };
  f32x16 acc[2][2] = {};
  // two LDS stages: chunk c is multiplied out of stage c & 1 while chunk c + 1 is written into the
  // other stage from registers and chunk c + 2 is in flight -> one barrier per chunk
  constexpr int STG = kKC * (TM + TN) * 2;
  // (not in the 1024-thread tile: its 128 registers have no room for the sums)
  constexpr bool CSOK = NT <= 512;
  const bool csum = CSOK && cs_part != nullptr && tn == 0;   // uniform per workgroup
  float cs[CSOK ? 8 : 1];
#pragma unroll
  for (int q = 0; q < (CSOK ? 8 : 1); ++q) cs[q] = 0.f;
  auto stage = [&](int c, int sb) {
    char* ab = smem + sb * STG;
    char* bb = ab + kKC * TM * 2;
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int e = tid + NT * j, row = e / CA, ch = e % CA;
      uint4 v = av[j];
      if constexpr (DPRO != DP_NONE) v = dpro(v, zv[HZ ? j : 0], mv[HM ? j : 0]);
      v = keep_if(c * kKC + row < P, v);
      *reinterpret_cast<uint4*>(ab + img_off<TM * 2>(row, ch)) = v;
      if constexpr (CSOK) if (csum) {
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          cs[2 * i] += __uint_as_float(w4[i] << 16);
          cs[2 * i + 1] += __uint_as_float(w4[i] & 0xffff0000u);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int e = tid + NT * j, row = e / CB, ch = e % CB;
      *reinterpret_cast<uint4*>(bb + img_off<TN * 2>(row, ch)) =
          keep_if(c * kKC + row < P, pro(bv[j]));
    }
  };
  if (c_lo < c_hi) {
    fetch(c_lo);
    stage(c_lo, 0);
    fetch(c_lo + 1 < c_hi ? c_lo + 1 : c_lo);
  }
  __syncthreads();
  for (int c = c_lo; c < c_hi; ++c) {
    const int sb = (c - c_lo) & 1;
    const char* ab = smem + sb * STG;
    const char* bb = ab + kKC * TM * 2;
#pragma unroll
    for (int ks = 0; ks < kKC / 16; ++ks) {
      bf16x8_t A[2], B[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int r0 = 16 * ks + 8 * h + q;
        const int cha = 8 * wm + 4 * b + 2 * (grp & 1) + (pq >> 1);   // co chunk in the tile
        const int chb = 8 * wn + 4 * b + 2 * (grp & 1) + (pq >> 1);   // ci chunk in the tile
        A[b] = cat(ld_tr(ab + img_off<TM * 2>(r0, cha) + 8 * (pq & 1)),
                   ld_tr(ab + img_off<TM * 2>(r0 + 4, cha) + 8 * (pq & 1)));
        B[b] = cat(ld_tr(bb + img_off<TN * 2>(r0, chb) + 8 * (pq & 1)),
                   ld_tr(bb + img_off<TN * 2>(r0 + 4, chb) + 8 * (pq & 1)));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(A[i], B[j], acc[i][j]);
    }
    if (c + 1 < c_hi) {                                // uniform branch; loads stay unconditional
      stage(c + 1, sb ^ 1);
    }
    fetch(c + 2 < c_hi ? c + 2 : c);                   // past the end: reload a valid chunk
    __syncthreads();
  }
  if constexpr (CSOK) if (csum) {   // fold the threads of each 8-channel group (tid % CA)
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int q = 0; q < 8; ++q) red[tid * 8 + q] = cs[q];
    __syncthreads();
    if (tid < CA) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v = 0.f;
        for (int k = tid; k < NT; k += CA) v += red[k * 8 + q];
        cs_part[static_cast<int64_t>(blockIdx.y) * Co + co0 + 8 * tid + q] = v;
      }
    }
  }
  // partial [split][Co][Ci]: lane r = ci column, register k = co row (k&3) + 8 (k>>2) + 4 h
  float* pw = part + static_cast<int64_t>(blockIdx.y) * Co * Ci;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int co = co0 + 64 * wm + 32 * i + (k & 3) + 8 * (k >> 2) + 4 * h;
        const int ci = ci0 + 64 * wn + 32 * j + r;
        pw[static_cast<int64_t>(co) * Ci + ci] = acc[i][j][k];
      }
}

// dW = sum over S splits (fixed order), 4 elements per thread, bf16 or fp32 out
template <bool BF16>
__global__ __launch_bounds__(256) void wgrad1x1_fold_kernel(const float* __restrict__ part, int S,
                                                           int64_t n, void* __restrict__ out) {
  const int64_t e = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (e >= n) return;
  // 8 loads in flight per round (a one-load-per-iteration loop was latency-bound at ~1.7 TB/s);
  // the sum order is fixed: round by round, then split by split within a round
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int k = 0;
  for (; k + 8 <= S; k += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = *reinterpret_cast<const float4*>(part + static_cast<int64_t>(k + u) * n + e);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s.x += v[u].x;
      s.y += v[u].y;
      s.z += v[u].z;
      s.w += v[u].w;
    }
  }
  for (; k < S; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(part + static_cast<int64_t>(k) * n + e);
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  if constexpr (BF16) {
    uint2 o;
    o.x = static_cast<uint32_t>(f2bf(s.x)) | (static_cast<uint32_t>(f2bf(s.y)) << 16);
    o.y = static_cast<uint32_t>(f2bf(s.z)) | (static_cast<uint32_t>(f2bf(s.w)) << 16);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + e) = o;
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + e) = s;
  }
}

// The same fold for many splits over few outputs (Gram matrices / column sums of 64-channel
// activations: S up to 2048 over n = 64..4096, where the kernel above runs 1-16 workgroups whose
// threads each walk all S rows, ~27 us per call). Here 16 split lanes share 64 outputs: lane sl
// sums splits sl, sl + 16, ... (8 loads in flight; a wave reads 4 split rows x 256 contiguous B),
// then lane 0 adds the 16 lane sums in lane order. Fixed order: deterministic.
template <bool BF16>
__global__ __launch_bounds__(256) void wgrad_fold_wide_kernel(const float* __restrict__ part,
                                                              int S, int64_t n,
                                                              void* __restrict__ out) {
  __shared__ float4 red[16][17];
  const int cg = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int64_t e = (static_cast<int64_t>(blockIdx.x) * 16 + cg) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n) {
    int k = sl;
    for (; k + 7 * 16 < S; k += 8 * 16) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = *reinterpret_cast<const float4*>(part + static_cast<int64_t>(k + 16 * u) * n + e);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s.x += v[u].x;
        s.y += v[u].y;
        s.z += v[u].z;
        s.w += v[u].w;
      }
    }
    for (; k < S; k += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + static_cast<int64_t>(k) * n + e);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  red[sl][cg] = s;
  __syncthreads();
  if (sl != 0 || e >= n) return;
#pragma unroll
  for (int j = 1; j < 16; ++j) {
    const float4 v = red[j][cg];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  if constexpr (BF16) {
    uint2 o;
    o.x = static_cast<uint32_t>(f2bf(s.x)) | (static_cast<uint32_t>(f2bf(s.y)) << 16);
    o.y = static_cast<uint32_t>(f2bf(s.z)) | (static_cast<uint32_t>(f2bf(s.w)) << 16);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + e) = o;
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + e) = s;
  }
}

// Splits from which the wide fold is used (CML_FOLD_WIDE_MIN, default 32; 0 disables it: A/B).
int fold_wide_min() {
  static const int v = [] {
    const char* e = getenv("CML_FOLD_WIDE_MIN");
    return e ? atoi(e) : 32;
  }();
  return v;
}

// out[0:n] = sum over S rows of part [S][n] (n % 4 == 0), fixed order, bf16 or fp32 out.
void fold_splits(const float* part, int S, int64_t n, void* out, bool out_bf16, hipStream_t st) {
  const int wmin = fold_wide_min();
  if (wmin > 0 && S >= wmin) {
    const int64_t b = (n + 63) / 64;
    if (out_bf16) wgrad_fold_wide_kernel<true><<<static_cast<unsigned>(b), 256, 0, st>>>(part, S, n, out);
    else wgrad_fold_wide_kernel<false><<<static_cast<unsigned>(b), 256, 0, st>>>(part, S, n, out);
    return;
  }
  const int fb = static_cast<int>((n / 4 + 255) / 256);
  if (out_bf16) wgrad1x1_fold_kernel<true><<<fb, 256, 0, st>>>(part, S, n, out);
  else wgrad1x1_fold_kernel<false><<<fb, 256, 0, st>>>(part, S, n, out);
}

}  // namespace

namespace {
// tile choice: cover as much of the smaller channel dimension as possible so the larger operand
// is streamed once (x is re-read Co / TM times, dy Ci / TN times)
// (memory-bound shapes, Co * Ci <= 128K); shapes with more MACs per byte take 128 x 128 tiles
// for more workgroups (tools/diag/wgrad1x1_bench.py)
void pick_tile(int Co, int Ci, int* TM, int* TN, bool pro = false) {
  if (Co == 64 && Ci == 64) {   // Gram matrix of a 64-channel activation: one wave per tile
    *TM = 64;
    *TN = 64;
    return;
  }
  if (static_cast<int64_t>(Co) * Ci >= 256 * 1024) {
    *TM = 128;
    *TN = 128;
    return;
  }
  *TM = Co % 256 == 0 ? 256 : 128;
  *TN = Ci == 64 ? 64 : (Ci % 256 == 0 ? 256 : 128);
  if (*TN == 64) *TM = 256;   // 4 waves
  if (pro && *TM == 256 && *TN == 256) *TN = 128;   // the 1024-thread tile has no prologue variant
}
}  // namespace

template <int TM, int TN, bool PRO, int DPRO>
void launch_one(dim3 grid, size_t lds, hipStream_t st, const uint16_t* dyp, const uint16_t* xp,
                float* part, int P, int Co, int Ci, int tiles_n, int cps, const float* sc,
                const float* bi, const DPro& dp,
                float* cs_part = nullptr) {
  auto k = &wgrad1x1_kernel<TM, TN, 64, PRO, DPRO>;
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  k<<<grid, (TM / 64) * (TN / 64) * 64, lds, st>>>(dyp, xp, part, P, Co, Ci, tiles_n, cps, sc, bi,
                                                    dp, cs_part);
}

template <bool PRO, int DPRO>
bool launch_tile(int TM, int TN, dim3 grid, size_t lds, hipStream_t st, const uint16_t* dyp,
                 const uint16_t* xp, float* part, int P, int Co, int Ci, int tiles_n, int cps,
                 const float* sc, const float* bi, const DPro& dp, float* cs_part) {
  // (no prologue variant of the 1024-thread 256 x 256 tile: it spills, and no ResNet shape needs
  // it)
  if (TM == 256 && TN == 256) {
    if constexpr (PRO || DPRO != DP_NONE) return false;
    else launch_one<256, 256, PRO, DPRO>(grid, lds, st, dyp, xp, part, P, Co, Ci, tiles_n, cps, sc, bi, dp, cs_part);
  } else if (TM == 256 && TN == 128) launch_one<256, 128, PRO, DPRO>(grid, lds, st, dyp, xp, part, P, Co, Ci, tiles_n, cps, sc, bi, dp, cs_part);
  else if (TM == 128 && TN == 256) launch_one<128, 256, PRO, DPRO>(grid, lds, st, dyp, xp, part, P, Co, Ci, tiles_n, cps, sc, bi, dp, cs_part);
  else if (TM == 128 && TN == 128) launch_one<128, 128, PRO, DPRO>(grid, lds, st, dyp, xp, part, P, Co, Ci, tiles_n, cps, sc, bi, dp, cs_part);
  else if (TM == 256 && TN == 64) launch_one<256, 64, PRO, DPRO>(grid, lds, st, dyp, xp, part, P, Co, Ci, tiles_n, cps, sc, bi, dp, cs_part);
  else if (TM == 64 && TN == 64) launch_one<64, 64, PRO, DPRO>(grid, lds, st, dyp, xp, part, P, Co, Ci, tiles_n, cps, sc, bi, dp, cs_part);
  else return false;
  return true;
}

// pixels per chunk (128-pixel chunks for the 128 x 128 tile measured 5-15 % slower: more
// registers, fewer chunks per workgroup)
int chunk_of(int, int) { return 64; }

void wgrad1x1_plan(int64_t P, int Co, int Ci, int* splits, int* cps, bool pro) {
  int TM, TN;
  pick_tile(Co, Ci, &TM, &TN, pro);
  const int KC = chunk_of(TM, TN);
  const int tiles = (Co / TM) * (Ci / TN);
  const int waves = (TM / 64) * (TN / 64);
  const int nchunk = static_cast<int>((P + KC - 1) / KC);
  const int target = 256 * 8 / waves;                  // ~8 waves per CU in flight
  int s = (target + tiles - 1) / tiles;
  s = s < 1 ? 1 : (s > nchunk ? nchunk : s);
  const int c = (nchunk + s - 1) / s;
  *cps = c;
  *splits = (nchunk + c - 1) / c;
}

hipError_t launch_wgrad1x1(const void* dy, const void* x, float* part, void* dw, bool dw_bf16,
                           int64_t P, int Co, int Ci, const float* pro_sc, const float* pro_bi,
                           hipStream_t st, const void* dz_z, const uint8_t* dz_mask,
                           const float* dz_a, const float* dz_b, const float* dz_c) {
  return launch_wgrad1x1_ex(dy, x, part, dw, dw_bf16, P, Co, Ci, pro_sc, pro_bi, st,
                            dz_z ? DP_FULL : DP_NONE, dz_z, dz_mask, dz_a, dz_b, dz_c, nullptr,
                            nullptr);
}

hipError_t launch_wgrad1x1_ex(const void* dy, const void* x, float* part, void* dw, bool dw_bf16,
                              int64_t P, int Co, int Ci, const float* pro_sc, const float* pro_bi,
                              hipStream_t st, int dmode, const void* dz_z, const uint8_t* dz_mask,
                              const float* dz_a, const float* dz_b, const float* dz_c,
                              float* cs_part, float* cs) {
  if (dmode == DP_FULL && (!dz_z || !dz_mask || !dz_a || !dz_b || !dz_c)) return hipErrorInvalidValue;
  if (dmode == DP_MASK && (!dz_mask || !dz_a || !dz_c)) return hipErrorInvalidValue;
  if (dmode == DP_BNRELU && (!dz_a || !dz_b)) return hipErrorInvalidValue;
  if (dmode < DP_NONE || dmode > DP_BNRELU || ((cs_part == nullptr) != (cs == nullptr)))
    return hipErrorInvalidValue;
  {
    int tm, tn;
    pick_tile(Co, Ci, &tm, &tn, pro_sc != nullptr || dmode != DP_NONE || cs != nullptr);
    if (cs && tm * tn > 32768) return hipErrorInvalidValue;   // no column sums in that tile
  }
  DPro dp{reinterpret_cast<const uint16_t*>(dz_z), dz_mask, dz_a, dz_b, dz_c};
  if (!(Co == 64 && Ci == 64) && (Ci == 64 ? Co % 256 != 0 : (Co % 128 || Ci % 128)))
    return hipErrorInvalidValue;
  if (P < 1 || P >= (1ll << 31)) return hipErrorInvalidValue;
  if ((pro_sc == nullptr) != (pro_bi == nullptr)) return hipErrorInvalidValue;
  int S, cps, TM, TN;
  // (the column sums have no 1024-thread tile either: it takes the prologue tiles)
  const bool anypro = pro_sc != nullptr || dmode != DP_NONE || cs != nullptr;
  wgrad1x1_plan(P, Co, Ci, &S, &cps, anypro);
  pick_tile(Co, Ci, &TM, &TN, anypro);
  const int KC = chunk_of(TM, TN);
  const int tiles_n = Ci / TN;
  const dim3 grid((Co / TM) * tiles_n, S);
  const auto* dyp = reinterpret_cast<const uint16_t*>(dy);
  const auto* xp = reinterpret_cast<const uint16_t*>(x);
  const size_t lds = 2 * static_cast<size_t>(KC) * (TM + TN) * 2;   // two stages
  const int Pi = static_cast<int>(P);
  bool ok;
  const float* sc = pro_sc;
  const float* bi = pro_bi;
#define CML_WG_TILE(P_, D_) \
  launch_tile<P_, D_>(TM, TN, grid, lds, st, dyp, xp, part, Pi, Co, Ci, tiles_n, cps, sc, bi, dp, cs_part)
  if (pro_sc) {
    switch (dmode) {
      case DP_FULL: ok = CML_WG_TILE(true, DP_FULL); break;
      case DP_MASK: ok = CML_WG_TILE(true, DP_MASK); break;
      case DP_BNRELU: ok = CML_WG_TILE(true, DP_BNRELU); break;
      default: ok = CML_WG_TILE(true, DP_NONE);
    }
  } else {
    switch (dmode) {
      case DP_FULL: ok = CML_WG_TILE(false, DP_FULL); break;
      case DP_MASK: ok = CML_WG_TILE(false, DP_MASK); break;
      case DP_BNRELU: ok = CML_WG_TILE(false, DP_BNRELU); break;
      default: ok = CML_WG_TILE(false, DP_NONE);
    }
  }
#undef CML_WG_TILE
  if (!ok) return hipErrorInvalidValue;
  if (cs) fold_splits(cs_part, S, Co, cs, false, st);
  fold_splits(part, S, static_cast<int64_t>(Co) * Ci, dw, dw_bf16, st);
  return hipGetLastError();
}

hipError_t launch_wgrad_fold(const float* part, int S, int64_t n, void* out, bool out_bf16,
                             hipStream_t st) {
  if (S < 1 || n % 4) return hipErrorInvalidValue;
  fold_splits(part, S, n, out, out_bf16, st);
  return hipGetLastError();
}

}  // namespace cml
