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

// ---- plain (no prologue) variant on LDS-DMA staging, deeper pipeline and 256-wide tiles.
//
// The register-staged kernel above keeps one 64-pixel chunk in flight per workgroup (the VGPRs
// it is prefetched into) and moves it to LDS with ds_write_b128 (~79 B/clk/CU); on the 14 x 14
// and 7 x 7 shapes that leaves it at 0.54-0.74 PFLOP/s, slower than MIOpen on (1024, 256) /
// (1024, 512) (profiles/r05_12/wgrad_lib.jsonl). Here:
//   * dy / x rows go global -> LDS by global_load_lds_dwordx4 (no VGPR staging, no LDS store
//     transfer), NS stages of 32 pixels, NS - 1 chunks in flight per workgroup; each wave waits
//     for its own DMAs of the chunk with a counted vmcnt, then one s_barrier per chunk (no
//     vmcnt(0) drain: __syncthreads would wait for the chunks still in flight);
//   * tiles of 256 (co) x 256 (ci) with 8 waves of 64 x 128 (x re-read Co / 256, dy Ci / 256
//     times instead of / 128), or 128 x 256 / 256 x 128 with 4 waves when a dimension is 128;
//   * the swizzle of the register-staged images (img_off) applied on the SOURCE side, since the
//     DMA writes each 1-KiB wave piece lane-linear; fragment reads unchanged (ds_read_b64_tr_b16);
//   * work items (split, tile) mapped XCD-aware: the tiles of one pixel range share an XCD's L2
//     (they read the same dy rows / x rows).
// Requires P % 32 == 0 and 16-B aligned rows (the launcher falls back otherwise).
constexpr int kDmaKC = 32;

// s_waitcnt vmcnt(N) expcnt(7) lgkmcnt(0) (gfx9 encoding: vmcnt bits 3:0 and 15:14)
template <int N>
__device__ __forceinline__ void vm_wait_lgkm0() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70);
}

// One staged chunk's MFMAs (wave tile 64 x 32 NB). The __restrict__ operands give the inlined
// LDS reads alias-scope metadata, which keeps the compiler's LDS-DMA tracking from putting a
// vmcnt(0) in front of them (it would wait for the chunks still in flight; the kernel orders the
// DMA itself: counted vmcnt + barrier).
template <int RA, int RB, int NB>
__device__ __forceinline__ void dma_chunk(const char* __restrict__ ab, const char* __restrict__ bb,
                                          f32x16 (&acc)[2][NB], int wm, int wn, int h, int q,
                                          int grp, int pq) {
#pragma unroll
  for (int ks = 0; ks < kDmaKC / 16; ++ks) {
    bf16x8_t A[2], B[NB];
    const int r0 = 16 * ks + 8 * h + q;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int cha = 8 * wm + 4 * e + 2 * (grp & 1) + (pq >> 1);
      A[e] = cat(ld_tr(ab + img_off<RA>(r0, cha) + 8 * (pq & 1)),
                 ld_tr(ab + img_off<RA>(r0 + 4, cha) + 8 * (pq & 1)));
    }
#pragma unroll
    for (int e = 0; e < NB; ++e) {
      const int chb = 4 * NB * wn + 4 * e + 2 * (grp & 1) + (pq >> 1);
      B[e] = cat(ld_tr(bb + img_off<RB>(r0, chb) + 8 * (pq & 1)),
                 ld_tr(bb + img_off<RB>(r0 + 4, chb) + 8 * (pq & 1)));
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int e = 0; e < NB; ++e) acc[a][e] = mfma(A[a], B[e], acc[a][e]);
  }
}

// S2: the B operand is the implicit im2col of a 3x3 / stride-2 / padding-1 conv's input:
// column n = tap * Ci + ci (tap = 3 dh + dw), row = output pixel o = (img, oh, ow) ->
// x[img][2 oh + dh - 1][2 ow + dw - 1][ci], or the zero row outside the image. A TN-wide column
// tile lies inside one tap (TN divides Ci), and the DMA source address is per lane, so the gather
// costs only its address arithmetic. dW comes out as [Co][tap][Ci] (channels_last [Co, Ci, 3, 3]).
struct DmaArgs {
  const uint16_t* dy;     // [P][Co]
  const uint16_t* x;      // [P][Ci] (1x1) or [img][H][W][Ci] (S2)
  const uint16_t* zero;   // >= 512 B of zeros (S2)
  float* part;            // [split][Co][ncol]
  int Co, ncol, Ci;       // ncol = Ci (1x1) or 9 Ci (S2)
  int tiles_n, tiles, nwork, nchunk, cps;
  int H, W, Ho, Wo;       // S2
  int tap0;               // S2: first tap (0: 3x3 / padding 1; 4: 1x1 / padding 0 = tap (1, 1) only)
  // XF modes (1x1 only): PRO x -> max(x sc + bi, 0); DPM dy -> da (mask ? dy : 0) + dc;
  // cs_part [split][Co]: column sums of the transformed dy (tn == 0 workgroups)
  const float* sc;
  const float* bi;
  const uint8_t* mask;    // [P][Co / 8]
  const float* da;
  const float* dc;
  float* cs_part;
  uint16_t* outb;         // one split: dW bf16 [Co][ncol] written directly (no partial, no fold)
};

// XF: the prologues of the register-staged kernel (PRO on x, DP_MASK on dy, column sums), applied
// once per element in LDS between the chunk's landing and its MFMAs (in place, 16-B items: a
// thread's items all cover the same 8 channels, so its affine constants sit in registers), with the
// same rounding points as the staging transforms above. Pipelined one chunk ahead: iteration i
// transforms chunk i + 1 while its waves multiply chunk i, so the transform costs LDS issue slots,
// not a serial phase. __restrict__ as in dma_chunk (no compiler vmcnt(0) before these accesses).
template <int RA, int RB, int NT, bool PRO, bool DPM>
__device__ __forceinline__ void dma_transform(char* __restrict__ ab, char* __restrict__ bb,
                                              const uint8_t* __restrict__ mk, int tid,
                                              const float (&psc)[8], const float (&pbi)[8],
                                              const float (&da)[8], const float (&dc)[8],
                                              float (&cs)[8], bool csum) {
  constexpr int CA = RA / 16, CB = RB / 16;   // 16-B chunks per row
  if constexpr (DPM) {
#pragma unroll
    for (int j = 0; j < kDmaKC * CA / NT; ++j) {
      const int e = tid + NT * j, row = e / CA, ch = e % CA;
      uint4* ptr = reinterpret_cast<uint4*>(ab + img_off<RA>(row, ch));
      const uint4 v = *ptr;
      const uint32_t bits = mk[row * CA + ch];
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float glo = ((bits >> (2 * i)) & 1u) ? __uint_as_float(w4[i] << 16) : 0.f;
        const float ghi = ((bits >> (2 * i + 1)) & 1u) ? __uint_as_float(w4[i] & 0xffff0000u) : 0.f;
        w4[i] = static_cast<uint32_t>(f2bf(fmaf(da[2 * i], glo, dc[2 * i]))) |
                (static_cast<uint32_t>(f2bf(fmaf(da[2 * i + 1], ghi, dc[2 * i + 1]))) << 16);
        if (csum) {
          cs[2 * i] += __uint_as_float(w4[i] << 16);
          cs[2 * i + 1] += __uint_as_float(w4[i] & 0xffff0000u);
        }
      }
      *ptr = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  }
  if constexpr (PRO) {
#pragma unroll
    for (int j = 0; j < kDmaKC * CB / NT; ++j) {
      const int e = tid + NT * j, row = e / CB, ch = e % CB;
      uint4* ptr = reinterpret_cast<uint4*>(bb + img_off<RB>(row, ch));
      const uint4 v = *ptr;
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float lo = fmaxf(fmaf(__uint_as_float(w4[i] << 16), psc[2 * i], pbi[2 * i]), 0.f);
        const float hi =
            fmaxf(fmaf(__uint_as_float(w4[i] & 0xffff0000u), psc[2 * i + 1], pbi[2 * i + 1]), 0.f);
        w4[i] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
      }
      *ptr = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  }
}

template <int TM, int TN, int NS, int WN, bool S2, bool PRO = false, bool DPM = false>
__global__ __launch_bounds__((TM / 64) * (TN / WN) * 64) void wgrad_dma_kernel(DmaArgs a) {
  constexpr int NW = (TM / 64) * (TN / WN), NB = WN / 32, NT = NW * 64;
  constexpr int RA = TM * 2, RB = TN * 2;                 // staged row bytes
  constexpr int LPA = RA / 16, LPB = RB / 16;             // lanes per row
  constexpr int IA = kDmaKC * LPA / 64, IB = kDmaKC * LPB / 64;   // 1-KiB pieces per chunk
  constexpr int L = (IA + IB) / NW;                       // pieces per wave per chunk
  constexpr bool XF = PRO || DPM;
  static_assert((IA + IB) % NW == 0 && IA % NW == 0, "piece split");
  static_assert(!DPM || TM == 256, "the mask tile is one 1-KiB piece: TM == 256");
  static_assert(!XF || (NT % LPA == 0 && NT % LPB == 0 && !S2), "transform items");
  constexpr int MSK = DPM ? kDmaKC * TM / 8 : 0;          // mask tile bytes per stage
  constexpr int STG = kDmaKC * (RA + RB) + MSK;
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) void g_void;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / (TN / WN), wn = wave % (TN / WN);
  const int h = lane >> 5, r = lane & 31;
  const int gi = lane & 15, grp = lane >> 4, q = gi >> 2, pq = gi & 3;

  // work item: bijective XCD remap (consecutive items on one XCD), tile fastest
  const int b = blockIdx.x, xcd = b & 7, q8 = a.nwork >> 3, r8 = a.nwork & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int split = t / a.tiles, tile = t - split * a.tiles;
  const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
  const int co0 = tm * TM, n0 = tn * TN;
  const int c_lo = split * a.cps;
  const int n = min(a.nchunk, c_lo + a.cps) - c_lo;
  // S2: this tile's tap and channel base (uniform)
  const int tq = S2 ? n0 / a.Ci : 0, tap = a.tap0 + tq, cb = S2 ? n0 - tq * a.Ci : n0;
  const int dh = tap / 3 - 1, dw = tap % 3 - 1;
  const int hw = a.Ho * a.Wo;

  // XF constants: a thread's transform items cover channels 8 (tid % (R / 16)) .. + 7
  float psc[8], pbi[8], da[8], dc[8], cs[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) psc[k] = pbi[k] = da[k] = dc[k] = cs[k] = 0.f;
  if constexpr (PRO) {
    const int c8 = cb + 8 * (tid % LPB);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      psc[k] = a.sc[c8 + k];
      pbi[k] = a.bi[c8 + k];
    }
  }
  if constexpr (DPM) {
    const int c8 = co0 + 8 * (tid % LPA);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      da[k] = a.da[c8 + k];
      dc[k] = a.dc[c8 + k];
    }
  }
  const bool csum = DPM && a.cs_part != nullptr && tn == 0;   // uniform per workgroup

  // this wave's pieces: j = wave + NW u; j < IA -> dy rows, else x rows; DPM: wave 0 also the
  // mask tile (32 rows x TM / 8 bytes = one piece)
  auto issue = [&](int c, int s) {
    char* base = smem + s * STG;
    const int64_t p0 = static_cast<int64_t>(c) * kDmaKC;
#pragma unroll
    for (int u = 0; u < L; ++u) {
      const int j = wave + NW * u;
      if (j < IA) {
        const int row0 = j * (64 / LPA), row = row0 + lane / LPA, pc = lane % LPA;
        const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
        __builtin_amdgcn_global_load_lds(
            (g_void*)(a.dy + (p0 + row) * a.Co + co0 + 8 * ch), (lds_void*)(base + row0 * RA), 16,
            0, 0);
      } else {
        const int jb = j - IA;
        const int row0 = jb * (64 / LPB), row = row0 + lane / LPB, pc = lane % LPB;
        const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
        const uint16_t* src;
        if constexpr (S2) {
          const int p = static_cast<int>(p0) + row, img = p / hw, rem = p - img * hw;
          const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
          const int ih = 2 * oh + dh, iw = 2 * ow + dw;
          src = (ih >= 0 && iw >= 0 && ih < a.H && iw < a.W)
                    ? a.x + ((static_cast<int64_t>(img) * a.H + ih) * a.W + iw) * a.Ci + cb + 8 * ch
                    : a.zero + 8 * ch;
        } else {
          src = a.x + (p0 + row) * a.Ci + cb + 8 * ch;
        }
        __builtin_amdgcn_global_load_lds((g_void*)src,
                                         (lds_void*)(base + kDmaKC * RA + row0 * RB), 16, 0, 0);
      }
    }
    if constexpr (DPM) {
      if (wave == 0)
        __builtin_amdgcn_global_load_lds(
            (g_void*)(a.mask + (p0 + (lane >> 1)) * (a.Co / 8) + co0 / 8 + 16 * (lane & 1)),
            (lds_void*)(base + kDmaKC * (RA + RB)), 16, 0, 0);
    }
  };
  auto xform = [&](int s) {
    char* ab = smem + s * STG;
    dma_transform<RA, RB, NT, PRO, DPM>(ab, ab + kDmaKC * RA,
                                        reinterpret_cast<const uint8_t*>(ab + kDmaKC * (RA + RB)),
                                        tid, psc, pbi, da, dc, cs, csum);
  };

  f32x16 acc[2][NB] = {};
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < n) issue(c_lo + s, s);
  // the DMA counts of this wave per chunk: L pieces (+ the mask piece on wave 0)
  const bool w0m = DPM && wave == 0;
  if constexpr (XF) {
    // chunk 0 landed everywhere, then transformed (the loop's first barrier publishes it)
    if (NS - 1 <= n) {
      if (w0m) vm_wait_lgkm0<(L + 1) * (NS - 2)>();
      else vm_wait_lgkm0<L * (NS - 2)>();
    } else {
      vm_wait_lgkm0<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    xform(0);
  }
  for (int i = 0; i < n; ++i) {
    if constexpr (XF) {
      // chunk i + 1 landed for this wave's pieces (and chunk i transformed: lgkmcnt(0)); every
      // wave done with chunk i - 1
      if (i + NS - 2 < n) {
        if (w0m) vm_wait_lgkm0<(L + 1) * (NS - 3)>();
        else vm_wait_lgkm0<L * (NS - 3)>();
      } else {
        vm_wait_lgkm0<0>();
      }
    } else {
      // chunk i landed for this wave's pieces; every wave done with chunk i - 1
      if (i + NS - 2 < n) vm_wait_lgkm0<L * (NS - 2)>();
      else vm_wait_lgkm0<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (i + NS - 1 < n) issue(c_lo + i + NS - 1, (i + NS - 1) % NS);
    if constexpr (XF)
      if (i + 1 < n) xform((i + 1) % NS);
    const char* ab = smem + (i % NS) * STG;
    dma_chunk<RA, RB, NB>(ab, ab + kDmaKC * RA, acc, wm, wn, h, q, grp, pq);
  }
  if constexpr (DPM) {
    if (csum) {   // fold the threads of each 8-channel group (tid % LPA), fixed order
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int k = 0; k < 8; ++k) red[tid * 8 + k] = cs[k];
      __syncthreads();
      if (tid < LPA) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float v = 0.f;
          for (int m = tid; m < NT; m += LPA) v += red[m * 8 + k];
          a.cs_part[static_cast<int64_t>(split) * a.Co + co0 + 8 * tid + k] = v;
        }
      }
    }
  }
  // partial [split][Co][ncol]: lane r = column, register k = co row (k&3) + 8 (k>>2) + 4 h
  if (a.outb != nullptr) {   // one split: bf16 dW, no fold (uniform branch)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < NB; ++e)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int co = co0 + 64 * wm + 32 * i + (k & 3) + 8 * (k >> 2) + 4 * h;
          const int col = n0 + WN * wn + 32 * e + r;
          a.outb[static_cast<int64_t>(co) * a.ncol + col] = f2bf(acc[i][e][k]);
        }
    return;
  }
  float* pw = a.part + static_cast<int64_t>(split) * a.Co * a.ncol;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < NB; ++e)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int co = co0 + 64 * wm + 32 * i + (k & 3) + 8 * (k >> 2) + 4 * h;
        const int col = n0 + WN * wn + 32 * e + r;
        pw[static_cast<int64_t>(co) * a.ncol + col] = acc[i][e][k];
      }
}

// dW = sum over S splits (fixed order), 4 elements per thread, bf16 or fp32 out
template <bool BF16>
__device__ __forceinline__ void fold_body(const float* __restrict__ part, int S, int64_t n,
                                          void* __restrict__ out, int64_t blk) {
  const int64_t e = (blk * 256 + threadIdx.x) * 4;
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

template <bool BF16>
__global__ __launch_bounds__(256) void wgrad1x1_fold_kernel(const float* __restrict__ part, int S,
                                                           int64_t n, void* __restrict__ out) {
  fold_body<BF16>(part, S, n, out, blockIdx.x);
}

// The same fold for many splits over few outputs (Gram matrices / column sums of 64-channel
// activations: S up to 2048 over n = 64..4096, where the kernel above runs 1-16 workgroups whose
// threads each walk all S rows, ~27 us per call). Here 16 split lanes share 64 outputs: lane sl
// sums splits sl, sl + 16, ... (8 loads in flight; a wave reads 4 split rows x 256 contiguous B),
// then lane 0 adds the 16 lane sums in lane order. Fixed order: deterministic.
template <bool BF16>
__device__ __forceinline__ void fold_wide_body(const float* __restrict__ part, int S, int64_t n,
                                               void* __restrict__ out, int64_t blk) {
  __shared__ float4 red[16][17];
  const int cg = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int64_t e = (blk * 16 + cg) * 4;
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

template <bool BF16>
__global__ __launch_bounds__(256) void wgrad_fold_wide_kernel(const float* __restrict__ part,
                                                              int S, int64_t n,
                                                              void* __restrict__ out) {
  fold_wide_body<BF16>(part, S, n, out, blockIdx.x);
}

// A weight gradient's two folds in one launch: blocks [0, b1) fold part -> out (dW, bf16 or fp32),
// blocks [b1, ..) fold part2 -> out2 (the column sums, fp32); the same per-element sums as two
// launches (the fold's fixed cost, ~5 us, is most of a column-sum fold)
template <bool WIDE, bool BF16>
__global__ __launch_bounds__(256) void fold_pair_kernel(const float* __restrict__ part, int64_t n,
                                                        void* __restrict__ out,
                                                        const float* __restrict__ part2,
                                                        int64_t n2, float* __restrict__ out2,
                                                        int S, int b1) {
  const int b = blockIdx.x;
  if (b < b1) {
    if constexpr (WIDE) fold_wide_body<BF16>(part, S, n, out, b);
    else fold_body<BF16>(part, S, n, out, b);
  } else {
    if constexpr (WIDE) fold_wide_body<false>(part2, S, n2, out2, b - b1);
    else fold_body<false>(part2, S, n2, out2, b - b1);
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

// dW = fold(part, n) and cs = fold(cs_part, ncs) (fp32) in one launch (cs null: dW only)
void fold_dw_cs(const float* part, int64_t n, void* dw, bool dw_bf16, const float* cs_part,
                int64_t ncs, float* cs, int S, hipStream_t st) {
  if (cs == nullptr) {
    fold_splits(part, S, n, dw, dw_bf16, st);
    return;
  }
  const int wmin = fold_wide_min();
  const bool wide = wmin > 0 && S >= wmin;
  const int64_t b1 = wide ? (n + 63) / 64 : (n / 4 + 255) / 256;
  const int64_t b2 = wide ? (ncs + 63) / 64 : (ncs / 4 + 255) / 256;
#define CML_FP(W, B)                                                                            \
  fold_pair_kernel<W, B><<<static_cast<unsigned>(b1 + b2), 256, 0, st>>>(part, n, dw, cs_part, \
                                                                        ncs, cs, S,            \
                                                                        static_cast<int>(b1))
  if (wide) {
    if (dw_bf16) CML_FP(true, true);
    else CML_FP(true, false);
  } else {
    if (dw_bf16) CML_FP(false, true);
    else CML_FP(false, false);
  }
#undef CML_FP
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

namespace {
// LDS-DMA kernel tile for a plain (no prologue / column sums) weight gradient, or false
// (CML_WGRAD_DMA=0 disables it: A/B)
bool dma_tile(int64_t P, int Co, int Ci, int* TM, int* TN) {
  static const bool on = [] {
    const char* e = getenv("CML_WGRAD_DMA");
    return !(e && e[0] == '0');
  }();
  if (!on || P < kDmaKC || P % kDmaKC || P >= (1ll << 31)) return false;
  if (Co % 256 == 0 && Ci % 256 == 0) { *TM = 256; *TN = 256; }
  else if (Co % 128 == 0 && Ci % 256 == 0) { *TM = 128; *TN = 256; }
  else if (Co % 256 == 0 && Ci % 128 == 0) { *TM = 256; *TN = 128; }
  else return false;
  return true;
}

void dma_plan(int64_t P, int Co, int ncol, int TM, int TN, int* splits, int* cps) {
  const int tiles = (Co / TM) * (ncol / TN);
  const int nchunk = static_cast<int>(P / kDmaKC);
  // one workgroup per CU (the LDS of the deep pipeline); two for the 64-KiB 128 x 128 tile
  int s = (TM == 128 && TN == 128 ? 512 : 256) / tiles;
  s = s < 1 ? 1 : (s > nchunk ? nchunk : s);
  const int c = (nchunk + s - 1) / s;
  *cps = c;
  *splits = (nchunk + c - 1) / c;
}

template <int TM, int TN, int NS, int WN, bool S2, bool PRO = false, bool DPM = false>
hipError_t launch_dma(DmaArgs a, int64_t P, int S, int cps, hipStream_t st) {
  constexpr int NW = (TM / 64) * (TN / WN);
  constexpr int lds = NS * (kDmaKC * (TM + TN) * 2 + (DPM ? kDmaKC * TM / 8 : 0));
  static_assert(lds <= 160 * 1024, "LDS");
  auto k = &wgrad_dma_kernel<TM, TN, NS, WN, S2, PRO, DPM>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  a.tiles_n = a.ncol / TN;
  a.tiles = (a.Co / TM) * a.tiles_n;
  a.nwork = a.tiles * S;
  a.nchunk = static_cast<int>(P / kDmaKC);
  a.cps = cps;
  k<<<a.nwork, NW * 64, lds, st>>>(a);
  return hipSuccess;
}

template <bool PRO, bool DPM>
hipError_t launch_dma_xf(int TM, int TN, const DmaArgs& a, int64_t P, int S, int cps,
                         hipStream_t st) {
  if (TM == 256 && TN == 256) return launch_dma<256, 256, 4, 128, false, PRO, DPM>(a, P, S, cps, st);
  if (TM == 256 && TN == 128) return launch_dma<256, 128, 6, 128, false, PRO, DPM>(a, P, S, cps, st);
  if constexpr (!DPM)
    if (TM == 128 && TN == 256) return launch_dma<128, 256, 6, 128, false, PRO, DPM>(a, P, S, cps, st);
  return hipErrorInvalidValue;
}

hipError_t launch_dma_tile(int TM, int TN, bool s2, const DmaArgs& a, int64_t P, int S, int cps,
                           hipStream_t st) {
  if (TM == 256 && TN == 256) return s2 ? launch_dma<256, 256, 4, 128, true>(a, P, S, cps, st)
                                        : launch_dma<256, 256, 4, 128, false>(a, P, S, cps, st);
  if (TM == 128 && TN == 256) return s2 ? launch_dma<128, 256, 6, 128, true>(a, P, S, cps, st)
                                        : launch_dma<128, 256, 6, 128, false>(a, P, S, cps, st);
  if (TM == 256 && TN == 128) return s2 ? launch_dma<256, 128, 6, 128, true>(a, P, S, cps, st)
                                        : launch_dma<256, 128, 6, 128, false>(a, P, S, cps, st);
  if (TM == 128 && TN == 128 && s2) {
    // 8 stages (1 workgroup / CU) or 4 (2 workgroups / CU): CML_WGRAD_DMA_NS128 (A/B)
    static const int ns = [] {
      const char* e = getenv("CML_WGRAD_DMA_NS128");
      return e ? atoi(e) : 4;
    }();
    return ns == 8 ? launch_dma<128, 128, 8, 64, true>(a, P, S, cps, st)
                   : launch_dma<128, 128, 4, 64, true>(a, P, S, cps, st);
  }
  return hipErrorInvalidValue;
}

// DMA eligibility of a wgrad1x1 call: plain; x prologue (PRO); DP_MASK dy prologue (TM 256),
// with its column sums. CML_WGRAD_DMA_XF=0 keeps the prologue variants on the register-staged
// kernel (A/B).
bool dma_ok(int64_t P, int Co, int Ci, bool pro, int dmode, bool cs, int* TM, int* TN) {
  static const bool xf = [] {
    const char* e = getenv("CML_WGRAD_DMA_XF");
    return !(e && e[0] == '0');
  }();
  if (dmode != DP_NONE && dmode != DP_MASK) return false;
  if (cs && dmode != DP_MASK) return false;
  if ((pro || dmode != DP_NONE) && !xf) return false;
  if (!dma_tile(P, Co, Ci, TM, TN)) return false;
  // the 4-wave 256 x 128 tile with prologues ran the layer-2 tail (Co 512, Ci 128, 1.6 M pixels)
  // at 727 us vs 459 on the staged kernel (profiles/r05_17/): one wave per SIMD carrying both the
  // transforms and the MFMAs
  if ((pro || dmode != DP_NONE) && *TN == 128) return false;
  return dmode != DP_MASK || *TM == 256;
}

// stride-2 3x3 tiles: TN divides Ci (a column tile inside one tap)
bool s2_tile(int N, int H, int W, int Co, int Ci, int* TM, int* TN) {
  if (N < 1 || H < 2 || W < 2 || (H & 1) || (W & 1) || Co % 128 || Ci % 128) return false;
  const int64_t P = static_cast<int64_t>(N) * (H / 2) * (W / 2);
  if (P % kDmaKC || P >= (1ll << 31) || static_cast<int64_t>(N) * H * W * Ci >= (1ll << 40))
    return false;
  *TM = Co % 256 == 0 ? 256 : 128;
  *TN = Ci % 256 == 0 ? 256 : 128;
  return true;
}
}  // namespace

void staged_plan(int64_t P, int Co, int Ci, int* splits, int* cps, bool pro);

void wgrad1x1_plan(int64_t P, int Co, int Ci, int* splits, int* cps, bool pro, int dmode,
                   bool cs) {
  int TM, TN;
  if (dma_ok(P, Co, Ci, pro, dmode, cs, &TM, &TN)) {
    dma_plan(P, Co, Ci, TM, TN, splits, cps);
    return;
  }
  staged_plan(P, Co, Ci, splits, cps, pro || dmode != DP_NONE || cs);
}

bool wgrad1x1_direct(int64_t P, int Co, int Ci, bool pro, int dmode, bool cs) {
  int TM, TN, S, cps;
  if (cs || !dma_ok(P, Co, Ci, pro, dmode, cs, &TM, &TN)) return false;
  dma_plan(P, Co, Ci, TM, TN, &S, &cps);
  return S == 1;
}

// plan of the register-staged kernel (pro: any prologue or column sums)
void staged_plan(int64_t P, int Co, int Ci, int* splits, int* cps, bool pro) {
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
  if (dma_ok(P, Co, Ci, pro_sc != nullptr, dmode, cs != nullptr, &TM, &TN)) {
    // (the caller sized `part` from this plan: no fallback to the staged kernel's splits)
    if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x)) % 16)
      return hipErrorInvalidValue;
    dma_plan(P, Co, Ci, TM, TN, &S, &cps);
    // one split, no column sums: the kernel writes dW itself (wgrad1x1_direct; part may be null)
    const bool direct = S == 1 && cs == nullptr;
    if (!direct && part == nullptr) return hipErrorInvalidValue;
    DmaArgs da{};
    da.dy = reinterpret_cast<const uint16_t*>(dy);
    da.x = reinterpret_cast<const uint16_t*>(x);
    da.part = direct && !dw_bf16 ? reinterpret_cast<float*>(dw) : part;
    da.outb = direct && dw_bf16 ? reinterpret_cast<uint16_t*>(dw) : nullptr;
    da.Co = Co;
    da.ncol = Ci;
    da.Ci = Ci;
    da.sc = pro_sc;
    da.bi = pro_bi;
    da.mask = dz_mask;
    da.da = dz_a;
    da.dc = dz_c;
    da.cs_part = cs_part;
    hipError_t e;
    const bool dpm = dmode == DP_MASK;
    if (pro_sc && dpm) e = launch_dma_xf<true, true>(TM, TN, da, P, S, cps, st);
    else if (pro_sc) e = launch_dma_xf<true, false>(TM, TN, da, P, S, cps, st);
    else if (dpm) e = launch_dma_xf<false, true>(TM, TN, da, P, S, cps, st);
    else e = launch_dma_tile(TM, TN, false, da, P, S, cps, st);
    if (e != hipSuccess) return e;
    if (direct) return hipGetLastError();
    fold_dw_cs(part, static_cast<int64_t>(Co) * Ci, dw, dw_bf16, cs_part, Co, cs, S, st);
    return hipGetLastError();
  }
  if (part == nullptr) return hipErrorInvalidValue;
  staged_plan(P, Co, Ci, &S, &cps, anypro);
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
  fold_dw_cs(part, static_cast<int64_t>(Co) * Ci, dw, dw_bf16, cs_part, Co, cs, S, st);
  return hipGetLastError();
}

bool wgrad3x3s2_plan(int N, int H, int W, int Co, int Ci, int* splits, int taps) {
  int TM, TN, cps;
  if ((taps != 9 && taps != 1) || !s2_tile(N, H, W, Co, Ci, &TM, &TN)) return false;
  dma_plan(static_cast<int64_t>(N) * (H / 2) * (W / 2), Co, taps * Ci, TM, TN, splits, &cps);
  return true;
}

hipError_t launch_wgrad3x3s2(const void* dy, const void* x, const void* zero, float* part,
                             void* dw, bool dw_bf16, int N, int H, int W, int Co, int Ci,
                             hipStream_t st, int taps) {
  int TM, TN, S, cps;
  if ((taps != 9 && taps != 1) || !s2_tile(N, H, W, Co, Ci, &TM, &TN)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) |
       reinterpret_cast<uintptr_t>(zero)) % 16)
    return hipErrorInvalidValue;
  const int64_t P = static_cast<int64_t>(N) * (H / 2) * (W / 2);
  dma_plan(P, Co, taps * Ci, TM, TN, &S, &cps);
  DmaArgs da{};
  da.dy = reinterpret_cast<const uint16_t*>(dy);
  da.x = reinterpret_cast<const uint16_t*>(x);
  da.zero = reinterpret_cast<const uint16_t*>(zero);
  da.part = part;
  da.Co = Co;
  da.ncol = taps * Ci;
  da.tap0 = taps == 1 ? 4 : 0;
  da.Ci = Ci;
  da.H = H;
  da.W = W;
  da.Ho = H / 2;
  da.Wo = W / 2;
  const hipError_t e = launch_dma_tile(TM, TN, true, da, P, S, cps, st);
  if (e != hipSuccess) return e;
  fold_splits(part, S, static_cast<int64_t>(Co) * taps * Ci, dw, dw_bf16, st);
  return hipGetLastError();
}

hipError_t launch_wgrad_fold(const float* part, int S, int64_t n, void* out, bool out_bf16,
                             hipStream_t st) {
  if (S < 1 || n % 4) return hipErrorInvalidValue;
  fold_splits(part, S, n, out, out_bf16, st);
  return hipGetLastError();
}

}  // namespace cml
