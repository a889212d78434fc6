// Fused 1x1 convolutions on the global_load_lds GEMM machinery of conv_gemm.hip: 256 x 256 output
// tiles, 8 waves of 64 (m) x 128 (n), both operands copied global -> LDS by the DMA path
// (global_load_lds_dwordx4, no VGPR staging), quad-phase ping-pong schedule (below). Same
// products and epilogues as conv1x1.hip:
//
//   y[m][n] = sum_k W[n][k] f(x[m][k])
//   f = identity                                   (PM_NONE)
//     = max(x sc[k] + bi[k], 0)                     (PM_BNRELU: the producer's BN + ReLU)
//     = a[k] (mask ? x : 0) + c[k]  for k < K1      (PM_CAT: a BN + ReLU backward of the block
//       max(x2 sc[k] + bi[k], 0)    for k >= K1      output gradient | a recomputed BN + ReLU
//                                                    output, one GEMM over two K-concatenated
//                                                    sources)
//
// conv1x1.hip transforms x while staging it through registers, which is what keeps its operand
// pipeline shallow (0.4-0.6 PFLOP/s on the compute-bound shapes). Here the DMA lands raw bf16 in
// LDS (its image must be lane-linear, so no transform on the way) and the prologue is applied in
// place in LDS once per staged x unit, with conv1x1.hip's arithmetic (same fmaf, same bf16
// rounding, packed VALU from common.h), so the operands -- and with the same k order the products
// -- are bit-identical. In production this kernel runs the downsample tails' forward GEMM (cat +
// BN + residual + ReLU epilogue) and the layer-2/3 recompute tails' data gradient (conv1x1g_pick);
// everything else is on conv1x1.hip.
//
// Epilogue: conv1x1_common.h's per-wave 64 x 64 block epilogue, called for each 64-channel half of
// the wave's tile through its own 8 KB LDS image (the staging buffers are free by then); BN
// statistics / BN-backward sums go to one partial row per (m-tile, wave row) of a tall slab that
// launch_bn_stats_finalize / launch_bnbwd_sums_finalize fold (fixed order, deterministic).
// Tiles are mapped XCD-aware: the n-tiles of one m-tile are consecutive on one XCD.
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "conv1x1_common.h"
#include "kernels.h"

namespace cml {
namespace {
using namespace c1;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

// f of one B fragment (8 channels k0 .. k0 + 7 of one pixel); sc / bi: the channels' coefficients
// MASKED: (bit ? x : 0) (the cat's first source; its BN-backward affine is folded into w and the
// epilogue bias), else max(x sc + bi, 0). Packed VALU (common.h): 4 / 5 instructions per pair.
template <bool MASKED>
__device__ __forceinline__ bf16x8_t prologue(bf16x8_t v, const float (&sc)[8], const float (&bi)[8],
                                             uint32_t bits) {
  uint4 u = *reinterpret_cast<const uint4*>(&v);
  if constexpr (MASKED) {
    u = make_uint4(mask_pk<0>(u.x, bits), mask_pk<1>(u.y, bits), mask_pk<2>(u.z, bits),
                   mask_pk<3>(u.w, bits));
  } else {
    u = make_uint4(bnrelu_pk(u.x, f32x2{sc[0], sc[1]}, f32x2{bi[0], bi[1]}),
                   bnrelu_pk(u.y, f32x2{sc[2], sc[3]}, f32x2{bi[2], bi[3]}),
                   bnrelu_pk(u.z, f32x2{sc[4], sc[5]}, f32x2{bi[4], bi[5]}),
                   bnrelu_pk(u.w, f32x2{sc[6], sc[7]}, f32x2{bi[6], bi[7]}));
  }
  return *reinterpret_cast<const bf16x8_t*>(&u);
}

// ---------------------------------------------------------------------------------------------
// Quad-phase ping-pong kernel (conv1x1q): 256 x 256 tiles for the compute-bound shapes (large K).
//
// A 2-buffer form (vmcnt(0) + barrier every k-step, so each step's DMA has one step of MFMA work
// to land in and every step ends in a drain; the "glds" family of rounds 2-3, slower than
// conv1x1.hip everywhere it was tried -- 128.7 ms/step with it everywhere, profiles/r03_17/ --
// and removed in round 4) is the baseline this replaces. Here the 64-deep k-step of a tile
// is split into four 16 KB "units" -- x rows 0-127 (X0), x rows 128-255 (X1), W rows 0-127 (W0)
// and W rows 128-255 (W1) -- with two slots each (k-step parity, 128 KB). Each k-step runs four
// phases; in each phase a wave multiplies one quadrant of its 64 (m) x 128 (n) output (32 pixels
// x 64 channels: its rows in x half mh, its channels in W half nh) over K = 64:
//
//   phase  quadrant   LDS reads (fragments)      DMA issued   wait        prologue (in LDS)
//     0    X0 x W0    X0 -> xf, W0 -> wc (kept)  X1(s+1)      -           X1(s)
//     1    X0 x W1    W1 -> wf                   W0(s+2)      -           -
//     2    X1 x W1    X1 -> xf                   X0(s+2)      X0(s+1)     -
//     3    X1 x W0    -                          W1(s+2)      X1(s+1)     X0(s+1)
//
// (the transforms sit in the phases with the fewest live fragment registers: the accumulators
// are 128 of the 256 registers a wave has at two waves per SIMD)
// so one unit is re-staged per phase, each into the slot its previous tile-step left one phase
// earlier, and 4 units (64 KB) stay in flight across barriers (counted vmcnt, raw s_barrier;
// a __syncthreads would drain the DMA queue). The prologue (f) is applied once per x unit, in
// place in LDS, by all threads, one phase after the wait that retired the unit's DMA and one
// phase before its first fragment read.
//
// Ping-pong: waves 4-7 (wn = 1) start one barrier late, so on every SIMD one wave multiplies while
// its partner reads fragments, issues DMA, transforms and waits. Each phase has two barriers: A
// (end of the load segment, after lgkmcnt(0): every ds_read / transform write of it has returned)
// and B (end of the MFMA segment). With the one-barrier stagger, a unit waited in phase p is
// visible to both groups from phase p + 1, and a slot whose last reads were in phase p may be
// re-staged from phase p + 1.
//
// Same products in the same k order and the same prologue arithmetic as conv1x1.hip: outputs are
// bit-identical to conv1x1.hip. Partial statistics rows per (m-tile, wave m-row), folded by the
// same finalize.
// The LDS accesses of the loop below, as functions with __restrict__ LDS operands: inlined, their
// loads and stores carry alias-scope metadata, which keeps hipcc's LDS-DMA tracking from putting
// an s_waitcnt vmcnt(0) in front of them (it drained every unit in flight twice per k-step,
// defeating the 4-units-in-flight schedule); the kernel orders the DMA itself (counted vmcnt +
// barriers, below).
__device__ __forceinline__ void q_rd_x(const char* __restrict__ sx, bf16x8_t (&xf)[4], int row,
                                       int h) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
    xf[kk] = *reinterpret_cast<const bf16x8_t*>(sx + swz(row, 2 * kk + h));
}
__device__ __forceinline__ void q_rd_w(const char* __restrict__ sw, bf16x8_t (&dst)[4][2],
                                       int row0, int h) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dst[kk][i] = *reinterpret_cast<const bf16x8_t*>(sw + swz(row0 + 32 * i, 2 * kk + h));
}
__device__ __forceinline__ void q_transform(char* __restrict__ sx, const float* __restrict__ sc_p,
                                            const float* __restrict__ bi_p,
                                            const uint8_t* __restrict__ smk, int tid,
                                            bool masked) {
  const int c = tid & 7;
  float sc[8], bi[8];
  ld8f(sc_p + 8 * c, sc);
  ld8f(bi_p + 8 * c, bi);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (tid >> 3) + 64 * i;
    bf16x8_t* q = reinterpret_cast<bf16x8_t*>(sx + swz(row, c));
    if (masked) *q = prologue<true>(*q, sc, bi, smk[row * 8 + c]);
    else *q = prologue<false>(*q, sc, bi, 0u);
  }
}

template <int PM, int SM, bool EL>
__global__ __launch_bounds__(512, 1) void conv1x1q_kernel(C1Args a) {
  constexpr int NT = 512, WM = 4, BM = 256, BN = 256;
  constexpr bool CAT = PM == PM_CAT, PRO = PM != PM_NONE;
  constexpr int UB = 128 * 128;                   // one unit: 128 rows x 128 B
  constexpr int GX = CAT ? 3 : 2;                 // DMA instructions per thread of an x unit
  constexpr int VQ = 4 + 2 * GX;                  // ... of the 4 units issued after a waited one
  constexpr int MKB = 2048;                       // CAT mask bytes per x slot (two copies)
  constexpr int SMASK = 8 * UB, SAFF = SMASK + (CAT ? 4 * MKB : 0);
  constexpr bool DM = CAT && SM == SM_BNBWD;
  constexpr bool STATS = SM == SM_BN || SM == SM_BNBWD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_aff = reinterpret_cast<float*>(smem + SAFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wn = wave >> 2;        // wn: the ping-pong group
  const int h = lane >> 5, r32 = lane & 31;
  const int G = a.ntn * a.mtiles, b = blockIdx.x, xcd = b & 7, q8 = G >> 3, r8 = G & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int mt = t / a.ntn, nt = t - mt * a.ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int K = a.K, KT = K / kBK;
  const int K1 = CAT ? a.K1 : K;

  if constexpr (PRO) fill_aff(a, CAT, s_aff, K, tid, NT);
  // staged rows of this thread in every unit: wave * 16 + 8 i + lane / 8 (i = 0, 1), 16-B chunk
  // lane & 7 of the row (source address inverse-swizzled: the DMA writes lane-linear)
  const int p = lane & 7, lrow = lane >> 3;
  // (addresses: a block-uniform base plus a 32-bit per-lane element offset, so the loop keeps
  // one register per DMA row instead of a 64-bit pointer per row and source)
  int xr[2][2];   // x row relative to m0 (clamped to M - 1: rows past M load a valid row)
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + 128 * u + wave * 16 + 8 * i + lrow;
      xr[u][i] = (m < a.M ? m : a.M - 1) - m0;
    }
  int mrow[2] = {0, 0};
  if constexpr (CAT) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = m0 + 128 * u + wm * 32 + (lane >> 1);
      mrow[u] = (m < a.M ? m : a.M - 1) - m0;
    }
  }
  auto slot = [&](int u, int s) { return smem + (((s & 1) << 2) + u) * UB; };
  auto mslot = [&](int u, int s) { return smem + SMASK + (((s & 1) << 1) + u) * MKB; };

  // unit u (0 X0, 1 X1, 2 W0, 3 W1) of k-step s: 2 DMA instructions per thread (+1 mask, CAT x)
  const int ab = a.ablate;
  auto issue = [&](int u, int s) {
    if (ab & 2) return;
    char* base = slot(u, s);
    const int k0 = s * kBK;
    if (u < 2) {
      const bool first = !CAT || k0 < K1;
      const int ld = first ? K1 : K - K1;
      const uint16_t* xb = first ? a.x + static_cast<int64_t>(m0) * K1 + k0
                                 : a.x2 + static_cast<int64_t>(m0) * (K - K1) + (k0 - K1);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = p ^ ((4 * i + (lrow >> 1)) & 7);   // (row >> 1) & 7 of row wave*16+8i+lrow
        __builtin_amdgcn_global_load_lds((g_void*)(xb + (xr[u][i] * ld + 8 * c)),
                                         (lds_void*)(base + (wave * 16 + 8 * i) * 128), 16, 0, 0);
      }
      if constexpr (CAT) {
        // 8 mask bytes per row at [row][8]; waves 4-7 load a second copy (every wave issues the
        // same DMA count). Second-source steps and cat_bnrelu: a dummy read, never used.
        const uint8_t* mb = a.cat_bnrelu ? reinterpret_cast<const uint8_t*>(a.x)
                                         : a.xm + static_cast<int64_t>(m0) * (K1 / 8) +
                                               (first ? k0 / 8 : 0);
        const int mo = a.cat_bnrelu ? 0 : mrow[u] * (K1 / 8) + 4 * (lane & 1);
        __builtin_amdgcn_global_load_lds((g_void*)(mb + mo), (lds_void*)(mslot(u, s) + wave * 256),
                                         4, 0, 0);
      }
    } else {
      const uint16_t* wb = a.w + static_cast<int64_t>(n0 + 128 * (u - 2)) * K + k0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = p ^ ((4 * i + (lrow >> 1)) & 7);
        __builtin_amdgcn_global_load_lds((g_void*)(wb + ((wave * 16 + 8 * i + lrow) * K + 8 * c)),
                                         (lds_void*)(base + (wave * 16 + 8 * i) * 128), 16, 0, 0);
      }
    }
  };
  // f in place on x unit u of step s: thread = chunk tid & 7 of rows tid / 8 and tid / 8 + 64
  auto transform = [&](int u, int s) {
    if (ab & 4) return;
    if constexpr (PRO) {
      const int k0 = s * kBK;
      const bool masked = CAT && k0 < K1 && !a.cat_bnrelu;
      if (CAT && k0 >= K1 && a.pro_sc2 == nullptr) return;   // identity second source
      q_transform(slot(u, s), s_aff + k0, s_aff + K + k0,
                  reinterpret_cast<const uint8_t*>(mslot(u, s)), tid, masked);
    }
  };

  bf16x8_t xf[4], wc[4][2], wf[4][2];
  auto rd_x = [&](int u, int s) { q_rd_x(slot(u, s), xf, wm * 32 + r32, h); };
  auto rd_w = [&](bf16x8_t (&dst)[4][2], int u, int s) {
    q_rd_w(slot(u, s), dst, wn * 64 + r32, h);
  };
  f32x16 acc[2][2][2];   // [x half][W half][32-channel fragment]
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[u][v][i][k] = 0.f;
  auto mma = [&](f32x16 (&ac)[2], const bf16x8_t (&wv)[4][2]) {
    if (ab & 1) return;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i) ac[i] = mfma32(wv[kk][i], xf[kk], ac[i]);
    __builtin_amdgcn_s_setprio(0);
  };
  // end of a load segment: this wave's LDS reads / writes returned, then the rendezvous
  auto bar_a = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto bar_b = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue: steps 0 and 1 (X1(1) is phase 0's DMA); X0(0) transformed, X1(0) landed
  // (in every phase the LDS reads and writes come before the DMA issue: hipcc waits vmcnt(0)
  // before an LDS access that follows a global_load_lds it cannot prove disjoint)
  issue(2, 0);
  issue(0, 0);
  issue(3, 0);
  issue(1, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // step 0 landed
  bar_a();                                           // ... in every wave
  transform(0, 0);
  issue(2, 1);
  issue(0, 1);
  issue(3, 1);
  bar_a();
  if (wn == 1) __builtin_amdgcn_s_barrier();   // ping-pong: group 1 one barrier behind

  for (int s = 0; s < KT; ++s) {
    const bool n1 = s + 1 < KT, n2 = s + 2 < KT;
    // ---- phase 0: X0 x W0
    rd_x(0, s);
    rd_w(wc, 2, s);
    transform(1, s);
    if (n1) issue(1, s + 1);
    bar_a();
    mma(acc[0][0], wc);
    bar_b();
    // ---- phase 1: X0 x W1
    rd_w(wf, 3, s);
    if (n2) issue(2, s + 2);
    bar_a();
    mma(acc[0][1], wf);
    bar_b();
    // ---- phase 2: X1 x W1
    rd_x(1, s);
    if (n2) issue(0, s + 2);
    if (n2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VQ) : "memory");   // X0(s+1), W0(s+1)
    else if (n1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + GX) : "memory");
    bar_a();
    mma(acc[1][1], wf);
    bar_b();
    // ---- phase 3: X1 x W0
    if (n1) transform(0, s + 1);
    if (n2) issue(3, s + 2);
    if (n2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 + GX) : "memory");   // X1(s+1), W1(s+1)
    else if (n1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar_a();
    mma(acc[1][0], wc);
    bar_b();
  }
  if (wn == 0) __builtin_amdgcn_s_barrier();   // equal barrier counts
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                             // staging area free for the epilogue images

  if (ab & 8) return;
  char* simg = smem + wave * 8192;
  float ss[8], sq[8], sh[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    ss[q] = 0.f;
    sq[q] = 0.f;
    sh[q] = 0.f;
  }
#pragma unroll
  for (int v = 0; v < 2; ++v) {               // W half: channels 128 v + 64 wn .. + 63
    const int ncol0 = 128 * v + 64 * wn;
    if constexpr (STATS) {
      if (a.shift) {
#pragma unroll
        for (int q = 0; q < 8; ++q) sh[q] = a.shift[n0 + ncol0 + 8 * (lane & 7) + q];
      }
    }
    f32x16 blk[2][2] = {{acc[0][v][0], acc[1][v][0]}, {acc[0][v][1], acc[1][v][1]}};
    epilogue<EL, SM, 2, DM, CAT && SM != SM_BNRES>(a, blk, ss, sq, sh, simg, m0 + wm * 32, ncol0,
                                                  n0, lane, m0 + 128 + wm * 32,
                                                  a.bias ? a.bias + n0 : nullptr);
    if (STATS && a.part) {
      float* pp = a.part + (static_cast<int64_t>(nt) * a.mtiles * WM + mt * WM + wm) * 2 * BN;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float sv = ss[q], qv = sq[q];
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) {
          sv += __shfl_xor(sv, o, 64);
          qv += __shfl_xor(qv, o, 64);
        }
        if (lane < 8) {
          pp[ncol0 + 8 * lane + q] = sv;
          pp[BN + ncol0 + 8 * lane + q] = qv;
        }
        ss[q] = 0.f;
        sq[q] = 0.f;
      }
    }
  }
}

struct GPlan {
  int BM, BN, WTN, ntn, mtiles;
  size_t lds;
};

GPlan gplan(int64_t M, int K, int N, int pm) {
  GPlan p{};
  p.BM = 256;
  p.BN = N % 256 == 0 ? 256 : 128;
  p.WTN = p.BN == 256 ? 128 : 64;
  p.ntn = N / p.BN;
  p.mtiles = static_cast<int>((M + p.BM - 1) / p.BM);
  const size_t sb = static_cast<size_t>(p.BM + p.BN) * 128 + (pm == PM_CAT ? p.BM * 8 : 0);
  p.lds = 2 * sb + (pm != PM_NONE ? static_cast<size_t>(2) * K * 4 : 0);
  return p;
}

size_t quad_lds(int K, int pm) {
  return static_cast<size_t>(8) * 128 * 128 + (pm == PM_CAT ? 4 * 2048 : 0) +
         (pm != PM_NONE ? static_cast<size_t>(2) * K * 4 : 0);
}

bool quad_eligible(int64_t M, int K, int N, int pm) {
  return N % 256 == 0 && K % kBK == 0 && K >= 2 * kBK && pm != PM_BNBWD &&
         quad_lds(K, pm) <= 160 * 1024;
}

template <int PM, int SM, bool EL>
hipError_t launch_q(const C1Args& a, const GPlan& p, hipStream_t st) {
  auto k = &conv1x1q_kernel<PM, SM, EL>;
  const size_t lds = quad_lds(a.K, PM);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  k<<<p.ntn * p.mtiles, 512, lds, st>>>(a);
  return hipGetLastError();
}

bool use_quad(int64_t M, int K, int N, int pm);

template <int PM, int SM, bool EL>
hipError_t launch_m(const C1Args& a, const GPlan& p, hipStream_t st) {
  if (use_quad(a.M, a.K, a.N, PM)) return launch_q<PM, SM, EL>(a, p, st);
  return hipErrorInvalidValue;   // conv1x1g_pick only picks quad-eligible shapes
}

}  // namespace

namespace {
// 0 off (conv1x1.hip), 2 auto (the shape policy below), 3 the quad-phase kernel wherever eligible
// (1, the removed 2-buffer kernel, reads as 0)
int g_mode = -1;

bool use_quad(int64_t M, int K, int N, int pm) {
  const int mode = conv1x1g_mode();
  if (!quad_eligible(M, K, N, pm)) return false;
  return mode == 3 || (mode == 2 && K >= 384);
}
}  // namespace

int conv1x1g_mode() {
  if (g_mode < 0) {
    const char* e = getenv("CML_C1G");
    g_mode = (!e || !strcmp(e, "auto")) ? 2 : atoi(e);
    if (g_mode < 0 || g_mode > 3) g_mode = 2;
    if (g_mode == 1) g_mode = 0;
  }
  return g_mode;
}

void set_conv1x1g_mode(int mode) { g_mode = mode == 1 ? 0 : mode; }

namespace {
int g_ablate = 0;
}  // namespace
void set_conv1x1g_ablate(int bits) { g_ablate = bits; }

bool conv1x1g_eligible(int64_t M, int K, int N, int pm) {
  if (K % kBK || N % 128 || K < kBK || M < 1 || M >= (1ll << 31) || N > 4096) return false;
  const GPlan p = gplan(M, K, N, pm);
  return p.lds <= 160 * 1024 && static_cast<int64_t>(p.ntn) * p.mtiles < (1ll << 31);
}

bool conv1x1g_pick(int64_t M, int K, int N, int pm, bool bnres) {
  const int mode = conv1x1g_mode();
  if (mode == 0 || !conv1x1g_eligible(M, K, N, pm)) return false;
  if (mode == 3) return use_quad(M, K, N, pm);
  // auto: since the packed prologues (round 3, profiles/r03_11_families.jsonl) the persistent
  // register-staged kernel is as fast or faster everywhere except the downsample tails' forward
  // GEMM (cat_bnres: 256 x 256 tiles, 1.14 / 0.92 vs 1.44 / 1.21 ms at batch 2048) ...
  // and the recompute tails' two-source data gradient with its BN-backward sums (K >= 384: layers
  // 2-3): 3.12 ms for its 6 calls vs ~3.46 on conv1x1.hip once the quad kernel's loop stopped
  // draining the DMA queue (profiles/r05_32/); CML_C1G_CAT=0 for the A/B
  static const bool cat = [] {
    const char* e = getenv("CML_C1G_CAT");
    return !(e && e[0] == '0');
  }();
  return pm == PM_CAT && (bnres || cat) && use_quad(M, K, N, pm);
}

size_t conv1x1g_part_floats(int64_t M, int K, int N, int pm) {
  const GPlan p = gplan(M, K, N, pm);
  const int R = p.mtiles * (p.BM / 64);
  return static_cast<size_t>(p.ntn) * (static_cast<size_t>(R) + bn_part_fold_slices(R, p.ntn)) *
         2 * p.BN;
}

hipError_t launch_conv1x1g(const C1Args& a0, int pm, int sm, bool el, hipStream_t st, int* R,
                           int* BN) {
  const GPlan p = gplan(a0.M, a0.K, a0.N, pm);
  C1Args a = a0;
  a.ablate = g_ablate;
  a.ntn = p.ntn;
  a.mtiles = p.mtiles;
  a.wgpn = 0;
  *R = p.mtiles * (p.BM / 64);
  *BN = p.BN;
  if (pm == PM_NONE && sm == SM_BN && !el) return launch_m<PM_NONE, SM_BN, false>(a, p, st);
  if (pm == PM_BNRELU && sm == SM_BN && !el) return launch_m<PM_BNRELU, SM_BN, false>(a, p, st);
  if (pm == PM_BNRELU && sm == SM_BNRES && !el) return launch_m<PM_BNRELU, SM_BNRES, false>(a, p, st);
  if (pm == PM_NONE && sm == SM_OFF && el) return launch_m<PM_NONE, SM_OFF, true>(a, p, st);
  if (pm == PM_NONE && sm == SM_BNBWD && el) return launch_m<PM_NONE, SM_BNBWD, true>(a, p, st);
  if (pm == PM_CAT && sm == SM_OFF && !el) return launch_m<PM_CAT, SM_OFF, false>(a, p, st);
  if (pm == PM_CAT && sm == SM_BNRES && !el) return launch_m<PM_CAT, SM_BNRES, false>(a, p, st);
  if (pm == PM_CAT && sm == SM_BNBWD && !el) return launch_m<PM_CAT, SM_BNBWD, false>(a, p, st);
  return hipErrorInvalidValue;
}

}  // namespace cml
