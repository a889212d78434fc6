// Dense bf16 NT GEMM on 128 x 128 tiles, gfx950 / CDNA4: y[m][n] = bf16(acc + bias[n]) [+ cin].
//
// gemm.hip's 256 x 256 eight-wave tiles need >= 128 tiles to fill the chip; the transformer
// shapes of a DP rank are tall and skinny (BERT-base per-rank step: M = 8192 tokens, N = 768
// outputs -> 96 tiles of 256 x 256, 37 % of the CUs; hipBLASLt takes 7.2 ms of that 13.4 ms step,
// profiles/r04_30/bert_v1_kernels.md). This kernel covers those grids with 4-wave 128 x 128 tiles
// (384 tiles at 8192 x 768), two workgroups per CU:
//   * waves as 2 (m) x 2 (n), 64 x 64 outputs each = 4 x 4 accumulators of
//     v_mfma_f32_16x16x32_bf16, computed transposed (C^T = B A^T) so a lane holds 4 consecutive
//     output channels of one row;
//   * K in 64-deep tiles through two LDS buffers (A and B images of 128 rows x 128 B, the
//     XOR-swizzled layout of gemm.hip, swizzle applied to the per-lane SOURCE address since
//     global_load_lds writes lane-linear): the DMA of tile k + 1 is issued right after the barrier
//     that retires tile k and runs under tile k's MFMAs; one barrier per K-tile (the guide's
//     minimal two-phase schedule);
//   * epilogue: bias added in fp32 and rounded into a per-wave bf16 LDS image, read back as 16-B
//     row pieces (whole 128-B row segments per store instruction), + cin (the residual-gradient
//     add of a data gradient) in fp32, rounded once more -- gemm.hip EP_STORE's rounding points;
//   * tiles mapped XCD-aware (consecutive ids = the n-tiles of one m-tile share an XCD's L2).
// Requirements (checked by the launcher): M % 128 == 0, N % 128 == 0, K % 64 == 0, 16-B aligned
// rows.
#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

constexpr int kT = 128;                 // tile edge
constexpr int kBK = 64;                 // K per tile step
constexpr int kThreads = 256;
constexpr int kImg = kT * 128;          // one operand image (128 rows x 128 B)
constexpr int kBuf = 2 * kImg;          // A image + B image
constexpr int kLds = 2 * kBuf;          // 64 KB

__device__ __forceinline__ int swz(int row, int c) { return row * 128 + 16 * (c ^ ((row >> 1) & 7)); }

__device__ __forceinline__ f32x4 mfma16(bf16x8_t a, bf16x8_t b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(kThreads, 2) void gemm128_nt_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // ---- tile (bijective XCD remap: consecutive ids share an XCD; n fastest)
  const int ntn = static_cast<int>(a.N / kT);
  const int G = static_cast<int>(a.M / kT) * ntn, b = blockIdx.x, xcd = b & 7, q8 = G >> 3,
            r8 = G & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int mtile = t / ntn, ntile = t - mtile * ntn;
  const int64_t m0 = static_cast<int64_t>(mtile) * kT, n0 = static_cast<int64_t>(ntile) * kT;
  const int nk = static_cast<int>(a.K / kBK);

  // ---- staging: A and B rows of K-tile kt (16 + 16 wave-instructions of 8 rows x 128 B; this
  // wave's 4 + 4), lane = 16-B slot (lane & 7) of row (lane >> 3)
  const int lrow = lane >> 3, lp = lane & 7;
  auto stage = [&](int kt, int buf) {
    const int64_t kofs = static_cast<int64_t>(kt) * kBK;
    char* base = smem + buf * kBuf;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int row0 = (wave + 4 * s) * 8;
      const int row = row0 + lrow;
      const int c = lp ^ ((row >> 1) & 7);
      __builtin_amdgcn_global_load_lds((g_void*)(a.a + (m0 + row) * a.lda + kofs + 8 * c),
                                       (lds_void*)(base + row0 * 128), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((g_void*)(a.b + (n0 + row) * a.ldb + kofs + 8 * c),
                                       (lds_void*)(base + kImg + row0 * 128), 16, 0, 0);
    }
  };

  const int fr = lane & 15, fc = lane >> 4;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  // tile 0 landed: the barrier itself does not wait for global_load_lds, so this wave's DMAs are
  // waited first (as before every barrier below)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, buf ^ 1);   // buffer buf ^ 1 was retired by the barrier above
    const char* A = smem + buf * kBuf;
    const char* B = A + kImg;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(A + swz(wm * 64 + i * 16 + fr, fc + 4 * ks));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(B + swz(wn * 64 + j * 16 + fr, fc + 4 * ks));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // tile kt + 1 landed; every wave is done reading buffer buf
  }

  // ---- epilogue: bf16(acc + bias) into this wave's [64 m][64 n] image (128-B rows, swizzled),
  // read back as 16-B row pieces (+ cin), whole row segments per store instruction
  char* img = smem + wave * (64 * 128);
  float bias[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (a.bias) {
      const uint2 bv =
          *reinterpret_cast<const uint2*>(a.bias + n0 + wn * 64 + j * 16 + 4 * fc);
      bias[j][0] = __uint_as_float(bv.x << 16);
      bias[j][1] = __uint_as_float(bv.x & 0xffff0000u);
      bias[j][2] = __uint_as_float(bv.y << 16);
      bias[j][3] = __uint_as_float(bv.y & 0xffff0000u);
    } else {
      bias[j][0] = bias[j][1] = bias[j][2] = bias[j][3] = 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = acc[i][j];
      const uint2 w = make_uint2(pk_bf16(v[0] + bias[j][0], v[1] + bias[j][1]),
                                 pk_bf16(v[2] + bias[j][2], v[3] + bias[j][3]));
      *reinterpret_cast<uint2*>(img + swz(i * 16 + fr, j * 2 + (fc >> 1)) + 8 * (fc & 1)) = w;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int64_t ncol = n0 + wn * 64 + 8 * lp;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int row = 8 * it + lrow;
    uint4 v = *reinterpret_cast<const uint4*>(img + swz(row, lp));
    const int64_t m = m0 + wm * 64 + row;
    if (a.cin) {
      const uint4 c = *reinterpret_cast<const uint4*>(a.cin + m * a.ldy + ncol);
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w}, cc[4] = {c.x, c.y, c.z, c.w};
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = pk_bf16(__uint_as_float(vv[e] << 16) + __uint_as_float(cc[e] << 16),
                       __uint_as_float(vv[e] & 0xffff0000u) + __uint_as_float(cc[e] & 0xffff0000u));
      v = make_uint4(o[0], o[1], o[2], o[3]);
    }
    *reinterpret_cast<uint4*>(a.y + m * a.ldy + ncol) = v;
  }
}

}  // namespace

bool gemm128_eligible(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N > 0 && K > 0 && M % kT == 0 && N % kT == 0 && K % kBK == 0 &&
         (M / kT) * (N / kT) < (1LL << 31);
}

hipError_t launch_gemm128_nt(const GemmArgs& a, hipStream_t st) {
  if (!gemm128_eligible(a.M, a.N, a.K)) return hipErrorInvalidValue;
  if ((a.lda % 8) || (a.ldb % 8) || (a.ldy % 8)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(a.a) | reinterpret_cast<uintptr_t>(a.b) |
       reinterpret_cast<uintptr_t>(a.y) | reinterpret_cast<uintptr_t>(a.cin)) % 16)
    return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(a.bias) % 8) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(gemm128_nt_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int tiles = static_cast<int>((a.M / kT) * (a.N / kT));
  gemm128_nt_kernel<<<tiles, kThreads, kLds, st>>>(a);
  return hipGetLastError();
}

}  // namespace cml
