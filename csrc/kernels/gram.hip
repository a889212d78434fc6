// Krum / Multi-Krum / Weiszfeld / centered-clipping pairwise geometry: G = X X^T on MFMA (N06).
//
// X is worker-major [n, D] with n <= 64 and D up to billions: a tall-skinny reduction over D, not
// a classic GEMM. For G the A operand (X rows) and the B operand (X^T columns) are the SAME data,
// and on gfx950 the 16x16x32 bf16 MFMA gives lane l A[l&15][8(l>>4)+j] and B[8(l>>4)+j][l&15]:
// both are X[row l&15][k0 + 8(l>>4) + j]. So one 16-byte load per lane feeds both operands —
// no LDS staging, no transpose. Rows are grouped in TT tiles of 16 (n <= 16*TT); each wave keeps
// the upper-triangle tile accumulators (TT(TT+1)/2 x 4 fp32) in AGPRs and walks its own
// 128-column (256 B per row) slices; D is split across every wave of the grid (split-K).
// fp32 inputs use the exact-f32 16x16x4 MFMA with the same lane trick (float4 per lane feeds 4
// MFMAs). The kernel is HBM-bound: 1 KiB per wave-instruction, 4 MFMAs per 4 loads.
//
// Stage 1 writes one [P, P] fp32 partial per workgroup (fixed-order LDS reduction of its 4
// waves); stage 2 sums the partials in fp64 in block order -> bitwise reproducible G.
// Rows >= n load a valid duplicate row (same cache lines, coalesced in the same instruction) and
// are zeroed by a select, so no lane-divergent branch sits in front of the loads.
#include "common.h"
#include "kernels.h"

namespace cml {

namespace {
constexpr int kGBlock = 256;   // 4 waves
constexpr int kGWaves = kGBlock / kWave;
constexpr int kMaxGramBlocks = 1024;

typedef __bf16 mfma_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ mfma_bf16x8 as_frag(uint4 u) {
  return __builtin_bit_cast(mfma_bf16x8, u);
}

// Columns per wave per iteration.
template <typename T> struct GramCols;
template <> struct GramCols<bf16> { static constexpr int value = 128; };   // 4 x (16 rows x 32)
template <> struct GramCols<float> { static constexpr int value = 64; };   // 4 x (16 rows x 16)

template <typename T, int TT>
__global__ __launch_bounds__(kGBlock) void gram_partial_kernel(const T* __restrict__ X, int64_t ld,
                                                              int n, const int* __restrict__ rows,
                                                              int64_t D, float* __restrict__ part) {
  constexpr int P = 16 * TT;
  constexpr int NT = TT * (TT + 1) / 2;
  constexpr int COLS = GramCols<T>::value;
  __shared__ float red[kGWaves][P * P];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int h = lane >> 4;

  const T* rowp[TT];
  bool valid[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int row = 16 * t + r;
    valid[t] = row < n;
    const int rr = valid[t] ? row : (row % n);
    rowp[t] = X + static_cast<int64_t>(rows ? rows[rr] : rr) * ld;
  }

  f32x4 acc[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t gw = static_cast<int64_t>(blockIdx.x) * kGWaves + wave;
  const int64_t W = static_cast<int64_t>(gridDim.x) * kGWaves;
  const int64_t Dmain = (D / COLS) * COLS;

  if constexpr (sizeof(T) == 2) {
    for (int64_t k0 = gw * COLS; k0 < Dmain; k0 += W * COLS) {
      uint4 u[4][TT];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int t = 0; t < TT; ++t)
          u[q][t] = *reinterpret_cast<const uint4*>(rowp[t] + k0 + 32 * q + 8 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        mfma_bf16x8 f[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          uint4 z = valid[t] ? u[q][t] : make_uint4(0, 0, 0, 0);
          f[t] = as_frag(z);
        }
        int idx = 0;
#pragma unroll
        for (int ta = 0; ta < TT; ++ta)
#pragma unroll
          for (int tb = ta; tb < TT; ++tb) {
            acc[idx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[ta], f[tb], acc[idx], 0, 0, 0);
            ++idx;
          }
      }
    }
    // Tail columns [Dmain, D): one wave, element-wise guarded loads.
    if (gw == 0 && Dmain < D) {
      for (int64_t k0 = Dmain; k0 < D; k0 += 32) {
        mfma_bf16x8 f[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          uint16_t tmp[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int64_t c = k0 + 8 * h + j;
            tmp[j] = (valid[t] && c < D) ? reinterpret_cast<const uint16_t*>(rowp[t])[c] : 0;
          }
          uint4 z;
          z.x = tmp[0] | (uint32_t(tmp[1]) << 16);
          z.y = tmp[2] | (uint32_t(tmp[3]) << 16);
          z.z = tmp[4] | (uint32_t(tmp[5]) << 16);
          z.w = tmp[6] | (uint32_t(tmp[7]) << 16);
          f[t] = as_frag(z);
        }
        int idx = 0;
#pragma unroll
        for (int ta = 0; ta < TT; ++ta)
#pragma unroll
          for (int tb = ta; tb < TT; ++tb) {
            acc[idx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[ta], f[tb], acc[idx], 0, 0, 0);
            ++idx;
          }
      }
    }
  } else {
    for (int64_t k0 = gw * COLS; k0 < Dmain; k0 += W * COLS) {
      float4 u[4][TT];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int t = 0; t < TT; ++t)
          u[q][t] = *reinterpret_cast<const float4*>(rowp[t] + k0 + 16 * q + 4 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 f[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) f[t] = valid[t] ? u[q][t] : make_float4(0.f, 0.f, 0.f, 0.f);
        int idx = 0;
#pragma unroll
        for (int ta = 0; ta < TT; ++ta)
#pragma unroll
          for (int tb = ta; tb < TT; ++tb) {
            acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[ta].x, f[tb].x, acc[idx], 0, 0, 0);
            acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[ta].y, f[tb].y, acc[idx], 0, 0, 0);
            acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[ta].z, f[tb].z, acc[idx], 0, 0, 0);
            acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[ta].w, f[tb].w, acc[idx], 0, 0, 0);
            ++idx;
          }
      }
    }
    if (gw == 0 && Dmain < D) {
      for (int64_t k0 = Dmain; k0 < D; k0 += 4) {
        float f[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          const int64_t c = k0 + h;
          f[t] = (valid[t] && c < D) ? rowp[t][c] : 0.f;
        }
        int idx = 0;
#pragma unroll
        for (int ta = 0; ta < TT; ++ta)
#pragma unroll
          for (int tb = ta; tb < TT; ++tb) {
            acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[ta], f[tb], acc[idx], 0, 0, 0);
            ++idx;
          }
      }
    }
  }

  // C/D layout (16x16, dtype independent on gfx950): col = lane & 15, row = 4*(lane>>4) + j.
  float* mine = red[wave];
  {
    int idx = 0;
#pragma unroll
    for (int ta = 0; ta < TT; ++ta)
#pragma unroll
      for (int tb = ta; tb < TT; ++tb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = 16 * ta + 4 * h + j;
          const int col = 16 * tb + r;
          mine[row * P + col] = acc[idx][j];
        }
        ++idx;
      }
  }
  __syncthreads();
  float* out = part + static_cast<int64_t>(blockIdx.x) * P * P;
  for (int e = threadIdx.x; e < P * P; e += kGBlock) {
    const int row = e / P, col = e % P;
    float v = 0.f;
    if ((row / 16) <= (col / 16)) {   // only upper tiles were written
#pragma unroll
      for (int w = 0; w < kGWaves; ++w) v += red[w][e];
    }
    out[e] = v;
  }
}

__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ part, int nblk,
                                                         int P, int n, double* __restrict__ G,
                                                         int accumulate) {
  // one workgroup per Gram element: 256 lanes stride the partials, then a fixed-order LDS tree
  // (deterministic; one launch of P*P small workgroups instead of a serial 1024-deep loop)
  __shared__ double red[256];
  const int e = blockIdx.x;
  const int row = e / P, col = e % P;
  if (row >= n || col >= n || (row / 16) > (col / 16)) return;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x)
    s += static_cast<double>(part[static_cast<int64_t>(b) * P * P + e]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double v = red[0];
    if (accumulate) v += G[row * n + col];
    G[row * n + col] = v;
    if ((row / 16) < (col / 16)) G[col * n + row] = v;   // mirror off-diagonal tiles
  }
}

int gram_tiles(int n) { return (n + 15) / 16; }

int gram_blocks(int64_t D, int cols) {
  int64_t b = (D + cols * kGWaves - 1) / (cols * kGWaves);
  if (b > kMaxGramBlocks) b = kMaxGramBlocks;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

template <typename T, int TT>
void launch_gram_t(const T* X, int64_t ld, int n, const int* rows, int64_t D, float* part,
                   double* G, int acc, hipStream_t st) {
  const int nb = gram_blocks(D, GramCols<T>::value);
  gram_partial_kernel<T, TT><<<nb, kGBlock, 0, st>>>(X, ld, n, rows, D, part);
  gram_reduce_kernel<<<(16 * TT) * (16 * TT), 256, 0, st>>>(part, nb, 16 * TT, n, G, acc);
}
}  // namespace

size_t gram_workspace_bytes(int n, int64_t D) {
  const int P = 16 * gram_tiles(n);
  return static_cast<size_t>(kMaxGramBlocks) * P * P * sizeof(float);
}

hipError_t launch_gram(int dtype, const void* X, int64_t ld, int n, const int* rows, int64_t D,
                       void* work, double* G, int accumulate, hipStream_t stream) {
  if (n < 1 || n > 64 || D < 1) return hipErrorInvalidValue;
  const int es = dtype == DT_BF16 ? 2 : 4;
  const int vec = 16 / es;
  if ((ld % vec) != 0 || (reinterpret_cast<uintptr_t>(X) % 16) != 0) return hipErrorInvalidValue;
  float* part = reinterpret_cast<float*>(work);
  const int TT = gram_tiles(n);
  if (dtype == DT_BF16) {
    const bf16* x = reinterpret_cast<const bf16*>(X);
    switch (TT) {
      case 1: launch_gram_t<bf16, 1>(x, ld, n, rows, D, part, G, accumulate, stream); break;
      case 2: launch_gram_t<bf16, 2>(x, ld, n, rows, D, part, G, accumulate, stream); break;
      case 3: launch_gram_t<bf16, 3>(x, ld, n, rows, D, part, G, accumulate, stream); break;
      default: launch_gram_t<bf16, 4>(x, ld, n, rows, D, part, G, accumulate, stream); break;
    }
  } else {
    const float* x = reinterpret_cast<const float*>(X);
    switch (TT) {
      case 1: launch_gram_t<float, 1>(x, ld, n, rows, D, part, G, accumulate, stream); break;
      case 2: launch_gram_t<float, 2>(x, ld, n, rows, D, part, G, accumulate, stream); break;
      case 3: launch_gram_t<float, 3>(x, ld, n, rows, D, part, G, accumulate, stream); break;
      default: launch_gram_t<float, 4>(x, ld, n, rows, D, part, G, accumulate, stream); break;
    }
  }
  return hipGetLastError();
}

}  // namespace cml
