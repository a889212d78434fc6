// Krum / Multi-Krum / Weiszfeld / centered-clipping pairwise geometry: G = X X^T on MFMA (N06).
//
// X is worker-major [n, D] with n <= 64 and D up to billions: a tall-skinny reduction over D, not
// a classic GEMM. For G the A operand (X rows) and the B operand (X^T columns) are the SAME data,
// and on gfx950 the 16x16x32 bf16 MFMA gives lane l A[l&15][8(l>>4)+j] and B[8(l>>4)+j][l&15]:
// both are X[row l&15][k0 + 8(l>>4) + j]. So one 16-byte load per lane feeds both operands —
// no LDS staging, no transpose. Rows are grouped in TT tiles of 16 (n <= 16*TT); each wave keeps
// the upper-triangle tile accumulators (TT(TT+1)/2 x 4 fp32) in AGPRs and walks its own column
// slices; D is split across every wave of the grid (split-K). fp32 inputs use the exact-f32
// 16x16x4 MFMA with the same lane trick (float4 per lane feeds 4 MFMAs).
//
// Small n (<= 8, the common "one row per GPU" case): a 16-row tile would leave 16-n lanes
// re-loading duplicate rows. Instead the 16 MFMA rows are G = 16/P2 "virtual rows" per real row
// (P2 = next pow2 >= n): virtual row g*P2 + i reads row i over column group g. The MFMA then
// produces a block matrix whose diagonal P2 x P2 blocks are partial Grams over disjoint column
// groups (off-diagonal blocks are cross-group products and are discarded); summing the diagonal
// blocks gives X X^T. Every lane loads unique bytes, so HBM bytes in flight per wave double
// (n = 8) or more. Each lane keeps Q 16-byte loads in flight per iteration (Q = 8 for n <= 32).
//
// Centered Gram (center != null): every row is taken relative to worker row *center,
// G'_ij = (x_i - x_c) . (x_j - x_c). Every quantity the Gram-space rules read is translation
// invariant (pairwise distances; distances to an affine combination sum_j a_j x_j with
// sum a = 1) -- and that holds coordinate by coordinate, so the center may be ANY vector: a
// non-finite element of row c is replaced by 0, which keeps every finite row finite when the
// center worker has turned non-finite. G' gives the same weights -- but without the
// cancellation of
// d_ij = G_ii + G_jj - 2 G_ij when the workers are near-duplicates (|x_i - x_j| << |x|): the fp32
// MFMA partials then carry ~1e-6 of |x|^2, which is all of d_ij for a tight honest cluster. The
// difference is formed in fp32 (exact for bf16 inputs) and rounded once to the MFMA input type.
// gram_center_kernel picks the center: the medoid (least summed squared distance to the finite
// rows) of a G; the engine uses the medoid of step t - 1 as step t's center, so one centered pass
// per step suffices (the medoid of an honest cluster stays inside it from step to step).
//
// A negative *center means "no center this step" (the weights kernel's guard sets it when a
// centered pass looked captured, see weights.hip): the pass runs uncentered.
//
// Stage 1 writes one [P, P] fp32 partial per workgroup (fixed-order LDS reduction of its 4
// waves, folded over column groups); stage 2 sums the partials in fp64 in block order ->
// bitwise reproducible G. Rows >= n load a valid duplicate row and are zeroed by a select, so
// no lane-divergent branch sits in front of the loads.
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

// Elements per lane-load (16 B) and columns covered by one load instruction of the wave.
template <typename T> struct GramVec;
template <> struct GramVec<bf16> { static constexpr int vec = 8, step = 32; };
template <> struct GramVec<float> { static constexpr int vec = 4, step = 16; };

template <int TT> struct GramQ { static constexpr int value = TT <= 2 ? 8 : 4; };

// Columns one wave consumes per main-loop iteration.
template <typename T, int TT, int G>
constexpr int gram_cols() { return G * GramQ<TT>::value * GramVec<T>::step; }

// acc[idx] += frag(ta) x frag(tb) over the upper-triangle tiles.
template <int TT>
__device__ __forceinline__ void gram_mfma(f32x4* acc, const uint4* u) {
  int idx = 0;
#pragma unroll
  for (int ta = 0; ta < TT; ++ta)
#pragma unroll
    for (int tb = ta; tb < TT; ++tb) {
      acc[idx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(u[ta]), as_frag(u[tb]), acc[idx],
                                                         0, 0, 0);
      ++idx;
    }
}

template <int TT>
__device__ __forceinline__ void gram_mfma(f32x4* acc, const float4* u) {
  int idx = 0;
#pragma unroll
  for (int ta = 0; ta < TT; ++ta)
#pragma unroll
    for (int tb = ta; tb < TT; ++tb) {
      acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[ta].x, u[tb].x, acc[idx], 0, 0, 0);
      acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[ta].y, u[tb].y, acc[idx], 0, 0, 0);
      acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[ta].z, u[tb].z, acc[idx], 0, 0, 0);
      acc[idx] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[ta].w, u[tb].w, acc[idx], 0, 0, 0);
      ++idx;
    }
}

template <typename T> struct GramLoad;
template <> struct GramLoad<bf16> {
  typedef uint4 type;
  static __device__ __forceinline__ uint4 zero() { return make_uint4(0, 0, 0, 0); }
  // a - c elementwise (fp32 difference of two bf16 values, rounded once to bf16); a non-finite
  // center element counts as 0 (the center may be any vector, see the header)
  static __device__ __forceinline__ uint4 sub(uint4 a, uint4 c) {
    const uint32_t av[4] = {a.x, a.y, a.z, a.w}, cv[4] = {c.x, c.y, c.z, c.w};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t clo = (cv[i] & 0x7f80u) == 0x7f80u ? 0u : (cv[i] << 16);
      const uint32_t chi = (cv[i] & 0x7f800000u) == 0x7f800000u ? 0u : (cv[i] & 0xffff0000u);
      const float lo = __uint_as_float(av[i] << 16) - __uint_as_float(clo);
      const float hi = __uint_as_float(av[i] & 0xffff0000u) - __uint_as_float(chi);
      o[i] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
  }
  // guarded load of 8 elements at p[c .. c+8) with columns >= D zero
  static __device__ __forceinline__ uint4 tail(const bf16* p, int64_t c, int64_t D) {
    if (c + 8 <= D) return *reinterpret_cast<const uint4*>(p + c);
    uint16_t t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = c + j < D ? reinterpret_cast<const uint16_t*>(p)[c + j] : 0;
    return make_uint4(t[0] | (uint32_t(t[1]) << 16), t[2] | (uint32_t(t[3]) << 16),
                      t[4] | (uint32_t(t[5]) << 16), t[6] | (uint32_t(t[7]) << 16));
  }
};
template <> struct GramLoad<float> {
  typedef float4 type;
  static __device__ __forceinline__ float4 zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ float fin(float c) { return isfinite(c) ? c : 0.f; }
  static __device__ __forceinline__ float4 sub(float4 a, float4 c) {
    return make_float4(a.x - fin(c.x), a.y - fin(c.y), a.z - fin(c.z), a.w - fin(c.w));
  }
  static __device__ __forceinline__ float4 tail(const float* p, int64_t c, int64_t D) {
    if (c + 4 <= D) return *reinterpret_cast<const float4*>(p + c);
    return make_float4(c < D ? p[c] : 0.f, c + 1 < D ? p[c + 1] : 0.f, c + 2 < D ? p[c + 2] : 0.f,
                       c + 3 < D ? p[c + 3] : 0.f);
  }
};

// G = column-group packing factor (1, or 16/P2 when TT == 1 and n <= 8).
// CENTER: rows relative to row *center (see the header).
template <typename T, int TT, int G, bool CENTER>
__device__ __forceinline__ void gram_partial_body(const T* __restrict__ X, int64_t ld, int n,
                                                  const int* __restrict__ rows, int64_t D,
                                                  float* __restrict__ part, int c,
                                                  float (*red)[16 * TT * 16 * TT]) {
  static_assert(G == 1 || TT == 1, "column-group packing is for a single row tile");
  typedef typename GramLoad<T>::type V;
  constexpr int P = 16 * TT;
  constexpr int NT = TT * (TT + 1) / 2;
  constexpr int Q = GramQ<TT>::value;
  constexpr int VEC = GramVec<T>::vec;
  constexpr int STEP = GramVec<T>::step;
  constexpr int GSPAN = Q * STEP;           // columns of one group per iteration
  constexpr int COLS = G * GSPAN;
  constexpr int P2 = 16 / G;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int h = lane >> 4;
  const int grp = r / P2;                   // 0 when G == 1
  const int vr = r % P2;

  const T* rowp[TT];
  bool valid[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int row = 16 * t + vr;
    valid[t] = row < n;
    const int rr = valid[t] ? row : (row % n);
    rowp[t] = X + static_cast<int64_t>(rows ? rows[rr] : rr) * ld + grp * GSPAN + VEC * h;
  }
  const T* cp = nullptr;
  if constexpr (CENTER) {
    c = c >= n ? n - 1 : c;
    cp = X + static_cast<int64_t>(rows ? rows[c] : c) * ld + grp * GSPAN + VEC * h;
  }

  f32x4 acc[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t gw = static_cast<int64_t>(blockIdx.x) * kGWaves + wave;
  const int64_t W = static_cast<int64_t>(gridDim.x) * kGWaves;
  const int64_t Dmain = (D / COLS) * COLS;

  for (int64_t k0 = gw * COLS; k0 < Dmain; k0 += W * COLS) {
    V u[Q][TT], cu[CENTER ? Q : 1];
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int t = 0; t < TT; ++t) u[q][t] = *reinterpret_cast<const V*>(rowp[t] + k0 + STEP * q);
    if constexpr (CENTER) {
#pragma unroll
      for (int q = 0; q < Q; ++q) cu[q] = *reinterpret_cast<const V*>(cp + k0 + STEP * q);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        if constexpr (CENTER) u[q][t] = GramLoad<T>::sub(u[q][t], cu[q]);
        u[q][t] = valid[t] ? u[q][t] : GramLoad<T>::zero();
      }
      gram_mfma<TT>(acc, u[q]);
    }
  }
  // Tail [Dmain, D): STEP-column chunks strided over all waves; only column group 0 loads
  // (the other groups' diagonal blocks just add zeros).
  for (int64_t k0 = Dmain + gw * STEP; k0 < D; k0 += W * STEP) {
    V u[TT], cu = GramLoad<T>::zero();
    if constexpr (CENTER) cu = GramLoad<T>::tail(cp - grp * GSPAN - VEC * h, k0 + VEC * h, D);
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      const T* base = rowp[t] - grp * GSPAN - VEC * h;
      u[t] = (valid[t] && grp == 0) ? GramLoad<T>::sub(GramLoad<T>::tail(base, k0 + VEC * h, D), cu)
                                    : GramLoad<T>::zero();
    }
    gram_mfma<TT>(acc, u);
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
    if constexpr (G == 1) {
      if ((row / 16) <= (col / 16)) {   // only upper tiles were written
#pragma unroll
        for (int w = 0; w < kGWaves; ++w) v += red[w][e];
      }
    } else {
      if (row < P2 && col < P2) {       // fold the diagonal column-group blocks
#pragma unroll
        for (int w = 0; w < kGWaves; ++w)
#pragma unroll
          for (int g = 0; g < G; ++g) v += red[w][(g * P2 + row) * P + g * P2 + col];
      }
    }
    out[e] = v;
  }
}

template <typename T, int TT, int G, bool CENTER>
__global__ __launch_bounds__(kGBlock) void gram_partial_kernel(const T* __restrict__ X, int64_t ld,
                                                              int n, const int* __restrict__ rows,
                                                              int64_t D, float* __restrict__ part,
                                                              const int* __restrict__ center) {
  __shared__ float red[kGWaves][16 * TT * 16 * TT];
  if constexpr (CENTER) {
    const int c = *center;   // uniform: one branch for the whole workgroup
    if (c < 0)
      gram_partial_body<T, TT, G, false>(X, ld, n, rows, D, part, 0, red);
    else
      gram_partial_body<T, TT, G, true>(X, ld, n, rows, D, part, c, red);
  } else {
    gram_partial_body<T, TT, G, false>(X, ld, n, rows, D, part, 0, red);
  }
}

// Deferred reduce of several buckets' stage-1 partials in ONE launch (the engine's early Grams:
// each bucket's partial kernel runs as its exchange lands, the reduces of all buckets run once in
// step()): G = sum over b in order of (fixed-order fp64 tree over bucket b's block partials) --
// the adds of one gram_reduce_kernel per bucket into a slot followed by gram_sum_kernel.
constexpr int kMaxRedBuckets = 32;
struct RedTable {
  const float* part[kMaxRedBuckets];
  int nblk[kMaxRedBuckets];
};

__global__ __launch_bounds__(256) void gram_reduce_multi_kernel(RedTable t, int nb, int P, int n,
                                                               double* __restrict__ G) {
  __shared__ double red[256];
  const int e = blockIdx.x;
  const int row = e / P, col = e % P;
  if (row >= n || col >= n || (row / 16) > (col / 16)) return;
  double acc = 0.0;
  for (int b = 0; b < nb; ++b) {
    const float* part = t.part[b];
    double s = 0.0;
    for (int k = threadIdx.x; k < t.nblk[b]; k += blockDim.x)
      s += static_cast<double>(part[static_cast<int64_t>(k) * P * P + e]);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    acc = b == 0 ? red[0] : acc + red[0];
    __syncthreads();   // red[] is reused by the next bucket
  }
  if (threadIdx.x == 0) {
    G[row * n + col] = acc;
    if ((row / 16) < (col / 16)) G[col * n + row] = acc;   // mirror off-diagonal tiles
  }
}

// G = sum over b of Gb[b] (fp64 [nb][E]), added in bucket order: the same adds as accumulating
// the per-bucket Grams into G one after another (the engine's early-Gram partials, one launch)
__global__ __launch_bounds__(256) void gram_sum_kernel(const double* __restrict__ Gb, int nb,
                                                      int64_t E, double* __restrict__ G) {
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; e < E;
       e += static_cast<int64_t>(gridDim.x) * 256) {
    double v = Gb[e];
    for (int b = 1; b < nb; ++b) v += Gb[static_cast<int64_t>(b) * E + e];
    G[e] = v;
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

// Medoid of the finite rows of G (n <= 64, one wave): score_i = sum over finite rows j of
// max(G_ii + G_jj - 2 G_ij, 0); non-finite rows / scores never win; ties -> lower index.
__global__ __launch_bounds__(64) void gram_center_kernel(const double* __restrict__ G, int n,
                                                         int* __restrict__ out) {
  const int i = threadIdx.x;
  double sc = __builtin_inf();
  if (i < n) {
    const double gii = G[i * n + i];
    if (isfinite(gii)) {
      double s = 0.0;
      for (int j = 0; j < n; ++j) {
        const double gjj = G[j * n + j];
        if (!isfinite(gjj)) continue;
        const double d = gii + gjj - 2.0 * G[i * n + j];
        s += d > 0.0 ? d : 0.0;
      }
      if (isfinite(s)) sc = s;
    }
  }
  int idx = i;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double s2 = __shfl_xor(sc, o, 64);
    const int i2 = __shfl_xor(idx, o, 64);
    if (s2 < sc || (s2 == sc && i2 < idx)) {
      sc = s2;
      idx = i2;
    }
  }
  if (i == 0) out[0] = (idx < n && isfinite(sc)) ? idx : 0;
}

int gram_tiles(int n) { return (n + 15) / 16; }

int gram_blocks(int64_t D, int cols) {
  int64_t b = (D + static_cast<int64_t>(cols) * kGWaves - 1) / (static_cast<int64_t>(cols) * kGWaves);
  if (b > kMaxGramBlocks) b = kMaxGramBlocks;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

// Stage 1 (and, with Gm != null, stage 2); returns the number of partial blocks.
template <typename T, int TT, int G>
int launch_gram_t(const T* X, int64_t ld, int n, const int* rows, int64_t D, float* part,
                  double* Gm, int acc, const int* center, hipStream_t st) {
  const int nb = gram_blocks(D, gram_cols<T, TT, G>());
  if (center)
    gram_partial_kernel<T, TT, G, true><<<nb, kGBlock, 0, st>>>(X, ld, n, rows, D, part, center);
  else
    gram_partial_kernel<T, TT, G, false><<<nb, kGBlock, 0, st>>>(X, ld, n, rows, D, part, nullptr);
  // (packed launches fold into the top-left block; the reduce skips elements >= n anyway)
  const int P = 16 * TT;
  if (Gm) gram_reduce_kernel<<<P * P, 256, 0, st>>>(part, nb, P, n, Gm, acc);
  return nb;
}

template <typename T>
int launch_gram_dispatch(const T* x, int64_t ld, int n, const int* rows, int64_t D, float* part,
                         double* G, int acc, const int* c, hipStream_t st) {
  if (n == 1) return launch_gram_t<T, 1, 16>(x, ld, n, rows, D, part, G, acc, c, st);
  if (n == 2) return launch_gram_t<T, 1, 8>(x, ld, n, rows, D, part, G, acc, c, st);
  if (n <= 4) return launch_gram_t<T, 1, 4>(x, ld, n, rows, D, part, G, acc, c, st);
  if (n <= 8) return launch_gram_t<T, 1, 2>(x, ld, n, rows, D, part, G, acc, c, st);
  if (n <= 16) return launch_gram_t<T, 1, 1>(x, ld, n, rows, D, part, G, acc, c, st);
  if (n <= 32) return launch_gram_t<T, 2, 1>(x, ld, n, rows, D, part, G, acc, c, st);
  if (n <= 48) return launch_gram_t<T, 3, 1>(x, ld, n, rows, D, part, G, acc, c, st);
  return launch_gram_t<T, 4, 1>(x, ld, n, rows, D, part, G, acc, c, st);
}
}  // namespace

size_t gram_workspace_bytes(int n, int64_t D) {
  const int P = 16 * gram_tiles(n);
  return static_cast<size_t>(kMaxGramBlocks) * P * P * sizeof(float);
}

hipError_t launch_gram(int dtype, const void* X, int64_t ld, int n, const int* rows, int64_t D,
                       void* work, double* G, int accumulate, hipStream_t stream,
                       const int* center) {
  if (n < 1 || n > 64 || D < 1) return hipErrorInvalidValue;
  const int es = dtype == DT_BF16 ? 2 : 4;
  const int vec = 16 / es;
  if ((ld % vec) != 0 || (reinterpret_cast<uintptr_t>(X) % 16) != 0) return hipErrorInvalidValue;
  float* part = reinterpret_cast<float*>(work);
  if (dtype == DT_BF16)
    launch_gram_dispatch(reinterpret_cast<const bf16*>(X), ld, n, rows, D, part, G, accumulate,
                         center, stream);
  else
    launch_gram_dispatch(reinterpret_cast<const float*>(X), ld, n, rows, D, part, G, accumulate,
                         center, stream);
  return hipGetLastError();
}

hipError_t launch_gram_partial(int dtype, const void* X, int64_t ld, int n, const int* rows,
                               int64_t D, void* work, hipStream_t stream, const int* center,
                               int* nblk) {
  if (n < 1 || n > 64 || D < 1) return hipErrorInvalidValue;
  const int es = dtype == DT_BF16 ? 2 : 4;
  if ((ld % (16 / es)) != 0 || (reinterpret_cast<uintptr_t>(X) % 16) != 0) return hipErrorInvalidValue;
  float* part = reinterpret_cast<float*>(work);
  *nblk = dtype == DT_BF16
              ? launch_gram_dispatch(reinterpret_cast<const bf16*>(X), ld, n, rows, D, part, nullptr,
                                     0, center, stream)
              : launch_gram_dispatch(reinterpret_cast<const float*>(X), ld, n, rows, D, part,
                                     nullptr, 0, center, stream);
  return hipGetLastError();
}

hipError_t launch_gram_reduce_multi(const float* const* parts, const int* nblks, int nb, int n,
                                    double* G, hipStream_t stream) {
  if (n < 1 || n > 64 || nb < 1 || nb > kMaxRedBuckets) return hipErrorInvalidValue;
  RedTable t{};
  for (int b = 0; b < nb; ++b) {
    t.part[b] = parts[b];
    t.nblk[b] = nblks[b];
  }
  const int P = 16 * gram_tiles(n);
  gram_reduce_multi_kernel<<<P * P, 256, 0, stream>>>(t, nb, P, n, G);
  return hipGetLastError();
}

hipError_t launch_gram_sum(const double* Gb, int nb, int64_t E, double* G, hipStream_t stream) {
  if (nb < 1 || E < 1) return hipErrorInvalidValue;
  int64_t blocks = (E + 255) / 256;
  if (blocks > 64) blocks = 64;
  gram_sum_kernel<<<static_cast<unsigned>(blocks), 256, 0, stream>>>(Gb, nb, E, G);
  return hipGetLastError();
}

hipError_t launch_gram_center(const double* G, int n, int* out, hipStream_t stream) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  gram_center_kernel<<<1, 64, 0, stream>>>(G, n, out);
  return hipGetLastError();
}

}  // namespace cml
