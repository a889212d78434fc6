// Fused robust aggregation + optimizer update (N04/N05/N08 of SURVEY.md §2.4).
//
// One pass over the n worker vectors of a coordinate shard: per coordinate either
//   * SORTED   : a compile-time Batcher network over NP >= n values held in VGPRs (padding rows
//                are +inf), then the mean of sorted ranks [lo, lo+cnt) -> median / trimmed mean
//                / Bulyan's coordinate phase, or
//   * WEIGHTED : sum_i w_i x_i over the non-zero weights only (Krum, Multi-Krum, Weiszfeld,
//                centered clipping, plain mean) — zero-weight rows are never read,
// and then SGD(momentum, nesterov, wd) or Adam/AdamW on the fp32 master, rewriting the bf16
// parameters in the same pass. The aggregated gradient never round-trips through HBM.
//
// Memory-bound streaming kernel: 16 B per lane per worker row (8 bf16 / 4 f32), grid-stride,
// <= 2048 workgroups of 256 threads. Row addresses are hoisted out of the loop; padded rows load
// a clamped (valid) row and are replaced by +inf with a select, so no per-row branch sits
// between the loads (hipcc would otherwise wait vmcnt(0) per row).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cml {

constexpr int kBlock = 256;
constexpr int kMaxRows = 64;
constexpr int kMaxSegs = 16;   // segments of one multi-segment launch

// Optimizer state of VEC coordinates, loaded BEFORE the combine so those HBM reads are in flight
// while the sort / weighted sum runs (hipcc does not hoist them above the VALU work by itself).
template <int VEC>
struct OptState {
  float p[VEC];   // fp32 master
  float a[VEC];   // momentum buffer / Adam m
  float b[VEC];   // Adam v
};

template <int VEC>
__device__ __forceinline__ void load_state(const UpdArgs& u, int opt, int64_t e, OptState<VEC>& st) {
  if (opt == OPT_NONE) return;
  load_vec<float, VEC>(u.master + e, st.p);
  if (opt == OPT_SGD) {
    if (u.momentum != 0.0f && !u.first) load_vec<float, VEC>(u.s1 + e, st.a);
  } else {
    load_vec<float, VEC>(u.s1 + e, st.a);
    load_vec<float, VEC>(u.s2 + e, st.b);
  }
}

template <int VEC>
__device__ __forceinline__ void update_and_store(const UpdArgs& u, int opt, int64_t e,
                                                 float (&g)[VEC], OptState<VEC>& st) {
  if (u.gscale != 1.0f) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) g[v] *= u.gscale;
  }
  if (u.gout) store_f32<VEC>(u.gout + e, g);
  if (opt == OPT_NONE) return;
  float (&p)[VEC] = st.p;
  if (opt == OPT_SGD) {
    if (u.weight_decay != 0.0f) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) g[v] = fmaf(u.weight_decay, p[v], g[v]);
    }
    if (u.momentum != 0.0f) {
      float (&b)[VEC] = st.a;
      if (u.first) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) b[v] = g[v];
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v) b[v] = fmaf(u.momentum, b[v], g[v]);
      }
      store_f32<VEC>(u.s1 + e, b);
      if (u.nesterov) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) g[v] = fmaf(u.momentum, b[v], g[v]);
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v) g[v] = b[v];
      }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) p[v] = fmaf(-u.lr, g[v], p[v]);
  } else {  // OPT_ADAM: decoupled weight decay (AdamW), or the L2 term of Adam (adam_l2)
    float (&m)[VEC] = st.a;
    float (&s)[VEC] = st.b;
    float decay = 1.0f - u.lr * u.weight_decay;
    if (u.adam_l2) {   // wave-uniform kernel argument
      decay = 1.0f;
#pragma unroll
      for (int v = 0; v < VEC; ++v) g[v] = fmaf(u.weight_decay, p[v], g[v]);
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      m[v] = fmaf(u.beta1, m[v], (1.0f - u.beta1) * g[v]);
      s[v] = fmaf(u.beta2, s[v], (1.0f - u.beta2) * g[v] * g[v]);
      const float denom = fmaf(sqrtf(s[v]), u.inv_sqrt_bc2, u.eps);
      p[v] = fmaf(-u.step_size, m[v] / denom, p[v] * decay);
    }
    store_f32<VEC>(u.s1 + e, m);
    store_f32<VEC>(u.s2 + e, s);
  }
  store_f32<VEC>(u.master + e, p);
  if (u.param_out) {
    if (u.param_f32) store_f32<VEC>(reinterpret_cast<float*>(u.param_out) + e, p);
    else store_bf16<VEC>(reinterpret_cast<bf16*>(u.param_out) + e, p);
  }
}

// ----------------------------------------------------------------------------- sorted combine
// fp32 rows (and the bf16 scalar tail): sort fp32 values. The rank window [lo, lo+cnt) is
// wave-uniform (kernel arguments), so the per-rank test is a scalar branch, not a VALU select.
template <typename T, int NP, int VEC, int OPT>
__device__ __forceinline__ void agg_sorted_body(const SrcArgs& s, const UpdArgs& u, int64_t base,
    int64_t nvec, int blk, int nblk) {
  const T* X = reinterpret_cast<const T*>(s.X);
  int64_t roff[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int r = i < s.n ? i : s.n - 1;
    roff[i] = static_cast<int64_t>(s.rows ? s.rows[r] : r) * s.ld + base;
  }
  const float inf = __builtin_inff();
  const float inv = 1.0f / static_cast<float>(s.cnt);
  const int64_t stride = static_cast<int64_t>(nblk) * kBlock;
  for (int64_t t = static_cast<int64_t>(blk) * kBlock + threadIdx.x; t < nvec; t += stride) {
    const int64_t e = t * VEC;
    float a[NP][VEC];
#pragma unroll
    for (int i = 0; i < NP; ++i) load_vec<T, VEC>(X + roff[i] + e, a[i]);
    OptState<VEC> st;
    load_state<VEC>(u, OPT, base + e, st);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const bool pad = i >= s.n;
#pragma unroll
      for (int v = 0; v < VEC; ++v) a[i][v] = (pad || a[i][v] != a[i][v]) ? inf : a[i][v];
    }
    sort_columns<float, NP, VEC>(a);
    float g[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) g[v] = 0.0f;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (i >= s.lo && i < s.lo + s.cnt) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) g[v] += a[i][v];
      }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) g[v] *= inv;
    update_and_store<VEC>(u, OPT, base + e, g, st);
  }
}

// bf16 rows: sort packed u16 keys (two coordinates per v_pk_min/max_u16, see bf16_key), decode
// only the cnt window ranks. VEC bf16 = VEC/2 32-bit words per row.
template <int W> struct Words;
template <> struct Words<4> {
  static __device__ __forceinline__ void load(const bf16* p, uint32_t (&w)[4]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
  }
};
template <> struct Words<2> {
  static __device__ __forceinline__ void load(const bf16* p, uint32_t (&w)[2]) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    w[0] = u.x; w[1] = u.y;
  }
};
template <> struct Words<1> {
  static __device__ __forceinline__ void load(const bf16* p, uint32_t (&w)[1]) {
    w[0] = *reinterpret_cast<const uint32_t*>(p);
  }
};

template <int NP, int VEC, int OPT>
__device__ __forceinline__ void agg_sorted_bf16_body(const SrcArgs& s, const UpdArgs& u, int64_t base,
    int64_t nvec, int blk, int nblk) {
  constexpr int W = VEC / 2;
  const bf16* X = reinterpret_cast<const bf16*>(s.X);
  int64_t roff[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int r = i < s.n ? i : s.n - 1;
    roff[i] = static_cast<int64_t>(s.rows ? s.rows[r] : r) * s.ld + base;
  }
  const float inv = 1.0f / static_cast<float>(s.cnt);
  const u16x2 kinf = {kKeyInf, kKeyInf};
  const int64_t stride = static_cast<int64_t>(nblk) * kBlock;
  for (int64_t t = static_cast<int64_t>(blk) * kBlock + threadIdx.x; t < nvec; t += stride) {
    const int64_t e = t * VEC;
    uint32_t raw[NP][W];
#pragma unroll
    for (int i = 0; i < NP; ++i) Words<W>::load(X + roff[i] + e, raw[i]);
    OptState<VEC> st;
    load_state<VEC>(u, OPT, base + e, st);
    u16x2 k[NP][W];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const bool pad = i >= s.n;
#pragma unroll
      for (int w = 0; w < W; ++w) k[i][w] = pad ? kinf : bf16_key(raw[i][w]);
    }
    sort_columns<u16x2, NP, W>(k);
    float g[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) g[v] = 0.0f;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (i >= s.lo && i < s.lo + s.cnt) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
          float lo, hi;
          bf16_unkey(k[i][w], lo, hi);
          g[2 * w] += lo;
          g[2 * w + 1] += hi;
        }
      }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) g[v] *= inv;
    update_and_store<VEC>(u, OPT, base + e, g, st);
  }
}

// ----------------------------------------------------------------------------- weighted combine
template <typename T, int VEC, int OPT>
__device__ __forceinline__ void agg_weighted_body(const SrcArgs& s, const UpdArgs& u, int64_t base,
    int64_t nvec, int blk, int nblk) {
  // Compact the non-zero weights once per workgroup (LDS, broadcast reads in the loop).
  __shared__ int64_t s_off[kMaxRows];
  __shared__ float s_w[kMaxRows];
  __shared__ int s_nz;
  if (threadIdx.x == 0) {
    int nz = 0;
    for (int i = 0; i < s.n; ++i) {
      const float wi = s.w ? s.w[i] : 1.0f;
      if (wi != 0.0f) {
        s_off[nz] = static_cast<int64_t>(s.rows ? s.rows[i] : i) * s.ld + base;
        s_w[nz] = wi;
        ++nz;
      }
    }
    s_nz = nz;
  }
  __syncthreads();
  const int nz = s_nz;
  const T* X = reinterpret_cast<const T*>(s.X);
  const int64_t stride = static_cast<int64_t>(nblk) * kBlock;
  for (int64_t t = static_cast<int64_t>(blk) * kBlock + threadIdx.x; t < nvec; t += stride) {
    const int64_t e = t * VEC;
    OptState<VEC> st;
    load_state<VEC>(u, OPT, base + e, st);
    float g[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) g[v] = 0.0f;
    int i = 0;
    for (; i + 4 <= nz; i += 4) {  // four rows in flight before the FMAs
      float x0[VEC], x1[VEC], x2[VEC], x3[VEC];
      load_vec<T, VEC>(X + s_off[i] + e, x0);
      load_vec<T, VEC>(X + s_off[i + 1] + e, x1);
      load_vec<T, VEC>(X + s_off[i + 2] + e, x2);
      load_vec<T, VEC>(X + s_off[i + 3] + e, x3);
      const float w0 = s_w[i], w1 = s_w[i + 1], w2 = s_w[i + 2], w3 = s_w[i + 3];
#pragma unroll
      for (int v = 0; v < VEC; ++v)
        g[v] = fmaf(w3, x3[v], fmaf(w2, x2[v], fmaf(w1, x1[v], fmaf(w0, x0[v], g[v]))));
    }
    for (; i < nz; ++i) {
      float x0[VEC];
      load_vec<T, VEC>(X + s_off[i] + e, x0);
      const float w0 = s_w[i];
#pragma unroll
      for (int v = 0; v < VEC; ++v) g[v] = fmaf(w0, x0[v], g[v]);
    }
    update_and_store<VEC>(u, OPT, base + e, g, st);
  }
}


// ----------------------------------------------------------------------------- kernels
// Single segment (one bucket / one vector): grid-stride over nvec vectors.
template <typename T, int NP, int VEC, int OPT>
__global__ __launch_bounds__(kBlock) void agg_sorted_kernel(SrcArgs s, UpdArgs u, int64_t base,
                                                            int64_t nvec) {
  agg_sorted_body<T, NP, VEC, OPT>(s, u, base, nvec, blockIdx.x, gridDim.x);
}
template <int NP, int VEC, int OPT>
__global__ __launch_bounds__(kBlock) void agg_sorted_bf16_kernel(SrcArgs s, UpdArgs u,
                                                                 int64_t base, int64_t nvec) {
  agg_sorted_bf16_body<NP, VEC, OPT>(s, u, base, nvec, blockIdx.x, gridDim.x);
}
template <typename T, int VEC, int OPT>
__global__ __launch_bounds__(kBlock) void agg_weighted_kernel(SrcArgs s, UpdArgs u, int64_t base,
                                                              int64_t nvec) {
  agg_weighted_body<T, VEC, OPT>(s, u, base, nvec, blockIdx.x, gridDim.x);
}

// Several segments in ONE launch (the sharded engine's buckets: per-bucket worker matrices and
// parameter shards, one fp32 optimizer-state vector): blockIdx.y = segment. Every segment is on
// the vector path (checked by the launcher).
struct SegTable {
  const void* X[kMaxSegs];
  int64_t ld[kMaxSegs];
  int64_t nvec[kMaxSegs];
  int64_t off[kMaxSegs];     // element offset into master / s1 / s2 / gout
  void* pout[kMaxSegs];
};

__device__ __forceinline__ void seg_args(const SegTable& t, int sg, SrcArgs& s, UpdArgs& u) {
  s.X = t.X[sg];
  s.ld = t.ld[sg];
  const int64_t o = t.off[sg];
  if (u.master) u.master += o;
  if (u.s1) u.s1 += o;
  if (u.s2) u.s2 += o;
  if (u.gout) u.gout += o;
  u.param_out = t.pout[sg];
}

template <typename T, int NP, int VEC, int OPT>
__global__ __launch_bounds__(kBlock) void agg_sorted_multi(SrcArgs s, UpdArgs u, SegTable t) {
  seg_args(t, blockIdx.y, s, u);
  agg_sorted_body<T, NP, VEC, OPT>(s, u, 0, t.nvec[blockIdx.y], blockIdx.x, gridDim.x);
}
template <int NP, int VEC, int OPT>
__global__ __launch_bounds__(kBlock) void agg_sorted_bf16_multi(SrcArgs s, UpdArgs u, SegTable t) {
  seg_args(t, blockIdx.y, s, u);
  agg_sorted_bf16_body<NP, VEC, OPT>(s, u, 0, t.nvec[blockIdx.y], blockIdx.x, gridDim.x);
}
template <typename T, int VEC, int OPT>
__global__ __launch_bounds__(kBlock) void agg_weighted_multi(SrcArgs s, UpdArgs u, SegTable t) {
  seg_args(t, blockIdx.y, s, u);
  agg_weighted_body<T, VEC, OPT>(s, u, 0, t.nvec[blockIdx.y], blockIdx.x, gridDim.x);
}

// ----------------------------------------------------------------------------- dispatch
// CML_AGG_GRID_CAP: the most workgroups of an update launch (default 0 = no cap: one vector per
// thread, the form that streams fastest on MI355X -- tools/diag/hbm_copy.py: a one-pass copy
// 6.0-6.6 TB/s vs 4.7-5.7 for grid-stride loops; the fused rule + SGD update 8.6-12.7 % faster
// than at the former cap of 2048 workgroups, profiles/r06_13/agg_*.jsonl).
static inline int grid_for(int64_t nvec) {
  static const int cap = [] {
    const char* e = getenv("CML_AGG_GRID_CAP");
    return e ? atoi(e) : 0;
  }();
  int64_t b = (nvec + kBlock - 1) / kBlock;
  if (cap > 0 && b > cap) b = cap;
  if (b > (1LL << 30)) b = 1LL << 30;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

template <typename T, int NP, int VEC>
static void launch_sorted_np(int opt, const SrcArgs& s, const UpdArgs& u, int64_t base,
                             int64_t nvec, hipStream_t st) {
  const int g = grid_for(nvec);
  if constexpr (sizeof(T) == 2 && VEC >= 2) {   // packed-key path
    switch (opt) {
      case OPT_NONE: agg_sorted_bf16_kernel<NP, VEC, OPT_NONE><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
      case OPT_SGD: agg_sorted_bf16_kernel<NP, VEC, OPT_SGD><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
      default: agg_sorted_bf16_kernel<NP, VEC, OPT_ADAM><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
    }
  } else {
    switch (opt) {
      case OPT_NONE: agg_sorted_kernel<T, NP, VEC, OPT_NONE><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
      case OPT_SGD: agg_sorted_kernel<T, NP, VEC, OPT_SGD><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
      default: agg_sorted_kernel<T, NP, VEC, OPT_ADAM><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
    }
  }
}

// Vector width per padded row count (sorted_vec below must agree): bf16 keys take half a VGPR
// per value, so bf16 keeps 16 B loads up to NP = 32; NP = 64 drops to 2 elements per lane.
template <typename T, bool VECTOR>
static void launch_sorted(int opt, const SrcArgs& s, const UpdArgs& u, int64_t base, int64_t D,
                          hipStream_t st) {
  // D: number of elements; VECTOR: D is a multiple of sorted_vec() and all pointers aligned.
  const int n = s.n;
  constexpr bool BF = sizeof(T) == 2;
  if constexpr (VECTOR) {
    if (n <= 2) launch_sorted_np<T, 2, BF ? 8 : 4>(opt, s, u, base, D / (BF ? 8 : 4), st);
    else if (n <= 4) launch_sorted_np<T, 4, BF ? 8 : 4>(opt, s, u, base, D / (BF ? 8 : 4), st);
    else if (n <= 8) launch_sorted_np<T, 8, BF ? 8 : 4>(opt, s, u, base, D / (BF ? 8 : 4), st);
    else if (n <= 16) launch_sorted_np<T, 16, BF ? 8 : 4>(opt, s, u, base, D / (BF ? 8 : 4), st);
    else if (n <= 32) launch_sorted_np<T, 32, BF ? 8 : 4>(opt, s, u, base, D / (BF ? 8 : 4), st);
    else launch_sorted_np<T, 64, 2>(opt, s, u, base, D / 2, st);
  } else {
    if (n <= 2) launch_sorted_np<T, 2, 1>(opt, s, u, base, D, st);
    else if (n <= 4) launch_sorted_np<T, 4, 1>(opt, s, u, base, D, st);
    else if (n <= 8) launch_sorted_np<T, 8, 1>(opt, s, u, base, D, st);
    else if (n <= 16) launch_sorted_np<T, 16, 1>(opt, s, u, base, D, st);
    else if (n <= 32) launch_sorted_np<T, 32, 1>(opt, s, u, base, D, st);
    else launch_sorted_np<T, 64, 1>(opt, s, u, base, D, st);
  }
}

template <typename T, int VEC>
static void launch_weighted(int opt, const SrcArgs& s, const UpdArgs& u, int64_t base, int64_t nvec,
                            hipStream_t st) {
  const int g = grid_for(nvec);
  switch (opt) {
    case OPT_NONE: agg_weighted_kernel<T, VEC, OPT_NONE><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
    case OPT_SGD: agg_weighted_kernel<T, VEC, OPT_SGD><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
    default: agg_weighted_kernel<T, VEC, OPT_ADAM><<<g, kBlock, 0, st>>>(s, u, base, nvec); break;
  }
}

static inline bool aligned(const void* p, int bytes) {
  return p == nullptr || (reinterpret_cast<uintptr_t>(p) % bytes) == 0;
}

static int sorted_vec(int dtype, int n) {
  if (n > 32) return 2;
  return dtype == DT_BF16 ? 8 : 4;
}

template <typename T>
static hipError_t agg_update_t(int combine, int opt, const SrcArgs& s, const UpdArgs& u, int64_t D,
                               hipStream_t st) {
  if (D <= 0) return hipSuccess;
  const int esz = sizeof(T);
  const int vec = combine == CMB_WEIGHTED ? (esz == 2 ? 8 : 4) : sorted_vec(esz == 2 ? DT_BF16 : DT_F32, s.n);
  // The vector path needs every row start and every state pointer aligned to VEC elements.
  bool ok = (s.ld % vec) == 0 && aligned(s.X, vec * esz) && aligned(u.master, vec * 4) &&
            aligned(u.s1, vec * 4) && aligned(u.s2, vec * 4) && aligned(u.gout, vec * 4) &&
            aligned(u.param_out, vec * (u.param_f32 ? 4 : 2));
  int64_t Dv = ok ? (D / vec) * vec : 0;
  if (Dv > 0) {
    if (combine == CMB_WEIGHTED) {
      if constexpr (sizeof(T) == 2) launch_weighted<T, 8>(opt, s, u, 0, Dv / 8, st);
      else launch_weighted<T, 4>(opt, s, u, 0, Dv / 4, st);
    } else {
      launch_sorted<T, true>(opt, s, u, 0, Dv, st);
    }
  }
  if (D > Dv) {  // scalar tail (or fully unaligned inputs)
    if (combine == CMB_WEIGHTED) launch_weighted<T, 1>(opt, s, u, Dv, D - Dv, st);
    else launch_sorted<T, false>(opt, s, u, Dv, D - Dv, st);
  }
  return hipGetLastError();
}

template <typename T, int NP, int VEC>
static void launch_sorted_multi_np(int opt, const SrcArgs& s, const UpdArgs& u, const SegTable& t,
                                   dim3 g, hipStream_t st) {
  if constexpr (sizeof(T) == 2 && VEC >= 2) {
    switch (opt) {
      case OPT_NONE: agg_sorted_bf16_multi<NP, VEC, OPT_NONE><<<g, kBlock, 0, st>>>(s, u, t); break;
      case OPT_SGD: agg_sorted_bf16_multi<NP, VEC, OPT_SGD><<<g, kBlock, 0, st>>>(s, u, t); break;
      default: agg_sorted_bf16_multi<NP, VEC, OPT_ADAM><<<g, kBlock, 0, st>>>(s, u, t); break;
    }
  } else {
    switch (opt) {
      case OPT_NONE: agg_sorted_multi<T, NP, VEC, OPT_NONE><<<g, kBlock, 0, st>>>(s, u, t); break;
      case OPT_SGD: agg_sorted_multi<T, NP, VEC, OPT_SGD><<<g, kBlock, 0, st>>>(s, u, t); break;
      default: agg_sorted_multi<T, NP, VEC, OPT_ADAM><<<g, kBlock, 0, st>>>(s, u, t); break;
    }
  }
}

template <typename T>
static hipError_t agg_update_multi_t(int combine, int opt, const SrcArgs& s, const UpdArgs& u,
                                     const AggSeg* segs, int nseg, hipStream_t st) {
  const int esz = sizeof(T);
  const int vec = combine == CMB_WEIGHTED ? (esz == 2 ? 8 : 4)
                                          : sorted_vec(esz == 2 ? DT_BF16 : DT_F32, s.n);
  bool ok = nseg >= 1 && nseg <= kMaxSegs;
  SegTable t{};
  int64_t maxv = 0;
  for (int i = 0; ok && i < nseg; ++i) {
    const AggSeg& g = segs[i];
    const int64_t o = g.off;
    ok = g.D > 0 && g.D % vec == 0 && (g.ld % vec) == 0 && aligned(g.X, vec * esz) &&
         o % vec == 0 && aligned(u.master, vec * 4) && aligned(u.s1, vec * 4) &&
         aligned(u.s2, vec * 4) && aligned(u.gout, vec * 4) &&
         aligned(g.param_out, vec * (u.param_f32 ? 4 : 2));
    t.X[i] = g.X;
    t.ld[i] = g.ld;
    t.nvec[i] = g.D / vec;
    t.off[i] = o;
    t.pout[i] = g.param_out;
    maxv = t.nvec[i] > maxv ? t.nvec[i] : maxv;
  }
  if (!ok) {   // per-segment launches (unaligned / ragged segments)
    for (int i = 0; i < nseg; ++i) {
      SrcArgs s1 = s;
      s1.X = segs[i].X;
      s1.ld = segs[i].ld;
      UpdArgs u1 = u;
      const int64_t o = segs[i].off;
      if (u1.master) u1.master += o;
      if (u1.s1) u1.s1 += o;
      if (u1.s2) u1.s2 += o;
      if (u1.gout) u1.gout += o;
      u1.param_out = segs[i].param_out;
      hipError_t e = agg_update_t<T>(combine, opt, s1, u1, segs[i].D, st);
      if (e != hipSuccess) return e;
    }
    return hipGetLastError();
  }
  int gx = grid_for(maxv);
  const int cap = 2048 / nseg;
  if (gx > cap) gx = cap < 1 ? 1 : cap;
  const dim3 g(static_cast<unsigned>(gx), static_cast<unsigned>(nseg));
  if (combine == CMB_WEIGHTED) {
    constexpr int V = sizeof(T) == 2 ? 8 : 4;
    switch (opt) {
      case OPT_NONE: agg_weighted_multi<T, V, OPT_NONE><<<g, kBlock, 0, st>>>(s, u, t); break;
      case OPT_SGD: agg_weighted_multi<T, V, OPT_SGD><<<g, kBlock, 0, st>>>(s, u, t); break;
      default: agg_weighted_multi<T, V, OPT_ADAM><<<g, kBlock, 0, st>>>(s, u, t); break;
    }
  } else {
    constexpr bool BF = sizeof(T) == 2;
    const int n = s.n;
    if (n <= 2) launch_sorted_multi_np<T, 2, BF ? 8 : 4>(opt, s, u, t, g, st);
    else if (n <= 4) launch_sorted_multi_np<T, 4, BF ? 8 : 4>(opt, s, u, t, g, st);
    else if (n <= 8) launch_sorted_multi_np<T, 8, BF ? 8 : 4>(opt, s, u, t, g, st);
    else if (n <= 16) launch_sorted_multi_np<T, 16, BF ? 8 : 4>(opt, s, u, t, g, st);
    else if (n <= 32) launch_sorted_multi_np<T, 32, BF ? 8 : 4>(opt, s, u, t, g, st);
    else launch_sorted_multi_np<T, 64, 2>(opt, s, u, t, g, st);
  }
  return hipGetLastError();
}

hipError_t launch_agg_update_multi(int dtype, int combine, int opt, const SrcArgs& src,
                                   const UpdArgs& upd, const AggSeg* segs, int nseg,
                                   hipStream_t stream) {
  if (src.n < 1 || src.n > kMaxRows || nseg < 1) return hipErrorInvalidValue;
  if (combine == CMB_SORTED && (src.cnt < 1 || src.lo < 0 || src.lo + src.cnt > src.n))
    return hipErrorInvalidValue;
  if (dtype == DT_BF16) return agg_update_multi_t<bf16>(combine, opt, src, upd, segs, nseg, stream);
  return agg_update_multi_t<float>(combine, opt, src, upd, segs, nseg, stream);
}

hipError_t launch_agg_update(int dtype, int combine, int opt, const SrcArgs& src,
                             const UpdArgs& upd, int64_t D, hipStream_t stream) {
  if (src.n < 1 || src.n > kMaxRows) return hipErrorInvalidValue;
  if (combine == CMB_SORTED && (src.cnt < 1 || src.lo < 0 || src.lo + src.cnt > src.n))
    return hipErrorInvalidValue;
  if (dtype == DT_BF16) return agg_update_t<bf16>(combine, opt, src, upd, D, stream);
  return agg_update_t<float>(combine, opt, src, upd, D, stream);
}

}  // namespace cml
