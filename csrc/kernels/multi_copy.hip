// Multi-tensor copy: gather a bucket's freshly produced gradient tensors into their slots of the
// flat gradient buffer in ONE launch (copy-on-ready capture, parallel/engine.py).
//
// PyTorch's _foreach_copy_ runs these at ~2.8 TB/s (11.6 ms of a 162 ms Llama-3-8B step moves
// 32 GB, profiles/r01_prof16_llama_fused_kernels.md): its multi_tensor_apply chunks are small and
// it launches per chunk-list. Here the table of up to kMaxCopy (src, dst, bytes) entries rides in
// the kernel arguments and every workgroup copies part of ONE entry: the launcher splits ~8192
// workgroups over the entries by size (prefix bpre), a workgroup finds its entry by a scalar
// search of that table, and the entry's workgroups stride over it with 4 16-B vectors per lane in
// flight. (The first form searched the entry per 16-B vector over the vector prefix, a divergent
// loop of dependent kernel-argument loads per element: 29 us for the ~10 MB of a batch-256 ResNet
// bucket, profiles/r05_19/kernels_b256.md; one 32-KiB slice per workgroup moved the 470 MB Llama
// buckets at only 2.9 TB/s, profiles/r05_25/.) The sub-16-B tails are copied in 2-B units by the first
// lanes of the grid.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kCB = 256;
constexpr int kU = 4;                    // 16-B vectors in flight per lane and iteration
constexpr int kSV = 2048;                // vectors per workgroup of a small copy (32 KiB)

__global__ __launch_bounds__(kCB) void multi_copy_kernel(MultiCopyArgs a) {
  const int b = blockIdx.x;
  int lo = 0, hi = a.n - 1;              // last entry with bpre[e] <= b (uniform: scalar loads)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a.bpre[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int e = lo;
  const int64_t nv = a.vpre[e + 1] - a.vpre[e];
  const uint4* src = reinterpret_cast<const uint4*>(a.src[e]);
  uint4* dst = reinterpret_cast<uint4*>(a.dst[e]);
  if (a.slice) {   // small copies: one kSV-vector slice per workgroup, all loads before the stores
    const int64_t v0 = static_cast<int64_t>(b - a.bpre[e]) * kSV + threadIdx.x;
    uint4 v[kSV / kCB];
#pragma unroll
    for (int u = 0; u < kSV / kCB; ++u) {
      const int64_t i = v0 + static_cast<int64_t>(u) * kCB;
      if (i < nv) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < kSV / kCB; ++u) {
      const int64_t i = v0 + static_cast<int64_t>(u) * kCB;
      if (i < nv) dst[i] = v[u];
    }
  } else {
  // the entry's workgroups stride over it together, kU vectors per lane in flight
  const int64_t stride = static_cast<int64_t>(a.bpre[e + 1] - a.bpre[e]) * kCB;
  for (int64_t i0 = static_cast<int64_t>(b - a.bpre[e]) * kCB + threadIdx.x; i0 < nv;
       i0 += kU * stride) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < nv) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < nv) dst[i] = v[u];
    }
  }
  }
  // tails: bytes [nvec * 16, bytes) of each entry, 2 B per lane
  if (b == 0) {
    for (int k = 0; k < a.n; ++k) {
      const int64_t nvk = a.vpre[k + 1] - a.vpre[k];
      const int64_t rem = (a.bytes[k] - nvk * 16) / 2;
      if (threadIdx.x < rem) {
        const int64_t h = nvk * 8 + threadIdx.x;
        reinterpret_cast<uint16_t*>(a.dst[k])[h] = reinterpret_cast<const uint16_t*>(a.src[k])[h];
      }
    }
  }
}

}  // namespace

namespace {
// dst [C][R] = src [R][C]^T (bf16, R % 64 == 0, C % 64 == 0, 16-B aligned rows): one 64 x 64
// tile per workgroup, 16-B loads into a padded LDS tile and 16-B stores of the transposed rows
// (the weight transposes of the data-gradient GEMMs: ATen's strided copy ran them at ~0.6 TB/s,
// 12 us per BERT weight, profiles/r04_06/bert_kernels.md)
__global__ __launch_bounds__(256) void transpose64_kernel(const uint16_t* __restrict__ src,
                                                         uint16_t* __restrict__ dst, int R, int C,
                                                         int64_t lds_, int64_t ldd) {
  __shared__ uint16_t t[64][64 + 2];   // +2: a row read down a column hits distinct banks
  const int tc = blockIdx.x, tr = blockIdx.y;
  const int r0 = tr * 64, c0 = tc * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 2; ++it) {   // 64 rows x 8 chunks of 8 elements
    const int i = tid + 256 * it, r = i >> 3, c = (i & 7) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(src + static_cast<int64_t>(r0 + r) * lds_ + c0 + c);
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      t[r][c + 2 * q] = static_cast<uint16_t>(w4[q] & 0xffffu);
      t[r][c + 2 * q + 1] = static_cast<uint16_t>(w4[q] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {   // output row c (a source column), 8 consecutive source rows
    const int i = tid + 256 * it, c = i >> 3, r = (i & 7) * 8;
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = static_cast<uint32_t>(t[r + 2 * q][c]) | (static_cast<uint32_t>(t[r + 2 * q + 1][c]) << 16);
    *reinterpret_cast<uint4*>(dst + static_cast<int64_t>(c0 + c) * ldd + r0 + r) =
        make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace

hipError_t launch_transpose_bf16(const void* src, void* dst, int R, int C, int64_t lds_,
                                 int64_t ldd, hipStream_t st) {
  if (R < 64 || C < 64 || R % 64 || C % 64 || lds_ % 8 || ldd % 8 ||
      ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15))
    return hipErrorInvalidValue;
  transpose64_kernel<<<dim3(C / 64, R / 64), 256, 0, st>>>(
      reinterpret_cast<const uint16_t*>(src), reinterpret_cast<uint16_t*>(dst), R, C, lds_, ldd);
  return hipGetLastError();
}

hipError_t launch_multi_copy(const MultiCopyArgs& a, hipStream_t st) {
  if (a.n < 1 || a.n > kMaxCopy) return hipErrorInvalidValue;
  for (int e = 0; e < a.n; ++e) {
    if ((reinterpret_cast<uintptr_t>(a.src[e]) & 15) || (reinterpret_cast<uintptr_t>(a.dst[e]) & 15) ||
        (a.bytes[e] & 1) || a.vpre[e + 1] - a.vpre[e] != a.bytes[e] / 16)
      return hipErrorInvalidValue;
  }
  MultiCopyArgs k = a;
  // Large copies (>= 8192 slices): 8192 workgroups split by size over the entries, striding
  // (the Llama-3-8B weight gradients at 4.88 TB/s, ATen's contiguous copy 4.84); small ones: one
  // 32-KiB slice per workgroup (a ResNet bucket's 10 MB in 11.5 us; striding grids of 664 / 8192
  // workgroups took 32 / 21 us, profiles/r05_25/, r05_26/). At least one workgroup per entry
  // (block 0 also copies the tails).
  const int64_t total = std::max<int64_t>(1, a.vpre[a.n]);
  k.slice = total < 8192ll * kSV ? 1 : 0;
  int64_t nb = 0;
  for (int e = 0; e < a.n; ++e) {
    k.bpre[e] = static_cast<int>(nb);
    const int64_t nv = a.vpre[e + 1] - a.vpre[e];
    if (k.slice) {
      nb += std::max<int64_t>(1, (nv + kSV - 1) / kSV);
    } else {
      const int64_t want = (nv * 8192 + total - 1) / total;
      const int64_t cap = (nv + kCB - 1) / kCB;   // no more workgroups than 256-vector slices
      nb += std::max<int64_t>(1, std::min(want, cap));
    }
  }
  k.bpre[a.n] = static_cast<int>(nb);
  multi_copy_kernel<<<static_cast<unsigned>(nb), kCB, 0, st>>>(k);
  return hipGetLastError();
}

}  // namespace cml
