// HBM stream-rate probes (tools/diag/hbm_copy.py): which access form reaches the measured
// ~6.3 TB/s float4-copy rate of MI355X_MICROARCH.md on this image, for the mixes the memory-bound
// training kernels have (1 read : 1 write copy, 2 : 1 add, write-only). Built standalone:
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/diag/hbm_copy.hip -o build/hbm_copy.so
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

// U 16-B vectors in flight per thread, grid-stride over n4 float4s; NT: nontemporal loads/stores
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_k(const v4f* __restrict__ a, v4f* __restrict__ c,
                                              int64_t n4) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * U;
  for (int64_t base = (static_cast<int64_t>(blockIdx.x) * 256) * U + threadIdx.x; base < n4;
       base += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i < n4) v[u] = NTL ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i < n4) {
        if (NTS) __builtin_nontemporal_store(v[u], c + i);
        else c[i] = v[u];
      }
    }
  }
}

template <int U, bool NTS>
__global__ __launch_bounds__(256) void add_k(const v4f* __restrict__ a, const v4f* __restrict__ b,
                                             v4f* __restrict__ c, int64_t n4) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * U;
  for (int64_t base = (static_cast<int64_t>(blockIdx.x) * 256) * U + threadIdx.x; base < n4;
       base += stride) {
    v4f v[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i < n4) {
        v[u] = a[i];
        w[u] = b[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i < n4) {
        const v4f r = v[u] + w[u];
        if (NTS) __builtin_nontemporal_store(r, c + i);
        else c[i] = r;
      }
    }
  }
}

template <int U, bool NTS>
__global__ __launch_bounds__(256) void fill_k(v4f* __restrict__ c, int64_t n4) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * U;
  const v4f z = {1.f, 2.f, 3.f, 4.f};
  for (int64_t base = (static_cast<int64_t>(blockIdx.x) * 256) * U + threadIdx.x; base < n4;
       base += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i < n4) {
        if (NTS) __builtin_nontemporal_store(z, c + i);
        else c[i] = z;
      }
    }
  }
}

}  // namespace

// kind: 0 copy, 1 add (2 reads : 1 write), 2 fill; variant bits: 1 = nt stores, 2 = nt loads
// (copy only); unroll U in {1, 2, 4, 8}; blocks: grid size (0: one pass, n4 / (256 U))
extern "C" int hbm_probe(int kind, int variant, int U, int blocks, const void* a, const void* b,
                         void* c, int64_t n4, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t one = (n4 + 256LL * U - 1) / (256LL * U);
  const int g = blocks > 0 ? blocks : static_cast<int>(one < (1LL << 31) ? one : (1LL << 31) - 1);
  const auto* A = reinterpret_cast<const v4f*>(a);
  const auto* B = reinterpret_cast<const v4f*>(b);
  auto* C = reinterpret_cast<v4f*>(c);
#define CP(UU)                                                                           \
  switch (variant & 3) {                                                                 \
    case 0: copy_k<UU, false, false><<<g, 256, 0, st>>>(A, C, n4); break;                \
    case 1: copy_k<UU, false, true><<<g, 256, 0, st>>>(A, C, n4); break;                 \
    case 2: copy_k<UU, true, false><<<g, 256, 0, st>>>(A, C, n4); break;                 \
    default: copy_k<UU, true, true><<<g, 256, 0, st>>>(A, C, n4); break;                 \
  }
#define AD(UU)                                                                           \
  if (variant & 1) add_k<UU, true><<<g, 256, 0, st>>>(A, B, C, n4);                      \
  else add_k<UU, false><<<g, 256, 0, st>>>(A, B, C, n4);
#define FL(UU)                                                                           \
  if (variant & 1) fill_k<UU, true><<<g, 256, 0, st>>>(C, n4);                           \
  else fill_k<UU, false><<<g, 256, 0, st>>>(C, n4);
#define DISPATCH(M)                                                                      \
  switch (U) {                                                                           \
    case 1: M(1) break;                                                                  \
    case 2: M(2) break;                                                                  \
    case 4: M(4) break;                                                                  \
    default: M(8) break;                                                                 \
  }
  if (kind == 0) { DISPATCH(CP) }
  else if (kind == 1) { DISPATCH(AD) }
  else { DISPATCH(FL) }
  return static_cast<int>(hipGetLastError());
}
