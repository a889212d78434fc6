// Stride-1 3x3 convolution (padding 1) of 64-channel NHWC bf16 images 56 pixels wide -- the
// ResNet-50 layer-1 3x3 conv (forward with its BN statistics, and its data gradient with bn1's
// backward sums) -- from an LDS-resident input PATCH instead of an implicit GEMM:
//
//   y[m][n] = sum_{tap, c} x[pix(m) + off(tap)][c] w[n][tap 64 + c]
//
// Why: the implicit GEMM (conv_gemm.hip / gemm.hip conv mode) re-stages every input pixel once per
// tap -- 9 x 128 B per output pixel copied L2 -> LDS, ~40 KB per 2.1 MFLOP k-step for a 256 x 64
// tile -- so at C = N = 64 it is bound by the LDS-DMA rate (~70 GB/s per CU), not by the MFMAs:
// 0.43-0.49 PFLOP/s (profiles/r04_12, conv_gemm_kernel<256, 64, ...>). Here a workgroup keeps the
// whole weight (9 taps x 64 x 64, 72 KB) resident and stages each tile's input rows ONCE: a tile is
// 4 output rows of one image (224 pixels), its patch the 6 input rows around them (43 KB,
// 1.5 x 128 B per output pixel); the 9 taps read shifted windows of the same patch.
//
// Layout (gfx950, one 448-thread workgroup per CU, persistent over a contiguous tile range):
//   LDS = W image [9 x 64 rows][128 B] | two patch buffers [336 rows][128 B] | a zero row --
//   156 KB. Rows are 128 B (64 channels), XOR-swizzled (16-B chunk c of row r at
//   c ^ ((r >> 1) & 7); the DMA image is lane-linear, so the swizzle is applied through the
//   per-lane SOURCE address, as in conv_gemm.hip).
//   Patch row q = pr 56 + pc holds input pixel (r0 - 1 + pr, pc); rows outside the image are
//   DMA'd from the zero buffer. Output pixel f of the tile (f = 56 tr + tc) reads tap (dy, dx)
//   at patch row q = f + 56 (1 + dy) + dx -- linear in f, so a 32-pixel fragment is 32
//   consecutive rows (conflict-free under the swizzle for any shift); a tap whose column falls
//   off the image (tc + dx outside [0, 56)) reads the zero row instead.
//   Waves: 7, wave w owns the 32-pixel fragment w of the tile and all 64 output channels:
//   2 accumulators of v_mfma_f32_32x32x16_bf16 (C^T = W X^T: a lane holds one pixel, 4 channels
//   per accumulator row group), 72 MFMAs per tile, 1 patch + 2 weight ds_read_b128 per 2 MFMAs,
//   read two steps ahead.
//   Epilogue: each wave rounds its 32 x 64 block into its own rows of the just-consumed patch
//   buffer and reads them back as whole 128-B rows (8 lanes per pixel): full-line 16-B stores,
//   8 fixed channels per lane. EP 1: shifted BN statistics of the stored bf16 values; EP 2: the
//   BN + ReLU backward sums of the data gradient (s += y', q += y' (z - mean),
//   y' = (z sc + bi > 0) ? y : 0), both accumulated per lane over the workgroup's tiles and
//   reduced once at the end into ONE partial row per workgroup (fixed order: deterministic),
//   folded by conv1x1.hip's finalize kernels.
//   Pipeline: once every wave has read its image back (the tile's third barrier), the patch of
//   tile j + 2 is DMA'd into that buffer, so each patch has a whole tile (MFMAs + epilogue) to
//   land; a counted vmcnt (the 4 stores of the last epilogue + the 6 DMA instructions of the next
//   patch stay in flight) retires exactly the current patch.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

constexpr int kWd = 56;                    // image width = tile width
constexpr int kTR = 4;                     // output rows per tile
constexpr int kTP = kTR * kWd;             // 224 pixels = 7 fragments of 32
constexpr int kNW = kTP / 32;              // waves
constexpr int kThr = 64 * kNW;             // 448
constexpr int kPQ = (kTR + 2) * kWd;       // 336 patch rows
constexpr int kWImg = 9 * 64 * 128;        // 73728 B
constexpr int kPImg = kPQ * 128;           // 43008 B
constexpr int kOffP = kWImg;
constexpr int kOffZ = kOffP + 2 * kPImg;   // 159744
constexpr int kLds = kOffZ + 128;          // 159872
constexpr int kPS = kPQ / 8 / kNW;         // 6 patch DMA instructions per wave
constexpr int kWI = 9 * 64 / 8;            // 72 weight DMA instructions
constexpr int kStores = 4;                 // epilogue stores per lane per tile (16 B each)
static_assert(kPS * 8 * kNW == kPQ, "patch rows split evenly over the waves");
static_assert(kLds <= 163840, "LDS budget");

struct P3Args {
  const uint16_t* x;      // [Nimg][H][56][64]
  const uint16_t* w;      // [64][9 * 64]: (n, tap 64 + c), tap = 3 (dy + 1) + dx + 1
  uint16_t* y;            // [Nimg H 56][64]
  const uint16_t* zero;   // >= 8 zero bf16, 16-B aligned
  float* part;            // EP >= 1: [gridDim.x][2][64]
  const float* shift;     // EP 1: statistics shift (or null); EP 2: the BN's mean
  const uint16_t* sz;     // EP 2: BN input z [M][64]
  const float* ep_sc;     // EP 2: that BN's affine (ReLU bit: z sc + bi > 0)
  const float* ep_bi;
  int H, tpi, tiles;      // image height, tiles per image (H / 4), tiles
  int dbg;                // bench/conv3x3p.py only: 1 skip the MFMAs, 2 skip the per-tile patch DMA
};

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// one 16-B LDS read; the caller waits for it (s_waitcnt lgkmcnt) before using the value
__device__ __forceinline__ bf16x8_t lds_rd(int addr) {
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(n) for the four counts the loop uses (n is wave-uniform)
__device__ __forceinline__ void wait_vm(int n) {
  if (n >= kPS + kStores) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if (n >= kPS) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= kStores) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
static_assert(kPS == 6 && kStores == 4, "wait_vm's immediates");

template <int EP>
__global__ __launch_bounds__(kThr, 1) __attribute__((amdgpu_waves_per_eu(1, 2))) void conv3x3p_kernel(
    P3Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, b = blockIdx.x;
  const int t0 = static_cast<int>(static_cast<int64_t>(a.tiles) * b / G);
  const int nloc = static_cast<int>(static_cast<int64_t>(a.tiles) * (b + 1) / G) - t0;
  const int lrow = lane >> 3, lp = lane & 7;

  // zero row; this lane's 8 epilogue channels' coefficients (plain loads: before any DMA is in
  // flight)
  if (tid < 8) *reinterpret_cast<uint4*>(smem + kOffZ + 16 * tid) = make_uint4(0u, 0u, 0u, 0u);
  const int c8 = lane & 7;   // epilogue: 16-B chunk (channels 8 c8 .. 8 c8 + 7) of a pixel row
  float sh[8], esc[8], ebi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sh[e] = EP >= 1 && a.shift ? a.shift[8 * c8 + e] : 0.f;
    esc[e] = EP == 2 ? a.ep_sc[8 * c8 + e] : 0.f;
    ebi[e] = EP == 2 ? a.ep_bi[8 * c8 + e] : 0.f;
  }

  // weight image: row tap 64 + n = w[n][tap 64 .. tap 64 + 63]
#pragma unroll
  for (int s = 0; s < (kWI + kNW - 1) / kNW; ++s) {
    const int i = wave + kNW * s;
    if (i < kWI) {
      const int row = 8 * i + lrow, tap = row >> 6, n = row & 63;
      const int c = lp ^ ((row >> 1) & 7);
      const uint16_t* src = a.w + static_cast<int64_t>(n) * 576 + tap * 64 + 8 * c;
      __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(smem + 8 * i * 128), 16, 0, 0);
    }
  }

  // this lane's patch rows (same for every tile): row q = 8 (wave + 7 s) + lrow
  int poff[kPS], prow[kPS];
#pragma unroll
  for (int s = 0; s < kPS; ++s) {
    const int q = 8 * (wave + kNW * s) + lrow;
    prow[s] = q / kWd;
    const int pc = q - prow[s] * kWd;
    poff[s] = pc * 64 + 8 * (lp ^ ((q >> 1) & 7));
  }
  auto stage = [&](int t, int buf) {
    const int img = t / a.tpi, r0 = (t - img * a.tpi) * kTR;
    char* dst0 = smem + kOffP + buf * kPImg;
#pragma unroll
    for (int s = 0; s < kPS; ++s) {
      const int ir = r0 - 1 + prow[s];
      const uint16_t* src =
          static_cast<unsigned>(ir) < static_cast<unsigned>(a.H)
              ? a.x + static_cast<int64_t>(img * a.H + ir) * (kWd * 64) + poff[s]
              : a.zero;
      __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(dst0 + 8 * (wave + kNW * s) * 128),
                                       16, 0, 0);
    }
  };

  // fragment addresses: lane pixel f (column r32 of the accumulators), k half h
  const int r32 = lane & 31, h = lane >> 5;
  const int f = 32 * wave + r32, tc = f % kWd;
  const int wl = r32 * 128 + 16 * (h ^ ((r32 >> 1) & 7));   // weight row r32 of a 32-row group
  int xo[9];                                                  // per tap, relative to the buffer
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int dy = tap / 3 - 1, dx = tap % 3 - 1;
    const int q = f + kWd * (1 + dy) + dx;
    const bool ok = dx == 0 || (dx < 0 ? tc > 0 : tc < kWd - 1);
    xo[tap] = ok ? kOffP + q * 128 + 16 * (h ^ ((q >> 1) & 7)) : -1;
  }

  float cs[8], cq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cs[e] = 0.f;
    cq[e] = 0.f;
  }

  if (nloc > 0) stage(t0, 0);
  if (nloc > 1) stage(t0 + 1, 1);

  for (int j = 0; j < nloc; ++j) {
    const int t = t0 + j, buf = j & 1;
    // retire patch j: younger are the last epilogue's stores and patch j + 1 (issued after them)
    wait_vm((j > 0 ? kStores : 0) + (j + 1 < nloc ? kPS : 0));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    // epilogue rows of this lane: tile pixels 32 wave + 8 k + lrow, chunk c8
    const int64_t mrow = static_cast<int64_t>(t) * kTP + 32 * wave + lrow;
    uint4 zr[EP == 2 ? 4 : 1];
    if constexpr (EP == 2) {   // the BN input at this lane's outputs (latency under the MFMAs)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        zr[k] = *reinterpret_cast<const uint4*>(a.sz + (mrow + 8 * k) * 64 + 8 * c8);
    }
    f32x16 acc[2];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      acc[0][k] = 0.f;
      acc[1][k] = 0.f;
    }
    const int pb = buf * kPImg;
    // 36 (tap, kk) steps, fragments of step s + 1 read before the MFMAs of step s
    int xb[9];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) xb[tap] = xo[tap] >= 0 ? xo[tap] + pb : kOffZ + 16 * h;
    // (sched_barriers pin the order: the reads of step s + 2 are issued before the MFMAs of step
    // s, so each MFMA pair waits only for reads two steps old)
    // The reads are inline asm with explicit counted lgkmcnt waits: the compiler's own waits for
    // this loop were lgkmcnt(0) every third step (draining the reads it had just issued).
    bf16x8_t fr[3][3];
    auto rd = [&](int s, bf16x8_t (&d)[3]) {
      const int tap = s >> 2, kk = s & 3;
      d[0] = lds_rd(xb[tap] ^ (32 * kk));
      d[1] = lds_rd(tap * 8192 + (wl ^ (32 * kk)));
      d[2] = lds_rd(tap * 8192 + 4096 + (wl ^ (32 * kk)));
    };
    if (!(a.dbg & 1)) {
    rd(0, fr[0]);
    rd(1, fr[1]);
#pragma unroll
    for (int s = 0; s < 36; ++s) {
      if (s + 2 < 36) rd(s + 2, fr[(s + 2) % 3]);
      // step s's reads retired; steps s + 1, s + 2 (3 reads each) may stay in flight
      if (s + 2 < 36) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
      else if (s + 1 < 36) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      acc[0] = mfma32(fr[s % 3][1], fr[s % 3][0], acc[0]);
      acc[1] = mfma32(fr[s % 3][2], fr[s % 3][0], acc[1]);
      __builtin_amdgcn_sched_barrier(0);
    }
    }
    bar();   // every wave is done with this buffer

    // epilogue: the wave's 32 pixels x 64 channels as a bf16 image in its own 32 rows of the
    // consumed buffer (same swizzle), read back as whole 128-B rows (8 lanes per pixel): full-line
    // 16-B stores, 8 fixed channels per lane for the statistics
    char* img = smem + kOffP + pb;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t lo = pk_bf16(acc[i][4 * g], acc[i][4 * g + 1]);
        const uint32_t hi = pk_bf16(acc[i][4 * g + 2], acc[i][4 * g + 3]);
        const int row = 32 * wave + r32, ch = 4 * i + g;
        *reinterpret_cast<uint2*>(img + row * 128 + 16 * (ch ^ ((row >> 1) & 7)) + 8 * h) =
            make_uint2(lo, hi);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = 32 * wave + 8 * k + lrow;
      const uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + 16 * (c8 ^ ((row >> 1) & 7)));
      *reinterpret_cast<uint4*>(a.y + (mrow + 8 * k) * 64 + 8 * c8) = v;
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      if constexpr (EP == 1) {   // shifted sums of the stored bf16 values
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float lo = __uint_as_float(w4[q] << 16) - sh[2 * q];
          const float hi = __uint_as_float(w4[q] & 0xffff0000u) - sh[2 * q + 1];
          cs[2 * q] += lo;
          cs[2 * q + 1] += hi;
          cq[2 * q] = fmaf(lo, lo, cq[2 * q]);
          cq[2 * q + 1] = fmaf(hi, hi, cq[2 * q + 1]);
        }
      } else if constexpr (EP == 2) {   // y' = relu'(z sc + bi) y; s += y', q += y' (z - mean)
        const uint32_t z4[4] = {zr[k].x, zr[k].y, zr[k].z, zr[k].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float zlo = __uint_as_float(z4[q] << 16), zhi = __uint_as_float(z4[q] & 0xffff0000u);
          const float lo = fmaf(zlo, esc[2 * q], ebi[2 * q]) > 0.f ? __uint_as_float(w4[q] << 16) : 0.f;
          const float hi = fmaf(zhi, esc[2 * q + 1], ebi[2 * q + 1]) > 0.f
                               ? __uint_as_float(w4[q] & 0xffff0000u) : 0.f;
          cs[2 * q] += lo;
          cs[2 * q + 1] += hi;
          cq[2 * q] = fmaf(lo, zlo - sh[2 * q], cq[2 * q]);
          cq[2 * q + 1] = fmaf(hi, zhi - sh[2 * q + 1], cq[2 * q + 1]);
        }
      }
    }
    if (j + 2 < nloc && !(a.dbg & 2)) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();   // every wave's image reads are done: the buffer takes patch j + 2
      stage(t + 2, buf);
    }
  }

  if constexpr (EP >= 1) {
    // lanes with equal c8 hold the same 8 channels: fixed-order xor tree over lane >> 3
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s1 = cs[e], s2 = cq[e];
#pragma unroll
      for (int k = 8; k < 64; k <<= 1) {
        s1 += __shfl_xor(s1, k, 64);
        s2 += __shfl_xor(s2, k, 64);
      }
      cs[e] = s1;
      cq[e] = s2;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    float* red = reinterpret_cast<float*>(smem + kOffP);   // [wave][2][64] over the dead patches
    if (lane < 8) {
      float* rp = red + wave * 128 + 8 * c8;
      reinterpret_cast<float4*>(rp)[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
      reinterpret_cast<float4*>(rp)[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
      reinterpret_cast<float4*>(rp + 64)[0] = make_float4(cq[0], cq[1], cq[2], cq[3]);
      reinterpret_cast<float4*>(rp + 64)[1] = make_float4(cq[4], cq[5], cq[6], cq[7]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (tid < 128) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kNW; ++w) s += red[w * 128 + tid];
      a.part[static_cast<int64_t>(b) * 128 + tid] = s;
    }
  }
}

int num_cus() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1)
      c = 256;
    return c;
  }();
  return n;
}

}  // namespace

// CML_CONV3P (A/B, default 1)
bool conv3x3p_eligible(int Nimg, int H, int W, int C, int N, int taps, int stride) {
  static const bool on = [] {
    const char* e = getenv("CML_CONV3P");
    return !e || e[0] != '0';
  }();
  return on && taps == 9 && stride == 1 && C == 64 && N == 64 && W == kWd && H > 0 && H % kTR == 0 &&
         Nimg > 0 && static_cast<int64_t>(Nimg) * H * kWd < (1LL << 31);
}

size_t conv3x3p_part_floats() { return static_cast<size_t>(num_cus()) * 128; }

hipError_t launch_conv3x3p(const void* x, const void* w, void* y, const void* zero, int Nimg, int H,
                           int ep, float* part, const float* shift, const void* z, const float* sc,
                           const float* bi, hipStream_t st, int* rows) {
  if (!conv3x3p_eligible(Nimg, H, kWd, 64, 64, 9, 1) || ep < 0 || ep > 2 || !x || !w || !y ||
      !zero || (ep >= 1 && !part) || (ep == 2 && (!z || !sc || !bi || !shift)))
    return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y) |
       reinterpret_cast<uintptr_t>(zero) | reinterpret_cast<uintptr_t>(z)) % 16)
    return hipErrorInvalidValue;
  P3Args a{};
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.w = reinterpret_cast<const uint16_t*>(w);
  a.y = reinterpret_cast<uint16_t*>(y);
  a.zero = reinterpret_cast<const uint16_t*>(zero);
  a.part = part;
  a.shift = shift;
  a.sz = reinterpret_cast<const uint16_t*>(z);
  a.ep_sc = sc;
  a.ep_bi = bi;
  a.H = H;
  a.tpi = H / kTR;
  a.tiles = Nimg * a.tpi;
  static const int dbg = [] {
    const char* d = getenv("CML_CONV3P_DBG");
    return d ? atoi(d) : 0;
  }();
  a.dbg = dbg;
  const int G = a.tiles < num_cus() ? a.tiles : num_cus();
  if (rows) *rows = G;
#define CML_P3(E)                                                                              \
  do {                                                                                         \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv3x3p_kernel<E>),                   \
                        hipFuncAttributeMaxDynamicSharedMemorySize, kLds);                     \
    conv3x3p_kernel<E><<<G, kThr, kLds, st>>>(a);                                              \
  } while (0)
  switch (ep) {
    case 0: CML_P3(0); break;
    case 1: CML_P3(1); break;
    default: CML_P3(2); break;
  }
#undef CML_P3
  return hipGetLastError();
}

}  // namespace cml
