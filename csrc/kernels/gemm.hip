// Dense bf16 GEMM with fused epilogues for the transformer FFN (BERT: bias + GELU forward, GELU
// backward + bias-gradient column sums), gfx950 / CDNA4:
//
//   y[m][n] = epi( sum_k A[m][k] B[n][k] )           A [M][K], B [N][K]: both K-contiguous ("NT",
//                                                     nn.Linear's x W^T)
//   EP_STORE   y = bf16(acc + bias[n]) [+ cin[m][n]]  (bias, cin optional; cin may alias y: the
//                                                     residual-gradient add of a data gradient)
//   EP_GELU    h = bf16(acc + bias[n]) -> aux,  y = bf16(gelu(h))   (erf GELU, from the bf16 h)
//   EP_DGELU   g = bf16(acc);  y = bf16(g * gelu'(aux[m][n])),  part[m / 128][n] = column sums of y
//
// The rounding points are those of the unfused PyTorch composition (GEMM output rounded to bf16,
// then the elementwise op in fp32 on the bf16 values), so the fused path changes only the GEMM's
// summation order.
//
// Tile and schedule (one 512-thread workgroup = 8 waves per 256 x 256 output tile, 1 per CU):
//   * waves as 2 (m) x 4 (n); each owns 128 x 64 outputs = 8 x 4 accumulators of
//     v_mfma_f32_16x16x32_bf16, computed transposed (C^T = B A^T) so that a lane holds 4
//     consecutive output channels of one row -- 8-B packed bf16 writes into the epilogue image;
//   * K in 64-deep tiles through two LDS buffers (2 x 64 KB: A then B image, 128-B rows,
//     XOR-swizzled so every ds_read_b128 lane group hits 16 distinct bank slots; the swizzle lives
//     in the per-lane SOURCE address since global_load_lds writes lane-linear);
//   * each K-tile is computed in 4 phases, one output quadrant (64 m x 32 n, 16 MFMAs) each; a
//     phase is a read section (fragment ds_reads, one staging issue, a counted vmcnt) and an
//     MFMA section, each closed by a raw s_barrier. The waves of m-row 1 (the second wave on
//     every SIMD) run one section behind m-row 0 (one extra barrier up front, one at the end for
//     m-row 0), so every SIMD alternates one wave's MFMAs with its partner's LDS reads.
//     Fragments read per phase: 1 = the wave's first 64 A rows + first 32 B rows, 2 = the second
//     32 B rows, 3 = the second 64 A rows, 4 = none. A tile is staged as 4 units matching that
//     order (U1 = A rows 0-63 of each 128-row half, U2 = B rows 0-31 of each 64-row group,
//     U3 = the other B rows, U4 = the other A rows), one unit (2 global_load_lds dwordx4 per
//     lane) per phase: U3, U4 of tile t+1 in phases 1, 2 and U1, U2 of tile t+2 in phases 3, 4.
//     With the one-section stagger a region may be restaged only 2 phases after its last read
//     (WAR: the lagging group retires its reads one barrier later), which this order meets
//     (U1: 2 phases, U2-U4: 3). Each read section ends with `s_waitcnt vmcnt(8)` (4 newer units
//     may stay in flight) before its barrier: that retires exactly the unit(s) the NEXT phase
//     reads, early enough for the lagging group (RAW); every unit has 4 phases of flight and the
//     queue never drains in the loop. Past the last K-tile the issues repeat the last tile into
//     dead buffers, so the counts stay uniform.
//   * epilogue: each wave rounds its 128 x 64 block into its own 16 KB LDS image and reads it
//     back as 16-B row pieces (8 lanes per 128-B row): whole-line global stores, 8 fixed
//     channels per lane for the column sums.
//   * tiles are mapped XCD-aware: the n-tiles of one m-tile get consecutive ids, and
//     consecutive ids share an XCD under round-robin placement (A read from HBM once).
// Requirements (checked by the launcher): M % 256 == 0, N % 256 == 0, K % 64 == 0, 16-B aligned
// rows. Other shapes go to hipBLASLt (ops/transformer.py).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

constexpr int kT = 256;                 // tile edge (square tiles)
constexpr int kBK = 64;                 // K per tile step
constexpr int kThreads = 512;

// Tile TM (m) x TN (n) with TM TN = 256 x 256: TM = 256 is the square tile; TM = 512 (TN = 128) is
// the tall tile of the 128-channel 3x3 convs (ResNet-50 layer 2), with the same 128 x 64 wave
// blocks (waves 4 (m) x 2 (n)) and therefore the same MFMA / fragment schedule; its A image is
// 512 rows, so a buffer is 80 KB and the two buffers take the whole 160 KB of LDS.
template <int TM>
struct Tile {
  static constexpr int TN = kT * kT / TM;
  static constexpr int WMR = TM / 128;            // wave m-rows
  static constexpr int WNC = 8 / WMR;             // wave n-columns
  static constexpr int ImgA = TM * 128, ImgB = TN * 128;
  static constexpr int Buf = ImgA + ImgB;
  static constexpr int Lds = 2 * Buf;
  static constexpr int IA = TM / 128, IB = TN / 128;   // wave-instructions per A / B unit
  static constexpr int VM = 2 * IA + 2 * IB;      // this wave's instructions of 4 units
  static_assert(TM == 256 || TM == 512, "tile");
  static_assert(Lds <= 160 * 1024, "LDS");
};

__device__ __forceinline__ int swz(int row, int c) { return row * 128 + 16 * (c ^ ((row >> 1) & 7)); }

__device__ __forceinline__ f32x4 mfma16(bf16x8_t a, bf16x8_t b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int EP, bool CONV, int TM = 256, bool S2 = false>
__global__ __launch_bounds__(kThreads, 2) void gemm_nt_kernel(GemmArgs a) {
  using T = Tile<TM>;
  constexpr int TN = T::TN;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / T::WNC, wn = wave % T::WNC;

  // ---- tile (bijective XCD remap: consecutive ids share an XCD; n fastest)
  const int ntn = a.N / TN;
  const int G = (a.M / TM) * ntn, b = blockIdx.x, xcd = b & 7, q8 = G >> 3, r8 = G & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  // a.gm > 1: groups of gm m-tiles with m fastest, so the tiles an XCD runs at once form a
  // gm x (32 / gm) block (each A panel serves 32 / gm tiles, each B panel gm) instead of one m-row
  int mtile, ntile;
  if (a.gm > 1) {
    const int mtn = static_cast<int>(a.M / TM);
    const int grp = t / (a.gm * ntn), gi = t - grp * (a.gm * ntn);
    const int gmr = min(a.gm, mtn - grp * a.gm);
    mtile = grp * a.gm + gi % gmr;
    ntile = gi / gmr;
  } else {
    mtile = t / ntn;
    ntile = t - mtile * ntn;
  }
  const int m0 = mtile * TM, n0 = ntile * TN;
  const int nk = a.K / kBK;

  // ---- staging: unit u (0..3 = U1..U4) of K-tile kt into buffer buf; this wave's IA (A units)
  // or IB (B units) of the unit's wave-instructions (8 rows x 128 B each)
  const int lrow = lane >> 3, lp = lane & 7;
  // CONV: this lane's TM / 64 A rows (j = 2 s + (u == 3): tile rows 64 j + 8 wave + lrow) as pixels
  constexpr int NJ = CONV ? TM / 64 : 1;
  int pbase[NJ], poh[NJ], pow_[NJ];
  if constexpr (CONV) {
    const int HW = a.H * a.W;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int m = m0 + 64 * j + 8 * wave + lrow;
      const int img = m / HW, rem = m - img * HW;
      pbase[j] = S2 ? img * (a.IH * a.IW) : img * HW;
      poh[j] = rem / a.W;
      pow_[j] = rem - poh[j] * a.W;
      if constexpr (S2) {   // the input pixel of tap (1, 1), (2 oh, 2 ow)
        poh[j] *= 2;
        pow_[j] *= 2;
      }
    }
  }
  auto stage = [&](int u, int kt, int buf) {
    kt = kt < nk ? kt : nk - 1;                 // past the end: a harmless repeat (dead buffer)
    const int64_t kofs = static_cast<int64_t>(kt) * kBK;
    const bool isA = (u == 0 || u == 3);
#pragma unroll
    for (int s = 0; s < (T::IA > T::IB ? T::IA : T::IB); ++s) {
      if (s >= (isA ? T::IA : T::IB)) break;
      const int i = wave + 8 * s;               // wave-instruction of the unit
      int row0;
      if (isA) row0 = (i >> 3) * 128 + (u == 3 ? 64 : 0) + (i & 7) * 8;   // A
      else row0 = (i >> 2) * 64 + (u == 2 ? 32 : 0) + (i & 3) * 8;        // B
      const int row = row0 + lrow;
      const int c = lp ^ ((row >> 1) & 7);
      const uint16_t* src;
      if (CONV && isA) {
        // k-tile kt = tap (C / 64) + cc: input pixel (oh + ky - 1, ow + kx - 1), channels cc 64 ..
        const int cs = a.C >> 6, tap = kt / cs, cc = kt - tap * cs;
        const int j = 2 * s + (u == 3 ? 1 : 0);
        const int ih = poh[j] + tap / 3 - 1, iw = pow_[j] + (tap - 3 * (tap / 3)) - 1;
        const int IH = S2 ? a.IH : a.H, IW = S2 ? a.IW : a.W;
        const bool ok = static_cast<unsigned>(ih) < static_cast<unsigned>(IH) &&
                        static_cast<unsigned>(iw) < static_cast<unsigned>(IW);
        src = ok ? a.a + (static_cast<int64_t>(pbase[j]) + ih * IW + iw) * a.C + cc * kBK + 8 * c
                 : a.zero;
      } else {
        src = isA ? a.a + static_cast<int64_t>(m0 + row) * a.lda + kofs + 8 * c
                  : a.b + static_cast<int64_t>(n0 + row) * a.ldb + kofs + 8 * c;
      }
      char* dst = smem + buf * T::Buf + (isA ? 0 : T::ImgA) + row0 * 128;
      __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)dst, 16, 0, 0);
    }
  };

  // ---- fragments: lane row lane & 15, 16-B chunk (lane >> 4) + 4 ks
  const int fr = lane & 15, fc = lane >> 4;
  bf16x8_t aF[2][4][2], bF[2][2][2];
  auto readA = [&](bf16x8_t (&f)[4][2], int mh, int buf) {
    const char* img = smem + buf * T::Buf;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        f[mt][ks] = *reinterpret_cast<const bf16x8_t*>(
            img + swz(wm * 128 + mh * 64 + mt * 16 + fr, fc + 4 * ks));
  };
  auto readB = [&](bf16x8_t (&f)[2][2], int nh, int buf) {
    const char* img = smem + buf * T::Buf + T::ImgA;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        f[nt][ks] = *reinterpret_cast<const bf16x8_t*>(
            img + swz(wn * 64 + nh * 32 + nt * 16 + fr, fc + 4 * ks));
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto quad = [&](int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[mh * 4 + mt][nh * 2 + nt] =
              mfma16(bF[nh][nt][ks], aF[mh][mt][ks], acc[mh * 4 + mt][nh * 2 + nt]);
    __builtin_amdgcn_s_setprio(0);
  };
  // 4 newer units may stay in flight (the 4 newest units are always one each of U1..U4)
  auto wait8 = [] { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::VM) : "memory"); };
  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- prologue: tile 0 whole, U1 + U2 of tile 1; retire U1, U2 of tile 0
  stage(0, 0, 0); stage(1, 0, 0); stage(2, 0, 0); stage(3, 0, 0);
  stage(0, 1, 1); stage(1, 1, 1);
  wait8();
  bar();
  // stagger: the second wave of every SIMD (waves 4-7) runs one section behind, so each SIMD
  // alternates one wave's MFMA section with its partner's read / issue section
  const bool lag = wave >= 4;
  if (lag) bar();

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    // phase 1: quadrant (0, 0)
    stage(2, kt + 1, buf ^ 1);
    readA(aF[0], 0, buf);
    readB(bF[0], 0, buf);
    wait8();                  // retires U3 of tile kt (read in phase 2)
    bar();
    quad(0, 0);
    bar();
    // phase 2: quadrant (0, 1)
    stage(3, kt + 1, buf ^ 1);
    readB(bF[1], 1, buf);
    wait8();                  // retires U4 of tile kt (phase 3)
    bar();
    quad(0, 1);
    bar();
    // phase 3: quadrant (1, 1)
    stage(0, kt + 2, buf);
    readA(aF[1], 1, buf);
    wait8();
    bar();
    quad(1, 1);
    bar();
    // phase 4: quadrant (1, 0), no fragment reads
    stage(1, kt + 2, buf);
    wait8();                  // retires U1, U2 of tile kt + 1 (next phase 1)
    bar();
    quad(1, 0);
    bar();
  }
  if (!lag) bar();            // balance the stagger barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();

  // ---- epilogue: bf16 image of the wave's 128 (m) x 64 (n) block, [m][128 B] swizzled
  // The second operand of the read-back (DGELU: h; STORE with cin: the residual gradient) is
  // loaded for all 16 read-back rows up front, so its latency overlaps the image writes instead
  // of stalling every row (a dependent load per row cost ~13 us per tile).
  const int c8 = lane & 7;
  const int ncol = n0 + wn * 64 + 8 * c8;
  constexpr bool kPre = EP == EP_DGELU || EP == EP_STORE || EP == EP_CONV_BB;
  const uint16_t* psrc = EP == EP_DGELU ? a.aux : (EP == EP_CONV_BB ? a.sz : a.cin);
  // (EP_CONV_BB holds more per-channel state: an 8-row window, each slot refilled with row it + 8
  // once row it is consumed, so 8 loads stay in flight without spilling)
  constexpr int kPN = EP == EP_CONV_BB ? 8 : 16;
  uint4 pre[kPre ? kPN : 1];
  auto pre_row = [&](int it) {
    return *reinterpret_cast<const uint4*>(
        psrc + static_cast<int64_t>(m0 + wm * 128 + 8 * it + lrow) * a.ldy + ncol);
  };
  if (kPre && psrc) {
#pragma unroll
    for (int it = 0; it < kPN; ++it) pre[it] = pre_row(it);
  }
  char* img = smem + wave * (128 * 128);
  // lane's 16 output channels (4 per accumulator column group): n = ni 16 + 4 fc + j
  float bias[4][4];
  if (a.bias) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const uint2 bv = *reinterpret_cast<const uint2*>(a.bias + n0 + wn * 64 + ni * 16 + 4 * fc);
      bias[ni][0] = __uint_as_float(bv.x << 16);
      bias[ni][1] = __uint_as_float(bv.x & 0xffff0000u);
      bias[ni][2] = __uint_as_float(bv.y << 16);
      bias[ni][3] = __uint_as_float(bv.y & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) bias[ni][j] = 0.f;
  }
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const f32x4 v = acc[mi][ni];
      const uint2 w = make_uint2(pk_bf16(v[0] + bias[ni][0], v[1] + bias[ni][1]),
                                 pk_bf16(v[2] + bias[ni][2], v[3] + bias[ni][3]));
      const int row = mi * 16 + fr;
      const int ch = ni * 2 + (fc >> 1);
      *reinterpret_cast<uint2*>(img + swz(row, ch) + 8 * (fc & 1)) = w;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();

  float cs[8], cq[8], sh[8], esc[8], ebi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cs[e] = 0.f;
    cq[e] = 0.f;
  }
  if constexpr (EP == EP_CONV_ST || EP == EP_CONV_BB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) sh[e] = a.shift ? a.shift[ncol + e] : 0.f;
  }
  if constexpr (EP == EP_CONV_BB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      esc[e] = a.ep_sc[ncol + e];
      ebi[e] = a.ep_bi[ncol + e];
    }
  }
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int row = 8 * it + lrow;
    const uint4 v = *reinterpret_cast<const uint4*>(img + swz(row, c8));
    const int64_t m = m0 + wm * 128 + row;
    uint16_t* yp = a.y + m * a.ldy + ncol;
    if constexpr (EP == EP_CONV_ST || EP == EP_CONV_BB) {
      *reinterpret_cast<uint4*>(yp) = v;
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      if constexpr (EP == EP_CONV_ST) {   // shifted sums of the stored bf16 values
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float lo = __uint_as_float(w4[q] << 16) - sh[2 * q];
          const float hi = __uint_as_float(w4[q] & 0xffff0000u) - sh[2 * q + 1];
          cs[2 * q] += lo;
          cs[2 * q + 1] += hi;
          cq[2 * q] = fmaf(lo, lo, cq[2 * q]);
          cq[2 * q + 1] = fmaf(hi, hi, cq[2 * q + 1]);
        }
      } else {   // BN + ReLU backward sums: y' = relu'(z sc + bi) y, s += y', q += y' (z - mean)
        const uint4 zv = pre[it % kPN];
        if (kPN == 8 && it + 8 < 16) pre[it % kPN] = pre_row(it + 8);
        const uint32_t z4[4] = {zv.x, zv.y, zv.z, zv.w};
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
    } else if constexpr (EP == EP_STORE) {
      if (a.cin) {   // y = bf16(bf16(acc + bias) + cin): a residual gradient added on the way out
        const uint4 cv = pre[it];
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w}, c4[4] = {cv.x, cv.y, cv.z, cv.w};
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = pk_bf16(__uint_as_float(w4[q] << 16) + __uint_as_float(c4[q] << 16),
                         __uint_as_float(w4[q] & 0xffff0000u) + __uint_as_float(c4[q] & 0xffff0000u));
        *reinterpret_cast<uint4*>(yp) = make_uint4(o[0], o[1], o[2], o[3]);
      } else {
        *reinterpret_cast<uint4*>(yp) = v;
      }
    } else if constexpr (EP == EP_GELU) {
      *reinterpret_cast<uint4*>(a.aux + m * a.ldy + ncol) = v;
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        o[q] = pk_bf16(gelu_f(__uint_as_float(w4[q] << 16)),
                       gelu_f(__uint_as_float(w4[q] & 0xffff0000u)));
      *reinterpret_cast<uint4*>(yp) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {   // EP_DGELU
      const uint4 hv = pre[it];
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w}, h4[4] = {hv.x, hv.y, hv.z, hv.w};
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        o[q] = pk_bf16(__uint_as_float(w4[q] << 16) * dgelu_f(__uint_as_float(h4[q] << 16)),
                       __uint_as_float(w4[q] & 0xffff0000u) *
                           dgelu_f(__uint_as_float(h4[q] & 0xffff0000u)));
        cs[2 * q] += __uint_as_float(o[q] << 16);
        cs[2 * q + 1] += __uint_as_float(o[q] & 0xffff0000u);
      }
      *reinterpret_cast<uint4*>(yp) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
  if constexpr (EP == EP_CONV_ST || EP == EP_CONV_BB) {
    // lanes with equal lane & 7 hold the same 8 channels: fixed-order xor tree over lane >> 3;
    // one partial row per (tile, wave row) of conv_gemm.hip's slab layout
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s1 = cs[e], s2 = cq[e];
      s1 += __shfl_xor(s1, 8, 64);
      s2 += __shfl_xor(s2, 8, 64);
      s1 += __shfl_xor(s1, 16, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      cs[e] = s1;
      cq[e] = s2;
    }
    if (lane < 8) {
      const int R = static_cast<int>(a.M / TM) * T::WMR;
      float* p = a.part + (static_cast<int64_t>(ntile) * R + mtile * T::WMR + wm) * 2 * TN +
                 wn * 64 + 8 * lane;
      reinterpret_cast<float4*>(p)[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
      reinterpret_cast<float4*>(p)[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
      reinterpret_cast<float4*>(p + TN)[0] = make_float4(cq[0], cq[1], cq[2], cq[3]);
      reinterpret_cast<float4*>(p + TN)[1] = make_float4(cq[4], cq[5], cq[6], cq[7]);
    }
  }
  if constexpr (EP == EP_DGELU) {
    if (a.part) {
      // lanes with equal lane & 7 hold the same 8 channels: fixed-order xor tree over lane >> 3
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float s = cs[e];
        s += __shfl_xor(s, 8, 64);
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        cs[e] = s;
      }
      if (lane < 8) {
        float* p = a.part + static_cast<int64_t>(mtile * T::WMR + wm) * a.N + ncol;
        reinterpret_cast<float4*>(p)[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
        reinterpret_cast<float4*>(p)[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
  }
}

// out[s][n] = sum over the 128-row blocks r of segment s (rows_per_seg / 128 of them, in order)
// of part[r][n]; bf16 or fp32 output
__global__ __launch_bounds__(256) void colsum_fold_kernel(const float* __restrict__ part, int nblk_seg,
                                                         int N, int64_t ldo, void* out, int out_f32) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int s = blockIdx.y;
  if (n >= N) return;
  const float* p = part + static_cast<int64_t>(s) * nblk_seg * N + n;
  float v = 0.f;
  for (int r = 0; r < nblk_seg; ++r) v += p[static_cast<int64_t>(r) * N];
  if (out_f32) reinterpret_cast<float*>(out)[static_cast<int64_t>(s) * ldo + n] = v;
  else reinterpret_cast<uint16_t*>(out)[static_cast<int64_t>(s) * ldo + n] = f2bf(v);
}

}  // namespace

bool gemm_nt_eligible(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N > 0 && K > 0 && M % kT == 0 && N % kT == 0 && K % kBK == 0 &&
         (M / kT) * (N / kT) < (1LL << 31);
}

namespace {
template <int TM>
hipError_t launch_tm(const GemmArgs& a, int ep, hipStream_t st) {
  using T = Tile<TM>;
  const int tiles = static_cast<int>((a.M / TM) * (a.N / T::TN));
#define CML_GEMM_S(E, CV, S)                                                                 \
  do {                                                                                       \
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_kernel<E, CV, TM, S>),         \
                        hipFuncAttributeMaxDynamicSharedMemorySize, T::Lds);                 \
    gemm_nt_kernel<E, CV, TM, S><<<tiles, kThreads, T::Lds, st>>>(a);                        \
  } while (0)
#define CML_GEMM(E, CV) CML_GEMM_S(E, CV, false)
  if (a.conv && a.s2) {   // stride-2 forward: plain or with the BN statistics
    switch (ep) {
      case EP_STORE: CML_GEMM_S(EP_STORE, true, true); break;
      case EP_CONV_ST: CML_GEMM_S(EP_CONV_ST, true, true); break;
      default: return hipErrorInvalidValue;
    }
  } else if (a.conv) {
    switch (ep) {
      case EP_STORE: CML_GEMM(EP_STORE, true); break;
      case EP_CONV_ST: CML_GEMM(EP_CONV_ST, true); break;
      case EP_CONV_BB: CML_GEMM(EP_CONV_BB, true); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    if constexpr (TM != 256) {
      return hipErrorInvalidValue;
    } else {
      switch (ep) {
        case EP_STORE: CML_GEMM(EP_STORE, false); break;
        case EP_GELU: CML_GEMM(EP_GELU, false); break;
        case EP_DGELU: CML_GEMM(EP_DGELU, false); break;
        default: return hipErrorInvalidValue;
      }
    }
  }
#undef CML_GEMM
#undef CML_GEMM_S
  return hipGetLastError();
}

bool check_ptrs(const GemmArgs& a, int ep) {
  if ((a.lda % 8) || (a.ldb % 8) || (a.ldy % 8)) return false;
  if ((reinterpret_cast<uintptr_t>(a.a) | reinterpret_cast<uintptr_t>(a.b) |
       reinterpret_cast<uintptr_t>(a.y)) % 16)
    return false;
  if ((ep == EP_GELU || ep == EP_DGELU) && (a.aux == nullptr || reinterpret_cast<uintptr_t>(a.aux) % 16))
    return false;
  return true;
}

// CML_GEMM2_TALL: the fewest 512 x 128 tiles for which a 128-channel 3x3 conv takes the tall
// tile (default 1024, four rounds of 256 CUs: batch 2048's 3136 tiles, not batch 256's 392;
// 0 disables it: A/B)
int tall_min_tiles() {
  static const int v = [] {
    const char* e = getenv("CML_GEMM2_TALL");
    return e ? atoi(e) : 1024;
  }();
  return v;
}
}  // namespace

// CML_GEMM_GM: m-tiles per tile group of the plain (non-conv) GEMM (default 4; 0 / 1: n
// fastest, the round-5 order). An XCD then runs a 4 (m) x 8 (n) block of tiles instead of one
// m-row: with 8, 8192^3 1.28 -> 1.35 PFLOP/s and the Llama-3-8B w13 / output-head forwards 1.34
// -> 1.44-1.46 (profiles/r06_15/); 4 is 1-4 % faster again on most Llama shapes (w13 forward /
// NT weight gradient, wo, w2 data gradient; w2 forward 1.5 % slower) and the Llama step -1.3 ms,
// ResNet unchanged (profiles/r06_32/, profiles/r06_33/)
int gemm_gm() {
  static const int v = [] {
    const char* e = getenv("CML_GEMM_GM");
    return e ? atoi(e) : 4;
  }();
  return v;
}

hipError_t launch_gemm_nt(const GemmArgs& a0, int ep, hipStream_t st) {
  if (!gemm_nt_eligible(a0.M, a0.N, a0.K) || !check_ptrs(a0, ep)) return hipErrorInvalidValue;
  GemmArgs a = a0;
  a.gm = gemm_gm();
  return launch_tm<256>(a, ep, st);
}

int gemm_conv_tm(int64_t M, int N, int C) {
  if (M <= 0 || M >= (1LL << 31) || C % kBK || 9LL * C > 65536) return 0;
  if (M % kT == 0 && N % kT == 0) return 256;
  const int tall = tall_min_tiles();
  if (tall > 0 && N % 128 == 0 && M % 512 == 0 && (M / 512) * (N / 128) >= tall) return 512;
  return 0;
}

bool gemm_conv_eligible(int64_t M, int N, int C) { return gemm_conv_tm(M, N, C) != 0; }

hipError_t launch_gemm_conv(const GemmArgs& a0, int ep, hipStream_t st) {
  GemmArgs a = a0;
  a.conv = 1;
  a.K = 9LL * a.C;
  a.lda = a.C;
  a.ldb = a.K;
  a.ldy = a.N;
  const int tm = gemm_conv_tm(a.M, static_cast<int>(a.N), a.C);
  if (!tm || !a.zero || !a.a || !a.b || !a.y) return hipErrorInvalidValue;
  if (static_cast<int64_t>(a.H) * a.W < 1 || a.M % (static_cast<int64_t>(a.H) * a.W))
    return hipErrorInvalidValue;
  // stride 2: the output grid must be the input's ((IH - 1) / 2 + 1) x ((IW - 1) / 2 + 1)
  if (a.s2 && (a.IH < 1 || a.IW < 1 || (a.IH - 1) / 2 + 1 != a.H || (a.IW - 1) / 2 + 1 != a.W ||
               static_cast<int64_t>(a.M / (static_cast<int64_t>(a.H) * a.W)) * a.IH * a.IW >=
                   (1LL << 31) || ep == EP_CONV_BB))
    return hipErrorInvalidValue;
  if ((ep == EP_CONV_ST || ep == EP_CONV_BB) && !a.part) return hipErrorInvalidValue;
  if (ep == EP_CONV_BB && (!a.sz || !a.ep_sc || !a.ep_bi)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(a.zero) % 16) || !check_ptrs(a, ep)) return hipErrorInvalidValue;
  return tm == 512 ? launch_tm<512>(a, ep, st) : launch_tm<256>(a, ep, st);
}

hipError_t launch_colsum_fold(const float* part, int64_t M, int N, int nseg, void* out, int64_t ldo,
                              int out_f32, hipStream_t st) {
  if (nseg < 1 || M % (128LL * nseg) != 0 || N % 8 != 0) return hipErrorInvalidValue;
  const int nblk_seg = static_cast<int>(M / 128 / nseg);
  dim3 grid((N + 255) / 256, nseg);
  colsum_fold_kernel<<<grid, 256, 0, st>>>(part, nblk_seg, N, ldo, out, out_f32);
  return hipGetLastError();
}

}  // namespace cml
