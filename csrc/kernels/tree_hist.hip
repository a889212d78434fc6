// Histogram split search for level-synchronous tree ensembles (random forest / gradient boosting,
// select/hist_trees.py; reference hot loops: randomForest 2k/5k/10k trees with proximity
// `cml_targetaml_seanalysis.Rmd:1037-1050`, xgboost / sklearn GB `scripts/model_comp.py:6-34`).
//
// One level of every tree in a chunk at once: for each (tree t, node) and each of its kk
// candidate features, build the (bin -> split statistics) histogram over the node's samples,
// scan the bins to score every threshold, and return the node's best (gain, feature slot, bin).
// The torch formulation materialises [T, n, kk] int64 histogram indices, scatter-adds them with
// float atomics (order-dependent sums), and writes / re-reads [T, L, kk, B, 2] histograms and
// gains; here one workgroup per (t, node) keeps each candidate feature's histogram in its own
// LDS slice, adds the samples in index order (deterministic), and only the per-node winners leave
// the chip. Empty nodes exit immediately, which at deep levels is most of them.
//
// crit 0 (Gini, stats = (w, w*y)): gain = gw(T) - gw(L) - gw(R), gw(s) = w - (wy^2 + (w-wy)^2) / w,
//                                  valid if both children have w >= 1;
// crit 1 (XGBoost, stats = (g, h)): gain = (G_L^2/(H_L+lam) + G_R^2/(H_R+lam) - G^2/(H+lam)) / 2,
//                                  valid if both children have h >= min_child.
// Ties resolve to the first (feature slot, bin) in row-major order, like torch.max.
#include <math.h>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kTW = 64;        // threads (candidate features in flight) per workgroup
constexpr int kMaxBins = 64;
constexpr int kHS = 2 * kMaxBins + 1;   // per-lane LDS histogram stride (odd: no bank conflicts)

__device__ __forceinline__ float gw(float w, float wy) {
  return w - (wy * wy + (w - wy) * (w - wy)) / fmaxf(w, 1e-12f);
}
__device__ __forceinline__ float sc(float g, float h, float lam) { return g * g / (h + lam); }

__global__ __launch_bounds__(kTW) void split_search_kernel(
    const uint8_t* __restrict__ Xb, const int* __restrict__ node_local,
    const float* __restrict__ stat, const int* __restrict__ feats, const float* __restrict__ tot,
    int L, int n, int p, int kk, int B, int crit, float lam, float min_child,
    float* __restrict__ out_gain, int* __restrict__ out_slot, int* __restrict__ out_bin) {
  __shared__ float hist[kTW * kHS];
  __shared__ float bg[kTW];
  __shared__ int bj[kTW], bb[kTW];
  const int tn = blockIdx.x;            // t * L + node
  const int t = tn / L, node = tn % L;
  const float T0 = tot[2 * tn], T1 = tot[2 * tn + 1];
  const int lane = threadIdx.x;
  float best = -INFINITY;
  int best_j = 0, best_b = 0;
  const bool empty = crit == 0 ? !(T0 > 0.f) : false;
  if (!empty) {
    const int* nl = node_local + static_cast<int64_t>(t) * n;
    const float* st = stat + static_cast<int64_t>(t) * n * 2;
    const int* fs = feats + static_cast<int64_t>(tn) * kk;
    const float tg = crit == 0 ? gw(T0, T1) : sc(T0, T1, lam);
    for (int j0 = 0; j0 < kk; j0 += kTW) {
      const int j = j0 + lane;
      const bool act = j < kk;
      const int f = act ? fs[j] : 0;
      float* hl = hist + lane * kHS;
      for (int b = 0; b < 2 * B; ++b) hl[b] = 0.f;
      for (int s = 0; s < n; ++s) {       // samples in index order: deterministic sums
        if (nl[s] != node) continue;       // wave-uniform branch
        const float s0 = st[2 * s], s1 = st[2 * s + 1];
        if (act) {
          const int b = Xb[static_cast<int64_t>(s) * p + f];
          hl[2 * b] += s0;
          hl[2 * b + 1] += s1;
        }
      }
      if (act) {
        float c0 = 0.f, c1 = 0.f;
        for (int b = 0; b + 1 < B; ++b) {   // threshold b: left = bins <= b
          c0 += hl[2 * b];
          c1 += hl[2 * b + 1];
          const float r0 = T0 - c0, r1 = T1 - c1;
          float g;
          if (crit == 0) {
            g = (c0 >= 1.f && r0 >= 1.f) ? tg - gw(c0, c1) - gw(r0, r1) : -INFINITY;
          } else {
            g = (c1 >= min_child && r1 >= min_child)
                    ? 0.5f * (sc(c0, c1, lam) + sc(r0, r1, lam) - tg) : -INFINITY;
          }
          if (g > best) {   // strict: first (slot, bin) wins ties
            best = g;
            best_j = j;
            best_b = b;
          }
        }
      }
    }
  }
  bg[lane] = best;
  bj[lane] = best_j;
  bb[lane] = best_b;
  __syncthreads();
  if (lane == 0) {
    float g = bg[0];
    int jj = bj[0], b = bb[0];
    for (int k = 1; k < kTW; ++k) {
      if (bg[k] > g || (bg[k] == g && (bj[k] < jj || (bj[k] == jj && bb[k] < b)))) {
        g = bg[k];
        jj = bj[k];
        b = bb[k];
      }
    }
    out_gain[tn] = g;
    out_slot[tn] = jj;
    out_bin[tn] = b;
  }
}

// Exact-threshold forests (select/hist_trees.py ExactForest): features binned by the rank of their
// distinct training values (B <= 128 bins, so every midpoint between consecutive distinct values is
// a candidate threshold, as in R randomForest's CART), and the node's mtry candidate features drawn
// HERE instead of from a [T, L, p] tensor of random keys (which at depth 12+ would be billions of
// floats): kk distinct features per (tree, node) by rounds of 64 counter-hashed draws, accepted in
// lane order against an LDS bitmap (sampling without replacement, deterministic for a seed).
// Returns the winning feature id (not its slot). Gini (crit 0) or XGBoost gain (crit 1).
constexpr int kXBins = 128;
constexpr int kXHS = 2 * kXBins + 1;
constexpr int kXMaxK = 512;          // candidate features per node
constexpr int kXMaxP = 65536;        // features (bitmap bits)

__device__ __forceinline__ uint32_t mix32(uint64_t z) {   // splitmix64 finaliser
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return static_cast<uint32_t>((z ^ (z >> 31)) >> 32);
}

__global__ __launch_bounds__(kTW) void split_search_sampled_kernel(
    const uint8_t* __restrict__ Xb, const int* __restrict__ node_local,
    const float* __restrict__ stat, const float* __restrict__ tot, int L, int n, int p, int kk,
    int B, int crit, float lam, float min_child, uint64_t seed, float* __restrict__ out_gain,
    int* __restrict__ out_feat, int* __restrict__ out_bin) {
  __shared__ float hist[kTW * kXHS];
  __shared__ uint32_t bitmap[kXMaxP / 32];
  __shared__ int cand[kXMaxK];
  __shared__ float bg[kTW];
  __shared__ int bj[kTW], bb[kTW];
  const int tn = blockIdx.x;            // t * L + node
  const int t = tn / L, node = tn % L;
  const float T0 = tot[2 * tn], T1 = tot[2 * tn + 1];
  const int lane = threadIdx.x;
  const bool empty = crit == 0 ? !(T0 > 0.f) : false;
  if (empty) {
    if (lane == 0) {
      out_gain[tn] = -INFINITY;
      out_feat[tn] = 0;
      out_bin[tn] = 0;
    }
    return;
  }
  // ---- kk distinct candidate features: rounds of 64 draws, lane-ordered acceptance
  for (int w = lane; w < (p + 31) / 32; w += kTW) bitmap[w] = 0u;
  __syncthreads();
  const uint64_t key = seed ^ (static_cast<uint64_t>(tn) * 0xd1b54a32d192ed03ull);
  int have = 0;
  for (int round = 0; have < kk; ++round) {
    const uint32_t r = mix32(key + static_cast<uint64_t>(round) * kTW + lane);
    const int f = static_cast<int>((static_cast<uint64_t>(r) * static_cast<uint32_t>(p)) >> 32);
    bool fresh = !((bitmap[f >> 5] >> (f & 31)) & 1u);
    for (int o = 0; o < kTW; ++o) {      // an earlier lane of this round drew the same feature
      const int fo = __shfl(f, o, kTW);
      if (o < lane && fo == f) fresh = false;
    }
    const uint64_t acc = __ballot(fresh);
    const int pos = have + __popcll(acc & ((1ull << lane) - 1ull));
    if (fresh && pos < kk) {
      cand[pos] = f;
      atomicOr(&bitmap[f >> 5], 1u << (f & 31));
    }
    have = min(kk, have + static_cast<int>(__popcll(acc)));
    __syncthreads();
  }
  // ---- histograms of the candidates (as split_search_kernel), best (gain, slot, bin)
  float best = -INFINITY;
  int best_j = 0, best_b = 0;
  const int* nl = node_local + static_cast<int64_t>(t) * n;
  const float* st = stat + static_cast<int64_t>(t) * n * 2;
  const float tg = crit == 0 ? gw(T0, T1) : sc(T0, T1, lam);
  for (int j0 = 0; j0 < kk; j0 += kTW) {
    const int j = j0 + lane;
    const bool act = j < kk;
    const int f = act ? cand[j] : 0;
    float* hl = hist + lane * kXHS;
    for (int b = 0; b < 2 * B; ++b) hl[b] = 0.f;
    for (int s = 0; s < n; ++s) {       // samples in index order: deterministic sums
      if (nl[s] != node) continue;       // wave-uniform branch
      const float s0 = st[2 * s], s1 = st[2 * s + 1];
      if (act) {
        const int b = Xb[static_cast<int64_t>(s) * p + f];
        hl[2 * b] += s0;
        hl[2 * b + 1] += s1;
      }
    }
    if (act) {
      float c0 = 0.f, c1 = 0.f;
      for (int b = 0; b + 1 < B; ++b) {   // threshold b: left = bins <= b
        c0 += hl[2 * b];
        c1 += hl[2 * b + 1];
        const float r0 = T0 - c0, r1 = T1 - c1;
        float g;
        if (crit == 0) {
          g = (c0 >= 1.f && r0 >= 1.f) ? tg - gw(c0, c1) - gw(r0, r1) : -INFINITY;
        } else {
          g = (c1 >= min_child && r1 >= min_child)
                  ? 0.5f * (sc(c0, c1, lam) + sc(r0, r1, lam) - tg) : -INFINITY;
        }
        if (g > best) {
          best = g;
          best_j = j;
          best_b = b;
        }
      }
    }
  }
  bg[lane] = best;
  bj[lane] = best_j;
  bb[lane] = best_b;
  __syncthreads();
  if (lane == 0) {
    float g = bg[0];
    int jj = bj[0], b = bb[0];
    for (int k = 1; k < kTW; ++k) {
      if (bg[k] > g || (bg[k] == g && (bj[k] < jj || (bj[k] == jj && bb[k] < b)))) {
        g = bg[k];
        jj = bj[k];
        b = bb[k];
      }
    }
    out_gain[tn] = g;
    out_feat[tn] = cand[jj];
    out_bin[tn] = b;
  }
}

}  // namespace

hipError_t launch_split_search(const uint8_t* Xb, const int* node_local, const float* stat,
                               const int* feats, const float* tot, int T, int L, int n, int p,
                               int kk, int B, int crit, float lam, float min_child,
                               float* out_gain, int* out_slot, int* out_bin, hipStream_t st) {
  if (T < 1 || L < 1 || n < 1 || p < 1 || kk < 1 || B < 2 || B > kMaxBins || (crit != 0 && crit != 1))
    return hipErrorInvalidValue;
  const int64_t blocks = static_cast<int64_t>(T) * L;
  if (blocks > 2147483647LL) return hipErrorInvalidValue;
  split_search_kernel<<<static_cast<unsigned>(blocks), kTW, 0, st>>>(
      Xb, node_local, stat, feats, tot, L, n, p, kk, B, crit, lam, min_child, out_gain, out_slot,
      out_bin);
  return hipGetLastError();
}

hipError_t launch_split_search_sampled(const uint8_t* Xb, const int* node_local,
                                       const float* stat, const float* tot, int T, int L, int n,
                                       int p, int kk, int B, int crit, float lam, float min_child,
                                       uint64_t seed, float* out_gain, int* out_feat, int* out_bin,
                                       hipStream_t st) {
  if (T < 1 || L < 1 || n < 1 || p < 1 || p > kXMaxP || kk < 1 || kk > kXMaxK || kk > p || B < 2 ||
      B > kXBins || (crit != 0 && crit != 1))
    return hipErrorInvalidValue;
  const int64_t blocks = static_cast<int64_t>(T) * L;
  if (blocks > 2147483647LL) return hipErrorInvalidValue;
  split_search_sampled_kernel<<<static_cast<unsigned>(blocks), kTW, 0, st>>>(
      Xb, node_local, stat, tot, L, n, p, kk, B, crit, lam, min_child, seed, out_gain, out_feat,
      out_bin);
  return hipGetLastError();
}

}  // namespace cml
