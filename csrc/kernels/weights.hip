// Robust weights from the n x n Gram matrix (one wave, fp64, no host round trip).
//
// Every vector-valued rule of the engine reduces to "weights over the worker rows" once the Gram
// matrix is known, because each iterate is a linear combination of the rows:
//   Krum / Multi-Krum   score_i = sum of the n-f-2 smallest d_ij, d_ij = G_ii + G_jj - 2 G_ij;
//                       the m lowest scores (ties -> lower index) get weight 1/m.
//   Weiszfeld (RFA)     z = sum_j a_j x_j  =>  ||x_i - z||^2 = G_ii - 2 (G a)_i + a^T G a, so all
//                       iterations run here on G and the data is read once more, by the fused
//                       weighted update, instead of once per iteration.
//   Centered clipping   same trick on the (n+1) Gram of [x_1..x_n, v_prev].
//   Bulyan              iterated Krum selects theta = n - 2f rows; the coordinate phase is the
//                       sorted kernel over those rows.
// Rows with a non-finite squared norm are Byzantine by definition: score +inf, weight 0.
// Lane i owns row i; ranks use (value, index) order so every rank computes identical weights.
//
// The same launch also (optionally) adds this step's selections to sel_counts, writes the
// medoid of G (the next step's Gram center, as gram_center_kernel) and -- for a G from the
// single centered pass around the PREVIOUS step's medoid -- guards against a captured center:
// a center worker that turns Byzantine with huge finite values overflows every honest centered
// row (x_i - x_c)^2, leaving its own all-zero row the only finite one. If at least half the
// worker rows are non-finite, the step is distrusted: gradient weights 0 (centered clipping
// keeps its previous aggregate), and the next center is -1 (the next Gram pass runs
// uncentered, where the overflowing row is the non-finite one).
#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kMax = 65;   // n <= 64 workers (+1 row for centered clipping)

__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
  return v;
}

// Sum of the k smallest of row i's distances to the rows in `mask` (excluding i).
__device__ double krum_score(const double* G, int n, int i, int k, const unsigned long long mask,
                             const bool* bad) {
  if (bad[i]) return __builtin_inf();
  if (k < 1) k = 1;   // floor: see ops/reference.py krum_scores
  if (k <= 0) return 0.0;
  double s = 0.0;
  const double gii = G[i * n + i];
  for (int j = 0; j < n; ++j) {
    if (j == i || !((mask >> j) & 1ull)) continue;
    double dj = bad[j] ? __builtin_inf() : fmax(gii + G[j * n + j] - 2.0 * G[i * n + j], 0.0);
    if (dj != dj) dj = __builtin_inf();
    // rank of d_ij among {d_il : l in mask, l != i} with index tie-break
    int rank = 0;
    for (int l = 0; l < n; ++l) {
      if (l == i || l == j || !((mask >> l) & 1ull)) continue;
      double dl = bad[l] ? __builtin_inf() : fmax(gii + G[l * n + l] - 2.0 * G[i * n + l], 0.0);
      if (dl != dl) dl = __builtin_inf();
      rank += (dl < dj) || (dl == dj && l < j);
    }
    if (rank < k) s += dj;
  }
  return s;
}

__device__ __forceinline__ void weights_rule(int rule, const double* __restrict__ G, int n, int f,
                                             int m, int iters, double eps, double tol, double tau,
                                             float* __restrict__ w, double* __restrict__ scores,
                                             int* __restrict__ sel, const bool* bad, double* sc,
                                             double* a) {
  const int i = threadIdx.x;

  if (rule == RULE_MEAN) {
    int good = 0;
    for (int r = 0; r < n; ++r) good += !bad[r];
    if (i < n) {
      w[i] = (!bad[i] && good > 0) ? 1.0f / good : 0.0f;
      if (scores) scores[i] = 0.0;
      if (sel) sel[i] = !bad[i];
    }
    return;
  }

  if (rule == RULE_KRUM || rule == RULE_MULTI_KRUM) {
    const unsigned long long all = n == 64 ? ~0ull : ((1ull << n) - 1ull);
    const int k = n - f - 2;
    if (i < n) sc[i] = krum_score(G, n, i, k, all, bad);
    __syncthreads();
    const int mm = rule == RULE_KRUM ? 1 : (m > 0 ? (m < n ? m : n) : n - f);
    if (i < n) {
      int rank = 0;
      for (int j = 0; j < n; ++j) rank += (sc[j] < sc[i]) || (sc[j] == sc[i] && j < i);
      const bool take = rank < mm;
      w[i] = take ? 1.0f / mm : 0.0f;
      if (scores) scores[i] = sc[i];
      if (sel) sel[i] = take;
    }
    return;
  }

  if (rule == RULE_BULYAN_SELECT) {
    // theta = n - 2f rounds; each round recomputes Krum over the remaining rows.
    __shared__ unsigned long long remaining;
    __shared__ int pick;
    if (i == 0) remaining = n == 64 ? ~0ull : ((1ull << n) - 1ull);
    __syncthreads();
    const int theta = n - 2 * f;
    unsigned long long chosen = 0;
    for (int round = 0; round < theta; ++round) {
      const unsigned long long rem = remaining;
      const int cnt = __popcll(rem);
      const bool mine = i < n && ((rem >> i) & 1ull);
      if (mine) sc[i] = krum_score(G, n, i, cnt - f - 2, rem, bad);
      __syncthreads();
      if (i == 0) {
        int best = -1;
        for (int j = 0; j < n; ++j) {
          if (!((rem >> j) & 1ull)) continue;
          if (best < 0 || sc[j] < sc[best]) best = j;
        }
        pick = best;
        remaining = rem & ~(1ull << best);
      }
      __syncthreads();
      chosen |= 1ull << pick;
      __syncthreads();
    }
    if (i == 0) {
      int c = 0;
      for (int j = 0; j < n; ++j)
        if ((chosen >> j) & 1ull) sel[c++] = j;
      sel[n] = c;
    }
    if (i < n) {
      w[i] = ((chosen >> i) & 1ull) ? 1.0f / theta : 0.0f;
      if (scores) scores[i] = 0.0;
    }
    return;
  }

  if (rule == RULE_GEOMED) {
    int good = 0;
    for (int r = 0; r < n; ++r) good += !bad[r];
    if (i < n) a[i] = (!bad[i] && good > 0) ? 1.0 / good : 0.0;
    __syncthreads();
    double dist = 0.0;
    for (int it = 0; it < iters; ++it) {
      double ga = 0.0;
      if (i < n && !bad[i])
        for (int j = 0; j < n; ++j)
          if (!bad[j]) ga += G[i * n + j] * a[j];
      const double aga = wave_sum(i < n ? a[i] * ga : 0.0);
      double b = 0.0;
      if (i < n && !bad[i]) {
        const double d2 = fmax(G[i * n + i] - 2.0 * ga + aga, 0.0);
        dist = sqrt(d2);
        b = 1.0 / fmax(dist, eps);
      }
      const double bs = wave_sum(b);
      const double an = bs > 0.0 ? b / bs : 0.0;
      const double delta = wmax(i < n ? fabs(an - a[i]) : 0.0);
      __syncthreads();
      if (i < n) a[i] = an;
      __syncthreads();
      if (tol > 0.0 && delta < tol) break;
    }
    if (i < n) {
      w[i] = static_cast<float>(a[i]);
      if (scores) scores[i] = dist;
      if (sel) sel[i] = a[i] > 0.0;
    }
    return;
  }

  if (rule == RULE_CCLIP) {
    // rows 0..n-1 workers, row n = previous aggregate v0; coefficients c over n+1 rows.
    const int N1 = n + 1;
    if (i <= n) a[i] = (i == n) ? 1.0 : 0.0;
    __syncthreads();
    for (int it = 0; it < iters; ++it) {
      // a non-finite worker row contributes nothing (its a[i] stays 0); its NaN / inf Gram row
      // must not reach gc either, or 0 * NaN poisons c^T G c for every lane (ops/reference.py
      // centered_clip_weights zeroes the bad rows and columns the same way)
      double gc = 0.0;
      if (i <= n && (i == n || !bad[i]))
        for (int j = 0; j <= n; ++j)
          if (!bad[j] || j == n) gc += G[i * N1 + j] * a[j];
      const double cgc = wave_sum(i <= n ? a[i] * gc : 0.0);
      double s = 0.0;
      if (i < n && !bad[i]) {
        const double d = sqrt(fmax(G[i * N1 + i] - 2.0 * gc + cgc, 0.0));
        s = fmin(tau / fmax(d, 1e-30), 1.0) / n;
      }
      const double ssum = wave_sum(s);
      double cn = 0.0;
      if (i <= n) cn = a[i] * (1.0 - ssum) + (i < n ? s : 0.0);
      __syncthreads();
      if (i <= n) a[i] = cn;
      __syncthreads();
    }
    if (i <= n) w[i] = static_cast<float>(a[i]);
    if (i < n) {
      if (scores) scores[i] = 0.0;
      if (sel) sel[i] = !bad[i];
    }
    return;
  }
}

__global__ __launch_bounds__(64) void robust_weights_kernel(int rule, const double* __restrict__ G,
                                                           int n, int f, int m, int iters,
                                                           double eps, double tol, double tau,
                                                           float* __restrict__ w,
                                                           double* __restrict__ scores,
                                                           int* __restrict__ sel, int guard,
                                                           int* __restrict__ center_out,
                                                           double* __restrict__ sel_counts,
                                                           int* __restrict__ nbad_io) {
  __shared__ bool bad[kMax];
  __shared__ double sc[kMax];
  __shared__ double a[kMax];
  const int i = threadIdx.x;
  const int nrows = rule == RULE_CCLIP ? n + 1 : n;   // Gram dimension
  // center_out holds the center THIS pass used (the engine passes one buffer): a pass that ran
  // uncentered (center < 0, e.g. the step after a trip) cannot have been captured, so the guard
  // is disarmed -- with half the rows genuinely non-finite it would otherwise trip every step
  // and freeze training instead of aggregating the finite rows
  const int center_in = center_out ? center_out[0] : 0;
  if (center_in < 0) guard = 0;
  // nbad_io: the previous pass's count of non-finite worker rows. A captured center shows as rows
  // that TURNED non-finite; workers that were already non-finite (genuine NaN / overflow, up to
  // half or more of them) are aggregated around as on an uncentered pass, every step
  const int nbad_prev = nbad_io ? nbad_io[0] : 0;
  for (int r = i; r < nrows; r += 64) {
    const double d = G[r * nrows + r];
    bad[r] = !(d == d) || d == __builtin_inf() || d == -__builtin_inf();
  }
  __syncthreads();
  weights_rule(rule, G, n, f, m, iters, eps, tol, tau, w, scores, sel, bad, sc, a);
  __syncthreads();
  int nbad = 0;
  for (int r = 0; r < n; ++r) nbad += bad[r];
  const bool trip = guard && 2 * nbad >= n && nbad > 0 && (!nbad_io || nbad > nbad_prev);
  if (nbad_io && i == 0) nbad_io[0] = nbad;
  if (trip) {
    if (i < nrows) w[i] = (rule == RULE_CCLIP && i == n) ? 1.0f : 0.0f;
    if (sel && rule != RULE_BULYAN_SELECT && i < n) sel[i] = 0;
  }
  if (sel_counts && i < n) sel_counts[i] += w[i] > 0.0f ? 1.0 : 0.0;
  if (center_out) {
    // medoid of the finite worker rows of G (gram_center_kernel's rule)
    double s_i = __builtin_inf();
    if (i < n) {
      const double gii = G[i * nrows + i];
      if (isfinite(gii)) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) {
          const double gjj = G[j * nrows + j];
          if (!isfinite(gjj)) continue;
          const double d = gii + gjj - 2.0 * G[i * nrows + j];
          s += d > 0.0 ? d : 0.0;
        }
        if (isfinite(s)) s_i = s;
      }
    }
    int idx = i;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double s2 = __shfl_xor(s_i, o, 64);
      const int i2 = __shfl_xor(idx, o, 64);
      if (s2 < s_i || (s2 == s_i && i2 < idx)) {
        s_i = s2;
        idx = i2;
      }
    }
    if (i == 0) center_out[0] = trip ? -1 : ((idx < n && isfinite(s_i)) ? idx : 0);
  }
}

}  // namespace

hipError_t launch_robust_weights(int rule, const double* G, int n, int f, int m, int iters,
                                 double eps, double tol, double tau, float* w, double* scores,
                                 int* sel, hipStream_t stream, int guard, int* center_out,
                                 double* sel_counts, int* nbad_io) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  if (rule == RULE_CCLIP && n > 63) return hipErrorInvalidValue;   // n + 1 rows, one per lane
  if (rule == RULE_BULYAN_SELECT && sel == nullptr) return hipErrorInvalidValue;
  robust_weights_kernel<<<1, 64, 0, stream>>>(rule, G, n, f, m, iters, eps, tol, tau, w, scores, sel,
                                              guard, center_out, sel_counts, nbad_io);
  return hipGetLastError();
}

}  // namespace cml
