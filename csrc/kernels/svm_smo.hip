// Batched dual C-SVC solver (SMO with libsvm's second-order working-set selection), one wave64
// per problem (select/svm.py C23/C33, MLSeq svmRadial C31).
//
//   min 1/2 a^T Q a - e^T a   s.t.  0 <= a <= C,  y^T a = 0,   Q_ts = y_t y_s K_ts
//
// The problems of the reference are small (n ~ 50-150 samples) and the algorithm is a long
// sequential chain of O(n) steps, so the design is latency-first: a single wave owns a problem,
// keeps a, G (dual gradient), y and diag(K) in LDS and reduces with cross-lane shuffles only (no
// workgroup barrier beyond the wave's own), and reads the two kernel rows i, j of each step from
// global memory (L2-resident: n^2 fp64 = 180 KB at n = 150). Many problems (CV folds x cost grid,
// the four runSVM fits) run as independent waves of one launch.
//
// Per step: i = argmax_{t in I_up} -y_t G_t,  stop when that minus min_{t in I_low} -y_t G_t < tol,
// j = argmin_{t in I_low, -y_t G_t < gmax} -(gmax + y_t G_t)^2 / (K_ii + K_tt - 2 K_it), the
// analytic two-variable update clipped to the box, then G += Q[:, i] da_i + Q[:, j] da_j.
// Ties resolve to the lowest index (numpy argmax / argmin order of the host oracle).
#include <hip/hip_runtime.h>

#include <climits>

#include "kernels.h"

namespace cml {
namespace {

constexpr int kWave = 64;

__device__ __forceinline__ void take_max(double& v, int& i, double v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}
__device__ __forceinline__ void take_min(double& v, int& i, double v2, int i2) {
  if (v2 < v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}
__device__ __forceinline__ void wave_argmax(double& v, int& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) take_max(v, i, __shfl_xor(v, off), __shfl_xor(i, off));
}
__device__ __forceinline__ void wave_argmin(double& v, int& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) take_min(v, i, __shfl_xor(v, off), __shfl_xor(i, off));
}

__global__ __launch_bounds__(kWave) void smo_kernel(const double* __restrict__ K,
                                                    const double* __restrict__ Y,
                                                    const int* __restrict__ ns, int nmax,
                                                    const double* __restrict__ Cs, double tol,
                                                    int max_iter, double* __restrict__ alpha,
                                                    double* __restrict__ grad,
                                                    int* __restrict__ iters) {
  extern __shared__ double smem[];
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = ns[b];
  const double C = Cs[b];
  const double tau = 1e-12;
  const double inf = __builtin_huge_val();
  const double* Kb = K + static_cast<size_t>(b) * nmax * nmax;
  double* a = smem;
  double* G = a + nmax;
  double* y = G + nmax;
  double* dg = y + nmax;
  for (int t = lane; t < n; t += kWave) {
    a[t] = 0.0;
    G[t] = -1.0;
    y[t] = Y[static_cast<size_t>(b) * nmax + t] > 0 ? 1.0 : -1.0;
    dg[t] = Kb[static_cast<size_t>(t) * nmax + t];
  }
  __syncthreads();
  int it = 0;
  for (; it < max_iter; ++it) {
    double vmax = -inf, vmin = inf;
    int imax = INT_MAX, imin = INT_MAX;
    for (int t = lane; t < n; t += kWave) {
      const double yt = y[t], at = a[t], v = -yt * G[t];
      const bool up = (yt > 0 && at < C) || (yt < 0 && at > 0);
      const bool lo = (yt > 0 && at > 0) || (yt < 0 && at < C);
      if (up) take_max(vmax, imax, v, t);
      if (lo) take_min(vmin, imin, v, t);
    }
    wave_argmax(vmax, imax);
    wave_argmin(vmin, imin);
    if (imax == INT_MAX || imin == INT_MAX || vmax - vmin < tol) break;
    const int i = imax;
    const double gmax = vmax;
    const double* Ki = Kb + static_cast<size_t>(i) * nmax;
    const double Kii = dg[i];
    double omin = inf;
    int j = INT_MAX;
    for (int t = lane; t < n; t += kWave) {
      const double yt = y[t], at = a[t], v = -yt * G[t];
      const bool lo = (yt > 0 && at > 0) || (yt < 0 && at < C);
      if (lo && v < gmax) {
        const double bb = gmax - v;
        double aa = Kii + dg[t] - 2.0 * Ki[t];
        if (!(aa > 0)) aa = tau;
        take_min(omin, j, -(bb * bb) / aa, t);
      }
    }
    wave_argmin(omin, j);
    if (j == INT_MAX || !(omin < inf)) break;
    // analytic two-variable step (every lane computes it: no broadcast needed)
    const double* Kj = Kb + static_cast<size_t>(j) * nmax;
    const double yi = y[i], yj = y[j];
    const double Qii = Kii, Qjj = dg[j], Qij = yi * yj * Ki[j];
    const double ai0 = a[i], aj0 = a[j];
    double ai, aj;
    if (yi != yj) {
      double quad = Qii + Qjj + 2.0 * Qij;
      if (quad < tau) quad = tau;
      const double delta = (-G[i] - G[j]) / quad;
      const double diff = ai0 - aj0;
      ai = ai0 + delta;
      aj = aj0 + delta;
      if (diff > 0 && aj < 0) {
        aj = 0;
        ai = diff;
      } else if (diff <= 0 && ai < 0) {
        ai = 0;
        aj = -diff;
      }
      if (diff > 0 && ai > C) {
        ai = C;
        aj = C - diff;
      } else if (diff <= 0 && aj > C) {
        aj = C;
        ai = C + diff;
      }
    } else {
      double quad = Qii + Qjj - 2.0 * Qij;
      if (quad < tau) quad = tau;
      const double delta = (G[i] - G[j]) / quad;
      const double s = ai0 + aj0;
      ai = ai0 - delta;
      aj = aj0 + delta;
      if (s > C && ai > C) {
        ai = C;
        aj = s - C;
      } else if (s <= C && aj < 0) {
        aj = 0;
        ai = s;
      }
      if (s > C && aj > C) {
        aj = C;
        ai = s - C;
      } else if (s <= C && ai < 0) {
        ai = 0;
        aj = s;
      }
    }
    const double dai = ai - ai0, daj = aj - aj0;
    __syncthreads();  // every lane has read a[i], a[j], G[i], G[j]
    for (int t = lane; t < n; t += kWave) {
      const double yt = y[t];
      G[t] += (Ki[t] * (yt * yi)) * dai + (Kj[t] * (yt * yj)) * daj;
    }
    if (lane == 0) {
      a[i] = ai;
      a[j] = aj;
    }
    __syncthreads();
  }
  for (int t = lane; t < n; t += kWave) {
    alpha[static_cast<size_t>(b) * nmax + t] = a[t];
    grad[static_cast<size_t>(b) * nmax + t] = G[t];
  }
  if (lane == 0) iters[b] = it;
}

}  // namespace

int smo_max_n() { return 2048; }

hipError_t launch_smo(const double* K, const double* y, const int* ns, int B, int nmax,
                      const double* C, double tol, int max_iter, double* alpha, double* grad,
                      int* iters, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if (nmax <= 0 || nmax > smo_max_n()) return hipErrorInvalidValue;
  const size_t lds = 4 * static_cast<size_t>(nmax) * sizeof(double);
  hipLaunchKernelGGL(smo_kernel, dim3(B), dim3(kWave), lds, stream, K, y, ns, nmax, C, tol,
                     max_iter, alpha, grad, iters);
  return hipGetLastError();
}

}  // namespace cml
