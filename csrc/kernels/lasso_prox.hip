// Batched FISTA for L1 / elastic-net logistic regression (select/lasso.py fista_logistic: the
// glmnet lambda path x LOOCV folds of `cml_targetaml_seanalysis.Rmd:68-123` solved as B
// independent problems at once; the reference's hot loop, `cv.glmnet(nfolds = n_train)`).
//
// Per iteration the two GEMMs z = X v and g = X^T r stay on hipBLASLt; everything else is these
// kernels on [p, B] / [n, B] column-per-lane layouts (B = problems, contiguous):
//   resid : r = (sigmoid(z + v0) - y) * M / nb, and the intercept gradient sum_i r  (one pass)
//   prox  : nbeta = soft(v - t (g + lam (1 - a) v), t lam a), and per-row-slice partial sums of
//           the adaptive-restart test (v - nbeta) . (nbeta - beta)               (one pass)
//   scal  : per problem: fold the partials (fixed order), restart / momentum / t_k, intercept
//   mom   : v = nbeta + mom (nbeta - beta), with per-slice max |d| and max |nbeta| partials on
//           convergence-check iterations                                        (one pass)
// i.e. 7 passes over [p, B] instead of ~15 elementwise torch kernels, and no host sync.
#include <math.h>

#include "common.h"
#include "kernels.h"

namespace cml {
namespace {

constexpr int kLB = 256;
constexpr int kRows = 64;     // rows per slice of the [p, B] kernels

__global__ __launch_bounds__(kLB) void lasso_resid_kernel(const float* __restrict__ z,
                                                         const float* __restrict__ v0,
                                                         const float* __restrict__ y,
                                                         const float* __restrict__ M,
                                                         const float* __restrict__ nb,
                                                         float* __restrict__ r,
                                                         float* __restrict__ rsum, int n, int B) {
  const int b = blockIdx.x * kLB + threadIdx.x;
  if (b >= B) return;
  const float off = v0 ? v0[b] : 0.f;
  const float inv = 1.f / nb[b];
  float s = 0.f;
  for (int i = 0; i < n; ++i) {
    const int64_t e = static_cast<int64_t>(i) * B + b;
    const float p = 1.f / (1.f + __expf(-(z[e] + off)));
    const float ri = (p - y[i]) * M[e] * inv;
    r[e] = ri;
    s += ri;
  }
  if (rsum) rsum[b] = s;
}

__global__ __launch_bounds__(kLB) void lasso_prox_kernel(const float* __restrict__ v,
                                                        const float* __restrict__ beta,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ step,
                                                        const float* __restrict__ lam, float alpha,
                                                        float* __restrict__ nbeta,
                                                        float* __restrict__ part, int p, int B) {
  const int b = blockIdx.x * kLB + threadIdx.x;
  if (b >= B) return;
  const float t = step[b], l = lam[b];
  const float thr = t * l * alpha, ridge = l * (1.f - alpha);
  const int i0 = blockIdx.y * kRows;
  const int i1 = i0 + kRows < p ? i0 + kRows : p;
  float dot = 0.f;
  for (int i = i0; i < i1; ++i) {
    const int64_t e = static_cast<int64_t>(i) * B + b;
    const float vi = v[e], bi = beta[e];
    const float u = vi - t * (g[e] + ridge * vi);
    const float nbi = copysignf(fmaxf(fabsf(u) - thr, 0.f), u);
    nbeta[e] = nbi;
    dot = fmaf(vi - nbi, nbi - bi, dot);
  }
  part[static_cast<int64_t>(blockIdx.y) * B + b] = dot;
}

// per problem: restart test, momentum, t_k; intercept step (v0 / b0 when given)
__global__ __launch_bounds__(kLB) void lasso_scal_kernel(const float* __restrict__ part, int ns,
                                                        float* __restrict__ tk,
                                                        float* __restrict__ mom,
                                                        const float* __restrict__ step,
                                                        const float* __restrict__ rsum,
                                                        float* __restrict__ v0,
                                                        float* __restrict__ b0, int B) {
  const int b = blockIdx.x * kLB + threadIdx.x;
  if (b >= B) return;
  float dot = 0.f;
  for (int s = 0; s < ns; ++s) dot += part[static_cast<int64_t>(s) * B + b];
  const float t = tk[b];
  const float tn = 0.5f * (1.f + sqrtf(1.f + 4.f * t * t));
  const bool up = dot > 0.f;
  const float m = up ? 0.f : (t - 1.f) / tn;
  tk[b] = up ? 1.f : tn;
  mom[b] = m;
  if (v0 != nullptr) {
    const float nb0 = v0[b] - step[b] * rsum[b];
    v0[b] = nb0 + m * (nb0 - b0[b]);
    b0[b] = nb0;
  }
}

__global__ __launch_bounds__(kLB) void lasso_mom_kernel(const float* __restrict__ nbeta,
                                                       float* __restrict__ beta,
                                                       float* __restrict__ v,
                                                       const float* __restrict__ mom,
                                                       float* __restrict__ part, int p, int B) {
  const int b = blockIdx.x * kLB + threadIdx.x;
  if (b >= B) return;
  const float m = mom[b];
  const int i0 = blockIdx.y * kRows;
  const int i1 = i0 + kRows < p ? i0 + kRows : p;
  float md = 0.f, mb = 0.f;
  for (int i = i0; i < i1; ++i) {
    const int64_t e = static_cast<int64_t>(i) * B + b;
    const float nbi = nbeta[e];
    const float d = nbi - beta[e];
    v[e] = nbi + m * d;
    beta[e] = nbi;
    md = fmaxf(md, fabsf(d));
    mb = fmaxf(mb, fabsf(nbi));
  }
  if (part) {
    part[(static_cast<int64_t>(blockIdx.y) * 2) * B + b] = md;
    part[(static_cast<int64_t>(blockIdx.y) * 2 + 1) * B + b] = mb;
  }
}

}  // namespace

int lasso_slices(int p) { return (p + kRows - 1) / kRows; }

hipError_t launch_lasso_resid(const float* z, const float* v0, const float* y, const float* M,
                              const float* nb, float* r, float* rsum, int n, int B,
                              hipStream_t st) {
  if (n < 1 || B < 1) return hipErrorInvalidValue;
  lasso_resid_kernel<<<(B + kLB - 1) / kLB, kLB, 0, st>>>(z, v0, y, M, nb, r, rsum, n, B);
  return hipGetLastError();
}

hipError_t launch_lasso_step(float* v, float* beta, const float* g, const float* step,
                             const float* lam, float alpha, float* tk, const float* rsum,
                             float* v0, float* b0, float* nbeta, float* mom, float* part,
                             float* conv_part, int p, int B, hipStream_t st) {
  if (p < 1 || B < 1) return hipErrorInvalidValue;
  const dim3 grid((B + kLB - 1) / kLB, lasso_slices(p));
  lasso_prox_kernel<<<grid, kLB, 0, st>>>(v, beta, g, step, lam, alpha, nbeta, part, p, B);
  lasso_scal_kernel<<<(B + kLB - 1) / kLB, kLB, 0, st>>>(part, lasso_slices(p), tk, mom, step,
                                                         rsum, v0, b0, B);
  lasso_mom_kernel<<<grid, kLB, 0, st>>>(nbeta, beta, v, mom, conv_part, p, B);
  return hipGetLastError();
}

}  // namespace cml
