// PyTorch bindings of the consensus kernels (_C extension). Argument checking lives here so the
// kernels stay torch-free; every launch goes on the caller's current HIP stream and none of them
// synchronises, so the whole aggregation step can be captured in a hipGraph.
#include <torch/extension.h>
#include <array>
#include <climits>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>

#include "kernels/kernels.h"

namespace {

using at::Tensor;
using c10::optional;

#define CML_CHECK_HIP(expr)                                                               \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    TORCH_CHECK(_e == hipSuccess, "consensusml_amd HIP error: ", hipGetErrorString(_e), " at " \
                #expr " (bindings.cpp:", __LINE__, ")");                                  \
  } while (0)

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dtype_of(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return cml::DT_BF16;
  TORCH_CHECK(t.scalar_type() == at::kFloat, "expected bf16 or fp32 tensor, got ", t.scalar_type());
  return cml::DT_F32;
}

void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}

template <typename T = void>
T* opt_ptr(const optional<Tensor>& t, at::ScalarType st, const char* name, int64_t min_numel) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_dev(*t, name);
  TORCH_CHECK(t->scalar_type() == st, name, " has dtype ", t->scalar_type(), ", expected ", st);
  TORCH_CHECK(t->is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t->numel() >= min_numel, name, " too small: ", t->numel(), " < ", min_numel);
  return reinterpret_cast<T*>(t->data_ptr());
}

// X: [R, C] rows of workers (row stride arbitrary, unit column stride). The aggregation uses n
// rows (rows[i] indexes X when given) and the first D columns.
void agg_update(const Tensor& X, int64_t n, int64_t D, const optional<Tensor>& rows, int64_t combine,
                int64_t lo, int64_t cnt, const optional<Tensor>& w, int64_t opt,
                const optional<Tensor>& master, const optional<Tensor>& s1,
                const optional<Tensor>& s2, const optional<Tensor>& param_out,
                const optional<Tensor>& gout, double lr, double momentum, double weight_decay,
                double beta1, double beta2, double eps, double step_size, double inv_sqrt_bc2,
                double gscale, bool nesterov, bool first) {
  check_dev(X, "X");
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "X must be 2-D with unit column stride");
  TORCH_CHECK(n >= 1 && n <= 64, "1 <= n <= 64 workers supported, got ", n);
  // opt 3 = Adam with the L2 term added to the gradient (torch.optim.Adam semantics)
  const int adam_l2 = opt == 3 ? 1 : 0;
  if (adam_l2) opt = cml::OPT_ADAM;
  TORCH_CHECK(D >= 0 && D <= X.size(1), "D out of range");
  const c10::DeviceGuard guard(X.device());
  cml::SrcArgs s{};
  s.X = X.data_ptr();
  s.ld = X.stride(0);
  s.n = static_cast<int>(n);
  s.rows = opt_ptr<const int>(rows, at::kInt, "rows", n);
  if (!s.rows) TORCH_CHECK(X.size(0) >= n, "X has fewer rows than n");
  s.w = opt_ptr<const float>(w, at::kFloat, "w", n);
  s.lo = static_cast<int>(lo);
  s.cnt = static_cast<int>(cnt);
  cml::UpdArgs u{};
  u.master = opt_ptr<float>(master, at::kFloat, "master", D);
  u.s1 = opt_ptr<float>(s1, at::kFloat, "s1", D);
  u.s2 = opt_ptr<float>(s2, at::kFloat, "s2", D);
  const bool pf32 = param_out.has_value() && param_out->defined() &&
                    param_out->scalar_type() == at::kFloat;
  u.param_out = opt_ptr<void>(param_out, pf32 ? at::kFloat : at::kBFloat16, "param_out", D);
  u.param_f32 = pf32 ? 1 : 0;
  u.gout = opt_ptr<float>(gout, at::kFloat, "gout", D);
  if (opt != cml::OPT_NONE) TORCH_CHECK(u.master, "optimizer update needs master weights");
  if (opt == cml::OPT_SGD && momentum != 0.0) TORCH_CHECK(u.s1, "SGD momentum needs s1");
  if (opt == cml::OPT_ADAM) TORCH_CHECK(u.s1 && u.s2, "Adam needs s1 and s2");
  if (opt == cml::OPT_NONE) TORCH_CHECK(u.gout, "OPT_NONE needs gout");
  u.lr = static_cast<float>(lr);
  u.momentum = static_cast<float>(momentum);
  u.weight_decay = static_cast<float>(weight_decay);
  u.beta1 = static_cast<float>(beta1);
  u.beta2 = static_cast<float>(beta2);
  u.eps = static_cast<float>(eps);
  u.step_size = static_cast<float>(step_size);
  u.inv_sqrt_bc2 = static_cast<float>(inv_sqrt_bc2);
  u.gscale = static_cast<float>(gscale);
  u.nesterov = nesterov ? 1 : 0;
  u.first = first ? 1 : 0;
  u.adam_l2 = adam_l2;
  CML_CHECK_HIP(cml::launch_agg_update(dtype_of(X), static_cast<int>(combine), static_cast<int>(opt),
                                       s, u, D, cur_stream()));
}

// The same rule + optimizer over several segments (the sharded engine's buckets) in one launch:
// segment i = worker rows Xs[i] (first Ds[i] columns), state elements [offs[i], offs[i] + Ds[i])
// of master / s1 / s2 / gout, parameters pouts[i] (bf16 or fp32, >= Ds[i] elements).
void agg_update_multi(const std::vector<Tensor>& Xs, const std::vector<int64_t>& Ds,
                      const std::vector<int64_t>& offs, const std::vector<Tensor>& pouts, int64_t n,
                      const optional<Tensor>& rows, int64_t combine, int64_t lo, int64_t cnt,
                      const optional<Tensor>& w, int64_t opt, const optional<Tensor>& master,
                      const optional<Tensor>& s1, const optional<Tensor>& s2,
                      const optional<Tensor>& gout, double lr, double momentum,
                      double weight_decay, double beta1, double beta2, double eps,
                      double step_size, double inv_sqrt_bc2, double gscale, bool nesterov,
                      bool first) {
  const size_t ns = Xs.size();
  TORCH_CHECK(ns >= 1 && ns <= 16 && Ds.size() == ns && offs.size() == ns && pouts.size() == ns,
              "agg_update_multi: 1..16 segments with matching Xs / Ds / offs / pouts");
  TORCH_CHECK(n >= 1 && n <= 64, "1 <= n <= 64 workers supported, got ", n);
  const int adam_l2 = opt == 3 ? 1 : 0;
  if (adam_l2) opt = cml::OPT_ADAM;
  const at::ScalarType xt = Xs[0].scalar_type();
  const bool pf32 = pouts[0].scalar_type() == at::kFloat;
  int64_t need = 0;
  std::vector<cml::AggSeg> segs(ns);
  for (size_t i = 0; i < ns; ++i) {
    const Tensor& X = Xs[i];
    check_dev(X, "X");
    TORCH_CHECK(X.get_device() == Xs[0].get_device() && X.scalar_type() == xt,
                "agg_update_multi: Xs on one device with one dtype");
    TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "X must be 2-D with unit column stride");
    TORCH_CHECK(Ds[i] >= 0 && Ds[i] <= X.size(1) && offs[i] >= 0, "segment D / off out of range");
    if (!(rows.has_value() && rows->defined())) TORCH_CHECK(X.size(0) >= n, "X has fewer rows than n");
    const Tensor& P = pouts[i];
    check_dev(P, "param_out");
    TORCH_CHECK(P.is_contiguous() && P.numel() >= Ds[i] &&
                    P.scalar_type() == (pf32 ? at::kFloat : at::kBFloat16),
                "param_out: contiguous, >= D elements, one dtype");
    segs[i] = cml::AggSeg{X.data_ptr(), X.stride(0), Ds[i], offs[i], P.data_ptr()};
    need = std::max(need, offs[i] + Ds[i]);
  }
  const c10::DeviceGuard guard(Xs[0].device());
  cml::SrcArgs s{};
  s.n = static_cast<int>(n);
  s.rows = opt_ptr<const int>(rows, at::kInt, "rows", n);
  s.w = opt_ptr<const float>(w, at::kFloat, "w", n);
  s.lo = static_cast<int>(lo);
  s.cnt = static_cast<int>(cnt);
  cml::UpdArgs u{};
  u.master = opt_ptr<float>(master, at::kFloat, "master", need);
  u.s1 = opt_ptr<float>(s1, at::kFloat, "s1", need);
  u.s2 = opt_ptr<float>(s2, at::kFloat, "s2", need);
  u.gout = opt_ptr<float>(gout, at::kFloat, "gout", need);
  u.param_f32 = pf32 ? 1 : 0;
  if (opt != cml::OPT_NONE) TORCH_CHECK(u.master, "optimizer update needs master weights");
  if (opt == cml::OPT_SGD && momentum != 0.0) TORCH_CHECK(u.s1, "SGD momentum needs s1");
  if (opt == cml::OPT_ADAM) TORCH_CHECK(u.s1 && u.s2, "Adam needs s1 and s2");
  if (opt == cml::OPT_NONE) TORCH_CHECK(u.gout, "OPT_NONE needs gout");
  u.lr = static_cast<float>(lr);
  u.momentum = static_cast<float>(momentum);
  u.weight_decay = static_cast<float>(weight_decay);
  u.beta1 = static_cast<float>(beta1);
  u.beta2 = static_cast<float>(beta2);
  u.eps = static_cast<float>(eps);
  u.step_size = static_cast<float>(step_size);
  u.inv_sqrt_bc2 = static_cast<float>(inv_sqrt_bc2);
  u.gscale = static_cast<float>(gscale);
  u.nesterov = nesterov ? 1 : 0;
  u.first = first ? 1 : 0;
  u.adam_l2 = adam_l2;
  CML_CHECK_HIP(cml::launch_agg_update_multi(dtype_of(Xs[0]), static_cast<int>(combine),
                                             static_cast<int>(opt), s, u, segs.data(),
                                             static_cast<int>(ns), cur_stream()));
}

int64_t gram_workspace_bytes(int64_t n, int64_t D) {
  return static_cast<int64_t>(cml::gram_workspace_bytes(static_cast<int>(n), D));
}

void gram(const Tensor& X, int64_t n, int64_t D, const optional<Tensor>& rows, Tensor& work,
          Tensor& G, bool accumulate, const optional<Tensor>& center) {
  check_dev(X, "X");
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "X must be 2-D with unit column stride");
  TORCH_CHECK(n >= 1 && n <= 64, "1 <= n <= 64 workers supported");
  TORCH_CHECK(D >= 1 && D <= X.size(1), "D out of range");
  const int* r = opt_ptr<const int>(rows, at::kInt, "rows", n);
  if (!r) TORCH_CHECK(X.size(0) >= n, "X has fewer rows than n");
  TORCH_CHECK(work.is_cuda() && work.is_contiguous() &&
                  work.numel() * work.element_size() >= gram_workspace_bytes(n, D),
              "gram workspace too small");
  TORCH_CHECK(G.is_cuda() && G.scalar_type() == at::kDouble && G.is_contiguous() && G.numel() >= n * n,
              "G must be a contiguous fp64 [n, n] GPU tensor");
  const int* c = opt_ptr<const int>(center, at::kInt, "center", 1);
  const c10::DeviceGuard guard(X.device());
  CML_CHECK_HIP(cml::launch_gram(dtype_of(X), X.data_ptr(), X.stride(0), static_cast<int>(n), r, D,
                                 work.data_ptr(), G.data_ptr<double>(), accumulate ? 1 : 0,
                                 cur_stream(), c));
}

// stage 1 of gram() into `work` (a per-bucket workspace); returns the partial block count
int64_t gram_partial(const Tensor& X, int64_t n, int64_t D, Tensor& work,
                     const optional<Tensor>& center) {
  check_dev(X, "X");
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1 && X.size(0) >= n, "X: 2-D, unit column stride, >= n rows");
  TORCH_CHECK(n >= 1 && n <= 64 && D >= 1 && D <= X.size(1), "gram_partial: 1 <= n <= 64, D in range");
  TORCH_CHECK(work.is_cuda() && work.is_contiguous() &&
                  work.numel() * work.element_size() >= gram_workspace_bytes(n, D),
              "gram workspace too small");
  const int* c = opt_ptr<const int>(center, at::kInt, "center", 1);
  const c10::DeviceGuard guard(X.device());
  int nblk = 0;
  CML_CHECK_HIP(cml::launch_gram_partial(dtype_of(X), X.data_ptr(), X.stride(0), static_cast<int>(n),
                                         nullptr, D, work.data_ptr(), cur_stream(), c, &nblk));
  return nblk;
}

// G [n, n] fp64 = the buckets' partials (works[b], nblks[b] blocks) reduced, summed in order
void gram_reduce_multi(const std::vector<Tensor>& works, const std::vector<int64_t>& nblks,
                       int64_t n, Tensor& G) {
  TORCH_CHECK(!works.empty() && works.size() == nblks.size() && works.size() <= 32,
              "gram_reduce_multi: 1..32 buckets");
  TORCH_CHECK(G.is_cuda() && G.scalar_type() == at::kDouble && G.is_contiguous() && G.numel() >= n * n,
              "G must be a contiguous fp64 [n, n] GPU tensor");
  std::vector<const float*> parts;
  std::vector<int> nb;
  const int P = 16 * static_cast<int>((n + 15) / 16);
  for (size_t b = 0; b < works.size(); ++b) {
    TORCH_CHECK(works[b].is_cuda() && works[b].scalar_type() == at::kFloat && works[b].is_contiguous() &&
                    works[b].get_device() == G.get_device() &&
                    works[b].numel() >= nblks[b] * P * P && nblks[b] >= 1,
                "gram_reduce_multi: fp32 workspaces holding nblk x P x P partials");
    parts.push_back(works[b].data_ptr<float>());
    nb.push_back(static_cast<int>(nblks[b]));
  }
  const c10::DeviceGuard guard(G.device());
  CML_CHECK_HIP(cml::launch_gram_reduce_multi(parts.data(), nb.data(), static_cast<int>(parts.size()),
                                              static_cast<int>(n), G.data_ptr<double>(), cur_stream()));
}

// out (int32 [1]) = medoid of the finite rows of G (fp64 [n, n])
void gram_center(const Tensor& G, int64_t n, Tensor& out) {
  TORCH_CHECK(G.is_cuda() && G.scalar_type() == at::kDouble && G.is_contiguous() && G.numel() >= n * n,
              "G must be a contiguous fp64 [n, n] GPU tensor");
  TORCH_CHECK(n >= 1 && n <= 64, "1 <= n <= 64");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kInt && out.numel() >= 1, "out: int32 [1]");
  const c10::DeviceGuard guard(G.device());
  CML_CHECK_HIP(cml::launch_gram_center(G.data_ptr<double>(), static_cast<int>(n),
                                        out.data_ptr<int>(), cur_stream()));
}

void robust_weights(const Tensor& G, int64_t rule, int64_t n, int64_t f, int64_t m, int64_t iters,
                    double eps, double tol, double tau, Tensor& w, const optional<Tensor>& scores,
                    const optional<Tensor>& sel, bool guard, const optional<Tensor>& center_out,
                    const optional<Tensor>& sel_counts) {
  TORCH_CHECK(G.is_cuda() && G.scalar_type() == at::kDouble && G.is_contiguous(), "G: fp64 GPU");
  const int64_t dim = rule == cml::RULE_CCLIP ? n + 1 : n;
  TORCH_CHECK(G.numel() >= dim * dim, "G too small");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.numel() >= dim, "w: fp32 GPU [n(+1)]");
  const c10::DeviceGuard guard_(G.device());
  double* sc = opt_ptr<double>(scores, at::kDouble, "scores", n);
  int* se = opt_ptr<int>(sel, at::kInt, "sel", n + 1);
  int* co = opt_ptr<int>(center_out, at::kInt, "center_out", 1);
  // a 2-element center buffer carries the guard's non-finite-row count of the previous pass
  int* nb = (co && center_out->numel() >= 2) ? co + 1 : nullptr;
  double* cnt = opt_ptr<double>(sel_counts, at::kDouble, "sel_counts", n);
  CML_CHECK_HIP(cml::launch_robust_weights(static_cast<int>(rule), G.data_ptr<double>(),
                                           static_cast<int>(n), static_cast<int>(f),
                                           static_cast<int>(m), static_cast<int>(iters), eps, tol,
                                           tau, w.data_ptr<float>(), sc, se, cur_stream(),
                                           guard ? 1 : 0, co, cnt, nb));
}

// G = sum over b of Gb[b] (fp64 [nb, r, r] -> [r, r]) in bucket order
void gram_sum(const Tensor& Gb, Tensor& G) {
  TORCH_CHECK(Gb.is_cuda() && Gb.scalar_type() == at::kDouble && Gb.is_contiguous() && Gb.dim() == 3,
              "Gb: contiguous fp64 [nb, r, r] GPU tensor");
  TORCH_CHECK(G.is_cuda() && G.scalar_type() == at::kDouble && G.is_contiguous() &&
                  G.numel() == Gb.size(1) * Gb.size(2) && G.get_device() == Gb.get_device(),
              "G: contiguous fp64 [r, r] on Gb's device");
  const c10::DeviceGuard guard(G.device());
  CML_CHECK_HIP(cml::launch_gram_sum(Gb.data_ptr<double>(), static_cast<int>(Gb.size(0)),
                                     G.numel(), G.data_ptr<double>(), cur_stream()));
}

int64_t gossip_workspace_bytes(int64_t D) {
  return static_cast<int64_t>(cml::gossip_workspace_bytes(D));
}

void gossip_mix(Tensor& master, const optional<Tensor>& param_out, const Tensor& left,
                const Tensor& right, double w0, double w1, double w2, double clip, Tensor& work) {
  check_dev(master, "master");
  TORCH_CHECK(master.scalar_type() == at::kFloat && master.is_contiguous(), "master: fp32 contiguous");
  const int64_t D = master.numel();
  TORCH_CHECK(left.scalar_type() == right.scalar_type() && left.is_contiguous() &&
                  right.is_contiguous() && left.numel() >= D && right.numel() >= D,
              "neighbours: contiguous, same dtype, master's size");
  TORCH_CHECK(work.numel() * work.element_size() >= gossip_workspace_bytes(D), "gossip workspace too small");
  void* p = opt_ptr<void>(param_out, left.scalar_type(), "param_out", D);
  const c10::DeviceGuard guard(master.device());
  CML_CHECK_HIP(cml::launch_gossip_mix(dtype_of(left), master.data_ptr<float>(), p, left.data_ptr(), right.data_ptr(),
                                       D, static_cast<float>(w0), static_cast<float>(w1),
                                       static_cast<float>(w2), static_cast<float>(clip),
                                       work.data_ptr(), cur_stream()));
}

void gossip_mix_k(Tensor& master, const optional<Tensor>& param_out, std::vector<Tensor> nbrs,
                  std::vector<double> w, double w0, double clip, Tensor& work,
                  const optional<Tensor>& param_out2) {
  check_dev(master, "master");
  TORCH_CHECK(master.scalar_type() == at::kFloat && master.is_contiguous(), "master: fp32 contiguous");
  const int64_t D = master.numel();
  const int k = static_cast<int>(nbrs.size());
  TORCH_CHECK(k >= 1 && k <= 8 && w.size() == nbrs.size(), "1..8 neighbours, one weight each");
  std::vector<const void*> ptr(k);
  std::vector<float> wf(k);
  for (int i = 0; i < k; ++i) {
    TORCH_CHECK(nbrs[i].scalar_type() == nbrs[0].scalar_type() && nbrs[i].is_contiguous() &&
                    nbrs[i].numel() >= D && nbrs[i].device() == master.device(),
                "neighbours: contiguous, same dtype and device, master's size");
    ptr[i] = nbrs[i].data_ptr();
    wf[i] = static_cast<float>(w[i]);
  }
  TORCH_CHECK(work.numel() * work.element_size() >= gossip_workspace_bytes(D), "gossip workspace too small");
  void* p = opt_ptr<void>(param_out, nbrs[0].scalar_type(), "param_out", D);
  void* p2 = opt_ptr<void>(param_out2, nbrs[0].scalar_type(), "param_out2", D);
  const c10::DeviceGuard guard(master.device());
  CML_CHECK_HIP(cml::launch_gossip_mix_k(dtype_of(nbrs[0]), master.data_ptr<float>(), p, ptr.data(),
                                         wf.data(), k, D, static_cast<float>(w0),
                                         static_cast<float>(clip), work.data_ptr(), cur_stream(), p2));
}

// x / res / y: NHWC-contiguous bf16 (4-D channels_last or 2-D [M, C]).
void check_nhwc(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  if (t.dim() == 4) {
    TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels_last");
  } else {
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  }
}

std::vector<Tensor> bn_fwd(const Tensor& x, const optional<Tensor>& res, const Tensor& gamma,
                           const Tensor& beta, const optional<Tensor>& rmean,
                           const optional<Tensor>& rvar, const optional<Tensor>& mean_in,
                           const optional<Tensor>& invstd_in, double eps, double momentum,
                           bool relu, bool training, bool want_mask) {
  check_nhwc(x, "x");
  const int64_t C = x.size(1) * (x.dim() == 4 ? 1 : 0) + (x.dim() == 2 ? x.size(1) : 0);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn: C must be 8 * (power of 2) <= 2048");
  if (res.has_value() && res->defined()) {
    check_nhwc(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "res shape mismatch");
  }
  TORCH_CHECK(gamma.scalar_type() == at::kBFloat16 && beta.scalar_type() == at::kBFloat16 &&
                  gamma.is_contiguous() && beta.is_contiguous() && gamma.numel() == C,
              "gamma/beta: contiguous bf16 [C]");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor y = at::empty_like(x);
  Tensor mean, invstd;
  if (training) {
    mean = at::empty({C}, f32);
    invstd = at::empty({C}, f32);
  } else {
    TORCH_CHECK(mean_in.has_value() && invstd_in.has_value(), "eval bn needs mean / invstd");
    mean = mean_in->contiguous();
    invstd = invstd_in->contiguous();
  }
  float* rm = opt_ptr<float>(rmean, at::kFloat, "running_mean", C);
  float* rv = opt_ptr<float>(rvar, at::kFloat, "running_var", C);
  Tensor work = at::empty({static_cast<int64_t>(cml::bn_workspace_bytes(M, static_cast<int>(C)) / 4 + 1)}, f32);
  const void* rp = (res.has_value() && res->defined()) ? res->data_ptr() : nullptr;
  Tensor mask;
  if (want_mask && rp && relu) mask = at::empty({M, C / 8}, x.options().dtype(at::kByte));
  CML_CHECK_HIP(cml::launch_bn_fwd(x.data_ptr(), rp, y.data_ptr(),
                                   mask.defined() ? mask.data_ptr() : nullptr, M,
                                   static_cast<int>(C), gamma.data_ptr(), beta.data_ptr(),
                                   mean.data_ptr<float>(), invstd.data_ptr<float>(), rm, rv,
                                   static_cast<float>(eps), static_cast<float>(momentum),
                                   relu ? 1 : 0, training ? 1 : 0, work.data_ptr(), cur_stream()));
  return {y, mean, invstd, mask};
}

// dy2 (optional): second part of the output gradient, summed on load. mask (optional): the
// forward's ReLU bit mask (required for relu with a residual). want_dres: also return the
// residual gradient.
// Reduction half of a training BN (+ ReLU) backward: {sdz, sdzx} fp32 [C] (sum dy', sum dy' xhat)
// for consumers that fold the apply into their own prologue (conv1x1_bnbwd, wgrad1x1 dz_*).
std::vector<Tensor> bn_bwd_sums(const Tensor& dy_in, const optional<Tensor>& dy2_in,
                                const Tensor& x, const optional<Tensor>& mask, const Tensor& gamma,
                                const Tensor& beta, const Tensor& mean, const Tensor& invstd,
                                bool relu) {
  check_nhwc(x, "x");
  Tensor dy = x.dim() == 4 ? dy_in.contiguous(at::MemoryFormat::ChannelsLast) : dy_in.contiguous();
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy shape mismatch");
  Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = x.dim() == 4 ? dy2_in->contiguous(at::MemoryFormat::ChannelsLast) : dy2_in->contiguous();
    check_nhwc(dy2, "dy2");
    TORCH_CHECK(dy2.sizes() == x.sizes(), "dy2 shape mismatch");
  }
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  const uint8_t* mp = opt_ptr<const uint8_t>(mask, at::kByte, "mask", M * (C / 8));
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor dgamma = at::empty({C}, gamma.options()), dbeta = at::empty({C}, beta.options());
  Tensor sdz = at::empty({C}, f32), sdzx = at::empty({C}, f32);
  Tensor work = at::empty({static_cast<int64_t>(cml::bn_workspace_bytes(M, static_cast<int>(C)) / 4 + 1)}, f32);
  CML_CHECK_HIP(cml::launch_bn_bwd(dy.data_ptr(), dy2.defined() ? dy2.data_ptr() : nullptr,
                                   x.data_ptr(), mp, nullptr, nullptr, M, static_cast<int>(C),
                                   gamma.data_ptr(), beta.data_ptr(), mean.data_ptr<float>(),
                                   invstd.data_ptr<float>(), dgamma.data_ptr(), dbeta.data_ptr(),
                                   sdz.data_ptr<float>(), sdzx.data_ptr<float>(), relu ? 1 : 0,
                                   work.data_ptr(), cur_stream()));
  return {sdz, sdzx};
}

std::vector<Tensor> bn_bwd(const Tensor& dy_in, const optional<Tensor>& dy2_in, const Tensor& x,
                           const optional<Tensor>& mask, const Tensor& gamma, const Tensor& beta,
                           const Tensor& mean, const Tensor& invstd, bool relu, bool want_dres) {
  check_nhwc(x, "x");
  auto as_nhwc = [&](const Tensor& t) {
    return x.dim() == 4 ? t.contiguous(at::MemoryFormat::ChannelsLast) : t.contiguous();
  };
  Tensor dy = as_nhwc(dy_in);
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy shape mismatch");
  Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = as_nhwc(*dy2_in);
    check_nhwc(dy2, "dy2");
    TORCH_CHECK(dy2.sizes() == x.sizes(), "dy2 shape mismatch");
  }
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  const bool has_mask = mask.has_value() && mask->defined();
  if (has_mask) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() == M * (C / 8) && mask->device() == x.device(),
                "mask: contiguous uint8 [M, C/8] on x's device");
  }
  TORCH_CHECK(!(relu && want_dres && !has_mask), "bn_bwd: relu + residual needs the forward mask");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor dx = at::empty_like(x);
  Tensor dres = want_dres ? at::empty_like(x) : Tensor();
  Tensor dgamma = at::empty({C}, gamma.options());
  Tensor dbeta = at::empty({C}, beta.options());
  Tensor sdz = at::empty({C}, f32), sdzx = at::empty({C}, f32);
  Tensor work = at::empty({static_cast<int64_t>(cml::bn_workspace_bytes(M, static_cast<int>(C)) / 4 + 1)}, f32);
  CML_CHECK_HIP(cml::launch_bn_bwd(dy.data_ptr(), dy2.defined() ? dy2.data_ptr() : nullptr,
                                   x.data_ptr(), has_mask ? mask->data_ptr() : nullptr,
                                   dx.data_ptr(), want_dres ? dres.data_ptr() : nullptr, M,
                                   static_cast<int>(C), gamma.data_ptr(), beta.data_ptr(),
                                   mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                   dgamma.data_ptr(), dbeta.data_ptr(), sdz.data_ptr<float>(),
                                   sdzx.data_ptr<float>(), relu ? 1 : 0, work.data_ptr(),
                                   cur_stream()));
  return {dx, dgamma, dbeta, dres};
}

// y = relu(bn1(x1) + bn2(x2)); returns (y, mean1, invstd1, mean2, invstd2, mask)
std::vector<Tensor> bn_fwd2(const Tensor& x1, const Tensor& x2, const Tensor& g1, const Tensor& b1,
                            const Tensor& g2, const Tensor& b2, const optional<Tensor>& rm1,
                            const optional<Tensor>& rv1, const optional<Tensor>& rm2,
                            const optional<Tensor>& rv2, const optional<Tensor>& mean1_in,
                            const optional<Tensor>& invstd1_in, const optional<Tensor>& mean2_in,
                            const optional<Tensor>& invstd2_in, double eps, double momentum,
                            bool training, bool want_mask) {
  check_nhwc(x1, "x1");
  check_nhwc(x2, "x2");
  TORCH_CHECK(x1.sizes() == x2.sizes() && x1.dim() == 4, "bn_fwd2: x1 / x2 same 4-D shape");
  const int64_t C = x1.size(1);
  const int64_t M = x1.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn: C must be 8 * (power of 2) <= 2048");
  for (const Tensor* t : {&g1, &b1, &g2, &b2})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->numel() == C,
                "gamma/beta: contiguous bf16 [C]");
  const c10::DeviceGuard guard(x1.device());
  auto f32 = x1.options().dtype(at::kFloat);
  Tensor y = at::empty_like(x1);
  Tensor m1, i1, m2, i2;
  if (training) {
    m1 = at::empty({C}, f32); i1 = at::empty({C}, f32); m2 = at::empty({C}, f32); i2 = at::empty({C}, f32);
  } else {
    TORCH_CHECK(mean1_in.has_value() && invstd1_in.has_value() && mean2_in.has_value() &&
                    invstd2_in.has_value(), "eval bn_fwd2 needs both means / invstds");
    m1 = mean1_in->contiguous(); i1 = invstd1_in->contiguous();
    m2 = mean2_in->contiguous(); i2 = invstd2_in->contiguous();
  }
  Tensor mask = want_mask ? at::empty({M, C / 8}, x1.options().dtype(at::kByte)) : Tensor();
  Tensor work = at::empty({static_cast<int64_t>(cml::bn_workspace_bytes(M, static_cast<int>(C)) / 4 + 1)}, f32);
  CML_CHECK_HIP(cml::launch_bn_fwd2(
      x1.data_ptr(), x2.data_ptr(), y.data_ptr(), want_mask ? mask.data_ptr() : nullptr, M,
      static_cast<int>(C), g1.data_ptr(), b1.data_ptr(), g2.data_ptr(), b2.data_ptr(),
      m1.data_ptr<float>(), i1.data_ptr<float>(), m2.data_ptr<float>(), i2.data_ptr<float>(),
      opt_ptr<float>(rm1, at::kFloat, "running_mean1", C), opt_ptr<float>(rv1, at::kFloat, "running_var1", C),
      opt_ptr<float>(rm2, at::kFloat, "running_mean2", C), opt_ptr<float>(rv2, at::kFloat, "running_var2", C),
      static_cast<float>(eps), static_cast<float>(momentum), training ? 1 : 0, work.data_ptr(),
      cur_stream()));
  return {y, m1, i1, m2, i2, mask};
}

// returns (dx1, dgamma1, dbeta1, dx2, dgamma2, dbeta2)
std::vector<Tensor> bn_bwd2(const Tensor& dy_in, const optional<Tensor>& dy2_in, const Tensor& x1,
                            const Tensor& x2, const Tensor& mask, const Tensor& g1,
                            const Tensor& g2, const Tensor& mean1, const Tensor& invstd1,
                            const Tensor& mean2, const Tensor& invstd2) {
  check_nhwc(x1, "x1");
  check_nhwc(x2, "x2");
  Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.sizes() == x1.sizes() && x2.sizes() == x1.sizes(), "bn_bwd2 shape mismatch");
  Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = dy2_in->contiguous(at::MemoryFormat::ChannelsLast);
    check_nhwc(dy2, "dy2");
    TORCH_CHECK(dy2.sizes() == x1.sizes(), "dy2 shape mismatch");
  }
  const int64_t C = x1.size(1);
  const int64_t M = x1.numel() / C;
  TORCH_CHECK(mask.scalar_type() == at::kByte && mask.is_contiguous() && mask.numel() == M * (C / 8),
              "mask: contiguous uint8 [M, C/8]");
  const c10::DeviceGuard guard(x1.device());
  auto f32 = x1.options().dtype(at::kFloat);
  Tensor dx1 = at::empty_like(x1), dx2 = at::empty_like(x2);
  Tensor dg1 = at::empty({C}, g1.options()), db1 = at::empty({C}, g1.options());
  Tensor dg2 = at::empty({C}, g2.options()), db2 = at::empty({C}, g2.options());
  Tensor sums = at::empty({4, C}, f32);
  Tensor work = at::empty({static_cast<int64_t>(cml::bn2_workspace_bytes(M, static_cast<int>(C)) / 4 + 1)}, f32);
  CML_CHECK_HIP(cml::launch_bn_bwd2(
      dy.data_ptr(), dy2.defined() ? dy2.data_ptr() : nullptr, x1.data_ptr(), x2.data_ptr(),
      mask.data_ptr(), dx1.data_ptr(), dx2.data_ptr(), M, static_cast<int>(C), g1.data_ptr(),
      g2.data_ptr(), mean1.data_ptr<float>(), invstd1.data_ptr<float>(), mean2.data_ptr<float>(),
      invstd2.data_ptr<float>(), dg1.data_ptr(), db1.data_ptr(), dg2.data_ptr(), db2.data_ptr(),
      sums.data_ptr<float>(), sums.data_ptr<float>() + C, sums.data_ptr<float>() + 2 * C,
      sums.data_ptr<float>() + 3 * C, work.data_ptr(), cur_stream()));
  return {dx1, dg1, db1, dx2, dg2, db2};
}

std::vector<Tensor> maxpool_fwd(const Tensor& x, int64_t k, int64_t s, int64_t p) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(1) % 8 == 0, "maxpool: 4-D NHWC with C % 8 == 0");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  const c10::DeviceGuard guard(x.device());
  Tensor y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor idx = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  CML_CHECK_HIP(cml::launch_maxpool_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C,
                                        OH, OW, k, s, p, cur_stream()));
  return {y, idx};
}

// maxpool(relu(bn(x))): returns (y_pool, idx, mean, invstd); training -> batch stats (running
// stats updated), else mean_in / invstd_in
std::vector<Tensor> bn_relu_maxpool_fwd(const Tensor& x, const Tensor& gamma, const Tensor& beta,
                                        const optional<Tensor>& rmean, const optional<Tensor>& rvar,
                                        const optional<Tensor>& mean_in,
                                        const optional<Tensor>& invstd_in, double eps,
                                        double momentum, bool training, int64_t k, int64_t s,
                                        int64_t p) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "bn_relu_maxpool: 4-D NHWC input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn: C must be 8 * (power of 2) <= 2048");
  TORCH_CHECK(gamma.scalar_type() == at::kBFloat16 && beta.scalar_type() == at::kBFloat16 &&
                  gamma.is_contiguous() && beta.is_contiguous() && gamma.numel() == C, "gamma/beta");
  const int64_t OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor mean, invstd;
  if (training) {
    mean = at::empty({C}, f32);
    invstd = at::empty({C}, f32);
    Tensor work = at::empty({static_cast<int64_t>(cml::bn_workspace_bytes(N * H * W, static_cast<int>(C)) / 4 + 1)}, f32);
    CML_CHECK_HIP(cml::launch_bn_stats(x.data_ptr(), N * H * W, static_cast<int>(C),
                                       mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                       opt_ptr<float>(rmean, at::kFloat, "running_mean", C),
                                       opt_ptr<float>(rvar, at::kFloat, "running_var", C),
                                       static_cast<float>(eps), static_cast<float>(momentum),
                                       work.data_ptr(), cur_stream()));
  } else {
    TORCH_CHECK(mean_in.has_value() && invstd_in.has_value(), "eval needs mean / invstd");
    mean = mean_in->contiguous();
    invstd = invstd_in->contiguous();
  }
  Tensor y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor idx = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  CML_CHECK_HIP(cml::launch_bn_relu_maxpool_fwd(x.data_ptr(), mean.data_ptr<float>(),
                                                invstd.data_ptr<float>(), gamma.data_ptr(),
                                                beta.data_ptr(), y.data_ptr(), idx.data_ptr(), N,
                                                H, W, C, OH, OW, k, s, p, cur_stream()));
  return {y, idx, mean, invstd};
}

// ResNet stem conv (7x7/s2/p3, C_in 3 or 4 -> 64) with the BatchNorm statistics in its epilogue.
// x: NHWC bf16 [N, C, H, W] channels_last; wpk: packed bf16 [64, 224]. Returns {z, mean, invstd}
// (mean / invstd undefined when !training).
std::vector<Tensor> stem_conv_fwd(const Tensor& x, const Tensor& wpk, const optional<Tensor>& rmean,
                                  const optional<Tensor>& rvar, double eps, double momentum,
                                  bool training) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "stem_conv: 4-D input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C == 3 || C == 4, "stem_conv: 3 or 4 input channels");
  TORCH_CHECK(wpk.scalar_type() == at::kBFloat16 && wpk.is_contiguous() && wpk.numel() == 64 * 224 &&
                  wpk.device() == x.device(), "stem_conv: packed bf16 weights [64, 224]");
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  const int grid = cml::stem_fwd_grid(N, OH, OW, C);
  Tensor part = at::empty({grid, 2, 64}, f32);
  Tensor z = at::empty({N, 64, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor mean, invstd;
  if (training) {
    mean = at::empty({64}, f32);
    invstd = at::empty({64}, f32);
  }
  CML_CHECK_HIP(cml::launch_stem_conv_fwd(
      x.data_ptr(), wpk.data_ptr(), z.data_ptr(), part.data_ptr<float>(), grid,
      training ? mean.data_ptr<float>() : nullptr, training ? invstd.data_ptr<float>() : nullptr,
      training ? opt_ptr<float>(rmean, at::kFloat, "running_mean", 64) : nullptr,
      training ? opt_ptr<float>(rvar, at::kFloat, "running_var", 64) : nullptr,
      static_cast<float>(eps), static_cast<float>(momentum), N, H, W, C, OH, OW, cur_stream()));
  return {z, mean, invstd};
}

// Stem backward through BN: g = ReLU-masked pool gradient (NHWC [N, 64, OH, OW]) with its channel
// sums gsum (maxpool_bwd_sum), z = conv output, x = conv input.
// Returns {dw [64, C, 7, 7] fp32, dgamma fp32 [64], dbeta fp32 [64]}.
std::vector<Tensor> stem_wgrad(const Tensor& g_in, const Tensor& z, const Tensor& x,
                               const Tensor& mean, const Tensor& invstd, const Tensor& gamma,
                               const Tensor& gsum) {
  check_nhwc(x, "x");
  check_nhwc(z, "z");
  Tensor g = g_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(g, "g");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(C == 3 || C == 4, "stem_wgrad: 3 or 4 input channels");
  TORCH_CHECK(z.size(0) == N && z.size(1) == 64 && z.size(2) == OH && z.size(3) == OW &&
                  g.sizes() == z.sizes(), "stem_wgrad: g / z shape");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && invstd.scalar_type() == at::kFloat &&
                  mean.numel() == 64 && invstd.numel() == 64 && mean.is_contiguous() &&
                  invstd.is_contiguous(), "stem_wgrad: fp32 mean / invstd [64]");
  TORCH_CHECK(gamma.scalar_type() == at::kBFloat16 && gamma.is_contiguous() && gamma.numel() == 64,
              "stem_wgrad: bf16 gamma [64]");
  TORCH_CHECK(gsum.scalar_type() == at::kFloat && gsum.is_contiguous() && gsum.numel() == 64 &&
                  gsum.device() == x.device(), "stem_wgrad: fp32 channel sums of g [64]");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  const int grid = cml::stem_bwd_grid(N, OH, OW, C);
  const int64_t pw = static_cast<int64_t>(cml::stem_wgrad_part_floats());
  Tensor part = at::empty({grid, pw}, f32);
  Tensor tot = at::empty({static_cast<int64_t>(cml::stem_wgrad_tot_doubles())},
                         x.options().dtype(at::kDouble));
  Tensor dw = at::empty({64, C, 7, 7}, f32);
  Tensor dg = at::empty({64}, f32), db = at::empty({64}, f32);
  Tensor cwork = at::empty({static_cast<int64_t>(cml::stem_cola_work_floats(N, H, W, C))}, f32);
  CML_CHECK_HIP(cml::launch_stem_wgrad(g.data_ptr(), z.data_ptr(), x.data_ptr(),
                                       mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                       gamma.data_ptr(), gsum.data_ptr<float>(),
                                       part.data_ptr<float>(), grid,
                                       tot.data_ptr<double>(), dw.data_ptr<float>(),
                                       dg.data_ptr<float>(), db.data_ptr<float>(), N, H, W, C, OH,
                                       OW, cur_stream(), nullptr, cwork.data_ptr<float>()));
  return {dw, dg, db};
}

// Stem backward straight from the max-pool's OUTPUT gradient dy [N, 64, PH, PW] (+ an optional
// second gradient dy2 of the same shape, summed into one pooled gradient first) and the pool's
// argmax bytes idx: stem_wgrad gathering each pixel's pool input gradient from its windows (the
// full-resolution pool gradient is never written), its mean handled through the column sums of
// the input patches. Same outputs as stem_wgrad.
std::vector<Tensor> stem_wgrad_pool(const Tensor& dy_in, const Tensor& idx,
                                    const optional<Tensor>& dy2_in, const Tensor& z,
                                    const Tensor& x, const Tensor& mean, const Tensor& invstd,
                                    const Tensor& gamma, bool bf16_out) {
  check_nhwc(x, "x");
  check_nhwc(z, "z");
  Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dy, "dy");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const int64_t PH = (OH - 1) / 2 + 1, PW = (OW - 1) / 2 + 1;
  TORCH_CHECK(C == 3 || C == 4, "stem_wgrad_pool: 3 or 4 input channels");
  TORCH_CHECK(z.size(0) == N && z.size(1) == 64 && z.size(2) == OH && z.size(3) == OW,
              "stem_wgrad_pool: z shape");
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == 64 && dy.size(2) == PH && dy.size(3) == PW,
              "stem_wgrad_pool: dy must be the 3x3 / s2 / p1 pool output gradient of z");
  // idx: the pool forward's argmax bytes, [N, PH, PW, 64] contiguous (bn_relu_maxpool_fwd)
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.numel() == dy.numel() && idx.is_contiguous() &&
                  idx.device() == dy.device(),
              "stem_wgrad_pool: idx");
  Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = dy2_in->contiguous(at::MemoryFormat::ChannelsLast);
    check_nhwc(dy2, "dy2");
    TORCH_CHECK(dy2.sizes() == dy.sizes() && dy2.device() == dy.device(), "stem_wgrad_pool: dy2");
  }
  TORCH_CHECK(mean.scalar_type() == at::kFloat && invstd.scalar_type() == at::kFloat &&
                  mean.numel() == 64 && invstd.numel() == 64 && mean.is_contiguous() &&
                  invstd.is_contiguous(), "stem_wgrad_pool: fp32 mean / invstd [64]");
  TORCH_CHECK(gamma.scalar_type() == at::kBFloat16 && gamma.is_contiguous() && gamma.numel() == 64,
              "stem_wgrad_pool: bf16 gamma [64]");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  const int64_t P = N * PH * PW;
  Tensor dsum;
  if (dy2.defined()) {   // one pooled gradient for the gather: dsum = bf16(dy + dy2)
    dsum = at::empty_like(dy);
    Tensor gs = at::empty({64}, f32);
    Tensor work = at::empty({static_cast<int64_t>(cml::pool_gsum_workspace_floats(P, 64))}, f32);
    CML_CHECK_HIP(cml::launch_pool_gsum(dy.data_ptr(), dy2.data_ptr(), idx.data_ptr(),
                                        dsum.data_ptr(), gs.data_ptr<float>(),
                                        work.data_ptr<float>(), P, 64, cur_stream()));
  }
  const Tensor& pg = dsum.defined() ? dsum : dy;
  Tensor cwork = at::empty({static_cast<int64_t>(cml::stem_cola_work_floats(N, H, W, C))}, f32);
  const int grid = cml::stem_bwd_grid(N, OH, OW, C);
  const int64_t pw = static_cast<int64_t>(cml::stem_wgrad_part_floats());
  Tensor part = at::empty({grid, pw}, f32);
  Tensor tot = at::empty({static_cast<int64_t>(cml::stem_wgrad_tot_doubles())},
                         x.options().dtype(at::kDouble));
  // bf16_out: the outputs in the (bf16) parameters' dtype from the final kernel itself
  auto odt = bf16_out ? x.options().dtype(at::kBFloat16) : f32;
  Tensor dw = at::empty({64, C, 7, 7}, odt);
  Tensor dg = at::empty({64}, odt), db = at::empty({64}, odt);
  CML_CHECK_HIP(cml::launch_stem_wgrad(pg.data_ptr(), z.data_ptr(), x.data_ptr(),
                                       mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                       gamma.data_ptr(), nullptr, part.data_ptr<float>(), grid,
                                       tot.data_ptr<double>(), dw.data_ptr(), dg.data_ptr(),
                                       db.data_ptr(), N, H, W, C, OH, OW, cur_stream(),
                                       idx.data_ptr<uint8_t>(), cwork.data_ptr<float>(),
                                       bf16_out));
  return {dw, dg, db};
}

Tensor maxpool_bwd(const Tensor& dy_in, const Tensor& idx, int64_t H, int64_t W, int64_t k,
                   int64_t s, int64_t p) {
  Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dy, "dy");
  const int64_t N = dy.size(0), C = dy.size(1), OH = dy.size(2), OW = dy.size(3);
  const c10::DeviceGuard guard(dy.device());
  Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  CML_CHECK_HIP(cml::launch_maxpool_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), N, H, W, C,
                                        OH, OW, k, s, p, cur_stream()));
  return dx;
}

// dW of a stride-1 1x1 conv: dy [N, Co, H, W], x [N, Ci, H, W] NHWC bf16 -> dW [Co, Ci, 1, 1]
// in `dtype` (bf16 or fp32).
Tensor wgrad1x1(const Tensor& dy_in, const Tensor& x, at::ScalarType dtype,
                const optional<Tensor>& pro_sc, const optional<Tensor>& pro_bi,
                const optional<Tensor>& dz_z, const optional<Tensor>& dz_mask,
                const optional<Tensor>& dz_a, const optional<Tensor>& dz_b,
                const optional<Tensor>& dz_c, const optional<Tensor>& out) {
  check_nhwc(x, "x");
  Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dy, "dy");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && dy.size(0) == x.size(0) && dy.size(2) == x.size(2) &&
                  dy.size(3) == x.size(3), "wgrad1x1: dy / x shapes");
  TORCH_CHECK(dtype == at::kBFloat16 || dtype == at::kFloat, "wgrad1x1: bf16 or fp32 output");
  const int64_t Co = dy.size(1), Ci = x.size(1);
  const int64_t P = x.numel() / Ci;
  TORCH_CHECK(Ci == 64 ? Co % 256 == 0 : (Co % 128 == 0 && Ci % 128 == 0),
              "wgrad1x1: channels must be multiples of 128 (or Ci 64 with Co % 256 == 0)");
  const float* sc = opt_ptr<const float>(pro_sc, at::kFloat, "pro_sc", Ci);
  const float* bi = opt_ptr<const float>(pro_bi, at::kFloat, "pro_bi", Ci);
  TORCH_CHECK((sc == nullptr) == (bi == nullptr), "wgrad1x1: pro_sc and pro_bi together");
  const void* zp = nullptr;
  if (dz_z.has_value() && dz_z->defined()) {
    check_nhwc(*dz_z, "dz_z");
    TORCH_CHECK(dz_z->sizes() == dy.sizes(), "wgrad1x1: dz_z must have dy's shape");
    zp = dz_z->data_ptr();
  }
  const uint8_t* zm = opt_ptr<const uint8_t>(dz_mask, at::kByte, "dz_mask", P * Co / 8);
  const float* za = opt_ptr<const float>(dz_a, at::kFloat, "dz_a", Co);
  const float* zb = opt_ptr<const float>(dz_b, at::kFloat, "dz_b", Co);
  const float* zc = opt_ptr<const float>(dz_c, at::kFloat, "dz_c", Co);
  TORCH_CHECK((zp == nullptr) == (zm == nullptr) && (zp == nullptr) == (za == nullptr) &&
                  (zp == nullptr) == (zb == nullptr) && (zp == nullptr) == (zc == nullptr),
              "wgrad1x1: dz_z, dz_mask, dz_a, dz_b, dz_c together");
  const c10::DeviceGuard guard(x.device());
  int S = 1, cps = 1;
  cml::wgrad1x1_plan(P, static_cast<int>(Co), static_cast<int>(Ci), &S, &cps, sc != nullptr,
                     zp != nullptr ? 1 : 0, false);
  // one-split long-K calls (transformer linears): the kernel writes dw itself, no partial slab
  const bool direct = cml::wgrad1x1_direct(P, static_cast<int>(Co), static_cast<int>(Ci),
                                           sc != nullptr, zp != nullptr ? 1 : 0, false);
  Tensor part = direct ? Tensor() : at::empty({S, Co, Ci}, x.options().dtype(at::kFloat));
  Tensor dw;
  if (out.has_value() && out->defined()) {   // caller's destination (e.g. a flat gradient row)
    check_dev(*out, "out");
    TORCH_CHECK(out->scalar_type() == dtype && out->is_contiguous() && out->numel() == Co * Ci &&
                    reinterpret_cast<uintptr_t>(out->data_ptr()) % 16 == 0,
                "wgrad1x1: out must be a contiguous 16-B aligned [Co, Ci] tensor of dtype");
    dw = *out;
  } else {
    dw = at::empty({Co, Ci, 1, 1}, x.options().dtype(dtype));
  }
  CML_CHECK_HIP(cml::launch_wgrad1x1(dy.data_ptr(), x.data_ptr(),
                                     direct ? nullptr : part.data_ptr<float>(),
                                     dw.data_ptr(), dtype == at::kBFloat16, P,
                                     static_cast<int>(Co), static_cast<int>(Ci), sc, bi,
                                     cur_stream(), zp, zm, za, zb, zc));
  return dw;
}

// wgrad1x1 with a general dy prologue (dmode: 0 none, 2 dz_a (mask ? dy : 0) + dz_c,
// 3 max(dy dz_a + dz_b, 0)) and optional column sums of the staged dz -> {dw fp32 [Co, Ci], cs [Co]}.
// Fixed-order fold of a split-K partial slab part [S, n] fp32 (n % 4 == 0) -> [n] fp32 / bf16 (the
// weight-gradient kernels' second stage; exposed for tests and the fold A/B).
Tensor split_fold(const Tensor& part, bool out_bf16) {
  check_dev(part, "part");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 2 &&
                  part.size(1) % 4 == 0 && part.size(0) >= 1 && part.size(0) < (1ll << 31),
              "split_fold: part must be contiguous fp32 [S, n] with n % 4 == 0");
  const c10::DeviceGuard guard(part.device());
  Tensor out = at::empty({part.size(1)}, part.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  CML_CHECK_HIP(cml::launch_wgrad_fold(part.data_ptr<float>(), static_cast<int>(part.size(0)),
                                       part.size(1), out.data_ptr(), out_bf16, cur_stream()));
  return out;
}

std::vector<Tensor> wgrad1x1_ex(const Tensor& dy_in, const Tensor& x, const optional<Tensor>& pro_sc,
                                const optional<Tensor>& pro_bi, int64_t dmode,
                                const optional<Tensor>& dz_mask, const optional<Tensor>& dz_a,
                                const optional<Tensor>& dz_b, const optional<Tensor>& dz_c,
                                bool colsum) {
  check_nhwc(x, "x");
  Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dy, "dy");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && dy.size(0) == x.size(0) && dy.size(2) == x.size(2) &&
                  dy.size(3) == x.size(3), "wgrad1x1_ex: dy / x shapes");
  TORCH_CHECK(dmode == 0 || dmode == 2 || dmode == 3, "wgrad1x1_ex: dmode 0, 2 or 3");
  const int64_t Co = dy.size(1), Ci = x.size(1), P = x.numel() / Ci;
  const float* sc = opt_ptr<const float>(pro_sc, at::kFloat, "pro_sc", Ci);
  const float* bi = opt_ptr<const float>(pro_bi, at::kFloat, "pro_bi", Ci);
  TORCH_CHECK((sc == nullptr) == (bi == nullptr), "wgrad1x1_ex: pro_sc and pro_bi together");
  const c10::DeviceGuard guard(x.device());
  int S = 1, cps = 1;
  cml::wgrad1x1_plan(P, static_cast<int>(Co), static_cast<int>(Ci), &S, &cps, sc != nullptr,
                     static_cast<int>(dmode), colsum);
  auto f32 = x.options().dtype(at::kFloat);
  Tensor part = at::empty({S, Co, Ci}, f32);
  Tensor dw = at::empty({Co, Ci}, f32);
  Tensor cs, cs_part;
  if (colsum) {
    cs = at::empty({Co}, f32);
    cs_part = at::empty({S, Co}, f32);
  }
  CML_CHECK_HIP(cml::launch_wgrad1x1_ex(
      dy.data_ptr(), x.data_ptr(), part.data_ptr<float>(), dw.data_ptr(), false, P,
      static_cast<int>(Co), static_cast<int>(Ci), sc, bi, cur_stream(), static_cast<int>(dmode),
      nullptr, opt_ptr<const uint8_t>(dz_mask, at::kByte, "dz_mask", P * Co / 8),
      opt_ptr<const float>(dz_a, at::kFloat, "dz_a", Co),
      opt_ptr<const float>(dz_b, at::kFloat, "dz_b", Co),
      opt_ptr<const float>(dz_c, at::kFloat, "dz_c", Co),
      colsum ? cs_part.data_ptr<float>() : nullptr, colsum ? cs.data_ptr<float>() : nullptr));
  return {dw, cs};
}

namespace {
// [Cout, Cin] bf16 weight given for a backward GEMM (already transposed by the caller)
void check_w2(const Tensor& w, int64_t K, const char* fn) {
  check_dev(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 &&
                  w.size(1) == K && w.size(0) % 64 == 0 && K % 64 == 0,
              fn, ": w must be contiguous bf16 [N, K] with N, K multiples of 64");
}
}  // namespace

// Data gradient through a BN + ReLU backward prologue (conv1x1.hip PM_BNBWD): g, z [N, K, H, W]
// NHWC bf16 (output gradient and input of the BN), mask [M, K/8] (the BN's ReLU bits), ca / cb /
// cc fp32 [K] (bn_bwd_coeffs), w [Nout, K] -> y [N, Nout, H, W] = (ca (m ? g : 0) + cb z + cc) w^T.
Tensor conv1x1_bnbwd(const Tensor& g, const Tensor& z, const Tensor& mask, const Tensor& ca,
                     const Tensor& cb, const Tensor& cc, const Tensor& w) {
  check_nhwc(g, "g");
  check_nhwc(z, "z");
  TORCH_CHECK(g.dim() == 4 && z.sizes() == g.sizes(), "conv1x1_bnbwd: g / z shapes");
  const int64_t N = g.size(0), K = g.size(1), H = g.size(2), W = g.size(3), M = N * H * W;
  check_w2(w, K, "conv1x1_bnbwd");
  const int64_t No = w.size(0);
  const uint8_t* mp = opt_ptr<const uint8_t>(mask, at::kByte, "mask", M * K / 8);
  const float* pa = opt_ptr<const float>(ca, at::kFloat, "ca", K);
  const float* pb = opt_ptr<const float>(cb, at::kFloat, "cb", K);
  const float* pc = opt_ptr<const float>(cc, at::kFloat, "cc", K);
  const c10::DeviceGuard guard(g.device());
  Tensor y = at::empty({N, No, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  CML_CHECK_HIP(cml::launch_conv1x1_bnbwd(g.data_ptr(), z.data_ptr(), mp, pa, pb, pc, w.data_ptr(),
                                          y.data_ptr(), M, static_cast<int>(K),
                                          static_cast<int>(No), cur_stream()));
  return y;
}

// Data gradient with the masked residual gradient added in the epilogue: x [N, K, H, W] NHWC bf16,
// w [Nout, K], link [N, Nout, H, W] + lmask [M, Nout/8] -> y = x w^T + (lmask ? link : 0). With sz /
// smask / mean / invstd (the BN + ReLU that consumes y): also {sdz, sdzx} = its backward sums.
std::vector<Tensor> conv1x1_link(const Tensor& x, const Tensor& w, const Tensor& link,
                                 const optional<Tensor>& lmask, const optional<Tensor>& sz,
                                 const optional<Tensor>& smask, const optional<Tensor>& mean,
                                 const optional<Tensor>& invstd) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "conv1x1_link: 4-D NHWC input");
  const int64_t N = x.size(0), K = x.size(1), H = x.size(2), W = x.size(3), M = N * H * W;
  check_w2(w, K, "conv1x1_link");
  const int64_t No = w.size(0);
  check_nhwc(link, "link");
  TORCH_CHECK(link.dim() == 4 && link.size(0) == N && link.size(1) == No && link.size(2) == H &&
                  link.size(3) == W, "conv1x1_link: link shape");
  const uint8_t* lm = opt_ptr<const uint8_t>(lmask, at::kByte, "lmask", M * No / 8);
  const bool sums = sz.has_value() && sz->defined();
  const void* szp = nullptr;
  if (sums) {
    check_nhwc(*sz, "sz");
    TORCH_CHECK(sz->sizes() == link.sizes(), "conv1x1_link: sz shape");
    szp = sz->data_ptr();
  }
  const uint8_t* sm = opt_ptr<const uint8_t>(smask, at::kByte, "smask", M * No / 8);
  const float* mu = opt_ptr<const float>(mean, at::kFloat, "mean", No);
  const float* is = opt_ptr<const float>(invstd, at::kFloat, "invstd", No);
  TORCH_CHECK(!sums || (sm && mu && is), "conv1x1_link: sz needs smask, mean, invstd");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor y = at::empty({N, No, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor part, sdz, sdzx;
  if (sums) {
    part = at::empty({static_cast<int64_t>(cml::conv1x1_link_part_floats(M, static_cast<int>(K),
                                                                       static_cast<int>(No)))}, f32);
    sdz = at::empty({No}, f32);
    sdzx = at::empty({No}, f32);
  }
  CML_CHECK_HIP(cml::launch_conv1x1_link(
      x.data_ptr(), w.data_ptr(), y.data_ptr(), link.data_ptr(), lm, szp, sums ? sm : nullptr,
      sums ? mu : nullptr, sums ? is : nullptr, sums ? part.data_ptr<float>() : nullptr,
      sums ? sdz.data_ptr<float>() : nullptr, sums ? sdzx.data_ptr<float>() : nullptr, M,
      static_cast<int>(K), static_cast<int>(No), cur_stream()));
  return {y, sdz, sdzx};
}

// BN + ReLU backward coefficients from its sums: {ca, cb, cc} fp32 [C] with dz = ca (m ? dy : 0) +
// cb z + cc, and {dgamma, dbeta} in gamma's dtype (bf16).
// BN training statistics of z = y W^T (1x1 conv, W [Co, P(, 1, 1)] bf16) from y's Gram matrix G
// [P, P] and column sums cy [P] over M rows (fp32, e.g. wgrad1x1_ex mode 3 / 0 with sums)
// -> {mean, invstd}; running stats updated in place when given.
std::vector<Tensor> bn_stats_gram(const Tensor& G, const Tensor& cy, const Tensor& w, int64_t M,
                                  const optional<Tensor>& rmean, const optional<Tensor>& rvar,
                                  double eps, double momentum, const optional<Tensor>& gamma,
                                  const optional<Tensor>& beta) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() > 0,
              "bn_stats_gram: contiguous bf16 weights");
  const int64_t Co = w.size(0), P = w.numel() / Co;
  TORCH_CHECK(G.is_cuda() && G.scalar_type() == at::kFloat && G.is_contiguous() && G.numel() == P * P,
              "bn_stats_gram: G fp32 [P, P]");
  const float* cp = opt_ptr<const float>(cy, at::kFloat, "cy", P);
  TORCH_CHECK(M >= 1, "bn_stats_gram: M >= 1");
  const c10::DeviceGuard guard(w.device());
  auto f32 = w.options().dtype(at::kFloat);
  TORCH_CHECK(P % 64 == 0, "bn_stats_gram: P must be a multiple of 64");
  Tensor mean = at::empty({Co}, f32), invstd = at::empty({Co}, f32);
  Tensor part = at::empty({P / 64, Co}, w.options().dtype(at::kDouble));
  // gamma / beta given: also the BN affine (sc, bi) of these statistics (bn_affine, no launch)
  const bool aff = gamma.has_value() && gamma->defined();
  const void* gp = aff ? opt_ptr<const void>(gamma, at::kBFloat16, "gamma", Co) : nullptr;
  const void* bp = aff ? opt_ptr<const void>(beta, at::kBFloat16, "beta", Co) : nullptr;
  TORCH_CHECK(!aff || bp, "bn_stats_gram: beta with gamma");
  Tensor sc = aff ? at::empty({Co}, f32) : Tensor(), bi = aff ? at::empty({Co}, f32) : Tensor();
  CML_CHECK_HIP(cml::launch_bn_stats_gram(G.data_ptr<float>(), cp, w.data_ptr(), static_cast<int>(P),
                                          static_cast<int>(Co), M, static_cast<float>(eps),
                                          static_cast<float>(momentum), mean.data_ptr<float>(),
                                          invstd.data_ptr<float>(),
                                          opt_ptr<float>(rmean, at::kFloat, "running_mean", Co),
                                          opt_ptr<float>(rvar, at::kFloat, "running_var", Co),
                                          part.data_ptr<double>(), cur_stream(), gp, bp,
                                          aff ? sc.data_ptr<float>() : nullptr,
                                          aff ? bi.data_ptr<float>() : nullptr));
  if (aff) return {mean, invstd, sc, bi};
  return {mean, invstd};
}

std::vector<Tensor> bn_bwd_coeffs(const Tensor& sdz, const Tensor& sdzx, const Tensor& gamma,
                                  const Tensor& mean, const Tensor& invstd, int64_t M) {
  const int64_t C = gamma.numel();
  TORCH_CHECK(gamma.scalar_type() == at::kBFloat16 && gamma.is_contiguous() && gamma.is_cuda(),
              "bn_bwd_coeffs: bf16 gamma");
  const float* s = opt_ptr<const float>(sdz, at::kFloat, "sdz", C);
  const float* q = opt_ptr<const float>(sdzx, at::kFloat, "sdzx", C);
  const float* mu = opt_ptr<const float>(mean, at::kFloat, "mean", C);
  const float* is = opt_ptr<const float>(invstd, at::kFloat, "invstd", C);
  const c10::DeviceGuard guard(gamma.device());
  auto f32 = gamma.options().dtype(at::kFloat);
  Tensor ca = at::empty({C}, f32), cb = at::empty({C}, f32), cc = at::empty({C}, f32);
  Tensor dg = at::empty_like(gamma), db = at::empty_like(gamma);
  CML_CHECK_HIP(cml::launch_bn_bwd_coeffs(s, q, gamma.data_ptr(), mu, is, static_cast<int>(C), M,
                                          ca.data_ptr<float>(), cb.data_ptr<float>(),
                                          cc.data_ptr<float>(), dg.data_ptr(), db.data_ptr(),
                                          cur_stream()));
  return {ca, cb, cc, dg, db};
}

// Recompute-tail backward algebra in two launches (tail_prep.hip): W bf16 [Co, p] (any shape with
// Co * p elements, contiguous), P fp32 [Co, p], s fp32 [Co], gram fp32 [p, p], cy fp32 [p], gamma
// bf16 [Co], mean / invstd fp32 [Co] -> {w_cat bf16 [p, Co + p], bias fp32 [p], dW bf16 [Co, p]
// (undefined unless need_dw), dgamma, dbeta bf16 [Co]}.
std::vector<Tensor> tail_bwd_prep(const Tensor& W, const Tensor& P, const Tensor& s,
                                  const Tensor& gram, const Tensor& cy, const Tensor& gamma,
                                  const Tensor& mean, const Tensor& invstd, int64_t M,
                                  bool need_dw) {
  TORCH_CHECK(P.dim() == 2, "tail_bwd_prep: P [Co, p]");
  const int64_t Co = P.size(0), p = P.size(1);
  TORCH_CHECK(W.is_cuda() && W.scalar_type() == at::kBFloat16 && W.is_contiguous() &&
                  W.numel() == Co * p, "tail_bwd_prep: W contiguous bf16 with Co * p elements");
  TORCH_CHECK(gamma.scalar_type() == at::kBFloat16 && gamma.is_contiguous() && gamma.numel() == Co,
              "tail_bwd_prep: gamma bf16 [Co]");
  TORCH_CHECK(Co % 64 == 0 && p % 64 == 0, "tail_bwd_prep: Co % 64 == 0 and p % 64 == 0");
  check_dev(W, "W");
  check_dev(gamma, "gamma");
  const float* Pp = opt_ptr<const float>(P, at::kFloat, "P", Co * p);
  const float* sp = opt_ptr<const float>(s, at::kFloat, "s", Co);
  const float* gp = opt_ptr<const float>(gram, at::kFloat, "gram", p * p);
  const float* cp = opt_ptr<const float>(cy, at::kFloat, "cy", p);
  const float* mp = opt_ptr<const float>(mean, at::kFloat, "mean", Co);
  const float* ip = opt_ptr<const float>(invstd, at::kFloat, "invstd", Co);
  const c10::DeviceGuard guard(W.device());
  auto f32 = P.options();
  Tensor work = at::empty({static_cast<int64_t>(
                              cml::tail_bwd_prep_work_floats(static_cast<int>(Co), static_cast<int>(p)))},
                          f32);
  Tensor wcat = at::empty({p, Co + p}, W.options());
  Tensor bias = at::empty({p}, f32);
  Tensor dW = need_dw ? at::empty({Co, p}, W.options()) : Tensor();
  Tensor dg = at::empty_like(gamma), db = at::empty_like(gamma);
  CML_CHECK_HIP(cml::launch_tail_bwd_prep(
      W.data_ptr(), Pp, sp, gp, cp, gamma.data_ptr(), mp, ip, static_cast<int>(Co),
      static_cast<int>(p), M, work.data_ptr<float>(), need_dw ? dW.data_ptr() : nullptr,
      wcat.data_ptr(), bias.data_ptr<float>(), dg.data_ptr(), db.data_ptr(), cur_stream()));
  return {wcat, bias, dW, dg, db};
}

// Optional bf16 [C] output tensors for a BN's parameter gradients bf16(sum dy' xhat) /
// bf16(sum dy'), written by the finalize launch of the sums that produce them (both or neither).
std::pair<void*, void*> dgb_ptrs(const optional<Tensor>& dgamma_out,
                                 const optional<Tensor>& dbeta_out, int64_t C, const Tensor& like,
                                 const char* name) {
  const bool want = dgamma_out.has_value() && dgamma_out->defined();
  TORCH_CHECK(want == (dbeta_out.has_value() && dbeta_out->defined()), name,
              ": dgamma_out and dbeta_out together");
  if (!want) return {nullptr, nullptr};
  for (const Tensor* t : {&*dgamma_out, &*dbeta_out}) {
    check_dev(*t, "dgamma_out / dbeta_out");
    TORCH_CHECK(t->device() == like.device() && t->scalar_type() == at::kBFloat16 &&
                    t->is_contiguous() && t->numel() == C,
                name, ": dgamma_out / dbeta_out must be contiguous bf16 [C]");
  }
  return {dgamma_out->data_ptr(), dbeta_out->data_ptr()};
}

// Optional BN affine output of a statistics finalize (gamma / beta: the BN's bf16 [C] parameters,
// both or neither): allocates sc / bi fp32 [C] and fills `out`; nullptr when not requested.
const cml::BnAffineOut* aff_out(const optional<Tensor>& gamma, const optional<Tensor>& beta,
                                int64_t C, const Tensor& like, const char* name, Tensor& sc,
                                Tensor& bi, cml::BnAffineOut& out) {
  const bool want = gamma.has_value() && gamma->defined();
  TORCH_CHECK(want == (beta.has_value() && beta->defined()), name, ": gamma and beta together");
  if (!want) return nullptr;
  for (const Tensor* t : {&*gamma, &*beta}) {
    check_dev(*t, "gamma / beta");
    TORCH_CHECK(t->device() == like.device() && t->scalar_type() == at::kBFloat16 &&
                    t->is_contiguous() && t->numel() == C,
                name, ": gamma / beta must be contiguous bf16 [C]");
  }
  auto f32 = like.options().dtype(at::kFloat);
  sc = at::empty({C}, f32);
  bi = at::empty({C}, f32);
  out = cml::BnAffineOut{gamma->data_ptr(), beta->data_ptr(), sc.data_ptr<float>(),
                         bi.data_ptr<float>()};
  return &out;
}

// Fused 1x1 conv forward (conv1x1.hip): x [N, K, H, W] NHWC bf16, w [Cout, K, 1, 1] bf16 ->
// {y [N, Cout, OH, OW] NHWC, mean, invstd} (mean / invstd: training BN statistics of y, undefined
// when !stats). pro_sc / pro_bi (fp32 [K]): apply max(x * sc + bi, 0) to the input on load.
// shift / rmean / rvar: fp32 [Cout] (statistics shift, running statistics updated in place).
std::vector<Tensor> conv1x1_bn_fwd(const Tensor& x, const Tensor& w, const optional<Tensor>& pro_sc,
                                   const optional<Tensor>& pro_bi, const optional<Tensor>& shift,
                                   const optional<Tensor>& rmean, const optional<Tensor>& rvar,
                                   int64_t stride, bool stats, double eps, double momentum,
                                   const optional<Tensor>& gamma, const optional<Tensor>& beta) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "conv1x1_bn_fwd: 4-D NHWC input");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 1 && w.size(3) == 1 &&
                  w.size(1) == x.size(1), "conv1x1_bn_fwd: w must be bf16 [Cout, Cin, 1, 1]");
  TORCH_CHECK(w.is_contiguous() || w.is_contiguous(at::MemoryFormat::ChannelsLast), "w layout");
  TORCH_CHECK(stride == 1 || stride == 2, "stride 1 or 2");
  const int64_t N = x.size(0), K = x.size(1), H = x.size(2), W = x.size(3), Co = w.size(0);
  TORCH_CHECK(K % 64 == 0 && Co % 64 == 0, "conv1x1_bn_fwd: channels must be multiples of 64");
  TORCH_CHECK(stride == 1 || (H % 2 == 0 && W % 2 == 0), "stride 2 needs even H, W");
  const int64_t OH = H / stride, OW = W / stride;
  const int64_t M = N * OH * OW;
  const bool pro = pro_sc.has_value() && pro_sc->defined();
  const float* sc = opt_ptr<const float>(pro_sc, at::kFloat, "pro_sc", K);
  const float* bi = opt_ptr<const float>(pro_bi, at::kFloat, "pro_bi", K);
  TORCH_CHECK(!pro || bi, "pro_bi needed with pro_sc");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor y = at::empty({N, Co, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor mean, invstd, part;
  if (stats) {
    mean = at::empty({Co}, f32);
    invstd = at::empty({Co}, f32);
    part = at::empty({static_cast<int64_t>(cml::conv1x1_bn_part_floats(M, static_cast<int>(K),
                                                                     static_cast<int>(Co), pro))}, f32);
  }
  Tensor asc, abi;
  cml::BnAffineOut ao{};
  const cml::BnAffineOut* aff = aff_out(gamma, beta, Co, x, "conv1x1_bn_fwd", asc, abi, ao);
  TORCH_CHECK(stats || !aff, "conv1x1_bn_fwd: the affine needs stats");
  CML_CHECK_HIP(cml::launch_conv1x1_bn_fwd(
      x.data_ptr(), w.data_ptr(), y.data_ptr(), stats ? part.data_ptr<float>() : nullptr, sc, bi,
      opt_ptr<const float>(shift, at::kFloat, "shift", Co), M, static_cast<int>(K),
      static_cast<int>(Co), static_cast<int>(stride), static_cast<int>(H), static_cast<int>(W),
      stats ? mean.data_ptr<float>() : nullptr, stats ? invstd.data_ptr<float>() : nullptr,
      stats ? opt_ptr<float>(rmean, at::kFloat, "running_mean", Co) : nullptr,
      stats ? opt_ptr<float>(rvar, at::kFloat, "running_var", Co) : nullptr,
      static_cast<float>(eps), static_cast<float>(momentum), cur_stream(), aff));
  if (aff) return {y, mean, invstd, asc, abi};
  return {y, mean, invstd};
}

// Statistics-only pass of a stride-1 1x1 conv with the BN + ReLU prologue (the product is not
// stored): {mean, invstd} of bf16(conv1x1(max(x sc + bi, 0))), running stats updated when given.
std::vector<Tensor> conv1x1_bn_stats_only(const Tensor& x, const Tensor& w,
                                          const optional<Tensor>& pro_sc,
                                          const optional<Tensor>& pro_bi, const optional<Tensor>& shift,
                                          const optional<Tensor>& rmean,
                                          const optional<Tensor>& rvar, double eps, double momentum) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4 && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 1 &&
                  w.size(3) == 1 && w.size(1) == x.size(1) && w.is_contiguous(),
              "conv1x1_bn_stats_only: x NHWC, w contiguous bf16 [Cout, Cin, 1, 1]");
  const int64_t K = x.size(1), Co = w.size(0), M = x.numel() / K;
  TORCH_CHECK(K % 64 == 0 && Co % 64 == 0, "conv1x1_bn_stats_only: channels multiples of 64");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({Co}, f32), invstd = at::empty({Co}, f32);
  const bool pro = pro_sc.has_value() && pro_sc->defined();
  TORCH_CHECK(pro == (pro_bi.has_value() && pro_bi->defined()), "pro_sc and pro_bi together");
  Tensor part = at::empty({static_cast<int64_t>(cml::conv1x1_bn_part_floats(
                              M, static_cast<int>(K), static_cast<int>(Co), pro))}, f32);
  CML_CHECK_HIP(cml::launch_conv1x1_bn_fwd(
      x.data_ptr(), w.data_ptr(), nullptr, part.data_ptr<float>(),
      opt_ptr<const float>(pro_sc, at::kFloat, "pro_sc", K),
      opt_ptr<const float>(pro_bi, at::kFloat, "pro_bi", K),
      opt_ptr<const float>(shift, at::kFloat, "shift", Co), M, static_cast<int>(K),
      static_cast<int>(Co), 1, 0, 0, mean.data_ptr<float>(), invstd.data_ptr<float>(),
      opt_ptr<float>(rmean, at::kFloat, "running_mean", Co),
      opt_ptr<float>(rvar, at::kFloat, "running_var", Co), static_cast<float>(eps),
      static_cast<float>(momentum), cur_stream()));
  return {mean, invstd};
}

// y = max(bf16(conv1x1(max(x sc + bi, 0))) ep_sc + ep_bi + res, 0) and its ReLU bit mask
// [M, Cout / 8] (uint8) -- the apply pass of a BN whose statistics came from
// conv1x1_bn_stats_only, recomputing the product instead of reading it.
std::vector<Tensor> conv1x1_bnres(const Tensor& x, const Tensor& w, const Tensor& pro_sc,
                                  const Tensor& pro_bi, const Tensor& ep_sc, const Tensor& ep_bi,
                                  const Tensor& res) {
  check_nhwc(x, "x");
  check_nhwc(res, "res");
  TORCH_CHECK(x.dim() == 4 && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 1 &&
                  w.size(3) == 1 && w.size(1) == x.size(1) && w.is_contiguous(),
              "conv1x1_bnres: x NHWC, w contiguous bf16 [Cout, Cin, 1, 1]");
  const int64_t N = x.size(0), K = x.size(1), H = x.size(2), W = x.size(3), Co = w.size(0);
  const int64_t M = N * H * W;
  TORCH_CHECK(res.dim() == 4 && res.size(0) == N && res.size(1) == Co && res.size(2) == H &&
                  res.size(3) == W, "conv1x1_bnres: res shape");
  TORCH_CHECK(K % 64 == 0 && Co % 64 == 0, "conv1x1_bnres: channels multiples of 64");
  const c10::DeviceGuard guard(x.device());
  Tensor y = at::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor mask = at::empty({M, Co / 8}, x.options().dtype(at::kByte));
  CML_CHECK_HIP(cml::launch_conv1x1_bnres(
      x.data_ptr(), w.data_ptr(), y.data_ptr(), mask.data_ptr<uint8_t>(),
      opt_ptr<const float>(pro_sc, at::kFloat, "pro_sc", K),
      opt_ptr<const float>(pro_bi, at::kFloat, "pro_bi", K),
      opt_ptr<const float>(ep_sc, at::kFloat, "ep_sc", Co),
      opt_ptr<const float>(ep_bi, at::kFloat, "ep_bi", Co), res.data_ptr(), M,
      static_cast<int>(K), static_cast<int>(Co), cur_stream()));
  return {y, mask};
}

namespace {
// shapes of a two-source 1x1 GEMM: {N, K1, H, W, K2, M, K, Co}
std::array<int64_t, 8> cat_shape(const Tensor& x1, const Tensor& x2, const Tensor& w,
                                 const char* what) {
  check_nhwc(x1, "x1");
  check_nhwc(x2, "x2");
  const int64_t N = x1.size(0), K1 = x1.size(1), H = x1.size(2), W = x1.size(3), K2 = x2.size(1);
  TORCH_CHECK(x2.dim() == 4 && x2.size(0) == N && x2.size(2) == H && x2.size(3) == W, what,
              ": x2 shape");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 2 &&
                  w.size(1) == K1 + K2 && w.is_contiguous() && w.size(0) % 64 == 0 &&
                  K1 % 64 == 0 && K2 % 64 == 0,
              what, ": w contiguous bf16 [Cout, K1 + K2], channels multiples of 64");
  return {N, K1, H, W, K2, N * H * W, K1 + K2, w.size(0)};
}
}  // namespace

// Downsample tail in one GEMM: y = max(bf16([max(x1 sc1 + bi1, 0) | f2(x2)] w^T) ep_sc + ep_bi, 0)
// and its ReLU bit mask; f2 = max(x2 sc2 + bi2, 0), or x2 itself when sc2 / bi2 are None (a ReLU
// output); sc / bi fp32 [K1] / [K2], w [Cout, K1 + K2] bf16.
std::vector<Tensor> conv1x1_cat_bnres(const Tensor& x1, const Tensor& x2, const Tensor& sc1,
                                      const Tensor& bi1, const optional<Tensor>& sc2,
                                      const optional<Tensor>& bi2, const Tensor& w,
                                      const Tensor& ep_sc, const Tensor& ep_bi) {
  const auto [N, K1, H, W, K2, M, K, Co] = cat_shape(x1, x2, w, "conv1x1_cat_bnres");
  const c10::DeviceGuard guard(x1.device());
  Tensor y = at::empty({N, Co, H, W}, x1.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor mask = at::empty({M, Co / 8}, x1.options().dtype(at::kByte));
  CML_CHECK_HIP(cml::launch_conv1x1_cat_bnres(
      x1.data_ptr(), x2.data_ptr(), opt_ptr<const float>(sc1, at::kFloat, "sc1", K1),
      opt_ptr<const float>(bi1, at::kFloat, "bi1", K1),
      opt_ptr<const float>(sc2, at::kFloat, "sc2", K2),
      opt_ptr<const float>(bi2, at::kFloat, "bi2", K2), w.data_ptr(),
      opt_ptr<const float>(ep_sc, at::kFloat, "ep_sc", Co),
      opt_ptr<const float>(ep_bi, at::kFloat, "ep_bi", Co), nullptr, y.data_ptr(),
      mask.data_ptr<uint8_t>(), M, static_cast<int>(K1), static_cast<int>(K),
      static_cast<int>(Co), cur_stream()));
  return {y, mask};
}

// y = [(mask ? g : 0) | f2(x2)] w^T + bias (two sources concatenated along K): g [N, K1, H, W],
// mask [M, K1 / 8], x2 [N, K2, H, W] NHWC bf16; f2 = max(x2 sc2 + bi2, 0) (fp32 [K2]) or x2 itself
// (None); bias fp32 [Cout] or None; w [Cout, K1 + K2] contiguous bf16 -> y [N, Cout, H, W] NHWC.
// A BN + ReLU backward on g (a (mask ? g : 0) + c) is folded by the caller: w[:, :K1] diag(a),
// bias += w[:, :K1] c (ops.conv.fold_cat).
Tensor conv1x1_cat(const Tensor& g, const Tensor& mask, const Tensor& x2,
                   const optional<Tensor>& sc2, const optional<Tensor>& bi2, const Tensor& w,
                   const optional<Tensor>& bias) {
  const auto [N, K1, H, W, K2, M, K, Co] = cat_shape(g, x2, w, "conv1x1_cat");
  const c10::DeviceGuard guard(g.device());
  Tensor y = at::empty({N, Co, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  CML_CHECK_HIP(cml::launch_conv1x1_cat(
      g.data_ptr(), opt_ptr<const uint8_t>(mask, at::kByte, "mask", M * K1 / 8), x2.data_ptr(),
      opt_ptr<const float>(sc2, at::kFloat, "sc2", K2),
      opt_ptr<const float>(bi2, at::kFloat, "bi2", K2),
      opt_ptr<const float>(bias, at::kFloat, "bias", Co), w.data_ptr(), y.data_ptr(), M,
      static_cast<int>(K1), static_cast<int>(K), static_cast<int>(Co), cur_stream()));
  return y;
}

// conv1x1_cat whose output dy2 is the gradient of relu(bn(x2)) (Cout = K2; sc2 / bi2 are that
// BN's affine): also that BN + ReLU backward's sums {sdz, sdzx} from the epilogue (mask
// recomputed from x2), so only bn_bwd_apply remains. mean / invstd fp32 [K2].
std::vector<Tensor> conv1x1_cat_bnsums(const Tensor& g, const Tensor& mask, const Tensor& x2,
                                       const Tensor& sc2, const Tensor& bi2, const Tensor& w,
                                       const optional<Tensor>& bias, const Tensor& mean,
                                       const Tensor& invstd, const optional<Tensor>& dgamma_out,
                                       const optional<Tensor>& dbeta_out) {
  const auto [N, K1, H, W, K2, M, K, Co] = cat_shape(g, x2, w, "conv1x1_cat_bnsums");
  TORCH_CHECK(Co == K2, "conv1x1_cat_bnsums: w must be [K2, K1 + K2]");
  const c10::DeviceGuard guard(g.device());
  auto f32 = g.options().dtype(at::kFloat);
  Tensor y = at::empty({N, Co, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor part = at::empty({static_cast<int64_t>(cml::conv1x1_cat_part_floats(M, K, Co))}, f32);
  Tensor sdz = at::empty({Co}, f32), sdzx = at::empty({Co}, f32);
  const auto [dg, db] = dgb_ptrs(dgamma_out, dbeta_out, Co, g, "conv1x1_cat_bnsums");
  CML_CHECK_HIP(cml::launch_conv1x1_cat(
      g.data_ptr(), opt_ptr<const uint8_t>(mask, at::kByte, "mask", M * K1 / 8), x2.data_ptr(),
      opt_ptr<const float>(sc2, at::kFloat, "sc2", K2),
      opt_ptr<const float>(bi2, at::kFloat, "bi2", K2),
      opt_ptr<const float>(bias, at::kFloat, "bias", Co), w.data_ptr(), y.data_ptr(), M,
      static_cast<int>(K1), static_cast<int>(K), static_cast<int>(Co), cur_stream(),
      opt_ptr<const float>(mean, at::kFloat, "mean", Co),
      opt_ptr<const float>(invstd, at::kFloat, "invstd", Co), part.data_ptr<float>(),
      sdz.data_ptr<float>(), sdzx.data_ptr<float>(), dg, db));
  return {y, sdz, sdzx};
}

// {sc, bi} fp32 [2, C]: sc = gamma invstd, bi = beta - mean sc (gamma / beta bf16 [C]).
Tensor bn_affine(const Tensor& gamma, const Tensor& beta, const Tensor& mean, const Tensor& invstd) {
  const int64_t C = gamma.numel();
  TORCH_CHECK(gamma.scalar_type() == at::kBFloat16 && beta.scalar_type() == at::kBFloat16 &&
                  gamma.is_contiguous() && beta.is_contiguous() && beta.numel() == C && C > 0,
              "bn_affine: contiguous bf16 gamma / beta [C]");
  check_dev(gamma, "gamma");
  check_dev(beta, "beta");
  const c10::DeviceGuard guard(gamma.device());
  Tensor out = at::empty({2, C}, gamma.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_bn_affine(gamma.data_ptr(), beta.data_ptr(),
                                      opt_ptr<const float>(mean, at::kFloat, "mean", C),
                                      opt_ptr<const float>(invstd, at::kFloat, "invstd", C),
                                      static_cast<int>(C), out.data_ptr<float>(),
                                      out.data_ptr<float>() + C, cur_stream()));
  return out;
}

// Apply half of a BN + ReLU backward (mask recomputed from x) from its sums: dy, x [N, C, H, W]
// NHWC bf16 -> dx.
Tensor bn_bwd_apply(const Tensor& dy_in, const Tensor& x, const Tensor& gamma, const Tensor& beta,
                    const Tensor& mean, const Tensor& invstd, const Tensor& sdz,
                    const Tensor& sdzx) {
  check_nhwc(x, "x");
  Tensor dy = x.dim() == 4 ? dy_in.contiguous(at::MemoryFormat::ChannelsLast) : dy_in.contiguous();
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "bn_bwd_apply: dy shape mismatch");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(gamma.scalar_type() == at::kBFloat16 && beta.scalar_type() == at::kBFloat16 &&
                  gamma.numel() == C && beta.numel() == C,
              "bn_bwd_apply: bf16 gamma / beta [C]");
  const c10::DeviceGuard guard(x.device());
  Tensor dx = at::empty_like(x);
  CML_CHECK_HIP(cml::launch_bn_bwd_apply(
      dy.data_ptr(), x.data_ptr(), dx.data_ptr(), M, static_cast<int>(C), gamma.data_ptr(),
      beta.data_ptr(), opt_ptr<const float>(mean, at::kFloat, "mean", C),
      opt_ptr<const float>(invstd, at::kFloat, "invstd", C),
      opt_ptr<const float>(sdz, at::kFloat, "sdz", C),
      opt_ptr<const float>(sdzx, at::kFloat, "sdzx", C), cur_stream()));
  return dx;
}

// dX = dY W (1x1, stride 1: x = dY [N, K, H, W] NHWC, w [No, K] -- W^T of the conv's weight)
// plus, at the even pixels, link [N, No, ceil(H/2), ceil(W/2)]: a parallel stride-2 conv's
// compact data gradient (never scattered to full resolution).
Tensor conv1x1_link_s2(const Tensor& x, const Tensor& w, const Tensor& link_in) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "conv1x1_link_s2: 4-D NHWC input");
  const int64_t N = x.size(0), K = x.size(1), H = x.size(2), W = x.size(3);
  check_w2(w, K, "conv1x1_link_s2");
  const int64_t No = w.size(0);
  Tensor link = link_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(link, "link");
  TORCH_CHECK(link.dim() == 4 && link.size(0) == N && link.size(1) == No &&
                  link.size(2) == (H + 1) / 2 && link.size(3) == (W + 1) / 2,
              "conv1x1_link_s2: link [N, No, ceil(H/2), ceil(W/2)]");
  const c10::DeviceGuard guard(x.device());
  Tensor y = at::empty({N, No, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  CML_CHECK_HIP(cml::launch_conv1x1_link_s2(x.data_ptr(), w.data_ptr(), y.data_ptr(),
                                            link.data_ptr(), static_cast<int>(N),
                                            static_cast<int>(H), static_cast<int>(W),
                                            static_cast<int>(K), static_cast<int>(No),
                                            cur_stream()));
  return y;
}

// x[:, :, ::2, ::2] of an NHWC bf16 tensor as a dense NHWC tensor, and the backward scatter
// (full resolution, zeros at the odd pixels; H, W: the full-resolution size).
Tensor subsample2(const Tensor& x) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(1) % 8 == 0, "subsample2: 4-D NHWC, C % 8 == 0");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const c10::DeviceGuard guard(x.device());
  Tensor y = at::empty({N, C, (H + 1) / 2, (W + 1) / 2},
                       x.options().memory_format(at::MemoryFormat::ChannelsLast));
  CML_CHECK_HIP(cml::launch_subsample2(x.data_ptr(), y.data_ptr(), static_cast<int>(N),
                                       static_cast<int>(H), static_cast<int>(W),
                                       static_cast<int>(C), cur_stream()));
  return y;
}

Tensor upsample2_scatter(const Tensor& g_in, int64_t H, int64_t W) {
  Tensor g = g_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(g, "g");
  const int64_t N = g.size(0), C = g.size(1);
  TORCH_CHECK(g.dim() == 4 && C % 8 == 0 && g.size(2) == (H + 1) / 2 && g.size(3) == (W + 1) / 2,
              "upsample2_scatter: g [N, C, ceil(H/2), ceil(W/2)], C % 8 == 0");
  const c10::DeviceGuard guard(g.device());
  Tensor dx = at::empty({N, C, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  CML_CHECK_HIP(cml::launch_upsample2_scatter(g.data_ptr(), dx.data_ptr(), static_cast<int>(N),
                                              static_cast<int>(H), static_cast<int>(W),
                                              static_cast<int>(C), cur_stream()));
  return dx;
}


// Weight gradient of a 3x3 / stride 1 / padding 1 conv (wgrad3x3.hip, nine taps per workgroup):
// dy [N, Co, H, W], x [N, Ci, H, W] NHWC bf16 -> dW [Co, Ci, 3, 3] in `dtype` (channels_last memory).
Tensor wgrad3x3(const Tensor& dy_in, const Tensor& x, at::ScalarType dtype,
                const optional<Tensor>& zero_in) {
  check_nhwc(x, "x");
  Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dy, "dy");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && dy.size(0) == x.size(0) && dy.size(2) == x.size(2) &&
                  dy.size(3) == x.size(3), "wgrad3x3: dy / x shapes");
  TORCH_CHECK(dtype == at::kBFloat16 || dtype == at::kFloat, "wgrad3x3: bf16 or fp32 output");
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3), Co = dy.size(1);
  const c10::DeviceGuard guard(x.device());
  int S = 1, T = 0;
  TORCH_CHECK(cml::wgrad3x3_direct_plan(static_cast<int>(N), static_cast<int>(H),
                                        static_cast<int>(W), static_cast<int>(Co),
                                        static_cast<int>(Ci), &S, &T),
              "wgrad3x3: no plan for this shape (check wgrad3x3_direct_ok first)");
  // all nine taps per workgroup (wgrad3x3.hip); dW in the channels_last order of [Co, Ci, 3, 3]
  Tensor zero;
  if (zero_in.has_value() && zero_in->defined()) {
    zero = *zero_in;
    TORCH_CHECK(zero.is_cuda() && zero.device() == x.device() && zero.scalar_type() == at::kBFloat16 &&
                    zero.is_contiguous() && zero.numel() >= 8, "wgrad3x3: zero must be >= 8 bf16");
  } else {
    zero = at::zeros({64}, x.options());
  }
  Tensor part = at::empty({S, Co, 9, Ci}, x.options().dtype(at::kFloat));
  Tensor dw = at::empty({Co, 3, 3, Ci}, x.options().dtype(dtype));
  CML_CHECK_HIP(cml::launch_wgrad3x3_direct(dy.data_ptr(), x.data_ptr(), zero.data_ptr(),
                                            part.data_ptr<float>(), dw.data_ptr(),
                                            dtype == at::kBFloat16, static_cast<int>(N),
                                            static_cast<int>(H), static_cast<int>(W),
                                            static_cast<int>(Co), static_cast<int>(Ci),
                                            cur_stream()));
  return dw.permute({0, 3, 1, 2});
}

bool wgrad3x3s2_ok(int64_t N, int64_t H, int64_t W, int64_t Co, int64_t Ci, int64_t taps) {
  int S = 0;
  return N < (1 << 30) && H < (1 << 15) && W < (1 << 15) && Co < (1 << 20) && Ci < (1 << 20) &&
         (taps == 9 || taps == 1) &&
         cml::wgrad3x3s2_plan(static_cast<int>(N), static_cast<int>(H), static_cast<int>(W),
                              static_cast<int>(Co), static_cast<int>(Ci), &S, static_cast<int>(taps));
}

// Weight gradient of a 3x3 / stride 2 / padding 1 conv (wgrad1x1.hip LDS-DMA kernel on the implicit
// im2col): dy [N, Co, H/2, W/2], x [N, Ci, H, W] NHWC bf16 -> dW [Co, Ci, 3, 3] in `dtype`
// (channels_last memory). taps = 1: a 1x1 / stride 2 / padding 0 conv -> dW [Co, Ci, 1, 1].
Tensor wgrad3x3s2(const Tensor& dy_in, const Tensor& x, at::ScalarType dtype,
                  const optional<Tensor>& zero_in, int64_t taps) {
  check_nhwc(x, "x");
  Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dy, "dy");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && dy.size(0) == x.size(0) &&
                  x.size(2) % 2 == 0 && x.size(3) % 2 == 0 && dy.size(2) * 2 == x.size(2) &&
                  dy.size(3) * 2 == x.size(3), "wgrad3x3s2: dy [N, Co, H/2, W/2], x [N, Ci, H, W]");
  TORCH_CHECK(dtype == at::kBFloat16 || dtype == at::kFloat, "wgrad3x3s2: bf16 or fp32 output");
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3), Co = dy.size(1);
  TORCH_CHECK(wgrad3x3s2_ok(N, H, W, Co, Ci, taps),
              "wgrad3x3s2: no plan for this shape (check wgrad3x3s2_ok first)");
  const c10::DeviceGuard guard(x.device());
  int S = 1;
  cml::wgrad3x3s2_plan(static_cast<int>(N), static_cast<int>(H), static_cast<int>(W),
                       static_cast<int>(Co), static_cast<int>(Ci), &S, static_cast<int>(taps));
  Tensor zero;
  if (zero_in.has_value() && zero_in->defined()) {
    zero = *zero_in;
    TORCH_CHECK(zero.is_cuda() && zero.device() == x.device() && zero.scalar_type() == at::kBFloat16 &&
                    zero.is_contiguous() && zero.numel() >= 256 && zero.data_ptr() != nullptr &&
                    reinterpret_cast<uintptr_t>(zero.data_ptr()) % 16 == 0,
                "wgrad3x3s2: zero must be >= 256 contiguous 16-B aligned bf16");
  } else {
    zero = at::zeros({256}, x.options());
  }
  const int64_t k = taps == 1 ? 1 : 3;
  Tensor part = at::empty({S, Co, taps, Ci}, x.options().dtype(at::kFloat));
  Tensor dw = at::empty({Co, k, k, Ci}, x.options().dtype(dtype));
  CML_CHECK_HIP(cml::launch_wgrad3x3s2(dy.data_ptr(), x.data_ptr(), zero.data_ptr(),
                                       part.data_ptr<float>(), dw.data_ptr(),
                                       dtype == at::kBFloat16, static_cast<int>(N),
                                       static_cast<int>(H), static_cast<int>(W),
                                       static_cast<int>(Co), static_cast<int>(Ci), cur_stream(),
                                       static_cast<int>(taps)));
  return dw.permute({0, 3, 1, 2});
}

// Implicit-GEMM conv (conv_gemm.hip): x [N, C, H, W] NHWC bf16, w [Cout, taps * C] contiguous
// bf16 (k = tap C + c), taps 1 or 9 (3x3, padding 1) -> y [N, Cout, H, W] NHWC.
// Stride-1 conv_gemm whose output is the gradient of relu(bn(z)) (z [N, Cout, H, W] NHWC bf16, sc /
// bi bn's affine, mean / invstd its batch statistics, fp32 [Cout]): {y, sdz, sdzx} with that BN +
// ReLU backward's sums from the epilogue (bn_bwd_apply finishes it).
// {wf or None, wr}: the GEMM layouts of a bf16 [Co, Ci, 3, 3] conv weight (any strides) for the
// implicit-GEMM forward (wf [Co, 9 Ci]) and data gradient (wr [Ci, 9 Co], rotated / transposed).
std::vector<Tensor> conv3x3_wlayouts(const Tensor& w, bool want_wf) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 3 &&
                  w.size(3) == 3, "conv3x3_wlayouts: bf16 [Co, Ci, 3, 3] CUDA weight");
  const int64_t Co = w.size(0), Ci = w.size(1);
  const c10::DeviceGuard guard(w.device());
  Tensor wr = at::empty({Ci, 9 * Co}, w.options().memory_format(at::MemoryFormat::Contiguous));
  Tensor wf;
  if (want_wf) wf = at::empty({Co, 9 * Ci}, w.options().memory_format(at::MemoryFormat::Contiguous));
  CML_CHECK_HIP(cml::launch_conv3x3_wlayouts(w.data_ptr(), static_cast<int>(Co),
                                             static_cast<int>(Ci), w.stride(0), w.stride(1),
                                             w.stride(2), w.stride(3),
                                             want_wf ? wf.data_ptr() : nullptr, wr.data_ptr(),
                                             cur_stream()));
  return {wf, wr};   // wf undefined (None) unless asked for
}

// Global-average-pool backward: g [N, C] bf16 -> dx [N, C, H, W] channels_last, g / (H W) at every
// pixel (one write-only pass; bit-identical to (g.float() / (H W)).to(bf16) broadcast).
Tensor avgpool_bwd(const Tensor& g_in, int64_t H, int64_t W) {
  Tensor g = g_in.contiguous();
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kBFloat16 && g.dim() == 2 && g.size(1) % 8 == 0,
              "avgpool_bwd: bf16 [N, C] CUDA gradient, C % 8 == 0");
  const c10::DeviceGuard guard(g.device());
  const int64_t N = g.size(0), C = g.size(1);
  Tensor dx = at::empty({N, C, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  CML_CHECK_HIP(cml::launch_avgpool_bwd(g.data_ptr(), dx.data_ptr(), static_cast<int>(N),
                                        static_cast<int>(H * W), static_cast<int>(C),
                                        cur_stream()));
  return dx;
}

// GEMM layouts of several conv weights (bf16, one device, any strides) in one launch: a 3x3
// [Co, Ci, 3, 3] gives (wf, wr) as conv3x3_wlayouts, a 1x1 [Co, Ci, 1, 1] gives (None, W^T
// [Ci, Co] contiguous) -- [(wf, wr), ...].
std::vector<std::vector<Tensor>> conv_wlayouts_multi(const std::vector<Tensor>& ws) {
  std::vector<std::vector<Tensor>> out;
  if (ws.empty()) return out;
  const c10::DeviceGuard guard(ws[0].device());
  std::vector<cml::WlDesc> d;
  for (const Tensor& w : ws) {
    TORCH_CHECK(w.is_cuda() && w.device() == ws[0].device() && w.scalar_type() == at::kBFloat16 &&
                    w.dim() == 4 && w.size(2) == w.size(3) && (w.size(2) == 3 || w.size(2) == 1),
                "conv_wlayouts_multi: bf16 [Co, Ci, 3, 3] or [Co, Ci, 1, 1] weights on one device");
    const int64_t Co = w.size(0), Ci = w.size(1), T = w.size(2) * w.size(3);
    Tensor wr = at::empty({Ci, T * Co}, w.options().memory_format(at::MemoryFormat::Contiguous));
    Tensor wf;
    if (T == 9) wf = at::empty({Co, 9 * Ci}, w.options().memory_format(at::MemoryFormat::Contiguous));
    d.push_back(cml::WlDesc{w.data_ptr(), T == 9 ? wf.data_ptr() : nullptr, wr.data_ptr(),
                            w.stride(0), w.stride(1), w.stride(2), w.stride(3),
                            static_cast<int>(Co), static_cast<int>(Ci), static_cast<int>(T)});
    out.push_back({wf, wr});
  }
  CML_CHECK_HIP(cml::launch_conv3x3_wlayouts_multi(d.data(), static_cast<int>(d.size()),
                                                   cur_stream()));
  return out;
}

// {w_cat bf16 [Co, k1 + k2] = [diag(s1) w1 | diag(s2) w2], bias fp32 [Co] = b1 + b2} in one
// launch (bit-identical to two torch.mul into the halves and one add).
std::vector<Tensor> scaled_cat_bias(const Tensor& w1, const Tensor& s1, const Tensor& w2,
                                    const Tensor& s2, const Tensor& b1, const Tensor& b2) {
  TORCH_CHECK(w1.is_cuda() && w2.device() == w1.device() && w1.scalar_type() == at::kBFloat16 &&
                  w2.scalar_type() == at::kBFloat16 && w1.dim() == 2 && w2.dim() == 2 &&
                  w1.is_contiguous() && w2.is_contiguous() && w1.size(0) == w2.size(0) &&
                  w1.size(1) % 8 == 0 && w2.size(1) % 8 == 0,
              "scaled_cat_bias: contiguous bf16 [Co, k1], [Co, k2] on one device, k % 8 == 0");
  const int64_t Co = w1.size(0), k1 = w1.size(1), k2 = w2.size(1);
  const c10::DeviceGuard guard(w1.device());
  Tensor out = at::empty({Co, k1 + k2}, w1.options());
  Tensor bias = at::empty({Co}, w1.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_scaled_cat_bias(
      w1.data_ptr(), opt_ptr<const float>(s1, at::kFloat, "s1", Co), static_cast<int>(k1),
      w2.data_ptr(), opt_ptr<const float>(s2, at::kFloat, "s2", Co), static_cast<int>(k2),
      opt_ptr<const float>(b1, at::kFloat, "b1", Co), opt_ptr<const float>(b2, at::kFloat, "b2", Co),
      static_cast<int>(Co), out.data_ptr(), bias.data_ptr<float>(), cur_stream()));
  return {out, bias};
}

std::vector<Tensor> conv_gemm_bnsums(const Tensor& x, const Tensor& w, int64_t taps,
                                     const Tensor& zero, const Tensor& z, const Tensor& sc,
                                     const Tensor& bi, const Tensor& mean, const Tensor& invstd,
                                     const optional<Tensor>& dgamma_out,
                                     const optional<Tensor>& dbeta_out) {
  check_nhwc(x, "x");
  check_nhwc(z, "z");
  TORCH_CHECK(x.dim() == 4, "conv_gemm_bnsums: 4-D NHWC input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(taps == 1 || taps == 9, "conv_gemm_bnsums: taps 1 or 9");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 &&
                  w.size(1) == taps * C && w.size(0) % 64 == 0 && C % 64 == 0,
              "conv_gemm_bnsums: w must be contiguous bf16 [Cout, taps * C], channels multiples of 64");
  const int64_t Co = w.size(0), M = N * H * W;
  TORCH_CHECK(z.dim() == 4 && z.size(0) == N && z.size(1) == Co && z.size(2) == H && z.size(3) == W,
              "conv_gemm_bnsums: z must be [N, Cout, H, W]");
  TORCH_CHECK(zero.is_cuda() && zero.device() == x.device() && zero.scalar_type() == at::kBFloat16 &&
                  zero.is_contiguous() && zero.numel() >= 64, "conv_gemm_bnsums: zero must be >= 64 bf16");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor y = at::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor part = at::empty({static_cast<int64_t>(cml::conv_gemm_part_floats(M, static_cast<int>(Co)))}, f32);
  Tensor sdz = at::empty({Co}, f32), sdzx = at::empty({Co}, f32);
  // optional: the BN's parameter gradients bf16(sdzx) / bf16(sdz) from the same finalize launch
  const auto [dg, db] = dgb_ptrs(dgamma_out, dbeta_out, Co, x, "conv_gemm_bnsums");
  CML_CHECK_HIP(cml::launch_conv_gemm_bnsums(
      x.data_ptr(), w.data_ptr(), y.data_ptr(), zero.data_ptr(), static_cast<int>(N),
      static_cast<int>(H), static_cast<int>(W), static_cast<int>(C), static_cast<int>(Co),
      static_cast<int>(taps), z.data_ptr(), opt_ptr<const float>(sc, at::kFloat, "sc", Co),
      opt_ptr<const float>(bi, at::kFloat, "bi", Co),
      opt_ptr<const float>(mean, at::kFloat, "mean", Co),
      opt_ptr<const float>(invstd, at::kFloat, "invstd", Co), part.data_ptr<float>(),
      sdz.data_ptr<float>(), sdzx.data_ptr<float>(), cur_stream(), dg, db));
  return {y, sdz, sdzx};
}

// Data gradient of a stride-2 / padding-1 3x3 conv with an even [2 Ho, 2 Wo] input: dy [N, Co, Ho,
// Wo] NHWC bf16, wr [Ci, 9 Co] (conv3x3_wlayouts) -> {dx [N, Ci, 2 Ho, 2 Wo] NHWC, sdz, sdzx}; with
// z (+ sc, bi, mean, invstd as conv_gemm_bnsums) the BN + ReLU backward sums dx feeds, else
// sdz / sdzx are undefined.
std::vector<Tensor> conv_gemm_s2dgrad(const Tensor& dy, const Tensor& wr, const Tensor& zero,
                                      const optional<Tensor>& z, const optional<Tensor>& sc,
                                      const optional<Tensor>& bi, const optional<Tensor>& mean,
                                      const optional<Tensor>& invstd,
                                      const optional<Tensor>& dgamma_out,
                                      const optional<Tensor>& dbeta_out) {
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.dim() == 4, "conv_gemm_s2dgrad: 4-D NHWC dy");
  const int64_t N = dy.size(0), Co = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(wr.is_cuda() && wr.scalar_type() == at::kBFloat16 && wr.is_contiguous() &&
                  wr.dim() == 2 && wr.size(1) == 9 * Co && wr.size(0) % 64 == 0 && Co % 64 == 0,
              "conv_gemm_s2dgrad: wr must be contiguous bf16 [Ci, 9 Co], channels multiples of 64");
  TORCH_CHECK(zero.is_cuda() && zero.device() == dy.device() && zero.scalar_type() == at::kBFloat16 &&
                  zero.is_contiguous() && zero.numel() >= 64, "conv_gemm_s2dgrad: zero must be >= 64 bf16");
  const int64_t Ci = wr.size(0);
  const bool sums = z.has_value() && z->defined();
  if (sums) {
    check_nhwc(*z, "z");
    TORCH_CHECK(z->dim() == 4 && z->size(0) == N && z->size(1) == Ci && z->size(2) == 2 * Ho &&
                    z->size(3) == 2 * Wo, "conv_gemm_s2dgrad: z must be [N, Ci, 2 Ho, 2 Wo]");
  }
  const c10::DeviceGuard guard(dy.device());
  auto f32 = dy.options().dtype(at::kFloat);
  Tensor dx = at::empty({N, Ci, 2 * Ho, 2 * Wo},
                        dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor part, sdz, sdzx;
  if (sums) {
    part = at::empty({static_cast<int64_t>(cml::conv_gemm_s2dgrad_part_floats(N * Ho * Wo,
                                                                              static_cast<int>(Ci)))}, f32);
    sdz = at::empty({Ci}, f32);
    sdzx = at::empty({Ci}, f32);
  }
  const auto [dg, db] = dgb_ptrs(dgamma_out, dbeta_out, Ci, dy, "conv_gemm_s2dgrad");
  TORCH_CHECK(sums || dg == nullptr, "conv_gemm_s2dgrad: dgamma_out needs z");
  CML_CHECK_HIP(cml::launch_conv_gemm_s2dgrad(
      dy.data_ptr(), wr.data_ptr(), dx.data_ptr(), zero.data_ptr(), static_cast<int>(N),
      static_cast<int>(Ho), static_cast<int>(Wo), static_cast<int>(Co), static_cast<int>(Ci),
      sums ? z->data_ptr() : nullptr,
      sums ? opt_ptr<const float>(sc, at::kFloat, "sc", Ci) : nullptr,
      sums ? opt_ptr<const float>(bi, at::kFloat, "bi", Ci) : nullptr,
      sums ? opt_ptr<const float>(mean, at::kFloat, "mean", Ci) : nullptr,
      sums ? opt_ptr<const float>(invstd, at::kFloat, "invstd", Ci) : nullptr,
      sums ? part.data_ptr<float>() : nullptr, sums ? sdz.data_ptr<float>() : nullptr,
      sums ? sdzx.data_ptr<float>() : nullptr, cur_stream(), dg, db));
  return {dx, sdz, sdzx};
}

Tensor conv_gemm(const Tensor& x, const Tensor& w, int64_t taps, const optional<Tensor>& zero_in,
                 int64_t stride) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "conv_gemm: 4-D NHWC input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(taps == 1 || taps == 9, "conv_gemm: taps 1 or 9");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 &&
                  w.size(1) == taps * C && w.size(0) % 64 == 0 && C % 64 == 0,
              "conv_gemm: w must be contiguous bf16 [Cout, taps * C], channels multiples of 64");
  TORCH_CHECK(stride == 1 || stride == 2, "conv_gemm: stride 1 or 2");
  const int64_t Co = w.size(0);
  const c10::DeviceGuard guard(x.device());
  Tensor y = at::empty({N, Co, (H - 1) / stride + 1, (W - 1) / stride + 1},
                       x.options().memory_format(at::MemoryFormat::ChannelsLast));
  // zero row for padded taps: pass a cached >= 64-element zero bf16 tensor to skip the per-call fill
  Tensor zero;
  if (zero_in.has_value() && zero_in->defined()) {
    zero = *zero_in;
    TORCH_CHECK(zero.is_cuda() && zero.device() == x.device() && zero.scalar_type() == at::kBFloat16 &&
                    zero.is_contiguous() && zero.numel() >= 64, "conv_gemm: zero must be >= 64 bf16");
  } else {
    zero = at::zeros({64}, x.options());
  }
  CML_CHECK_HIP(cml::launch_conv_gemm(x.data_ptr(), w.data_ptr(), y.data_ptr(), zero.data_ptr(),
                                      static_cast<int>(N), static_cast<int>(H), static_cast<int>(W),
                                      static_cast<int>(C), static_cast<int>(Co),
                                      static_cast<int>(taps), cur_stream(), nullptr, nullptr,
                                      nullptr, nullptr, nullptr, nullptr, 1e-5f, 0.1f,
                                      static_cast<int>(stride)));
  return y;
}

// conv_gemm + the training BatchNorm statistics of its bf16 output (shifted by `shift`, e.g. the
// running mean) in the epilogue -> {y, mean, invstd}; running stats updated in place when given.
std::vector<Tensor> conv_gemm_bn(const Tensor& x, const Tensor& w, int64_t taps,
                                 const optional<Tensor>& zero_in, const optional<Tensor>& shift,
                                 const optional<Tensor>& rmean, const optional<Tensor>& rvar,
                                 double eps, double momentum, int64_t stride,
                                 const optional<Tensor>& gamma, const optional<Tensor>& beta) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "conv_gemm_bn: 4-D NHWC input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(taps == 1 || taps == 9, "conv_gemm_bn: taps 1 or 9");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 &&
                  w.size(1) == taps * C && w.size(0) % 64 == 0 && C % 64 == 0,
              "conv_gemm_bn: w must be contiguous bf16 [Cout, taps * C], channels multiples of 64");
  TORCH_CHECK(stride == 1 || stride == 2, "conv_gemm_bn: stride 1 or 2");
  const int64_t OH = (H - 1) / stride + 1, OW = (W - 1) / stride + 1;
  const int64_t Co = w.size(0), M = N * OH * OW;
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor y = at::empty({N, Co, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor zero;
  if (zero_in.has_value() && zero_in->defined()) {
    zero = *zero_in;
    TORCH_CHECK(zero.is_cuda() && zero.device() == x.device() && zero.scalar_type() == at::kBFloat16 &&
                    zero.is_contiguous() && zero.numel() >= 64, "conv_gemm_bn: zero must be >= 64 bf16");
  } else {
    zero = at::zeros({64}, x.options());
  }
  Tensor mean = at::empty({Co}, f32), invstd = at::empty({Co}, f32);
  Tensor part = at::empty({static_cast<int64_t>(cml::conv_gemm_part_floats(M, static_cast<int>(Co)))}, f32);
  Tensor asc, abi;
  cml::BnAffineOut ao{};
  const cml::BnAffineOut* aff = aff_out(gamma, beta, Co, x, "conv_gemm_bn", asc, abi, ao);
  CML_CHECK_HIP(cml::launch_conv_gemm(
      x.data_ptr(), w.data_ptr(), y.data_ptr(), zero.data_ptr(), static_cast<int>(N),
      static_cast<int>(H), static_cast<int>(W), static_cast<int>(C), static_cast<int>(Co),
      static_cast<int>(taps), cur_stream(), part.data_ptr<float>(),
      opt_ptr<const float>(shift, at::kFloat, "shift", Co), mean.data_ptr<float>(),
      invstd.data_ptr<float>(), opt_ptr<float>(rmean, at::kFloat, "running_mean", Co),
      opt_ptr<float>(rvar, at::kFloat, "running_var", Co), static_cast<float>(eps),
      static_cast<float>(momentum), static_cast<int>(stride), aff));
  if (aff) return {y, mean, invstd, asc, abi};
  return {y, mean, invstd};
}

// BatchNorm training statistics only: x NHWC bf16 -> {mean, invstd} (fp32 [C]); running stats
// updated in place when given.
std::vector<Tensor> bn_stats(const Tensor& x, const optional<Tensor>& rmean,
                             const optional<Tensor>& rvar, double eps, double momentum) {
  check_nhwc(x, "x");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn: C must be 8 * (power of 2) <= 2048");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({C}, f32), invstd = at::empty({C}, f32);
  Tensor work = at::empty({static_cast<int64_t>(cml::bn_workspace_bytes(M, static_cast<int>(C)) / 4 + 1)}, f32);
  CML_CHECK_HIP(cml::launch_bn_stats(x.data_ptr(), M, static_cast<int>(C), mean.data_ptr<float>(),
                                     invstd.data_ptr<float>(),
                                     opt_ptr<float>(rmean, at::kFloat, "running_mean", C),
                                     opt_ptr<float>(rvar, at::kFloat, "running_var", C),
                                     static_cast<float>(eps), static_cast<float>(momentum),
                                     work.data_ptr(), cur_stream()));
  return {mean, invstd};
}

// 3x3/s2/p1 max-pool backward + per-channel sums of the result: {dx, sums fp32 [C]}. dy2: an
// optional second output gradient of dy's shape, summed on load.
std::vector<Tensor> maxpool_bwd_sum(const Tensor& dy_in, const Tensor& idx, int64_t H, int64_t W,
                                    const optional<Tensor>& dy2_in) {
  Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dy, "dy");
  Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = dy2_in->contiguous(at::MemoryFormat::ChannelsLast);
    check_nhwc(dy2, "dy2");
    TORCH_CHECK(dy2.sizes() == dy.sizes() && dy2.device() == dy.device(), "maxpool_bwd_sum: dy2");
  }
  const int64_t N = dy.size(0), C = dy.size(1), OH = dy.size(2), OW = dy.size(3);
  TORCH_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1, "maxpool_bwd_sum: 3x3/s2/p1 shapes");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.numel() == dy.numel(), "maxpool_bwd_sum: idx");
  const c10::DeviceGuard guard(dy.device());
  Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor sums = at::empty({C}, dy.options().dtype(at::kFloat));
  const size_t wb = cml::maxpool_bwd_sum_workspace_bytes(N, H, W, C);
  Tensor work = at::empty({static_cast<int64_t>(wb / 4 + 1)}, dy.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_maxpool_bwd_sum(dy.data_ptr(),
                                            dy2.defined() ? dy2.data_ptr() : nullptr,
                                            idx.data_ptr(), dx.data_ptr(),
                                            sums.data_ptr<float>(), work.data_ptr(), N, H, W, C,
                                            OH, OW, cur_stream()));
  return {dx, sums};
}

// dsts[i].copy_(srcs[i]) for same-dtype, same-numel contiguous 16-B aligned tensors, in launches of
// up to kMaxCopy entries. Returns the indices that did not qualify (the caller copies those).
std::vector<int64_t> multi_copy(const std::vector<Tensor>& dsts, const std::vector<Tensor>& srcs) {
  TORCH_CHECK(dsts.size() == srcs.size(), "multi_copy: list length mismatch");
  std::vector<int64_t> rest;
  cml::MultiCopyArgs a{};
  int64_t nv = 0;
  auto flush = [&]() {
    if (a.n == 0) return;
    a.vpre[a.n] = nv;
    CML_CHECK_HIP(cml::launch_multi_copy(a, cur_stream()));
    a = cml::MultiCopyArgs{};
    nv = 0;
  };
  c10::optional<c10::DeviceGuard> guard;
  for (size_t i = 0; i < dsts.size(); ++i) {
    const Tensor& d = dsts[i];
    const Tensor& s = srcs[i];
    // both contiguous, or both dense with identical sizes and strides (channels_last conv
    // weights and their gradients): either way the bytes are in the same order, starting at
    // data_ptr (positive strides)
    const bool same_dense = d.sizes() == s.sizes() && d.strides() == s.strides() &&
                            d.is_non_overlapping_and_dense();
    const bool ok = d.is_cuda() && s.is_cuda() && d.device() == s.device() &&
                    d.scalar_type() == s.scalar_type() && d.numel() == s.numel() &&
                    ((d.is_contiguous() && s.is_contiguous()) || same_dense) &&
                    d.element_size() % 2 == 0 &&
                    (reinterpret_cast<uintptr_t>(d.data_ptr()) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(s.data_ptr()) & 15) == 0;
    if (!ok) {
      rest.push_back(static_cast<int64_t>(i));
      continue;
    }
    if (!guard) guard.emplace(d.device());
    const int64_t bytes = d.numel() * d.element_size();
    a.src[a.n] = s.data_ptr();
    a.dst[a.n] = d.data_ptr();
    a.bytes[a.n] = bytes;
    a.vpre[a.n] = nv;
    nv += bytes / 16;
    if (++a.n == cml::kMaxCopy) flush();
  }
  flush();
  return rest;
}

// x [N, C, H, W] channels_last bf16, C <= 4 -> [N, 4, H, W] channels_last, zero channels C..3
Tensor pad_c4(const Tensor& x) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(1) >= 1 && x.size(1) <= 4, "pad_c4: 4-D NHWC with C <= 4");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const c10::DeviceGuard guard(x.device());
  Tensor y = at::empty({N, 4, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  CML_CHECK_HIP(cml::launch_pad_c4(x.data_ptr(), y.data_ptr(), N * H * W, static_cast<int>(C),
                                   cur_stream()));
  return y;
}

void fault(Tensor& g, int64_t kind, double scale, double sigma, int64_t seed) {
  check_dev(g, "g");
  TORCH_CHECK(g.is_contiguous(), "g must be contiguous");
  const c10::DeviceGuard guard(g.device());
  CML_CHECK_HIP(cml::launch_fault(dtype_of(g), g.data_ptr(), g.numel(), static_cast<int>(kind),
                                  static_cast<float>(scale), static_cast<float>(sigma),
                                  static_cast<uint64_t>(seed), cur_stream()));
}

// ---------------------------------------------------------------- transformer ops
void check_bf16c(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name, " must be 16-B aligned");
}

// logits [R, V] bf16 contiguous, labels [R] int64 -> (lse fp32 [R], loss fp32 [R])
// logits [R, V] with unit column stride; rows contiguous (ld = V) or row-strided (ld % 8 == 0,
// a padded logits buffer)
int64_t ce_row_stride(const Tensor& logits) {
  check_dev(logits, "logits");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16, "logits must be bf16");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [R, V] with unit column stride");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(logits.data_ptr()) & 15) == 0, "logits must be 16-B aligned");
  const int64_t V = logits.size(1), ld = logits.stride(0);
  TORCH_CHECK(ld == V || (ld >= V && ld % 8 == 0) || logits.size(0) == 1,
              "logits rows must be contiguous or 16-B aligned (row stride % 8 == 0)");
  return logits.size(0) == 1 ? V : ld;
}

std::vector<Tensor> ce_fwd(const Tensor& logits, const Tensor& labels, int64_t ignore) {
  const int64_t ld = ce_row_stride(logits);
  const int64_t R = logits.size(0), V = logits.size(1);
  TORCH_CHECK(R >= 1 && R <= 2147483647LL && V >= 1 && V <= 2147483647LL, "bad logits shape");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                  labels.numel() == R, "labels: contiguous int64 [R] on the GPU");
  const c10::DeviceGuard guard(logits.device());
  auto f32 = logits.options().dtype(at::kFloat);
  Tensor lse = at::empty({R}, f32), loss = at::empty({R}, f32);
  CML_CHECK_HIP(cml::launch_ce_fwd(logits.data_ptr(), R, static_cast<int>(V), ld,
                                   labels.data_ptr<int64_t>(), ignore, lse.data_ptr<float>(),
                                   loss.data_ptr<float>(), cur_stream()));
  return {lse, loss};
}

// Fused backward over row-strided logits (ld % 8 == 0, R % 64 == 0): (grad [R, V] view of an
// [R, ld] buffer, part [R / 64, ld] fp32 column sums per 64-row block) -- ce_part_fold turns part
// into the logits bias gradient.
std::vector<Tensor> ce_bwd_cs(const Tensor& logits, const Tensor& labels, const Tensor& lse,
                              const Tensor& scale, int64_t ignore, const optional<Tensor>& div) {
  const int64_t ld = ce_row_stride(logits);
  const int64_t R = logits.size(0), V = logits.size(1);
  TORCH_CHECK(ld % 8 == 0 && R % 64 == 0, "ce_bwd_cs: needs a row stride % 8 == 0 and R % 64 == 0");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.numel() == R &&
                  labels.is_contiguous(), "labels: contiguous int64 [R]");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.numel() == R &&
                  lse.is_contiguous(), "lse: fp32 [R]");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() >= 1,
              "scale: fp32 GPU scalar");
  const c10::DeviceGuard guard(logits.device());
  Tensor gbuf = at::empty({R, ld}, logits.options());
  Tensor part = at::empty({R / 64, ld}, logits.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_ce_bwd_cs(logits.data_ptr(), R, static_cast<int>(V), ld,
                                      labels.data_ptr<int64_t>(), ignore, lse.data_ptr<float>(),
                                      scale.data_ptr<float>(), gbuf.data_ptr(),
                                      part.data_ptr<float>(), cur_stream(),
                                      opt_ptr<const float>(div, at::kFloat, "div", 1)));
  return {gbuf.narrow(1, 0, V), part};
}

// w.t().contiguous() for bf16 [R, C] with R, C multiples of 64 (LDS-tiled kernel); other inputs
// fall back to ATen
Tensor transpose_bf16(const Tensor& w) {
  check_dev(w, "w");
  TORCH_CHECK(w.dim() == 2, "transpose_bf16: 2-D");
  const int64_t R = w.size(0), C = w.size(1);
  if (w.scalar_type() != at::kBFloat16 || w.stride(1) != 1 || R % 64 || C % 64 || w.stride(0) % 8 ||
      (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15))
    return w.t().contiguous();
  const c10::DeviceGuard guard(w.device());
  Tensor out = at::empty({C, R}, w.options());
  CML_CHECK_HIP(cml::launch_transpose_bf16(w.data_ptr(), out.data_ptr(), static_cast<int>(R),
                                           static_cast<int>(C), w.stride(0), R, cur_stream()));
  return out;
}

Tensor gelu_bwd(const Tensor& da, const Tensor& h) {
  check_bf16c(da, "da");
  check_bf16c(h, "h");
  TORCH_CHECK(da.numel() == h.numel() && da.numel() % 8 == 0, "gelu_bwd: same size, % 8 == 0");
  const c10::DeviceGuard guard(da.device());
  Tensor dh = at::empty_like(h);
  CML_CHECK_HIP(cml::launch_gelu_bwd(da.data_ptr(), h.data_ptr(), dh.data_ptr(), da.numel(),
                                     cur_stream()));
  return dh;
}

// out [nseg, V] (bf16 or fp32, unit column stride) = per-segment sums of ce_bwd_cs's partials
void ce_part_fold(const Tensor& part, int64_t V, int64_t nseg, Tensor& out) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 2 &&
                  part.is_contiguous(), "part: fp32 [R / 64, ld]");
  TORCH_CHECK(out.is_cuda() && (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat) &&
                  out.dim() == 2 && out.size(0) == nseg && out.size(1) == V && out.stride(1) == 1,
              "out must be [nseg, V] bf16 / fp32");
  const c10::DeviceGuard guard(part.device());
  CML_CHECK_HIP(cml::launch_ce_part_fold(part.data_ptr<float>(), part.size(0) * 64,
                                         static_cast<int>(V), part.size(1), static_cast<int>(nseg),
                                         out.data_ptr(), out.stride(0),
                                         out.scalar_type() == at::kFloat ? 1 : 0, cur_stream()));
}

Tensor ce_bwd(const Tensor& logits, const Tensor& labels, const Tensor& lse, const Tensor& scale,
              int64_t ignore, const optional<Tensor>& div) {
  check_bf16c(logits, "logits");
  const int64_t R = logits.size(0), V = logits.size(1);
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.numel() == R &&
                  labels.is_contiguous(), "labels: contiguous int64 [R]");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.numel() == R &&
                  lse.is_contiguous(), "lse: fp32 [R]");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() >= 1,
              "scale: fp32 GPU scalar");
  const c10::DeviceGuard guard(logits.device());
  Tensor g = at::empty_like(logits);
  CML_CHECK_HIP(cml::launch_ce_bwd(logits.data_ptr(), R, static_cast<int>(V),
                                   labels.data_ptr<int64_t>(), ignore, lse.data_ptr<float>(),
                                   scale.data_ptr<float>(), g.data_ptr(), cur_stream(),
                                   opt_ptr<const float>(div, at::kFloat, "div", 1)));
  return g;
}

// {mean loss (0-dim), n_valid [1]} fp32 from ce_fwd's per-row losses in one launch (fixed-order
// fp64 sums; n_valid = max(#labels != ignore, 1)).
std::vector<Tensor> ce_mean(const Tensor& loss, const Tensor& labels, int64_t ignore) {
  TORCH_CHECK(loss.is_cuda() && loss.scalar_type() == at::kFloat && loss.is_contiguous() &&
                  labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                  labels.numel() == loss.numel() && loss.numel() >= 1,
              "ce_mean: contiguous fp32 loss [R] and int64 labels [R] on the GPU");
  const c10::DeviceGuard guard(loss.device());
  Tensor out = at::empty({}, loss.options()), count = at::empty({1}, loss.options());
  CML_CHECK_HIP(cml::launch_ce_mean(loss.data_ptr<float>(), labels.data_ptr<int64_t>(),
                                    loss.numel(), ignore, out.data_ptr<float>(),
                                    count.data_ptr<float>(), cur_stream()));
  return {out, count};
}

// x (and res) [.., D] bf16 contiguous; w (and b) [D] bf16. Returns (y, sum|undef, mean|undef, rstd).
std::vector<Tensor> norm_fwd(const Tensor& x, const optional<Tensor>& res, const Tensor& w,
                             const optional<Tensor>& b, double eps) {
  check_bf16c(x, "x");
  const int64_t D = x.size(-1);
  const int64_t M = x.numel() / D;
  check_bf16c(w, "w");
  TORCH_CHECK(w.numel() == D, "w must be [D]");
  const bool ln = b.has_value() && b->defined();
  if (ln) {
    check_bf16c(*b, "b");
    TORCH_CHECK(b->numel() == D, "b must be [D]");
  }
  const bool has_res = res.has_value() && res->defined();
  if (has_res) {
    check_bf16c(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "res shape mismatch");
  }
  TORCH_CHECK(D % 8 == 0 && D <= 4096, "norm: D % 8 == 0 and D <= 4096");
  const c10::DeviceGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor y = at::empty_like(x);
  Tensor sum = has_res ? at::empty_like(x) : Tensor();
  Tensor mean = ln ? at::empty({M}, f32) : Tensor();
  Tensor rstd = at::empty({M}, f32);
  CML_CHECK_HIP(cml::launch_norm_fwd(ln ? 1 : 0, x.data_ptr(), has_res ? res->data_ptr() : nullptr,
                                     w.data_ptr(), ln ? b->data_ptr() : nullptr, y.data_ptr(),
                                     has_res ? sum.data_ptr() : nullptr,
                                     ln ? mean.data_ptr<float>() : nullptr, rstd.data_ptr<float>(),
                                     M, static_cast<int>(D), static_cast<float>(eps),
                                     cur_stream()));
  return {y, sum, mean, rstd};
}

// Returns (dx, dw, db|undef). dres (optional) is added to dx.
std::vector<Tensor> norm_bwd(const Tensor& dy_in, const optional<Tensor>& dres_in, const Tensor& x,
                             const Tensor& w, const optional<Tensor>& mean, const Tensor& rstd) {
  check_bf16c(x, "x");
  const int64_t D = x.size(-1);
  const int64_t M = x.numel() / D;
  Tensor dy = dy_in.contiguous();
  check_bf16c(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy shape mismatch");
  Tensor dres;
  if (dres_in.has_value() && dres_in->defined()) {
    dres = dres_in->contiguous();
    check_bf16c(dres, "dres");
    TORCH_CHECK(dres.sizes() == x.sizes(), "dres shape mismatch");
  }
  check_bf16c(w, "w");
  const bool ln = mean.has_value() && mean->defined();
  TORCH_CHECK(rstd.is_cuda() && rstd.scalar_type() == at::kFloat && rstd.numel() == M, "rstd: fp32 [M]");
  if (ln) TORCH_CHECK(mean->scalar_type() == at::kFloat && mean->numel() == M, "mean: fp32 [M]");
  TORCH_CHECK(D % 8 == 0 && D <= 4096, "norm: D % 8 == 0 and D <= 4096");
  const c10::DeviceGuard guard(x.device());
  Tensor dx = at::empty_like(x);
  Tensor dw = at::empty_like(w);
  Tensor db = ln ? at::empty_like(w) : Tensor();
  Tensor work = at::empty({static_cast<int64_t>(cml::norm_workspace_bytes(M, static_cast<int>(D)) / 4 + 1)},
                          x.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_norm_bwd(ln ? 1 : 0, dy.data_ptr(), dres.defined() ? dres.data_ptr() : nullptr,
                                     x.data_ptr(), w.data_ptr(), ln ? mean->data_ptr<float>() : nullptr,
                                     rstd.data_ptr<float>(), dx.data_ptr(), dw.data_ptr(),
                                     ln ? db.data_ptr() : nullptr, M, static_cast<int>(D),
                                     work.data_ptr(), cur_stream()));
  return {dx, dw, db};
}

void check_rope_tables(const optional<Tensor>& c, const optional<Tensor>& s, int64_t S, int64_t hd) {
  if (!(c.has_value() && c->defined())) return;
  TORCH_CHECK(s.has_value() && s->defined(), "rope: cos without sin");
  for (const Tensor* t : {&*c, &*s}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                    t->numel() >= S * (hd / 2), "rope tables: contiguous fp32 [S, hd/2]");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "rope tables must be 16-B aligned");
  }
}

std::vector<Tensor> rope_fwd(const Tensor& qkv, const optional<Tensor>& cosb,
                             const optional<Tensor>& sinb, int64_t H, int64_t KV, int64_t hd) {
  check_bf16c(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == (H + 2 * KV) * hd && hd % 8 == 0,
              "qkv must be [B, S, (H + 2 KV) hd] with hd % 8 == 0");
  const int64_t B = qkv.size(0), S = qkv.size(1);
  check_rope_tables(cosb, sinb, S, hd);
  const c10::DeviceGuard guard(qkv.device());
  Tensor q = at::empty({B, H, S, hd}, qkv.options());
  Tensor k = at::empty({B, KV, S, hd}, qkv.options());
  Tensor v = at::empty({B, KV, S, hd}, qkv.options());
  const bool rot = cosb.has_value() && cosb->defined();
  CML_CHECK_HIP(cml::launch_rope_fwd(qkv.data_ptr(), rot ? cosb->data_ptr<float>() : nullptr,
                                     rot ? sinb->data_ptr<float>() : nullptr, q.data_ptr(),
                                     k.data_ptr(), v.data_ptr(), B, S, H, KV, hd, cur_stream()));
  return {q, k, v};
}

Tensor rope_bwd(const Tensor& dq_in, const Tensor& dk_in, const Tensor& dv_in,
                const optional<Tensor>& cosb, const optional<Tensor>& sinb, int64_t grp) {
  Tensor dq = dq_in.contiguous(), dk = dk_in.contiguous(), dv = dv_in.contiguous();
  check_bf16c(dq, "dq");
  check_bf16c(dk, "dk");
  check_bf16c(dv, "dv");
  TORCH_CHECK(dq.dim() == 4 && dk.dim() == 4 && dk.sizes() == dv.sizes() &&
                  dq.size(0) == dk.size(0) && dq.size(2) == dk.size(2) && dq.size(3) == dk.size(3),
              "dq [B, H, S, hd], dk / dv [B, KV grp, S, hd]");
  TORCH_CHECK(grp >= 1 && dk.size(1) % grp == 0, "rope_bwd: dk heads must be a multiple of grp");
  const int64_t B = dq.size(0), H = dq.size(1), S = dq.size(2), hd = dq.size(3),
                KV = dk.size(1) / grp;
  TORCH_CHECK(hd % 8 == 0, "hd % 8 == 0");
  check_rope_tables(cosb, sinb, S, hd);
  const c10::DeviceGuard guard(dq.device());
  Tensor dqkv = at::empty({B, S, (H + 2 * KV) * hd}, dq.options());
  const bool rot = cosb.has_value() && cosb->defined();
  CML_CHECK_HIP(cml::launch_rope_bwd(dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                                     rot ? cosb->data_ptr<float>() : nullptr,
                                     rot ? sinb->data_ptr<float>() : nullptr, dqkv.data_ptr(), B,
                                     S, H, KV, hd, cur_stream(), static_cast<int>(grp)));
  return dqkv;
}

// Flash attention (csrc/kernels/flash_attn.hip): q [B, H, S, 128], k / v [B, KV, S, 128] bf16
// contiguous -> (o [B, S, H * 128], lse fp32 [B, H, S])
void check_flash_qkv(const Tensor& q, const Tensor& k, const Tensor& v) {
  check_bf16c(q, "q");
  check_bf16c(k, "k");
  check_bf16c(v, "v");
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && k.sizes() == v.sizes() && q.size(0) == k.size(0) &&
                  q.size(2) == k.size(2) && q.size(3) == 128 && k.size(3) == 128,
              "flash: q [B, H, S, 128], k / v [B, KV, S, 128]");
  TORCH_CHECK(q.size(1) % k.size(1) == 0, "flash: H % KV == 0");
  TORCH_CHECK(q.get_device() == k.get_device() && q.get_device() == v.get_device(),
              "flash: q / k / v on one device");
  for (const Tensor* t : {&q, &k, &v})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "flash: 16-B aligned q / k / v");
}

std::vector<Tensor> flash_fwd(const Tensor& q, const Tensor& k, const Tensor& v, bool causal,
                              double scale, double rescale_thr) {
  check_flash_qkv(q, k, v);
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), KV = k.size(1);
  const c10::DeviceGuard guard(q.device());
  Tensor o = at::empty({B, S, H * 128}, q.options());
  Tensor lse = at::empty({B, H, S}, q.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                      lse.data_ptr<float>(), static_cast<int>(B), static_cast<int>(H),
                                      static_cast<int>(KV), static_cast<int>(S),
                                      static_cast<float>(scale), causal, cur_stream(),
                                      static_cast<float>(rescale_thr)));
  return {o, lse};
}

// -> (dq [B, H, S, 128], dk / dv per query head [B, H, S, 128])
std::vector<Tensor> flash_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                              const Tensor& dout_in, const Tensor& lse, bool causal, double scale) {
  check_flash_qkv(q, k, v);
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), KV = k.size(1);
  Tensor dout = dout_in.contiguous();
  check_bf16c(o, "o");
  check_bf16c(dout, "dout");
  TORCH_CHECK(o.numel() == B * S * H * 128 && dout.numel() == o.numel() && o.is_contiguous(),
              "flash_bwd: o / dout [B, S, H * 128]");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(o.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(dout.data_ptr()) & 15) == 0,
              "flash_bwd: 16-B aligned o / dout");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() &&
                  lse.numel() == B * H * S && lse.get_device() == q.get_device(),
              "flash_bwd: lse fp32 [B, H, S]");
  const c10::DeviceGuard guard(q.device());
  Tensor dq = at::empty_like(q);
  Tensor dk = at::empty({B, H, S, 128}, q.options());
  Tensor dv = at::empty({B, H, S, 128}, q.options());
  Tensor dsum = at::empty({B, H, S}, lse.options());
  CML_CHECK_HIP(cml::launch_flash_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                      dout.data_ptr(), lse.data_ptr<float>(), dsum.data_ptr<float>(),
                                      dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                                      static_cast<int>(B), static_cast<int>(H), static_cast<int>(KV),
                                      static_cast<int>(S), static_cast<float>(scale), causal,
                                      cur_stream()));
  return {dq, dk, dv};
}

Tensor swiglu_fwd(const Tensor& h) {
  check_bf16c(h, "h");
  const int64_t F2 = h.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "swiglu: last dim must be 2F with F % 8 == 0");
  const int64_t M = h.numel() / F2;
  const c10::DeviceGuard guard(h.device());
  auto sizes = h.sizes().vec();
  sizes.back() = F2 / 2;
  Tensor y = at::empty(sizes, h.options());
  CML_CHECK_HIP(cml::launch_swiglu_fwd(h.data_ptr(), y.data_ptr(), M, static_cast<int>(F2 / 2),
                                       cur_stream()));
  return y;
}

Tensor swiglu_bwd(const Tensor& dy_in, const Tensor& h) {
  check_bf16c(h, "h");
  Tensor dy = dy_in.contiguous();
  check_bf16c(dy, "dy");
  const int64_t F2 = h.size(-1);
  const int64_t M = h.numel() / F2;
  TORCH_CHECK(F2 % 16 == 0 && dy.numel() == M * (F2 / 2), "swiglu_bwd shape mismatch");
  const c10::DeviceGuard guard(h.device());
  Tensor dh = at::empty_like(h);
  CML_CHECK_HIP(cml::launch_swiglu_bwd(dy.data_ptr(), h.data_ptr(), dh.data_ptr(), M,
                                       static_cast<int>(F2 / 2), cur_stream()));
  return dh;
}

// qkv [B, S, 3 H 64] bf16 contiguous -> (O [B, S, H 64], lse fp32 [B, H, S])
std::vector<Tensor> attn_fwd(const Tensor& qkv, int64_t H, double scale) {
  check_bf16c(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == 3 * H * 64, "attn: qkv must be [B, S, 3 H 64]");
  const int64_t B = qkv.size(0), S = qkv.size(1);
  TORCH_CHECK(S % 32 == 0 && S >= 32 && S <= 128, "attn: S % 32 == 0 and S <= 128");
  const c10::DeviceGuard guard(qkv.device());
  Tensor out = at::empty({B, S, H * 64}, qkv.options());
  Tensor lse = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr<float>(),
                                     static_cast<int>(B), static_cast<int>(S), static_cast<int>(H),
                                     static_cast<float>(scale), cur_stream()));
  return {out, lse};
}

Tensor attn_bwd(const Tensor& qkv, const Tensor& out, const Tensor& dout_in, const Tensor& lse,
                int64_t H, double scale) {
  check_bf16c(qkv, "qkv");
  check_bf16c(out, "out");
  Tensor dout = dout_in.contiguous();
  check_bf16c(dout, "dout");
  const int64_t B = qkv.size(0), S = qkv.size(1);
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == 3 * H * 64 && S % 32 == 0 && S <= 128,
              "attn_bwd: qkv must be [B, S, 3 H 64], S % 32 == 0, S <= 128");
  TORCH_CHECK(out.sizes() == dout.sizes() && out.dim() == 3 && out.size(0) == B && out.size(1) == S &&
                  out.size(2) == H * 64, "attn_bwd: out / dout must be [B, S, H 64]");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() &&
                  lse.numel() == B * H * S, "attn_bwd: lse fp32 [B, H, S]");
  const c10::DeviceGuard guard(qkv.device());
  Tensor dqkv = at::empty_like(qkv);
  CML_CHECK_HIP(cml::launch_attn_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(),
                                     lse.data_ptr<float>(), dqkv.data_ptr(), static_cast<int>(B),
                                     static_cast<int>(S), static_cast<int>(H),
                                     static_cast<float>(scale), cur_stream()));
  return dqkv;
}

std::vector<Tensor> split_search(const Tensor& Xb, const Tensor& node_local, const Tensor& stat,
                                 const Tensor& feats, const Tensor& tot, int64_t n_bins,
                                 int64_t crit, double lam, double min_child) {
  check_dev(Xb, "Xb");
  TORCH_CHECK(Xb.scalar_type() == at::kByte && Xb.dim() == 2 && Xb.is_contiguous(), "Xb: uint8 [n, p]");
  const int64_t n = Xb.size(0), p = Xb.size(1);
  TORCH_CHECK(node_local.is_cuda() && node_local.scalar_type() == at::kInt && node_local.dim() == 2 &&
                  node_local.size(1) == n && node_local.is_contiguous(), "node_local: int32 [T, n]");
  const int64_t T = node_local.size(0);
  TORCH_CHECK(stat.is_cuda() && stat.scalar_type() == at::kFloat && stat.is_contiguous() &&
                  stat.numel() == T * n * 2, "stat: fp32 [T, n, 2]");
  TORCH_CHECK(feats.is_cuda() && feats.scalar_type() == at::kInt && feats.dim() == 3 &&
                  feats.size(0) == T && feats.is_contiguous(), "feats: int32 [T, L, kk]");
  const int64_t L = feats.size(1), kk = feats.size(2);
  TORCH_CHECK(tot.is_cuda() && tot.scalar_type() == at::kFloat && tot.is_contiguous() &&
                  tot.numel() == T * L * 2, "tot: fp32 [T, L, 2]");
  TORCH_CHECK(n_bins >= 2 && n_bins <= 64, "split_search: 2 <= n_bins <= 64");
  TORCH_CHECK(Xb.device() == stat.device() && Xb.device() == feats.device(), "device mismatch");
  const c10::DeviceGuard guard(Xb.device());
  Tensor gain = at::empty({T, L}, stat.options());
  Tensor slot = at::empty({T, L}, feats.options());
  Tensor bin = at::empty({T, L}, feats.options());
  CML_CHECK_HIP(cml::launch_split_search(Xb.data_ptr<uint8_t>(), node_local.data_ptr<int>(),
                                         stat.data_ptr<float>(), feats.data_ptr<int>(),
                                         tot.data_ptr<float>(), static_cast<int>(T),
                                         static_cast<int>(L), static_cast<int>(n),
                                         static_cast<int>(p), static_cast<int>(kk),
                                         static_cast<int>(n_bins), static_cast<int>(crit),
                                         static_cast<float>(lam), static_cast<float>(min_child),
                                         gain.data_ptr<float>(), slot.data_ptr<int>(),
                                         bin.data_ptr<int>(), cur_stream()));
  return {gain, slot, bin};
}

// split_search with in-kernel candidate sampling (kk distinct features per node from `seed`) and up
// to 128 bins: {gain [T, L], feature [T, L], bin [T, L]} (select/hist_trees.py ExactForest).
std::vector<Tensor> split_search_sampled(const Tensor& Xb, const Tensor& node_local,
                                         const Tensor& stat, const Tensor& tot, int64_t L,
                                         int64_t kk, int64_t n_bins, int64_t crit, double lam,
                                         double min_child, int64_t seed) {
  check_dev(Xb, "Xb");
  TORCH_CHECK(Xb.scalar_type() == at::kByte && Xb.dim() == 2 && Xb.is_contiguous(), "Xb: uint8 [n, p]");
  const int64_t n = Xb.size(0), p = Xb.size(1);
  TORCH_CHECK(node_local.is_cuda() && node_local.scalar_type() == at::kInt && node_local.dim() == 2 &&
                  node_local.size(1) == n && node_local.is_contiguous(), "node_local: int32 [T, n]");
  const int64_t T = node_local.size(0);
  TORCH_CHECK(stat.is_cuda() && stat.scalar_type() == at::kFloat && stat.is_contiguous() &&
                  stat.numel() == T * n * 2, "stat: fp32 [T, n, 2]");
  TORCH_CHECK(tot.is_cuda() && tot.scalar_type() == at::kFloat && tot.is_contiguous() &&
                  tot.numel() == T * L * 2, "tot: fp32 [T, L, 2]");
  TORCH_CHECK(n_bins >= 2 && n_bins <= 128 && kk >= 1 && kk <= 512 && kk <= p && p <= 65536,
              "split_search_sampled: 2 <= n_bins <= 128, 1 <= kk <= min(512, p), p <= 65536");
  const c10::DeviceGuard guard(Xb.device());
  Tensor gain = at::empty({T, L}, stat.options());
  Tensor feat = at::empty({T, L}, node_local.options());
  Tensor bin = at::empty({T, L}, node_local.options());
  CML_CHECK_HIP(cml::launch_split_search_sampled(
      Xb.data_ptr<uint8_t>(), node_local.data_ptr<int>(), stat.data_ptr<float>(),
      tot.data_ptr<float>(), static_cast<int>(T), static_cast<int>(L), static_cast<int>(n),
      static_cast<int>(p), static_cast<int>(kk), static_cast<int>(n_bins), static_cast<int>(crit),
      static_cast<float>(lam), static_cast<float>(min_child), static_cast<uint64_t>(seed),
      gain.data_ptr<float>(), feat.data_ptr<int>(), bin.data_ptr<int>(), cur_stream()));
  return {gain, feat, bin};
}

float* f32p(const Tensor& t, const char* name, int64_t numel) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == numel,
              name, ": contiguous fp32 GPU tensor with ", numel, " elements");
  return t.data_ptr<float>();
}
float* f32opt(const optional<Tensor>& t, const char* name, int64_t numel) {
  return (t.has_value() && t->defined()) ? f32p(*t, name, numel) : nullptr;
}

std::vector<Tensor> svm_smo(const Tensor& K, const Tensor& y, const std::vector<int64_t>& ns,
                            const Tensor& C, double tol, int64_t max_iter) {
  TORCH_CHECK(K.is_cuda() && K.scalar_type() == at::kDouble && K.is_contiguous() && K.dim() == 3 &&
                  K.size(1) == K.size(2),
              "svm_smo: K must be a contiguous fp64 GPU tensor [B, n, n]");
  const int64_t B = K.size(0), nmax = K.size(1);
  TORCH_CHECK(nmax >= 1 && nmax <= cml::smo_max_n(), "svm_smo: n must be in [1, ",
              cml::smo_max_n(), "]");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kDouble && y.is_contiguous() &&
                  y.numel() == B * nmax, "svm_smo: y must be fp64 [B, n]");
  TORCH_CHECK(C.is_cuda() && C.scalar_type() == at::kDouble && C.is_contiguous() &&
                  C.numel() == B, "svm_smo: C must be fp64 [B]");
  TORCH_CHECK(static_cast<int64_t>(ns.size()) == B, "svm_smo: one size per problem");
  for (int64_t v : ns) TORCH_CHECK(v >= 1 && v <= nmax, "svm_smo: problem size out of range");
  TORCH_CHECK(max_iter >= 0 && max_iter <= INT_MAX, "svm_smo: max_iter");
  const c10::DeviceGuard guard(K.device());
  std::vector<int> ns32(ns.begin(), ns.end());
  Tensor nsd = at::from_blob(ns32.data(), {B}, at::TensorOptions().dtype(at::kInt)).to(K.device());
  Tensor alpha = at::zeros({B, nmax}, K.options());
  Tensor grad = at::zeros({B, nmax}, K.options());
  Tensor iters = at::zeros({B}, nsd.options());
  CML_CHECK_HIP(cml::launch_smo(K.data_ptr<double>(), y.data_ptr<double>(), nsd.data_ptr<int>(),
                                static_cast<int>(B), static_cast<int>(nmax), C.data_ptr<double>(),
                                tol, static_cast<int>(max_iter), alpha.data_ptr<double>(),
                                grad.data_ptr<double>(), iters.data_ptr<int>(), cur_stream()));
  return {alpha, grad, iters};
}

void lasso_resid(const Tensor& z, const optional<Tensor>& v0, const Tensor& y, const Tensor& M,
                 const Tensor& nb, Tensor& r, const optional<Tensor>& rsum) {
  TORCH_CHECK(z.dim() == 2, "z: [n, B]");
  const int64_t n = z.size(0), B = z.size(1);
  const c10::DeviceGuard guard(z.device());
  CML_CHECK_HIP(cml::launch_lasso_resid(f32p(z, "z", n * B), f32opt(v0, "v0", B), f32p(y, "y", n),
                                        f32p(M, "M", n * B), f32p(nb, "nb", B), f32p(r, "r", n * B),
                                        f32opt(rsum, "rsum", B), static_cast<int>(n),
                                        static_cast<int>(B), cur_stream()));
}

void lasso_step(Tensor& v, Tensor& beta, const Tensor& g, const Tensor& step, const Tensor& lam,
                double alpha, Tensor& tk, const optional<Tensor>& rsum, const optional<Tensor>& v0,
                const optional<Tensor>& b0, Tensor& nbeta, Tensor& mom, Tensor& part,
                const optional<Tensor>& conv_part) {
  TORCH_CHECK(v.dim() == 2, "v: [p, B]");
  const int64_t p = v.size(0), B = v.size(1);
  const int64_t ns = cml::lasso_slices(static_cast<int>(p));
  const bool icpt = v0.has_value() && v0->defined();
  TORCH_CHECK(!icpt || (rsum.has_value() && rsum->defined() && b0.has_value() && b0->defined()),
              "lasso_step: the intercept needs rsum, v0 and b0");
  const c10::DeviceGuard guard(v.device());
  CML_CHECK_HIP(cml::launch_lasso_step(
      f32p(v, "v", p * B), f32p(beta, "beta", p * B), f32p(g, "g", p * B), f32p(step, "step", B),
      f32p(lam, "lam", B), static_cast<float>(alpha), f32p(tk, "tk", B),
      icpt ? f32opt(rsum, "rsum", B) : nullptr, icpt ? f32opt(v0, "v0", B) : nullptr,
      icpt ? f32opt(b0, "b0", B) : nullptr, f32p(nbeta, "nbeta", p * B), f32p(mom, "mom", B),
      f32p(part, "part", ns * B), f32opt(conv_part, "conv_part", ns * 2 * B), static_cast<int>(p),
      static_cast<int>(B), cur_stream()));
}

int64_t lasso_slices(int64_t p) { return cml::lasso_slices(static_cast<int>(p)); }

// Dense NT GEMM with fused epilogues (gemm.hip). y = epi(a [M, K] @ b [N, K]^T).
// ep 0: + bias; ep 1: aux <- h = a b^T + bias, y = gelu(h); ep 2: y = (a b^T) * gelu'(aux) and,
// with colsum_out, its column sums per row segment (colsum_out [nseg, N], bf16 or fp32, unit
// column stride, any row stride).
// EP_STORE tile choice: the 256 x 256 kernel once it has >= 128 tiles (it fills the chip), else
// the 128 x 128 kernel (bench/gemm.py: BERT per-rank and Llama shapes), 0 = neither eligible.
int64_t gemm_nt_pick(int64_t M, int64_t N, int64_t K) {
  if (cml::gemm_nt_eligible(M, N, K) && (M / 256) * (N / 256) >= 128) return 256;
  if (cml::gemm128_eligible(M, N, K)) return 128;
  if (cml::gemm_nt_eligible(M, N, K)) return 256;
  return 0;
}

Tensor gemm_nt(const Tensor& a, const Tensor& b, int64_t ep, const optional<Tensor>& bias,
               const optional<Tensor>& aux, const optional<Tensor>& out,
               const optional<Tensor>& colsum_out, const optional<Tensor>& cin, int64_t tile) {
  check_dev(a, "a");
  check_dev(b, "b");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16, "gemm_nt: bf16");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1,
              "gemm_nt: 2-D operands with unit column stride");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_nt: K mismatch");
  if (tile == 0) tile = ep == cml::EP_STORE ? gemm_nt_pick(M, N, K) : 256;
  TORCH_CHECK(tile == 128 || tile == 256, "gemm_nt: tile must be 0 (auto), 128 or 256");
  TORCH_CHECK(tile == 256 || ep == cml::EP_STORE, "gemm_nt: the 128 x 128 kernel has ep 0 only");
  TORCH_CHECK(tile == 128 ? cml::gemm128_eligible(M, N, K) : cml::gemm_nt_eligible(M, N, K),
              "gemm_nt: needs M, N multiples of the tile (", tile, ") and K % 64 == 0");
  // every operand on a's device and aligned for its vector width (16-B rows of a / b / y / aux /
  // cin, 8-B bias reads): a misaligned pointer must be a TORCH_CHECK, not a device fault
  auto same_dev = [&](const optional<Tensor>& t, const char* name) {
    if (t.has_value() && t->defined()) {
      TORCH_CHECK(t->is_cuda() && t->get_device() == a.get_device(), "gemm_nt: ", name,
                  " must be on a's device");
    }
  };
  auto aligned = [](const Tensor& t, int bytes) {
    return (reinterpret_cast<uintptr_t>(t.data_ptr()) % bytes) == 0;
  };
  TORCH_CHECK(b.get_device() == a.get_device(), "gemm_nt: b must be on a's device");
  same_dev(bias, "bias");
  same_dev(aux, "aux");
  same_dev(out, "out");
  same_dev(colsum_out, "colsum_out");
  same_dev(cin, "cin");
  TORCH_CHECK(aligned(a, 16) && aligned(b, 16) && a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0,
              "gemm_nt: a / b need 16-B aligned rows");
  const bool has_bias = bias.has_value() && bias->defined(), has_cin = cin.has_value() && cin->defined();
  const bool has_aux = aux.has_value() && aux->defined();
  TORCH_CHECK(!has_bias || aligned(*bias, 8), "gemm_nt: bias must be 8-B aligned");
  TORCH_CHECK(!has_cin || aligned(*cin, 16), "gemm_nt: cin must be 16-B aligned");
  TORCH_CHECK(!has_aux || aligned(*aux, 16), "gemm_nt: aux must be 16-B aligned");
  TORCH_CHECK(!(colsum_out.has_value() && colsum_out->defined()) ||
                  colsum_out->scalar_type() == at::kFloat || colsum_out->scalar_type() == at::kBFloat16,
              "colsum_out: bf16 or fp32");
  const c10::DeviceGuard guard(a.device());
  Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.dim() == 2 && y.size(0) == M &&
                y.size(1) == N && y.stride(1) == 1 && aligned(y, 16) && y.stride(0) % 8 == 0,
                "gemm_nt: out must be bf16 [M, N] with 16-B aligned rows");
  } else {
    y = at::empty({M, N}, a.options());
  }
  cml::GemmArgs g{};
  g.a = reinterpret_cast<const uint16_t*>(a.data_ptr());
  g.b = reinterpret_cast<const uint16_t*>(b.data_ptr());
  g.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  g.M = M; g.N = N; g.K = K;
  g.lda = a.stride(0); g.ldb = b.stride(0); g.ldy = y.stride(0);
  g.bias = opt_ptr<const uint16_t>(bias, at::kBFloat16, "bias", N);
  if (cin.has_value() && cin->defined()) {
    TORCH_CHECK(ep == cml::EP_STORE, "gemm_nt: cin only with ep 0");
    TORCH_CHECK(cin->scalar_type() == at::kBFloat16 && cin->dim() == 2 && cin->size(0) == M &&
                cin->size(1) == N && cin->stride(1) == 1 && cin->stride(0) == y.stride(0),
                "gemm_nt: cin must be bf16 [M, N] with out's row stride");
    g.cin = reinterpret_cast<const uint16_t*>(cin->data_ptr());
  }
  if (ep == cml::EP_GELU || ep == cml::EP_DGELU) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "gemm_nt: ep ", ep, " needs aux");
    TORCH_CHECK(aux->scalar_type() == at::kBFloat16 && aux->dim() == 2 && aux->size(0) == M &&
                aux->size(1) == N && aux->stride(1) == 1 && aux->stride(0) == y.stride(0),
                "gemm_nt: aux must be bf16 [M, N] with out's row stride");
    g.aux = reinterpret_cast<uint16_t*>(aux->data_ptr());
  }
  Tensor part;
  const bool cs = colsum_out.has_value() && colsum_out->defined();
  if (cs) {
    TORCH_CHECK(ep == cml::EP_DGELU, "gemm_nt: column sums only with ep 2");
    TORCH_CHECK(colsum_out->dim() == 2 && colsum_out->size(1) == N && colsum_out->stride(1) == 1,
                "gemm_nt: colsum_out must be [nseg, N]");
    part = at::empty({M / 128, N}, a.options().dtype(at::kFloat));
    g.part = part.data_ptr<float>();
  }
  if (tile == 128) {
    CML_CHECK_HIP(cml::launch_gemm128_nt(g, cur_stream()));
  } else {
    CML_CHECK_HIP(cml::launch_gemm_nt(g, static_cast<int>(ep), cur_stream()));
  }
  if (cs) {
    const bool f32 = colsum_out->scalar_type() == at::kFloat;
    CML_CHECK_HIP(cml::launch_colsum_fold(part.data_ptr<float>(), M, static_cast<int>(N),
                                          static_cast<int>(colsum_out->size(0)),
                                          colsum_out->data_ptr(), colsum_out->stride(0),
                                          f32 ? 1 : 0, cur_stream()));
  }
  return y;
}

bool gemm_nt_ok(int64_t M, int64_t N, int64_t K) { return cml::gemm_nt_eligible(M, N, K); }
int64_t gemm_conv_tm(int64_t M, int64_t N, int64_t C) {
  return cml::gemm_conv_tm(M, static_cast<int>(N), static_cast<int>(C));
}

// column sums of x viewed as [M, N] (N = last dim) -> bf16 [N]
// Dense GEMM on gemm_w4.hip (4 waves x 128 x 128 per 256 x 256 tile, every operand layout):
// y [M, N] = A B^T (+ bias[N]) (+ cin), A(m, k) = a[m][k] (mode bit 0 clear) or a[k][m] (set),
// B(n, k) = b[n][k] (bit 1 clear) or b[k][n] (set). So a linear layer's three products run
// without a transpose: forward gemm_w4(x, W, 0), data gradient gemm_w4(dy, W, 2), weight
// gradient gemm_w4(dy, x, 3). K % 64 == 0, M, N multiples of 8.
Tensor gemm_w4(const Tensor& a, const Tensor& b, int64_t mode, const optional<Tensor>& out,
               const optional<Tensor>& bias, const optional<Tensor>& cin) {
  check_dev(a, "a");
  check_dev(b, "b");
  TORCH_CHECK(mode >= 0 && mode < 4, "gemm_w4: mode 0..3");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16, "gemm_w4: bf16");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1,
              "gemm_w4: 2-D operands with unit column stride");
  TORCH_CHECK(b.get_device() == a.get_device(), "gemm_w4: b must be on a's device");
  const bool at_ = mode & 1, bt_ = mode & 2;
  const int64_t M = at_ ? a.size(1) : a.size(0), K = at_ ? a.size(0) : a.size(1);
  const int64_t N = bt_ ? b.size(1) : b.size(0), Kb = bt_ ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "gemm_w4: K mismatch (", K, " vs ", Kb, ")");
  TORCH_CHECK(cml::gemm_w4_eligible(M, N, K, static_cast<int>(mode)),
              "gemm_w4: needs K % 64 == 0 and M, N multiples of 8 (M ", M, ", N ", N, ", K ", K, ")");
  auto aligned = [](const Tensor& t, int bytes) {
    return (reinterpret_cast<uintptr_t>(t.data_ptr()) % bytes) == 0;
  };
  TORCH_CHECK(aligned(a, 16) && aligned(b, 16) && a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0,
              "gemm_w4: a / b need 16-B aligned rows");
  const c10::DeviceGuard guard(a.device());
  Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    TORCH_CHECK(y.is_cuda() && y.get_device() == a.get_device(), "gemm_w4: out must be on a's device");
    TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.dim() == 2 && y.size(0) == M &&
                y.size(1) == N && y.stride(1) == 1 && aligned(y, 16) && y.stride(0) % 8 == 0,
                "gemm_w4: out must be bf16 [M, N] with 16-B aligned rows");
  } else {
    y = at::empty({M, N}, a.options());
  }
  cml::GemmArgs g{};
  g.a = reinterpret_cast<const uint16_t*>(a.data_ptr());
  g.b = reinterpret_cast<const uint16_t*>(b.data_ptr());
  g.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  g.M = M; g.N = N; g.K = K;
  g.lda = a.stride(0); g.ldb = b.stride(0); g.ldy = y.stride(0);
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->get_device() == a.get_device() && aligned(*bias, 8),
                "gemm_w4: bias must be on a's device, 8-B aligned");
    g.bias = opt_ptr<const uint16_t>(bias, at::kBFloat16, "bias", N);
  }
  if (cin.has_value() && cin->defined()) {
    TORCH_CHECK(cin->is_cuda() && cin->get_device() == a.get_device(), "gemm_w4: cin device");
    TORCH_CHECK(cin->scalar_type() == at::kBFloat16 && cin->dim() == 2 && cin->size(0) == M &&
                cin->size(1) == N && cin->stride(1) == 1 && cin->stride(0) == y.stride(0) &&
                aligned(*cin, 16),
                "gemm_w4: cin must be bf16 [M, N] with out's row stride");
    g.cin = reinterpret_cast<const uint16_t*>(cin->data_ptr());
  }
  CML_CHECK_HIP(cml::launch_gemm_w4(g, static_cast<int>(mode), cur_stream()));
  return y;
}

Tensor colsum(const Tensor& x_in) {
  Tensor x = x_in.contiguous();
  check_bf16c(x, "x");
  const int64_t N = x.size(-1);
  const int64_t M = x.numel() / N;
  TORCH_CHECK(N % 8 == 0 && M >= 1 && (M + 63) / 64 <= 65535, "colsum: N % 8 == 0, M <= 4M rows");
  const c10::DeviceGuard guard(x.device());
  Tensor out = at::empty({N}, x.options());
  Tensor work = at::empty({static_cast<int64_t>(cml::colsum_workspace_bytes(M, static_cast<int>(N)) / 4 + 1)},
                          x.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_colsum(x.data_ptr(), M, static_cast<int>(N), out.data_ptr(),
                                   work.data_ptr(), cur_stream()));
  return out;
}

// Per-segment column sums of x [M, N] (nseg equal row segments) into out [nseg, N] (bf16, any row
// stride: e.g. the per-worker rows of the engine's flat gradient buffer).
void colsum_seg(const Tensor& x_in, int64_t nseg, Tensor& out) {
  Tensor x = x_in.contiguous();
  check_bf16c(x, "x");
  const int64_t N = x.size(-1);
  const int64_t M = x.numel() / N;
  TORCH_CHECK(out.is_cuda() && out.device() == x.device() && out.scalar_type() == at::kBFloat16 &&
                  out.dim() == 2 && out.size(0) == nseg && out.size(1) == N && out.stride(1) == 1,
              "colsum_seg: out must be bf16 [nseg, N] with unit column stride");
  const c10::DeviceGuard guard(x.device());
  Tensor work = at::empty({static_cast<int64_t>(cml::colsum_workspace_bytes(M, static_cast<int>(N)) / 4 + 1)},
                          x.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_colsum_seg(x.data_ptr(), M, static_cast<int>(N), static_cast<int>(nseg),
                                       out.data_ptr(), out.stride(0), work.data_ptr(), cur_stream()));
}

// Segmented norm backward: dx for all rows; dgamma / dbeta of segment z into dw_out[z] / db_out[z]
// (bf16 [nseg, D] views with one common row stride).
Tensor norm_bwd_seg(const Tensor& dy_in, const optional<Tensor>& dres_in, const Tensor& x,
                    const Tensor& w, const optional<Tensor>& mean, const Tensor& rstd,
                    int64_t nseg, Tensor& dw_out, const optional<Tensor>& db_out) {
  check_bf16c(x, "x");
  const int64_t D = x.size(-1);
  const int64_t M = x.numel() / D;
  Tensor dy = dy_in.contiguous();
  check_bf16c(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy shape mismatch");
  Tensor dres;
  if (dres_in.has_value() && dres_in->defined()) {
    dres = dres_in->contiguous();
    check_bf16c(dres, "dres");
    TORCH_CHECK(dres.sizes() == x.sizes(), "dres shape mismatch");
  }
  check_bf16c(w, "w");
  const bool ln = mean.has_value() && mean->defined();
  TORCH_CHECK(rstd.is_cuda() && rstd.scalar_type() == at::kFloat && rstd.numel() == M, "rstd: fp32 [M]");
  if (ln) TORCH_CHECK(mean->scalar_type() == at::kFloat && mean->numel() == M, "mean: fp32 [M]");
  TORCH_CHECK(D % 8 == 0 && D <= 4096, "norm: D % 8 == 0 and D <= 4096");
  TORCH_CHECK(nseg >= 1 && M % nseg == 0, "norm_bwd_seg: rows must split into nseg equal segments");
  auto chk = [&](const Tensor& o, const char* nm) {
    TORCH_CHECK(o.is_cuda() && o.device() == x.device() && o.scalar_type() == at::kBFloat16 &&
                    o.dim() == 2 && o.size(0) == nseg && o.size(1) == D && o.stride(1) == 1,
                nm, ": bf16 [nseg, D] with unit column stride");
  };
  chk(dw_out, "dw_out");
  void* dbp = nullptr;
  if (ln) {
    TORCH_CHECK(db_out.has_value() && db_out->defined(), "norm_bwd_seg: LayerNorm needs db_out");
    chk(*db_out, "db_out");
    TORCH_CHECK(db_out->stride(0) == dw_out.stride(0), "dw_out / db_out: one row stride");
    dbp = db_out->data_ptr();
  }
  const c10::DeviceGuard guard(x.device());
  Tensor dx = at::empty_like(x);
  Tensor work = at::empty({static_cast<int64_t>(cml::norm_workspace_bytes_seg(M, static_cast<int>(D),
                                                                              static_cast<int>(nseg)) / 4 + 1)},
                          x.options().dtype(at::kFloat));
  CML_CHECK_HIP(cml::launch_norm_bwd_seg(ln ? 1 : 0, dy.data_ptr(), dres.defined() ? dres.data_ptr() : nullptr,
                                         x.data_ptr(), w.data_ptr(), ln ? mean->data_ptr<float>() : nullptr,
                                         rstd.data_ptr<float>(), dx.data_ptr(), dw_out.data_ptr(), dbp,
                                         M, static_cast<int>(D), static_cast<int>(nseg),
                                         dw_out.stride(0), work.data_ptr(), cur_stream()));
  return dx;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "consensusml_amd native HIP kernels for gfx950 (MI355X)";
  m.def("agg_update", &agg_update, "fused robust aggregation + optimizer update");
  m.def("gram_workspace_bytes", &gram_workspace_bytes);
  m.def("gram", &gram, "G = X X^T (fp64) on MFMA; center: rows relative to that row",
        py::arg("X"), py::arg("n"), py::arg("D"), py::arg("rows"), py::arg("work"), py::arg("G"),
        py::arg("accumulate"), py::arg("center") = py::none());
  m.def("gram_center", &gram_center, "medoid of the finite rows of a Gram matrix");
  m.def("robust_weights", &robust_weights, "robust weights from a Gram matrix (+ selection counts, "
        "next center and the centered-pass guard in the same launch)",
        py::arg("G"), py::arg("rule"), py::arg("n"), py::arg("f"), py::arg("m"), py::arg("iters"),
        py::arg("eps"), py::arg("tol"), py::arg("tau"), py::arg("w"), py::arg("scores"),
        py::arg("sel"), py::arg("guard") = false, py::arg("center_out") = py::none(),
        py::arg("sel_counts") = py::none());
  m.def("gram_sum", &gram_sum, "sum of per-bucket Gram partials in bucket order");
  m.def("gram_partial", &gram_partial, "Gram stage 1 into a per-bucket workspace (block count)",
        py::arg("X"), py::arg("n"), py::arg("D"), py::arg("work"), py::arg("center") = py::none());
  m.def("gram_reduce_multi", &gram_reduce_multi,
        "reduce several buckets' Gram partials into G in one launch (bucket order)");
  m.def("agg_update_multi", &agg_update_multi,
        "fused robust aggregation + optimizer step over several buckets in one launch");
  m.def("gossip_workspace_bytes", &gossip_workspace_bytes);
  m.def("gossip_mix", &gossip_mix, "ring gossip mixing with neighbour clipping");
  m.def("gossip_mix_k", &gossip_mix_k, "k-neighbour gossip mixing with neighbour clipping (optional "
        "second parameter output: the delayed-gossip send buffer)", py::arg("master"),
        py::arg("param_out"), py::arg("nbrs"), py::arg("w"), py::arg("w0"), py::arg("clip"),
        py::arg("work"), py::arg("param_out2") = py::none());
  m.def("colsum_seg", &colsum_seg, "per-segment column sums into strided rows");
  m.def("norm_bwd_seg", &norm_bwd_seg, "LayerNorm / RMSNorm backward with per-segment dgamma / dbeta");
  m.def("conv1x1g_mode", &cml::conv1x1g_mode, "fused 1x1 kernel family: 0 old, 1 glds, 2 auto");
  m.def("set_conv1x1g_mode", &cml::set_conv1x1g_mode, "select the fused 1x1 kernel family");
  m.def("set_conv1x1g_ablate", &cml::set_conv1x1g_ablate, "diagnostics: quad kernel ablation bits");
  m.def("fault", &fault, "Byzantine fault injection");
  m.def("bn_fwd", &bn_fwd, "fused NHWC BatchNorm(+res)(+ReLU) forward");
  m.def("bn_bwd", &bn_bwd, "fused NHWC BatchNorm(+res)(+ReLU) backward");
  m.def("bn_fwd2", &bn_fwd2, "relu(BN(x1) + BN(x2)) forward (downsample-block tail)");
  m.def("bn_bwd2", &bn_bwd2, "relu(BN(x1) + BN(x2)) backward");
  m.def("bn_relu_maxpool_fwd", &bn_relu_maxpool_fwd, "maxpool(relu(BN(x))) forward (stem)");
  m.def("stem_conv_fwd", &stem_conv_fwd, "ResNet stem 7x7/s2 conv + BN statistics (MFMA)");
  m.def("stem_wgrad", &stem_wgrad, "ResNet stem weight gradient through BN (MFMA, one pass)");
  m.def("maxpool_fwd", &maxpool_fwd, "NHWC bf16 max-pool forward (uint8 argmax)");
  m.def("maxpool_bwd", &maxpool_bwd, "NHWC bf16 max-pool backward (gather)");
  m.def("conv1x1_bn_fwd", &conv1x1_bn_fwd, py::arg("x"), py::arg("w"), py::arg("pro_sc"),
        py::arg("pro_bi"), py::arg("shift"), py::arg("running_mean"), py::arg("running_var"),
        py::arg("stride"), py::arg("stats"), py::arg("eps"), py::arg("momentum"),
        py::arg("gamma") = py::none(), py::arg("beta") = py::none(),
        "fused 1x1 conv forward (MFMA) + BN statistics epilogue + optional BN-ReLU prologue "
        "(+ with gamma / beta that BN's affine sc, bi from the statistics' finalize)");
  m.def("bn_stats", &bn_stats, "training BatchNorm statistics (mean, invstd) only");
  m.def("wgrad1x1", &wgrad1x1, py::arg("dy"), py::arg("x"), py::arg("dtype"),
        py::arg("pro_sc") = py::none(), py::arg("pro_bi") = py::none(),
        py::arg("dz_z") = py::none(), py::arg("dz_mask") = py::none(), py::arg("dz_a") = py::none(),
        py::arg("dz_b") = py::none(), py::arg("dz_c") = py::none(), py::arg("out") = py::none(),
        "weight gradient of a stride-1 1x1 conv (MFMA, split-K)");
  m.def("wgrad3x3s2_ok", &wgrad3x3s2_ok, py::arg("N"), py::arg("H"), py::arg("W"),
        py::arg("Co"), py::arg("Ci"), py::arg("taps") = 9);
  m.def("wgrad3x3s2", &wgrad3x3s2, py::arg("dy"), py::arg("x"), py::arg("dtype"),
        py::arg("zero") = py::none(), py::arg("taps") = 9);
  m.def("wgrad3x3", &wgrad3x3, py::arg("dy"), py::arg("x"), py::arg("dtype"),
        py::arg("zero") = py::none(),
        "weight gradient of a 3x3 stride-1 conv (MFMA, split-K, all nine taps per workgroup: "
        "wgrad3x3.hip) for shapes with wgrad3x3_direct_ok");
  m.def("conv1x1_link_s2", &conv1x1_link_s2,
        "1x1 data gradient + a stride-2 conv's compact data gradient at the even pixels");
  m.def("subsample2", &subsample2, "x[:, :, ::2, ::2] of an NHWC bf16 tensor, dense NHWC");
  m.def("upsample2_scatter", &upsample2_scatter, py::arg("g"), py::arg("H"), py::arg("W"),
        "full-resolution NHWC tensor with g at the even pixels, zeros elsewhere");
  m.def("wgrad3x3_direct_ok", [](int64_t B, int64_t H, int64_t W, int64_t Co, int64_t Ci) {
    int S, T;
    return cml::wgrad3x3_direct_plan(static_cast<int>(B), static_cast<int>(H), static_cast<int>(W),
                                     static_cast<int>(Co), static_cast<int>(Ci), &S, &T);
  }, "whether wgrad3x3 takes the nine-tap kernel for this shape");
  m.def("conv_gemm_bnsums", &conv_gemm_bnsums, py::arg("x"), py::arg("w"), py::arg("taps"),
        py::arg("zero"), py::arg("z"), py::arg("sc"), py::arg("bi"), py::arg("mean"),
        py::arg("invstd"), py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(),
        "stride-1 conv_gemm + the sums of the BN + ReLU backward its output feeds (+ optionally "
        "that BN's parameter gradients)");
  m.def("conv_gemm_s2dgrad", &conv_gemm_s2dgrad, py::arg("dy"), py::arg("wr"), py::arg("zero"),
        py::arg("z") = py::none(), py::arg("sc") = py::none(), py::arg("bi") = py::none(),
        py::arg("mean") = py::none(), py::arg("invstd") = py::none(),
        py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(),
        "stride-2 3x3 data gradient as four parity-class implicit GEMMs (+ BN + ReLU backward sums, "
        "+ optionally that BN's parameter gradients)");
  m.def("conv_gemm", &conv_gemm, py::arg("x"), py::arg("w"), py::arg("taps"),
        py::arg("zero") = py::none(), py::arg("stride") = 1,
        "implicit-GEMM NHWC conv (1x1 / 3x3 padding 1, stride 1 or 2), glds staging");
  m.def("conv1x1_bn_stats_only", &conv1x1_bn_stats_only, py::arg("x"), py::arg("w"),
        py::arg("pro_sc"), py::arg("pro_bi"), py::arg("shift") = py::none(),
        py::arg("running_mean") = py::none(), py::arg("running_var") = py::none(),
        py::arg("eps") = 1e-5, py::arg("momentum") = 0.1,
        "BN statistics of conv1x1(bnrelu(x)) without storing the product");
  m.def("conv1x1_bnres", &conv1x1_bnres, "recomputed conv1x1 + BN apply + residual + ReLU -> {y, mask}");
  m.def("conv1x1_cat_bnres", &conv1x1_cat_bnres,
        "two BN'd 1x1 convs summed + ReLU in one K-concatenated GEMM -> {y, mask}");
  m.def("conv1x1_cat_bnsums", &conv1x1_cat_bnsums, py::arg("g"), py::arg("mask"), py::arg("x2"),
        py::arg("sc2"), py::arg("bi2"), py::arg("w"), py::arg("bias"), py::arg("mean"),
        py::arg("invstd"), py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(),
        "conv1x1_cat + the sums of the BN + ReLU backward its output feeds (+ optionally that "
        "BN's parameter gradients)");
  m.def("bn_affine", &bn_affine, "BN affine (gamma invstd, beta - mean sc) of batch statistics");
  m.def("bn_bwd_apply", &bn_bwd_apply, "apply half of a BN + ReLU backward from its sums");
  m.def("split_search_sampled", &split_search_sampled,
        "tree split search with in-kernel candidate sampling, <= 128 bins -> {gain, feature, bin}");
  m.def("tail_bwd_prep", &tail_bwd_prep,
        "recompute-tail backward algebra: {w_cat, bias, dW, dgamma, dbeta}");
  m.def("conv1x1_cat", &conv1x1_cat, "two-source (masked | BN-ReLU or identity) 1x1 conv along K, + bias");
  m.def("split_fold", &split_fold, "fixed-order fold of a split-K partial slab");
  m.def("wgrad1x1_ex", &wgrad1x1_ex, py::arg("dy"), py::arg("x"), py::arg("pro_sc") = py::none(),
        py::arg("pro_bi") = py::none(), py::arg("dmode") = 0, py::arg("dz_mask") = py::none(),
        py::arg("dz_a") = py::none(), py::arg("dz_b") = py::none(), py::arg("dz_c") = py::none(),
        py::arg("colsum") = false, "1x1 weight gradient with dy prologue modes and column sums");
  m.def("conv_gemm_bn", &conv_gemm_bn, py::arg("x"), py::arg("w"), py::arg("taps"),
        py::arg("zero") = py::none(), py::arg("shift") = py::none(),
        py::arg("running_mean") = py::none(), py::arg("running_var") = py::none(),
        py::arg("eps") = 1e-5, py::arg("momentum") = 0.1, py::arg("stride") = 1,
        py::arg("gamma") = py::none(), py::arg("beta") = py::none(),
        "implicit-GEMM conv + BN statistics of the output in the epilogue -> {y, mean, invstd} "
        "(+ sc, bi: the BN's affine from the finalize, with gamma / beta)");
  m.def("conv1x1_bnbwd", &conv1x1_bnbwd, "1x1 data gradient through a BN + ReLU backward prologue");
  m.def("conv1x1_link", &conv1x1_link, py::arg("x"), py::arg("w"), py::arg("link"),
        py::arg("lmask"), py::arg("sz") = py::none(), py::arg("smask") = py::none(),
        py::arg("mean") = py::none(), py::arg("invstd") = py::none(),
        "1x1 data gradient + masked residual gradient (lmask None: plain residual add) (+ the "
        "consumer BN's backward sums)");
  m.def("bn_stats_gram", &bn_stats_gram, py::arg("G"), py::arg("cy"), py::arg("w"), py::arg("M"),
        py::arg("running_mean") = py::none(), py::arg("running_var") = py::none(),
        py::arg("eps") = 1e-5, py::arg("momentum") = 0.1, py::arg("gamma") = py::none(),
        py::arg("beta") = py::none(),
        "BN statistics of a 1x1 conv's output from its input's Gram matrix and column sums "
        "(+ the BN affine sc, bi when gamma / beta are given)");
  m.def("bn_bwd_coeffs", &bn_bwd_coeffs, "BN + ReLU backward coefficients from its sums");
  m.def("bn_bwd_sums", &bn_bwd_sums, "reduction half of a BN (+ ReLU) backward");
  m.def("stem_wgrad_pool", &stem_wgrad_pool, py::arg("dy"), py::arg("idx"), py::arg("dy2"),
        py::arg("z"), py::arg("x"), py::arg("mean"), py::arg("invstd"), py::arg("gamma"),
        py::arg("bf16_out") = false,
        "stem backward (conv weight gradient through BN, dgamma, dbeta) from the pool output "
        "gradient, the pool input gradient gathered inside the kernel");
  m.def("avgpool_bwd", &avgpool_bwd, py::arg("g"), py::arg("H"), py::arg("W"),
        "global-average-pool backward into NHWC in one write-only pass");
  m.def("conv_wlayouts_multi", &conv_wlayouts_multi, py::arg("ws"),
        "GEMM layouts of several 3x3 / 1x1 conv weights in one launch -> [(wf, wr), ...]");
  m.def("scaled_cat_bias", &scaled_cat_bias, py::arg("w1"), py::arg("s1"), py::arg("w2"),
        py::arg("s2"), py::arg("b1"), py::arg("b2"),
        "[diag(s1) w1 | diag(s2) w2] (bf16) and b1 + b2 in one launch");
  m.def("conv3x3_wlayouts", &conv3x3_wlayouts, py::arg("w"), py::arg("want_wf"),
        "forward / data-gradient GEMM layouts of a 3x3 conv weight in one launch");
  m.def("maxpool_bwd_sum", &maxpool_bwd_sum, "3x3/s2 max-pool backward + channel sums of dx",
        py::arg("dy"), py::arg("idx"), py::arg("H"), py::arg("W"), py::arg("dy2") = py::none());
  m.def("multi_copy", &multi_copy, "multi-tensor copy in one launch per 32 tensors");
  m.def("pad_c4", &pad_c4, "NHWC bf16 channel zero-padding to 4");
  m.def("ce_fwd", &ce_fwd, "fused cross-entropy forward over bf16 logits (lse, per-row loss)");
  m.def("ce_bwd", &ce_bwd, py::arg("logits"), py::arg("labels"), py::arg("lse"), py::arg("scale"),
        py::arg("ignore"), py::arg("div") = py::none(),
        "fused cross-entropy backward (bf16 logits gradient; scale / div when div is given)");
  m.def("ce_bwd_cs", &ce_bwd_cs, py::arg("logits"), py::arg("labels"), py::arg("lse"),
        py::arg("scale"), py::arg("ignore"), py::arg("div") = py::none(),
        "cross-entropy backward over row-strided logits + bias-gradient column partials");
  m.def("ce_mean", &ce_mean, py::arg("loss"), py::arg("labels"), py::arg("ignore"),
        "{mean loss, n_valid} from ce_fwd's per-row losses in one launch");
  m.def("transpose_bf16", &transpose_bf16, "w.t().contiguous() (LDS-tiled bf16 transpose)");
  m.def("gelu_bwd", &gelu_bwd, "dh = da * gelu'(h) (erf GELU), bf16");
  m.def("ce_part_fold", &ce_part_fold, "per-segment fold of ce_bwd_cs's column partials");
  m.def("norm_fwd", &norm_fwd, "LayerNorm / RMSNorm (+ residual add) forward");
  m.def("norm_bwd", &norm_bwd, "LayerNorm / RMSNorm backward (+ residual gradient)");
  m.def("rope_fwd", &rope_fwd, "QKV split + RoPE into head-major q / k / v");
  m.def("rope_bwd", &rope_bwd, "inverse of rope_fwd (grp > 1: sums per-query-head dk / dv)",
        py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("cos"), py::arg("sin"),
        py::arg("grp") = 1);
  m.def("flash_fwd", &flash_fwd, "flash attention forward, head dim 128, GQA, causal / full",
        py::arg("q"), py::arg("k"), py::arg("v"), py::arg("causal"), py::arg("scale"),
        py::arg("rescale_thr") = 8.0);
  m.def("flash_bwd", &flash_bwd, "flash attention backward (dq, per-query-head dk / dv)");
  m.def("swiglu_fwd", &swiglu_fwd, "silu(a) * b over [a | b]");
  m.def("swiglu_bwd", &swiglu_bwd, "SwiGLU backward");
  m.def("attn_fwd", &attn_fwd, "short-sequence MFMA attention forward (fused qkv in)");
  m.def("attn_bwd", &attn_bwd, "short-sequence MFMA attention backward (fused dqkv out)");
  m.def("split_search", &split_search, "tree-ensemble histogram split search (one level)");
  m.def("svm_smo", &svm_smo, "batched dual C-SVC SMO (one wave per problem)");
  m.def("smo_max_n", &cml::smo_max_n);
  m.def("lasso_resid", &lasso_resid, "batched logistic-lasso residual (+ intercept gradient)");
  m.def("lasso_step", &lasso_step, "batched FISTA prox / restart / momentum step");
  m.def("lasso_slices", &lasso_slices);
  m.def("colsum", &colsum, "column sums of a bf16 matrix (bias gradient)");
  m.def("gemm_nt", &gemm_nt, "NT GEMM with fused epilogues (bias / bias+GELU / GELU backward + "
        "column sums)", py::arg("a"), py::arg("b"), py::arg("ep"), py::arg("bias") = py::none(),
        py::arg("aux") = py::none(), py::arg("out") = py::none(),
        py::arg("colsum_out") = py::none(), py::arg("cin") = py::none(), py::arg("tile") = 0);
  m.def("gemm_w4", &gemm_w4, "GEMM on 4-wave 256 x 256 tiles, any operand layout (mode bit 0: a is "
        "[K, M], bit 1: b is [K, N])", py::arg("a"), py::arg("b"), py::arg("mode") = 0,
        py::arg("out") = py::none(), py::arg("bias") = py::none(), py::arg("cin") = py::none());
  m.def("gemm_nt_ok", &gemm_nt_ok, "shape eligibility of gemm_nt's 256 x 256 kernel");
  m.def("gemm_conv_tm", &gemm_conv_tm, "m-tile of gemm.hip's 3x3 conv mode for M x N, C (256, 512, 0)");
  m.def("gemm_nt_pick", &gemm_nt_pick, "EP_STORE tile choice of gemm_nt: 256, 128 or 0 (none)");
  m.attr("CMB_SORTED") = static_cast<int>(cml::CMB_SORTED);
  m.attr("CMB_WEIGHTED") = static_cast<int>(cml::CMB_WEIGHTED);
  m.attr("OPT_NONE") = static_cast<int>(cml::OPT_NONE);
  m.attr("OPT_SGD") = static_cast<int>(cml::OPT_SGD);
  m.attr("OPT_ADAM") = static_cast<int>(cml::OPT_ADAM);
  m.attr("RULE_MEAN") = static_cast<int>(cml::RULE_MEAN);
  m.attr("RULE_KRUM") = static_cast<int>(cml::RULE_KRUM);
  m.attr("RULE_MULTI_KRUM") = static_cast<int>(cml::RULE_MULTI_KRUM);
  m.attr("RULE_GEOMED") = static_cast<int>(cml::RULE_GEOMED);
  m.attr("RULE_CCLIP") = static_cast<int>(cml::RULE_CCLIP);
  m.attr("RULE_BULYAN_SELECT") = static_cast<int>(cml::RULE_BULYAN_SELECT);
}
