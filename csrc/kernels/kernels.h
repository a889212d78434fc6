// Host-side launch API of the consensus kernels (no torch headers: included by bindings.cpp and
// by every .hip translation unit). All launches are asynchronous on the given stream and never
// allocate, synchronise or copy to the host, so callers may capture them in a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cml {

enum DType : int { DT_BF16 = 0, DT_F32 = 1 };
enum Combine : int { CMB_SORTED = 0, CMB_WEIGHTED = 1 };
enum Opt : int { OPT_NONE = 0, OPT_SGD = 1, OPT_ADAM = 2 };
enum Rule : int {
  RULE_MEAN = 0,
  RULE_KRUM = 1,
  RULE_MULTI_KRUM = 2,
  RULE_GEOMED = 3,
  RULE_CCLIP = 4,
  RULE_BULYAN_SELECT = 5,
};

// Worker rows of a [n, ld] matrix: row i of the aggregation is X + rows[i]*ld (rows == nullptr:
// identity). Sorted combine averages sorted ranks [lo, lo+cnt); weighted combine computes
// sum_i w[i] x_i (w == nullptr: all ones), skipping zero-weight rows.
struct SrcArgs {
  const void* X;
  int64_t ld;
  int n;
  const int* rows;
  const float* w;
  int lo, cnt;
};

// Optimizer state is fp32 and indexed like the aggregate. Any pointer may be null when unused.
struct UpdArgs {
  float* master;     // fp32 master weights (SGD/Adam)
  float* s1;         // momentum (SGD) or exp_avg (Adam)
  float* s2;         // exp_avg_sq (Adam)
  void* param_out;   // model parameters rewritten from the master (bf16, or fp32 if param_f32)
  float* gout;       // aggregated gradient (fp32), optional
  float lr, momentum, weight_decay, beta1, beta2, eps, step_size, inv_sqrt_bc2, gscale;
  int nesterov, first;
  int param_f32;
  int adam_l2;       // Adam: torch.optim.Adam's L2 term (g += wd p) instead of AdamW's decay
};

// Aggregate n worker vectors of length D and apply the optimizer in the same pass.
// Returns hipSuccess or the launch error.
hipError_t launch_agg_update(int dtype, int combine, int opt, const SrcArgs& src,
                             const UpdArgs& upd, int64_t D, hipStream_t stream);
// The same over up to 16 segments in ONE launch (the sharded engine's buckets): segment i reads
// worker rows from X (row stride ld) over D elements, updates the optimizer state at element
// offset off and writes param_out; src / upd carry the shared rule, weights and state bases
// (upd.param_out unused). Ragged or unaligned segments fall back to one launch each.
struct AggSeg {
  const void* X;
  int64_t ld;
  int64_t D;
  int64_t off;
  void* param_out;
};
hipError_t launch_agg_update_multi(int dtype, int combine, int opt, const SrcArgs& src,
                                   const UpdArgs& upd, const AggSeg* segs, int nseg,
                                   hipStream_t stream);

// Gram matrix G = X X^T (fp64, [n, n], row-major) of n <= 64 worker rows. ``work`` must hold
// gram_workspace_bytes(n, D) bytes. accumulate != 0: G += X X^T (bucket-by-bucket Gram).
size_t gram_workspace_bytes(int n, int64_t D);
// center (device int, may be null): rows relative to worker row *center (centered Gram,
// translation-invariant for every Gram-space rule, no cancellation for near-duplicate workers).
hipError_t launch_gram(int dtype, const void* X, int64_t ld, int n, const int* rows, int64_t D,
                       void* work, double* G, int accumulate, hipStream_t stream,
                       const int* center = nullptr);
// out[0] = the medoid of the finite rows of G [n, n] (the centered Gram's center).
hipError_t launch_gram_center(const double* G, int n, int* out, hipStream_t stream);

// Robust weights from a Gram matrix (single workgroup). Outputs:
//   w[n_out] fp32 (n_out = n, or n+1 for centered clipping whose last row is the previous
//   aggregate), scores[n] fp64 (Krum scores / final distances), sel[n+1] int32
//   (Bulyan: sorted selected indices then sel[n] = count; others: sel[i] = 1 if w_i > 0).
// Optional, in the same launch: sel_counts[n] fp64 += (w_i > 0); center_out[0] = medoid of G
// (the next step's Gram center); guard != 0 (G from a pass centered on the previous step's
// medoid): if at least half the worker rows are non-finite the weights are zeroed (centered
// clipping: the previous aggregate kept) and center_out = -1 (next pass uncentered).
hipError_t launch_robust_weights(int rule, const double* G, int n, int f, int m, int iters,
                                 double eps, double tol, double tau, float* w, double* scores,
                                 int* sel, hipStream_t stream, int guard = 0,
                                 int* center_out = nullptr, double* sel_counts = nullptr,
                                 int* nbad_io = nullptr);
// Stage 1 of launch_gram only: per-workgroup [P, P] fp32 partials into work (*nblk of them, P =
// 16 ceil(n / 16)); launch_gram_reduce_multi then reduces nb buckets' partials into G in ONE
// launch, bit-identical to one launch_gram per bucket into slots summed by launch_gram_sum.
hipError_t launch_gram_partial(int dtype, const void* X, int64_t ld, int n, const int* rows,
                               int64_t D, void* work, hipStream_t stream, const int* center,
                               int* nblk);
hipError_t launch_gram_reduce_multi(const float* const* parts, const int* nblks, int nb, int n,
                                    double* G, hipStream_t stream);
// G[e] = sum_b Gb[b][e] in b order (the early-Gram per-bucket partials), e < E.
hipError_t launch_gram_sum(const double* Gb, int nb, int64_t E, double* G, hipStream_t stream);

// Gossip: x <- (w0+w1+w2) x + w1*clip(left-x) + w2*clip(right-x); writes fp32 master and bf16
// params. clip <= 0 disables clipping. ``work`` must hold gossip_workspace_bytes(D) bytes.
// The fused 1x1-conv kernel family used by launch_conv1x1_* (conv1x1g.hip policy): 0 = the
// register-staged conv1x1.hip kernels only, 1 = the global_load_lds kernels wherever eligible,
// 2 = per-shape auto (default; env CML_C1G = 0 / 1 / auto).
int conv1x1g_mode();
void set_conv1x1g_mode(int mode);
// diagnostics: ablation bits passed to the quad-phase kernel (see C1Args::ablate)
void set_conv1x1g_ablate(int bits);

size_t gossip_workspace_bytes(int64_t D);
// k-neighbour mix (1 <= k <= 8): x <- (w0 + sum w_k) x + sum_k w_k clip_k(nbrs[k] - x)
hipError_t launch_gossip_mix_k(int dtype, float* master, void* param_out, const void* const* nbrs,
                               const float* w, int k, int64_t D, float w0, float clip, void* work,
                               hipStream_t stream, void* param_out2 = nullptr);
hipError_t launch_gossip_mix(int dtype, float* master, void* param_out, const void* left,
                             const void* right, int64_t D, float w0, float w1, float w2,
                             float clip, void* work, hipStream_t stream);

// Fused training BatchNorm (+ residual add) (+ ReLU) on NHWC bf16 rows x[M, C] (C % 8 == 0,
// C <= 2048). Forward with training != 0 computes batch statistics into mean / invstd (fp32 [C])
// and updates the fp32 running stats (nullable); training == 0 uses the given mean / invstd.
// Backward recomputes the ReLU mask from x, writes dx (and dres = dz when res != null), dgamma /
// dbeta (bf16) and the per-channel sums sdz / sdzx (fp32 [C]). ``work``: bn_workspace_bytes.
size_t bn_workspace_bytes(int64_t M, int C);
// mask (optional, only with res && relu): [M, C/8] bytes, one ReLU bit per element.
hipError_t launch_bn_fwd(const void* x, const void* res, void* y, void* mask, int64_t M, int C,
                         const void* gamma, const void* beta, float* mean, float* invstd,
                         float* rmean, float* rvar, float eps, float momentum, int relu,
                         int training, void* work, hipStream_t stream);
// Backward: output gradient dy (+ dy2 if non-null); ReLU from the forward's bit mask when given,
// else recomputed from x (only valid without a residual); dres (optional) receives the masked
// output gradient (the residual input's gradient). dx == null: the reduction only (sums, dgamma,
// dbeta), for consumers that apply the backward in their own prologue.
// Apply half of a training BN + ReLU backward (ReLU mask recomputed from x) from its sums
// (sdz = sum dy', sdzx = sum dy' xhat): dx = gamma invstd (dy' - sdz / M - xhat sdzx / M).
// BN affine of batch statistics: sc = gamma invstd, bi = beta - mean sc (fp32 [C]; gamma / beta bf16)
hipError_t launch_bn_affine(const void* gamma, const void* beta, const float* mean,
                            const float* invstd, int C, float* sc, float* bi, hipStream_t st);
hipError_t launch_bn_bwd_apply(const void* dy, const void* x, void* dx, int64_t M, int C,
                               const void* gamma, const void* beta, const float* mean,
                               const float* invstd, const float* sdz, const float* sdzx,
                               hipStream_t st);
hipError_t launch_bn_bwd(const void* dy, const void* dy2, const void* x, const void* mask,
                         void* dx, void* dres, int64_t M, int C, const void* gamma,
                         const void* beta, const float* mean, const float* invstd, void* dgamma,
                         void* dbeta, float* sdz, float* sdzx, int relu, void* work,
                         hipStream_t stream);

// Downsample-block tail y = relu(bn1(x1) + bn2(x2)) (two training BNs of the same shape, one
// ReLU, optional 1-bit mask). Forward work: bn_workspace_bytes; backward: bn2_workspace_bytes.
// Backward writes dx1, dx2, both BNs' dgamma / dbeta and their per-channel sums (sdz, sdzx1) and
// (sdz_b, sdzx2).
hipError_t launch_bn_fwd2(const void* x1, const void* x2, void* y, void* mask, int64_t M, int C,
                          const void* gamma1, const void* beta1, const void* gamma2,
                          const void* beta2, float* mean1, float* invstd1, float* mean2,
                          float* invstd2, float* rmean1, float* rvar1, float* rmean2,
                          float* rvar2, float eps, float momentum, int training, void* work,
                          hipStream_t stream);
size_t bn2_workspace_bytes(int64_t M, int C);
hipError_t launch_bn_bwd2(const void* dy, const void* dy2, const void* x1, const void* x2,
                          const void* mask, void* dx1, void* dx2, int64_t M, int C,
                          const void* gamma1, const void* gamma2, const float* mean1,
                          const float* invstd1, const float* mean2, const float* invstd2,
                          void* dgamma1, void* dbeta1, void* dgamma2, void* dbeta2, float* sdz,
                          float* sdzx1, float* sdz_b, float* sdzx2, void* work,
                          hipStream_t stream);

// y = x[:, ::2, ::2, :] of NHWC bf16 x [N][H][W][C] (y [N][ceil(H/2)][ceil(W/2)][C]); the
// scatter writes the full-resolution dx with g at the even pixels and zeros elsewhere. C % 8 == 0.
hipError_t launch_subsample2(const void* x, void* y, int N, int H, int W, int C, hipStream_t st);
// Global-average-pool backward: g bf16 [N][C] -> dx NHWC bf16 [N][HW][C], bf16(g / HW) everywhere.
hipError_t launch_avgpool_bwd(const void* g, void* dx, int N, int HW, int C, hipStream_t st);
hipError_t launch_upsample2_scatter(const void* g, void* dx, int N, int H, int W, int C,
                                    hipStream_t st);
// NHWC bf16 max-pool with a one-byte argmax per output element; backward is a gather.
hipError_t launch_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C,
                              int OH, int OW, int k, int s, int p, hipStream_t stream);
hipError_t launch_maxpool_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W,
                              int C, int OH, int OW, int k, int s, int p, hipStream_t stream);

// Multi-tensor copy of up to kMaxCopy (src -> dst, bytes) entries in one launch (16-B aligned
// pointers, even byte counts). vpre[e] = number of whole 16-B vectors before entry e; bpre[e] =
// first workgroup of entry e (filled by launch_multi_copy).
constexpr int kMaxCopy = 32;
struct MultiCopyArgs {
  const void* src[kMaxCopy];
  void* dst[kMaxCopy];
  int64_t bytes[kMaxCopy];
  int64_t vpre[kMaxCopy + 1];
  int bpre[kMaxCopy + 1];
  int n;
  int slice;    // 1: one 32-KiB slice per workgroup (small copies), 0: striding workgroups
};
hipError_t launch_multi_copy(const MultiCopyArgs& args, hipStream_t stream);
// dst [C][R] = src [R][C]^T, bf16, R and C multiples of 64, row strides lds / ldd (% 8 == 0)
hipError_t launch_transpose_bf16(const void* src, void* dst, int R, int C, int64_t lds, int64_t ldd,
                                 hipStream_t stream);

// 3x3/s2/p1 max-pool backward that also returns the channel sums of dx (fp32 [C]; the stem BN's
// dbeta). dy2 (nullable): a second output gradient, summed on load. work:
// maxpool_bwd_sum_workspace_bytes.
size_t maxpool_bwd_sum_workspace_bytes(int N, int H, int W, int C);
// Channel sums of a max-pool's routed output gradient: sums[c] = sum over pooled pixels whose
// argmax byte is not 255 of dy (+ dy2) (= the channel sums of the pool's input gradient, which is
// never formed); with dy2, dsum = bf16(dy + dy2) as well. P pooled pixels, C channels (C / 8
// divides 256); work: pool_gsum_workspace_floats(P, C) floats.
size_t pool_gsum_workspace_floats(int64_t P, int C);
hipError_t launch_pool_gsum(const void* dy, const void* dy2, const void* idx, void* dsum,
                            float* sums, float* work, int64_t P, int C, hipStream_t st);
hipError_t launch_maxpool_bwd_sum(const void* dy, const void* dy2, const void* idx, void* dx,
                                  float* sums, void* work, int N, int H, int W, int C, int OH,
                                  int OW, hipStream_t stream);
// Stem: y = maxpool(relu(bn(x))) with the BN affine (training statistics from launch_bn_stats,
// or running statistics) applied to every window tap; idx as launch_maxpool_fwd.
hipError_t launch_bn_stats(const void* x, int64_t M, int C, float* mean, float* invstd,
                           float* rmean, float* rvar, float eps, float momentum, void* work,
                           hipStream_t stream);
hipError_t launch_bn_relu_maxpool_fwd(const void* x, const float* mean, const float* invstd,
                                      const void* gamma, const void* beta, void* y, void* idx,
                                      int N, int H, int W, int C, int OH, int OW, int k, int s,
                                      int p, hipStream_t stream);

// NHWC bf16 channel zero-padding C (<= 4) -> 4 over npix pixels (y 8-B aligned).
hipError_t launch_pad_c4(const void* x, void* y, int64_t npix, int C, hipStream_t stream);

// Elementwise fault injection on a local gradient (Byzantine simulation, N10).
hipError_t launch_fault(int dtype, void* g, int64_t D, int kind, float scale, float sigma,
                        uint64_t seed, hipStream_t stream);

// ---- transformer ops (transformer.hip); bf16 activations, fp32 statistics.
// Cross-entropy over contiguous bf16 logits [R, V] (16-B aligned base): forward writes the
// per-row logsumexp and loss (0 for ignored rows); backward writes
// grad = (*scale) * (softmax - onehot) (0 rows for ignored labels), scale = dloss / n_valid.
hipError_t launch_ce_fwd(const void* logits, int64_t R, int V, int64_t ld, const int64_t* labels,
                         int64_t ignore, float* lse, float* loss, hipStream_t stream);
// div (optional): scale = scale[0] / div[0] in the kernel (grad_output / n_valid, no divide launch)
hipError_t launch_ce_bwd(const void* logits, int64_t R, int V, const int64_t* labels,
                         int64_t ignore, const float* lse, const float* scale, void* grad,
                         hipStream_t stream, const float* div = nullptr);
// The mean loss from the forward's per-row losses in one launch (one workgroup, fixed order, fp64
// sums): *out = sum(loss) / n_valid, *count = n_valid = max(#labels != ignore, 1) (fp32).
hipError_t launch_ce_mean(const float* loss, const int64_t* labels, int64_t R, int64_t ignore,
                          float* out, float* count, hipStream_t stream);
// Row-strided form (ld % 8 == 0, R % 64 == 0): grad gets the same stride (columns [V, ld) = 0),
// and part [R / 64][ld] fp32 the column sums of each 64-row block of the stored gradient;
// launch_ce_part_fold sums them per segment of R / nseg rows into out [nseg][ldo] (bf16 / fp32).
hipError_t launch_ce_bwd_cs(const void* logits, int64_t R, int V, int64_t ld,
                            const int64_t* labels, int64_t ignore, const float* lse,
                            const float* scale, void* grad, float* part, hipStream_t stream,
                            const float* div = nullptr);
hipError_t launch_ce_part_fold(const float* part, int64_t R, int V, int64_t ld, int nseg, void* out,
                               int64_t ldo, int out_f32, hipStream_t stream);
// dh = bf16(da * gelu'(h)) (erf GELU), n % 8 == 0, 16-B aligned
hipError_t launch_gelu_bwd(const void* da, const void* h, void* dh, int64_t n, hipStream_t stream);
// LayerNorm (ln = 1, with bias b and mean) or RMSNorm (ln = 0) over rows of D (D % 8 == 0,
// D <= 4096). res != null: normalise x + res and write the bf16 sum to `sum`.
// Backward: dx (+ dres if given) and dw (+ db) via norm_workspace_bytes of partials.
size_t norm_workspace_bytes(int64_t M, int D);
hipError_t launch_norm_fwd(int ln, const void* x, const void* res, const void* w, const void* b,
                           void* y, void* sum, float* mean, float* rstd, int64_t M, int D,
                           float eps, hipStream_t stream);
hipError_t launch_norm_bwd(int ln, const void* dy, const void* dres, const void* x,
                           const void* w, const float* mean, const float* rstd, void* dx,
                           void* dw, void* db, int64_t M, int D, void* work, hipStream_t stream);
// Segmented backward (batched virtual workers): the M rows are nseg equal segments; segment z's
// dgamma / dbeta go to dw / db + z ostride (bf16). Workspace: norm_workspace_bytes_seg.
size_t norm_workspace_bytes_seg(int64_t M, int D, int nseg);
hipError_t launch_norm_bwd_seg(int ln, const void* dy, const void* dres, const void* x,
                               const void* w, const float* mean, const float* rstd, void* dx,
                               void* dw, void* db, int64_t M, int D, int nseg, int64_t ostride,
                               void* work, hipStream_t stream);
// qkv [B, S, (H + 2 KV) hd] -> q [B, H, S, hd], k / v [B, KV, S, hd] with interleaved-pair RoPE
// on q / k from fp32 cos / sin [S, hd / 2] (null: no rotation); backward is the inverse.
hipError_t launch_rope_fwd(const void* qkv, const float* cosb, const float* sinb, void* q, void* k,
                           void* v, int B, int S, int H, int KV, int hd, hipStream_t stream);
// grp > 1: dk / dv hold one gradient per QUERY head ([B, KV grp, S, hd]); each kv head's grp
// heads are summed (fp32) on the way into dqkv.
hipError_t launch_rope_bwd(const void* dq, const void* dk, const void* dv, const float* cosb,
                           const float* sinb, void* dqkv, int B, int S, int H, int KV, int hd,
                           hipStream_t stream, int grp = 1);
// Flash attention, head dim 128, causal or full, grouped-query heads (H % KV == 0):
// q [B, H, S, 128], k / v [B, KV, S, 128] -> o [B, S, H, 128], lse fp32 [B, H, S] (log2
// domain). Backward: dq [B, H, S, 128], dk / dv per query head [B, H, S, 128]; dsum [B, H, S]
// fp32 scratch (D = rowsum(dO * O)). csrc/kernels/flash_attn.hip.
// rescale_thr: deferred online-softmax rescale threshold in log2 units (0 = rescale at every
// max increase; 8 = scores exponentiated against a max up to 2^8 stale, see flash_attn.hip).
hipError_t launch_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B,
                            int H, int KV, int S, float scale, bool causal, hipStream_t stream,
                            float rescale_thr = 8.f);
hipError_t launch_flash_bwd(const void* q, const void* k, const void* v, const void* o,
                            const void* dout, const float* lse, float* dsum, void* dq, void* dk,
                            void* dv, int B, int H, int KV, int S, float scale, bool causal,
                            hipStream_t stream);
// SwiGLU over h = [a | b] ([M, 2F]): y = silu(a) * b; backward writes dh [M, 2F].
hipError_t launch_swiglu_fwd(const void* h, void* y, int64_t M, int F, hipStream_t stream);
hipError_t launch_swiglu_bwd(const void* dy, const void* h, void* dh, int64_t M, int F,
                             hipStream_t stream);
// Short-sequence attention (S % 32 == 0, S <= 128, head dim 64, no mask) on MFMA: reads the
// fused projection qkv [B, S, 3, H, 64], writes O [B, S, H * 64] and lse fp32 [B, H, S];
// backward writes dqkv in the fused layout.
hipError_t launch_attn_fwd(const void* qkv, void* out, float* lse, int B, int S, int H,
                           float scale, hipStream_t stream);
hipError_t launch_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse,
                           void* dqkv, int B, int S, int H, float scale, hipStream_t stream);
// Tree-ensemble split search, one level of T trees x L nodes: per (tree, node) the best
// (gain, candidate slot, bin) over its kk candidate features (feats [T, L, kk]) from the binned
// samples Xb [n, p] (uint8, B <= 64 bins) of that node (node_local [T, n], -1 = not in the level),
// with split statistics stat [T, n, 2] and node totals tot [T, L, 2]; crit 0 Gini, 1 XGBoost.
hipError_t launch_split_search(const uint8_t* Xb, const int* node_local, const float* stat,
                               const int* feats, const float* tot, int T, int L, int n, int p,
                               int kk, int B, int crit, float lam, float min_child,
                               float* out_gain, int* out_slot, int* out_bin, hipStream_t stream);
// Exact-threshold variant: B <= 128 rank bins, kk distinct candidate features per (tree, node)
// drawn in the kernel from `seed` (no feats tensor); returns the winning feature id.
hipError_t launch_split_search_sampled(const uint8_t* Xb, const int* node_local,
                                       const float* stat, const float* tot, int T, int L, int n,
                                       int p, int kk, int B, int crit, float lam, float min_child,
                                       uint64_t seed, float* out_gain, int* out_feat, int* out_bin,
                                       hipStream_t stream);
// Batched FISTA logistic lasso (lasso_prox.hip), problems along columns (B contiguous):
// r = (sigmoid(z + v0) - y) M / nb [n, B] (+ rsum = column sums of r), then the prox / restart /
// momentum step in place on v, beta [p, B] (tk, mom [B]; v0, b0 [B] when fitting an intercept).
// part: lasso_slices(p) x B floats; conv_part (optional): lasso_slices(p) x 2 x B (max |d|,
// max |beta| per row slice for the convergence test).
int lasso_slices(int p);
hipError_t launch_lasso_resid(const float* z, const float* v0, const float* y, const float* M,
                              const float* nb, float* r, float* rsum, int n, int B,
                              hipStream_t stream);
hipError_t launch_lasso_step(float* v, float* beta, const float* g, const float* step,
                             const float* lam, float alpha, float* tk, const float* rsum,
                             float* v0, float* b0, float* nbeta, float* mom, float* part,
                             float* conv_part, int p, int B, hipStream_t stream);
// Column sums of a bf16 [M, N] matrix (bias gradients), fp32 accumulation, bf16 out.
size_t colsum_workspace_bytes(int64_t M, int N);
hipError_t launch_colsum(const void* x, int64_t M, int N, void* out, void* work,
                         hipStream_t stream);
// Per-segment column sums (nseg equal row segments, (M / nseg) % 32 == 0): segment z -> out +
// z ostride. Workspace: colsum_workspace_bytes(M, N).
hipError_t launch_colsum_seg(const void* x, int64_t M, int N, int nseg, void* out,
                             int64_t ostride, void* work, hipStream_t stream);

// ResNet stem 7x7/s2/p3 convolution, C_in 3 or 4 -> 64, NHWC bf16 (stem_conv.hip).
// Forward: z = conv(x, wpk) with wpk the packed weights [64][224] (k = (ky*8 + kx)*4 + c, zero for
// kx = 7 / c >= C_in); part [grid][2][64] receives per-workgroup channel sums and sums of squares
// and, when mean != nullptr, mean / invstd (and running stats) are finalized from them.
// Backward: from g (ReLU-masked max-pool gradient) and its channel sums gsum, z, x and the forward
// mean / invstd, the weight gradient of the conv THROUGH the BatchNorm (dw [64][C][7][7] fp32) and
// dgamma / dbeta (fp32);
// part: grid x stem_wgrad_part_floats() floats, tot: stem_wgrad_part_floats() doubles.
int stem_fwd_grid(int N, int OH, int OW, int C);
int stem_bwd_grid(int N, int OH, int OW, int C);
size_t stem_wgrad_part_floats();
hipError_t launch_stem_conv_fwd(const void* x, const void* wpk, void* z, float* part, int grid,
                                float* mean, float* invstd, float* rmean, float* rvar, float eps,
                                float momentum, int N, int H, int W, int C, int OH, int OW,
                                hipStream_t stream);
hipError_t launch_stem_wgrad(const void* g, const void* z, const void* x, const float* mean,
                             const float* invstd, const void* gamma, const float* gsum,
                             float* part, int grid,
                             double* tot, void* dw, void* dgamma, void* dbeta, int N, int H,
                             int W, int C, int OH, int OW, hipStream_t stream,
                             const uint8_t* pidx = nullptr, float* cola_work = nullptr,
                             bool out_bf16 = false);
// pidx != nullptr: g is the 3x3 / s2 / p1 max-pool's output gradient [N][PH][PW][64] and pidx its
// forward argmax bytes; the kernel gathers the pool's input gradient itself and takes dbeta and
// mean(g) from its own sums (gsum unused). cola_work (always): stem_cola_work_floats floats.
// out_bf16: dw / dgamma / dbeta written as bf16 (else fp32).
// tot: stem_wgrad_tot_doubles() doubles.
size_t stem_wgrad_tot_doubles();
size_t stem_cola_work_floats(int N, int H, int W, int C);

// Weight gradient of a stride-1 1x1 conv, NHWC bf16: dW[co][ci] = sum_p dy[p][co] x[p][ci]
// (wgrad1x1.hip). Co, Ci multiples of 128, or Ci == 64 with Co a multiple of 256. part: splits x
// Co x Ci floats (wgrad1x1_plan); dw: bf16 (dw_bf16) or fp32 [Co][Ci]. pro_sc / pro_bi (fp32
// [Ci], both or neither): x is replaced by max(x * sc + bi, 0) (a BN + ReLU never materialised).
// pro: a dy or x prologue is applied (the plan then avoids the 1024-thread tile)
// pro: x prologue; dmode: dy prologue (0 none, 1 full, 2 mask, 3 BN-ReLU); cs: column sums
void wgrad1x1_plan(int64_t P, int Co, int Ci, int* splits, int* cps, bool pro = false,
                   int dmode = 0, bool cs = false);
// True when that call runs as one split on the LDS-DMA kernel without column sums: the kernel then
// writes dw itself (bf16 or fp32) and `part` may be null (long-K shapes, e.g. transformer linears).
bool wgrad1x1_direct(int64_t P, int Co, int Ci, bool pro = false, int dmode = 0, bool cs = false);
// dz_z / dz_mask / dz_a / dz_b / dz_c (all or none): dy is the output gradient of a BN + ReLU that
// consumed the conv output z = dz_z; the staging uses dz = a (mask ? dy : 0) + b z + c instead.
// General form: dmode 0 none, 1 the dz_* BN-backward prologue above, 2 dz = dz_a (mask ? dy : 0)
// + dz_c (no z), 3 dz = max(dy dz_a + dz_b, 0); Co = Ci = 64 also allowed. cs_part (splits x Co
// floats) / cs: column sums of the staged dz over the pixels -> cs [Co] (fp32).
hipError_t launch_wgrad1x1_ex(const void* dy, const void* x, float* part, void* dw, bool dw_bf16,
                              int64_t P, int Co, int Ci, const float* pro_sc, const float* pro_bi,
                              hipStream_t st, int dmode, const void* dz_z, const uint8_t* dz_mask,
                              const float* dz_a, const float* dz_b, const float* dz_c,
                              float* cs_part, float* cs);
hipError_t launch_wgrad1x1(const void* dy, const void* x, float* part, void* dw, bool dw_bf16,
                           int64_t P, int Co, int Ci, const float* pro_sc, const float* pro_bi,
                           hipStream_t stream, const void* dz_z = nullptr,
                           const uint8_t* dz_mask = nullptr, const float* dz_a = nullptr,
                           const float* dz_b = nullptr, const float* dz_c = nullptr);

// dW = sum of S fp32 partial slabs of n floats (n % 4 == 0), fixed order, bf16 or fp32 out.
// Weight gradient of a 3x3 / stride 2 / padding 1 conv (wgrad1x1.hip's LDS-DMA kernel on the
// implicit im2col of x): dy [N][H/2][W/2][Co], x [N][H][W][Ci] NHWC bf16 -> dw [Co][3][3][Ci]
// (bf16 or fp32). H, W even; Co, Ci multiples of 128; N (H/2) (W/2) % 32 == 0. zero: >= 512 B
// of zeros (the padding rows). part: splits x Co x taps Ci floats (wgrad3x3s2_plan).
// taps = 1: the 1x1 / stride 2 / padding 0 conv (a downsample's weight gradient, the single tap
// at (2 oh, 2 ow)) -> dw [Co][Ci].
bool wgrad3x3s2_plan(int N, int H, int W, int Co, int Ci, int* splits, int taps = 9);
hipError_t launch_wgrad3x3s2(const void* dy, const void* x, const void* zero, float* part,
                             void* dw, bool dw_bf16, int N, int H, int W, int Co, int Ci,
                             hipStream_t st, int taps = 9);
hipError_t launch_wgrad_fold(const float* part, int S, int64_t n, void* out, bool out_bf16,
                             hipStream_t st);
// 3x3 / stride 1 / padding 1 weight gradient with all nine taps per workgroup (wgrad3x3.hip):
// dy [B][H][W][Co], x [B][H][W][Ci] bf16, zero: >= 8 zero bf16, part: splits x Co x 9 x Ci floats,
// dw [Co][3][3][Ci] (bf16 or fp32). Co % 64 == 0, Ci == 64 or Ci % 128 == 0; the plan also needs a
// chunk geometry that fits LDS (false: the library's weight gradient).
bool wgrad3x3_direct_plan(int B, int H, int W, int Co, int Ci, int* splits, int* tci);
hipError_t launch_wgrad3x3_direct(const void* dy, const void* x, const void* zero, float* part,
                                  void* dw, bool dw_bf16, int B, int H, int W, int Co, int Ci,
                                  hipStream_t st);

// Fused 1x1 convolution forward (conv1x1.hip): y[M][N] = f(x)[src(m)][K] W[N][K]^T on NHWC bf16,
// f = identity or max(x * pro_sc + pro_bi, 0) per input channel (pro_sc != null), src(m) = m
// (stride 1) or the stride-2 pixel of an [*, H, W] input. With part / mean non-null also the
// training BatchNorm statistics of y (shifted by `shift`, e.g. the running mean; finalize updates
// rmean / rvar when non-null). K % 64 == 0, N % 64 == 0. part: conv1x1_bn_part_floats floats.
size_t conv1x1_bn_part_floats(int64_t M, int K, int N, bool pro);
// Optional output of a BN statistics finalize: the BN's affine sc = gamma invstd,
// bi = beta - mean sc (fp32, from the stored fp32 mean / invstd, bit-identical to bn_affine) for
// bf16 gamma / beta -- the consumer's bn_affine launch folded into the finalize.
struct BnAffineOut {
  const void* gamma;
  const void* beta;
  float* sc;
  float* bi;
};
hipError_t launch_conv1x1_bn_fwd(const void* x, const void* w, void* y, float* part,
                                 const float* pro_sc, const float* pro_bi, const float* shift,
                                 int64_t M, int K, int N, int stride, int H, int W, float* mean,
                                 float* invstd, float* rmean, float* rvar, float eps,
                                 float momentum, hipStream_t st, const BnAffineOut* aff = nullptr);

// Implicit-GEMM NHWC conv, stride 1, 1x1 (taps 1) or 3x3 padding 1 (taps 9), global_load_lds
// double-buffered (conv_gemm.hip): x [Nimg][H][W][C], w [N][taps][C], y [Nimg][H][W][N]; zero:
// >= 64 zero bf16 (padding rows).
// With part / mean non-null also the training BatchNorm statistics of y (shifted by `shift`),
// finalized like conv1x1_bn_fwd (running stats updated when rmean / rvar are non-null); part:
// conv_gemm_part_floats floats.
size_t conv_gemm_part_floats(int64_t M, int N);
// 3x3 (or 1x1) stride-1 implicit GEMM whose output y is the gradient of relu(bn(z)) (z [M][N],
// bn's affine sc / bi and batch statistics mean / invstd): also that backward's sums {sdz, sdzx}
// (part: conv_gemm_part_floats floats).
hipError_t launch_conv_gemm_bnsums(const void* x, const void* w, void* y, const void* zero,
                                   int Nimg, int H, int W, int C, int N, int taps, const void* z,
                                   const float* sc, const float* bi, const float* mean,
                                   const float* invstd, float* part, float* sdz, float* sdzx,
                                   hipStream_t st, void* dgamma = nullptr, void* dbeta = nullptr);
// dgamma / dbeta (bf16 [N], both or neither): also bf16(sdzx) / bf16(sdz), the BN's parameter
// gradients (bn_bwd_coeffs' values), written by the same finalize launch
hipError_t launch_bnbwd_sums_finalize(const float* part, int R, int BN, int N, const float* invstd,
                                      float* sdz, float* sdzx, hipStream_t st, float* fold,
                                      void* dgamma = nullptr, void* dbeta = nullptr);
// Data gradient dx [Nimg][2 Ho][2 Wo][Ci] of a stride-2 / padding-1 3x3 conv (even input) from dy
// [Nimg][Ho][Wo][Co] and wr [Ci][9 Co] (launch_conv3x3_wlayouts), as four output-parity-class
// implicit GEMMs of 4 / 2 / 2 / 1 taps. With z non-null also the sums of the BN + ReLU backward
// dx feeds, as launch_conv_gemm_bnsums (part: conv_gemm_s2dgrad_part_floats(Nimg Ho Wo, Ci)).
size_t conv_gemm_s2dgrad_part_floats(int64_t Mc, int N);
hipError_t launch_conv_gemm_s2dgrad(const void* dy, const void* wr, void* dx, const void* zero,
                                    int Nimg, int Ho, int Wo, int Co, int Ci, const void* z,
                                    const float* sc, const float* bi, const float* mean,
                                    const float* invstd, float* part, float* sdz, float* sdzx,
                                    hipStream_t st, void* dgamma = nullptr, void* dbeta = nullptr);
// The forward (wf [Co][9 Ci], k = (3 ky + kx) Ci + ci) and data-gradient (wr [Ci][9 Co], rotated
// and transposed: wr[ci][(3 ky + kx) Co + co] = w[co][ci][2 - ky][2 - kx]) GEMM layouts of a bf16
// 3x3 conv weight with strides s0..s3 (elements), in one launch; wf may be null.
hipError_t launch_conv3x3_wlayouts(const void* w, int Co, int Ci, int64_t s0, int64_t s1,
                                   int64_t s2, int64_t s3, void* wf, void* wr, hipStream_t st);
// The same for n weights in ceil(n / kWlMax) launches (descriptors passed by value); taps 1: a
// 1x1 weight [Co][Ci][1][1], wr = its transpose [Ci][Co] (a 1x1 data gradient's GEMM operand).
struct WlDesc {
  const void* w;
  void* wf;   // may be null
  void* wr;
  int64_t s0, s1, s2, s3;
  int Co, Ci, taps;
};
constexpr int kWlMax = 24;
hipError_t launch_conv3x3_wlayouts_multi(const WlDesc* d, int n, hipStream_t st);
// Stride-1 3x3 conv of 64 -> 64 channels on 56-wide images from an LDS-resident input patch
// (conv3x3p.hip; launch_conv_gemm / launch_conv_gemm_bnsums route there when eligible). ep 0: y
// only; 1: + shifted BN statistics; 2: + BN + ReLU backward sums (z, sc, bi, shift = mean); one
// partial row [2][64] per workgroup into part (*rows of them).
bool conv3x3p_eligible(int Nimg, int H, int W, int C, int N, int taps, int stride);
size_t conv3x3p_part_floats();
hipError_t launch_conv3x3p(const void* x, const void* w, void* y, const void* zero, int Nimg, int H,
                           int ep, float* part, const float* shift, const void* z, const float* sc,
                           const float* bi, hipStream_t st, int* rows);
hipError_t launch_conv_gemm(const void* x, const void* w, void* y, const void* zero, int Nimg,
                            int H, int W, int C, int N, int taps, hipStream_t st,
                            float* part = nullptr, const float* shift = nullptr,
                            float* mean = nullptr, float* invstd = nullptr,
                            float* rmean = nullptr, float* rvar = nullptr, float eps = 1e-5f,
                            float momentum = 0.1f, int stride = 1,
                            const BnAffineOut* aff = nullptr);
// BN statistics from a [ntn][R][2][BN] partial slab of shifted sums (conv1x1.hip's finalize).
// With `fold` (>= ntn * bn_part_fold_slices(R, ntn) * 2 * BN floats) a tall slab is first folded
// to bn_part_fold_slices rows per column tile by a wide kernel.
int bn_part_fold_slices(int R, int ntn);
hipError_t launch_bn_stats_finalize(const float* part, int R, int BN, int N, int64_t M,
                                   const float* shift, float eps, float momentum, float* mean,
                                   float* invstd, float* rmean, float* rvar, hipStream_t st,
                                   float* fold = nullptr, const BnAffineOut* aff = nullptr);

// Backward variants of the fused 1x1 conv (conv1x1.hip), stride 1, W given as [N][K] (for a data
// gradient: the forward weight transposed).
//   bnbwd: y = f(g) W^T with f = ca (mask ? g : 0) + cb z + cc per input channel (a BN + ReLU
//          backward applied while staging: dz never materialised).
//   link:  y = bf16(x W^T) + (lm ? link : 0) (masked residual gradient added in the epilogue); with
//          sz non-null also the backward sums of the BN + ReLU that consumes y: sdz = sum m y,
//          sdzx = sum m y (sz - mean) invstd (m = sm's bit). part: conv1x1_link_part_floats.
size_t conv1x1_link_part_floats(int64_t M, int K, int N);

// Identity-block tail without a stored z3 (ops.conv._RecomputeTailFn):
// y = max(conv1x1(max(x sc + bi, 0)) ep_sc + ep_bi + res, 0) with its ReLU bit mask ymask
// [M][N / 8]; the product is rounded to bf16 exactly as conv1x1_bn_fwd's statistics pass (same
// plan) rounded it, so the statistics describe the values normalised here.
hipError_t launch_conv1x1_bnres(const void* x, const void* w, void* y, uint8_t* ymask,
                                const float* pro_sc, const float* pro_bi, const float* ep_sc,
                                const float* ep_bi, const void* res, int64_t M, int K, int N,
                                hipStream_t st);
// Two-source GEMMs (K = K1 + K2 channels from g / x1 [M][K1] and x2 [M][K2]; w [N][K]):
// y = max(bf16([max(x1 sc + bi, 0) | max(x2 sc + bi, 0)] W^T) ep_sc + ep_bi (+ res), 0) and its
// ReLU bit mask: two BN'd convs summed before a ReLU (a downsample block's tail) in one GEMM.
// x1 staged as max(x1 sc1 + bi1, 0) (sc1 / bi1 [K1]), x2 as max(x2 sc2 + bi2, 0) ([K - K1]) or as
// is (sc2 / bi2 null)
hipError_t launch_conv1x1_cat_bnres(const void* x1, const void* x2, const float* sc1,
                                    const float* bi1, const float* sc2, const float* bi2,
                                    const void* w, const float* ep_sc, const float* ep_bi,
                                    const void* res, void* y, uint8_t* ymask, int64_t M, int K1,
                                    int K, int N, hipStream_t st);
// y = [(mask ? g : 0) | f2(x2)] w^T + bias: f2 = max(x2 sc2 + bi2, 0) ([K - K1]) or the identity
// (sc2 / bi2 null); bias [N] or null. mean / invstd (optional): also the sums {sdz, sdzx} of the
// backward of the BN + ReLU whose input is x2 (N = K - K1, needs sc2 / bi2: its mask is
// recomputed from x2); part: conv1x1_cat_part_floats floats
hipError_t launch_conv1x1_cat(const void* g, const uint8_t* mask, const void* x2, const float* sc2,
                              const float* bi2, const float* bias, const void* w, void* y,
                              int64_t M, int K1, int K, int N, hipStream_t st,
                              const float* mean = nullptr, const float* invstd = nullptr,
                              float* part = nullptr, float* sdz = nullptr, float* sdzx = nullptr,
                              void* dgamma = nullptr, void* dbeta = nullptr);
size_t conv1x1_cat_part_floats(int64_t M, int K, int N);
hipError_t launch_conv1x1_bnbwd(const void* g, const void* z, const uint8_t* mask, const float* ca,
                                const float* cb, const float* cc, const void* w, void* y,
                                int64_t M, int K, int N, hipStream_t st);
// (lm null: the link is added everywhere)
hipError_t launch_conv1x1_link(const void* x, const void* w, void* y, const void* link,
                               const uint8_t* lm, const void* sz, const uint8_t* sm,
                               const float* mean, const float* invstd, float* part, float* sdz,
                               float* sdzx, int64_t M, int K, int N, hipStream_t st);
// dz = ca (mask ? dy : 0) + cb z + cc coefficients of a training BN + ReLU backward from its sums
// (sdz, sdzx); dgamma = sdzx, dbeta = sdz (bf16).
// 1x1 data gradient y = x w^T (x = dY [Nimg][H][W][K], w [N][K]) plus, at the even pixels, a
// stride-2 conv's compact data gradient link [Nimg][ceil(H/2)][ceil(W/2)][N] (conv1x1.hip EL).
hipError_t launch_conv1x1_link_s2(const void* x, const void* w, void* y, const void* link,
                                  int Nimg, int H, int W, int K, int N, hipStream_t st);
// BN training statistics (mean, invstd; running stats updated when given) of z = y W^T from the
// Gram matrix G = y^T y [P][P] and column sums cy [P] of y over M rows; W [Co][P] bf16 (conv1x1.hip).
// part: fp64 scratch [P / 64][Co]; P % 64 == 0. sc != nullptr: also the BN affine
// sc = gamma invstd, bi = beta - mean sc (gamma / beta bf16 [Co]) bit-identical to launch_bn_affine.
hipError_t launch_bn_stats_gram(const float* G, const float* cy, const void* w, int P, int Co,
                                int64_t M, float eps, float momentum, float* mean, float* invstd,
                                float* rmean, float* rvar, double* part, hipStream_t st,
                                const void* gamma = nullptr, const void* beta = nullptr,
                                float* sc = nullptr, float* bi = nullptr);
// Recompute-tail backward algebra (tail_prep.hip): from conv3's W bf16 [Co][p], P = u^T y2 and
// s = sum u (fp32), y2's Gram / column sums and bn3's gamma (bf16) / mean / invstd: bn3's backward
// coefficients, dgamma / dbeta (bf16 [Co]), conv3's weight gradient dW (bf16 [Co][p], skipped when
// null), w_cat = [W^T diag(a) | W^T diag(b) W] (bf16 [p][Co + p]) and bias = W^T c (fp32 [p]).
// work: tail_bwd_prep_work_floats(Co, p) fp32 scratch. Co % 64 == 0, p % 64 == 0.
hipError_t launch_tail_bwd_prep(const void* W, const float* P, const float* s, const float* gram,
                                const float* cy, const void* gamma, const float* mean,
                                const float* invstd, int Co, int p, int64_t M, float* work,
                                void* dW, void* wcat, float* bias, void* dgamma, void* dbeta,
                                hipStream_t st);
size_t tail_bwd_prep_work_floats(int Co, int p);
// w_cat = [diag(s1) w1 | diag(s2) w2] (bf16 [Co][k1 + k2], each product rounded once from fp32)
// and bias = b1 + b2 (fp32 [Co]) in one launch (the downsample recompute tail's folded weights).
hipError_t launch_scaled_cat_bias(const void* w1, const float* s1, int k1, const void* w2,
                                  const float* s2, int k2, const float* b1, const float* b2,
                                  int Co, void* out, float* bias, hipStream_t st);
hipError_t launch_bn_bwd_coeffs(const float* sdz, const float* sdzx, const void* gamma,
                                const float* mean, const float* invstd, int C, int64_t M,
                                float* ca, float* cb, float* cc, void* dgamma, void* dbeta,
                                hipStream_t st);

// Batched dual C-SVC (svm_smo.hip): one wave per problem b, SMO with second-order working-set
// selection on K [B][nmax][nmax] fp64 (problem b uses its leading ns[b] x ns[b] block), labels y
// [B][nmax] (> 0 -> +1), box C [B]; alpha / grad (dual gradient) [B][nmax], iters [B].
// nmax <= smo_max_n().
int smo_max_n();
hipError_t launch_smo(const double* K, const double* y, const int* ns, int B, int nmax,
                      const double* C, double tol, int max_iter, double* alpha, double* grad,
                      int* iters, hipStream_t stream);

// Dense NT GEMM with fused epilogues (gemm.hip): y[M][N] = epi(A[M][K] B[N][K]^T), bf16 in/out,
// fp32 accumulation. EP_STORE: + bias[N] (bf16, optional); EP_GELU: aux = h = bf16(acc + bias),
// y = bf16(gelu(h)); EP_DGELU: y = bf16(bf16(acc) * gelu'(aux)) and, when part is set, fp32
// column sums of y per 128-row block into part [M / 128][N]. M % 256 == 0, N % 256 == 0,
// K % 64 == 0, leading dimensions % 8 == 0, 16-B aligned bases.
enum { EP_STORE = 0, EP_GELU = 1, EP_DGELU = 2, EP_CONV_ST = 3, EP_CONV_BB = 4 };
struct GemmArgs {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* y;
  uint16_t* aux;
  const uint16_t* bias;
  float* part;
  const uint16_t* cin;    // EP_STORE: y = bf16(bf16(acc + bias) + cin), cin [M][ldy] (may be y)
  int64_t M, N, K;
  int64_t lda, ldb, ldy;
  // implicit-GEMM 3x3 / stride 1 / padding 1 convolution (conv = 1): A = the NHWC input x
  // [Nimg][H][W][C] gathered per tap (a = x, K = 9 C, b = wf [N][9 C]); padded taps read `zero`.
  // EP_CONV_ST: the BN statistics of the stored bf16 output (minus shift[n]) as partial rows
  // part[(ntile R + WMR mtile + wave row)][2][TN], R = WMR M / TM (gemm_conv_tm; WMR = TM / 128,
  // TN = 65536 / TM; the square tile: R = 2 M / 256, TN = 256); EP_CONV_BB: instead the sums of
  // the BN + ReLU backward that y feeds (z = sz [M][N], ReLU bit z ep_sc + ep_bi > 0, shift = mean)
  int conv, C, H, W;       // H, W: the output grid
  int s2, IH, IW;         // conv: stride 2 with an IH x IW input grid (s2 = 1), else unused
  int gm;                 // gemm.hip tile order: > 1 = groups of gm m-tiles, m fastest
  const uint16_t* zero;
  const float* shift;
  const uint16_t* sz;
  const float* ep_sc;
  const float* ep_bi;
};
bool gemm_nt_eligible(int64_t M, int64_t N, int64_t K);
hipError_t launch_gemm_nt(const GemmArgs& a, int ep, hipStream_t st);
// 128 x 128-tile NT GEMM (gemm128.hip), EP_STORE only (bias, cin): M % 128 == 0, N % 128 == 0,
// K % 64 == 0 -- the grids that 256 x 256 tiles leave under-filled.
bool gemm128_eligible(int64_t M, int64_t N, int64_t K);
hipError_t launch_gemm128_nt(const GemmArgs& a, hipStream_t st);
// the conv form (a.conv = 1; M % 256 == 0, N % 256 == 0, C % 64 == 0), ep EP_STORE /
// EP_CONV_ST / EP_CONV_BB (conv_gemm.hip's 256 x 256 path for stride-1 3x3 convs)
bool gemm_conv_eligible(int64_t M, int N, int C);
// the m-tile launch_gemm_conv takes: 256 (256 x 256 tiles, N % 256 == 0), 512 (512 x 128 tiles:
// 128-channel convs with enough tiles, CML_GEMM2_TALL), 0 = not eligible; partial slabs of
// EP_CONV_ST / EP_CONV_BB then have R = (M / TM) (TM / 128) rows of 2 x (65536 / TM) floats
int gemm_conv_tm(int64_t M, int N, int C);
hipError_t launch_gemm_conv(const GemmArgs& a, int ep, hipStream_t st);
// 4-wave 256 x 256-tile GEMM (gemm_w4.hip), EP_STORE (bias, cin), any operand layout: mode bit 0 =
// A stored [K][M] (lda >= M), bit 1 = B stored [K][N]; K % 64 == 0, M, N multiples of 8.
bool gemm_w4_eligible(int64_t M, int64_t N, int64_t K, int mode);
hipError_t launch_gemm_w4(const GemmArgs& a, int mode, hipStream_t st);
// out[s][n] = sum of the 128-row partial column sums of segment s of M rows (nseg equal
// segments, fixed order); out bf16 [nseg][ldo] or fp32 when out_f32
hipError_t launch_colsum_fold(const float* part, int64_t M, int N, int nseg, void* out, int64_t ldo,
                              int out_f32, hipStream_t st);

}  // namespace cml
