/*
 * catseg_hip_train.h — C ABI of the training-side kernels in libcatseg_hip.so: the
 * backward of the CAT-Seg aggregation head and the CATSeg ConvTranspose upsamplers
 * (reference cat_seg/cat_seg_model.py:57-75,189-203,
 * cat_seg/modeling/transformer/model.py:51-225,256-424,520-555, train_net.py:174-258).
 *
 * Conventions are those of catseg_hip.h: device pointers, int64 sizes / strides in
 * ELEMENTS, the HIP stream as `void*`, int status (catseg_last_error()), caller-allocated
 * outputs and workspaces (size queries below), no allocation or synchronisation inside,
 * hipGraph-capturable.  Everything here is fp32 (the reference trains in fp32).  Every
 * reduction runs in a fixed order on a grid that depends only on the shape: gradients are
 * bit-reproducible.  `beta` flags: 0 = overwrite, 1 = accumulate into the output.
 * The Python mirror is cat-seg_amd/cat_seg/train_ops.py; the autograd functions that use
 * these entry points are cat-seg_amd/cat_seg/training.py.
 */
#ifndef CATSEG_HIP_TRAIN_H
#define CATSEG_HIP_TRAIN_H
#include <stdint.h>
#include "catseg_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------
 * catseg_gemm_ex — C[m][n] = alpha * sum_k A(m,k) B(k,n) + beta * C[m][n], fp32, exact-f32 MFMA.
 * A(m,k) = A[m*a_sm + k*a_sk], B(k,n) = B[k*b_sk + n*b_sn]; one stride of each operand must be 1
 * (its contiguous dimension, read as 16-byte vectors: that extent and the other stride % 4 == 0).
 * Serves every nn.Linear backward (dX = dY.W: A = dY rows, B = W; dW = dY^T.X: a_sm = 1, K = rows)
 * and the cost-volume einsum backward (model.py:648-652).  Large K is split over the grid into
 * fp32 partials reduced in a fixed order: workspace >= catseg_gemm_ex_workspace(M, N, K) bytes.
 * ------------------------------------------------------------------------- */
typedef struct {
  const void* A; int64_t a_sm, a_sk;
  const void* B; int64_t b_sk, b_sn;
  int64_t M, N, K;
  void* C; int64_t ldc;
  float alpha; int beta;
  void* workspace; int64_t workspace_bytes;
  /* optional activation-backward epilogue (act != CATSEG_ACT_NONE; beta must be 0): C[m][n] =
   * alpha * sum_k A B * act'(act_u[m*ld_u + n]) -- the MLP's dU = (dY . W2) * act'(U) in one pass
   * (act_u may be C itself: each element is read before it is written by the same lane) */
  const void* act_u; int64_t ld_u; int act;
} CatsegGemmExArgs;
int catseg_gemm_ex(const CatsegGemmExArgs* args, void* stream);
int64_t catseg_gemm_ex_workspace(int64_t M, int64_t N, int64_t K);

/* catseg_colsum — out[c] = alpha * sum_r x[r*ld + c] + beta * out[c]: bias gradients of Linear /
 * Conv2d / ConvTranspose2d.  workspace >= catseg_colsum_workspace(rows, cols) bytes. */
int catseg_colsum(const float* x, int64_t ld, int64_t rows, int64_t cols, float* out, float alpha, int beta,
                  void* workspace, int64_t workspace_bytes, void* stream);
int64_t catseg_colsum_workspace(int64_t rows, int64_t cols);

/* ---------------------------------------------------------------------------
 * Normalisation / activation backward
 * ------------------------------------------------------------------------- */
/* catseg_layernorm_backward — nn.LayerNorm backward (model.py:152,158,233,368-369; the LN
 * statistics are recomputed from x): dx (+)= rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma;
 * dgamma (+)= sum_r dy xhat, dbeta (+)= sum_r dy (NULL both to skip; then no workspace needed).
 * cols in {64, 128, 256, 512, 768, 1024}.  workspace >= catseg_layernorm_backward_workspace bytes. */
int catseg_layernorm_backward(const float* x, int64_t ld_x, const float* gamma, const float* dy, int64_t ld_dy,
                              float* dx, int64_t ld_dx, int acc_dx, int64_t rows, int64_t cols, float eps,
                              float* dgamma, float* dbeta, int acc_param, void* workspace, int64_t workspace_bytes,
                              void* stream);
int64_t catseg_layernorm_backward_workspace(int64_t rows, int64_t cols);

/* catseg_act_forward — a = act(u); catseg_act_backward — du = dy * act'(u).  act: CATSEG_ACT_RELU,
 * _GELU (exact erf, timm Mlp model.py:159), _QUICKGELU (model_vpt.py:165-167); n % 4 == 0. */
int catseg_act_forward(const float* u, float* a, int64_t n, int act, void* stream);
int catseg_act_backward(const float* u, const float* dy, float* du, int64_t n, int act, void* stream);

/* catseg_groupnorm_stats_rows — nn.GroupNorm statistics (model.py:529,532) of an NHWC map
 * x[S][HW][C], groups of cpg channels: mean / rstd [S][C/cpg] (biased variance, eps).  Pixel chunks
 * of 16384/C pixels reduce {sum, M2} in registers, chunks combine in order (pairwise update).
 * C/4 a power of two <= 256, cpg % 4 == 0, x 16-byte aligned.
 * workspace >= catseg_groupnorm_stats_rows_workspace(S, HW, C, cpg) bytes. */
int catseg_groupnorm_stats_rows(const float* x, int64_t S, int64_t HW, int C, int cpg, float eps, float* mean,
                                float* rstd, void* workspace, int64_t workspace_bytes, void* stream);
int64_t catseg_groupnorm_stats_rows_workspace(int64_t S, int64_t HW, int C, int cpg);

/* catseg_groupnorm_relu_backward — backward of y = relu(GroupNorm(x)) (model.py:529-533) given
 * dy = dL/dy: dx (overwritten), dgamma / dbeta (+= when acc_param).  C/4 a power of two <= 256,
 * cpg % 4 == 0, x / dy / dx / gamma / beta 16-byte aligned.
 * workspace >= catseg_groupnorm_relu_backward_workspace(S, HW, C) bytes. */
int catseg_groupnorm_relu_backward(const float* x, const float* dy, float* dx, int64_t S, int64_t HW, int C, int cpg,
                                   const float* mean, const float* rstd, const float* gamma, const float* beta,
                                   float* dgamma, float* dbeta, int acc_param, void* workspace,
                                   int64_t workspace_bytes, void* stream);
int64_t catseg_groupnorm_relu_backward_workspace(int64_t S, int64_t HW, int C);

/* catseg_l2normalize_backward — F.normalize backward (model.py:649-650, cat_seg_predictor.py:216):
 * dx[outmap(r)] (+)= (dy[r] - y (y . dy[r])) / max(|x|, eps), x = x[inmap(r)], y = x / max(|x|, eps). */
int catseg_l2normalize_backward(const float* x, int64_t ld_x, CatsegRowMap inmap, const float* dy, int64_t ld_dy,
                                float* dx, int64_t ld_dx, CatsegRowMap outmap, int beta, int64_t rows, int64_t cols,
                                float eps, void* stream);

/* catseg_axpby — out = alpha * x + beta * y (y may be NULL), n % 4 == 0: the residual branches'
 * gradient sums.  catseg_add_dev_scalar — x[i] += *s (s a device scalar: the head conv's bias
 * without a host read, model.py:634). */
int catseg_axpby(const float* x, const float* y, float* out, int64_t n, float alpha, float beta, void* stream);
/* catseg_scatter_rows — out[idx[r]] = in[r] (fp32 rows): the backward of the text encoder's EOT gather
 * (model_vpt.py:436, catseg_eot_gather). */
int catseg_scatter_rows(const float* in, int64_t ld_in, const int32_t* idx, int64_t rows, int64_t cols, float* out,
                        int64_t ld_out, void* stream);
int catseg_add_dev_scalar(float* x, int64_t n, const float* s, void* stream);

/* ---------------------------------------------------------------------------
 * Reductions and layout transposes of the rows layout X[b][t][p][c]
 * ------------------------------------------------------------------------- */
/* catseg_sum_classes — out[b*HW + p] (+)= sum_t x[(b*T + t)*HW + p] (C columns, row strides ld):
 * the backward of guidance repeated over classes (model.py:249 repeat, :551-554 repeat). */
int catseg_sum_classes(const float* x, int64_t ld_x, int64_t B, int T, int64_t HW, int C, float* out, int64_t ld_out,
                       int beta, void* stream);
/* catseg_sum_pixels — out[t] (+)= sum_{b, p} x[(b*T + t)*HW + p]: the backward of the per-class
 * text guidance broadcast over images and pixels (model.py:405-409). */
int catseg_sum_pixels(const float* x, int64_t ld_x, int64_t B, int T, int64_t HW, int C, float* out, int64_t ld_out,
                      int beta, void* stream);
/* catseg_avgpool_backward_rows — AvgPool2d(ph, pw) backward (model.py:374-385) on [S][H][W][C]. */
int catseg_avgpool_backward_rows(const float* dxp, int64_t S, int H, int W, int C, int ph, int pw, float* dx, int beta,
                                 void* stream);
/* catseg_upsample_ac_backward_rows — backward of bilinear(align_corners=True) [S][Hp][Wp][C] ->
 * [S][H][W][C] (model.py:415-416), gather form (no atomics). */
int catseg_upsample_ac_backward_rows(const float* dy, int64_t S, int H, int W, int C, int Hp, int Wp, float* dxp,
                                     int beta, void* stream);
/* catseg_convt_gather — the gradient of a ConvTranspose2d(k, stride k) output [S][hin*k][win*k] (pixel
 * stride ld, cout channels) as GEMM rows g[(s, y, x)][(ky, kx, co)]: with it dX = g . Wg and
 * dWg = g^T . X (catseg_gemm_ex), Wg = the ConvTranspose weight as [(ky, kx, co)][ci]
 * (cat_seg_model.py:81-82, model.py:546). */
int catseg_convt_gather(const float* dout, int64_t ld, int64_t S, int hin, int win, int k, int cout, float* g,
                        void* stream);

/* ---------------------------------------------------------------------------
 * Attention backward
 * ------------------------------------------------------------------------- */
/* catseg_window_attention_backward — WindowAttention backward (model.py:86-114, shift / -100 region mask
 * of model.py:161-216), rows as catseg_attention mode 1: q/k/v the forward projections (heads
 * concatenated, scale NOT applied), o the forward attention output, dout = dL/do.  Writes dq, dk, dv
 * (row stride ld_dqkv, head h at columns h*head_dim).  head_dim 32, window^2 % 16 == 0, <= 144. */
typedef struct {
  const void* q; const void* k; const void* v; int64_t ld_qkv;
  const void* o; int64_t ld_o;
  const void* dout; int64_t ld_dout;
  void* dq; void* dk; void* dv; int64_t ld_dqkv;
  int64_t S; int img_h, img_w, window, shift, n_heads, head_dim; float scale;
} CatsegWinAttnBwdArgs;
int catseg_window_attention_backward(const CatsegWinAttnBwdArgs* args, void* stream);

/* catseg_attention_backward — dense softmax attention backward for catseg_attention mode 0 rows
 * (the CLIP blocks' nn.MultiheadAttention, model_vpt.py:169-182,202-206; causal = the text encoder's
 * triu mask, model_vpt.py:400-406): sequence s, token i at row s*seq_len + i; q/k/v the forward
 * projections (scale not applied), o the forward output, dout = dL/do.  Writes dq, dk, dv.
 * head_dim 64.  workspace >= catseg_attention_backward_workspace bytes (softmax statistics). */
typedef struct {
  const void* q; const void* k; const void* v; int64_t ld_qkv;
  const void* o; int64_t ld_o;
  const void* dout; int64_t ld_dout;
  void* dq; void* dk; void* dv; int64_t ld_dqkv;
  int64_t n_seq; int seq_len; int n_heads; int head_dim; float scale; int causal;
  void* workspace; int64_t workspace_bytes;
} CatsegAttnBwdArgs;
int catseg_attention_backward(const CatsegAttnBwdArgs* args, void* stream);
int64_t catseg_attention_backward_workspace(int64_t n_seq, int seq_len, int n_heads);

/* catseg_linear_attention_backward — LinearAttention backward (model.py:256-286) for the rows of
 * catseg_linear_attention: dy = dL/d(attention output).  Writes dq, dk, dv; with n_pad > 0 also
 * dk_pad / dv_pad [heads*head_dim] = the gradients of the padding tokens' constant k / v projections
 * (summed over their n_pad copies and every pixel).  4 heads x 32.  workspace >=
 * catseg_linear_attention_backward_workspace(B, HW) bytes when n_pad > 0. */
typedef struct {
  const void* q; const void* k; const void* v; int64_t ld_qkv;
  const void* dy; int64_t ld_dy;
  void* dq; void* dk; void* dv; int64_t ld_dqkv;
  int64_t B; int T; int HW; int n_heads; int head_dim;
  int n_pad; const float* k_pad; const float* v_pad; float eps;
  float* dk_pad; float* dv_pad;
  void* workspace; int64_t workspace_bytes;
} CatsegLinAttnBwdArgs;
int catseg_linear_attention_backward(const CatsegLinAttnBwdArgs* args, void* stream);
int64_t catseg_linear_attention_backward_workspace(int64_t B, int HW);

/* ---------------------------------------------------------------------------
 * Convolutions (stride 1, pad = ksize / 2, NHWC)
 * ------------------------------------------------------------------------- */
/* catseg_conv2d_nhwc — y[p][co] = alpha * act(sum_{tap, ci} x[p + tap][ci] w[(tap*cin + ci)*ld_w + co]
 * + bias[co]) + beta * y[p][co]; act NONE / RELU.  Forward of the guidance projections and DoubleConv
 * (model.py:528-531,616,627), and every conv's data gradient (x = dY, w = the flipped, transposed
 * weight).  catseg_conv2d_wgrad — dw[(tap*cin + ci)*cout + co] = alpha * sum_p x[p + tap][ci] y[p][co]
 * + beta * dw (y = dY; weight gradient, corr_embed's 7x7 included); workspace >=
 * catseg_conv2d_wgrad_workspace(args) bytes.  cout % 4 == 0. */
typedef struct {
  const void* x; int64_t ld_x;
  int64_t S; int H, W; int cin;
  const void* w; int64_t ld_w;
  int cout; int ksize; int pad;
  const float* bias; int act;
  void* y; int64_t ld_y;
  float alpha; int beta;
  void* dw;
  void* workspace; int64_t workspace_bytes;
} CatsegConv2dArgs;
int catseg_conv2d_nhwc(const CatsegConv2dArgs* args, void* stream);
int catseg_conv2d_wgrad(const CatsegConv2dArgs* args, void* stream);
int64_t catseg_conv2d_wgrad_workspace(const CatsegConv2dArgs* args);

/* catseg_corr_embed_backward_input — the data gradient of corr_embed's Conv2d(1, D, k, pad k/2)
 * (model.py:613,654-659): dcorr[s][q] = sum_{tap, co} dX[s][q - tap][co] weight[co][tap]; dX rows
 * [S*H*W][D], weight [D][k*k] (the Conv2d weight (D, 1, k, k)), dcorr [S][H*W].  D % 32 == 0. */
int catseg_corr_embed_backward_input(const float* dX, const float* weight, float* dcorr, int64_t S, int H, int W,
                                     int D, int ksize, void* stream);

/* catseg_head_conv_backward — the head conv C -> 1 (3x3, model.py:634,679) backward: x the forward
 * input [S][H][W][C], dlogits [S][H][W]; dx [S][H][W][C] (overwritten), dw [9][C] (tap-major,
 * overwritten).  The bias gradient is catseg_colsum over dlogits.  workspace >=
 * catseg_head_conv_backward_workspace bytes. */
int catseg_head_conv_backward(const float* x, const float* dlogits, const float* weight, float* dx, float* dw,
                              int64_t S, int H, int W, int C, void* workspace, int64_t workspace_bytes, void* stream);
int64_t catseg_head_conv_backward_workspace(int64_t S, int H, int W, int C);

/* ---------------------------------------------------------------------------
 * Optimizer: torch.optim.AdamW inside the reference's FullModelGradientClippingOptimizer
 * (train_net.py:228-253), every parameter of every group in one multi-tensor pass.
 * ------------------------------------------------------------------------- */
/* One parameter tensor (fp32, contiguous, numel elements) and its group's hyper-parameters; an array
 * of these lives in DEVICE memory.  bias_correction1/2 = 1 - beta^step of the step being taken. */
typedef struct {
  float* param; float* grad; float* exp_avg; float* exp_avg_sq;
  int64_t numel;
  float lr; float weight_decay; float bias_correction1; float bias_correction2;
} CatsegAdamWTensor;
/* The chunk table: 4096-element chunks over the tensors, entry = (tensor << 40) | chunk; host-side,
 * computed once per parameter set (catseg_adamw_chunks gives its length). */
int64_t catseg_adamw_chunks(const int64_t* numels, int n_tensors);
int catseg_adamw_chunk_table(const int64_t* numels, int n_tensors, int64_t* table);
/* catseg_adamw_step — with max_grad_norm > 0: total = ||all grads||_2 (fixed-order sum), coef =
 * min(1, max_grad_norm / (total + 1e-6)), grads scaled in place (torch.nn.utils.clip_grad_norm_),
 * norm_out[0] = total, norm_out[1] = coef (device floats; workspace >= n_chunks floats); then the AdamW
 * update of torch.optim.AdamW (decoupled weight decay, lerp first moment, bias-corrected step). */
int catseg_adamw_step(const CatsegAdamWTensor* tensors, const int64_t* chunk_table, int64_t n_chunks, float beta1,
                      float beta2, float eps, float max_grad_norm, float* norm_out, void* workspace,
                      int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CATSEG_HIP_TRAIN_H */
