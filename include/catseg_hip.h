/*
 * catseg_hip.h — C ABI of libcatseg_hip.so, the MI355X (gfx950) kernels of the
 * CAT-Seg dense-inference hot path.
 *
 * Conventions
 *   - Plain pointers to DEVICE memory, int64 sizes/strides in ELEMENTS, a dtype
 *     enum, and the HIP stream as `void*` (a hipStream_t; NULL = default stream).
 *   - Caller-allocated outputs and workspaces; no entry point allocates,
 *     synchronises or copies to the host, so every one is hipGraph-capturable.
 *   - Return 0 on success, < 0 on error; catseg_last_error() then holds a
 *     thread-local message.  Arguments are validated on the host before launch.
 *   - Row-major, channels-last layouts.  The aggregation cost tensor is
 *     X[b][t][h][w][c] (the reference's B C T H W, model.py:683-725, with C moved
 *     innermost), i.e. rows of `hidden` channels ordered (image, class, pixel).
 *
 * Each entry names the reference function(s) it replaces (paths relative to the
 * reference repo root).  The Python host mirror is cat-seg_amd/cat_seg/ops.py.
 * Kernel variants are chosen automatically per shape; the A/B knobs used by the tests and
 * tools/ live behind a separate diagnostics header (catseg_hip_tuning.h), not in this ABI.
 */
#ifndef CATSEG_HIP_H
#define CATSEG_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { CATSEG_OK = 0, CATSEG_ERR_ARG = -1, CATSEG_ERR_HIP = -2 };
enum { CATSEG_F32 = 0, CATSEG_BF16 = 1, CATSEG_FP8 = 2 /* OCP e4m3fn bytes */ };
enum { CATSEG_ACT_NONE = 0, CATSEG_ACT_RELU = 1, CATSEG_ACT_GELU = 2, CATSEG_ACT_QUICKGELU = 3,
       CATSEG_ACT_SIGMOID = 4 };

const char* catseg_last_error(void);
int catseg_abi_version(void);

/* r(m) = ((m / d1) % m1) * s1 + ((m / d2) % m2) * s2 + off   (identity: {1,BIG,1,1,1,0,0}) */
typedef struct {
  int64_t d1, m1, s1, d2, m2, s2, off;
} CatsegRowMap;

/* ---------------------------------------------------------------------------
 * catseg_gemm — every dense contraction on the path.  Replaces nn.Linear /
 * F.linear calls of model_vpt.py:193-236 (ViT q/k/v, out_proj, c_fc+QuickGELU,
 * c_proj), model_vpt.py:312 (ln_post @ proj), model_vpt.py:289 (patch conv as
 * im2col GEMM), model.py:77-112 + 159 (Swin q/k/v/proj/Mlp), model.py:327-366
 * (class-attention q/k/v/MLP), model.py:648-652 (cost-volume einsum),
 * model.py:546 / cat_seg_model.py:81-82 (ConvTranspose2d k=s via store_mode 1).
 *   out[store(m,n)] = act(A[amap(m),:] . W[n,:] + bias[n] + add[addmap(m), n<add_ncols]) * alpha
 *                     + res[m,n] + res2[m,n]
 * W: [N][K] (nn.Linear layout).  bias: fp32 [N] or NULL.  add/res/res2/out share
 * dtype_out.  store_mode 1: m = (s, y, x) over (cvt_hin, cvt_win), n = (ky, kx, co),
 * out NHWC [s][y*k+ky][x*k+kx][co].
 * ------------------------------------------------------------------------- */
typedef struct {
  const void* A; int64_t lda; CatsegRowMap amap;
  const void* W; int64_t ldw;
  int64_t M, N, K;
  const float* bias;
  const void* add; int64_t ld_add; CatsegRowMap addmap; int64_t add_ncols;
  int act; float alpha;
  const void* res; int64_t ld_res;
  const void* res2; int64_t ld_res2;
  void* out; int64_t ldo;
  int store_mode; int cvt_k, cvt_hin, cvt_win, cvt_cout;
  int dtype_a, dtype_out;
} CatsegGemmArgs;
int catseg_gemm(const CatsegGemmArgs* args, void* stream);

/* ---------------------------------------------------------------------------
 * fp8 ViT GEMMs ("fp8 MFMA ViT GEMMs").  The reference runs the
 * same nn.Linear calls (model_vpt.py:193-236) in fp32/fp16; here A and W are OCP e4m3
 * with one fp32 dequant scale per row of each (scale_a [M], scale_w [N], 16B aligned):
 *   out = epilogue( (A8[r,:] . W8[n,:]) * scale_a[r] * scale_w[n] ), r = amap(m)   (epilogue as catseg_gemm)
 * dtype_a = CATSEG_FP8; K, lda, ldw in bytes (K % 128 == 0); N % 128 == 0; row-major
 * store only; dtype_out f32 or bf16.  Block-scaled K=128 MFMA at unit block scales.
 * ------------------------------------------------------------------------- */
int catseg_gemm_fp8(const CatsegGemmArgs* args, const float* scale_a, const float* scale_w, void* stream);

/* Per-row e4m3 quantization: scale[r] = max|x[r,:]| / 448, q[r,c] = rne_e4m3(x[r,c] / scale[r]).
 * x: f32 or bf16 (dtype), q: bytes.  cols <= 4096; cols, ld_x, ld_q multiples of 8.  Used for the
 * weights at load and the activations ahead of catseg_gemm_fp8. */
int catseg_quant_fp8_rows(const void* x, int dtype, int64_t ld_x, int64_t rows, int64_t cols, void* q,
                          int64_t ld_q, float* scale, void* stream);
/* LayerNorm straight to e4m3 rows (ln_1 / ln_2 ahead of the fp8 QKV / c_fc GEMMs,
 * model_vpt.py:208-217): y = LN(x[inmap(r)]) in fp32 as catseg_layernorm, then quantized as
 * catseg_quant_fp8_rows.  cols <= 4096, multiples of 8. */
int catseg_layernorm_fp8(const void* x, int64_t ld_x, CatsegRowMap inmap, int dtype_x, void* q, int64_t ld_q,
                         float* scale, const float* gamma, const float* beta, int64_t rows, int64_t cols, float eps,
                         void* stream);


/* ---------------------------------------------------------------------------
 * Row-block kernels over the 128-channel cost-embedding rows (K = 128).
 * Epilogue (applied on full output rows, 16-byte vectors): v = acc + bias[n]
 * (+ add[addmap(m), n < add_ncols]); v = act(v); v += res[m, n] + res2[m, n];
 * stored row-major (ldo) or ConvTranspose-scattered (store_mode 1, as catseg_gemm).
 * add/res/res2/out have the kernel dtype; bias is fp32.
 * ------------------------------------------------------------------------- */
typedef struct {
  const float* bias;
  const void* add; int64_t ld_add; CatsegRowMap addmap; int64_t add_ncols;
  int act;
  const void* res; int64_t ld_res;
  const void* res2; int64_t ld_res2;
  void* out; int64_t ldo;
  int store_mode; int cvt_k, cvt_hin, cvt_win, cvt_cout;
} CatsegRowsEpi;

/* catseg_rows_gemm — out = epi(LN?(X) . W^T), X: [M][128], W: [N][128].  LayerNorm
 * (ln_gamma/ln_beta, eps; NULL = none) is applied to X on load.  Replaces LN + q/k/v of
 * SwinTransformerBlock / AttentionLayer (model.py:191-196, 94-96, 344-346, 412), the
 * Swin output proj + residual (:112, :222) and the decoder ConvTranspose2d (:546). */
int catseg_rows_gemm(const void* x, int64_t ld_x, int64_t M, const float* ln_gamma,
                     const float* ln_beta, float eps, const void* w, int64_t N,
                     const CatsegRowsEpi* epi, int dtype, void* stream);

/* catseg_swin_proj_mlp — the rest of a Swin block after its window attention, in one pass
 * (model.py:112 proj, :222-223 shortcut + Mlp(norm2)):
 *   x1 = bf16(x + attn . w_proj^T + b_proj),  out = x1 + GELU(LN(x1) . W1^T + b1) . W2^T + b2,
 * x1 kept on chip.  bf16 rows of 128, hidden 512, exact-erf GELU; out may alias x (ld_out == ld_x).
 * Same arithmetic as catseg_rows_gemm (proj + residual) followed by catseg_rows_mlp. */
int catseg_swin_proj_mlp(const void* attn, int64_t ld_attn, const void* x, int64_t ld_x, int64_t M,
                         const void* w_proj, const float* b_proj, const float* ln_gamma, const float* ln_beta,
                         float eps, const void* w1, const float* b1, int64_t hidden, const void* w2,
                         const float* b2, void* out, int64_t ld_out, void* stream);

/* catseg_rows_mlp — out = epi(act(LN(Y) . W1^T + b1) . W2^T): the whole token MLP with
 * the hidden activations kept on chip.  Y: [M][128], W1: [hidden][128], b1 fp32,
 * W2: [128][hidden], epi.bias = b2.  Replaces timm Mlp after norm2 (model.py:223, GELU)
 * and the class-attention MLP (model.py:362-366,413, ReLU). */
int catseg_rows_mlp(const void* y, int64_t ld_y, int64_t M, const float* ln_gamma,
                    const float* ln_beta, float eps, const void* w1, const float* b1,
                    int64_t hidden, int act, const void* w2, const CatsegRowsEpi* epi,
                    int dtype, void* stream);

/* catseg_convt64_gn — bf16: out = ConvTranspose2d(k=2, s=2)(relu(GroupNorm(X))) for 64-channel
 * NHWC rows X [M][64] (slice = row / HW, HW % 64 == 0): the second guided-upsampler stage
 * (model.py:546) fused with DoubleConv's last GroupNorm+ReLU (:532-533).  W: [N=4*cout][64],
 * epi: bias + store_mode 1 scatter (cvt_k = 2). */
int catseg_convt64_gn(const void* x, int64_t M, int64_t HW, const float* mean, const float* rstd,
                      const float* gamma, const float* beta, int cpg, const void* w, int64_t N,
                      const CatsegRowsEpi* epi, void* stream);



/* catseg_layernorm — LayerNorm over the last dim (fp32 math).  Replaces
 * model_vpt.py:156-162 (ln_pre/ln_1/ln_2/ln_post/ln_final) and the nn.LayerNorm of
 * model.py:152,158,233,368-369.  in rows use `inmap`. */
int catseg_layernorm(const void* in, int64_t ld_in, CatsegRowMap inmap, int dtype_in,
                     void* out, int64_t ld_out, int dtype_out,
                     const float* gamma, const float* beta, int64_t rows, int64_t cols,
                     float eps, void* stream);

/* catseg_l2normalize — x / max(||x||, eps) per row (F.normalize, model.py:649-650,
 * cat_seg_predictor.py:216, model.py:714). */
int catseg_l2normalize(const void* in, int64_t ld_in, CatsegRowMap inmap, int dtype_in,
                       void* out, int64_t ld_out, int dtype_out, int64_t rows, int64_t cols,
                       float eps, void* stream);

/* ---------------------------------------------------------------------------
 * catseg_attention — softmax attention, flash-style (online softmax, K/V tiles
 * staged in LDS, MFMA for QK^T and PV).
 *   mode 0 (dense sequences): nn.MultiheadAttention of model_vpt.py:202-206
 *     (ViT, 16/12 heads x 64) and the causal text encoder (:400-406).
 *     Sequence s, token i lives at row s*seq_len + i.
 *   mode 1 (Swin windows): WindowAttention of model.py:86-114 with the cyclic
 *     shift and -100 region mask of model.py:161-216.  Sequence s = (slice,
 *     window); token i maps to pixel ((wy*ws + i/ws + shift) % H, ...) of slice.
 *   mode 2 (dense, log2-scaled q): as mode 0 with the q rows already multiplied
 *     by scale * log2(e) (the engine folds it into the ViT q projection), so
 *     softmax(scale q.k) = 2^(q.k - max) / sum; `scale` is not read.  bf16,
 *     head_dim 64, non-causal only.
 *   q/k/v: row pointers (columns of one head at + h*head_dim), row stride ld_qkv.
 *   out:   row stride ld_out, head h at columns h*head_dim.
 * ------------------------------------------------------------------------- */
typedef struct {
  const void* q; const void* k; const void* v; int64_t ld_qkv;
  void* out; int64_t ld_out;
  int64_t n_seq; int seq_len; int n_heads; int head_dim;
  float scale; int causal;
  int mode; int img_h, img_w, window, shift;
  int dtype;
} CatsegAttnArgs;
int catseg_attention(const CatsegAttnArgs* args, void* stream);

/* catseg_linear_attention — class aggregation attention (LinearAttention,
 * model.py:256-286, inside AttentionLayer model.py:338-354 and the padding of
 * ClassTransformerLayer model.py:397-410).  For every pixel (b, p) the sequence is
 * the T classes, rows (b*T + t)*HW + p of q/k/v (heads x head_dim columns).
 * n_pad learned padding tokens with constant projections k_pad/v_pad (fp32,
 * heads*head_dim) join the K/V sums; S = T + n_pad is the reference's v_length.
 *   y[row] = x[row] + LinearAttn(q, k, v)[row]            (x/y: ld_xy, may alias) */
typedef struct {
  const void* q; const void* k; const void* v; int64_t ld_qkv;
  const void* x; void* y; int64_t ld_xy;
  int64_t B; int T; int HW; int n_heads; int head_dim;
  int n_pad; const float* k_pad; const float* v_pad; float eps;
  int dtype;
} CatsegLinAttnArgs;
int catseg_linear_attention(const CatsegLinAttnArgs* args, void* stream);

/* catseg_class_seq_pack / catseg_class_seq_unpack_add — ATTENTION_TYPE "full" (FullAttention,
 * model.py:289-320, in AttentionLayer model.py:331-334 and ClassTransformerLayer :387-424).
 * The softmax itself is catseg_attention (mode 0, head_dim 32) over sequence-major rows:
 *   pack:       qkv rows (b*T + t)*HW + p ([q | k | v], C columns each) -> packed rows
 *               (b*HW + p)*(T + n_pad) + t; pad rows t >= T get q = 0, k = k_pad, v = v_pad
 *               (the learned padding's constant projections, fp32, model.py:397-410)
 *   unpack_add: y[(b*T + t)*HW + p] = x[same] + o[(b*HW + p)*(T + n_pad) + t], t < T
 *               (the pad rows' outputs are discarded as in model.py:419-421; x/y may alias) */
typedef struct {
  const void* qkv; int64_t ld_qkv;
  void* packed; int64_t ld_packed;
  const void* o; int64_t ld_o;
  const void* x; void* y; int64_t ld_xy;
  int64_t B; int T; int HW; int C;
  int n_pad; const float* k_pad; const float* v_pad;
  int dtype;
} CatsegClassSeqArgs;
int catseg_class_seq_pack(const CatsegClassSeqArgs* args, void* stream);
int catseg_class_seq_unpack_add(const CatsegClassSeqArgs* args, void* stream);

/* ---------------------------------------------------------------------------
 * catseg_conv3x3 — 3x3 / pad 1 convolution as an MFMA implicit GEMM over NHWC.
 * Replaces nn.Conv2d of model.py:528,531 (DoubleConv), 616, 627 (guidance
 * projections).  Input channels are the concatenation [src1 (c1) || src2 (c2)]
 * without materialising it (model.py:551-554): src1 per slice s, src2 per image
 * s / src2_div (the decoder guidance repeated over T).  Optional GroupNorm+ReLU
 * prologue on src1 (gn_mean/gn_rstd per (s, group of gn_cpg channels), gamma/
 * beta per channel).  Epilogue: + bias, act, optional GroupNorm partial stats
 * (per (s, tile, group): count-weighted mean and M2) for catseg_groupnorm_stats.
 *   weight: [c_out][3][3][c1+c2] (K contiguous).  out: [S][H][W][c_out].
 * ------------------------------------------------------------------------- */
typedef struct {
  const void* src1; int64_t s1_slice_stride; int64_t s1_offset; int c1;
  const void* src2; int64_t s2_slice_stride; int64_t s2_offset; int c2; int64_t src2_div;
  int64_t S; int H; int W;
  const void* weight; int c_out;
  const float* bias; int act;
  const float* gn_mean; const float* gn_rstd; const float* gn_gamma; const float* gn_beta; int gn_cpg;
  void* out; float* stats; int stats_cpg;
  int dtype;
  /* optional fp32 addend joined before the activation / statistics (the guidance half
   * of the conv computed once per image): addend[(s / addend_div) * addend_slice_stride
   * + pixel * c_out + co] */
  const float* addend; int64_t addend_slice_stride; int64_t addend_div;
  /* optional caller-allocated scratch (catseg_conv3x3_workspace bytes) for split-K of
   * small-grid convs; without it the conv runs unsplit */
  void* workspace; int64_t workspace_bytes;
} CatsegConvArgs;
int catseg_conv3x3(const CatsegConvArgs* args, void* stream);

/* catseg_conv3x3_partial — the conv over a channel subset, fp32 out, once per image:
 * out[b][pix][co] = sum_{tap, ci} weight[co][tap][ci] * g[b][pix + tap][ci] (zero pad, no
 * bias).  With g = the decoder guidance (model.py:551-554, repeated over classes by the
 * reference) this is the class-independent half of conv(concat[x, g]); it enters the
 * per-class conv over x as its `addend`.  g: NHWC [B][H][W][cin]; weight fp32 [cout][9][cin]. */
int catseg_conv3x3_partial(const void* g, int64_t B, int H, int W, int cin, const float* weight, int cout,
                           float* out, int dtype, void* stream);
/* catseg_upconv3x3 — ConvTranspose2d(k=2, s=2) followed by the 3x3 / pad-1 conv of
 * DoubleConv, with the ConvTranspose output never materialised (Up.forward, model.py:546-555:
 * up -> concat guidance -> conv).  Per output parity (a, b) the pair is a 2x2-tap conv over the
 * ConvTranspose INPUT; args as catseg_conv3x3 with
 *   src1 = the ConvTranspose input [S][H][W][c1] (optional GroupNorm+ReLU prologue as there),
 *   weight = composite bf16 [4 * cout][3][3][c1], row block p = 2a + b holding parity (a, b)'s
 *            taps (rows a..a+1, columns b..b+1; the other taps unused),
 *   c_out = 4 * cout, addend = fp32 [S / addend_div][H*W][4 * cout] (catseg_upconv_addend: the
 *            guidance half of the conv and the ConvTranspose bias through the in-image taps),
 *   out = bf16 [S][2H][2W][cout], stats = GroupNorm partials of the 2H x 2W map:
 *            [S][4 * H*W / catseg_upconv3x3_stats_tile()][cout / 16][2].
 * Instantiated for c1 = 64, cout = 32, 48 <= W <= 50 (the second Up block of CAT-Seg). */
int catseg_upconv3x3(const CatsegConvArgs* args, void* stream);
int catseg_upconv3x3_stats_tile(void);
/* catseg_upconv_addend — catseg_conv3x3_partial on the 2H x 2W guidance grid plus, per pixel,
 * tap_bias[tap][co] (the ConvTranspose bias through conv tap `tap`, fp32 [9][cout], may be NULL)
 * summed over the taps inside the image, written in catseg_upconv3x3's parity addend layout
 * out[b][(y/2)*(W2/2) + x/2][((y%2)*2 + x%2)*cout + co].  bf16 g with 16 or 32 channels. */
int catseg_upconv_addend(const void* g, int64_t B, int H2, int W2, int cin, const float* weight,
                         const float* tap_bias, int cout, float* out, int dtype, void* stream);
/* Rows per conv tile of the im2col kernel (128). */
int catseg_conv_tile_rows(void);
/* Pixels per GroupNorm partial ("tile") of the kernel catseg_conv3x3 picks for `args`:
 * stats is [S][H*W/tile][c_out/stats_cpg][2] (the row-ring kernel emits one partial per
 * wave pixel block, 32-128 pixels; the others 128). */
int catseg_conv3x3_stats_tile(const CatsegConvArgs* args);
/* Bytes of split-K scratch catseg_conv3x3 would use for `args` (0 = none). */
int64_t catseg_conv3x3_workspace(const CatsegConvArgs* args);

/* catseg_groupnorm_stats — combine the conv partials into mean / rstd per
 * (slice, group) (nn.GroupNorm statistics, model.py:529,532; eps 1e-5). */
int catseg_groupnorm_stats(const float* partials, int64_t S, int tiles, int groups, int64_t tile_count,
                           float eps, float* mean, float* rstd, void* stream);

/* catseg_groupnorm_relu — y = relu((x - mean[s,g]) * rstd[s,g] * gamma[c] + beta[c]) over
 * NHWC [S][HW][C] (GroupNorm + ReLU of model.py:529-533). */
int catseg_groupnorm_relu(const void* x, void* y, int64_t S, int64_t HW, int C, int cpg,
                          const float* mean, const float* rstd, const float* gamma,
                          const float* beta, int dtype, void* stream);

/* catseg_conv3x3_head — the final head conv3x3 c_in -> 1 with bias (model.py:634,679)
 * writing fp32 logits into out[b][cls(b, t)][H][W], cls = classes[b*T + t] (or t if
 * classes == NULL); out has T_out class planes (the top-k scatter of model.py:721-724). */
int catseg_conv3x3_head(const void* x, int64_t B, int T, int H, int W, int C,
                        const float* weight, float bias, const int32_t* classes, int T_out,
                        float* out, int dtype, void* stream);
/* Same, with the preceding GroupNorm+ReLU (mean/rstd per (slice, group of cpg
 * channels), gamma/beta per channel) applied to x on load.  weight: [9][C]. */
int catseg_conv3x3_head_gn(const void* x, int64_t B, int T, int H, int W, int C,
                           const float* weight, float bias, const float* mean, const float* rstd,
                           const float* gamma, const float* beta, int cpg,
                           const int32_t* classes, int T_out, float* out, int dtype, void* stream);

/* catseg_corr_embed — Conv2d(1, hidden, 7, pad 3) on every cost slice
 * (Aggregator.corr_embed, model.py:654-659).  corr: fp32, slice (b, t) read from
 * corr + cls(b,t)*corr_t_stride + b*corr_b_stride (cls = classes[b*T+t] or t),
 * H*W contiguous.  out: X rows [(b*T + t)*H*W + p][hidden]. */
int catseg_corr_embed(const float* corr, int64_t corr_t_stride, int64_t corr_b_stride,
                      const int32_t* classes, int64_t B, int T, int H, int W,
                      const float* weight, const float* bias, int hidden,
                      void* out, int dtype, void* stream);

/* catseg_topk_classes — per image, the top-k classes by max-over-pixels cosine
 * (model.py:694-696), written sorted by (max descending, class index ascending): the set
 * torch.topk selects, ties to the lower class index.  corr fp32 laid out as
 * corr[t*corr_t_stride + b*corr_b_stride + p]; workspace: B*T floats (the class maxima). */
int catseg_topk_classes(const float* corr, int64_t corr_t_stride, int64_t corr_b_stride,
                        int64_t B, int T, int HW, int k, int32_t* classes, float* workspace, void* stream);

/* catseg_transpose_rows — out[b][c][r] = in[b*in_bstride + r][c] for r < rows, 0 for
 * rows <= r < ld_out (the transposed text-guidance k half of catseg_class_attention). */
int catseg_transpose_rows(const void* in, int64_t ld_in, int64_t rows, int64_t cols, int64_t batch,
                          int64_t in_bstride, void* out, int64_t ld_out, int dtype, void* stream);

/* catseg_gather_rows — out[r] = in[idx[r]] for fp32/bf16 rows (text guidance gather
 * of model.py:697-698). */
int catseg_gather_rows(const void* in, int64_t ld_in, const int32_t* idx, int64_t rows, int64_t cols,
                       void* out, int64_t ld_out, int dtype, void* stream);

/* catseg_convert — out[r] = (dtype_out) in[inmap(r)] (hook / feature casts, CLS drop of
 * cat_seg_model.py:178-183). */
int catseg_convert(const void* in, int64_t ld_in, CatsegRowMap inmap, int dtype_in,
                   void* out, int64_t ld_out, int dtype_out, int64_t rows, int64_t cols, void* stream);

/* catseg_fill_f32 — out[i] = value (the -100 canvas of model.py:722). */
int catseg_fill_f32(float* out, int64_t n, float value, void* stream);

/* ---------------------------------------------------------------------------
 * Image side
 * ------------------------------------------------------------------------- */
/* catseg_preprocess_im2col — cat_seg_model.py:149-154 + the patch conv's im2col:
 * normalize (mean/std), ImageList zero-pad (value 0 after normalization) to the
 * padded canvas (Hp, Wp), bilinear resize (align_corners=False) to res x res, then
 * unfold res/patch x res/patch patches into rows (b, gy, gx) of K = 3*patch*patch
 * columns ordered (c, ky, kx), zero-padded to ld_out.  raw: fp32 [B][3][Hp][Wp]
 * (0..255), sizes: int32 [B][2] valid (h, w) per image. */
int catseg_preprocess_im2col(const float* raw, const int32_t* sizes, int64_t B, int Hp, int Wp,
                             const float* mean, const float* std, int res, int patch,
                             void* out, int64_t ld_out, int dtype, void* stream);

/* catseg_vit_embed — VisualTransformer.forward head (model_vpt.py:290-300):
 * x[b, 0] = cls + pos[0]; x[b, 1+p] = patches[b*G2 + p] + pos[1+p]; then ln_pre.
 * patches fp32 [B*G2][width]; x fp32 [B*(G2+1)][width]. */
int catseg_vit_embed(const float* patches, const float* cls, const float* pos,
                     const float* gamma, const float* beta, int64_t B, int G2, int width,
                     float* x, void* stream);

/* catseg_bicubic_resize — VisualTransformer.resized_pos_embed (model_vpt.py:316-329),
 * bicubic (A = -0.75) align_corners=False on a [S_in][S_in][D] grid -> [S_out][S_out][D]. */
int catseg_bicubic_resize(const float* in, int S_in, int D, float* out, int S_out, void* stream);

/* catseg_postprocess — sigmoid then bilinear (align_corners=False) of fp32 logits
 * [B][T][h][w] cropped to (crop_h, crop_w) to [B][T][H][W] fp32
 * (cat_seg_model.py:222-227 + detectron2 sem_seg_postprocess). */
int catseg_postprocess(const float* logits, int64_t B, int T, int h, int w, int crop_h, int crop_w,
                       float* out, int H, int W, void* stream);
/* catseg_resize_bilinear — catseg_postprocess without the sigmoid: the final
 * sem_seg_postprocess of the sliding branch (cat_seg_model.py:215-217). */
int catseg_resize_bilinear(const float* in, int64_t B, int T, int h, int w, int crop_h, int crop_w,
                           float* out, int H, int W, void* stream);

/* ---------------------------------------------------------------------------
 * catseg_swin_window_attention — fused LayerNorm(norm1) + [q|k|v] projection (+ the
 * per-image guidance half of q and k) + shifted-window multi-head attention, one
 * workgroup per (slice, window); q/k/v never reach HBM.  Replaces, per Swin block,
 * model.py:191-199 (norm1, concat guidance_norm(guidance), roll, window_partition) and
 * WindowAttention.forward model.py:86-114 up to the output projection (which stays a
 * catseg_rows_gemm with the residual).  bf16; 24x24 map, 12x12 windows, 4 heads x 32.
 *   out[row] = attention rows (heads concatenated), same row order as x;
 *   q|k|v[row] = LN(x[row]) . w_qkv^T + b_qkv (+ gqk[gmap(row)] on the q and k columns)
 * ------------------------------------------------------------------------- */
typedef struct {
  const void* x; int64_t ld_x;
  const float* ln_g; const float* ln_b; float eps;
  const void* w_qkv; const float* b_qkv;          /* [3*128][128], [3*128] */
  const void* gqk; int64_t ld_g; CatsegRowMap gmap; /* [.][256] guidance halves of q, k */
  void* out; int64_t ld_out;
  int64_t S; int img_h, img_w, window, shift, n_heads, head_dim; float scale;
  int dtype;
} CatsegSwinAttnArgs;
int catseg_swin_window_attention(const CatsegSwinAttnArgs* args, void* stream);

/* ---------------------------------------------------------------------------
 * catseg_class_attention — fused LayerNorm(norm1) + [q|k|v] projection (+ the
 * per-class text-guidance half of q and k) + linear class attention + the attention
 * residual, persistent workgroups over pixels; q/k/v never reach HBM.  Replaces, per
 * class layer, model.py:397-413 up to `x_pool + attention(norm1(x_pool), guidance)`
 * (AttentionLayer model.py:338-354, LinearAttention model.py:256-286), i.e. the
 * catseg_rows_gemm + catseg_linear_attention pair.  bf16; 4 heads x 32.
 *   rows of pixel (b, p): (b*T + t)*HW + p, t < T;  tg row of class t: b*tg_bstride + t
 *   (tg = [.][256] guidance halves of q | k, without bias; tg_bstride 0 = shared);
 *   y[row] = x[row] + LinearAttention(q, k, v)[row] with the n_pad learned padding
 *   tokens' constant projections k_pad / v_pad (fp32) in the sums, S = T + n_pad.
 * ------------------------------------------------------------------------- */
typedef struct {
  const void* x; int64_t ld_x;
  const float* ln_g; const float* ln_b; float eps;
  const void* w_qkv; const float* b_qkv;          /* [3*128][128], [3*128] */
  const void* tg; int64_t ld_tg; int64_t tg_bstride;
  int n_pad; const float* k_pad; const float* v_pad; float attn_eps;
  void* y; int64_t ld_y;
  int64_t B; int T; int HW; int n_heads; int head_dim;
  int dtype;
  /* the k half of tg transposed, [128][ld_tgk_t] per image (catseg_transpose_rows), image b
   * at element offset b*tgk_t_bstride (0 = shared); ld_tgk_t >= round_up(T, 16), zero past T.
   * Required by the default kernel (variant 0); null selects variant 1. */
  const void* tgk_t; int64_t ld_tgk_t; int64_t tgk_t_bstride;
} CatsegClassAttnArgs;
int catseg_class_attention(const CatsegClassAttnArgs* args, void* stream);

/* ---------------------------------------------------------------------------
 * Class-attention pooling (POOLING_SIZES != [1,1]; ClassTransformerLayer,
 * model.py:374-423) on the rows layout [S][H][W][C] (S = B*T slices).
 * ------------------------------------------------------------------------- */
/* catseg_avgpool_rows — nn.AvgPool2d(ph, pw) (stride = kernel, no padding) per slice:
 * [S][H][W][C] -> [S][H/ph][W/pw][C]  (pool_features, model.py:374-385). */
int catseg_avgpool_rows(const void* in, int64_t S, int H, int W, int C, int ph, int pw, void* out,
                        int dtype, void* stream);
/* catseg_upsample_add_rows — x[S][H][W][C] += bilinear(xp[S][Hp][Wp][C] -> H x W,
 * align_corners=True)  (model.py:415-423: interpolate, crop padding, x + x_pool). */
int catseg_upsample_add_rows(const void* xp, int64_t S, int Hp, int Wp, int C, void* x, int H, int W,
                             int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * Sliding-window inference (TEST.SLIDING_WINDOW, cat_seg_model.py:156-176,204-218).
 * ------------------------------------------------------------------------- */
/* catseg_sliding_crops — per image n of a zero-padded fp32 canvas raw[N][3][Hc][Wc] with
 * valid sizes[n] = (h, w): bilinear resize to out_res², nn.Unfold(kernel, stride) into
 * nb² crops (nb = (out_res - kernel) / stride + 1, row-major blocks), plus the bilinear
 * kernel² resize of the whole image:  crops[N*(nb²+1)][3][kernel][kernel], 0-255
 * (normalisation and the CLIP-resolution resize follow in catseg_preprocess_im2col). */
int catseg_sliding_crops(const float* raw, const int32_t* sizes, int64_t N, int Hc, int Wc, int out_res,
                         int kernel, int stride, float* crops, void* stream);
/* catseg_sliding_merge — logits[N*(nb²+1)][T][h][w] -> out[N][T][out_res][out_res]:
 * interpolate each crop to kernel² + sigmoid; Fold(tiles) / Fold(Unfold(ones));
 * average with the global crop interpolated to out_res²  (cat_seg_model.py:204-213). */
int catseg_sliding_merge(const float* logits, int64_t N, int T, int h, int w, int kernel, int stride,
                         int out_res, float* out, void* stream);

/* ---------------------------------------------------------------------------
 * Text side (CLIP.encode_text, model_vpt.py:421-438)
 * ------------------------------------------------------------------------- */
/* catseg_token_embed — x[n, i] = tok_emb[tokens[n, i]] + pos[i]  (fp32 out). */
int catseg_token_embed(const int32_t* tokens, int64_t n, int ctx, const float* tok_emb,
                       const float* pos, int width, float* x, void* stream);
/* catseg_eot_gather — out[n] = x[n*ctx + argmax_i tokens[n, i]] (first max). */
int catseg_eot_gather(const float* x, const int32_t* tokens, int64_t n, int ctx, int width,
                      float* out, void* stream);

/* catseg_bce_onehot_loss — the training branch's loss (cat_seg_model.py:189-203):
 * logits [B][T][h][w] fp32, bilinearly upsampled (align_corners=False) to the target size,
 * BCE-with-logits against one-hot targets built from targets [B][H][W] int32 (ignore_value
 * pixels have an all-zero target row and still count), mean over B*H*W*T -> *loss (fp32, device).
 * workspace: >= B*H doubles (caller-allocated).  Deterministic (fixed-order fp64 partial sums).
 * Its gradient w.r.t. the logits is catseg_bce_onehot_loss_backward. */
int catseg_bce_onehot_loss(const float* logits, int64_t B, int T, int h, int w, const int32_t* targets, int H, int W,
                           int ignore_value, double* workspace, float* loss, void* stream);
/* catseg_bce_onehot_loss_backward — d loss / d logits of catseg_bce_onehot_loss (what autograd
 * computes for cat_seg_model.py:192-203: the BCE-with-logits mean's backward through
 * F.interpolate's bilinear backward): grad_logits[B][T][h][w] = *grad_loss / (B*H*W*T) *
 * U^T (sigmoid(U logits) - onehot), U the bilinear upsample.  grad_loss: device fp32 scalar (the
 * upstream gradient; NULL = 1).  workspace: >= B*T*H*w floats.  Gather form, no atomics:
 * deterministic.  Needs B*T < 65536. */
int catseg_bce_onehot_loss_backward(const float* logits, int64_t B, int T, int h, int w, const int32_t* targets,
                                    int H, int W, int ignore_value, const float* grad_loss, float* workspace,
                                    float* grad_logits, void* stream);

/* ---------------------------------------------------------------------------
 * catseg_semseg_confusion — the confusion-matrix update of detectron2's
 * SemSegEvaluator.process as CAT-Seg's evaluators use it (plain_train_net.py:107-116,
 * train_net.py:55-67): pred = argmax over T of probs [T][H][W] (first maximum wins);
 * pred >= clamp_pred -> clamp_pred (VOC-b; clamp_pred < 0 disables); gt [H][W] int32 with
 * ignore_label -> num_classes; conf[(num_classes+1) * pred + gt] += 1 (int64,
 * (num_classes+1)^2, caller-zeroed, accumulated across calls).  Labels outside
 * [0, num_classes] are not binned but counted in *n_invalid (int64).
 * ------------------------------------------------------------------------- */
int catseg_semseg_confusion(const float* probs, int64_t T, int64_t H, int64_t W, const int32_t* gt,
                            int num_classes, int ignore_label, int clamp_pred, int64_t* conf,
                            int64_t* n_invalid, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CATSEG_HIP_H */
