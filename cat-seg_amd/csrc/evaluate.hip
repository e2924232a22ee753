// Semantic-segmentation evaluation on the device: the confusion-matrix update of
// detectron2's SemSegEvaluator.process as CAT-Seg's evaluators use it
// (plain_train_net.py:107-116 SemSegGzeroEvaluator, train_net.py:55-67 VOCbEvaluator):
//
//   pred = sem_seg.argmax(0)                      (first maximum wins, as torch.argmax)
//   pred[pred >= clamp_pred] = clamp_pred         (VOC-b background fold; clamp_pred < 0: off)
//   gt[gt == ignore_label] = num_classes
//   conf += bincount((num_classes + 1) * pred + gt)
//
// One thread per pixel; the argmax walks the T class planes with the pixel index on the
// lanes (each class plane read once, coalesced).  Bins are 64-bit integer atomics, so the
// matrix is exact and independent of the order in which pixels land.  Labels outside
// [0, num_classes] after the ignore fold (the reference's bincount would then fail its
// reshape) are counted in *n_invalid instead of being binned.
#include "common.h"
#include "capi.h"

namespace {

__global__ __launch_bounds__(256) void confusion_kernel(const float* __restrict__ probs, int64_t T, int64_t HW,
                                                        const int32_t* __restrict__ gt, int num_classes,
                                                        int ignore_label, int clamp_pred,
                                                        unsigned long long* __restrict__ conf,
                                                        unsigned long long* __restrict__ n_invalid) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HW) return;
  float best = probs[p];
  int arg = 0;
  for (int64_t t = 1; t < T; ++t) {
    const float v = probs[t * HW + p];
    // strict >: the first maximum wins; NaN ranks above every number (torch.argmax).  NaN is
    // tested on the bits, so the rule holds whatever float mode the file is built with
    const bool best_nan = (__float_as_uint(best) & 0x7fffffffu) > 0x7f800000u;
    const bool v_nan = (__float_as_uint(v) & 0x7fffffffu) > 0x7f800000u;
    if (!best_nan && (v_nan || v > best)) {
      best = v;
      arg = (int)t;
    }
  }
  if (clamp_pred >= 0 && arg >= clamp_pred) arg = clamp_pred;
  int g = gt[p];
  if (g == ignore_label) g = num_classes;
  const int64_t n1 = (int64_t)num_classes + 1;
  if (g < 0 || g > num_classes || arg > num_classes) {
    atomicAdd(n_invalid, 1ull);
    return;
  }
  atomicAdd(conf + n1 * arg + g, 1ull);
}

// ---- training-branch loss (cat_seg_model.py:189-203): BCE-with-logits of the logits,
// bilinearly upsampled (align_corners=False) to the target size, against one-hot targets
// (ignore_value pixels: all-zero rows, still averaged), mean over B*H*W*T.  One block per
// (image, target row); per-thread fp32 sums over the classes of a pixel, fp64 block partials,
// then one block sums the partials in a fixed order (deterministic).
DEV void bce_lin(int dst, int in_size, float scale, int& i0, int& i1, float& l1) {
  const float src = fmaxf(scale * ((float)dst + 0.5f) - 0.5f, 0.f);
  i0 = (int)src;
  i1 = i0 + ((i0 < in_size - 1) ? 1 : 0);
  l1 = src - (float)i0;
}

__global__ __launch_bounds__(256) void bce_rows_kernel(const float* __restrict__ logits, int T, int h, int w,
                                                       const int32_t* __restrict__ tgt, int H, int W, int ignore,
                                                       double* __restrict__ partial) {
  const int y = blockIdx.x, b = blockIdx.y;
  int y0, y1;
  float ly;
  bce_lin(y, h, (float)h / (float)H, y0, y1, ly);
  double acc = 0.0;
  for (int x = threadIdx.x; x < W; x += blockDim.x) {
    int x0, x1;
    float lx;
    bce_lin(x, w, (float)w / (float)W, x0, x1, lx);
    const int cls = tgt[((int64_t)b * H + y) * W + x];
    // the class planes' taps are independent loads: unrolled so a batch is in flight per round trip;
    // softplus(-|v|) as log(1 + e) with the hardware log / exp (absolute error ~1e-7 per term)
    const float* L0 = logits + (int64_t)b * T * h * w + (int64_t)y0 * w;
    const float* L1 = logits + (int64_t)b * T * h * w + (int64_t)y1 * w;
    const int64_t plane = (int64_t)h * w;
    float s = 0.f;
#pragma unroll 8
    for (int t = 0; t < T; ++t) {
      const float v = (1.f - ly) * ((1.f - lx) * L0[t * plane + x0] + lx * L0[t * plane + x1]) +
                      ly * ((1.f - lx) * L1[t * plane + x0] + lx * L1[t * plane + x1]);
      s += fmaxf(v, 0.f) + __logf(1.f + __expf(-fabsf(v)));
    }
    if (cls != ignore && cls >= 0 && cls < T) {
      const float v = (1.f - ly) * ((1.f - lx) * L0[cls * plane + x0] + lx * L0[cls * plane + x1]) +
                      ly * ((1.f - lx) * L1[cls * plane + x0] + lx * L1[cls * plane + x1]);
      s -= v;
    }
    acc += (double)s;
  }
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[(int64_t)b * H + y] = red[0];
}

__global__ __launch_bounds__(256) void bce_final_kernel(const double* __restrict__ partial, int64_t n, double denom,
                                                        float* __restrict__ loss) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) acc += partial[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = (float)(red[0] / denom);
}

// ---- its gradient w.r.t. the logits: dL/dlogits = U^T (sigmoid(U logits) - onehot) * g / denom,
// U the separable bilinear upsample.  Gather form (each output element sums its own
// contributions in a fixed order -- no atomics, deterministic), in two passes:
//   pass 1 (one block per (image, target row y)): G[b][t][y][j] = sum over the target columns x
//          whose taps include logit column j of wx(x, j) * (sigmoid(v(y, x)) - z(y, x)), v computed
//          from the 4 logits taps exactly as the forward does;
//   pass 2 (one thread per logit): grad[b][t][i][j] = g / denom * sum over the target rows y
//          whose taps include i of wy(y, i) * G[b][t][y][j].
// The x (y) range of logit column j (row i) is the contiguous run of targets with x0(x) in {j-1, j}
// (x0 is nondecreasing); the scan starts a few targets below the analytic start.
DEV int bce_first_src(int j, int in_size, int out_size) {
  // first target index whose floor source index can be >= j-1, minus a margin of 2
  const int s = (int)floorf(((float)j - 1.5f) * (float)out_size / (float)in_size) - 2;
  return s < 0 ? 0 : s;
}

// the contributing run [a, b) of targets for source index j (index arithmetic only)
DEV void bce_run(int j, int in_size, int out_size, float scale, int& a, int& b) {
  a = bce_first_src(j, in_size, out_size);
  for (; a < out_size; ++a) {
    int i0, i1;
    float l1;
    bce_lin(a, in_size, scale, i0, i1, l1);
    if (i1 >= j) break;
  }
  for (b = a; b < out_size; ++b) {
    int i0, i1;
    float l1;
    bce_lin(b, in_size, scale, i0, i1, l1);
    if (i0 > j) break;
  }
}

// pass 1: one block per (image, target row y).  Per chunk of TC classes the residuals
// r[t][x] = sigmoid(v) - z of the whole target row are computed once into LDS (x on the lanes:
// the logits taps of a class plane are neighbouring loads), then every (class, logit column j)
// sums its run of x from LDS.  The per-column runs are computed once per block.
__global__ __launch_bounds__(256) void bce_grad_rows_kernel(const float* __restrict__ logits, int T, int h, int w,
                                                            const int32_t* __restrict__ tgt, int H, int W, int ignore,
                                                            int TC, float* __restrict__ G) {
  extern __shared__ float lds[];
  float* R = lds;                                  // [TC][W]
  int* run = reinterpret_cast<int*>(lds + TC * W); // [w][2]
  const int y = blockIdx.x, b = blockIdx.y;
  int y0, y1;
  float ly;
  bce_lin(y, h, (float)h / (float)H, y0, y1, ly);
  const float sx = (float)w / (float)W;
  const int32_t* trow = tgt + ((int64_t)b * H + y) * W;
  const int64_t plane = (int64_t)h * w;
  const float* L0 = logits + (int64_t)b * T * plane + (int64_t)y0 * w;
  const float* L1 = logits + (int64_t)b * T * plane + (int64_t)y1 * w;
  for (int j = threadIdx.x; j < w; j += blockDim.x) bce_run(j, w, W, sx, run[2 * j], run[2 * j + 1]);
  for (int t0 = 0; t0 < T; t0 += TC) {
    const int nt = min(TC, T - t0);
    __syncthreads();                               // runs written / previous chunk consumed
    // a lane owns target column x and walks the chunk's classes: the taps of 8 classes in flight
    // per round trip (one class per iteration would pay a round trip each)
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
      int x0, x1;
      float lx;
      bce_lin(x, w, sx, x0, x1, lx);
      const int cls = trow[x];
      const int zt = (cls != ignore) ? cls - t0 : -1;
#pragma unroll 8
      for (int tt = 0; tt < nt; ++tt) {
        const float* r0 = L0 + (int64_t)(t0 + tt) * plane;
        const float* r1 = L1 + (int64_t)(t0 + tt) * plane;
        const float v = (1.f - ly) * ((1.f - lx) * r0[x0] + lx * r0[x1]) + ly * ((1.f - lx) * r1[x0] + lx * r1[x1]);
        R[tt * W + x] = __builtin_amdgcn_rcpf(1.f + __expf(-v)) - (tt == zt ? 1.f : 0.f);
      }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nt * w; idx += blockDim.x) {
      const int tt = idx / w, j = idx - tt * w;
      const float* Rt = R + tt * W;
      float acc = 0.f;
      for (int x = run[2 * j]; x < run[2 * j + 1]; ++x) {
        int x0, x1;
        float lx;
        bce_lin(x, w, sx, x0, x1, lx);
        acc += ((x0 == j ? 1.f - lx : 0.f) + (x1 == j ? lx : 0.f)) * Rt[x];
      }
      G[(((int64_t)b * T + t0 + tt) * H + y) * w + j] = acc;
    }
  }
}

// pass 2: one thread per logit (class plane bt, row i, column j); grid (ceil(h*w / 256), B*T).
__global__ __launch_bounds__(256) void bce_grad_cols_kernel(const float* __restrict__ G, int h, int w, int H,
                                                            const float* __restrict__ gscale, float inv_denom,
                                                            float* __restrict__ grad) {
  const int64_t bt = blockIdx.y;
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= h * w) return;
  const int i = o / w, j = o - i * w;
  const float sy = (float)h / (float)H;
  const float scale = (gscale ? gscale[0] : 1.f) * inv_denom;
  const float* Gp = G + bt * H * w + j;
  int ya, yb;
  bce_run(i, h, H, sy, ya, yb);
  float acc = 0.f;
#pragma unroll 4
  for (int y = ya; y < yb; ++y) {
    int y0, y1;
    float ly;
    bce_lin(y, h, sy, y0, y1, ly);
    acc += ((y0 == i ? 1.f - ly : 0.f) + (y1 == i ? ly : 0.f)) * Gp[(int64_t)y * w];
  }
  grad[bt * h * w + o] = acc * scale;
}

}  // namespace

int g_bce_classes = 0;   // classes per LDS chunk in the loss backward's rows pass (0 = auto)
CATSEG_KNOB(g_bce_classes, "bce_classes");

extern "C" int catseg_bce_onehot_loss_backward(const float* logits, int64_t B, int T, int h, int w,
                                               const int32_t* targets, int H, int W, int ignore_value,
                                               const float* grad_loss, float* workspace, float* grad_logits,
                                               void* stream) {
  CATSEG_CHECK(logits && targets && workspace && grad_logits, "bce_onehot_loss_backward: null pointer");
  CATSEG_CHECK(B > 0 && T > 0 && h > 0 && w > 0 && H > 0 && W > 0 && B * T < 65536 && B < 65536,
               "bce_onehot_loss_backward: bad shape");
  // LDS for the rows pass: TC class rows of W residuals + the w column runs.  Auto: 16 classes
  // (24 KB at W = 384), capped at 32 KB; at the training shape 4 / 8 / 16 / 21 / 32 classes measured
  // 355 / 315 / 306 / 415 / 404 us (tools/micro_bce.py)
  const int TC = std::max(1, std::min(T, g_bce_classes > 0 ? g_bce_classes : std::min(16, 8192 / W)));
  const size_t lds = (size_t)TC * W * 4 + (size_t)w * 8;
  CATSEG_CHECK(lds <= 64 * 1024, "bce_onehot_loss_backward: target or logits rows too wide");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bce_grad_rows_kernel, dim3((unsigned)H, (unsigned)B), dim3(256), lds, st, logits, T, h, w,
                     targets, H, W, ignore_value, TC, workspace);
  hipLaunchKernelGGL(bce_grad_cols_kernel, dim3((unsigned)((h * w + 255) / 256), (unsigned)(B * T)), dim3(256), 0,
                     st, workspace, h, w, H, grad_loss, (float)(1.0 / ((double)B * H * W * T)), grad_logits);
  return catseg_launch_status("bce_onehot_loss_backward");
}

extern "C" int catseg_bce_onehot_loss(const float* logits, int64_t B, int T, int h, int w, const int32_t* targets,
                                      int H, int W, int ignore_value, double* workspace, float* loss, void* stream) {
  CATSEG_CHECK(logits && targets && workspace && loss, "bce_onehot_loss: null pointer");
  CATSEG_CHECK(B > 0 && T > 0 && h > 0 && w > 0 && H > 0 && W > 0 && B < 65536, "bce_onehot_loss: bad shape");
  CATSEG_CHECK(((uintptr_t)workspace % 8) == 0, "bce_onehot_loss: workspace must be 8-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bce_rows_kernel, dim3((unsigned)H, (unsigned)B), dim3(256), 0, st, logits, T, h, w, targets, H, W,
                     ignore_value, workspace);
  hipLaunchKernelGGL(bce_final_kernel, dim3(1), dim3(256), 0, st, workspace, B * H, (double)B * H * W * T, loss);
  return catseg_launch_status("bce_onehot_loss");
}

extern "C" int catseg_semseg_confusion(const float* probs, int64_t T, int64_t H, int64_t W, const int32_t* gt,
                                       int num_classes, int ignore_label, int clamp_pred, int64_t* conf,
                                       int64_t* n_invalid, void* stream) {
  CATSEG_CHECK(probs && gt && conf && n_invalid, "semseg_confusion: null pointer");
  CATSEG_CHECK(T > 0 && H > 0 && W > 0 && num_classes > 0, "semseg_confusion: empty shape");
  CATSEG_CHECK(((uintptr_t)conf % 8) == 0 && ((uintptr_t)n_invalid % 8) == 0, "semseg_confusion: misaligned counters");
  const int64_t HW = H * W;
  const int64_t blocks = (HW + 255) / 256;
  CATSEG_CHECK(blocks < ((int64_t)1 << 31), "semseg_confusion: image too large");
  hipLaunchKernelGGL(confusion_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, probs, T, HW, gt,
                     num_classes, ignore_label, clamp_pred, (unsigned long long*)conf,
                     (unsigned long long*)n_invalid);
  return catseg_launch_status("semseg_confusion");
}
