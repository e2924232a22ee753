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
    // strict >: the first maximum wins; NaN ranks above every number (torch.argmax)
    if (best == best && (v > best || v != v)) {
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

}  // namespace

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
