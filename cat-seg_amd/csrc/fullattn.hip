// ATTENTION_TYPE "full" for the class aggregation: FullAttention (reference
// cat_seg/modeling/transformer/model.py:289-320) inside AttentionLayer (:331-334,338-354) of
// ClassTransformerLayer (:387-424).
//
// The softmax attention itself runs on the MFMA flash kernel (catseg_attention, mode 0,
// head_dim 32); what differs from the ViT MHA is only where a sequence's rows live.  The class
// aggregation keeps its rows class-major, (b*T + t)*HW + p, so a pixel's T class rows are HW
// rows apart, and the reference pads every sequence to pad_len with learned tokens whose k / v
// projections are constant (model.py:397-410).  Two HBM passes around the attention:
//   pack:        qkv rows (b, t, p) -> sequence-major rows (b, p, t), t < T + n_pad; the pad
//                rows get k_pad / v_pad (their queries are zero: the reference discards the pad
//                rows' outputs, :419-421, so their values never matter)
//   unpack_add:  y[(b, t, p)] = x[(b, t, p)] + o[(b, p, t)] for t < T (the residual, :413)
// One thread per 4 columns of a row; a wave covers whole rows, so both sides stay coalesced.
#include "common.h"
#include "capi.h"

namespace {

template <typename E>
__global__ __launch_bounds__(256) void class_seq_pack_kernel(CatsegClassSeqArgs a, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int g3 = 3 * a.C / 4;                   // 4-column groups per [q | k | v] row
  const int Lp = a.T + a.n_pad;
  const int64_t pr = i / g3;
  const int col = (int)(i % g3) * 4;
  const int64_t seq = pr / Lp;
  const int t = (int)(pr % Lp);
  const int64_t b = seq / a.HW;
  const int p = (int)(seq % a.HW);
  float v[4];
  if (t < a.T) {
    load4<E>(reinterpret_cast<const E*>(a.qkv) + ((b * a.T + t) * a.HW + p) * a.ld_qkv + col, v);
  } else if (col < a.C) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = 0.f;
  } else {
    const float* src = col < 2 * a.C ? a.k_pad + (col - a.C) : a.v_pad + (col - 2 * a.C);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = src[e];
  }
  store4<E>(reinterpret_cast<E*>(a.packed) + pr * a.ld_packed + col, v);
}

template <typename E>
__global__ __launch_bounds__(256) void class_seq_unpack_add_kernel(CatsegClassSeqArgs a, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int g = a.C / 4;
  const int64_t r = i / g;                      // class-major row (b*T + t)*HW + p
  const int col = (int)(i % g) * 4;
  const int64_t bt = r / a.HW;
  const int p = (int)(r % a.HW);
  const int64_t b = bt / a.T;
  const int t = (int)(bt % a.T);
  const int64_t pr = (b * a.HW + p) * (a.T + a.n_pad) + t;
  float x[4], o[4];
  load4<E>(reinterpret_cast<const E*>(a.x) + r * a.ld_xy + col, x);
  load4<E>(reinterpret_cast<const E*>(a.o) + pr * a.ld_o + col, o);
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] += o[e];
  store4<E>(reinterpret_cast<E*>(a.y) + r * a.ld_xy + col, x);
}

int check(const CatsegClassSeqArgs* a, const char* who) {
  CATSEG_CHECK(a && a->B > 0 && a->T > 0 && a->HW > 0 && a->n_pad >= 0, who);
  CATSEG_CHECK(a->C > 0 && a->C % 8 == 0, who);
  CATSEG_CHECK(a->dtype == CATSEG_BF16 || a->dtype == CATSEG_F32, who);
  return 0;
}

}  // namespace

extern "C" int catseg_class_seq_pack(const CatsegClassSeqArgs* a, void* stream) {
  if (check(a, "class_seq_pack: bad shape / dtype")) return -1;
  CATSEG_CHECK(a->qkv && a->packed, "class_seq_pack: null pointer");
  CATSEG_CHECK(a->n_pad == 0 || (a->k_pad && a->v_pad), "class_seq_pack: padding projections missing");
  CATSEG_CHECK(a->ld_qkv >= 3 * a->C && a->ld_packed >= 3 * a->C, "class_seq_pack: row strides too small");
  CATSEG_CHECK(a->ld_qkv % 4 == 0 && a->ld_packed % 4 == 0 && (uintptr_t)a->qkv % 16 == 0 &&
               (uintptr_t)a->packed % 16 == 0, "class_seq_pack: rows must allow 4-element vector access");
  const int64_t n = a->B * a->HW * (int64_t)(a->T + a->n_pad) * (3 * a->C / 4);
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (a->dtype == CATSEG_BF16)
    hipLaunchKernelGGL(class_seq_pack_kernel<bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, *a, n);
  else
    hipLaunchKernelGGL(class_seq_pack_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, *a, n);
  return catseg_launch_status("class_seq_pack");
}

extern "C" int catseg_class_seq_unpack_add(const CatsegClassSeqArgs* a, void* stream) {
  if (check(a, "class_seq_unpack_add: bad shape / dtype")) return -1;
  CATSEG_CHECK(a->o && a->x && a->y, "class_seq_unpack_add: null pointer");
  CATSEG_CHECK(a->ld_o >= a->C && a->ld_xy >= a->C, "class_seq_unpack_add: row strides too small");
  CATSEG_CHECK(a->ld_o % 4 == 0 && a->ld_xy % 4 == 0 && (uintptr_t)a->o % 16 == 0 && (uintptr_t)a->x % 16 == 0 &&
               (uintptr_t)a->y % 16 == 0, "class_seq_unpack_add: rows must allow 4-element vector access");
  const int64_t n = a->B * (int64_t)a->T * a->HW * (a->C / 4);
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (a->dtype == CATSEG_BF16)
    hipLaunchKernelGGL(class_seq_unpack_add_kernel<bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, *a, n);
  else
    hipLaunchKernelGGL(class_seq_unpack_add_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, *a, n);
  return catseg_launch_status("class_seq_unpack_add");
}
