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
// pack: one thread per 16-byte chunk of a row; unpack: one thread per 4 columns.  A wave covers whole
// rows, so both sides stay coalesced.
#include "common.h"
#include "capi.h"

namespace {

template <typename E>
__global__ __launch_bounds__(256) void class_seq_pack_kernel(CatsegClassSeqArgs a, int64_t n) {
  // one 16-byte chunk per thread (8 bf16 / 4 fp32); 32-bit index math (host-checked n < 2^31)
  constexpr int VN = 16 / sizeof(E);
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i >= (unsigned)n) return;
  const unsigned g3 = 3u * (unsigned)a.C / VN;   // chunks per [q | k | v] row
  const unsigned Lp = (unsigned)(a.T + a.n_pad);
  const unsigned pr = i / g3;
  const int col = (int)(i - pr * g3) * VN;
  const unsigned seq = pr / Lp;
  const int t = (int)(pr - seq * Lp);
  const unsigned b = seq / (unsigned)a.HW;
  const int p = (int)(seq - b * (unsigned)a.HW);
  E* dst = reinterpret_cast<E*>(a.packed) + (int64_t)pr * a.ld_packed + col;
  if (t < a.T) {
    const E* src = reinterpret_cast<const E*>(a.qkv) + (((int64_t)b * a.T + t) * a.HW + p) * a.ld_qkv + col;
    st16(dst, ld16(src));
  } else if (col < a.C) {
    st16(dst, make_uint4(0u, 0u, 0u, 0u));
  } else {
    const float* src = col < 2 * a.C ? a.k_pad + (col - a.C) : a.v_pad + (col - 2 * a.C);
#pragma unroll
    for (int h = 0; h < VN / 4; ++h) store4<E>(dst + 4 * h, src + 4 * h);
  }
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
  const int vn = a->dtype == CATSEG_BF16 ? 8 : 4;
  CATSEG_CHECK(a->ld_qkv % vn == 0 && a->ld_packed % vn == 0, "class_seq_pack: rows must allow 16-byte chunks");
  const int64_t n = a->B * a->HW * (int64_t)(a->T + a->n_pad) * (3 * a->C / vn);
  CATSEG_CHECK(n < (1LL << 31), "class_seq_pack: too many chunks for 32-bit indexing");
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
