// Linear ("Transformers are RNNs") class attention of the CAT-Seg class aggregation
// (reference cat_seg/modeling/transformer/model.py:256-286 LinearAttention, called
// by AttentionLayer :338-354 inside ClassTransformerLayer :387-424).
//
// For every pixel (b, p) the sequence is the T classes (rows (b*T + t)*HW + p of the
// q/k/v projections), padded to S = T + n_pad with learned tokens whose projections
// k_pad / v_pad are constant (model.py:397-410): they enter the sums as
// n_pad * phi(k_pad) (x) v_pad and n_pad * phi(k_pad), and their own output rows are
// discarded by the reference (:419-421), so they are never computed here.
//   phi = elu + 1;  KV_h = sum_s phi(k_s,h)^T (v_s,h / S);  Z = 1 / (phi(q).ksum + eps)
//   y = x + (phi(q_h) . KV_h) * Z * S
// One 256-thread workgroup per pixel; KV (4 x 32 x 32) and ksum live in LDS.
#include "common.h"
#include "capi.h"

namespace {

constexpr int CH = 32;      // classes staged per chunk
constexpr int NT = 256;
constexpr int C = 128;      // n_heads * head_dim (host-checked: 4 x 32)
constexpr int D = 32;

DEV float phi(float x) { return x > 0.f ? x + 1.f : __expf(x); }   // elu(x) + 1

template <typename E>
DEV void load16(const E* src, float* dst);   // 16 consecutive elements
template <> DEV void load16<float>(const float* s, float* d) {
#pragma unroll
  for (int i = 0; i < 4; ++i) load4<float>(s + 4 * i, d + 4 * i);
}
template <> DEV void load16<bf16>(const bf16* s, float* d) {
#pragma unroll
  for (int i = 0; i < 4; ++i) load4<bf16>(s + 4 * i, d + 4 * i);
}

template <typename E>
__global__ __launch_bounds__(NT) void linattn_kernel(CatsegLinAttnArgs a) {
  __shared__ float sk[CH][C + 4];
  __shared__ float sv[CH][C + 4];
  __shared__ float skv[C][D + 1];      // [h*32 + i][j]
  __shared__ float sks[C];

  const int tid = threadIdx.x;
  const int64_t pix = blockIdx.x;
  const int64_t b = pix / a.HW;
  const int p = (int)(pix % a.HW);
  const int Tn = a.T;
  const E* Q = reinterpret_cast<const E*>(a.q);
  const E* K = reinterpret_cast<const E*>(a.k);
  const E* V = reinterpret_cast<const E*>(a.v);
  auto row_of = [&](int t) -> int64_t { return (b * Tn + t) * (int64_t)a.HW + p; };

  // ---- phase 1: KV and ksum ----
  const int h = tid >> 6, i = (tid >> 1) & 31, j0 = (tid & 1) * 16;
  float kv[16];
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) kv[jj] = 0.f;
  float ks = 0.f;
  const int srow = tid >> 3, scol = (tid & 7) * 16;
  for (int c0 = 0; c0 < Tn; c0 += CH) {
    float kk[16], vv[16];
    const int t = c0 + srow;
    if (t < Tn) {
      const int64_t r = row_of(t);
      load16<E>(K + r * a.ld_qkv + scol, kk);
      load16<E>(V + r * a.ld_qkv + scol, vv);
#pragma unroll
      for (int e = 0; e < 16; ++e) kk[e] = phi(kk[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) { kk[e] = 0.f; vv[e] = 0.f; }
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) { sk[srow][scol + e] = kk[e]; sv[srow][scol + e] = vv[e]; }
    __syncthreads();
    const int cn = min(CH, Tn - c0);
    for (int c = 0; c < cn; ++c) {
      const float kx = sk[c][h * D + i];
      ks += kx;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) kv[jj] += kx * sv[c][h * D + j0 + jj];
    }
    __syncthreads();
  }
  const float S = (float)(Tn + a.n_pad);
  if (a.n_pad > 0) {
    const float kp = (float)a.n_pad * phi(a.k_pad[h * D + i]);
    ks += kp;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) kv[jj] += kp * a.v_pad[h * D + j0 + jj];
  }
  const float invS = 1.f / S;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) skv[h * D + i][j0 + jj] = kv[jj] * invS;
  if (j0 == 0) sks[h * D + i] = ks;
  __syncthreads();

  // ---- phase 2: outputs ----
  const int c = tid & (C - 1), hh = c >> 5, j = c & 31, par = tid >> 7;
  const E* X = reinterpret_cast<const E*>(a.x);
  E* Y = reinterpret_cast<E*>(a.y);
  for (int c0 = 0; c0 < Tn; c0 += CH) {
    float qq[16];
    const int t = c0 + srow;
    if (t < Tn) {
      load16<E>(Q + row_of(t) * a.ld_qkv + scol, qq);
#pragma unroll
      for (int e = 0; e < 16; ++e) qq[e] = phi(qq[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) qq[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) sk[srow][scol + e] = qq[e];
    __syncthreads();
    const int cn = min(CH, Tn - c0);
    for (int rr = par; rr < cn; rr += 2) {
      float acc = 0.f, z = 0.f;
#pragma unroll
      for (int ii = 0; ii < D; ++ii) {
        const float qv = sk[rr][hh * D + ii];
        acc += qv * skv[hh * D + ii][j];
        z += qv * sks[hh * D + ii];
      }
      const float out = acc * (1.f / (z + a.eps)) * S;
      const int64_t r = row_of(c0 + rr);
      Y[r * a.ld_xy + c] = from_f<E>(to_f<E>(X[r * a.ld_xy + c]) + out);
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int catseg_linear_attention(const CatsegLinAttnArgs* a, void* stream) {
  CATSEG_CHECK(a && a->q && a->k && a->v && a->x && a->y, "linear_attention: null pointer");
  CATSEG_CHECK(a->n_heads * a->head_dim == C && a->head_dim == D, "linear_attention: needs 4 heads x 32");
  CATSEG_CHECK(a->B > 0 && a->T > 0 && a->HW > 0, "linear_attention: empty shape");
  CATSEG_CHECK(a->n_pad == 0 || (a->k_pad && a->v_pad), "linear_attention: padding projections missing");
  const int vn = a->dtype == CATSEG_BF16 ? 8 : 4;
  CATSEG_CHECK(a->ld_qkv % vn == 0, "linear_attention: ld_qkv alignment");
  const unsigned grid = (unsigned)(a->B * a->HW);
  if (a->dtype == CATSEG_BF16)
    hipLaunchKernelGGL(linattn_kernel<bf16>, dim3(grid), dim3(NT), 0, (hipStream_t)stream, *a);
  else
    hipLaunchKernelGGL(linattn_kernel<float>, dim3(grid), dim3(NT), 0, (hipStream_t)stream, *a);
  return catseg_launch_status("linear_attention");
}
