// Training-side normalisation, activation, reduction and layout kernels.
// fp32 throughout; every reduction runs in a fixed order over a grid that depends on the
// shape only, so gradients are bit-reproducible run to run.
//
//   catseg_layernorm_backward        nn.LayerNorm backward (model.py:152,158,233,368-369)
//   catseg_act_forward / _backward   GELU (exact erf, timm Mlp model.py:159), ReLU (model.py:362-366,
//                                    616-630), QuickGELU (model_vpt.py:165-167)
//   catseg_groupnorm_stats_rows      nn.GroupNorm statistics of an NHWC map (model.py:529,532)
//   catseg_groupnorm_relu_backward   GroupNorm + ReLU backward (dx, dgamma, dbeta)
//   catseg_sum_classes / _pixels     the reductions behind repeat/expand over T (model.py:249,551-554)
//                                    and the per-class guidance broadcast (model.py:405-409)
//   catseg_avgpool_backward_rows     nn.AvgPool2d backward (model.py:374-385)
//   catseg_upsample_ac_backward_rows bilinear align_corners=True backward (model.py:415-416)
//   catseg_l2normalize_backward      F.normalize backward (model.py:649-650)
//   catseg_convt_gather              the ConvTranspose2d(k, stride k) output grad as GEMM rows
#include "common.h"
#include "capi.h"
#include "catseg_hip_train.h"

namespace {

// ---------------------------------------------------------------------------------- LayerNorm
constexpr int LN_WG_MAX = 1024;

int ln_grid(int64_t rows) {
  const int64_t wg = (rows + 3) / 4;
  return (int)(wg < LN_WG_MAX ? wg : LN_WG_MAX);
}

// one wave per row, VPL = cols / 64 values per lane (column c = lane + 64 j)
template <int VPL>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x, int64_t ld_x,
                                                     const float* __restrict__ gamma, const float* __restrict__ dy,
                                                     int64_t ld_dy, float* __restrict__ dx, int64_t ld_dx, int acc_dx,
                                                     int64_t rows, int cols, float eps, float* __restrict__ part) {
  __shared__ float red[4][2 * 64 * VPL];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  float gm[VPL], dg[VPL], db[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) { gm[j] = gamma[lane + 64 * j]; dg[j] = 0.f; db[j] = 0.f; }
  const float inv = 1.f / (float)cols;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < rows; r += nwaves) {
    float xv[VPL], dv[VPL];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      xv[j] = x[r * ld_x + lane + 64 * j];
      dv[j] = dy[r * ld_dy + lane + 64 * j];
      s += xv[j];
    }
    const float mu = wave_sum(s) * inv;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) { const float d = xv[j] - mu; q += d * d; }
    const float rstd = 1.f / sqrtf(wave_sum(q) * inv + eps);
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      xv[j] = (xv[j] - mu) * rstd;                 // xhat
      const float g = dv[j] * gm[j];
      a += g;
      b += g * xv[j];
      dg[j] += dv[j] * xv[j];
      db[j] += dv[j];
    }
    a = wave_sum(a) * inv;
    b = wave_sum(b) * inv;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      float v = rstd * (dv[j] * gm[j] - a - xv[j] * b);
      float* p = dx + r * ld_dx + lane + 64 * j;
      if (acc_dx) v += *p;
      *p = v;
    }
  }
  if (!part) return;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    red[wave][lane + 64 * j] = dg[j];
    red[wave][64 * VPL + lane + 64 * j] = db[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * 64 * VPL; c += 256)
    part[(int64_t)blockIdx.x * 2 * cols + c] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

// dgamma / dbeta = sum of the per-workgroup partials: 16 columns x 16 partial lanes per workgroup
// (lane z takes partials z, z + 16, ...), then a fixed tree over the lanes
__global__ __launch_bounds__(256) void ln_param_final_kernel(const float* __restrict__ part, int nwg, int cols,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             int acc) {
  __shared__ float red[256];
  const int ci = threadIdx.x & 15, zl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + ci;
  float s = 0.f;
  if (c < 2 * cols) {
#pragma unroll 8
    for (int w = zl; w < nwg; w += 16) s += part[(int64_t)w * 2 * cols + c];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off >= 16; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x < 16 && c < 2 * cols) {
    float* o = c < cols ? dgamma + c : dbeta + (c - cols);
    *o = acc ? *o + red[threadIdx.x] : red[threadIdx.x];
  }
}

// ---------------------------------------------------------------------------------- activations
constexpr float INV_SQRT2 = 0.70710678118654752f, INV_SQRT2PI = 0.39894228040143268f;

DEV float act_f(float v, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_GELU: return 0.5f * v * (1.f + erff(v * INV_SQRT2));
    case ACT_QUICKGELU: return v / (1.f + expf(-1.702f * v));
    default: return v;
  }
}
DEV float act_d(float v, int act) {   // d act / d v
  switch (act) {
    case ACT_RELU: return v > 0.f ? 1.f : 0.f;
    case ACT_GELU: return 0.5f * (1.f + erff(v * INV_SQRT2)) + v * INV_SQRT2PI * expf(-0.5f * v * v);
    case ACT_QUICKGELU: {
      const float s = 1.f / (1.f + expf(-1.702f * v));
      return s + 1.702f * v * s * (1.f - s);
    }
    default: return 1.f;
  }
}

__global__ __launch_bounds__(256) void act_fwd_kernel(const float* __restrict__ u, float* __restrict__ a, int64_t n4,
                                                      int act) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 v = reinterpret_cast<const float4*>(u)[i];
  v.x = act_f(v.x, act); v.y = act_f(v.y, act); v.z = act_f(v.z, act); v.w = act_f(v.w, act);
  reinterpret_cast<float4*>(a)[i] = v;
}
__global__ __launch_bounds__(256) void act_bwd_kernel(const float* __restrict__ u, const float* __restrict__ dy,
                                                      float* __restrict__ du, int64_t n4, int act) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4 v = reinterpret_cast<const float4*>(u)[i];
  float4 d = reinterpret_cast<const float4*>(dy)[i];
  d.x *= act_d(v.x, act); d.y *= act_d(v.y, act); d.z *= act_d(v.z, act); d.w *= act_d(v.w, act);
  reinterpret_cast<float4*>(du)[i] = d;
}

// ---------------------------------------------------------------------------------- GroupNorm
// NHWC slices x[s][p][c] (S slices of HW pixels x C channels), groups of cpg consecutive channels.
// The slice is cut into chunks of GN_PPC(C) pixels; one 256-thread workgroup per (chunk, slice),
// thread t owns channel quad t % (C/4) (a float4) and pixels t / (C/4) + k * (1024 / C), k < 16,
// so every load is a coalesced float4 and a chunk is 16 float4 per thread, held in registers.
// Partials reduce across the threads of one quad by a fixed binary tree (strides 128 .. C/4),
// chunks combine in chunk order: deterministic, grid a function of the shape only.
// Requires C/4 a power of two <= 256 and cpg % 4 == 0 (the decoder: C 32 / 64 / 128, cpg 16).
constexpr int GN_K = 16;                       // float4 per thread per chunk
DEV int gn_ppc(int C) { return GN_K * 1024 / C; }
int gn_chunks(int64_t HW, int C) { return (int)((HW + GN_K * 1024 / C - 1) / (GN_K * 1024 / C)); }
bool gn_shape_ok(int C, int cpg) {
  const int nq = C / 4;
  return C % 4 == 0 && nq > 0 && nq <= 256 && (nq & (nq - 1)) == 0 && cpg % 4 == 0 && C % cpg == 0;
}

// in-place tree over red[NV][256]: afterwards red[v][q], q < nq, holds quad q's sum (fixed order)
template <int NV>
DEV void quad_tree(float (*red)[256], int nq) {
  for (int off = 128; off >= nq; off >>= 1) {
    if ((int)threadIdx.x < off) {
#pragma unroll
      for (int v = 0; v < NV; ++v) red[v][threadIdx.x] += red[v][threadIdx.x + off];
    }
    __syncthreads();
  }
}

// statistics, pass 1: per (slice, chunk, group) {sum, M2 about the chunk's own group mean}
__global__ __launch_bounds__(256) void gn_stats_chunk_kernel(const float* __restrict__ x, int64_t HW, int C, int cpg,
                                                             float* __restrict__ part) {
  __shared__ float red[1][256];
  __shared__ float gmean[256];
  const int nq = C >> 2, G = C / cpg, qpg = cpg >> 2;
  const int q = threadIdx.x & (nq - 1), pl = threadIdx.x / nq, ppi = 256 / nq;
  const int64_t s = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * gn_ppc(C);
  const int64_t pend = p0 + gn_ppc(C) < HW ? p0 + gn_ppc(C) : HW;
  const float4* xs = reinterpret_cast<const float4*>(x + s * HW * C) + q;
  float4 v[GN_K];
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < GN_K; ++k) {
    const int64_t p = p0 + pl + (int64_t)k * ppi;
    v[k] = p < pend ? xs[p * nq] : make_float4(0.f, 0.f, 0.f, 0.f);
    acc += ((v[k].x + v[k].y) + v[k].z) + v[k].w;
  }
  red[0][threadIdx.x] = acc;
  __syncthreads();
  quad_tree<1>(red, nq);
  const float cnt = (float)((pend - p0) * cpg);
  if ((int)threadIdx.x < G) {
    float t = 0.f;
    for (int j = 0; j < qpg; ++j) t += red[0][threadIdx.x * qpg + j];
    gmean[threadIdx.x] = t / cnt;
    part[((s * gridDim.x + blockIdx.x) * G + threadIdx.x) * 2 + 0] = t;
  }
  __syncthreads();
  const float mu = gmean[(q * 4) / cpg];
  acc = 0.f;
#pragma unroll
  for (int k = 0; k < GN_K; ++k) {
    const int64_t p = p0 + pl + (int64_t)k * ppi;
    if (p < pend) {
      const float a = v[k].x - mu, b = v[k].y - mu, c = v[k].z - mu, d = v[k].w - mu;
      acc += ((a * a + b * b) + c * c) + d * d;
    }
  }
  red[0][threadIdx.x] = acc;
  __syncthreads();
  quad_tree<1>(red, nq);
  if ((int)threadIdx.x < G) {
    float t = 0.f;
    for (int j = 0; j < qpg; ++j) t += red[0][threadIdx.x * qpg + j];
    part[((s * gridDim.x + blockIdx.x) * G + threadIdx.x) * 2 + 1] = t;
  }
}

// statistics, pass 2: one thread per (slice, group) combines its chunks in order (Chan et al.'s
// pairwise mean / M2 update) -> mean, rstd (biased variance, as nn.GroupNorm)
__global__ __launch_bounds__(256) void gn_stats_final_kernel(const float* __restrict__ part, int64_t S, int64_t HW,
                                                             int C, int cpg, int nch, float eps, float* __restrict__ mean,
                                                             float* __restrict__ rstd) {
  const int G = C / cpg;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= S * G) return;
  const int64_t s = i / G;
  const int g = (int)(i % G);
  const int ppc = gn_ppc(C);
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int k = 0; k < nch; ++k) {
    const int64_t px = (k + 1) * (int64_t)ppc < HW ? ppc : HW - (int64_t)k * ppc;
    const float nb = (float)(px * cpg);
    const float* pp = part + ((s * nch + k) * G + g) * 2;
    const float mb = pp[0] / nb;
    const float nn = n + nb;
    const float dl = mb - mu;
    mu += dl * (nb / nn);
    m2 += pp[1] + dl * dl * (n * nb / nn);
    n = nn;
  }
  mean[i] = mu;
  rstd[i] = 1.f / sqrtf(m2 / n + eps);
}

// GroupNorm+ReLU backward, pass 1: per (slice, chunk, channel) S1 = sum dyr, S2 = sum dyr * xhat,
// dyr = dy where the ReLU passed (gamma * xhat + beta > 0)
__global__ __launch_bounds__(256) void gn_bwd_chunk_reduce_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                                  int64_t HW, int C, int cpg,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ rstd,
                                                                  const float* __restrict__ gamma,
                                                                  const float* __restrict__ beta, float* __restrict__ part) {
  __shared__ float red[8][256];
  const int nq = C >> 2, G = C / cpg;
  const int q = threadIdx.x & (nq - 1), pl = threadIdx.x / nq, ppi = 256 / nq;
  const int64_t s = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * gn_ppc(C);
  const int64_t pend = p0 + gn_ppc(C) < HW ? p0 + gn_ppc(C) : HW;
  const int64_t sg = s * G + (q * 4) / cpg;
  const float mu = mean[sg], rs = rstd[sg];
  const float4 ga = reinterpret_cast<const float4*>(gamma)[q], be = reinterpret_cast<const float4*>(beta)[q];
  const float4* xs = reinterpret_cast<const float4*>(x + s * HW * C) + q;
  const float4* ds = reinterpret_cast<const float4*>(dy + s * HW * C) + q;
  float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k = 0; k < GN_K; ++k) {
    const int64_t p = p0 + pl + (int64_t)k * ppi;
    if (p < pend) {
      const float4 xv = xs[p * nq], dv = ds[p * nq];
      const float xh[4] = {(xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs};
      const float gg[4] = {ga.x, ga.y, ga.z, ga.w}, bb[4] = {be.x, be.y, be.z, be.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = (gg[j] * xh[j] + bb[j]) > 0.f ? dd[j] : 0.f;
        a[j] += d;
        b[j] += d * xh[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) { red[j][threadIdx.x] = a[j]; red[4 + j][threadIdx.x] = b[j]; }
  __syncthreads();
  quad_tree<8>(red, nq);
  if ((int)threadIdx.x < nq) {
    float* out = part + ((s * gridDim.x + blockIdx.x) * C + threadIdx.x * 4) * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) { out[2 * j] = red[j][threadIdx.x]; out[2 * j + 1] = red[4 + j][threadIdx.x]; }
  }
}

// pass 2: per (slice, channel) totals over the chunks, in chunk order -> sums[s][c][2]
__global__ __launch_bounds__(256) void gn_bwd_chan_kernel(const float* __restrict__ part, int64_t S, int C, int nch,
                                                          float* __restrict__ sums) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= S * C) return;
  const int64_t s = i / C;
  const int c = (int)(i % C);
  float a = 0.f, b = 0.f;
  for (int k = 0; k < nch; ++k) {
    const float* pp = part + ((s * nch + k) * C + c) * 2;
    a += pp[0];
    b += pp[1];
  }
  sums[i * 2 + 0] = a;
  sums[i * 2 + 1] = b;
}

// pass 3: dx = rstd * (dyr * gamma - (A_g + xhat * B_g) / n), A_g = sum_c gamma_c S1_c, B_g = sum_c gamma_c S2_c
// (A_g, B_g formed once per thread, channels in ascending order)
__global__ __launch_bounds__(256) void gn_bwd_chunk_apply_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                                 float* __restrict__ dx, int64_t HW, int C, int cpg,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ rstd,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta,
                                                                 const float* __restrict__ sums) {
  const int nq = C >> 2, G = C / cpg;
  const int q = threadIdx.x & (nq - 1), pl = threadIdx.x / nq, ppi = 256 / nq;
  const int64_t s = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * gn_ppc(C);
  const int64_t pend = p0 + gn_ppc(C) < HW ? p0 + gn_ppc(C) : HW;
  const int g = (q * 4) / cpg;
  const int64_t sg = s * G + g;
  float A = 0.f, Bv = 0.f;
  for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
    A += gamma[c] * sums[(s * C + c) * 2 + 0];
    Bv += gamma[c] * sums[(s * C + c) * 2 + 1];
  }
  const float inv_n = 1.f / (float)(HW * cpg);
  const float mu = mean[sg], rs = rstd[sg];
  const float4 ga = reinterpret_cast<const float4*>(gamma)[q], be = reinterpret_cast<const float4*>(beta)[q];
  const float gg[4] = {ga.x, ga.y, ga.z, ga.w}, bb[4] = {be.x, be.y, be.z, be.w};
  const float4* xs = reinterpret_cast<const float4*>(x + s * HW * C) + q;
  const float4* ds = reinterpret_cast<const float4*>(dy + s * HW * C) + q;
  float4* os = reinterpret_cast<float4*>(dx + s * HW * C) + q;
#pragma unroll 4
  for (int k = 0; k < GN_K; ++k) {
    const int64_t p = p0 + pl + (int64_t)k * ppi;
    if (p < pend) {
      const float4 xv = xs[p * nq], dv = ds[p * nq];
      const float xx[4] = {xv.x, xv.y, xv.z, xv.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xh = (xx[j] - mu) * rs;
        const float d = (gg[j] * xh + bb[j]) > 0.f ? dd[j] : 0.f;
        o[j] = rs * (d * gg[j] - (A + xh * Bv) * inv_n);
      }
      os[p * nq] = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

// pass 4: dgamma[c] = sum_s S2[s][c], dbeta[c] = sum_s S1[s][c]; one workgroup per channel,
// thread t takes slices t, t + 256, ..., then a fixed tree over the 256 threads
__global__ __launch_bounds__(256) void gn_param_kernel(const float* __restrict__ sums, int64_t S, int C,
                                                       float* __restrict__ dgamma, float* __restrict__ dbeta, int acc) {
  __shared__ float red[2][256];
  const int c = blockIdx.x;
  float a = 0.f, b = 0.f;
  for (int64_t s = threadIdx.x; s < S; s += 256) { a += sums[(s * C + c) * 2 + 0]; b += sums[(s * C + c) * 2 + 1]; }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  quad_tree<2>(red, 1);
  if (threadIdx.x == 0) {
    dgamma[c] = acc ? dgamma[c] + red[1][0] : red[1][0];
    dbeta[c] = acc ? dbeta[c] + red[0][0] : red[0][0];
  }
}

// ---------------------------------------------------------------------------------- reductions
// out[b*HW + p][c] (+)= sum_t x[((b*T + t)*HW + p)*ld_x + c]
__global__ __launch_bounds__(256) void sum_classes_kernel(const float* __restrict__ x, int64_t ld_x, int64_t B, int T,
                                                          int64_t HW, int C, float* __restrict__ out, int64_t ld_out,
                                                          int beta) {
  const int c4n = C / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= B * HW * c4n) return;
  const int c = (int)(i % c4n) * 4;
  const int64_t bp = i / c4n, b = bp / HW, p = bp % HW;
  float4 s = make_float4(0, 0, 0, 0);
#pragma unroll 8
  for (int t = 0; t < T; ++t) {
    const float4 v = *reinterpret_cast<const float4*>(x + ((b * T + t) * HW + p) * ld_x + c);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  float4* o = reinterpret_cast<float4*>(out + bp * ld_out + c);
  if (beta) { const float4 v = *o; s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w; }
  *o = s;
}

// out[t][c] (+)= sum_{b, p} x[((b*T + t)*HW + p)*ld_x + c]: one workgroup per (t, 64 columns)
__global__ __launch_bounds__(256) void sum_pixels_kernel(const float* __restrict__ x, int64_t ld_x, int64_t B, int T,
                                                         int64_t HW, int C, float* __restrict__ out, int64_t ld_out,
                                                         int beta) {
  __shared__ float red[4][64];
  const int t = blockIdx.x;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  float s = 0.f;
  if (c < C)
    for (int64_t b = 0; b < B; ++b) {
      const float* base = x + (b * T + t) * HW * ld_x + c;
#pragma unroll 8
      for (int64_t p = q; p < HW; p += 4) s += base[p * ld_x];
    }
  red[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && c < C) {
    const int l = threadIdx.x;
    float v = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
    float* o = out + (int64_t)t * ld_out + c;
    *o = beta ? *o + v : v;
  }
}

// ---------------------------------------------------------------------------------- pooling / resampling
// dx[s][y][x][c] (+)= dxp[s][y/ph][x/pw][c] / (ph*pw) inside the pooled region, else 0 (+ nothing)
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const float* __restrict__ dxp, int64_t S, int H, int W, int C,
                                                          int ph, int pw, float* __restrict__ dx, int beta) {
  const int c4n = C / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= S * H * W * c4n) return;
  const int c = (int)(i % c4n) * 4;
  const int64_t pix = i / c4n;
  const int xw = (int)(pix % W), yh = (int)((pix / W) % H);
  const int64_t s = pix / ((int64_t)H * W);
  const int Hp = H / ph, Wp = W / pw;
  float4 v = make_float4(0, 0, 0, 0);
  if (yh / ph < Hp && xw / pw < Wp) {
    v = *reinterpret_cast<const float4*>(dxp + ((s * Hp + yh / ph) * Wp + xw / pw) * C + c);
    const float k = 1.f / (float)(ph * pw);
    v.x *= k; v.y *= k; v.z *= k; v.w *= k;
  }
  float4* o = reinterpret_cast<float4*>(dx + pix * C + c);
  if (beta) { const float4 u = *o; v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w; }
  *o = v;
}

// align_corners=True source coordinate and its two taps (as the forward kernel / torch compute them)
DEV void ac_taps(int y, int H, int Hp, int& y0, int& y1, float& w1) {
  const float sc = H > 1 ? (float)(Hp - 1) / (float)(H - 1) : 0.f;
  const float src = sc * (float)y;
  y0 = (int)src;
  if (y0 > Hp - 1) y0 = Hp - 1;
  y1 = y0 + 1 < Hp ? y0 + 1 : Hp - 1;
  w1 = src - (float)y0;
}

// dxp[s][qy][qx][c] (+)= sum_{y, x} wy(y, qy) wx(x, qx) dy[s][y][x][c]  (gather form, no atomics)
__global__ __launch_bounds__(256) void upsample_ac_bwd_kernel(const float* __restrict__ dy, int64_t S, int H, int W,
                                                              int C, int Hp, int Wp, float* __restrict__ dxp, int beta) {
  const int c4n = C / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= S * Hp * Wp * c4n) return;
  const int c = (int)(i % c4n) * 4;
  const int64_t pix = i / c4n;
  const int qx = (int)(pix % Wp), qy = (int)((pix / Wp) % Hp);
  const int64_t s = pix / ((int64_t)Hp * Wp);
  // fine rows whose taps can reach qy: src in (qy - 1, qy + 1]
  const float sy = Hp > 1 ? (float)(H - 1) / (float)(Hp - 1) : 0.f, sx = Wp > 1 ? (float)(W - 1) / (float)(Wp - 1) : 0.f;
  int ylo = (int)floorf((float)(qy - 1) * sy) - 1, yhi = (int)ceilf((float)(qy + 1) * sy) + 1;
  int xlo = (int)floorf((float)(qx - 1) * sx) - 1, xhi = (int)ceilf((float)(qx + 1) * sx) + 1;
  ylo = ylo < 0 ? 0 : ylo; xlo = xlo < 0 ? 0 : xlo;
  yhi = yhi > H - 1 ? H - 1 : yhi; xhi = xhi > W - 1 ? W - 1 : xhi;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int y = ylo; y <= yhi; ++y) {
    int y0, y1; float ly;
    ac_taps(y, H, Hp, y0, y1, ly);
    const float wy = (y0 == qy ? 1.f - ly : 0.f) + (y1 == qy ? ly : 0.f);
    if (wy == 0.f) continue;
    for (int x = xlo; x <= xhi; ++x) {
      int x0, x1; float lx;
      ac_taps(x, W, Wp, x0, x1, lx);
      const float wx = (x0 == qx ? 1.f - lx : 0.f) + (x1 == qx ? lx : 0.f);
      if (wx == 0.f) continue;
      const float w = wy * wx;
      const float4 v = *reinterpret_cast<const float4*>(dy + ((s * H + y) * W + x) * C + c);
      acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
    }
  }
  float4* o = reinterpret_cast<float4*>(dxp + pix * C + c);
  if (beta) { const float4 u = *o; acc.x += u.x; acc.y += u.y; acc.z += u.z; acc.w += u.w; }
  *o = acc;
}

// ---------------------------------------------------------------------------------- l2 normalize
template <int VPL>
__global__ __launch_bounds__(256) void l2n_bwd_kernel(const float* __restrict__ x, int64_t ld_x, RowMap inmap,
                                                      const float* __restrict__ dy, int64_t ld_dy, float* __restrict__ dx,
                                                      int64_t ld_dx, RowMap outmap, int beta, int64_t rows, int cols,
                                                      float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + rowmap(inmap, r) * ld_x;
  const float* dr = dy + r * ld_dy;
  float xv[VPL], dv[VPL];
  float ss = 0.f, dd = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    xv[j] = c < cols ? xr[c] : 0.f;
    dv[j] = c < cols ? dr[c] : 0.f;
    ss += xv[j] * xv[j];
    dd += xv[j] * dv[j];
  }
  const float nrm = sqrtf(wave_sum(ss));
  dd = wave_sum(dd);
  const float den = fmaxf(nrm, eps);
  // y = x / den; dx = (dy - y (y . dy)) / den when ||x|| > eps, else dy / eps
  const float k = nrm > eps ? dd / (den * den) : 0.f;
  float* o = dx + rowmap(outmap, r) * ld_dx;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c >= cols) continue;
    float v = (dv[j] - xv[j] * k) / den;
    if (beta) v += o[c];
    o[c] = v;
  }
}

// ---------------------------------------------------------------------------------- ConvTranspose gather
// g[m][(ky*k + kx)*cout + co] = dout[s][y*k + ky][x*k + kx][co] (dout pixel stride ld), m = (s, y, x)
__global__ __launch_bounds__(256) void convt_gather_kernel(const float* __restrict__ dout, int64_t ld, int64_t M,
                                                           int hin, int win, int k, int cout, float* __restrict__ g) {
  const int n4 = k * k * cout / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * n4) return;
  const int64_t m = i / n4;
  const int n = (int)(i % n4) * 4;
  const int co = n % cout, kk = n / cout, ky = kk / k, kx = kk % k;
  const int xw = (int)(m % win), yh = (int)((m / win) % hin);
  const int64_t s = m / ((int64_t)hin * win);
  const int64_t src = ((s * hin * k + (int64_t)yh * k + ky) * ((int64_t)win * k) + (int64_t)xw * k + kx) * ld + co;
  *reinterpret_cast<float4*>(g + m * (int64_t)k * k * cout + n) = *reinterpret_cast<const float4*>(dout + src);
}

// ---------------------------------------------------------------------------------- elementwise
__global__ __launch_bounds__(256) void axpby_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                    float* __restrict__ out, int64_t n4, float alpha, float beta) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4 a = reinterpret_cast<const float4*>(x)[i];
  float4 v = make_float4(alpha * a.x, alpha * a.y, alpha * a.z, alpha * a.w);
  if (y) {
    const float4 b = reinterpret_cast<const float4*>(y)[i];
    v.x += beta * b.x; v.y += beta * b.y; v.z += beta * b.z; v.w += beta * b.w;
  }
  reinterpret_cast<float4*>(out)[i] = v;
}
// out[idx[r]][c] = in[r][c] (the EOT gather's backward, model_vpt.py:436)
__global__ __launch_bounds__(256) void scatter_rows_kernel(const float* __restrict__ in, int64_t ld_in,
                                                           const int32_t* __restrict__ idx, int64_t rows, int64_t cols,
                                                           float* __restrict__ out, int64_t ld_out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols, c = i % cols;
  out[(int64_t)idx[r] * ld_out + c] = in[r * ld_in + c];
}
__global__ __launch_bounds__(256) void add_dev_scalar_kernel(float* __restrict__ x, int64_t n, const float* __restrict__ s) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] += *s;
}

bool rowmap_ok(const CatsegRowMap& m) { return m.d1 > 0 && m.m1 > 0 && m.d2 > 0 && m.m2 > 0; }
RowMap rm(const CatsegRowMap& m) { return RowMap{m.d1, m.m1, m.s1, m.d2, m.m2, m.s2, m.off}; }

unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" int64_t catseg_layernorm_backward_workspace(int64_t rows, int64_t cols) {
  return rows > 0 && cols > 0 ? (int64_t)ln_grid(rows) * 2 * cols * (int64_t)sizeof(float) : 0;
}

extern "C" int catseg_layernorm_backward(const float* x, int64_t ld_x, const float* gamma, const float* dy, int64_t ld_dy,
                                         float* dx, int64_t ld_dx, int acc_dx, int64_t rows, int64_t cols, float eps,
                                         float* dgamma, float* dbeta, int acc_param, void* workspace,
                                         int64_t workspace_bytes, void* stream) {
  CATSEG_CHECK(x && gamma && dy && dx && rows > 0, "layernorm_backward: bad args");
  CATSEG_CHECK(cols % 64 == 0 && cols >= 64 && cols <= 1024, "layernorm_backward: cols must be a multiple of 64, <= 1024");
  CATSEG_CHECK(!dgamma == !dbeta, "layernorm_backward: dgamma and dbeta go together");
  const int grid = ln_grid(rows);
  if (dgamma)
    CATSEG_CHECK(workspace && workspace_bytes >= (int64_t)grid * 2 * cols * (int64_t)sizeof(float),
                 "layernorm_backward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = dgamma ? (float*)workspace : nullptr;
  const int vpl = (int)(cols / 64);
#define LNB(V) hipLaunchKernelGGL((ln_bwd_kernel<V>), dim3(grid), dim3(256), 0, st, x, ld_x, gamma, dy, ld_dy, dx, ld_dx, \
                                  acc_dx, rows, (int)cols, eps, part)
  switch (vpl) {
    case 1: LNB(1); break;
    case 2: LNB(2); break;
    case 4: LNB(4); break;
    case 8: LNB(8); break;
    case 12: LNB(12); break;
    case 16: LNB(16); break;
    default: CATSEG_FAIL("layernorm_backward: cols must be 64, 128, 256, 512, 768 or 1024");
  }
#undef LNB
  if (dgamma)
    hipLaunchKernelGGL(ln_param_final_kernel, dim3((unsigned)((2 * cols + 15) / 16)), dim3(256), 0, st,
                       (const float*)part, grid, (int)cols, dgamma, dbeta, acc_param);
  return catseg_launch_status("layernorm_backward");
}

extern "C" int catseg_act_forward(const float* u, float* a, int64_t n, int act, void* stream) {
  CATSEG_CHECK(u && a && n > 0 && n % 4 == 0, "act_forward: bad args (n % 4 == 0)");
  CATSEG_CHECK(act == ACT_NONE || act == ACT_RELU || act == ACT_GELU || act == ACT_QUICKGELU, "act_forward: bad act");
  hipLaunchKernelGGL(act_fwd_kernel, dim3(blocks(n / 4)), dim3(256), 0, (hipStream_t)stream, u, a, n / 4, act);
  return catseg_launch_status("act_forward");
}

extern "C" int catseg_act_backward(const float* u, const float* dy, float* du, int64_t n, int act, void* stream) {
  CATSEG_CHECK(u && dy && du && n > 0 && n % 4 == 0, "act_backward: bad args (n % 4 == 0)");
  CATSEG_CHECK(act == ACT_NONE || act == ACT_RELU || act == ACT_GELU || act == ACT_QUICKGELU, "act_backward: bad act");
  hipLaunchKernelGGL(act_bwd_kernel, dim3(blocks(n / 4)), dim3(256), 0, (hipStream_t)stream, u, dy, du, n / 4, act);
  return catseg_launch_status("act_backward");
}

extern "C" int64_t catseg_groupnorm_stats_rows_workspace(int64_t S, int64_t HW, int C, int cpg) {
  if (S <= 0 || HW <= 0 || C <= 0 || cpg <= 0 || !gn_shape_ok(C, cpg)) return 0;
  return S * gn_chunks(HW, C) * (C / cpg) * 2 * (int64_t)sizeof(float);
}

extern "C" int catseg_groupnorm_stats_rows(const float* x, int64_t S, int64_t HW, int C, int cpg, float eps, float* mean,
                                           float* rstd, void* workspace, int64_t workspace_bytes, void* stream) {
  CATSEG_CHECK(x && mean && rstd && S > 0 && HW > 0 && cpg > 0, "groupnorm_stats_rows: bad args");
  CATSEG_CHECK(gn_shape_ok(C, cpg), "groupnorm_stats_rows: needs C/4 a power of two <= 256 and cpg % 4 == 0");
  CATSEG_CHECK(((uintptr_t)x % 16) == 0, "groupnorm_stats_rows: x must be 16-byte aligned");
  const int nch = gn_chunks(HW, C);
  CATSEG_CHECK(S < 65536 && nch < (1 << 30), "groupnorm_stats_rows: too many slices");
  CATSEG_CHECK(workspace && workspace_bytes >= S * nch * (C / cpg) * 2 * (int64_t)sizeof(float),
               "groupnorm_stats_rows: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)workspace;
  hipLaunchKernelGGL(gn_stats_chunk_kernel, dim3((unsigned)nch, (unsigned)S), dim3(256), 0, st, x, HW, C, cpg, part);
  hipLaunchKernelGGL(gn_stats_final_kernel, dim3(blocks(S * (C / cpg))), dim3(256), 0, st, (const float*)part, S, HW, C,
                     cpg, nch, eps, mean, rstd);
  return catseg_launch_status("groupnorm_stats_rows");
}

extern "C" int64_t catseg_groupnorm_relu_backward_workspace(int64_t S, int64_t HW, int C) {
  if (S <= 0 || HW <= 0 || C <= 0 || C % 4 != 0) return 0;
  return (S * gn_chunks(HW, C) * C * 2 + S * C * 2) * (int64_t)sizeof(float);
}

extern "C" int catseg_groupnorm_relu_backward(const float* x, const float* dy, float* dx, int64_t S, int64_t HW, int C,
                                              int cpg, const float* mean, const float* rstd, const float* gamma,
                                              const float* beta, float* dgamma, float* dbeta, int acc_param,
                                              void* workspace, int64_t workspace_bytes, void* stream) {
  CATSEG_CHECK(x && dy && dx && mean && rstd && gamma && beta && dgamma && dbeta, "groupnorm_relu_backward: null pointer");
  CATSEG_CHECK(S > 0 && HW > 0 && cpg > 0, "groupnorm_relu_backward: bad shape");
  CATSEG_CHECK(gn_shape_ok(C, cpg), "groupnorm_relu_backward: needs C/4 a power of two <= 256 and cpg % 4 == 0");
  CATSEG_CHECK(((uintptr_t)x % 16) == 0 && ((uintptr_t)dy % 16) == 0 && ((uintptr_t)dx % 16) == 0 &&
                   ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0,
               "groupnorm_relu_backward: x, dy, dx, gamma, beta must be 16-byte aligned");
  const int nch = gn_chunks(HW, C);
  CATSEG_CHECK(S < 65536, "groupnorm_relu_backward: too many slices");
  CATSEG_CHECK(workspace && workspace_bytes >= (S * nch * C * 2 + S * C * 2) * (int64_t)sizeof(float),
               "groupnorm_relu_backward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)workspace;
  float* sums = part + S * nch * C * 2;
  const dim3 grid((unsigned)nch, (unsigned)S);
  hipLaunchKernelGGL(gn_bwd_chunk_reduce_kernel, grid, dim3(256), 0, st, x, dy, HW, C, cpg, mean, rstd, gamma, beta, part);
  hipLaunchKernelGGL(gn_bwd_chan_kernel, dim3(blocks(S * C)), dim3(256), 0, st, (const float*)part, S, C, nch, sums);
  hipLaunchKernelGGL(gn_bwd_chunk_apply_kernel, grid, dim3(256), 0, st, x, dy, dx, HW, C, cpg, mean, rstd, gamma, beta,
                     (const float*)sums);
  hipLaunchKernelGGL(gn_param_kernel, dim3((unsigned)C), dim3(256), 0, st, (const float*)sums, S, C, dgamma, dbeta,
                     acc_param);
  return catseg_launch_status("groupnorm_relu_backward");
}

extern "C" int catseg_sum_classes(const float* x, int64_t ld_x, int64_t B, int T, int64_t HW, int C, float* out,
                                  int64_t ld_out, int beta, void* stream) {
  CATSEG_CHECK(x && out && B > 0 && T > 0 && HW > 0 && C > 0 && C % 4 == 0 && ld_x % 4 == 0 && ld_out % 4 == 0,
               "sum_classes: bad args");
  hipLaunchKernelGGL(sum_classes_kernel, dim3(blocks(B * HW * (C / 4))), dim3(256), 0, (hipStream_t)stream, x, ld_x, B, T,
                     HW, C, out, ld_out, beta);
  return catseg_launch_status("sum_classes");
}

extern "C" int catseg_sum_pixels(const float* x, int64_t ld_x, int64_t B, int T, int64_t HW, int C, float* out,
                                 int64_t ld_out, int beta, void* stream) {
  CATSEG_CHECK(x && out && B > 0 && T > 0 && HW > 0 && C > 0, "sum_pixels: bad args");
  hipLaunchKernelGGL(sum_pixels_kernel, dim3((unsigned)T, (unsigned)((C + 63) / 64)), dim3(256), 0, (hipStream_t)stream,
                     x, ld_x, B, T, HW, C, out, ld_out, beta);
  return catseg_launch_status("sum_pixels");
}

extern "C" int catseg_avgpool_backward_rows(const float* dxp, int64_t S, int H, int W, int C, int ph, int pw, float* dx,
                                            int beta, void* stream) {
  CATSEG_CHECK(dxp && dx && S > 0 && H > 0 && W > 0 && C % 4 == 0 && ph > 0 && pw > 0, "avgpool_backward_rows: bad args");
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(blocks(S * H * W * (C / 4))), dim3(256), 0, (hipStream_t)stream, dxp, S, H,
                     W, C, ph, pw, dx, beta);
  return catseg_launch_status("avgpool_backward_rows");
}

extern "C" int catseg_upsample_ac_backward_rows(const float* dy, int64_t S, int H, int W, int C, int Hp, int Wp,
                                                float* dxp, int beta, void* stream) {
  CATSEG_CHECK(dy && dxp && S > 0 && H > 0 && W > 0 && Hp > 0 && Wp > 0 && C % 4 == 0, "upsample_ac_backward: bad args");
  hipLaunchKernelGGL(upsample_ac_bwd_kernel, dim3(blocks(S * Hp * Wp * (C / 4))), dim3(256), 0, (hipStream_t)stream, dy, S,
                     H, W, C, Hp, Wp, dxp, beta);
  return catseg_launch_status("upsample_ac_backward_rows");
}

extern "C" int catseg_l2normalize_backward(const float* x, int64_t ld_x, CatsegRowMap inmap, const float* dy,
                                           int64_t ld_dy, float* dx, int64_t ld_dx, CatsegRowMap outmap, int beta,
                                           int64_t rows, int64_t cols, float eps, void* stream) {
  CATSEG_CHECK(x && dy && dx && rows > 0 && cols > 0 && cols <= 1024, "l2normalize_backward: bad args (cols <= 1024)");
  CATSEG_CHECK(rowmap_ok(inmap) && rowmap_ok(outmap), "l2normalize_backward: bad row map");
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((rows + 3) / 4);
  const int vpl = (int)((cols + 63) / 64);
#define L2B(V) hipLaunchKernelGGL((l2n_bwd_kernel<V>), dim3(grid), dim3(256), 0, st, x, ld_x, rm(inmap), dy, ld_dy, dx, \
                                  ld_dx, rm(outmap), beta, rows, (int)cols, eps)
  if (vpl <= 2) L2B(2);
  else if (vpl <= 4) L2B(4);
  else if (vpl <= 8) L2B(8);
  else if (vpl <= 12) L2B(12);
  else L2B(16);
#undef L2B
  return catseg_launch_status("l2normalize_backward");
}

extern "C" int catseg_convt_gather(const float* dout, int64_t ld, int64_t S, int hin, int win, int k, int cout, float* g,
                                   void* stream) {
  CATSEG_CHECK(dout && g && S > 0 && hin > 0 && win > 0 && k > 0 && cout > 0, "convt_gather: bad args");
  CATSEG_CHECK(cout % 4 == 0 && ld % 4 == 0 && ld >= cout, "convt_gather: cout and ld must be multiples of 4");
  const int64_t M = S * hin * win;
  hipLaunchKernelGGL(convt_gather_kernel, dim3(blocks(M * (k * k * cout / 4))), dim3(256), 0, (hipStream_t)stream, dout,
                     ld, M, hin, win, k, cout, g);
  return catseg_launch_status("convt_gather");
}

extern "C" int catseg_axpby(const float* x, const float* y, float* out, int64_t n, float alpha, float beta, void* stream) {
  CATSEG_CHECK(x && out && n > 0 && n % 4 == 0, "axpby: bad args (n % 4 == 0)");
  hipLaunchKernelGGL(axpby_kernel, dim3(blocks(n / 4)), dim3(256), 0, (hipStream_t)stream, x, y, out, n / 4, alpha, beta);
  return catseg_launch_status("axpby");
}

extern "C" int catseg_scatter_rows(const float* in, int64_t ld_in, const int32_t* idx, int64_t rows, int64_t cols,
                                   float* out, int64_t ld_out, void* stream) {
  CATSEG_CHECK(in && idx && out && rows > 0 && cols > 0 && ld_in >= cols && ld_out >= cols, "scatter_rows: bad args");
  hipLaunchKernelGGL(scatter_rows_kernel, dim3(blocks(rows * cols)), dim3(256), 0, (hipStream_t)stream, in, ld_in, idx,
                     rows, cols, out, ld_out);
  return catseg_launch_status("scatter_rows");
}

extern "C" int catseg_add_dev_scalar(float* x, int64_t n, const float* s, void* stream) {
  CATSEG_CHECK(x && s && n > 0, "add_dev_scalar: bad args");
  hipLaunchKernelGGL(add_dev_scalar_kernel, dim3(blocks(n)), dim3(256), 0, (hipStream_t)stream, x, n, s);
  return catseg_launch_status("add_dev_scalar");
}
