// Row-wise and data-movement kernels of the CAT-Seg path (HBM-bound; vectorised,
// one wave per row where a row reduction is needed) and the C-ABI error state.
#include <stdarg.h>
#include <string.h>
#include "common.h"
#include "capi.h"

static thread_local char g_err[512] = "";

void catseg_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* catseg_last_error(void) { return g_err; }

int catseg_device_cus() {
  static int cached[64];   // per device ordinal; 0 = not yet queried
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}
extern "C" int catseg_abi_version(void) { return 1; }

namespace {

constexpr int MAXV = 8;   // <= 8 float4 per lane -> cols <= 2048

// ---------------- LayerNorm / L2 normalise (one wave per row) -------------------
template <typename TI, typename TO, bool LN>
__global__ void rownorm_kernel(const TI* __restrict__ in, int64_t ld_in, RowMap inmap, TO* __restrict__ out,
                               int64_t ld_out, const float* gamma, const float* beta, int64_t rows, int cols,
                               float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TI* x = in + rowmap(inmap, row) * ld_in;
  float v[MAXV][4];
  float4 gv[LN ? MAXV : 1], bv[LN ? MAXV : 1];
  // the row and (LayerNorm) gamma / beta are all requested before the first reduction, so the
  // affine parameters do not add a dependent global-load round trip after it
#pragma unroll
  for (int it = 0; it < MAXV; ++it) {
    const int c = (it * 64 + lane) * 4;
    if (c < cols) {
      load4<TI>(x + c, v[it]);
      if constexpr (LN) {
        gv[it] = *reinterpret_cast<const float4*>(gamma + c);
        bv[it] = *reinterpret_cast<const float4*>(beta + c);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < MAXV; ++it)
    if ((it * 64 + lane) * 4 < cols) s += v[it][0] + v[it][1] + v[it][2] + v[it][3];
  if (LN) {
    const float mean = warp_sum(s) / cols;
    float q = 0.f;
#pragma unroll
    for (int it = 0; it < MAXV; ++it) {
      const int c = (it * 64 + lane) * 4;
      if (c < cols)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[it][r] -= mean;
          q += v[it][r] * v[it][r];
        }
    }
    const float rstd = rsqrtf(warp_sum(q) / cols + eps);
#pragma unroll
    for (int it = 0; it < MAXV; ++it) {
      const int c = (it * 64 + lane) * 4;
      if (c < cols) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = v[it][r] * rstd * (&gv[it].x)[r] + (&bv[it].x)[r];
        store4<TO>(out + row * ld_out + c, o);
      }
    }
  } else {
    float q = 0.f;
#pragma unroll
    for (int it = 0; it < MAXV; ++it) {
      const int c = (it * 64 + lane) * 4;
      if (c < cols)
#pragma unroll
        for (int r = 0; r < 4; ++r) q += v[it][r] * v[it][r];
    }
    const float inv = 1.f / fmaxf(sqrtf(warp_sum(q)), eps);
#pragma unroll
    for (int it = 0; it < MAXV; ++it) {
      const int c = (it * 64 + lane) * 4;
      if (c < cols) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = v[it][r] * inv;
        store4<TO>(out + row * ld_out + c, o);
      }
    }
  }
}

// ---------------- LayerNorm, fp32 rows -> bf16, NV float4 per lane (cols = 256 NV) --------
// The ViT's ln_1 / ln_2 / ln_post (1024-wide fp32 residual stream -> bf16 GEMM operand):
// persistent waves walk rows r, r + nw, ... with the next row's loads issued before the
// current row is reduced and stored, so each wave keeps a load and a store stream in flight
// (the one-row-per-wave form loads every row, then stores every row: 8.4 us per 4616 x 1024
// launch against 28 MB / 6 TB/s = 4.7 us).  Same arithmetic as rownorm_kernel, bit for bit.
template <int NV, bool WT = false>
__global__ __launch_bounds__(256) void ln_pipe_kernel(const float* __restrict__ in, int64_t ld_in, RowMap inmap,
                                                      bf16* __restrict__ out, int64_t ld_out, const float* gamma,
                                                      const float* beta, int64_t rows, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  float4 gv[NV], bv[NV], cur[NV], nxt[NV];
#pragma unroll
  for (int it = 0; it < NV; ++it) {
    const int c = (it * 64 + lane) * 4;
    gv[it] = *reinterpret_cast<const float4*>(gamma + c);
    bv[it] = *reinterpret_cast<const float4*>(beta + c);
  }
  auto load = [&](int64_t r, float4 (&v)[NV]) {
    const float* x = in + rowmap(inmap, r) * ld_in;
#pragma unroll
    for (int it = 0; it < NV; ++it) v[it] = *reinterpret_cast<const float4*>(x + (it * 64 + lane) * 4);
  };
  if (row < rows) load(row, cur);
  for (; row < rows; row += nw) {
    if (row + nw < rows) load(row + nw, nxt);
    float s = 0.f;
#pragma unroll
    for (int it = 0; it < NV; ++it) s += cur[it].x + cur[it].y + cur[it].z + cur[it].w;
    const float mean = warp_sum(s) / (NV * 256);
    float q = 0.f;
    float v[NV][4];
#pragma unroll
    for (int it = 0; it < NV; ++it) {
      v[it][0] = cur[it].x - mean; v[it][1] = cur[it].y - mean; v[it][2] = cur[it].z - mean; v[it][3] = cur[it].w - mean;
#pragma unroll
      for (int r = 0; r < 4; ++r) q += v[it][r] * v[it][r];
    }
    const float rstd = rsqrtf(warp_sum(q) / (NV * 256) + eps);
#pragma unroll
    for (int it = 0; it < NV; ++it) {
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = v[it][r] * rstd * (&gv[it].x)[r] + (&bv[it].x)[r];
      if constexpr (WT) {   // sc1 write-through: the rows leave the XCD's L2 as they are written
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000);
        const uint2 u = make_uint2(f2bf2(o[0], o[1]), f2bf2(o[2], o[3]));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i32_t, u), rs, (int)((row * ld_out + (it * 64 + lane) * 4) * 2), 0, 16);
      } else {
        store4<bf16>(out + row * ld_out + (it * 64 + lane) * 4, o);
      }
    }
#pragma unroll
    for (int it = 0; it < NV; ++it) cur[it] = nxt[it];
  }
}

int g_ln_variant = 0;   // 0 = pipelined persistent fp32 -> bf16 LayerNorm where it applies, 1 = one row per wave
CATSEG_KNOB(g_ln_variant, "ln_variant");
int g_ln_store = 1;     // ln_pipe stores: 0 = plain, 1 = sc1 write-through (same box, whole step: 9.445 -> 9.385 ms)
CATSEG_KNOB(g_ln_store, "ln_store");

template <bool LN>
int rownorm(const void* in, int64_t ld_in, CatsegRowMap m, int dti, void* out, int64_t ld_out, int dto,
            const float* gamma, const float* beta, int64_t rows, int64_t cols, float eps, void* stream) {
  CATSEG_CHECK(in && out && rows > 0 && cols > 0, "rownorm: bad args");
  CATSEG_CHECK(cols % 4 == 0 && cols <= 64 * 4 * MAXV, "rownorm: cols must be a multiple of 4 and <= 2048");
  CATSEG_CHECK(ld_in % 4 == 0 && ld_out % 4 == 0, "rownorm: strides must be multiples of 4");
  CATSEG_CHECK(!LN || (gamma && beta), "layernorm: gamma/beta missing");
  CATSEG_CHECK(!LN || ((uintptr_t)gamma % 16 == 0 && (uintptr_t)beta % 16 == 0), "layernorm: gamma/beta must be 16B aligned");
  CATSEG_CHECK(m.d1 > 0 && m.m1 > 0 && m.d2 > 0 && m.m2 > 0, "rownorm: bad row map");
  RowMap rm{m.d1, m.m1, m.s1, m.d2, m.m2, m.s2, m.off};
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (LN && g_ln_variant != 1 && dti == CATSEG_F32 && dto == CATSEG_BF16 && cols == 1024 && rows >= 2048) {
    // 2 waves per SIMD over the 256 CUs: ~2-5 rows per wave at the ViT's 2308-4616 rows
    const int64_t cap = g_ln_variant == 2 ? 256 : g_ln_variant == 3 ? 1024 : 512;
    const unsigned pg = (unsigned)std::min<int64_t>((rows + 3) / 4, cap);
    if (g_ln_store) hipLaunchKernelGGL((ln_pipe_kernel<4, true>), dim3(pg), block, 0, st, (const float*)in, ld_in, rm, (bf16*)out, ld_out,
                                       gamma, beta, rows, eps);
    else hipLaunchKernelGGL((ln_pipe_kernel<4>), dim3(pg), block, 0, st, (const float*)in, ld_in, rm, (bf16*)out, ld_out,
                       gamma, beta, rows, eps);
    return catseg_launch_status("layernorm");
  }
#define RN_LAUNCH(TI, TO)                                                                                   \
  hipLaunchKernelGGL((rownorm_kernel<TI, TO, LN>), grid, block, 0, st, (const TI*)in, ld_in, rm, (TO*)out, \
                     ld_out, gamma, beta, rows, (int)cols, eps)
  if (dti == CATSEG_F32 && dto == CATSEG_F32) RN_LAUNCH(float, float);
  else if (dti == CATSEG_F32 && dto == CATSEG_BF16) RN_LAUNCH(float, bf16);
  else if (dti == CATSEG_BF16 && dto == CATSEG_BF16) RN_LAUNCH(bf16, bf16);
  else RN_LAUNCH(bf16, float);
#undef RN_LAUNCH
  return catseg_launch_status(LN ? "layernorm" : "l2normalize");
}

// ---------------- corr_embed: Conv2d(1, hidden, 7, pad 3) per cost slice ------------
template <typename TO>
__global__ void corr_embed_kernel(const float* corr, int64_t ts, int64_t bs, const int32_t* classes, int Tn, int H,
                                  int W, const float* w, const float* bias, int hidden, TO* out) {
  extern __shared__ float sm[];
  const int PW = W + 6, PH = H + 6;
  float* sin = sm;                     // [PH][PW]
  float* sw = sm + PH * PW;            // [49][hidden]
  const int64_t s = blockIdx.x;
  const int64_t b = s / Tn;
  const int t = (int)(s % Tn);
  const int cls = classes ? classes[s] : t;
  const float* src = corr + (int64_t)cls * ts + b * bs;
  for (int i = threadIdx.x; i < PH * PW; i += blockDim.x) {
    const int y = i / PW - 3, x = i % PW - 3;
    sin[i] = (y >= 0 && y < H && x >= 0 && x < W) ? src[y * W + x] : 0.f;
  }
  for (int i = threadIdx.x; i < 49 * hidden; i += blockDim.x) {
    const int tap = i / hidden, c = i % hidden;
    sw[i] = w[c * 49 + tap];
  }
  __syncthreads();
  const int c = threadIdx.x % hidden;
  const int step = blockDim.x / hidden;
  const float bc = bias[c];
  for (int pix = threadIdx.x / hidden; pix < H * W; pix += step) {
    const int y = pix / W, x = pix % W;
    float acc = bc;
#pragma unroll
    for (int ky = 0; ky < 7; ++ky)
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) acc += sin[(y + ky) * PW + x + kx] * sw[(ky * 7 + kx) * hidden + c];
    out[(s * H * W + pix) * hidden + c] = from_f<TO>(acc);
  }
}

// corr_embed on the MFMA (bf16 output, hidden = 128): the 7x7 conv of a cost slice is the
// GEMM out[pix][c] = sum_k patch[pix][k] . W[c][k] over the 49 taps (K padded to 64).  fp32
// operands enter as bf16 hi + lo pairs (hi.hi + hi.lo + lo.hi: ~16-bit mantissa products,
// fp32 accumulation), so the result matches the fp32 conv to well below the bf16 output
// rounding.  One 4-wave workgroup per slice: the zero-padded slice sits in LDS, every wave
// keeps all 128 x 64 weights as MFMA A fragments in registers and walks 16-pixel tiles:
// D[c][pix] with 4 consecutive channels per lane (8-byte stores).
int g_corr_mfma = 1;   // A/B switch (catseg_set_corr_mfma): 1 = MFMA, weights staged in LDS; 2 = MFMA, weights gathered from global; 0 = VALU

DEV void split_bf16(float v, bf16& hi, bf16& lo) {
  hi = f2bf(v);
  lo = f2bf(v - bf2f(hi));
}

__global__ __launch_bounds__(256) void corr_embed_mfma_kernel(const float* corr, int64_t ts, int64_t bs,
                                                              const int32_t* classes, int64_t S, int Tn, int H,
                                                              int W, const float* w, const float* bias, bf16* out,
                                                              int stage_w) {
  constexpr int HID = 128;
  __shared__ float sin[1024];          // (H + 6) x (W + 6) zero-padded slice (host-checked)
  __shared__ float sbias[HID];
  __shared__ float sw[HID * 49];       // stage_w: the [128][49] weights, one coalesced sweep
  // each wave's 16-pixel x 128-channel bf16 output tile, transposed through LDS so the stores are
  // whole 256-byte pixel rows (16 lanes x 16 B) instead of 8-byte pieces 16 rows apart
  constexpr int OLD = HID + 8;
  __shared__ __attribute__((aligned(16))) bf16 sout[4][16 * OLD];
  const int PW = W + 6, PH = H + 6;
  const int HW = H * W;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  // persistent over slices: the hi/lo weight fragments are built once per workgroup, from LDS
  // (stage_w: 25 KB read coalesced; a fragment's 8 k values of one row are 8 scattered scalar
  // loads otherwise, 128 per thread)
  const float* wsrc = w;
  if (stage_w) {
    for (int i = threadIdx.x; i < HID * 49; i += 256) sw[i] = w[i];
    __syncthreads();
    wsrc = sw;
  }
  s16x8 whi[8][2], wlo[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16 h[8], l[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * ks + 8 * q + j;
        split_bf16(k < 49 ? wsrc[(16 * i + r16) * 49 + k] : 0.f, h[j], l[j]);
      }
      whi[i][ks] = *reinterpret_cast<const s16x8*>(h);
      wlo[i][ks] = *reinterpret_cast<const s16x8*>(l);
    }
  if (threadIdx.x < HID) sbias[threadIdx.x] = bias[threadIdx.x];
  int toff[2][8];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * ks + 8 * q + j;
      toff[ks][j] = k < 49 ? (k / 7) * PW + k % 7 : -1;
    }
  // the slice's HW (<= 576, host-checked) values: up to 3 per thread, prefetched a slice ahead
  float pv[3];
  auto fetch = [&](int64_t s) {
    const int64_t b = s / Tn;
    const int t = (int)(s % Tn);
    const int cls = classes ? classes[s] : t;
    const float* src = corr + (int64_t)cls * ts + b * bs;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int i = threadIdx.x + 256 * k;
      pv[k] = i < HW ? src[i] : 0.f;
    }
  };
  if (blockIdx.x < S) fetch(blockIdx.x);
  for (int i = threadIdx.x; i < PH * PW; i += 256) sin[i] = 0.f;   // the halo stays zero
  for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
    __syncthreads();                   // previous slice's gathers done (and the halo zeroed)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < HW) sin[(i / W + 3) * PW + i % W + 3] = pv[k];
    }
    __syncthreads();
    if (s + gridDim.x < S) fetch(s + gridDim.x);
    const int ntiles = (HW + 15) / 16;
    for (int tile = wave; tile < ntiles; tile += 4) {
      const int pix = tile * 16 + r16;
      const bool valid = pix < HW;
      const int y = valid ? pix / W : 0, x = valid ? pix % W : 0;
      const int base = y * PW + x;
      s16x8 bhi[2], blo[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16 h[8], l[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) split_bf16(toff[ks][j] >= 0 ? sin[base + toff[ks][j]] : 0.f, h[j], l[j]);
        bhi[ks] = *reinterpret_cast<const s16x8*>(h);
        blo[ks] = *reinterpret_cast<const s16x8*>(l);
      }
      f32x4 acc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          acc[i] = mfma_bf16(whi[i][ks], bhi[ks], acc[i]);
          acc[i] = mfma_bf16(whi[i][ks], blo[ks], acc[i]);
          acc[i] = mfma_bf16(wlo[i][ks], bhi[ks], acc[i]);
        }
      }
      bf16* so = sout[wave];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = 16 * i + 4 * q;
        const float4 bb = *reinterpret_cast<const float4*>(sbias + c);
        *reinterpret_cast<uint2*>(so + r16 * OLD + c) = make_uint2(f2bf2(acc[i][0] + bb.x, acc[i][1] + bb.y),
                                                                  f2bf2(acc[i][2] + bb.z, acc[i][3] + bb.w));
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = 4 * k + (lane >> 4), c8 = (lane & 15) * 8;
        const uint4 v = *reinterpret_cast<const uint4*>(so + row * OLD + c8);
        if (tile * 16 + row < HW) st16(out + (s * HW + tile * 16 + row) * HID + c8, v);
      }
    }
  }
}

// ---------------- top-k classes per image --------------------------------------------
// (1) class maxima: one wave per (image, class) row of HW contiguous costs, 4 waves per
//     workgroup, the grid spread over every CU (a single workgroup per image is bound by one
//     CU's load rate: ~80 us for 847 x 576 costs);  the maxima go to the caller's workspace.
// (2) selection, one 1024-thread workgroup per image: class t's rank is the number of classes
//     ordered before it by (max descending, index ascending) -- a broadcast LDS scan, every rank
//     distinct -- and the classes of rank < k are written at their rank: the k largest, sorted.
constexpr int TOPK_NT = 1024;
__global__ __launch_bounds__(256) void class_max_kernel(const float* corr, int64_t ts, int64_t bs, int Tn, int HW,
                                                        float* cmax) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = blockIdx.y;
  if (t >= Tn) return;
  const float* src = corr + (int64_t)t * ts + b * bs;
  float m = -INFINITY;
#pragma unroll 4
  for (int p = lane; p < HW; p += 64) m = fmaxf(m, src[p]);
  m = warp_max(m);
  if (lane == 0) cmax[b * Tn + t] = m;
}

__global__ __launch_bounds__(TOPK_NT) void topk_select_kernel(const float* cmax, int Tn, int k, int32_t* classes) {
  // 16-byte broadcast reads of the maxima (one ds_read_b128 per 4 classes: the scan is LDS-issue
  // bound with 4-byte reads); entries past Tn are -inf and rank after every real class
  __shared__ __attribute__((aligned(16))) float sv[2048];
  const int64_t b = blockIdx.x;
  const int T4 = (Tn + 3) & ~3;
  for (int t = threadIdx.x; t < T4; t += TOPK_NT) sv[t] = t < Tn ? cmax[b * Tn + t] : -INFINITY;
  __syncthreads();
  for (int t = threadIdx.x; t < Tn; t += TOPK_NT) {
    const float v = sv[t];
    int r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    for (int u = 0; u < T4; u += 4) {
      const float4 w = *reinterpret_cast<const float4*>(&sv[u]);
      r0 += (w.x > v) | ((w.x == v) & (u < t));
      r1 += (w.y > v) | ((w.y == v) & (u + 1 < t));
      r2 += (w.z > v) | ((w.z == v) & (u + 2 < t));
      r3 += (w.w > v) | ((w.w == v) & (u + 3 < t));
    }
    const int rank = (r0 + r1) + (r2 + r3);
    if (rank < k) classes[b * k + rank] = t;
  }
}

template <typename E>
__global__ void gather_rows_kernel(const E* in, int64_t ld_in, const int32_t* idx, int64_t rows, int64_t cols, E* out,
                                   int64_t ld_out) {
  const int64_t total = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols, c = i % cols;
    out[r * ld_out + c] = in[(int64_t)idx[r] * ld_in + c];
  }
}

__global__ void fill_kernel(float* out, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = v;
}

// ---------------- preprocess + im2col --------------------------------------------
// torch bilinear, align_corners=False: src = max(scale*(dst+0.5)-0.5, 0), scale = in/out
DEV void lin_idx(int dst, int in_size, float scale, int& i0, int& i1, float& l1) {
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  src = fmaxf(src, 0.f);
  i0 = (int)src;
  i1 = i0 + ((i0 < in_size - 1) ? 1 : 0);
  l1 = src - (float)i0;
}

constexpr int PRE_NT = 256;

template <typename TO, int PATCH>
__global__ __launch_bounds__(PRE_NT) void pre_im2col_kernel(const float* raw, const int32_t* sizes, int64_t B, int Hp, int Wp, const float* mean,
                                  const float* stdv, int res, int patch_rt, TO* out, int64_t ld_out) {
  const int patch = PATCH ? PATCH : patch_rt;   // 14 (L/14) and 16 (B/16) compiled: divisions by constants
  // one workgroup per patch row m = (b, gy, gx): the row's image / patch coordinates are found once
  // and the K columns are walked with 32-bit index math (per-element 64-bit div / mod before: 22 us)
  const int G = res / patch;
  const int P2 = patch * patch;
  const int Kc = 3 * P2;
  const int64_t m = blockIdx.x;
  const int64_t b = m / (G * G);
  const int gp = (int)(m - b * (G * G)), gy = gp / G, gx = gp - gy * G;
  const float sy = (float)Hp / (float)res, sx = (float)Wp / (float)res;
  const int h = sizes[2 * b], w = sizes[2 * b + 1];
  TO* orow = out + m * ld_out;
  for (int kcol = threadIdx.x; kcol < ld_out; kcol += blockDim.x) {
    float v = 0.f;
    if (kcol < Kc) {
      const int c = kcol / P2, kk = kcol - c * P2, ky = kk / patch, kx = kk - ky * patch;
      const int oy = gy * patch + ky, ox = gx * patch + kx;
      int y0, y1, x0, x1;
      float ly, lx;
      lin_idx(oy, Hp, sy, y0, y1, ly);
      lin_idx(ox, Wp, sx, x0, x1, lx);
      const float* img = raw + (b * 3 + c) * (int64_t)Hp * Wp;
      const float mu = mean[c], inv = 1.f / stdv[c];
      auto px = [&](int y, int x) -> float { return (y < h && x < w) ? (img[y * Wp + x] - mu) * inv : 0.f; };
      v = (1.f - ly) * ((1.f - lx) * px(y0, x0) + lx * px(y0, x1)) + ly * ((1.f - lx) * px(y1, x0) + lx * px(y1, x1));
    }
    orow[kcol] = from_f<TO>(v);
  }
}

// ---------------- ViT embed: [cls; patches] + pos -> ln_pre ------------------------
__global__ void vit_embed_kernel(const float* patches, const float* cls, const float* pos, const float* gamma,
                                 const float* beta, int64_t B, int G2, int width, float* x) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int L = G2 + 1;
  if (row >= B * L) return;
  const int64_t b = row / L;
  const int tok = (int)(row % L);
  const float* src = tok == 0 ? cls : patches + (b * G2 + tok - 1) * width;
  const float* pp = pos + (int64_t)tok * width;
  float v[MAXV][4];
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < MAXV; ++it) {
    const int c = (it * 64 + lane) * 4;
    if (c < width) {
      float a[4], q[4];
      load4<float>(src + c, a);
      load4<float>(pp + c, q);
#pragma unroll
      for (int r = 0; r < 4; ++r) { v[it][r] = a[r] + q[r]; s += v[it][r]; }
    }
  }
  const float mean = warp_sum(s) / width;
  float q2 = 0.f;
#pragma unroll
  for (int it = 0; it < MAXV; ++it) {
    const int c = (it * 64 + lane) * 4;
    if (c < width)
#pragma unroll
      for (int r = 0; r < 4; ++r) { v[it][r] -= mean; q2 += v[it][r] * v[it][r]; }
  }
  const float rstd = rsqrtf(warp_sum(q2) / width + 1e-5f);
#pragma unroll
  for (int it = 0; it < MAXV; ++it) {
    const int c = (it * 64 + lane) * 4;
    if (c < width) {
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = v[it][r] * rstd * gamma[c + r] + beta[c + r];
      store4<float>(x + row * width + c, o);
    }
  }
}

// ---------------- bicubic (torch upsample_bicubic2d, A = -0.75, align_corners=False) ----
DEV float cc1(float x, float A) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; }
DEV float cc2(float x, float A) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; }

__global__ void bicubic_kernel(const float* in, int Si, int D, float* out, int So) {
  const int64_t total = (int64_t)So * So * D;
  const float scale = (float)Si / (float)So;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int op = (int)(i / D), oy = op / So, ox = op % So;
    const float ry = scale * (oy + 0.5f) - 0.5f, rx = scale * (ox + 0.5f) - 0.5f;
    const int iy = (int)floorf(ry), ix = (int)floorf(rx);
    const float ty = ry - iy, tx = rx - ix;
    const float A = -0.75f;
    const float wy[4] = {cc2(ty + 1.f, A), cc1(ty, A), cc1(1.f - ty, A), cc2(2.f - ty, A)};
    const float wx[4] = {cc2(tx + 1.f, A), cc1(tx, A), cc1(1.f - tx, A), cc2(2.f - tx, A)};
    float acc = 0.f;
    for (int a = 0; a < 4; ++a) {
      const int yy = min(max(iy - 1 + a, 0), Si - 1);
      float row = 0.f;
      for (int c = 0; c < 4; ++c) {
        const int xx = min(max(ix - 1 + c, 0), Si - 1);
        row += in[((int64_t)yy * Si + xx) * D + d] * wx[c];
      }
      acc += row * wy[a];
    }
    out[i] = acc;
  }
}

// ---------------- postprocess: sigmoid + bilinear resize -----------------------------
template <bool SIG>
__global__ void post_kernel(const float* lg, int64_t planes, int h, int w, int ch, int cw, float* out, int H, int W) {
  const int64_t total = planes * (int64_t)H * W;
  const float sy = (float)ch / (float)H, sx = (float)cw / (float)W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % W);
    const int y = (int)((i / W) % H);
    const int64_t pl = i / ((int64_t)H * W);
    int y0, y1, x0, x1;
    float ly, lx;
    lin_idx(y, ch, sy, y0, y1, ly);
    lin_idx(x, cw, sx, x0, x1, lx);
    const float* src = lg + pl * (int64_t)h * w;
    auto sg = [&](int yy, int xx) -> float {
      const float v = src[yy * w + xx];
      return SIG ? 1.f / (1.f + expf(-v)) : v;
    };
    out[i] = (1.f - ly) * ((1.f - lx) * sg(y0, x0) + lx * sg(y0, x1)) + ly * ((1.f - lx) * sg(y1, x0) + lx * sg(y1, x1));
  }
}

// One workgroup per (plane, band of output rows): the crop region's sigmoids are computed
// ONCE into LDS (each source logit feeds ~(H/ch)^2 outputs), then every thread writes 4
// consecutive outputs of a row (16-byte stores) from 4 LDS taps each.
constexpr int POST_ROWS = 48;    // output rows per workgroup
template <bool SIG>
__global__ __launch_bounds__(256) void post_band_kernel(const float* lg, int h, int w, int ch, int cw, float* out,
                                                        int H, int W) {
  extern __shared__ float sgm[];           // sigmoid of the source rows this band reads [rows][cw]
  const int64_t pl = blockIdx.y;
  const int oy0 = blockIdx.x * POST_ROWS, oy1 = min(H, oy0 + POST_ROWS);
  const float sy = (float)ch / (float)H, sx = (float)cw / (float)W;
  int ya, yb, yt;
  float lt;
  lin_idx(oy0, ch, sy, ya, yt, lt);
  lin_idx(oy1 - 1, ch, sy, yt, yb, lt);
  const int nrows = yb - ya + 1;
  const float* src = lg + pl * (int64_t)h * w;
  for (int i = threadIdx.x; i < nrows * cw; i += 256) {
    const int r = i / cw, c = i - r * cw;
    const float v = src[(int64_t)(ya + r) * w + c];
    sgm[i] = SIG ? 1.f / (1.f + __expf(-v)) : v;
  }
  __syncthreads();
  const int W4 = W / 4;
  float* o = out + pl * (int64_t)H * W;
  for (int idx = threadIdx.x; idx < (oy1 - oy0) * W4; idx += 256) {
    const int ry = idx / W4, x4 = (idx - ry * W4) * 4;
    const int y = oy0 + ry;
    int y0, y1;
    float ly;
    lin_idx(y, ch, sy, y0, y1, ly);
    const float* r0 = sgm + (y0 - ya) * cw;
    const float* r1 = sgm + (y1 - ya) * cw;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int x0, x1;
      float lx;
      lin_idx(x4 + k, cw, sx, x0, x1, lx);
      const float top = fmaf(lx, r0[x1] - r0[x0], r0[x0]);
      const float bot = fmaf(lx, r1[x1] - r1[x0], r1[x0]);
      v[k] = fmaf(ly, bot - top, top);
    }
    *reinterpret_cast<float4*>(o + (int64_t)y * W + x4) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Separable band kernel (default for W % 4 == 0): the band's source rows are sigmoid'ed into LDS,
// then interpolated HORIZONTALLY once per source row into full output-width rows (LDS, float4
// writes), and every output row is one vertical lerp of two of them: 2 conflict-free 16-byte LDS
// reads + 4 fma pairs per 16-byte store (post_band_kernel: 16 scalar reads with bank conflicts per
// store).  The horizontal value is exactly post_band_kernel's `top` / `bot` (same taps, same fma),
// and the vertical step its last fma: bit-identical.
template <bool SIG>
__global__ __launch_bounds__(256) void post_sep_kernel(const float* lg, int h, int w, int ch, int cw, float* out,
                                                        int H, int W) {
  extern __shared__ float smem[];          // [nrows][cw] sigmoid | [nrows][W] horizontal rows
  const int64_t pl = blockIdx.y;
  const int oy0 = blockIdx.x * POST_ROWS, oy1 = min(H, oy0 + POST_ROWS);
  const float sy = (float)ch / (float)H, sx = (float)cw / (float)W;
  int ya, yb, yt;
  float lt;
  lin_idx(oy0, ch, sy, ya, yt, lt);
  lin_idx(oy1 - 1, ch, sy, yt, yb, lt);
  const int nrows = yb - ya + 1;
  float* sgm = smem;
  float* hr = smem + ((nrows * cw + 3) & ~3);
  const float* src = lg + pl * (int64_t)h * w;
  if (cw == w && (w & 3) == 0) {
    // the band's source rows are one contiguous run: 16-byte loads, all of a thread's issued
    // before the first LDS write (one round trip per band instead of one per loop trip)
    const float4* s4 = reinterpret_cast<const float4*>(src + (int64_t)ya * w);
    const int n4 = nrows * cw / 4;
    constexpr int B4 = 4;
    for (int base = 0; base < n4; base += 256 * B4) {
      float4 v[B4];
#pragma unroll
      for (int m = 0; m < B4; ++m) v[m] = s4[min(base + (int)threadIdx.x + 256 * m, n4 - 1)];
#pragma unroll
      for (int m = 0; m < B4; ++m) {
        const int i = base + (int)threadIdx.x + 256 * m;
        if (i < n4) {
          float e[4] = {v[m].x, v[m].y, v[m].z, v[m].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) e[k] = SIG ? 1.f / (1.f + __expf(-e[k])) : e[k];
          *reinterpret_cast<float4*>(sgm + 4 * i) = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
    }
  } else {
    for (int i = threadIdx.x; i < nrows * cw; i += 256) {
      const int r = i / cw, c = i - r * cw;
      const float v = src[(int64_t)(ya + r) * w + c];
      sgm[i] = SIG ? 1.f / (1.f + __expf(-v)) : v;
    }
  }
  __syncthreads();
  const int W4 = W >> 2;
  for (int i = threadIdx.x; i < nrows * W4; i += 256) {
    const int r = i / W4, x4 = (i - r * W4) * 4;
    const float* rs = sgm + r * cw;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int x0, x1;
      float lx;
      lin_idx(x4 + k, cw, sx, x0, x1, lx);
      v[k] = fmaf(lx, rs[x1] - rs[x0], rs[x0]);
    }
    *reinterpret_cast<float4*>(hr + r * W + x4) = make_float4(v[0], v[1], v[2], v[3]);
  }
  __syncthreads();
  float* o = out + pl * (int64_t)H * W;
  for (int idx = threadIdx.x; idx < (oy1 - oy0) * W4; idx += 256) {
    const int ry = idx / W4, x4 = (idx - ry * W4) * 4;
    const int y = oy0 + ry;
    int y0, y1;
    float ly;
    lin_idx(y, ch, sy, y0, y1, ly);
    const float4 t = *reinterpret_cast<const float4*>(hr + (y0 - ya) * W + x4);
    const float4 b = *reinterpret_cast<const float4*>(hr + (y1 - ya) * W + x4);
    *reinterpret_cast<float4*>(o + (int64_t)y * W + x4) =
        make_float4(fmaf(ly, b.x - t.x, t.x), fmaf(ly, b.y - t.y, t.y), fmaf(ly, b.z - t.z, t.z), fmaf(ly, b.w - t.w, t.w));
  }
}

// ---------------- text: token embedding + EOT gather ------------------------------
__global__ void token_embed_kernel(const int32_t* tok, int64_t n, int ctx, const float* emb, const float* pos, int width,
                                   float* x) {
  const int64_t total = n * ctx * (int64_t)width;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % width);
    const int64_t r = i / width;
    const int pi = (int)(r % ctx);
    x[i] = emb[(int64_t)tok[r] * width + c] + pos[(int64_t)pi * width + c];
  }
}

__global__ void eot_kernel(const float* x, const int32_t* tok, int64_t n, int ctx, int width, float* out) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  __shared__ int arg;
  if (threadIdx.x == 0) {
    int best = 0, bv = tok[r * ctx];
    for (int i = 1; i < ctx; ++i)
      if (tok[r * ctx + i] > bv) { bv = tok[r * ctx + i]; best = i; }
    arg = best;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < width; c += blockDim.x) out[r * width + c] = x[(r * ctx + arg) * width + c];
}

inline unsigned grid_for(int64_t n, int64_t cap = 16384) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  return (unsigned)(g < cap ? g : cap);
}

}  // namespace

extern "C" int catseg_layernorm(const void* in, int64_t ld_in, CatsegRowMap inmap, int dtype_in, void* out,
                                int64_t ld_out, int dtype_out, const float* gamma, const float* beta, int64_t rows,
                                int64_t cols, float eps, void* stream) {
  return rownorm<true>(in, ld_in, inmap, dtype_in, out, ld_out, dtype_out, gamma, beta, rows, cols, eps, stream);
}

extern "C" int catseg_l2normalize(const void* in, int64_t ld_in, CatsegRowMap inmap, int dtype_in, void* out,
                                  int64_t ld_out, int dtype_out, int64_t rows, int64_t cols, float eps, void* stream) {
  return rownorm<false>(in, ld_in, inmap, dtype_in, out, ld_out, dtype_out, nullptr, nullptr, rows, cols, eps, stream);
}

CATSEG_KNOB(g_corr_mfma, "corr_mfma");

extern "C" int catseg_corr_embed(const float* corr, int64_t corr_t_stride, int64_t corr_b_stride,
                                 const int32_t* classes, int64_t B, int T, int H, int W, const float* weight,
                                 const float* bias, int hidden, void* out, int dtype, void* stream) {
  CATSEG_CHECK(corr && weight && bias && out && B > 0 && T > 0 && H > 0 && W > 0, "corr_embed: bad args");
  CATSEG_CHECK(hidden > 0 && 256 % hidden == 0, "corr_embed: hidden must divide 256");
  const size_t sh = ((H + 6) * (W + 6) + 49 * hidden) * sizeof(float);
  CATSEG_CHECK(sh <= 64 * 1024, "corr_embed: slice too large for LDS");
  const unsigned grid = (unsigned)(B * T);
  if (dtype == CATSEG_BF16 && hidden == 128 && (H + 6) * (W + 6) <= 1024 && H * W <= 768 && g_corr_mfma) {
    const int cus = catseg_device_cus();
    const unsigned pgrid = (unsigned)std::min<int64_t>(B * T, (int64_t)cus * 2);
    hipLaunchKernelGGL(corr_embed_mfma_kernel, dim3(pgrid), dim3(256), 0, (hipStream_t)stream, corr, corr_t_stride,
                       corr_b_stride, classes, B * (int64_t)T, T, H, W, weight, bias, (bf16*)out, g_corr_mfma != 2 ? 1 : 0);
  }
  else if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL(corr_embed_kernel<bf16>, dim3(grid), dim3(256), sh, (hipStream_t)stream, corr, corr_t_stride,
                       corr_b_stride, classes, T, H, W, weight, bias, hidden, (bf16*)out);
  else
    hipLaunchKernelGGL(corr_embed_kernel<float>, dim3(grid), dim3(256), sh, (hipStream_t)stream, corr, corr_t_stride,
                       corr_b_stride, classes, T, H, W, weight, bias, hidden, (float*)out);
  return catseg_launch_status("corr_embed");
}

extern "C" int catseg_topk_classes(const float* corr, int64_t corr_t_stride, int64_t corr_b_stride, int64_t B, int T,
                                   int HW, int k, int32_t* classes, float* workspace, void* stream) {
  CATSEG_CHECK(corr && classes && workspace && B > 0 && T > 0 && HW > 0, "topk: bad args");
  CATSEG_CHECK(T <= 2048 && k > 0 && k <= T, "topk: need 0 < k <= T <= 2048");
  CATSEG_CHECK(B <= 65535, "topk: at most 65535 images per call");
  hipLaunchKernelGGL(class_max_kernel, dim3((unsigned)((T + 3) / 4), (unsigned)B), dim3(256), 0, (hipStream_t)stream,
                     corr, corr_t_stride, corr_b_stride, T, HW, workspace);
  hipLaunchKernelGGL(topk_select_kernel, dim3((unsigned)B), dim3(TOPK_NT), 0, (hipStream_t)stream, workspace, T, k,
                     classes);
  return catseg_launch_status("topk");
}

extern "C" int catseg_gather_rows(const void* in, int64_t ld_in, const int32_t* idx, int64_t rows, int64_t cols,
                                  void* out, int64_t ld_out, int dtype, void* stream) {
  CATSEG_CHECK(in && idx && out && rows > 0 && cols > 0, "gather_rows: bad args");
  if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL(gather_rows_kernel<bf16>, dim3(grid_for(rows * cols)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)in, ld_in, idx, rows, cols, (bf16*)out, ld_out);
  else
    hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(grid_for(rows * cols)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)in, ld_in, idx, rows, cols, (float*)out, ld_out);
  return catseg_launch_status("gather_rows");
}

// out[b][c][r] = in[b * in_bstride + r][c] (r < rows), 0 for rows <= r < ld_out
template <typename E>
__global__ void transpose_rows_kernel(const E* in, int64_t ld_in, int64_t rows, int64_t cols, int64_t in_bstride,
                                      E* out, int64_t ld_out, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i % ld_out, bc = i / ld_out, c = bc % cols, b = bc / cols;
    out[i] = r < rows ? in[(b * in_bstride + r) * ld_in + c] : (E)0;
  }
}

extern "C" int catseg_transpose_rows(const void* in, int64_t ld_in, int64_t rows, int64_t cols, int64_t batch,
                                     int64_t in_bstride, void* out, int64_t ld_out, int dtype, void* stream) {
  CATSEG_CHECK(in && out && rows > 0 && cols > 0 && batch > 0 && ld_out >= rows && ld_in >= cols,
               "transpose_rows: bad args");
  const int64_t total = batch * cols * ld_out;
  if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL(transpose_rows_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)in, ld_in, rows, cols, in_bstride, (bf16*)out, ld_out, total);
  else
    hipLaunchKernelGGL(transpose_rows_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)in, ld_in, rows, cols, in_bstride, (float*)out, ld_out, total);
  return catseg_launch_status("transpose_rows");
}

extern "C" int catseg_fill_f32(float* out, int64_t n, float value, void* stream) {
  CATSEG_CHECK(out && n > 0, "fill: bad args");
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, out, n, value);
  return catseg_launch_status("fill");
}

extern "C" int catseg_preprocess_im2col(const float* raw, const int32_t* sizes, int64_t B, int Hp, int Wp,
                                        const float* mean, const float* stdv, int res, int patch, void* out,
                                        int64_t ld_out, int dtype, void* stream) {
  CATSEG_CHECK(raw && sizes && mean && stdv && out && B > 0 && Hp > 0 && Wp > 0, "preprocess: bad args");
  CATSEG_CHECK(patch > 0 && res % patch == 0 && ld_out >= 3 * patch * patch, "preprocess: bad geometry");
  CATSEG_CHECK((int64_t)Hp * Wp < (1ll << 31), "preprocess: canvas too large");
  const int G = res / patch;
  const dim3 grid((unsigned)(B * G * G));
  auto go = [&](auto kern, auto* o) {
    hipLaunchKernelGGL(kern, grid, dim3(PRE_NT), 0, (hipStream_t)stream, raw, sizes, B, Hp, Wp, mean, stdv, res, patch, o,
                       ld_out);
  };
  if (dtype == CATSEG_BF16) {
    if (patch == 14) go(pre_im2col_kernel<bf16, 14>, (bf16*)out);
    else if (patch == 16) go(pre_im2col_kernel<bf16, 16>, (bf16*)out);
    else go(pre_im2col_kernel<bf16, 0>, (bf16*)out);
  } else {
    if (patch == 14) go(pre_im2col_kernel<float, 14>, (float*)out);
    else if (patch == 16) go(pre_im2col_kernel<float, 16>, (float*)out);
    else go(pre_im2col_kernel<float, 0>, (float*)out);
  }
  return catseg_launch_status("preprocess_im2col");
}

extern "C" int catseg_vit_embed(const float* patches, const float* cls, const float* pos, const float* gamma,
                                const float* beta, int64_t B, int G2, int width, float* x, void* stream) {
  CATSEG_CHECK(patches && cls && pos && gamma && beta && x && B > 0 && G2 > 0, "vit_embed: bad args");
  CATSEG_CHECK(width % 4 == 0 && width <= 64 * 4 * MAXV, "vit_embed: bad width");
  const int64_t rows = B * (G2 + 1);
  hipLaunchKernelGGL(vit_embed_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, patches,
                     cls, pos, gamma, beta, B, G2, width, x);
  return catseg_launch_status("vit_embed");
}

extern "C" int catseg_bicubic_resize(const float* in, int S_in, int D, float* out, int S_out, void* stream) {
  CATSEG_CHECK(in && out && S_in > 0 && S_out > 0 && D > 0, "bicubic: bad args");
  const int64_t total = (int64_t)S_out * S_out * D;
  hipLaunchKernelGGL(bicubic_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, in, S_in, D, out, S_out);
  return catseg_launch_status("bicubic");
}

namespace {
int g_post_variant = 0;   // 0 = separable band kernel, 1 = the direct band kernel (A/B; bit-identical)
template <bool SIG>
int launch_post(const char* what, const float* logits, int64_t B, int T, int h, int w, int crop_h, int crop_w,
                float* out, int H, int W, void* stream) {
  CATSEG_CHECK(logits && out && B > 0 && T > 0 && H > 0 && W > 0, "postprocess/resize: bad args");
  CATSEG_CHECK(crop_h > 0 && crop_h <= h && crop_w > 0 && crop_w <= w, "postprocess/resize: bad crop");
  const int64_t total = B * T * (int64_t)H * W;
  // banded kernels: source rows of one band (<= POST_ROWS * ch / H + 2) fit LDS
  const int64_t band_src_rows = (int64_t)POST_ROWS * crop_h / H + 3;
  const dim3 grid((unsigned)((H + POST_ROWS - 1) / POST_ROWS), (unsigned)(B * T));
  const int64_t sep_bytes = (((band_src_rows * crop_w + 3) & ~3LL) + band_src_rows * W) * 4;
  if (W % 4 == 0 && g_post_variant == 0 && sep_bytes <= 64 * 1024) {
    hipLaunchKernelGGL(post_sep_kernel<SIG>, grid, dim3(256), (size_t)sep_bytes, (hipStream_t)stream, logits, h, w,
                       crop_h, crop_w, out, H, W);
    return catseg_launch_status(what);
  }
  if (W % 4 == 0 && band_src_rows * crop_w * 4 <= 64 * 1024) {
    hipLaunchKernelGGL(post_band_kernel<SIG>, grid, dim3(256), (size_t)(band_src_rows * crop_w * 4), (hipStream_t)stream,
                       logits, h, w, crop_h, crop_w, out, H, W);
    return catseg_launch_status(what);
  }
  hipLaunchKernelGGL(post_kernel<SIG>, dim3(grid_for(total, 65536)), dim3(256), 0, (hipStream_t)stream, logits,
                     B * T, h, w, crop_h, crop_w, out, H, W);
  return catseg_launch_status(what);
}
}  // namespace

CATSEG_KNOB(g_post_variant, "post_variant");

extern "C" int catseg_postprocess(const float* logits, int64_t B, int T, int h, int w, int crop_h, int crop_w,
                                  float* out, int H, int W, void* stream) {
  return launch_post<true>("postprocess", logits, B, T, h, w, crop_h, crop_w, out, H, W, stream);
}

extern "C" int catseg_resize_bilinear(const float* in, int64_t B, int T, int h, int w, int crop_h, int crop_w,
                                      float* out, int H, int W, void* stream) {
  return launch_post<false>("resize_bilinear", in, B, T, h, w, crop_h, crop_w, out, H, W, stream);
}

extern "C" int catseg_token_embed(const int32_t* tokens, int64_t n, int ctx, const float* tok_emb, const float* pos,
                                  int width, float* x, void* stream) {
  CATSEG_CHECK(tokens && tok_emb && pos && x && n > 0 && ctx > 0 && width > 0, "token_embed: bad args");
  hipLaunchKernelGGL(token_embed_kernel, dim3(grid_for(n * ctx * width)), dim3(256), 0, (hipStream_t)stream, tokens,
                     n, ctx, tok_emb, pos, width, x);
  return catseg_launch_status("token_embed");
}

extern "C" int catseg_eot_gather(const float* x, const int32_t* tokens, int64_t n, int ctx, int width, float* out,
                                 void* stream) {
  CATSEG_CHECK(x && tokens && out && n > 0, "eot_gather: bad args");
  hipLaunchKernelGGL(eot_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, x, tokens, n, ctx, width, out);
  return catseg_launch_status("eot_gather");
}

// ---------------- dtype conversion with a row map (hook / feature casts) ------------
namespace {
template <typename TI, typename TO>
__global__ void convert_kernel(const TI* in, int64_t ld_in, RowMap m, TO* out, int64_t ld_out, int64_t rows,
                               int64_t cols4) {
  const int64_t total = rows * cols4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols4, c = (i % cols4) * 4;
    float v[4];
    load4<TI>(in + rowmap(m, r) * ld_in + c, v);
    store4<TO>(out + r * ld_out + c, v);
  }
}
}  // namespace

extern "C" int catseg_convert(const void* in, int64_t ld_in, CatsegRowMap inmap, int dtype_in, void* out,
                              int64_t ld_out, int dtype_out, int64_t rows, int64_t cols, void* stream) {
  CATSEG_CHECK(in && out && rows > 0 && cols > 0 && cols % 4 == 0 && ld_in % 4 == 0 && ld_out % 4 == 0,
               "convert: bad args");
  CATSEG_CHECK(inmap.d1 > 0 && inmap.m1 > 0 && inmap.d2 > 0 && inmap.m2 > 0, "convert: bad row map");
  RowMap rm{inmap.d1, inmap.m1, inmap.s1, inmap.d2, inmap.m2, inmap.s2, inmap.off};
  const unsigned grid = grid_for(rows * cols / 4);
  hipStream_t st = (hipStream_t)stream;
  if (dtype_in == CATSEG_F32 && dtype_out == CATSEG_BF16)
    hipLaunchKernelGGL((convert_kernel<float, bf16>), dim3(grid), dim3(256), 0, st, (const float*)in, ld_in, rm,
                       (bf16*)out, ld_out, rows, cols / 4);
  else if (dtype_in == CATSEG_F32 && dtype_out == CATSEG_F32)
    hipLaunchKernelGGL((convert_kernel<float, float>), dim3(grid), dim3(256), 0, st, (const float*)in, ld_in, rm,
                       (float*)out, ld_out, rows, cols / 4);
  else if (dtype_in == CATSEG_BF16 && dtype_out == CATSEG_F32)
    hipLaunchKernelGGL((convert_kernel<bf16, float>), dim3(grid), dim3(256), 0, st, (const bf16*)in, ld_in, rm,
                       (float*)out, ld_out, rows, cols / 4);
  else
    hipLaunchKernelGGL((convert_kernel<bf16, bf16>), dim3(grid), dim3(256), 0, st, (const bf16*)in, ld_in, rm,
                       (bf16*)out, ld_out, rows, cols / 4);
  return catseg_launch_status("convert");
}
