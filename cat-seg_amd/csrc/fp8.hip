// e4m3 producers of the config-5 fp8 ViT GEMMs (catseg_gemm_fp8, gemm.hip).
//
// One wave per row, the whole row held in registers (<= 8 chunks of 8 values per lane,
// cols <= 4096): one HBM read and one byte-wide write per element.
//   quant:      scale = max|x| / 448,           q = rne_e4m3(x * (448 / max|x|))
//   layernorm:  y = (x - mean) * rstd * g + b (as catseg_layernorm, fp32), then quant(y)
// The LayerNorm form replaces catseg_layernorm + a bf16 round trip ahead of the QKV and
// c_fc GEMMs (model_vpt.py:208-217 ln_1 / ln_2), so the GEMM operand is quantized from
// the fp32 normalized row, not from its bf16 rounding.
#include "common.h"
#include "capi.h"

namespace {

constexpr int MAXC = 8;   // 8-value chunks per lane -> cols <= 64 * 8 * 8 = 4096

DEV void load8(const float* p, float v[8]) { load4<float>(p, v); load4<float>(p + 4, v + 4); }
DEV void load8(const bf16* p, float v[8]) {
  const uint4 u = ld16(p);
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
}

template <typename TI, bool LN>
__global__ __launch_bounds__(256) void fp8_rows_kernel(const TI* __restrict__ in, int64_t ld_in, RowMap inmap,
                                                       uint8_t* __restrict__ q, int64_t ld_q, float* __restrict__ scale,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       int64_t rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TI* x = in + rowmap(inmap, row) * ld_in;
  float v[MAXC][8];
#pragma unroll
  for (int it = 0; it < MAXC; ++it) {
    const int c = (it * 64 + lane) * 8;
    if (c < cols) load8(x + c, v[it]);
  }
  if (LN) {
    float s = 0.f;
#pragma unroll
    for (int it = 0; it < MAXC; ++it)
      if ((it * 64 + lane) * 8 < cols)
#pragma unroll
        for (int r = 0; r < 8; ++r) s += v[it][r];
    const float mean = warp_sum(s) / cols;
    float ss = 0.f;
#pragma unroll
    for (int it = 0; it < MAXC; ++it)
      if ((it * 64 + lane) * 8 < cols)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          v[it][r] -= mean;
          ss += v[it][r] * v[it][r];
        }
    const float rstd = rsqrtf(warp_sum(ss) / cols + eps);
#pragma unroll
    for (int it = 0; it < MAXC; ++it) {
      const int c = (it * 64 + lane) * 8;
      if (c < cols) {
        float g[8], b[8];
        load8(gamma + c, g);
        load8(beta + c, b);
#pragma unroll
        for (int r = 0; r < 8; ++r) v[it][r] = v[it][r] * rstd * g[r] + b[r];
      }
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int it = 0; it < MAXC; ++it)
    if ((it * 64 + lane) * 8 < cols)
#pragma unroll
      for (int r = 0; r < 8; ++r) amax = fmaxf(amax, fabsf(v[it][r]));
  amax = fmaxf(warp_max(amax), 1e-30f);
  const float inv = 448.f / amax;
  if (lane == 0) scale[row] = amax / 448.f;
  uint8_t* qr = q + row * ld_q;
#pragma unroll
  for (int it = 0; it < MAXC; ++it) {
    const int c = (it * 64 + lane) * 8;
    if (c < cols) {
      float t[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) t[r] = fminf(fmaxf(v[it][r] * inv, -448.f), 448.f);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(t[0], t[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(t[2], t[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(t[4], t[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(t[6], t[7], hi, true);
      *reinterpret_cast<uint2*>(qr + c) = make_uint2((unsigned)lo, (unsigned)hi);
    }
  }
}

template <bool LN>
int fp8_rows(const void* x, int dtype, int64_t ld_x, CatsegRowMap m, int64_t rows, int64_t cols, void* q,
             int64_t ld_q, float* scale, const float* gamma, const float* beta, float eps, void* stream) {
  const char* what = LN ? "layernorm_fp8" : "quant_fp8_rows";
  CATSEG_CHECK(x && q && scale, what);
  CATSEG_CHECK(rows > 0 && cols > 0 && cols <= 64 * 8 * MAXC, "fp8 rows: need 0 < cols <= 4096");
  CATSEG_CHECK(cols % 8 == 0 && ld_x % 8 == 0 && ld_q % 8 == 0, "fp8 rows: cols / ld must be multiples of 8");
  CATSEG_CHECK(dtype == CATSEG_BF16 || dtype == CATSEG_F32, "fp8 rows: dtype must be f32 or bf16");
  CATSEG_CHECK(!LN || (gamma && beta && ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0),
               "layernorm_fp8: gamma/beta missing or misaligned");
  CATSEG_CHECK(((uintptr_t)x % 16) == 0 && ((uintptr_t)q % 8) == 0, "fp8 rows: misaligned pointer");
  CATSEG_CHECK(m.d1 > 0 && m.m1 > 0 && m.d2 > 0 && m.m2 > 0, "fp8 rows: bad row map");
  RowMap rm{m.d1, m.m1, m.s1, m.d2, m.m2, m.s2, m.off};
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((rows + 3) / 4);
  if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL((fp8_rows_kernel<bf16, LN>), dim3(grid), dim3(256), 0, st, (const bf16*)x, ld_x, rm,
                       (uint8_t*)q, ld_q, scale, gamma, beta, rows, (int)cols, eps);
  else
    hipLaunchKernelGGL((fp8_rows_kernel<float, LN>), dim3(grid), dim3(256), 0, st, (const float*)x, ld_x, rm,
                       (uint8_t*)q, ld_q, scale, gamma, beta, rows, (int)cols, eps);
  return catseg_launch_status(what);
}

}  // namespace

extern "C" int catseg_quant_fp8_rows(const void* x, int dtype, int64_t ld_x, int64_t rows, int64_t cols, void* q,
                                     int64_t ld_q, float* scale, void* stream) {
  const CatsegRowMap ident{1, (int64_t)1 << 62, 1, 1, 1, 0, 0};
  return fp8_rows<false>(x, dtype, ld_x, ident, rows, cols, q, ld_q, scale, nullptr, nullptr, 0.f, stream);
}

extern "C" int catseg_layernorm_fp8(const void* x, int64_t ld_x, CatsegRowMap inmap, int dtype, void* q, int64_t ld_q,
                                    float* scale, const float* gamma, const float* beta, int64_t rows, int64_t cols,
                                    float eps, void* stream) {
  return fp8_rows<true>(x, dtype, ld_x, inmap, rows, cols, q, ld_q, scale, gamma, beta, eps, stream);
}
