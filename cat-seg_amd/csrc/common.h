// Common device helpers for the CAT-Seg gfx950 kernels.
//
// Element types: activations are either fp32 or bf16 (raw ushort storage,
// round-to-nearest-even conversion).  MFMA: bf16 uses
// v_mfma_f32_16x16x32_bf16, fp32 uses the exact-f32 v_mfma_f32_16x16x4_f32
// (gfx950 has no xf32).  Both share the 16x16 C/D layout
// (col = lane & 15, row = 4 * (lane >> 4) + reg), see
// /opt/skills/guides/cdna_hip_programming.md §3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <type_traits>

typedef unsigned short bf16;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef int v2i32_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));

#define DEV __device__ __forceinline__

DEV float bf2f(bf16 v) { return __uint_as_float(((unsigned)v) << 16); }
// fp32 -> bf16, round-to-nearest-even: the native __bf16 conversion lowers to gfx950's
// v_cvt_pk_bf16_f32 (one instruction per PAIR), vs ~6 VALU for the bit-trick form.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
DEV bf16 f2bf(float f) { return __builtin_bit_cast(bf16, (__bf16)f); }
DEV unsigned f2bf2(float lo, float hi) {
  const bf16x2_t h = __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t);
  return __builtin_bit_cast(unsigned, h);
}

// ReLU of a packed bf16 pair: a signed 16-bit max with 0 (v_pk_max_i16) maps every negative value
// and -0 to +0 and keeps the rest, the same bits as rounding the ReLU'd floats
typedef short s16x2_t __attribute__((ext_vector_type(2)));
DEV unsigned relu_bf16x2(unsigned v) {
  const s16x2_t r = __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, v), (s16x2_t){0, 0});
  return __builtin_bit_cast(unsigned, r);
}

template <typename T> DEV float to_f(T v);
template <> DEV float to_f<float>(float v) { return v; }
template <> DEV float to_f<bf16>(bf16 v) { return bf2f(v); }
template <typename T> DEV T from_f(float v);
template <> DEV float from_f<float>(float v) { return v; }
template <> DEV bf16 from_f<bf16>(float v) { return f2bf(v); }

// 16-byte vector of T: 4 floats or 8 bf16
template <typename T> struct Vec16;
template <> struct Vec16<float> { static constexpr int N = 4; };
template <> struct Vec16<bf16> { static constexpr int N = 8; };

DEV uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
DEV void st16(void* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }
// sc1 write-through stores at a byte offset (< 2^31) from a wave-uniform base: the line leaves the
// XCD's L2 as it is written, so the kernel-end writeback has no dirty lines of it left to flush
DEV void st16_wt(void* base, int64_t byte_off, uint4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, v), r, (int)byte_off, 0, 16);
}
DEV void st8_wt(void* base, int64_t byte_off, uint2 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i32_t, v), r, (int)byte_off, 0, 16);
}

// load 4 consecutive elements as floats
template <typename T> DEV void load4(const T* p, float out[4]);
template <> DEV void load4<float>(const float* p, float out[4]) {
  float4 v = *reinterpret_cast<const float4*>(p);
  out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
}
template <> DEV void load4<bf16>(const bf16* p, float out[4]) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  out[0] = __uint_as_float(v.x << 16); out[1] = __uint_as_float(v.x & 0xffff0000u);
  out[2] = __uint_as_float(v.y << 16); out[3] = __uint_as_float(v.y & 0xffff0000u);
}
template <typename T> DEV void store4(T* p, const float v[4]);
template <> DEV void store4<float>(float* p, const float v[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> DEV void store4<bf16>(bf16* p, const float v[4]) {
  uint2 o;
  o.x = f2bf2(v[0], v[1]);
  o.y = f2bf2(v[2], v[3]);
  *reinterpret_cast<uint2*>(p) = o;
}

// LDS-DMA (global_load_lds, 16 B per lane, lane-linear LDS destination) and counted vmcnt waits
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
// Workgroups are dealt round-robin over the 8 XCDs (observed, speed only): remap the linear
// block id so each XCD owns a contiguous range (neighbouring tiles share one L2).
DEV int xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

DEV void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}
template <int N>
DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // gfx9 s_waitcnt encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

DEV f32x4 mfma_bf16(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
DEV f32x4 mfma_f32(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Reductions on the DPP crossbar (no LDS-pipe ds_bpermute round trips, which cost ~100+
// cycles each in the LayerNorm prologues of the row kernels).  Every step adds a value to
// its partner's, so all lanes of a group end with bit-identical sums; fixed order:
// deterministic.
template <int CTRL, int ROWMASK = 0xF>
DEV float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWMASK, 0xF, false));
}
// sum over the 16 lanes of each DPP row (lanes 16r .. 16r+15), result in all 16
DEV float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);          // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);          // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);         // row_half_mirror
  v += dpp_mov<0x140>(v);         // row_mirror
  return v;
}
// full-wave sum: row sums, then row broadcasts into lane 63, read back uniformly
DEV float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);          // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);          // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);         // row_half_mirror
  v += dpp_mov<0x140>(v);         // row_mirror: every lane holds its row's sum
  v += dpp_mov<0x142, 0xA>(v);    // row_bcast:15 into rows 1, 3
  v += dpp_mov<0x143, 0xC>(v);    // row_bcast:31 into rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
DEV float warp_sum(float v) { return wave_sum(v); }
// sum / max over the 4 lanes l, l^16, l^32, l^48 (the same MFMA column in each 16-lane row):
// gfx950 v_permlane16_swap / v_permlane32_swap exchange whole rows / halves in registers
DEV float xrow4_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
DEV float xrow4_max(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
DEV float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Activations (epilogues).  GELU is the exact erf form (nn.GELU default, timm Mlp);
// QuickGELU is CLIP's x*sigmoid(1.702x) (model_vpt.py:165-167).
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_QUICKGELU = 3, ACT_SIGMOID = 4 };

// erf via Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7): one exp + one rcp + 5 FMAs,
// branch-free (ocml erff is a multi-branch polynomial that dominated the Swin MLP).
DEV float fast_erf(float x) {
  const float a = fabsf(x);
  const float t = __frcp_rn(fmaf(0.3275911f, a, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.f - p * t * __expf(-a * a);
  return copysignf(y, x);
}

// GELU(x) = 0.5 x (1 + erf(x / sqrt 2)), erf(x / sqrt 2) ~= xc P(xc^2), xc = clamp(x, +-3 sqrt 2):
// P is a degree-8 minimax fit of the GELU error (x/2)|dt| (linear program on a 3000-point grid),
// max 3.0e-5 inside the clamp evaluated in fp32; no transcendental (v_exp / v_rcp cost 8 issue
// cycles).  Written on scalars: whether the fp32 chain is packed (v_pk_fma_f32) is left to the
// compiler's SLP pass, which measured neutral for the MLP and positive for most kernels.
typedef float f32x2 __attribute__((ext_vector_type(2)));
DEV float erf_t1(float x) {
  constexpr float XC = 4.242640495f;
  const float xc = __builtin_amdgcn_fmed3f(x, -XC, XC);
  const float s = xc * xc;
  float p = 9.1976350e-11f;
  p = __builtin_fmaf(p, s, -9.1081507e-09f);
  p = __builtin_fmaf(p, s, 3.9963419e-07f);
  p = __builtin_fmaf(p, s, -1.0334782e-05f);
  p = __builtin_fmaf(p, s, 1.7735695e-04f);
  p = __builtin_fmaf(p, s, -2.1602388e-03f);
  p = __builtin_fmaf(p, s, 1.9443829e-02f);
  p = __builtin_fmaf(p, s, -1.3238958e-01f);
  p = __builtin_fmaf(p, s, 7.9764283e-01f);
  return xc * p;
}
DEV f32x2 erf_t2(f32x2 x) { return f32x2{erf_t1(x.x), erf_t1(x.y)}; }
// GELU for the bf16 paths: beyond the clamp t = xc P(xc^2) ~= erf(3) = 1 - 2.2e-5 instead of +-1,
// a relative error < 1e-4 (bf16 keeps 3.9e-3): no saturation select (12 VALU per value)
DEV float gelu1(float x) {   // x (0.5 + 0.5 erf): 12 VALU
  return x * __builtin_fmaf(0.5f, erf_t1(x), 0.5f);
}
DEV f32x2 gelu2(f32x2 x) { return f32x2{gelu1(x.x), gelu1(x.y)}; }
// exact-saturation GELU (fp32 paths)
DEV float gelu_erf(float v) {
  float t = erf_t1(v);
  t = fabsf(v) < 4.242640495f ? t : copysignf(1.f, v);
  const float h = 0.5f * v;
  return h + h * t;
}

// QuickGELU x * sigmoid(1.702 x) as x * rcp(1 + 2^(-1.702 log2(e) x)): v_exp_f32 + v_rcp_f32
// (~1 ulp each) instead of the IEEE division sequence (div_scale x2 / div_fmas / div_fixup + rcp
// + 4 fma per value), which dominated the fc1 epilogue.  x -> -inf: 2^(+inf) = inf, rcp = 0,
// result -0; x -> +inf: rcp(1) = 1, result x.
DEV float quick_gelu(float v) {
  return v * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.4554670f * v));   // 1.702 * log2(e)
}

template <int ACT> DEV float act_t(float v) {
  if constexpr (ACT == ACT_RELU) return fmaxf(v, 0.f);
  else if constexpr (ACT == ACT_GELU) return gelu_erf(v);
  else if constexpr (ACT == ACT_QUICKGELU) return quick_gelu(v);
  else if constexpr (ACT == ACT_SIGMOID) return 1.f / (1.f + __expf(-v));
  else return v;
}

DEV float apply_act(float v, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_GELU: return gelu_erf(v);
    case ACT_QUICKGELU: return quick_gelu(v);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    default: return v;
  }
}

// Row map: r(m) = ((m / d1) % m1) * s1 + ((m / d2) % m2) * s2 + off.
// Identity = {1, INT64 big, 1, 1, 1, 0, 0}.  Used to gather A rows (hook tokens
// without CLS) and to broadcast per-image / per-class guidance terms.
// ConvTranspose2d(k, stride k) scatter of GEMM output (m, n): m = (s, y, x) over
// (hin, win), n = (ky, kx, co); NHWC destination [s][y*k+ky][x*k+kx][co].  32-bit index
// math (m < 2^31 and n < 2^31, host-checked): the 64-bit div/mod form cost the decoder's
// ConvTranspose epilogue more than its MFMAs.
DEV int64_t convt_offset(int64_t m, int64_t n, int k, int hin, int win, int cout) {
  const unsigned mu = (unsigned)m, nu = (unsigned)n, hw = (unsigned)(hin * win), kc = (unsigned)(k * cout);
  const unsigned s = mu / hw, rem = mu - s * hw, y = rem / (unsigned)win, x = rem - y * (unsigned)win;
  const unsigned ky = nu / kc, r2 = nu - ky * kc, kx = r2 / (unsigned)cout, co = r2 - kx * (unsigned)cout;
  return (((int64_t)s * hin * k + (int64_t)y * k + ky) * ((int64_t)win * k) + (int64_t)x * k + kx) * cout + co;
}

struct RowMap {
  int64_t d1, m1, s1, d2, m2, s2, off;
};
// 32-bit unsigned quotient with the common divisor-1 case skipped (uniform branches)
DEV uint32_t udiv32(uint32_t a, uint32_t d) { return d == 1 ? a : a / d; }
DEV uint32_t umod32(uint32_t a, uint32_t d) { return d == 1 ? 0u : a % d; }
DEV int64_t rowmap(const RowMap& r, int64_t m) {
  constexpr int64_t LIM = 0x7fffffffLL;
  // Every row count on the path is < 2^31: 32-bit division is ~10x cheaper in VALU than
  // the 64-bit emulation (which dominated epilogues that gather rows per element).
  if (m <= LIM && r.d1 <= LIM && r.d2 <= LIM) {
    const uint32_t mu = (uint32_t)m;
    const uint32_t a = udiv32(mu, (uint32_t)r.d1), b = udiv32(mu, (uint32_t)r.d2);
    const int64_t x = r.m1 <= LIM ? (int64_t)umod32(a, (uint32_t)r.m1) : (int64_t)a;
    const int64_t y = r.m2 <= LIM ? (int64_t)umod32(b, (uint32_t)r.m2) : (int64_t)b;
    return x * r.s1 + y * r.s2 + r.off;
  }
  return ((m / r.d1) % r.m1) * r.s1 + ((m / r.d2) % r.m2) * r.s2 + r.off;
}
