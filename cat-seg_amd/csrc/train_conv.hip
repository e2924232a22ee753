// Convolutions of the aggregation head for training, fp32, NHWC, stride 1,
// "same" padding: the guidance projections (model.py:615-630), DoubleConv (model.py:520-533),
// corr_embed's 7x7 conv (model.py:613,654-659) and the head conv (model.py:634,679).
//
// catseg_conv2d_nhwc — implicit GEMM  y[p][co] = alpha * act(sum_{tap, ci} x[p + tap][ci] w[tap][ci][co]
//   + bias[co]) + beta * y[p][co].  The same kernel is the data gradient of a conv: dX = conv(dY, w')
//   with w'[tap][co][ci] = w[ci... flipped] (the host passes the flipped, transposed weight).
// catseg_conv2d_wgrad — dw[tap][ci][co] = alpha * sum_p x[p + tap][ci] dy[p][co] + beta * dw: a GEMM
//   with the pixel count as its reduction, split over the grid into fp32 partials summed in a fixed
//   order (deterministic, no atomics).
// catseg_head_conv_backward — conv 32 -> 1 (3x3, bias): dx, dw, db in one pass over x (a 1-channel
//   output leaves an MFMA tile 1/16 used, so this one is VALU).
// MFMA: exact-f32 16x16x4, D^T = W^T . X^T so a lane ends with 4 consecutive output channels.
#include "common.h"
#include "capi.h"
#include "catseg_hip_train.h"

namespace {

constexpr int CBK = 16, CNT = 256;
// Tiles (pixels or (tap, ci) rows x output channels): 128 x 64 (four waves of 32 x 64) for cout > 32,
// 256 x 32 (four waves of 64 x 32) for cout <= 32, so the 32-channel decoder convs spend no MFMA on
// zero weight columns; either way a wave issues 8 MFMAs per 4-deep k-step.
// [k][m] images: element (k, m) at k * pitch + (m ^ swz(k)): the transposing stores (8 m x 4 k-quads
// per 32-lane group) hit 32 distinct banks, fragment reads (16 m x 2 k per group) stay conflict-free
DEV int swz(int k) { return ((k >> 2) & 3) << 3; }

template <bool VEC, int BMT, int BNT>
__global__ __launch_bounds__(CNT) void conv_fwd_kernel(CatsegConv2dArgs a, int tiles_n) {
  constexpr int CLA = BMT + 16, CLB = BNT + 16;
  constexpr int WM = BMT / 4, FM = WM / 16, FN = BNT / 16;
  __shared__ __attribute__((aligned(16))) float As[2][CBK * CLA];
  __shared__ __attribute__((aligned(16))) float Bs[2][CBK * CLB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t m0 = (int64_t)(lin / tiles_n) * BMT;
  const int n0 = (lin % tiles_n) * BNT;
  const float* x = (const float*)a.x;
  const float* w = (const float*)a.w;
  const int H = a.H, W = a.W, cin = a.cin, cout = a.cout, ks = a.ksize, pad = a.pad;
  const int64_t HWp = (int64_t)H * W, M = a.S * HWp;
  const int nkc = (cin + CBK - 1) / CBK;
  const int nslab = ks * ks * nkc;

  // per-thread A rows (fixed over K): VEC chunks of 4 channels, else scalars
  constexpr int NA = VEC ? BMT / 64 : BMT / 16;
  int64_t a_base[NA]; int a_y[NA], a_x[NA], a_k[NA], a_m[NA]; bool a_ok[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int c = tid + i * CNT;
    a_m[i] = VEC ? c >> 2 : c >> 4;
    a_k[i] = VEC ? (c & 3) * 4 : c & 15;
    const int64_t m = m0 + a_m[i];
    a_ok[i] = m < M;
    const int64_t mm = a_ok[i] ? m : 0;
    const int64_t s = mm / HWp, rem = mm % HWp;
    a_y[i] = (int)(rem / W); a_x[i] = (int)(rem % W);
    a_base[i] = s * HWp;
  }
  float4 ra[VEC ? NA : 1];
  float rs[VEC ? 1 : NA];
  float4 rb;
  constexpr int BQ = BNT / 4;                 // float4 per weight row of the tile
  const bool b_on = tid < CBK * BQ;
  auto gload = [&](int slab) {
    const int tap = slab / nkc, ci0 = (slab % nkc) * CBK;
    const int dy = tap / ks - pad, dx = tap % ks - pad;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int sy = a_y[i] + dy, sx = a_x[i] + dx, ci = ci0 + a_k[i];
      const bool ok = a_ok[i] && sy >= 0 && sy < H && sx >= 0 && sx < W && ci < cin;
      const float* p = x + (a_base[i] + (int64_t)sy * W + sx) * a.ld_x + ci;
      if constexpr (VEC) ra[i] = ok ? *reinterpret_cast<const float4*>(p) : make_float4(0, 0, 0, 0);
      else rs[i] = ok ? *p : 0.f;
    }
    const int kr = tid / BQ, n4 = (tid % BQ) * 4;
    const int ci = ci0 + kr, n = n0 + n4;
    rb = (b_on && ci < cin && n < cout) ? *reinterpret_cast<const float4*>(w + ((int64_t)tap * cin + ci) * a.ld_w + n)
                                        : make_float4(0, 0, 0, 0);
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (VEC) {
        float* d = &As[buf][a_k[i] * CLA + (a_m[i] ^ swz(a_k[i]))];
        d[0] = ra[i].x; d[CLA] = ra[i].y; d[2 * CLA] = ra[i].z; d[3 * CLA] = ra[i].w;
      } else {
        As[buf][a_k[i] * CLA + (a_m[i] ^ swz(a_k[i]))] = rs[i];
      }
    }
    if (b_on) *reinterpret_cast<float4*>(&Bs[buf][(tid / BQ) * CLB + (tid % BQ) * 4]) = rb;
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  gload(0);
  sstore(0);
  __syncthreads();
  for (int sl = 0; sl < nslab; ++sl) {
    const int buf = sl & 1;
    if (sl + 1 < nslab) gload(sl + 1);
#pragma unroll
    for (int kk = 0; kk < CBK; kk += 4) {
      float av[FM], bv[FN];
#pragma unroll
      for (int j = 0; j < FM; ++j) av[j] = As[buf][(kk + g) * CLA + ((wave * WM + 16 * j + r) ^ swz(kk))];
#pragma unroll
      for (int i = 0; i < FN; ++i) bv[i] = Bs[buf][(kk + g) * CLB + 16 * i + r];
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_f32(bv[i], av[j], acc[i][j]);
    }
    if (sl + 1 < nslab) sstore(buf ^ 1);
    __syncthreads();
  }
  float* y = (float*)a.y;
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + 16 * i + 4 * g;
    if (n >= cout) continue;
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias) {
#pragma unroll
      for (int u = 0; u < 4; ++u) bias[u] = a.bias[n + u];
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int64_t m = m0 + wave * WM + 16 * j + r;
      if (m >= M) continue;
      float* p = y + m * a.ld_y + n;
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = acc[i][j][u] + bias[u];
        if (a.act == ACT_RELU) t = fmaxf(t, 0.f);
        t *= a.alpha;
        if (a.beta) t += p[u];
        v[u] = t;
      }
      *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

template <bool VEC, int BMT, int BNT>
__global__ __launch_bounds__(CNT) void conv_wgrad_kernel(CatsegConv2dArgs a, int tiles_n, int64_t k_chunk,
                                                         float* __restrict__ part) {
  constexpr int CLA = BMT + 16, CLB = BNT + 16;
  constexpr int WM = BMT / 4, FM = WM / 16, FN = BNT / 16;
  __shared__ __attribute__((aligned(16))) float As[2][CBK * CLA];
  __shared__ __attribute__((aligned(16))) float Bs[2][CBK * CLB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (lin / tiles_n) * BMT;
  const int n0 = (lin % tiles_n) * BNT;
  const float* x = (const float*)a.x;
  const float* dy = (const float*)a.y;
  const int H = a.H, W = a.W, cin = a.cin, cout = a.cout, ks = a.ksize, pad = a.pad;
  const int64_t HWp = (int64_t)H * W, K = a.S * HWp;
  const int M = ks * ks * cin;
  const int64_t kb = (int64_t)blockIdx.y * k_chunk;
  const int64_t ke = kb + k_chunk < K ? kb + k_chunk : K;

  // per-thread A columns (tap, ci) fixed over K; pixel row a_kk of the 16-pixel slab
  constexpr int AQ = VEC ? BMT / 4 : BMT;     // A items per slab row
  constexpr int NA = CBK * AQ / CNT;
  int a_kk[NA], a_mm[NA], a_dy[NA], a_dx[NA], a_ci[NA]; bool a_ok[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int c = tid + i * CNT;
    a_kk[i] = c / AQ;
    a_mm[i] = VEC ? (c % AQ) * 4 : c % AQ;
    const int m = m0 + a_mm[i];
    a_ok[i] = m < M;
    const int tap = a_ok[i] ? m / cin : 0;
    a_ci[i] = a_ok[i] ? m % cin : 0;
    a_dy[i] = tap / ks - pad;
    a_dx[i] = tap % ks - pad;
  }
  // the (slice, row, column) of each A pixel, divided out once and advanced by CBK pixels per slab
  // (no 64-bit division in the loop: it was most of this kernel's VALU)
  int64_t c_s[NA];
  int c_y[NA], c_x[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int64_t p0 = kb + a_kk[i];
    c_s[i] = p0 / HWp;
    const int64_t rem = p0 % HWp;
    c_y[i] = (int)(rem / W);
    c_x[i] = (int)(rem % W);
  }
  float4 ra[VEC ? NA : 1];
  float rs[VEC ? 1 : NA];
  float4 rb;
  constexpr int BQ = BNT / 4;
  const bool b_on = tid < CBK * BQ;
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int64_t pix = k0 + a_kk[i];
      const int sy = c_y[i] + a_dy[i], sx = c_x[i] + a_dx[i];
      const bool ok = a_ok[i] && pix < ke && sy >= 0 && sy < H && sx >= 0 && sx < W;
      const float* p = x + (c_s[i] * HWp + (int64_t)sy * W + sx) * a.ld_x + a_ci[i];
      if constexpr (VEC) ra[i] = ok ? *reinterpret_cast<const float4*>(p) : make_float4(0, 0, 0, 0);
      else rs[i] = ok ? *p : 0.f;
      c_x[i] += CBK;
      while (c_x[i] >= W) {
        c_x[i] -= W;
        if (++c_y[i] == H) { c_y[i] = 0; ++c_s[i]; }
      }
    }
    const int kr = tid / BQ, n4 = (tid % BQ) * 4;
    const int64_t pix = k0 + kr;
    const int n = n0 + n4;
    rb = (b_on && pix < ke && n < cout) ? *reinterpret_cast<const float4*>(dy + pix * a.ld_y + n)
                                        : make_float4(0, 0, 0, 0);
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (VEC) *reinterpret_cast<float4*>(&As[buf][a_kk[i] * CLA + (a_mm[i] ^ swz(a_kk[i]))]) = ra[i];
      else As[buf][a_kk[i] * CLA + (a_mm[i] ^ swz(a_kk[i]))] = rs[i];
    }
    if (b_on) *reinterpret_cast<float4*>(&Bs[buf][(tid / BQ) * CLB + (tid % BQ) * 4]) = rb;
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = ke > kb ? (int)((ke - kb + CBK - 1) / CBK) : 0;
  if (nk > 0) {
    gload(kb);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kb + (int64_t)(kt + 1) * CBK);
#pragma unroll
    for (int kk = 0; kk < CBK; kk += 4) {
      float av[FM], bv[FN];
#pragma unroll
      for (int j = 0; j < FM; ++j) av[j] = As[buf][(kk + g) * CLA + ((wave * WM + 16 * j + r) ^ swz(kk))];
#pragma unroll
      for (int i = 0; i < FN; ++i) bv[i] = Bs[buf][(kk + g) * CLB + 16 * i + r];
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_f32(bv[i], av[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
  float* dst = part ? part + (int64_t)blockIdx.y * M * cout : (float*)a.dw;
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + 16 * i + 4 * g;
    if (n >= cout) continue;
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wave * WM + 16 * j + r;
      if (m >= M) continue;
      float* p = dst + (int64_t)m * cout + n;
      float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      if (!part) {
        v.x *= a.alpha; v.y *= a.alpha; v.z *= a.alpha; v.w *= a.alpha;
        if (a.beta) { const float4 o = *reinterpret_cast<const float4*>(p); v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w; }
      }
      *reinterpret_cast<float4*>(p) = v;
    }
  }
}

// dw[i] = alpha * sum_z part[z][i] + beta * dw[i]: 16 outputs x 16 split lanes per workgroup, fixed tree
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int64_t n,
                                                           float* __restrict__ dw, float alpha, int beta) {
  __shared__ float red[256];
  const int ci = threadIdx.x & 15, zl = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + ci;
  float s = 0.f;
  if (i < n) {
#pragma unroll 8
    for (int z = zl; z < splits; z += 16) s += part[(int64_t)z * n + i];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off >= 16; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x < 16 && i < n) dw[i] = alpha * red[threadIdx.x] + (beta ? dw[i] : 0.f);
}

// the tile for an output-channel count
struct ConvTile { int bm, bn; };
ConvTile conv_tile(int cout) { return cout <= 32 ? ConvTile{256, 32} : ConvTile{128, 64}; }
// weight gradient: M = taps x cin rows; 192-row tiles where they waste fewer rows than 256 (M = 576:
// 3 full tiles instead of 2 + a quarter-used one; M = 288: 2 tiles at 75 % instead of 56 %)
ConvTile wgrad_tile(int64_t M, int cout) {
  if (cout > 32) return ConvTile{128, 64};
  const int64_t t256 = (M + 255) / 256, t192 = (M + 191) / 192;
  return t192 * 192 < t256 * 256 ? ConvTile{192, 32} : ConvTile{256, 32};
}

int wgrad_splits(const CatsegConv2dArgs* a) {
  const int64_t M = (int64_t)a->ksize * a->ksize * a->cin;
  const ConvTile t = wgrad_tile(M, a->cout);
  const int64_t tiles = ((M + t.bm - 1) / t.bm) * ((a->cout + t.bn - 1) / t.bn);
  const int64_t K = a->S * a->H * a->W;
  // one round of resident workgroups: LDS per workgroup 2 x 16 x (bm + 16 + bn + 16) floats
  // (256 x 32: 41 KB -> 3 per CU; 128 x 64: 29 KB -> 5 per CU); floor, so no tail round
  const int64_t lds = 2LL * CBK * (t.bm + 16 + t.bn + 16) * 4;
  const int64_t slots = 256 * ((160 * 1024) / lds);
  int64_t s = slots / tiles;
  const int64_t kmax = K / (CBK * 64);
  if (s > kmax) s = kmax;
  if (s > 512) s = 512;
  return s < 1 ? 1 : (int)s;
}

// ------------------------------------------------------------------------------ head conv backward
// thread item i = (pixel q, 4-channel chunk); the grid stride is a multiple of C/4, so a thread's
// channel chunk is fixed and it accumulates dw[tap][c..c+3] for the pixels it visits.
constexpr int HC_WG = 1024;
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dl,
                                                       const float* __restrict__ w, float* __restrict__ dx, int64_t S,
                                                       int H, int W, int C, float* __restrict__ part) {
  __shared__ float red[256][37];
  const int c4n = C / 4;
  const int cq = (threadIdx.x % c4n) * 4;
  float wr[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) wr[t][u] = w[t * C + cq + u];
  float acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[t][u] = 0.f;
  const int64_t HW = (int64_t)H * W, total = S * HW * c4n;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
    const int64_t q = i / c4n;
    const int64_t s = q / HW;
    const int rem = (int)(q % HW), yq = rem / W, xq = rem % W;
    const float4 xv = *reinterpret_cast<const float4*>(x + q * C + cq);
    const float xa[4] = {xv.x, xv.y, xv.z, xv.w};
    float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // y[p] reads x[p + (ky-1, kx-1)] through tap t, so x[q] feeds y[q - (ky-1, kx-1)]
      const int py = yq - (t / 3 - 1), px = xq - (t % 3 - 1);
      const float d = (py >= 0 && py < H && px >= 0 && px < W) ? dl[s * HW + py * W + px] : 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        o[u] += d * wr[t][u];
        acc[t][u] += d * xa[u];
      }
    }
    *reinterpret_cast<float4*>(dx + q * C + cq) = make_float4(o[0], o[1], o[2], o[3]);
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) red[threadIdx.x][t * 4 + u] = acc[t][u];
  __syncthreads();
  // threads with the same channel chunk: threadIdx % c4n; sum them in thread order
  for (int e = threadIdx.x; e < 9 * C; e += 256) {
    const int t = e / C, c = e % C, ch = c / 4, u = c % 4;
    float s = 0.f;
    for (int th = ch; th < 256; th += c4n) s += red[th][t * 4 + u];
    part[(int64_t)blockIdx.x * 9 * C + e] = s;
  }
}

__global__ __launch_bounds__(256) void head_final_kernel(const float* __restrict__ part, int nwg, int n,
                                                         float* __restrict__ dw) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int z = 0; z < nwg; ++z) s += part[(int64_t)z * n + i];
  dw[i] = s;
}

// ------------------------------------------------------------------------------ corr_embed input grad
// dcorr[s][q] = sum_{tap, co} dX[s][q - off(tap)][co] w[co][tap]: the 7x7 conv's data gradient with a
// single output channel (an MFMA tile would be 1/16 used).  One workgroup per slice; 32-channel chunks
// of the slice's dX staged in LDS, the weights transposed to [tap][co] beside them.
constexpr int CEC = 32, CEP = CEC + 4;
__global__ __launch_bounds__(256) void corr_dgrad_kernel(const float* __restrict__ dX, const float* __restrict__ w,
                                                         float* __restrict__ dcorr, int H, int W, int D, int k) {
  extern __shared__ float sm[];
  const int HW = H * W, taps = k * k, pad = k / 2;
  float* xs = sm;                        // [HW][CEP]
  float* wt = sm + HW * CEP;             // [taps][CEC]
  const int64_t s = blockIdx.x;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < D; c0 += CEC) {
    __syncthreads();
    for (int e = threadIdx.x; e < HW * (CEC / 4); e += 256) {
      const int p = e / (CEC / 4), c = (e % (CEC / 4)) * 4;
      *reinterpret_cast<float4*>(xs + p * CEP + c) =
          *reinterpret_cast<const float4*>(dX + (s * HW + p) * (int64_t)D + c0 + c);
    }
    for (int e = threadIdx.x; e < taps * CEC; e += 256) {
      const int co = e / taps, t = e % taps;
      wt[t * CEC + co] = w[(int64_t)(c0 + co) * taps + t];
    }
    __syncthreads();
    int slot = 0;
    for (int q = threadIdx.x; q < HW; q += 256, ++slot) {
      const int y = q / W, x = q % W;
      float a = 0.f;
      for (int t = 0; t < taps; ++t) {
        const int py = y - (t / k - pad), px = x - (t % k - pad);
        if (py < 0 || py >= H || px < 0 || px >= W) continue;
        const float* xr = xs + (py * W + px) * CEP;
        const float* wr = wt + t * CEC;
#pragma unroll
        for (int c = 0; c < CEC; c += 4) {
          const float4 xv = *reinterpret_cast<const float4*>(xr + c);
          const float4 wv = *reinterpret_cast<const float4*>(wr + c);
          a += xv.x * wv.x + xv.y * wv.y + xv.z * wv.z + xv.w * wv.w;
        }
      }
      if (slot < 4) acc[slot] += a;
    }
  }
  int slot = 0;
  for (int q = threadIdx.x; q < HW && slot < 4; q += 256, ++slot) dcorr[s * HW + q] = acc[slot];
}

int head_grid(int64_t S, int H, int W, int C) {
  const int64_t items = S * H * W * (C / 4);
  const int64_t wg = (items + 256 * 16 - 1) / (256 * 16);
  return (int)(wg < HC_WG ? (wg < 1 ? 1 : wg) : HC_WG);
}

int check_conv(const CatsegConv2dArgs* a, bool wgrad) {
  CATSEG_CHECK(a && a->x && a->w == a->w && a->y, "conv2d: null pointer");
  CATSEG_CHECK(a->S > 0 && a->H > 0 && a->W > 0 && a->cin > 0 && a->cout > 0, "conv2d: empty shape");
  CATSEG_CHECK(a->ksize > 0 && a->ksize % 2 == 1 && a->pad == a->ksize / 2, "conv2d: odd ksize, pad = ksize / 2 only");
  CATSEG_CHECK(a->cout % 4 == 0, "conv2d: cout must be a multiple of 4");
  CATSEG_CHECK(a->ld_x >= a->cin && a->ld_y >= (wgrad ? a->cout : a->cout), "conv2d: bad row strides");
  CATSEG_CHECK(a->ld_y % 4 == 0 && ((uintptr_t)a->y % 16) == 0, "conv2d: y rows must be 16-byte aligned");
  if (a->cin % 4 == 0) CATSEG_CHECK(a->ld_x % 4 == 0 && ((uintptr_t)a->x % 16) == 0, "conv2d: x rows must be 16-byte aligned");
  return CATSEG_OK;
}

}  // namespace

extern "C" int catseg_conv2d_nhwc(const CatsegConv2dArgs* a, void* stream) {
  if (int e = check_conv(a, false)) return e;
  CATSEG_CHECK(a->w && a->ld_w >= a->cout && a->ld_w % 4 == 0 && ((uintptr_t)a->w % 16) == 0, "conv2d: bad weight");
  CATSEG_CHECK(a->act == ACT_NONE || a->act == ACT_RELU, "conv2d: act must be none or relu");
  const int64_t M = a->S * a->H * a->W;
  const ConvTile t = conv_tile(a->cout);
  const int64_t tm = (M + t.bm - 1) / t.bm, tn = (a->cout + t.bn - 1) / t.bn;
  CATSEG_CHECK(tm * tn < (1LL << 31), "conv2d: too many tiles");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(tm * tn));
  const bool vec = a->cin % 4 == 0;
  if (t.bn == 32) {
    if (vec) hipLaunchKernelGGL((conv_fwd_kernel<true, 256, 32>), grid, dim3(CNT), 0, st, *a, (int)tn);
    else hipLaunchKernelGGL((conv_fwd_kernel<false, 256, 32>), grid, dim3(CNT), 0, st, *a, (int)tn);
  } else {
    if (vec) hipLaunchKernelGGL((conv_fwd_kernel<true, 128, 64>), grid, dim3(CNT), 0, st, *a, (int)tn);
    else hipLaunchKernelGGL((conv_fwd_kernel<false, 128, 64>), grid, dim3(CNT), 0, st, *a, (int)tn);
  }
  return catseg_launch_status("conv2d_nhwc");
}

extern "C" int64_t catseg_conv2d_wgrad_workspace(const CatsegConv2dArgs* a) {
  if (!a || a->S <= 0 || a->cin <= 0 || a->cout <= 0 || a->ksize <= 0) return 0;
  const int s = wgrad_splits(a);
  return s > 1 ? (int64_t)s * a->ksize * a->ksize * a->cin * a->cout * (int64_t)sizeof(float) : 0;
}

extern "C" int catseg_conv2d_wgrad(const CatsegConv2dArgs* a, void* stream) {
  if (int e = check_conv(a, true)) return e;
  CATSEG_CHECK(a->dw && ((uintptr_t)a->dw % 16) == 0, "conv2d_wgrad: dw missing / unaligned");
  const int64_t M = (int64_t)a->ksize * a->ksize * a->cin;
  CATSEG_CHECK(M < (1LL << 30), "conv2d_wgrad: weight too large");
  const ConvTile t = wgrad_tile(M, a->cout);
  const int64_t tm = (M + t.bm - 1) / t.bm, tn = (a->cout + t.bn - 1) / t.bn;
  const int splits = wgrad_splits(a);
  const int64_t need = splits > 1 ? (int64_t)splits * M * a->cout * (int64_t)sizeof(float) : 0;
  if (splits > 1) CATSEG_CHECK(a->workspace && a->workspace_bytes >= need, "conv2d_wgrad: workspace too small");
  const int64_t K = a->S * a->H * a->W;
  int64_t kc = (K + splits - 1) / splits;
  kc = (kc + CBK - 1) / CBK * CBK;
  hipStream_t st = (hipStream_t)stream;
  float* part = splits > 1 ? (float*)a->workspace : nullptr;
  dim3 grid((unsigned)(tm * tn), (unsigned)splits);
  const bool vec = a->cin % 4 == 0;
  if (t.bm == 192) {
    if (vec) hipLaunchKernelGGL((conv_wgrad_kernel<true, 192, 32>), grid, dim3(CNT), 0, st, *a, (int)tn, kc, part);
    else hipLaunchKernelGGL((conv_wgrad_kernel<false, 192, 32>), grid, dim3(CNT), 0, st, *a, (int)tn, kc, part);
  } else if (t.bn == 32) {
    if (vec) hipLaunchKernelGGL((conv_wgrad_kernel<true, 256, 32>), grid, dim3(CNT), 0, st, *a, (int)tn, kc, part);
    else hipLaunchKernelGGL((conv_wgrad_kernel<false, 256, 32>), grid, dim3(CNT), 0, st, *a, (int)tn, kc, part);
  } else {
    if (vec) hipLaunchKernelGGL((conv_wgrad_kernel<true, 128, 64>), grid, dim3(CNT), 0, st, *a, (int)tn, kc, part);
    else hipLaunchKernelGGL((conv_wgrad_kernel<false, 128, 64>), grid, dim3(CNT), 0, st, *a, (int)tn, kc, part);
  }
  if (splits > 1) {
    const int64_t n = M * a->cout;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, st, (const float*)part,
                       splits, n, (float*)a->dw, a->alpha, a->beta);
  }
  return catseg_launch_status("conv2d_wgrad");
}

extern "C" int catseg_corr_embed_backward_input(const float* dX, const float* weight, float* dcorr, int64_t S, int H,
                                                int W, int D, int ksize, void* stream) {
  CATSEG_CHECK(dX && weight && dcorr && S > 0 && H > 0 && W > 0 && ksize > 0 && ksize % 2 == 1,
               "corr_embed_backward_input: bad args");
  CATSEG_CHECK(D % CEC == 0, "corr_embed_backward_input: hidden must be a multiple of 32");
  CATSEG_CHECK((int64_t)H * W <= 4 * 256, "corr_embed_backward_input: at most 1024 pixels per slice");
  const size_t sh = ((size_t)H * W * CEP + (size_t)ksize * ksize * CEC) * sizeof(float);
  CATSEG_CHECK(sh <= 160 * 1024, "corr_embed_backward_input: slice too large for LDS");
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_dgrad_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    configured = true;
  }
  CATSEG_CHECK(S < (1LL << 31), "corr_embed_backward_input: too many slices");
  hipLaunchKernelGGL(corr_dgrad_kernel, dim3((unsigned)S), dim3(256), sh, (hipStream_t)stream, dX, weight, dcorr, H, W, D,
                     ksize);
  return catseg_launch_status("corr_embed_backward_input");
}

extern "C" int64_t catseg_head_conv_backward_workspace(int64_t S, int H, int W, int C) {
  if (S <= 0 || H <= 0 || W <= 0 || C <= 0) return 0;
  return (int64_t)head_grid(S, H, W, C) * 9 * C * (int64_t)sizeof(float);
}

extern "C" int catseg_head_conv_backward(const float* x, const float* dlogits, const float* weight, float* dx, float* dw,
                                         int64_t S, int H, int W, int C, void* workspace, int64_t workspace_bytes,
                                         void* stream) {
  CATSEG_CHECK(x && dlogits && weight && dx && dw && S > 0 && H > 0 && W > 0, "head_conv_backward: bad args");
  CATSEG_CHECK(C % 4 == 0 && C <= 64 && 256 % (C / 4) == 0, "head_conv_backward: C must be a multiple of 4, <= 64");
  const int grid = head_grid(S, H, W, C);
  CATSEG_CHECK(workspace && workspace_bytes >= (int64_t)grid * 9 * C * (int64_t)sizeof(float),
               "head_conv_backward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(head_bwd_kernel, dim3(grid), dim3(256), 0, st, x, dlogits, weight, dx, S, H, W, C, (float*)workspace);
  hipLaunchKernelGGL(head_final_kernel, dim3((unsigned)((9 * C + 255) / 256)), dim3(256), 0, st,
                     (const float*)workspace, grid, 9 * C, dw);
  return catseg_launch_status("head_conv_backward");
}
