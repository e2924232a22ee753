// bf16 3x3 / pad-1 convolution with an LDS-resident input tile (decoder convs of the
// guided upsampler, reference model.py:528-533 DoubleConv inside Up, :540-555).
//
// A workgroup computes 128 consecutive output pixels of one NHWC slice (H*W % 128 == 0,
// so a tile never crosses slices) for all COUT channels.  The input rows the tile needs
// (<= 6 rows incl. the 1-pixel halo) are loaded ONCE into LDS — channels [0, c1) from the
// per-slice tensor (optionally GroupNorm+ReLU'd on load with per-channel scale/shift),
// [c1, C) from the per-image guidance tensor (the concat + repeat of Up.forward,
// model.py:551-554, never materialised) — and the 9 taps are formed by LDS addressing,
// so each input element crosses L2 once per tile instead of 9 times (the im2col kernel
// in conv.hip).  Weights stream through LDS one tap at a time ([COUT][C] slabs, double
// buffered).  MFMA D = W_tap . A_tap^T; epilogue: bias, act, optional GroupNorm partials
// (per tile mean / M2, as conv.hip), fp32 stage -> 16-byte row stores.
#include "common.h"
#include "capi.h"

namespace {

constexpr int TP = 128;          // output pixels per tile
constexpr int NT = 256;          // 4 waves, each 32 pixels x COUT

struct LdsConvP {
  const bf16* s1; int64_t s1_ss; int c1;
  const bf16* s2; int64_t s2_ss; int c2; int64_t s2_div;
  int64_t S; int H; int W; int maxr;
  const bf16* w; const float* bias; int act;
  const float* gmean; const float* grstd; const float* ggamma; const float* gbeta; int gcpg;
  bf16* out; float* stats;
};

template <int C, int COUT>
__global__ __launch_bounds__(NT) void conv_lds_kernel(LdsConvP p) {
  constexpr int CP = C + 8;                 // LDS pixel stride (elements): 16 B pad vs bank conflicts
  constexpr int CPR = C / 8;                // 16-byte chunks per pixel
  constexpr int FN = COUT / 16, FM = 2;     // wave: COUT x 32 pixels
  constexpr int WLD = C + 8;                // weight slab row stride
  constexpr int SLD = COUT + 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int W = p.W, WP = W + 2;
  bf16* sIn = reinterpret_cast<bf16*>(smem);                                  // [MAXR][W+2][CP]
  const int in_bytes = ((p.maxr * WP * CP * 2) + 15) / 16 * 16;
  bf16* sW = reinterpret_cast<bf16*>(smem + in_bytes);                        // [2][COUT][WLD]
  float* gsc = reinterpret_cast<float*>(smem + in_bytes + 2 * COUT * WLD * 2); // [C]
  float* gsh = gsc + C;
  float* red = gsh + C;                                                       // [4][8]
  float* st = reinterpret_cast<float*>(smem);                                 // stage reuses sIn

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int64_t HW = (int64_t)p.H * W;
  const int64_t m0 = (int64_t)blockIdx.x * TP;
  const int64_t s = m0 / HW;
  const int pix0 = (int)(m0 % HW);
  const int y0 = pix0 / W;                         // first output row of the tile
  const int nrows = (pix0 + TP - 1) / W - y0 + 3;  // staged rows y0-1 .. ylast+1

  if (p.gmean) {
    const int ngroups = p.c1 / p.gcpg;
    for (int c = tid; c < p.c1; c += NT) {
      const float sc = p.grstd[s * ngroups + c / p.gcpg] * p.ggamma[c];
      gsc[c] = sc;
      gsh[c] = p.gbeta[c] - p.gmean[s * ngroups + c / p.gcpg] * sc;
    }
  }
  // weights: tap t+1 is loaded into registers before tap t's MFMAs and written to the
  // other LDS buffer after them, so the global latency hides behind the MFMAs.
  constexpr int WCH = (COUT * CPR + NT - 1) / NT;
  uint4 wr[WCH];
  auto load_w = [&](int tap) {
#pragma unroll
    for (int k = 0; k < WCH; ++k) {
      const int i = tid + k * NT;
      if (i < COUT * CPR) wr[k] = ld16(p.w + ((int64_t)(i / CPR) * 9 + tap) * C + (i % CPR) * 8);
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int k = 0; k < WCH; ++k) {
      const int i = tid + k * NT;
      if (i < COUT * CPR) st16(&sW[(buf * COUT + i / CPR) * WLD + (i % CPR) * 8], wr[k]);
    }
  };
  load_w(0);
  store_w(0);
  __syncthreads();    // gsc/gsh ready
  // ---- stage the input rows (zero halo / outside rows) ----
  // Batches of SU independent 16-byte loads per thread are issued before any LDS store,
  // so the global latencies overlap instead of serialising one load-store pair per step.
  constexpr int SU = 8;
  const int total = nrows * WP * CPR;
  const bf16* s1base = p.s1 + s * p.s1_ss;
  const bf16* s2base = p.s2 ? p.s2 + (s / p.s2_div) * p.s2_ss : nullptr;
  for (int i0 = 0; i0 < total; i0 += NT * SU) {
    uint4 u[SU];
#pragma unroll
    for (int j = 0; j < SU; ++j) {
      const int i = i0 + j * NT + tid;
      const int ch = i % CPR, pc = i / CPR;
      const int lr = pc / WP, lc = pc - lr * WP;
      const int yy = y0 - 1 + lr, xx = lc - 1;
      const int ci = ch * 8;
      u[j] = make_uint4(0, 0, 0, 0);
      if (i < total && yy >= 0 && yy < p.H && xx >= 0 && xx < W) {
        const int pix = yy * W + xx;
        if (ci < p.c1) u[j] = ld16(s1base + (int64_t)pix * p.c1 + ci);
        else u[j] = ld16(s2base + (int64_t)pix * p.c2 + (ci - p.c1));
      }
    }
#pragma unroll
    for (int j = 0; j < SU; ++j) {
      const int i = i0 + j * NT + tid;
      if (i < total) {
        const int ch = i % CPR, pc = i / CPR;
        const int ci = ch * 8;
        const int lr = pc / WP, lc = pc - lr * WP;
        const int yy = y0 - 1 + lr, xx = lc - 1;
        if (p.gmean && ci < p.c1 && yy >= 0 && yy < p.H && xx >= 0 && xx < W) {
          bf16* e = reinterpret_cast<bf16*>(&u[j]);
#pragma unroll
          for (int k = 0; k < 8; ++k) e[k] = f2bf(fmaxf(fmaf(bf2f(e[k]), gsc[ci + k], gsh[ci + k]), 0.f));
        }
        st16(&sIn[pc * CP + ci], u[j]);
      }
    }
  }
  __syncthreads();

  // per-lane pixel base offsets (tap (1,1) = centre) for the wave's two 16-pixel tiles
  int base[FM];
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int pp = pix0 + wave * 32 + 16 * j + r16;
    const int lr = pp / W - y0 + 1, lc = pp % W + 1;
    base[j] = (lr * WP + lc) * CP + 8 * q;
  }
  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int tap = 0; tap < 9; ++tap) {
    const int buf = tap & 1;
    if (tap + 1 < 9) load_w(tap + 1);
    const int toff = ((tap / 3 - 1) * WP + (tap % 3 - 1)) * CP;
    const bf16* wb = sW + buf * COUT * WLD;
#pragma unroll
    for (int kc = 0; kc < C / 32; ++kc) {
      s16x8 xf[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) xf[j] = *reinterpret_cast<const s16x8*>(&sIn[base[j] + toff + kc * 32]);
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const s16x8 wf = *reinterpret_cast<const s16x8*>(&wb[(16 * i + r16) * WLD + kc * 32 + 8 * q]);
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(wf, xf[j], acc[i][j]);
      }
    }
    if (tap + 1 < 9) store_w(buf ^ 1);               // other buffer: free since the last barrier
    __syncthreads();
  }

  // ---- epilogue: bias/act, GroupNorm partials, stage, coalesced store ----
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[i][j][r];
        if (p.bias) v += p.bias[16 * i + 4 * q + r];
        acc[i][j][r] = apply_act(v, p.act);
      }
  if (p.stats) {
    // groups of 16 channels: tile i of the wave's FN tiles is group i; reduce over the
    // wave's 32 pixels, then the 4 waves
    float gsum[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) a += acc[i][j][r];
      gsum[i] = warp_sum(a);
    }
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < FN; ++i) red[wave * 8 + i] = gsum[i];
    __syncthreads();
    float gmean[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i)
      gmean[i] = (red[i] + red[8 + i] + red[16 + i] + red[24 + i]) * (1.f / (TP * 16));
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) { const float d = acc[i][j][r] - gmean[i]; a += d * d; }
      gsum[i] = warp_sum(a);
    }
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < FN; ++i) red[wave * 8 + i] = gsum[i];
    __syncthreads();
    if (tid < FN) {
      const int ntiles = (int)(HW / TP), tile = pix0 / TP;
      float* o = p.stats + ((s * ntiles + tile) * FN + tid) * 2;
      o[0] = gmean[tid];
      o[1] = red[tid] + red[8 + tid] + red[16 + tid] + red[24 + tid];
    }
  }
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j)
      *reinterpret_cast<f32x4*>(&st[(wave * 32 + 16 * j + r16) * SLD + 16 * i + 4 * q]) = acc[i][j];
  __syncthreads();
  constexpr int CH = COUT / 8;
  for (int i = tid; i < TP * CH; i += NT) {
    const int r = i / CH, c = (i % CH) * 8;
    const float* sv = &st[r * SLD + c];
    const uint4 o = make_uint4(f2bf2(sv[0], sv[1]), f2bf2(sv[2], sv[3]), f2bf2(sv[4], sv[5]), f2bf2(sv[6], sv[7]));
    st16(p.out + (m0 + r) * COUT + c, o);
  }
}

template <int C, int COUT>
size_t lds_bytes(const LdsConvP& p) {
  constexpr int CP = C + 8, WLD = C + 8;
  const int WP = p.W + 2;
  const size_t in_bytes = ((p.maxr * WP * CP * 2) + 15) / 16 * 16;
  size_t sh = in_bytes + 2 * COUT * WLD * 2 + (2 * C + 32) * 4;
  const size_t stage = (size_t)TP * (COUT + 4) * 4;
  if (stage > in_bytes) sh += stage - in_bytes;   // stage reuses the input tile region
  return sh;
}

// Measured (MI355X, config 3, B=8 T=150): the LDS-tile conv beats the im2col conv for
// 96x96 C64->32 (1.53 vs 2.15 ms), 96x96 C32->32 (0.96 vs 2.05), 48x48 C64->64 (0.55 vs
// 1.20) but not for 48x48 C128->64 (1.20 vs 1.14), whose 116 KiB tile leaves one
// workgroup per CU.
constexpr size_t LDS_LIMIT = 96 * 1024;

template <int C, int COUT>
int launch(const LdsConvP& p, hipStream_t st) {
  const size_t sh = lds_bytes<C, COUT>(p);
  if (sh > LDS_LIMIT) return 1;
  const unsigned grid = (unsigned)(p.S * p.H * p.W / TP);
  static size_t configured = 0;
  if (sh > configured) {   // > 64 KiB dynamic LDS must be opted into (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_lds_kernel<C, COUT>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    configured = sh;
  }
  hipLaunchKernelGGL((conv_lds_kernel<C, COUT>), dim3(grid), dim3(NT), sh, st, p);
  return 0;
}

}  // namespace

// bf16 fast path of catseg_conv3x3 (conv.hip): 0 = launched, 1 = not applicable.
int catseg_conv3x3_lds(const CatsegConvArgs* a, hipStream_t st) {
  if (a->dtype != CATSEG_BF16) return 1;
  const int C = a->c1 + a->c2;
  const int64_t HW = (int64_t)a->H * a->W;
  if (HW % TP != 0 || a->W < 48 || a->W > 96) return 1;
  if (a->s1_offset != 0 || a->s2_offset != 0) return 1;
  if (a->addend) return 1;                      // (the epilogue addend is ring / im2col only)
  if (a->stats && a->stats_cpg != 16) return 1;
  if (a->gn_mean && (a->c1 % 8 != 0)) return 1;
  LdsConvP p;
  p.s1 = (const bf16*)a->src1; p.s1_ss = a->s1_slice_stride; p.c1 = a->c1;
  p.s2 = (const bf16*)a->src2; p.s2_ss = a->s2_slice_stride; p.c2 = a->c2; p.s2_div = a->src2_div > 0 ? a->src2_div : 1;
  p.S = a->S; p.H = a->H; p.W = a->W;
  p.maxr = (a->W - 1 + TP - 1) / a->W + 3;     // tile span + 1-row halo above and below
  p.w = (const bf16*)a->weight; p.bias = a->bias; p.act = a->act;
  p.gmean = a->gn_mean; p.grstd = a->gn_rstd; p.ggamma = a->gn_gamma; p.gbeta = a->gn_beta; p.gcpg = a->gn_cpg;
  p.out = (bf16*)a->out; p.stats = a->stats;
  if (C == 128 && a->c_out == 64) return launch<128, 64>(p, st);
  if (C == 64 && a->c_out == 64) return launch<64, 64>(p, st);
  if (C == 64 && a->c_out == 32) return launch<64, 32>(p, st);
  if (C == 32 && a->c_out == 32) return launch<32, 32>(p, st);
  return 1;
}
