// bf16 3x3 / pad-1 convolution with a sliding ring of input rows in LDS and the weights
// in registers (decoder convs of the guided upsampler, reference model.py:528-533
// DoubleConv inside Up, :540-555).
//
// A workgroup walks a band of consecutive 128-pixel chunks of one NHWC slice.  The
// input rows live in a 6-row LDS ring (row y in slot (y + 1) % 6, one zero halo column
// each side, rows outside the image zero) and each row is loaded from HBM ONCE per band:
// while the MFMAs of chunk c run, the rows chunk c+1 adds are already in flight in
// registers (global -> VGPR), and are written into the slots chunk c+1 no longer needs
// after the chunk's barrier.  Channels [0, c1) come from the per-slice tensor
// (GroupNorm+ReLU'd on the way in when the conv consumes relu(GN(x))), [c1, C) from the
// per-image guidance tensor (the concat + repeat of Up.forward, model.py:551-554, never
// materialised).  The 16-byte channel chunks of a ring pixel are XOR-swizzled by its
// position so the 16 pixels of a fragment read hit distinct LDS bank slots.
//
// Each wave keeps ITS slice of the weights for all 9 taps as MFMA A fragments in
// registers for the life of the workgroup (WCO waves split COUT, WPX split the chunk's
// pixels), so the LDS traffic is the pixel fragments only.  D = W_tap . X_tap^T; the
// epilogue adds bias, applies the activation, emits the per-(128-pixel tile, group)
// GroupNorm mean / M2 partials in the layout of conv.hip, and stores bf16 rows.
#include "common.h"
#include "capi.h"

namespace {

constexpr int CH = 128;          // output pixels per chunk (= GroupNorm partial tile)
constexpr int NT = 256;          // 4 waves
constexpr int NR = 6;            // ring rows (a chunk spans <= 4 rows + 2 halo at W >= 48)

struct RingP {
  const bf16* s1; int64_t s1_ss; int c1;
  const bf16* s2; int64_t s2_ss; int c2; int64_t s2_div;
  int64_t S; int H; int W; int chunks_per_band; int bands;
  const bf16* w; const float* bias; int act;
  const float* gmean; const float* grstd; const float* ggamma; const float* gbeta; int gcpg;
  bf16* out; float* stats;
};

template <int C>
DEV int ring_off(int pos, int ch) {        // element offset of 16-byte chunk ch of ring position pos
  constexpr int CPX = C / 8;               // chunks per pixel
  constexpr int PPB = CPX >= 16 ? 1 : 16 / CPX;   // pixels per 256-byte bank row
  return pos * C + ((ch ^ ((pos / PPB) % CPX)) << 3);
}

template <int C, int COUT, int WPX, int WCO, int NPOS>
__global__ __launch_bounds__(NT, 2) void conv_ring_kernel(RingP p) {
  constexpr int CPX = C / 8;
  constexpr int MAXPF = (NPOS * CPX + NT - 1) / NT;     // prefetch chunks per thread
  constexpr int PXW = CH / WPX, FM = PXW / 16;          // pixels per wave, their 16-px tiles
  constexpr int COW = COUT / WCO, FN = COW / 16;        // output channels per wave
  constexpr int KC = C / 32;                            // MFMA k-steps per tap
  static_assert(WPX * WCO == 4 && FM >= 1 && FN >= 1, "wave grid");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* ring = reinterpret_cast<bf16*>(smem);
  const int W = p.W, WP = W + 2, H = p.H;
  const int ring_elems = NR * WP * C;
  float* gsc = reinterpret_cast<float*>(smem + (size_t)ring_elems * 2);   // [C]
  float* gsh = gsc + C;                                                    // [C]
  float* red = gsh + C;                                                    // [4][4]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int wpx = wave % WPX, wco = wave / WPX;
  const int64_t s = blockIdx.x / p.bands;
  const int band = blockIdx.x % p.bands;
  const int HW = H * W;
  const int nchunks = HW / CH;
  const int c_begin = band * p.chunks_per_band;
  const int c_end = min(nchunks, c_begin + p.chunks_per_band);
  if (c_begin >= c_end) return;

  // ---- weights of this wave's output channels, all taps, in registers ----
  s16x8 wf[9][KC][FN];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = wco * COW + 16 * i + r16;
        uint4 u = ld16(p.w + ((int64_t)n * 9 + tap) * C + kc * 32 + 8 * q);
        wf[tap][kc][i] = *reinterpret_cast<s16x8*>(&u);
      }
  if (p.gmean) {
    const int ngroups = p.c1 / p.gcpg;
    for (int c = tid; c < p.c1; c += NT) {
      const float sc = p.grstd[s * ngroups + c / p.gcpg] * p.ggamma[c];
      gsc[c] = sc;
      gsh[c] = p.gbeta[c] - p.gmean[s * ngroups + c / p.gcpg] * sc;
    }
  }
  const bf16* s1base = p.s1 + s * p.s1_ss;
  const bf16* s2base = p.s2 ? p.s2 + (s / p.s2_div) * p.s2_ss : nullptr;

  // load 16-byte chunk (row y, ring column xc, chunk ch) from HBM (zero outside the image)
  auto gload = [&](int y, int xc, int ch) -> uint4 {
    const int x = xc - 1, ci = ch * 8;
    if (y < 0 || y >= H || x < 0 || x >= W) return make_uint4(0, 0, 0, 0);
    const int pix = y * W + x;
    return ci < p.c1 ? ld16(s1base + (int64_t)pix * p.c1 + ci) : ld16(s2base + (int64_t)pix * p.c2 + (ci - p.c1));
  };
  auto lput = [&](int y, int xc, int ch, uint4 u) {
    const int ci = ch * 8;
    if (p.gmean && ci < p.c1 && y >= 0 && y < H && xc >= 1 && xc <= W) {
      bf16* e = reinterpret_cast<bf16*>(&u);
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = f2bf(fmaxf(fmaf(bf2f(e[k]), gsc[ci + k], gsh[ci + k]), 0.f));
    }
    const int pos = ((y + 1) % NR) * WP + xc;
    st16(&ring[ring_off<C>(pos, ch)], u);
  };
  const int row_items = WP * CPX;

  // ---- prime: rows needed by the first chunk ----
  __syncthreads();   // gsc/gsh
  int loaded_to;     // rows [.., loaded_to] are in the ring
  {
    const int p0 = c_begin * CH;
    const int ya = p0 / W - 1, yb = (p0 + CH - 1) / W + 1;
    const int total = (yb - ya + 1) * row_items;
    for (int i0 = 0; i0 < total; i0 += NT * 8) {
      uint4 u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + j * NT + tid;
        u[j] = i < total ? gload(ya + i / row_items, (i % row_items) / CPX, i % CPX) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + j * NT + tid;
        if (i < total) lput(ya + i / row_items, (i % row_items) / CPX, i % CPX, u[j]);
      }
    }
    loaded_to = yb;
  }
  // per-thread prefetch items, decoded once: (row offset << 16) | (ring column << 4) | chunk
  int pf_code[MAXPF];
#pragma unroll
  for (int k = 0; k < MAXPF; ++k) {
    const int i = tid + k * NT;
    pf_code[k] = ((i / row_items) << 16) | (((i % row_items) / CPX) << 4) | (i % CPX);
  }
  __syncthreads();

  for (int c = c_begin; c < c_end; ++c) {
    const int p0 = c * CH;
    // ---- prefetch the rows the next chunk adds ----
    uint4 pf[MAXPF];
    int nnew = 0;
    if (c + 1 < c_end) {
      const int yb_next = min((p0 + 2 * CH - 1) / W + 1, H);
      nnew = yb_next - loaded_to;
    }
#pragma unroll
    for (int k = 0; k < MAXPF; ++k)
      pf[k] = (pf_code[k] >> 16) < nnew
                  ? gload(loaded_to + 1 + (pf_code[k] >> 16), (pf_code[k] >> 4) & 0xfff, pf_code[k] & 15)
                  : make_uint4(0, 0, 0, 0);

    // ---- MFMAs: 9 taps x KC k-steps over the ring ----
    int prow[FM], pcol[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int pp = p0 + wpx * PXW + 16 * j + r16;
      prow[j] = pp / W;
      pcol[j] = pp - prow[j] * W + 1;        // ring column of the centre tap
    }
    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      int rbase[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) rbase[j] = ((prow[j] + dy) % NR) * WP + pcol[j] - 1;   // slot of row y+dy-1
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int tap = dy * 3 + dx;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          s16x8 xf[FM];
#pragma unroll
          for (int j = 0; j < FM; ++j)
            xf[j] = *reinterpret_cast<const s16x8*>(&ring[ring_off<C>(rbase[j] + dx, kc * 4 + q)]);
#pragma unroll
          for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(wf[tap][kc][i], xf[j], acc[i][j]);
        }
      }
    }

    // ---- epilogue: bias / act, GroupNorm partials, bf16 stores ----
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r];
          if (p.bias) v += p.bias[wco * COW + 16 * i + 4 * q + r];
          acc[i][j][r] = apply_act(v, p.act);
        }
    if (p.stats) {
      // group of 16 channels = one n-tile; reduce the wave's PXW pixels, then the WPX
      // waves that share the wave's channel range
      float gs[FN];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < FM; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) a += acc[i][j][r];
        gs[i] = warp_sum(a);
      }
      if (lane == 0)
#pragma unroll
        for (int i = 0; i < FN; ++i) red[wave * 4 + i] = gs[i];
      __syncthreads();
      float gm[FN];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        float a = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < WPX; ++w2) a += red[(wco * WPX + w2) * 4 + i];
        gm[i] = a * (1.f / (CH * 16));
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < FM; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) { const float d = acc[i][j][r] - gm[i]; a += d * d; }
        gs[i] = warp_sum(a);
      }
      if (lane == 0)
#pragma unroll
        for (int i = 0; i < FN; ++i) red[wave * 4 + i] = gs[i];
      __syncthreads();
      if (wpx == 0 && lane < FN) {
        float m2 = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < WPX; ++w2) m2 += red[(wco * WPX + w2) * 4 + lane];
        float gml = gm[0];
#pragma unroll
        for (int i = 1; i < FN; ++i) if (lane == i) gml = gm[i];
        const int grp = (wco * COW) / 16 + lane;
        float* o = p.stats + (((int64_t)s * nchunks + c) * (COUT / 16) + grp) * 2;
        o[0] = gml;
        o[1] = m2;
      }
    }
    bf16* ob = p.out + ((int64_t)s * HW + p0 + wpx * PXW) * COUT + wco * COW;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        store4<bf16>(ob + (int64_t)(16 * j + r16) * COUT + 16 * i + 4 * q, v);
      }

    // ---- rotate the ring: prefetched rows into the slots the next chunk no longer needs ----
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MAXPF; ++k)
      if ((pf_code[k] >> 16) < nnew) lput(loaded_to + 1 + (pf_code[k] >> 16), (pf_code[k] >> 4) & 0xfff, pf_code[k] & 15, pf[k]);
    loaded_to += nnew > 0 ? nnew : 0;
    __syncthreads();
  }
}

template <int C>
size_t ring_lds(int W) { return (size_t)NR * (W + 2) * C * 2 + (2 * C + 16) * 4; }

// NPOS bounds the ring positions one chunk adds: ceil(128 / W) rows of W + 2 columns,
// <= 156 for 48 <= W <= 50 and <= 198 for any 48 <= W <= 96.
template <int C, int COUT, int WPX, int WCO, int NPOS>
int launch_ring(const RingP& p0, hipStream_t st) {
  RingP p = p0;
  const int nchunks = p.H * p.W / CH;
  // bands of ~24 chunks (a band re-primes its ring once), at least 2 workgroups per CU
  int bands = (nchunks + 23) / 24;
  while (p.S * bands < 2048 && bands * 4 <= nchunks) bands *= 2;
  p.bands = bands;
  p.chunks_per_band = (nchunks + bands - 1) / bands;
  const size_t sh = ring_lds<C>(p.W);
  static size_t configured = 0;
  if (sh > configured) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_ring_kernel<C, COUT, WPX, WCO, NPOS>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    configured = sh;
  }
  hipLaunchKernelGGL((conv_ring_kernel<C, COUT, WPX, WCO, NPOS>), dim3((unsigned)(p.S * bands)), dim3(NT), sh, st, p);
  return 0;
}

}  // namespace

// bf16 fast path of catseg_conv3x3 (conv.hip): 0 = launched, 1 = not applicable.
int catseg_conv3x3_ring(const CatsegConvArgs* a, hipStream_t st) {
  if (a->dtype != CATSEG_BF16) return 1;
  const int C = a->c1 + a->c2;
  const int64_t HW = (int64_t)a->H * a->W;
  if (HW % CH != 0 || a->W < 48 || a->W > 96) return 1;
  if (a->s1_offset != 0 || a->s2_offset != 0) return 1;
  if (a->stats && a->stats_cpg != 16) return 1;
  if (a->gn_mean && (a->c1 % 8 != 0)) return 1;
  RingP p;
  p.s1 = (const bf16*)a->src1; p.s1_ss = a->s1_slice_stride; p.c1 = a->c1;
  p.s2 = (const bf16*)a->src2; p.s2_ss = a->s2_slice_stride; p.c2 = a->c2; p.s2_div = a->src2_div > 0 ? a->src2_div : 1;
  p.S = a->S; p.H = a->H; p.W = a->W;
  p.w = (const bf16*)a->weight; p.bias = a->bias; p.act = a->act;
  p.gmean = a->gn_mean; p.grstd = a->gn_rstd; p.ggamma = a->gn_gamma; p.gbeta = a->gn_beta; p.gcpg = a->gn_cpg;
  p.out = (bf16*)a->out; p.stats = a->stats;
  // weights in registers: 9 taps x C/32 x COUT/WCO/16 fragments (<= 36 = 144 VGPRs)
  const bool narrow = a->W <= 50;
  if (C == 64 && a->c_out == 32) return narrow ? launch_ring<64, 32, 4, 1, 156>(p, st) : launch_ring<64, 32, 4, 1, 198>(p, st);
  if (C == 32 && a->c_out == 32) return narrow ? launch_ring<32, 32, 4, 1, 156>(p, st) : launch_ring<32, 32, 4, 1, 198>(p, st);
  if (C == 64 && a->c_out == 64 && narrow) return launch_ring<64, 64, 1, 4, 156>(p, st);
  return 1;
}
