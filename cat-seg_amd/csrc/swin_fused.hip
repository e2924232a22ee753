// catseg_swin_window_attention: argument checks and dispatch (the default kernel is the
// head-per-SIMD form in swin_window.hip) plus the row-tile-wave kernel kept as its A/B reference.
// Fused Swin window attention for the CAT-Seg spatial aggregation (bf16):
//   LayerNorm(norm1) + [q|k|v] projection (+ the per-image guidance half of q, k)
//   + shifted-window multi-head attention, one workgroup per (slice, window).
// Reference: SwinTransformerBlock.forward model.py:191-199 (norm1, concat guidance,
// roll, window_partition) and WindowAttention.forward model.py:86-114 up to (and not
// including) the output projection; the -100 region mask of model.py:161-183.
//
// The 144 x 384 q/k/v of a window never leave the CU: per head, the 144 x 96 slice is
// produced by MFMA from the LayerNorm'd window rows held in registers, written to LDS in the
// layouts the attention loop reads (K [key][d (+ region one-hot)], V^T [d][key],
// Q [query][d]), and consumed at once.  HBM traffic per window: the 144 input rows,
// the 144 output rows, the guidance rows (shared by every class of an image: L2/MALL).
//
// Persistent: one 9-wave workgroup per CU stages all of W_qkv in LDS once and walks the
// windows; wave w owns rows / queries 16w .. 16w+15 of every window: its rows (prefetched
// one window ahead) are LayerNorm'd straight into MFMA B fragments (no LDS).
// Window geometry is compile-time (24 x 24 feature map, 12 x 12 windows: CAT-Seg's
// FEATURE_RESOLUTION / window_size, host-checked).
#include "common.h"
#include "capi.h"

namespace {

constexpr int IMG = 24, WS = 12, NWIN = 4, L = WS * WS;   // 144 tokens per window
constexpr int C = 128, D = 32, NH = 4;
constexpr int NW = 9, NT = NW * 64;
constexpr int XD = 32;                // region one-hot dims appended to K / -100 dims to Q
constexpr int KC = (D + XD) / 8;      // 16-byte chunks of a K row (d | region one-hot)
constexpr int KB = 160;               // key columns of V^T (5 x 32-key MFMA steps)
constexpr int VP = KB + 4;            // V^T row stride
constexpr int KTV = L / 16;           // 9 key tiles

struct SwinP {
  const bf16* x; int64_t ld_x;
  const float* ln_g; const float* ln_b; float eps;
  const bf16* w; const float* bias;
  const bf16* g; int64_t ld_g; RowMap gmap;
  bf16* out; int64_t ld_out;
  int shift; float scale;
};

// LDS images of bf16 rows are chunk-major with a row XOR swizzle (16-byte chunk c of row r
// at slot c * ROWS + (r ^ (c & 15))): MFMA fragment reads (16 rows x 1 chunk per 16 lanes)
// and row writes hit distinct bank slots (the padded row-major images ran ~35 % bank
// conflicts, rocprofv3 SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
template <int ROWS>
DEV int cslot(int c, int r) { return (c * ROWS + (r ^ (c & 15))) * 8; }
// the same slot for r = rbase + rlo (rbase % 16 == 0, rlo < 16): the swizzle stays in the
// low 4 bits, so per-tile addresses are one base + immediate offsets
template <int ROWS>
DEV int cslot16(int c, int rbase, int rlo) { return (c * ROWS + rbase + (rlo ^ (c & 15))) * 8; }

DEV int win_row(int slice, int wloc, int i, int shift) {       // roll(-shift) + partition
  const int Y = (wloc >> 1) * WS + i / WS, X = (wloc & 1) * WS + i % WS;
  const int y = Y + shift < IMG ? Y + shift : Y + shift - IMG;
  const int x = X + shift < IMG ? X + shift : X + shift - IMG;
  return slice * IMG * IMG + y * IMG + x;
}

DEV int region(int wloc, int i, int shift) {                    // model.py:161-176 label
  const int Y = (wloc >> 1) * WS + i / WS, X = (wloc & 1) * WS + i % WS;
  const int hb = Y < IMG - WS ? 0 : (Y < IMG - shift ? 1 : 2);
  const int wb = X < IMG - WS ? 0 : (X < IMG - shift ? 1 : 2);
  return hb * 3 + wb;
}


// Region one-hot dims (chunks 4..7 of every K row) of window location wloc: one key per item,
// 4 x 16-byte stores.  They depend on (wloc, shift) only, and a persistent workgroup strided by
// a multiple of NWIN windows always sees the same wloc, so the kernels write them once.
DEV void put_onehot(bf16* Ks, int wloc, int shift, int tid, int nt) {
  for (int key = tid; key < L; key += nt) {
    const int reg = region(wloc, key, shift);
#pragma unroll
    for (int c = 0; c < XD / 8; ++c) {
      unsigned w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e0 = c * 8 + 2 * j;
        w[j] = (e0 == reg ? 0x3F80u : 0u) | (e0 + 1 == reg ? 0x3F800000u : 0u);
      }
      st16(&Ks[cslot<L>((D >> 3) + c, key)], make_uint4(w[0], w[1], w[2], w[3]));
    }
  }
}

// ---- pipelined row-tile-wave form (A/B reference of swin_window.hip): head h+1's q/k/v projection runs in the same barrier interval
// as head h's attention.  K and V^T are double-buffered in LDS (Q stays in registers: the
// projection leaves lane (row, g) holding q[row][4g..4g+3 | 16+4g..16+4g+3], which is exactly a
// B fragment when the K rows use the same permuted d order inside each 16-byte chunk, so K is
// stored with one 16-byte write per lane and Qs is gone -- that is what makes the second K/V
// buffer fit).  One barrier per head instead of two; the projection MFMAs of one head overlap
// the softmax VALU of the other inside every wave.
template <bool SWM>
__global__ __launch_bounds__(NT) void swin_fused2_kernel(SwinP p, int nwin_total) {
  __shared__ __attribute__((aligned(16))) bf16 sW[3 * C * C];      // all of W_qkv, staged once
  __shared__ __attribute__((aligned(16))) bf16 Ks_[2][L * KC * 8];
  __shared__ __attribute__((aligned(16))) bf16 Vt_[2][D * VP];
  __shared__ __attribute__((aligned(16))) float sP[2 * C + 3 * C];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int qi = wave * 16 + r16;                           // this lane's row / query in a window
  for (int i = tid; i < 5 * C; i += NT) sP[i] = i < C ? p.ln_g[i] : i < 2 * C ? p.ln_b[i - C] : p.bias[i - 2 * C];
  for (int c = tid; c < 3 * C * 16; c += NT) {
    const int lr = c >> 4, ch = c & 15;
    st16(&sW[cslot<3 * C>(ch, lr)], ld16(p.w + (int64_t)lr * C + ch * 8));
  }
  for (int i = tid; i < 2 * D * (KB - L); i += NT) {
    const int b = i / (D * (KB - L)), j = i % (D * (KB - L));
    Vt_[b][(j / (KB - L)) * VP + L + j % (KB - L)] = 0;
  }
  __syncthreads();
  s16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)0x3F80;
  const float sl2 = p.scale * 1.4426950408889634f;

  uint4 nx[4];
  auto fetch = [&](int win) {
    const int64_t row = win_row(win / NWIN, win % NWIN, qi, p.shift);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) nx[ks] = ld16(p.x + row * p.ld_x + ks * 32 + 8 * g);
  };
  int win = blockIdx.x;
  if (win < nwin_total) fetch(win);
  for (; win < nwin_total; win += gridDim.x) {
    const int slice = win / NWIN, wloc = win % NWIN;
    const int64_t qrow = win_row(slice, wloc, qi, p.shift);
    s16x8 hf[4];
    {
      float v[4][8], s = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16* e = reinterpret_cast<const bf16*>(&nx[ks]);
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[ks][j] = bf2f(e[j]); s += v[ks][j]; }
      }
      s = xrow4_sum(s);
      const float mean = s * (1.f / C);
      float q = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[ks][j] -= mean; q += v[ks][j] * v[ks][j]; }
      q = xrow4_sum(q);
      const float rstd = rsqrtf(q * (1.f / C) + p.eps);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int c0 = ks * 32 + 8 * g;
        float o8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o8[j] = v[ks][j] * rstd * sP[c0 + j] + sP[C + c0 + j];
        uint4 u = make_uint4(f2bf2(o8[0], o8[1]), f2bf2(o8[2], o8[3]), f2bf2(o8[4], o8[5]), f2bf2(o8[6], o8[7]));
        hf[ks] = *reinterpret_cast<s16x8*>(&u);
      }
    }
    // region one-hot of every key, in both K buffers (the previous window's last barrier
    // retired every read of them); once per workgroup when its windows share one location
    if constexpr (SWM) {
      if (gridDim.x % NWIN != 0 || win == (int)blockIdx.x) {
        put_onehot(Ks_[0], wloc, p.shift, tid, NT);
        put_onehot(Ks_[1], wloc, p.shift, tid, NT);
      }
    }
    const int qreg = SWM ? region(wloc, qi, p.shift) : 0;
    const bf16* grow_p = p.g + rowmap(p.gmap, qrow) * p.ld_g;

    // q (registers), k, v^T (LDS buffer b) of head h for this wave's 16 rows
    auto proj = [&](int h, int b, s16x8& qout) {
      int r16_ = lane & 15, g_ = lane >> 4;
      asm volatile("" : "+v"(r16_), "+v"(g_));
#pragma unroll 1
      for (int part = 0; part < 3; ++part) {
        float v[2][4];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int n0 = part * C + h * D + dt * 16;
          f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            a = mfma_bf16(*reinterpret_cast<const s16x8*>(&sW[cslot16<3 * C>(ks * 4 + g_, n0, r16_)]), hf[ks], a);
          const int n = n0 + 4 * g_;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[dt][r] = a[r] + sP[2 * C + n + r];
          if (part < 2) {
            float gv[4];
            load4<bf16>(grow_p + n, gv);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[dt][r] += gv[r];
          }
        }
        if (part < 2) {
          // 16-byte chunk g_ = d {4g..4g+3, 16+4g..16+4g+3} (the permuted order of Q and K)
          const uint4 u = make_uint4(f2bf2(v[0][0], v[0][1]), f2bf2(v[0][2], v[0][3]), f2bf2(v[1][0], v[1][1]),
                                     f2bf2(v[1][2], v[1][3]));
          if (part == 0) qout = __builtin_bit_cast(s16x8, u);
          else st16(&Ks_[b][cslot16<L>(g_, wave * 16, r16_)], u);
        } else {
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int r = 0; r < 4; ++r) Vt_[b][(dt * 16 + 4 * g_ + r) * VP + qi] = f2bf(v[dt][r]);
        }
      }
    };
    s16x8 qcur;
    proj(0, 0, qcur);
    __syncthreads();
#pragma unroll 1
    for (int h = 0; h < NH; ++h) {
      const int b = h & 1;
      s16x8 qnext;
      if (h + 1 < NH) proj(h + 1, b ^ 1, qnext);
      // the next window's rows are requested during the last head (not across the whole window:
      // their 16 VGPRs would be live beside the attention state of every head)
      else if (win + (int)gridDim.x < nwin_total) fetch(win + gridDim.x);
      const bf16* Ks = Ks_[b];
      const bf16* Vt = Vt_[b];
      int r16_ = lane & 15, g_ = lane >> 4;
      asm volatile("" : "+v"(r16_), "+v"(g_));
      s16x8 qmask;             // -100/scale on the dims of every other region (rebuilt per head: 4 VGPRs fewer)
      if constexpr (SWM) {
        const short neg = (short)f2bf(-100.f / p.scale);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int dim = 8 * g_ + j;
          qmask[j] = dim < 9 && dim != qreg ? neg : (short)0;
        }
      }
      f32x4 st[KTV + 1];
#pragma unroll
      for (int kt = 0; kt < KTV; ++kt) {
        f32x4 a = mfma_bf16(*reinterpret_cast<const s16x8*>(&Ks[cslot16<L>(g_, kt * 16, r16_)]), qcur,
                            f32x4{0.f, 0.f, 0.f, 0.f});
        if constexpr (SWM) a = mfma_bf16(*reinterpret_cast<const s16x8*>(&Ks[cslot16<L>(4 + g_, kt * 16, r16_)]), qmask, a);
        st[kt] = a;
      }
      float mx = -1e30f;
#pragma unroll
      for (int kt = 0; kt < KTV; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, st[kt][r]);
      mx = xrow4_max(mx);
      const float nb = -mx * sl2;
#pragma unroll
      for (int kt = 0; kt < KTV; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[kt][r] = __builtin_amdgcn_exp2f(fmaf(st[kt][r], sl2, nb));
      st[KTV] = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, osum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < KB / 32; ++u) {
        uint4 pu = make_uint4(f2bf2(st[2 * u][0], st[2 * u][1]), f2bf2(st[2 * u][2], st[2 * u][3]),
                              f2bf2(st[2 * u + 1][0], st[2 * u + 1][1]), f2bf2(st[2 * u + 1][2], st[2 * u + 1][3]));
        const s16x8 pb = *reinterpret_cast<s16x8*>(&pu);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16* vr = &Vt[(dt * 16 + r16_) * VP + 32 * u + 4 * g_];
          const uint2 lo = *reinterpret_cast<const uint2*>(vr);
          const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16);
          uint4 va = make_uint4(lo.x, lo.y, hi.x, hi.y);
          o[dt] = mfma_bf16(*reinterpret_cast<s16x8*>(&va), pb, o[dt]);
        }
        osum = mfma_bf16(ones, pb, osum);
      }
      const float inv = 1.f / osum[0];
      bf16* O = p.out + qrow * p.ld_out + h * D;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
        *reinterpret_cast<uint2*>(O + dt * 16 + 4 * g_) =
            make_uint2(f2bf2(o[dt][0] * inv, o[dt][1] * inv), f2bf2(o[dt][2] * inv, o[dt][3] * inv));
      __syncthreads();    // buffer b is rewritten by the projection of head h + 2 / the next window
      qcur = qnext;
    }
  }
}

// 0 (default) = the register-resident kernel (swin_window.hip swin_win5: two 4-wave workgroups per
// CU, wave h holding head h's k / v^T / q in registers after the projection), 1 = the head-per-SIMD
// kernel (swin_win3) with the builtin LDS-DMA and a row map per tile, 2 = the row-tile-wave kernel
// (swin_fused2_kernel), 3 = swin_win3 with the opaque (inline-asm) LDS-DMA and the per-window
// guidance base (the default until round 3), 16 = variant 3 with phase stamps (diagnostics,
// tools/stamps_swin.py).  Row maps that are not base + pixel per slice run swin_win3.
// (A barrier-free form with two 4-wave workgroups per CU, every head wave LayerNorming its window's
// rows itself, measured 314 / 410 us vs 259 / 271 us: the per-wave load -> LayerNorm -> MFMA chains
// left their latency exposed.)
int g_swin_variant = 0;

}  // namespace

CATSEG_KNOB(g_swin_variant, "swin_variant");

int swin_win3_launch(const CatsegSwinAttnArgs* a, int n_cu, hipStream_t st, bool asm_dma, bool glin, bool stamps);   // swin_window.hip
int swin_win5_launch(const CatsegSwinAttnArgs* a, int n_cu, hipStream_t st, bool glin);

// the guidance row map restricted to one slice is rowmap(slice * 576) + pixel (swin_win3 then adds the pixel)
static bool gmap_linear_in_pixel(const CatsegRowMap& m) {
  const int64_t P = IMG * IMG;
  return (m.d2 == 1 && m.s2 == 1 && m.m2 % P == 0 && m.d1 % P == 0) ||
         (m.d1 == 1 && m.s1 == 1 && m.m1 % P == 0 && m.d2 % P == 0);
}

extern "C" int catseg_swin_window_attention(const CatsegSwinAttnArgs* a, void* stream) {
  CATSEG_CHECK(a && a->x && a->ln_g && a->ln_b && a->w_qkv && a->b_qkv && a->gqk && a->out,
               "swin_window_attention: null pointer");
  CATSEG_CHECK(a->dtype == CATSEG_BF16, "swin_window_attention: bf16 only");
  CATSEG_CHECK(a->img_h == IMG && a->img_w == IMG && a->window == WS, "swin_window_attention: 24x24 map, 12x12 windows");
  CATSEG_CHECK(a->n_heads == NH && a->head_dim == D, "swin_window_attention: 4 heads x 32");
  CATSEG_CHECK(a->shift >= 0 && a->shift < WS, "swin_window_attention: bad shift");
  CATSEG_CHECK(a->S > 0 && a->S * NWIN < (1LL << 31), "swin_window_attention: bad slice count");
  CATSEG_CHECK(a->ld_x % 8 == 0 && a->ld_g % 4 == 0 && a->ld_out % 4 == 0, "swin_window_attention: row alignment");
  CATSEG_CHECK(a->gmap.d1 > 0 && a->gmap.m1 > 0 && a->gmap.d2 > 0 && a->gmap.m2 > 0, "swin_window_attention: bad gmap");
  SwinP p;
  p.x = (const bf16*)a->x; p.ld_x = a->ld_x;
  p.ln_g = a->ln_g; p.ln_b = a->ln_b; p.eps = a->eps;
  p.w = (const bf16*)a->w_qkv; p.bias = a->b_qkv;
  p.g = (const bf16*)a->gqk; p.ld_g = a->ld_g;
  p.gmap = RowMap{a->gmap.d1, a->gmap.m1, a->gmap.s1, a->gmap.d2, a->gmap.m2, a->gmap.s2, a->gmap.off};
  p.out = (bf16*)a->out; p.ld_out = a->ld_out;
  p.shift = a->shift; p.scale = a->scale;
  // persistent: one workgroup per CU (W_qkv staged once per CU), windows strided over them
  const int n_cu = catseg_device_cus();
  const int nwin_total = (int)(a->S * NWIN);
  const dim3 grid((unsigned)std::min(nwin_total, n_cu));
  const bool glin = gmap_linear_in_pixel(a->gmap);
  if (glin && g_swin_variant == 0) {
    swin_win5_launch(a, n_cu, (hipStream_t)stream, true);
  } else if (g_swin_variant != 2) {
    // (variant 0 with a row map that is not base + pixel per slice runs swin_win3's row-map form)
    const bool v3 = g_swin_variant != 1;
    swin_win3_launch(a, n_cu, (hipStream_t)stream, v3, v3 && glin, g_swin_variant == 16);
  } else {
    if (a->shift > 0)
      hipLaunchKernelGGL(swin_fused2_kernel<true>, grid, dim3(NT), 0, (hipStream_t)stream, p, nwin_total);
    else
      hipLaunchKernelGGL(swin_fused2_kernel<false>, grid, dim3(NT), 0, (hipStream_t)stream, p, nwin_total);
  }
  return catseg_launch_status("swin_window_attention");
}
