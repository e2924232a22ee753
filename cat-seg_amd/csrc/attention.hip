// Flash-style softmax attention for gfx950 (MFMA, online softmax, LDS-staged K/V).
//
// One workgroup = NW waves; each wave owns QT query tiles of 16 queries of one
// (sequence, head), so one staged K/V block serves 16*NW*QT queries.  Per 16-key tile
// a wave computes S^T = K . Q^T: the 16x16 C/D layout then puts ONE query per lane
// column (col = lane & 15) and 4 keys per register group (row = 4*(lane>>4) + r), so
// the per-query max / sum need only the two xor-16/32 shuffles, and the exponentiated
// tile is already the B operand of O^T = V^T . P^T (k order permuted inside each 32-key
// step; V^T is read from LDS in the same permuted order — cdna_hip_programming.md §3
// "An accumulator tile as the next MFMA's operand").  K tiles are stored [key][d],
// V tiles transposed [d][key].
//
// mode 0: dense sequences (CLIP ViT MHA, model_vpt.py:202-206; causal text encoder,
//         model_vpt.py:400-406).  KB = 64-key blocks, online softmax across blocks.
// mode 1: Swin windows with cyclic shift + -100 region mask (model.py:86-114,
//         161-216); the roll/partition/reverse are folded into the row index.  The
//         whole 144-key window is one block (KB = 160), so one workgroup does all 144
//         queries of a (window, head) from a single K/V staging.
#include "common.h"
#include "capi.h"

namespace {

struct AttnP {
  const void* q; const void* k; const void* v; int64_t ld;
  void* out; int64_t ldo;
  int64_t n_seq; int L; int H; float scale; int causal;
  int mode; int img_h, img_w, ws, shift;
  int skip_tail;   // skip the MFMAs of key tiles wholly past L (catseg_set_attn_tail_skip A/B)
};

// GEO != 0: the window geometry is compile-time (GEO x GEO image, GEO/2 windows — CAT-Seg's
// 24x24 feature map with 12x12 windows), so every index division is by a constant.
template <int GEO>
DEV int64_t seq_row(const AttnP& p, int s, int i) {
  if (p.mode == 0) return (int64_t)s * p.L + i;
  const int IH = GEO ? GEO : p.img_h, IW = GEO ? GEO : p.img_w, WS = GEO ? GEO / 2 : p.ws;
  const int nwx = IW / WS, nwin = (IH / WS) * nwx;
  const int slice = s / nwin, w = s % nwin;
  const int Y = (w / nwx) * WS + i / WS, X = (w % nwx) * WS + i % WS;
  const int y = (Y + p.shift) % IH, x = (X + p.shift) % IW;
  return (int64_t)slice * IH * IW + y * IW + x;
}

template <int GEO>
DEV int swin_region(const AttnP& p, int wloc, int i) {
  const int IH = GEO ? GEO : p.img_h, IW = GEO ? GEO : p.img_w, WS = GEO ? GEO / 2 : p.ws;
  const int nwx = IW / WS;
  const int Y = (wloc / nwx) * WS + i / WS, X = (wloc % nwx) * WS + i % WS;
  const int hb = Y < IH - WS ? 0 : (Y < IH - p.shift ? 1 : 2);
  const int wb = X < IW - WS ? 0 : (X < IW - p.shift ? 1 : 2);
  return hb * 3 + wb;
}

// SWM: the shifted-window -100 region mask (model.py:161-183) is applied by the MFMA
// itself: each staged key row gets XD extra dims holding the one-hot of its region
// (3 x 3 regions) and each query fragment the matching dims -100/scale for every other
// region, so S = q.k + mask comes out of the same instruction chain and the softmax
// loop carries no per-score mask work (this kernel is VALU-bound: head_dim 32 gives one
// 16x16x32 MFMA per 256 scores).  The softmax row sums come from the MFMA too: a
// constant all-ones A fragment times P^T adds one MFMA per 32 keys instead of one VALU
// add per score.
template <typename T, int D, int NW, int KB, int QT, int GEO, bool SWM, bool CAUSAL>
__global__ __launch_bounds__(NW * 64) void attn_kernel(AttnP p) {
  constexpr int NT = NW * 64;
  constexpr bool BF = sizeof(T) == 2;
  constexpr int VN = Vec16<T>::N;
  constexpr int XD = SWM ? (BF ? 32 : 12) : 0;          // region dims appended to K / Q
  // bf16: K and V both staged row-major [key][d] with 16-element row padding: the K
  // fragment reads (ds_read_b128, 16-B slot 10*row + g mod 16 for D + XD = 64) and the V
  // transposed reads (ds_read_b64_tr_b16, 8 rows x 32 B per 32-lane half, row stride 24 or
  // 40 dwords) are conflict-free; fp32 keeps V^T [d][key]
  constexpr int KP = D + XD + (BF ? 16 : 4);            // K row stride (elements)
  constexpr int VP = BF ? D + 16 : KB + 4;              // V row stride (bf16) / V^T row stride (fp32)
  constexpr int VROWS = BF ? KB : D;
  constexpr int DT = D / 16;                            // d tiles of O^T
  constexpr int KT = KB / 16;                           // key tiles per block
  constexpr int KS = BF ? 32 : 4;                       // K depth of one MFMA
  constexpr int QF = D / KS, QX = XD / KS;
  constexpr int LC = GEO ? (GEO / 2) * (GEO / 2) : 0;   // compile-time sequence length
  constexpr int KTV = LC ? (LC + 15) / 16 : KT;         // key tiles that can hold a key
  static_assert(!LC || (LC <= KB && LC % 16 == 0), "fixed window must fill whole key tiles");
  using QFrag = typename std::conditional<BF, s16x8, float>::type;
  __shared__ __attribute__((aligned(16))) T Ks[KB * KP];
  __shared__ __attribute__((aligned(16))) T Vt[VROWS * VP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lin = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  const int bx = lin % gridDim.x, by = lin / gridDim.x;   // query blocks of one head on one XCD
  const int s = by / p.H;
  const int h = by % p.H;
  const int g = lane >> 4;
  const int L = LC ? LC : p.L;
  const T* Kg = reinterpret_cast<const T*>(p.k);
  const T* Vg = reinterpret_cast<const T*>(p.v);
  const int nwin = p.mode == 1 ? (GEO ? 4 : (p.img_h / p.ws) * (p.img_w / p.ws)) : 1;
  const int wloc = p.mode == 1 ? s % nwin : 0;
  const float sl2 = p.scale * 1.4426950408889634f;   // exp(x) = exp2(x * log2 e)

  int qi[QT];
  int64_t qrow[QT];
  bool q_ok[QT], tile_live[QT];
  QFrag qf[QT][QF + QX];
  f32x4 o[QT][DT], osum[QT];
  float m_run[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int q0 = (bx * NW * QT + wave * QT + t) * 16;
    tile_live[t] = q0 < L;
    qi[t] = q0 + (lane & 15);
    q_ok[t] = qi[t] < L;
    qrow[t] = seq_row<GEO>(p, s, q_ok[t] ? qi[t] : 0);
    const T* Q = reinterpret_cast<const T*>(p.q) + qrow[t] * p.ld + h * D;
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < QF; ++ks) {
        uint4 u = q_ok[t] ? ld16(Q + ks * 32 + 8 * g) : make_uint4(0, 0, 0, 0);
        qf[t][ks] = *reinterpret_cast<s16x8*>(&u);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < QF; ++ks) qf[t][ks] = q_ok[t] ? to_f<T>(Q[4 * ks + g]) : 0.f;
    }
    if constexpr (SWM) {
      const int qreg = swin_region<GEO>(p, wloc, q_ok[t] ? qi[t] : 0);
      const float neg = -100.f / p.scale;                // raw-score units (scores are scaled later)
      if constexpr (BF) {
        s16x8 f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int dim = 8 * g + j;
          f[j] = (short)f2bf(dim < 9 && dim != qreg ? neg : 0.f);
        }
        qf[t][QF] = f;
      } else {
#pragma unroll
        for (int e = 0; e < QX; ++e) {
          const int dim = 4 * e + g;
          qf[t][QF + e] = dim < 9 && dim != qreg ? neg : 0.f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < DT; ++i) o[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    osum[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    m_run[t] = -1e30f;
  }
  QFrag ones;
  if constexpr (BF) {
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (short)0x3F80;   // bf16 1.0
  } else {
    ones = 1.f;
  }

  const int nblk = (L + KB - 1) / KB;
  for (int blk = 0; blk < nblk; ++blk) {
    const int k0 = blk * KB;
    // ---- stage K [key][d (+ region one-hot)] and V^T [d][key] ----
    constexpr int CPK = D / VN;
    for (int c = tid; c < KB * CPK; c += NT) {
      const int kk = c / CPK, d0 = (c % CPK) * VN;
      const int key = k0 + kk;
      uint4 ku = make_uint4(0, 0, 0, 0), vu = make_uint4(0, 0, 0, 0);
      if (key < L) {
        const int64_t r = seq_row<GEO>(p, s, key);
        ku = ld16(Kg + r * p.ld + h * D + d0);
        vu = ld16(Vg + r * p.ld + h * D + d0);
      }
      st16(&Ks[kk * KP + d0], ku);
      if constexpr (BF) {
        st16(&Vt[kk * VP + d0], vu);
      } else {
        const T* ve = reinterpret_cast<const T*>(&vu);
#pragma unroll
        for (int j = 0; j < VN; ++j) Vt[(d0 + j) * VP + kk] = ve[j];
      }
      if constexpr (SWM) {
        if (d0 == 0) {
          const int kreg = key < L ? swin_region<GEO>(p, wloc, key) : -1;
#pragma unroll
          for (int e = 0; e < XD; ++e) Ks[kk * KP + D + e] = from_f<T>(e == kreg ? 1.f : 0.f);
        }
      }
    }
    __syncthreads();
    const bool tail = !LC && k0 + KB > L;                 // block-uniform: keys past L exist

#pragma unroll
    for (int t = 0; t < QT; ++t) {
      if (!tile_live[t]) continue;
      // ---- S^T tiles (raw q.k, + region mask dims) ----
      f32x4 st[KT];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        // a key tile wholly past L (the tail block: L = 577 leaves one key in the last 64-key
        // block) is all -inf after the mask below: its MFMAs are skipped (block-uniform branch)
        if (kt < KTV && (!tail || !p.skip_tail || k0 + kt * 16 < L)) {
          const int kr = kt * 16 + (lane & 15);
#pragma unroll
          for (int ks = 0; ks < QF + QX; ++ks) {
            if constexpr (BF) {
              const s16x8 kf = *reinterpret_cast<const s16x8*>(&Ks[kr * KP + ks * 32 + 8 * g]);
              a = mfma_bf16(kf, qf[t][ks], a);
            } else {
              a = mfma_f32(Ks[kr * KP + 4 * ks + g], qf[t][ks], a);
            }
          }
        }
        st[kt] = a;
      }
      if (tail || CAUSAL) {
#pragma unroll
        for (int kt = 0; kt < KTV; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + kt * 16 + 4 * g + r;
            if (key >= L || (CAUSAL && key > qi[t])) st[kt][r] = -INFINITY;
          }
      }
      // ---- online softmax (per query column): max, then exp2(s * sl2 - m * sl2) ----
      float bmax = -1e30f;
#pragma unroll
      for (int kt = 0; kt < KTV; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) bmax = fmaxf(bmax, st[kt][r]);
      bmax = xrow4_max(bmax);
      const float m_new = fmaxf(m_run[t], bmax);
      const float alpha = __builtin_amdgcn_exp2f((m_run[t] - m_new) * sl2);
      m_run[t] = m_new;
      const float nb = -m_new * sl2;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          st[kt][r] = kt < KTV ? __builtin_amdgcn_exp2f(fmaf(st[kt][r], sl2, nb)) : 0.f;
      if (blk > 0) {
#pragma unroll
        for (int i = 0; i < DT; ++i) o[t][i] *= alpha;
        osum[t] *= alpha;
      }

      // ---- O^T += V^T . P^T ; row sums += 1 . P^T ----
      if constexpr (BF) {
#pragma unroll
        for (int u = 0; u < KB / 32; ++u) {
          if (2 * u >= KTV) continue;
          if (tail && p.skip_tail && k0 + 32 * u >= L) continue;          // P = 0 on all 32 keys: O, l unchanged
          uint4 pu = make_uint4(f2bf2(st[2 * u][0], st[2 * u][1]), f2bf2(st[2 * u][2], st[2 * u][3]),
                                f2bf2(st[2 * u + 1][0], st[2 * u + 1][1]), f2bf2(st[2 * u + 1][2], st[2 * u + 1][3]));
          const s16x8 pb = *reinterpret_cast<s16x8*>(&pu);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            // V^T fragment by transposed reads: lane 4q'+p' of group g addresses key row
            // 32u + 4g + q' (and + 16), columns 16 dt + 4p' .. +3; lane i receives d = 16 dt + i
            // over those 4 keys -- P's permuted key order (keys 32u + 4g + r, then + 16)
            const int i16 = lane & 15;
            const T* vr = &Vt[(32 * u + 4 * g + (i16 >> 2)) * VP + dt * 16 + 4 * (i16 & 3)];
            typedef short s16x4 __attribute__((ext_vector_type(4)));
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(vr));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(vr + 16 * VP));
            const s16x8 va = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            o[t][dt] = mfma_bf16(va, pb, o[t][dt]);
          }
          osum[t] = mfma_bf16(ones, pb, osum[t]);
        }
      } else {
#pragma unroll
        for (int kt = 0; kt < KTV; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
              const float va = to_f<T>(Vt[(dt * 16 + (lane & 15)) * VP + kt * 16 + 4 * g + r]);
              o[t][dt] = mfma_f32(va, st[kt][r], o[t][dt]);
            }
            osum[t] = mfma_f32(ones, st[kt][r], osum[t]);
          }
      }
    }
    __syncthreads();
  }

  // ---- normalize + store: lane holds O^T[d = dt*16 + 4g + r][q]; osum rows all = l[q] ----
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    if (!q_ok[t]) continue;
    const float inv = 1.f / osum[t][0];
    T* O = reinterpret_cast<T*>(p.out) + qrow[t] * p.ldo + h * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      float v[4] = {o[t][dt][0] * inv, o[t][dt][1] * inv, o[t][dt][2] * inv, o[t][dt][3] * inv};
      store4<T>(O + dt * 16 + 4 * g, v);
    }
  }
}

// ------------------------------------------------------------------------------------
// CLIP ViT MHA (bf16, head_dim 64, dense, non-causal; model_vpt.py:202-206), one wave per
// 16 queries of one (image, head), NW waves sharing 64-key K/V blocks.  LDS-DMA ring: the K / V
// blocks arrive by global_load_lds (no staging VGPRs, no staging VALU) into a 4-slot ring with two
// blocks in flight beyond the one being read, so the load latency is covered by two blocks of
// compute; one raw barrier per block (each wave retires its own pieces with a counted vmcnt
// first).  The LDS images are unpadded 128-byte rows with the 16-byte chunk XOR-swizzled by
// row & 7 (applied to the per-lane DMA source, so the lane-linear DMA destination lands the
// swizzled image): K fragment reads (ds_read_b128) and V^T transposed reads (ds_read_b64_tr_b16)
// are conflict-free.
//   * Defer-max online softmax (cdna_hip_programming.md T13): the running max m of a query
//     moves only when a block's scores exceed it by more than 2^THR in exp2 units, so the
//     common block costs one max chain per lane and one wave vote -- no cross-lane reduction,
//     no rescale of O.  The softmax is invariant to the subtracted constant; p <= 2^THR.
//   * Row sums l from the MFMA (all-ones A fragment times P^T), as attn_kernel.
//   * Rows past L read the clamped row L-1 (no per-element branch); their scores are masked.
// ------------------------------------------------------------------------------------
// L2S (mode 2): the q rows arrive multiplied by scale * log2(e) (folded into the q projection's
// weights and bias), so S = K Q^T is already the exponent in log2 units.  The running max then
// enters as the MFMA's accumulator input (C = -m), S - m comes out of the matrix pipe, and the
// softmax is one v_exp per score (no scale / subtract FMA); block 0 seeds the max.
template <int NW, int QT, bool L2S = false, bool WT = false>
__global__ __launch_bounds__(NW * 64, (2 * NW + 3) / 4) void vit_attn3_kernel(AttnP p) {   // two workgroups per CU
  constexpr int D = 64, KB = 64, NBUF = 4, AHEAD = 2;
  constexpr int BLK = 2 * KB * D;                       // elements of one ring slot (K rows, then V rows)
  constexpr int NI = (16 + NW - 1) / NW;                // DMA pieces (1 KiB) per wave per block
  constexpr float THR = 16.f;                           // defer-max threshold (log2 units)
  __shared__ __attribute__((aligned(16))) bf16 smem[NBUF * BLK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // all query blocks of one (sequence, head) on one XCD: its K / V are fetched into one L2
  const int lin = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  const int bx = lin % gridDim.x, by = lin / gridDim.x;
  const int s = by / p.H, h = by % p.H;
  const int g = lane >> 4, col = lane & 15;
  const int L = p.L;
  const float sl2 = p.scale * 1.4426950408889634f;
  const int q0 = (bx * NW + wave) * 16 * QT;
  const bool live = q0 < L;                             // wave-uniform
  const int64_t row0 = (int64_t)s * L;

  // QT query tiles of 16 per wave: every K fragment / V^T read feeds QT MFMAs
  s16x8 qf[QT][2];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int qi = q0 + 16 * t + col;
    const bf16* Q = reinterpret_cast<const bf16*>(p.q) + (row0 + (qi < L ? qi : 0)) * p.ld + h * D;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 u = qi < L ? ld16(Q + ks * 32 + 8 * g) : make_uint4(0, 0, 0, 0);
      qf[t][ks] = *reinterpret_cast<s16x8*>(&u);
    }
  }
  // DMA pieces: piece j = 8 key rows (j % 8) * 8 .. +7 of K (j < 8) or V; lane l lands in slot l
  // of the piece = row r = (j % 8) * 8 + l / 8, swizzled chunk l % 8 = chunk c ^ (r & 7).
  // Every wave issues NI pieces (wave-uniform counted vmcnt); surplus waves repeat pieces (benign
  // duplicate writes of identical bytes)
  const bf16* psrc[NI];
  int prow[NI], pdst[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int j = (wave * NI + i) % 16, which = j >> 3;
    const int r = (j & 7) * 8 + (lane >> 3), c = (lane & 7) ^ (r & 7);
    prow[i] = r;
    psrc[i] = reinterpret_cast<const bf16*>(which ? p.v : p.k) + row0 * p.ld + h * D + c * 8;
    pdst[i] = which * KB * D + (j & 7) * 8 * D;          // element offset of the piece in a slot
  }
  auto issue = [&](int blk) {
    bf16* slot = smem + (blk % NBUF) * BLK;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int key = min(blk * KB + prow[i], L - 1);    // rows past L re-read row L-1 (masked)
      dma16(psrc[i] + (int64_t)key * p.ld, slot + pdst[i]);
    }
  };

  f32x4 o[QT][4], osum[QT];
  float m_run[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) o[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    osum[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    m_run[t] = -1e30f;
  }
  s16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)0x3F80;   // bf16 1.0
  // per-lane byte offsets in a slot: K fragment rows kt*16 + col, chunks ks*4 + g (swizzle col & 7);
  // V^T transposed reads rows 32u + 4g + col/4 (+16), chunk 2dt + ((col & 3) >> 1), half col & 1
  const int kswz = col & 7;
  const int koff0 = col * 128 + ((g ^ kswz) << 4), koff1 = col * 128 + (((4 + g) ^ kswz) << 4);
  const int vrow = 4 * g + (col >> 2), vswz = vrow & 7;
  int voff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
    voff[dt] = KB * D * 2 + vrow * 128 + (((2 * dt + ((col & 3) >> 1)) ^ vswz) << 4) + (col & 1) * 8;

  // scores + softmax of block blk -> P fragments (bf16) in pb
  auto scores = [&](int blk, auto tail_tag, s16x8 (&pb)[QT][2]) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    const char* S0 = reinterpret_cast<const char*>(smem + (blk % NBUF) * BLK);
    const int k0 = blk * KB;
    f32x4 st[QT][4];
    f32x4 cinit[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const float c = L2S && blk > 0 ? -m_run[t] : 0.f;
      cinit[t] = f32x4{c, c, c, c};
    }
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int t = 0; t < QT; ++t) st[t][kt] = cinit[t];
      if (!TAIL || k0 + kt * 16 < L) {
        const s16x8 k0f = *reinterpret_cast<const s16x8*>(S0 + kt * 16 * 128 + koff0);
        const s16x8 k1f = *reinterpret_cast<const s16x8*>(S0 + kt * 16 * 128 + koff1);
#pragma unroll
        for (int t = 0; t < QT; ++t) st[t][kt] = mfma_bf16(k1f, qf[t][1], mfma_bf16(k0f, qf[t][0], st[t][kt]));
      }
    }
    if constexpr (TAIL) {
#pragma unroll
      for (int t = 0; t < QT; ++t)
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (k0 + kt * 16 + 4 * g + r >= L) st[t][kt][r] = -INFINITY;
    }
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      float lm = fmaxf(fmaxf(st[t][0][0], st[t][0][1]), fmaxf(st[t][0][2], st[t][0][3]));
#pragma unroll
      for (int kt = 1; kt < 4; ++kt)
        lm = fmaxf(lm, fmaxf(fmaxf(st[t][kt][0], st[t][kt][1]), fmaxf(st[t][kt][2], st[t][kt][3])));
      if constexpr (L2S) {
        // st = S - m_run already (block 0: S, with m_run unset); rescale when a query's block max
        // passes the running max by more than THR (block 0: always, to seed it)
        if (blk == 0 || __any(lm > THR)) {
          const float d = blk == 0 ? xrow4_max(lm) : fmaxf(xrow4_max(lm), 0.f);
          if (blk > 0) {
            const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
            for (int i = 0; i < 4; ++i) o[t][i] *= alpha;
            osum[t] *= alpha;
            m_run[t] += d;
          } else {
            m_run[t] = d;
          }
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) st[t][kt] -= f32x4{d, d, d, d};
        }
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) st[t][kt][r] = __builtin_amdgcn_exp2f(st[t][kt][r]);
      } else {
      if (__any((lm - m_run[t]) * sl2 > THR)) {          // rare after the first block
        const float m_new = fmaxf(m_run[t], xrow4_max(lm));
        const float alpha = __builtin_amdgcn_exp2f((m_run[t] - m_new) * sl2);
        m_run[t] = m_new;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[t][i] *= alpha;
        osum[t] *= alpha;
      }
      const float nb = -m_run[t] * sl2;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[t][kt][r] = __builtin_amdgcn_exp2f(fmaf(st[t][kt][r], sl2, nb));
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        uint4 pu = make_uint4(f2bf2(st[t][2 * u][0], st[t][2 * u][1]), f2bf2(st[t][2 * u][2], st[t][2 * u][3]),
                              f2bf2(st[t][2 * u + 1][0], st[t][2 * u + 1][1]),
                              f2bf2(st[t][2 * u + 1][2], st[t][2 * u + 1][3]));
        pb[t][u] = *reinterpret_cast<s16x8*>(&pu);
      }
    }
  };
  // O += P V and the row sums over block blk
  auto pv = [&](int blk, auto tail_tag, const s16x8 (&pb)[QT][2]) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    const char* S0 = reinterpret_cast<const char*>(smem + (blk % NBUF) * BLK);
    const int k0 = blk * KB;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (TAIL && k0 + 32 * u >= L) continue;            // P = 0 on all 32 keys
      // the transposed reads go through inline asm: hipcc treats the ds_read_tr builtin as
      // aliasing the in-flight LDS-DMA and would drain every block in flight (vmcnt(0)) first;
      // their completion is waited for here explicitly (lgkmcnt(0), MFMAs fenced behind it)
      s16x4 lo[4], hi[4];
      const unsigned vb = (unsigned)(uintptr_t)(S0 + 32 * u * 128);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo[dt]) : "v"(vb + voff[dt]));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hi[dt]) : "v"(vb + voff[dt]));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const s16x8 va = s16x8{lo[dt][0], lo[dt][1], lo[dt][2], lo[dt][3], hi[dt][0], hi[dt][1], hi[dt][2], hi[dt][3]};
#pragma unroll
        for (int t = 0; t < QT; ++t) o[t][dt] = mfma_bf16(va, pb[t][u], o[t][dt]);
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) osum[t] = mfma_bf16(ones, pb[t][u], osum[t]);
    }
  };

  const int nblk = (L + KB - 1) / KB;
  const int nfull = L / KB;                              // blocks with every key < L
  s16x8 pb[QT][2];
#pragma unroll
  for (int b = 0; b <= AHEAD; ++b)
    if (b < nblk) issue(b);
  for (int blk = 0; blk < nblk; ++blk) {
    // this wave's pieces of blocks blk+1 .. min(blk+AHEAD, nblk-1) may stay in flight
    const int after = min(AHEAD, nblk - 1 - blk);
    if (after >= 2) wait_vmcnt<2 * NI>();
    else if (after == 1) wait_vmcnt<NI>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();                         // every wave's pieces of block blk landed;
    __builtin_amdgcn_sched_barrier(0);                    // every wave is done with block blk - 1
    if (blk + AHEAD + 1 < nblk) issue(blk + AHEAD + 1);   // into block blk - 1's slot
    if (live) {
      if (blk < nfull) {
        scores(blk, std::false_type{}, pb);
        pv(blk, std::false_type{}, pb);
      } else {
        scores(blk, std::true_type{}, pb);
        pv(blk, std::true_type{}, pb);
      }
    }
  }
  // 16-byte stores: per pair of 16-channel tiles (dt, dt + 1) the lane pair (g, g ^ 1) of a query
  // swaps halves so that each lane holds 8 consecutive channels (even g: 4g .. 4g+7 of tile dt, odd g:
  // 4(g-1) .. +7 of tile dt + 1); the swaps run on every lane, the stores only for queries < L
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int qi = q0 + 16 * t + col;
    const float inv = 1.f / osum[t][0];
    bf16* O = reinterpret_cast<bf16*>(p.out) + (row0 + (qi < L ? qi : 0)) * p.ldo + h * D;
#pragma unroll
    for (int dp = 0; dp < 2; ++dp) {
      const f32x4 a0 = o[t][2 * dp] * inv, a1 = o[t][2 * dp + 1] * inv;
      const uint2 y0 = make_uint2(f2bf2(a0[0], a0[1]), f2bf2(a0[2], a0[3]));
      const uint2 y1 = make_uint2(f2bf2(a1[0], a1[1]), f2bf2(a1[2], a1[3]));
      const uint2 give = (g & 1) ? y0 : y1;
      const uint2 got = make_uint2((unsigned)__shfl_xor((int)give.x, 16, 64), (unsigned)__shfl_xor((int)give.y, 16, 64));
      if (qi < L) {
        bf16* dst = O + 32 * dp + ((g & 1) ? 12 + 4 * g : 4 * g);
        const uint4 val = (g & 1) ? make_uint4(got.x, got.y, y1.x, y1.y) : make_uint4(y0.x, y0.y, got.x, got.y);
        if constexpr (WT) {   // sc1 write-through (attn_store knob)
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, 0x7fffffff, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, val), rs,
                                                 (int)((dst - reinterpret_cast<bf16*>(p.out)) * 2), 0, 16);
        } else {
          st16(dst, val);
        }
      }
    }
  }
}

int g_attn_store = 1;   // vit_attn3 output stores: 0 = plain, 1 = sc1 write-through (same box, whole step: 9.232 -> 9.175 ms)
CATSEG_KNOB(g_attn_store, "attn_store");
template <int NW, int QT, bool L2S = false>
void launch_vit3(const AttnP& p, hipStream_t st) {
  dim3 grid((unsigned)((p.L + 16 * NW * QT - 1) / (16 * NW * QT)), (unsigned)(p.n_seq * p.H));
  if (g_attn_store) hipLaunchKernelGGL((vit_attn3_kernel<NW, QT, L2S, true>), grid, dim3(NW * 64), 0, st, p);
  else hipLaunchKernelGGL((vit_attn3_kernel<NW, QT, L2S>), grid, dim3(NW * 64), 0, st, p);
}

template <typename T, int D, int NW, int KB, int QT, int GEO, bool SWM, bool CAUSAL>
void launch(const AttnP& p, hipStream_t st) {
  constexpr int QW = 16 * NW * QT;
  dim3 grid((unsigned)((p.L + QW - 1) / QW), (unsigned)(p.n_seq * p.H));
  hipLaunchKernelGGL((attn_kernel<T, D, NW, KB, QT, GEO, SWM, CAUSAL>), grid, dim3(NW * 64), 0, st, p);
}

template <typename T, int D, int NW, int KB, int QT, int GEO>
void launch_win(const AttnP& p, hipStream_t st) {
  if (p.shift > 0) launch<T, D, NW, KB, QT, GEO, true, false>(p, st);
  else launch<T, D, NW, KB, QT, GEO, false, false>(p, st);
}

int g_attn_tail_skip = 1;
int g_attn_variant = 0;   // dense path: 0 = default, 7 = the generic tiling (tests)

template <typename T, int D>
void launch_dense(const AttnP& p, hipStream_t st) {
  if (p.causal) { launch<T, D, 4, 64, 2, 0, false, true>(p, st); return; }
  if constexpr (sizeof(T) == 2 && D == 64) {
    // the ViT MHA kernel (LDS-DMA ring, 8 waves, XCD-remapped grid); attn_variant 7 forces the
    // generic tiling (the exact-max cross-check of the defer-max tests)
    if (g_attn_variant != 7) { launch_vit3<8, 1>(p, st); return; }
  }
  // generic tiling: 10 waves x 16 queries when that needs fewer query blocks than 8 x 16 (ViT
  // L = 577: 4 blocks of 160 vs 5 of 128 -> 512 workgroups, two per CU, no ragged third round)
  if ((p.L + 159) / 160 < (p.L + 127) / 128) launch<T, D, 10, 64, 1, 0, false, false>(p, st);
  else launch<T, D, 8, 64, 1, 0, false, false>(p, st);
}


template <typename T>
int dispatch(const AttnP& p, int head_dim, hipStream_t st) {
  if (p.mode == 2) {
    if constexpr (sizeof(T) != 2) return -1;
    if (head_dim != 64 || p.causal) return -1;
    // (measured and not kept: 10 waves x 16 queries, 512 workgroups in one round, 29.4 vs 27.4 us;
    // waves 4-7 half a block behind on a 5-slot ring, 29.3 vs 28.1 us; the block loop software-
    // pipelined one block deep -- block b+1's S MFMAs and softmax issued before block b's P.V, the
    // rescale deferred behind it -- on a 4- / 5-slot ring, 28.9 / 28.7 vs 26.9 us; 9 waves x 16
    // queries, so that 576 of the 577 queries fill four workgroups per (image, head): 27.0 vs 27.0 us)
    launch_vit3<8, 1, true>(p, st);
    return 0;
  }
  if (p.mode == 1) {
    if (head_dim == 32 && p.img_h == 24 && p.img_w == 24 && p.ws == 12) { launch_win<T, 32, 9, 160, 1, 24>(p, st); return 0; }
    if (head_dim == 32 && p.L <= 160) { launch_win<T, 32, 9, 160, 1, 0>(p, st); return 0; }
    if (head_dim == 32) { launch_win<T, 32, 4, 64, 2, 0>(p, st); return 0; }
  } else {
    if (head_dim == 64) { launch_dense<T, 64>(p, st); return 0; }
    if (head_dim == 32) { launch_dense<T, 32>(p, st); return 0; }
  }
  return -1;
}

}  // namespace

CATSEG_KNOB(g_attn_variant, "attn_variant");
CATSEG_KNOB(g_attn_tail_skip, "attn_tail_skip");

extern "C" int catseg_attention(const CatsegAttnArgs* a, void* stream) {
  CATSEG_CHECK(a && a->q && a->k && a->v && a->out, "attention: null pointer");
  CATSEG_CHECK(a->n_seq > 0 && a->seq_len > 0 && a->n_heads > 0, "attention: empty shape");
  const int vn = a->dtype == CATSEG_BF16 ? 8 : 4;
  CATSEG_CHECK(a->ld_qkv % vn == 0 && a->ld_out % 4 == 0, "attention: row strides must allow 16B loads");
  CATSEG_CHECK(((uintptr_t)a->q % 16) == 0 && ((uintptr_t)a->k % 16) == 0 && ((uintptr_t)a->v % 16) == 0,
               "attention: q/k/v must be 16B aligned");
  AttnP p;
  p.q = a->q; p.k = a->k; p.v = a->v; p.ld = a->ld_qkv; p.out = a->out; p.ldo = a->ld_out;
  p.n_seq = a->n_seq; p.L = a->seq_len; p.H = a->n_heads; p.scale = a->scale; p.causal = a->causal;
  p.skip_tail = g_attn_tail_skip;
  p.mode = a->mode; p.img_h = a->img_h; p.img_w = a->img_w; p.ws = a->window; p.shift = a->shift;
  if (a->mode == 1) {
    CATSEG_CHECK(a->window > 0 && a->img_h % a->window == 0 && a->img_w % a->window == 0,
                 "attention: image must tile into windows");
    CATSEG_CHECK(a->seq_len == a->window * a->window, "attention: seq_len must be window^2");
    CATSEG_CHECK(a->shift >= 0 && a->shift < a->window, "attention: bad shift");
    CATSEG_CHECK(!a->causal, "attention: causal not supported for windows");
  } else if (a->mode == 2) {
    CATSEG_CHECK(a->dtype == CATSEG_BF16 && a->head_dim == 64 && !a->causal,
                 "attention: mode 2 (log2-scaled q) is bf16, head_dim 64, non-causal");
  } else {
    CATSEG_CHECK(a->mode == 0, "attention: bad mode");
  }
  hipStream_t st = (hipStream_t)stream;
  int rc = a->dtype == CATSEG_BF16 ? dispatch<bf16>(p, a->head_dim, st)
                                   : dispatch<float>(p, a->head_dim, st);
  CATSEG_CHECK(rc == 0, "attention: unsupported head_dim/mode combination");
  return catseg_launch_status("attention");
}
