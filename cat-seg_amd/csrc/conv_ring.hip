// bf16 3x3 / pad-1 convolution with a sliding ring of input rows in LDS and the weights
// in registers (decoder convs of the guided upsampler, reference model.py:528-533
// DoubleConv inside Up, :540-555).
//
// A workgroup walks a band of consecutive 128-pixel chunks of one NHWC slice.  The
// input rows live in an NR-row LDS ring (row y in slot (y + 1) % NR, one zero halo column
// each side, rows outside the image zero) and each pixel is loaded from HBM ONCE per band:
// while the MFMAs of chunk c run, the CH pixels chunk c+1 adds (the linear pixel stream
// one row + one pixel ahead of it) are already in flight in registers (global -> VGPR), and
// are written into the slots chunk c+1 no longer needs after the chunk's MFMAs.  Channels [0, c1) come from the per-slice tensor
// (GroupNorm+ReLU'd on the way in when the conv consumes relu(GN(x))), [c1, C) from the
// per-image guidance tensor (the concat + repeat of Up.forward, model.py:551-554, never
// materialised).  An optional fp32 per-image addend (the guidance half of the conv,
// computed once per image by catseg_conv3x3_partial) joins in the epilogue instead.
//
// Ring layout: pixel-major with a pixel stride PS of C*2 rounded up to 32 (mod 64) bytes.
// With that stride the 16 pixels x 4 k-chunks of a ds_read_b128 fragment read fall in 16
// distinct 16-byte bank slots in every lane group (checked exhaustively for the gfx950
// b128 lane grouping), and every fragment address is one per-(pixel tile, row) base plus a
// compile-time offset (dx * PS + k), so the tap loop issues LDS reads with immediate
// offsets and no per-read VALU (the XOR-swizzled image this replaces spent ~7 VALU per
// read and still measured 25-35 % SQ_LDS_BANK_CONFLICT).
//
// Each wave keeps ITS slice of the weights for all 9 taps as MFMA A fragments in
// registers for the life of the workgroup (WCO waves split COUT, WPX split the chunk's
// pixels), so the LDS traffic is the pixel fragments only.  D = W_tap . X_tap^T; C need
// not be a multiple of 32: the trailing 16 channels of two taps share one K=32 step.  The
// epilogue adds bias / addend, applies the activation, emits the per-(128-pixel tile,
// group) GroupNorm mean / M2 partials in the layout of conv.hip, and stores bf16 rows.
#include "common.h"
#include "capi.h"

#define DEV_HOST_CONST __host__ __device__ constexpr

namespace {

constexpr int NT = 256;          // 4 waves
int g_ring_onebar = 1;           // 1 = the one-barrier-per-chunk rings (OB) where instantiated (default: bit-identical,
                                 // Up1 fold 365 -> 347 us, the other three decoder convs within 1 %), 0 = two barriers
int g_ring_persist = 2;          // persistent workgroups over (slice, band) units: 2 = >= 4 units each (bands by that), 1 = one-unit band rule, 0 = one unit per workgroup

struct RingP {
  const bf16* s1; int64_t s1_ss; int c1;
  const bf16* s2; int64_t s2_ss; int c2; int64_t s2_div;
  int64_t S; int H; int W; int chunks_per_band; int bands;
  const bf16* w; const float* bias; int act;
  const float* gmean; const float* grstd; const float* ggamma; const float* gbeta; int gcpg;
  const float* add; int64_t add_ss; int64_t add_div;
  bf16* out; float* stats;
  int up_split;   // UP: output channels of a parity split over this many workgroups (1, 2 or 4)
  int wt;         // output pixels through sc1 write-through stores (ring_store knob)
};

template <int C>
struct RingGeom {
  static_assert(C % 16 == 0, "channels in 16-channel steps");
  static constexpr int PSB = (C * 2) % 64 == 32 ? C * 2 : C * 2 + 32;   // pixel stride, bytes
  static constexpr int PS = PSB / 2;                                     // ... elements
  // ring row pitch = (W + 2) pixels + RPAD: a 16-pixel fragment that wraps from column W-1 of one
  // row to column 0 of the next skips the two halo columns; the pad makes that step -2 pixel
  // strides mod 256 bytes, so the wrapped lanes land on the banks of a contiguous run (W = 24:
  // 1/3 more LDS cycles per fragment read without it; widths that are multiples of 16 never wrap)
  static constexpr int RPADB = (256 - (2 * PSB) % 256) % 256;
  static DEV_HOST_CONST int pitch(int W) { return (W + 2) * PS + RPADB / 2; }   // elements
};


// OCC: waves per SIMD the register budget is sized for (2 = 256 VGPRs; 1 = 512 with AGPRs,
// for the 96-channel variant whose 108 weight VGPRs leave no room at 2)
// NR: ring rows = rows a chunk can span + 2 halo rows (CH = 128: 4 + 2 at W >= 48, 3 + 2 at
// W >= 64; CH = 64: 3 + 2 at W >= 48)
// UP: the 4-parity form of ConvTranspose2d(k=2, s=2) followed by this conv (catseg_upconv3x3):
// the source grid is the ConvTranspose INPUT, wave wco computes output parity
// (a, b) = (wco >> 1, wco & 1) with its 2x2 of the 9 taps (rows a, a+1; columns b, b+1), and
// channel block wco of COUT lands at pixel (2y + a, 2x + b) of the 2H x 2W output map.
// WFIX > 0: the map width as a compile-time constant (UP variants; the per-pixel row / column
// divisions become multiplies), 0 = p.W
// OB: one barrier per chunk -- the rows chunk c+1 adds are written into the ring right after chunk
// c's epilogue, before the end-of-chunk barrier, into slots chunk c does not read; needs NR >= the
// rows a chunk spans + the rows the next one adds (the two-barrier form writes them after a barrier
// that retires chunk c's reads, so NR only has to cover one chunk + its additions in sequence)
template <int C, int COUT, int WPX, int WCO, int NPOS, int CH, int OCC, int NR, bool ADD, bool UP = false, int WFIX = 0,
          bool OB = false>
__global__ __launch_bounds__(NT, OCC) void conv_ring_kernel(RingP p) {
  constexpr int CPX = C / 8;
  constexpr int PS = RingGeom<C>::PS;
  constexpr int PXW = CH / WPX, FM = PXW / 16;          // pixels per wave, their 16-px tiles
  constexpr int COW = COUT / WCO, FN = COW / 16;        // output channels per wave
  constexpr int KC = C / 32;                            // full MFMA k-steps per tap
  constexpr bool KT = (C % 32) == 16;                   // trailing 16 channels per tap
  constexpr int NTP = KT ? 5 : 0;                       // tap pairs (0,1) (2,3) (4,5) (6,7) (8,-)
  static_assert(WPX * WCO == 4 && FM >= 1 && FN >= 1, "wave grid");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* ring = reinterpret_cast<bf16*>(smem);
  const int W = WFIX > 0 ? WFIX : p.W, WP = W + 2, H = p.H;
  const int RPE = RingGeom<C>::pitch(W);                  // ring row pitch, elements
  const int ring_elems = NR * RPE;
  float* gsc = reinterpret_cast<float*>(smem + (size_t)ring_elems * 2);   // [C]
  float* gsh = gsc + C;                                                    // [C]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int wpx = wave % WPX, wco = wave / WPX;
  // UP with up_split > 1: workgroup `half` computes channel block half of every parity
  // (COW of the CO = COW * up_split channels per parity); the source ring is read per block
  // Persistent over units (slice, band): workgroup g keeps channel block half = g % nsplit (its
  // weights stay in registers) and walks units g / nsplit, + gridDim.x / nsplit, ...
  const int nsplit = UP ? p.up_split : 1;
  const int half = UP ? (int)(blockIdx.x % nsplit) : 0;
  const int64_t nunits = p.S * p.bands, ustride = gridDim.x / nsplit;
  const int CO = COW * nsplit;                          // UP: channels per parity in the output map
  const int ch0 = wco * CO + half * COW;                // first weight row / addend channel of this wave
  const int HW = H * W;
  const int nchunks = HW / CH;

  // ---- weights of this wave's output channels, all taps, in registers ----
  // The trailing 16 channels of two taps share one K=32 step: lanes q < 2 carry tap 2p's
  // channels KC*32 + 8q.., lanes q >= 2 tap 2p+1's (zero weights past tap 8) -- the k order
  // inside an MFMA step is free as long as A and B agree.
  static_assert(!UP || (WPX == 1 && WCO == 4 && !KT), "UP: one output parity per wave, C % 32 == 0");
  constexpr int NTAP = UP ? 4 : 9;
  const int pa = UP ? (wco >> 1) : 0, pb = UP ? (wco & 1) : 0;     // UP: this wave's output parity
  s16x8 wf[NTAP][KC > 0 ? KC : 1][FN];
  s16x8 wt[NTP > 0 ? NTP : 1][FN];
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = ch0 + 16 * i + r16;
#pragma unroll
    for (int t = 0; t < NTAP; ++t) {
      const int tap = UP ? (pa + t / 2) * 3 + pb + t % 2 : t;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        uint4 u = ld16(p.w + ((int64_t)n * 9 + tap) * C + kc * 32 + 8 * q);
        wf[t][kc][i] = *reinterpret_cast<s16x8*>(&u);
      }
    }
#pragma unroll
    for (int tp = 0; tp < NTP; ++tp) {
      const int tap = 2 * tp + (q >> 1);
      uint4 u = make_uint4(0, 0, 0, 0);
      if (tap < 9) u = ld16(p.w + ((int64_t)n * 9 + tap) * C + KC * 32 + 8 * (q & 1));
      wt[tp][i] = *reinterpret_cast<s16x8*>(&u);
    }
  }
  float bv[FN][4];                      // bias of this lane's output channels (0 without)
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[i][r] = p.bias ? p.bias[ch0 + 16 * i + 4 * q + r] : 0.f;

  // ---- the halo columns (ring columns 0 and W + 1) of every slot are zeroed once: the pixel
  // loads below never write them ----
  for (int i = tid; i < NR * 2 * CPX; i += NT) {
    const int slot = i / (2 * CPX), side = (i / CPX) & 1;
    st16(&ring[slot * RPE + (side ? W + 1 : 0) * PS + (i % CPX) * 8], make_uint4(0, 0, 0, 0));
  }
  // Ring loads are PIXEL-granular: the image is one linear pixel stream P = y * W + x (row -1 and
  // rows >= H read as zeros), and the ring holds pixels [.., lp) of it.  Chunk c needs pixels up to
  // the bottom-right neighbour of its last pixel, p0 + CH + W (exclusive end p0 + CH + W + 1), so
  // each chunk adds exactly CH pixels = CH * CPX 16-byte items, MAXPF per thread, with no idle
  // passes for partial rows and no halo writes.  (When a chunk ends at a row end the last of
  // those pixels is column 0 of the row after the bottom halo row; its slot cannot alias a row in
  // use -- that case spans one row less than the worst case the NR of each variant is sized
  // for, ring_plan_ok() checks every launch.)
  constexpr int MAXPF = CH * CPX / NT;
  static_assert(MAXPF * NT == CH * CPX, "a chunk's pixels fill whole passes of the workgroup");
  // ring-write item order: with 4 chunks per pixel (C = 32, 96-byte pixel stride) the 8 lanes of a
  // ds_write_b128 group would write pixels p, p+1 and hit 8 banks twice; swapping bits 2 and 3 of
  // the item index gives them pixels p, p+2 (distinct 16-byte bank slots), a bijection on every
  // aligned block of 16 items
  auto perm = [](int i) { return CPX == 4 ? (i & ~12) | ((i & 4) << 1) | ((i & 8) >> 1) : i; };
  // per-thread prefetch items, decoded once: (pixel offset << 8) | 16-byte channel chunk
  int pf_code[MAXPF];
#pragma unroll
  for (int k = 0; k < MAXPF; ++k) {
    const int i = perm(tid + k * NT);
    pf_code[k] = ((i / CPX) << 8) | (i % CPX);
  }
  // ring element offset of pixel P (P >= -W), channel chunk ch
  auto ring_at = [&](int P, int ch) {
    const unsigned y1 = (unsigned)(P + W) / (unsigned)W;           // y + 1 >= 0
    const int x = P + W - (int)y1 * W;
    return (int)(y1 % NR) * RPE + (x + 1) * PS + ch * 8;
  };

  for (int64_t unit = blockIdx.x / nsplit; unit < nunits; unit += ustride) {
  const int64_t s = unit / p.bands;
  const int band = (int)(unit % p.bands);
  const int c_begin = band * p.chunks_per_band;
  const int c_end = min(nchunks, c_begin + p.chunks_per_band);
  if (c_begin >= c_end) continue;       // uniform over the workgroup
  // (the previous unit ended on a barrier after its last ring reads / GN-table reads)
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
  const bool gn = p.gmean != nullptr;

  // 16-byte item (pixel P, channel chunk ch) from HBM: the address of pixel P when it is in the
  // image, else of pixel 0 (the caller zero-selects)
  auto gsrc = [&](int P, int ch) -> const bf16* {
    const int ci = ch * 8;
    return ci < p.c1 ? s1base + (int64_t)__umul24(P, p.c1) + ci : s2base + (int64_t)__umul24(P, p.c2) + (ci - p.c1);
  };
  // write an item into the ring, GroupNorm+ReLU'd when it is an in-image s1 channel chunk
  // (ReLU on the rounded bf16 pair as a signed 16-bit max with 0: the same bits as rounding the
  // ReLU'd float)
  auto lput = [&](int P, int ch, bool in_image, uint4 u) {
    const int ci = ch * 8;
    if (gn && in_image && ci < p.c1) {
      const float4 a0 = *reinterpret_cast<const float4*>(gsc + ci), a1 = *reinterpret_cast<const float4*>(gsc + ci + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(gsh + ci), b1 = *reinterpret_cast<const float4*>(gsh + ci + 4);
      const float sc[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float sh[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = __uint_as_float(w[e] << 16), hi = __uint_as_float(w[e] & 0xffff0000u);
        const unsigned r = f2bf2(fmaf(lo, sc[2 * e], sh[2 * e]), fmaf(hi, sc[2 * e + 1], sh[2 * e + 1]));
        w[e] = relu_bf16x2(r);
      }
      u = make_uint4(w[0], w[1], w[2], w[3]);
    }
    st16(&ring[ring_at(P, ch)], in_image ? u : make_uint4(0, 0, 0, 0));
  };

  // ---- prime: from the top halo row of the first chunk to its bottom-right neighbour ----
  __syncthreads();   // gsc/gsh (and, first unit, the halo columns)
  int lp;            // pixels [.., lp) are in the ring
  {
    const int p0 = c_begin * CH;
    const int pa = (p0 / W - 1) * W, pe = p0 + CH + W + 1;
    const int total = (pe - pa) * CPX;
    for (int i0 = 0; i0 < total; i0 += NT * 8) {
      uint4 u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = perm(i0 + j * NT + tid);
        const int P = pa + i / CPX;
        u[j] = i < total && P >= 0 && P < HW ? ld16(gsrc(P, i % CPX)) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = perm(i0 + j * NT + tid);
        const int P = pa + i / CPX;
        if (i < total) lput(P, i % CPX, P >= 0 && P < HW, u[j]);
      }
    }
    lp = pe;
  }
  // the ring row / column of each of this wave's pixel tiles (pixel p0 + wpx * PXW + 16 j + r16),
  // advanced by CH pixels per chunk: slot of the row above (y - 1 + 1) % NR and column x
  int srow[FM], pcol[FM];
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int pp = c_begin * CH + wpx * PXW + 16 * j + r16;
    srow[j] = (pp / W) % NR;
    pcol[j] = pp % W;
  }
  __syncthreads();

  for (int c = c_begin; c < c_end; ++c) {
    const int p0 = c * CH;
    // the per-image addend of this chunk (L2-resident) first, so that waiting for it does
    // not also wait for the row prefetch issued after it (vmcnt retires in issue order)
    // LATE_ADD (the 512-register UP variant): the addend is read in the epilogue instead, so its
    // 4 x FN x FM registers are not live across the MFMAs
    constexpr bool LATE_ADD = UP && ((C >= 128 && OCC > 1) || CH >= 128);
    const float* addb = ADD ? p.add + (s / p.add_div) * p.add_ss + (int64_t)(p0 + wpx * PXW) * COUT * nsplit + ch0 : nullptr;
    float4 ad[FN][FM];
    if constexpr (ADD && !LATE_ADD) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          ad[i][j] = *reinterpret_cast<const float4*>(addb + (16 * j + r16) * COUT * nsplit + 16 * i + 4 * q);
    }
    if constexpr (ADD) __builtin_amdgcn_sched_barrier(0);     // (the addend loads issue before the prefetch loads)
    // ---- prefetch the CH pixels the next chunk adds, [lp, lp + CH): unconditional loads from
    // clamped addresses (zero-selected at the ring write), so the code is straight-line and every
    // wait is an exact vmcnt count ----
    uint4 pf[MAXPF];
#pragma unroll
    for (int k = 0; k < MAXPF; ++k) {
      const int P = lp + (pf_code[k] >> 8);
      pf[k] = ld16(gsrc(P < HW ? P : 0, pf_code[k] & 255));
    }
    // with an addend, its loads and the prefetch loads stay ahead of the MFMAs (left to itself the
    // scheduler sinks them below the tap loop, and the epilogue then waits out their full latency;
    // without one, sinking the prefetch measured faster: 48-wide 64-channel conv 312 -> 272 us)
    if constexpr (ADD) __builtin_amdgcn_sched_barrier(0);

    // ---- MFMAs: 9 taps x (KC + tail) k-steps over the ring ----
    auto wrap = [](int r) { return r >= NR ? r - NR : r; };
    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (UP) {
      // taps (pa + sy, pb + sx): ring row y + pa + sy - 1, column x + pb + sx - 1
      int rbu[2][FM];
#pragma unroll
      for (int sy = 0; sy < 2; ++sy)
#pragma unroll
        for (int j = 0; j < FM; ++j) rbu[sy][j] = wrap(srow[j] + pa + sy) * RPE + (pcol[j] + pb) * PS;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          s16x8 xf[FM];
#pragma unroll
          for (int j = 0; j < FM; ++j)
            xf[j] = *reinterpret_cast<const s16x8*>(ring + rbu[t / 2][j] + 8 * q + (t % 2) * PS + kc * 32);
#pragma unroll
          for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(wf[t][kc][i], xf[j], acc[i][j]);
        }
      }
    }
    int rb[3][FM];                            // pixel (row y+dy-1, column x-1) of each tile row
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int j = 0; j < FM; ++j) rb[dy][j] = wrap(srow[j] + dy) * RPE + pcol[j] * PS;
#pragma unroll
    for (int dy = 0; dy < (UP ? 0 : 3); ++dy) {
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int tap = dy * 3 + dx;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          s16x8 xf[FM];
#pragma unroll
          for (int j = 0; j < FM; ++j) xf[j] = *reinterpret_cast<const s16x8*>(ring + rb[dy][j] + 8 * q + dx * PS + kc * 32);
#pragma unroll
          for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(wf[UP ? 0 : tap][kc][i], xf[j], acc[i][j]);
        }
      }
    }
#pragma unroll
    for (int tp = 0; tp < NTP; ++tp) {
      // lanes q < 2: tap 2tp, q >= 2: tap 2tp+1 (tap 9 reads tap 8's pixels against zero weights)
      const int ta = 2 * tp, tb = 2 * tp + 1 < 9 ? 2 * tp + 1 : 8;
      const bool hi = q >= 2;
      s16x8 xf[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int a0 = rb[ta / 3][j] + (ta % 3) * PS, b0 = rb[tb / 3][j] + (tb % 3) * PS;
        xf[j] = *reinterpret_cast<const s16x8*>(ring + (hi ? b0 : a0) + KC * 32 + 8 * (q & 1));
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(wt[tp][i], xf[j], acc[i][j]);
    }

    // ---- epilogue: bias / addend / act, GroupNorm partials, bf16 stores ----
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        float adv[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (ADD) {
          const float4 av = LATE_ADD ? *reinterpret_cast<const float4*>(addb + (16 * j + r16) * COUT * nsplit + 16 * i + 4 * q)
                                     : ad[i][j];
          adv[0] = av.x; adv[1] = av.y; adv[2] = av.z; adv[3] = av.w;
        }
#pragma unroll
        // (acc + addend) + bias: no addend-only subexpression the scheduler could hoist above the
        // tap loop (it would wait there for the addend loads)
        for (int r = 0; r < 4; ++r) acc[i][j][r] = (ADD ? acc[i][j][r] + adv[r] : acc[i][j][r]) + bv[i][r];
        if (p.act != ACT_NONE)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = apply_act(acc[i][j][r], p.act);
      }
    if (p.stats) {
      // GroupNorm partials per (wave pixel block = PXW pixels, group of 16 channels = one
      // n-tile): mean and M2 of the wave's own accumulators, no cross-wave reduction
      const int ntiles = HW / PXW, tile = c * WPX + wpx;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < FM; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) a += acc[i][j][r];
        const float gm = wave_sum(a) * (1.f / (PXW * 16));
        float m2 = 0.f;
#pragma unroll
        for (int j = 0; j < FM; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) { const float d = acc[i][j][r] - gm; m2 += d * d; }
        m2 = wave_sum(m2);
        if (lane == 0) {
          const int grp = ch0 / 16 + i;
          float* o = p.stats + (((int64_t)s * ntiles + tile) * (COUT * nsplit / 16) + grp) * 2;
          o[0] = gm;
          o[1] = m2;
        }
      }
    }
    // bf16 stores of a pixel's 16 n-tile channels: with two n-tiles (32 channels of the pixel per
    // wave) the lane pair (q, q ^ 1) swaps halves so that each lane holds 8 consecutive channels
    // (even q: 4q .. 4q+7, odd q: 16 + 4(q-1) .. +7) and writes them as one 16-byte store -- the
    // pixel's 64 bytes in one instruction instead of two 32-byte pieces
    auto store_px = [&](bf16* ob, int j) {
      if constexpr (FN == 2) {
        const uint2 y0 = make_uint2(f2bf2(acc[0][j][0], acc[0][j][1]), f2bf2(acc[0][j][2], acc[0][j][3]));
        const uint2 y1 = make_uint2(f2bf2(acc[1][j][0], acc[1][j][1]), f2bf2(acc[1][j][2], acc[1][j][3]));
        const uint2 give = (q & 1) ? y0 : y1;
        const uint2 got = make_uint2((unsigned)__shfl_xor((int)give.x, 16, 64), (unsigned)__shfl_xor((int)give.y, 16, 64));
        bf16* dst = ob + ((q & 1) ? 12 + 4 * q : 4 * q);
        const uint4 val = (q & 1) ? make_uint4(got.x, got.y, y1.x, y1.y) : make_uint4(y0.x, y0.y, got.x, got.y);
        if (p.wt) st16_wt(p.out, (dst - p.out) * 2, val);
        else st16(dst, val);
      } else {
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          bf16* dst = ob + 16 * i + 4 * q;
          const uint2 val = make_uint2(f2bf2(acc[i][j][0], acc[i][j][1]), f2bf2(acc[i][j][2], acc[i][j][3]));
          if (p.wt) st8_wt(p.out, (dst - p.out) * 2, val);
          else *reinterpret_cast<uint2*>(dst) = val;
        }
      }
    };
    if constexpr (UP) {
      // parity (pa, pb) of source pixel (y, x) -> pixel (2y + pa, 2x + pb) of the 2H x 2W map, COW channels
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int pp = p0 + 16 * j + r16, yy = pp / W, xx = pp - yy * W;
        store_px(p.out + ((int64_t)s * 4 * HW + (2 * yy + pa) * (2 * W) + 2 * xx + pb) * CO + half * COW, j);
      }
    } else {
      bf16* ob = p.out + ((int64_t)s * HW + p0 + wpx * PXW) * COUT + wco * COW;
#pragma unroll
      for (int j = 0; j < FM; ++j) store_px(ob + (int64_t)(16 * j + r16) * COUT, j);
    }

    // ---- the prefetched pixels into the ring (slots the next chunk's rows own), and the pixel
    // tiles one chunk on ----
    if constexpr (!OB) __syncthreads();
    if (c + 1 < c_end) {
#pragma unroll
      for (int k = 0; k < MAXPF; ++k) {
        const int P = lp + (pf_code[k] >> 8);
        lput(P, pf_code[k] & 255, P < HW, pf[k]);
      }
    }
    lp += CH;
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      pcol[j] += CH % W;
      srow[j] += CH / W;
      if (pcol[j] >= W) { pcol[j] -= W; srow[j] += 1; }
      srow[j] = wrap(srow[j]);
    }
    __syncthreads();
  }
  }   // units
}

// The pixel-granular ring plan on an H x W map with CH-pixel chunks and NR slots: for every chunk
// (any chunk may start a band), the band prime's rows fit the ring, and the rows chunk c's prefetch
// writes never share a slot with a row a chunk still reads (OB: chunk c's own rows, which other
// waves may still be reading; two-barrier: chunk c+1's).
static bool ring_plan_ok(int H, int W, int CH, int NR, bool OB) {
  const int nchunks = H * W / CH;
  for (int c = 0; c < nchunks; ++c) {
    const int p0 = c * CH;
    const int first = p0 / W - 1;                         // top halo row of chunk c
    const int prime_last = (p0 + CH + W) / W;             // row of the prime's last pixel
    if (prime_last - first + 1 > NR) return false;
    if (c + 1 == nchunks) break;
    const int wr_last = (p0 + 2 * CH + W) / W;            // row of the prefetch's last pixel
    const int oldest = OB ? first : (p0 + CH) / W - 1;    // oldest row still read
    if (wr_last - oldest + 1 > NR) return false;
  }
  return true;
}

template <int C>
size_t ring_lds(int W, int NR) { return (size_t)NR * RingGeom<C>::pitch(W) * 2 + 2 * C * 4; }

// NPOS: the ring positions one chunk added under round 4's row-granular loads (W + 2 columns per
// new row: 156 / 198 for CH = 128 at W = 48 / 96, 104 for CH = 64 at W = 48); with pixel-granular
// loads it no longer sizes anything and only names the width class of a variant (launch_ring).
template <int C, int COUT, int WPX, int WCO, int NPOS, int CH, int OCC, int NR, bool ADD, bool UP = false, int WFIX = 0,
          bool OB = false>
int launch_ring_t(const RingP& p0, hipStream_t st) {
  RingP p = p0;
  const int nchunks = p.H * p.W / CH;
  // bands of ~3072 pixels on narrow maps, ~6144 on wide ones (a band re-primes its ring once:
  // the measured sweep, tools/micro_ring.py, favours longer bands at W = 96), at least 2
  // workgroups per CU
  const int base = p.W >= 64 ? 6144 : 3072;
  const int per_band = base / CH;
  int bands = (nchunks + per_band - 1) / per_band;
  const size_t sh = ring_lds<C>(p.W, NR);
  const int nsplit = UP ? p.up_split : 1;
  // persistent grid: the workgroups that fit at once (OCC per CU, LDS permitting), a multiple of
  // nsplit; g_ring_persist 0 = one unit per workgroup (A/B)
  const int per_cu = std::max(1, std::min(OCC, (int)((160 * 1024) / std::max<size_t>(sh, 1))));
  const int64_t cap = (int64_t)(catseg_device_cus() * per_cu / nsplit) * nsplit;
  // enough units for every workgroup: >= 2048 workgroups when each takes one unit, >= 4 units
  // per workgroup when persistent (ring_persist 2; 1 keeps the one-unit band rule)
  const int64_t want = g_ring_persist == 2 ? 4 * cap / nsplit : 2048;
  while (p.S * bands < want && bands * 4 <= nchunks) bands *= 2;
  p.bands = bands;
  p.chunks_per_band = (nchunks + bands - 1) / bands;
  static size_t configured = 0;
  if (sh > configured) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_ring_kernel<C, COUT, WPX, WCO, NPOS, CH, OCC, NR, ADD, UP, WFIX, OB>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    configured = sh;
  }
  if (nsplit < 1 || nsplit > 4 || (COUT / WCO) % 16 != 0 || ((int64_t)p.H * p.W) % CH != 0 || (WFIX > 0 && p.W != WFIX)) {
    catseg_set_error("conv ring: bad channel split %d or H*W %% %d != 0", nsplit, CH);
    return -1;
  }
  if (!ring_plan_ok(p.H, p.W, CH, NR, OB)) {
    catseg_set_error("conv ring: %d ring slots do not cover %d-pixel chunks on a %d-wide map", NR, CH, p.W);
    return -1;
  }
  int64_t grid = p.S * bands * nsplit;
  if (g_ring_persist) grid = std::min(grid, cap);
  hipLaunchKernelGGL((conv_ring_kernel<C, COUT, WPX, WCO, NPOS, CH, OCC, NR, ADD, UP, WFIX, OB>), dim3((unsigned)grid),
                     dim3(NT), sh, st, p);
  return 0;
}

// the CAT-Seg decoder widths (48, 96) get a compile-time width; others run with p.W
template <int C, int COUT, int WPX, int WCO, int NPOS, int CH = 128, int OCC = 2, int NR = 6, bool OB = false>
int launch_ring(const RingP& p0, hipStream_t st) {
  constexpr int WF = NPOS > 160 ? 96 : 48;      // the width class a variant is sized for
  if (p0.W == WF) {
    if (p0.add) return launch_ring_t<C, COUT, WPX, WCO, NPOS, CH, OCC, NR, true, false, WF, OB>(p0, st);
    return launch_ring_t<C, COUT, WPX, WCO, NPOS, CH, OCC, NR, false, false, WF, OB>(p0, st);
  }
  if constexpr (OB) {
    return 1;                                   // the one-barrier rings are sized for their width class only
  } else {
    if (p0.add) return launch_ring_t<C, COUT, WPX, WCO, NPOS, CH, OCC, NR, true>(p0, st);
    return launch_ring_t<C, COUT, WPX, WCO, NPOS, CH, OCC, NR, false>(p0, st);
  }
}

// ---- per-image partial conv (fp32 out): the guidance half of a conv over [x | g] ----
// out[b][pix][co] = sum_{tap, ci} w[co][tap][ci] * g[b][pix + tap][ci]  (zero padded),
// one thread per (pixel, 4 output channels); weights staged in LDS as [tap][ci][co].
template <typename T>
__global__ __launch_bounds__(256) void conv_partial_kernel(const T* __restrict__ g, int64_t B, int H, int W, int cin,
                                                           const float* __restrict__ w, int cout, float* out) {
  extern __shared__ float sw[];        // [9][cin][cout]
  for (int i = threadIdx.x; i < 9 * cin * cout; i += blockDim.x) {
    const int co = i % cout, ci = (i / cout) % cin, tap = i / (cout * cin);
    sw[i] = w[((int64_t)co * 9 + tap) * cin + ci];
  }
  __syncthreads();
  const int groups = cout / 4;
  const int64_t total = B * H * W * groups;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
    const int cg = (int)(idx % groups);
    const int64_t pixg = idx / groups;
    const int64_t b = pixg / (H * W);
    const int pix = (int)(pixg % (H * W));
    const int y = pix / W, x = pix % W;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int tap = 0; tap < 9; ++tap) {
      const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      const T* src = g + ((b * H + yy) * W + xx) * cin;
      const float* wt = sw + tap * cin * cout + cg * 4;
      for (int ci = 0; ci < cin; ++ci) {
        const float v = to_f<T>(src[ci]);
        const float4 ww = *reinterpret_cast<const float4*>(wt + ci * cout);
        a0 += v * ww.x; a1 += v * ww.y; a2 += v * ww.z; a3 += v * ww.w;
      }
    }
    *reinterpret_cast<float4*>(out + pixg * cout + cg * 4) = make_float4(a0, a1, a2, a3);
  }
}

// bf16 guidance with CIN % 8 == 0 channels: the same sum, the pixel's channels of a tap read
// as 16-byte vectors (the scalar 2-byte loads above issue one VMEM instruction per FMA group
// and bound the kernel at ~10 TF/s); weights stay fp32 in LDS, summation order tap-major as above
// PAR (catseg_upconv_addend): also + tap_bias[tap][co] for every in-image tap, and the output in
// the parity layout of catseg_upconv3x3's addend: [b][(y/2)*(W/2) + x/2][((y%2)*2 + x%2)*cout + co]
template <int CIN, bool PAR = false>
__global__ __launch_bounds__(256) void conv_partial_vec_kernel(const bf16* __restrict__ g, int64_t B, int H, int W,
                                                              const float* __restrict__ w, int cout, float* out,
                                                              const float* __restrict__ tap_bias = nullptr) {
  extern __shared__ float sw[];        // [9][CIN][cout + 4] (+ PAR: [9][cout] tap bias)
  // Transposing staging: 32 lanes = 8 consecutive ci (32 contiguous global bytes) x 4 co, so a
  // wave-load touches 8 cache lines (indexing in LDS order made each lane touch its own line),
  // and the LDS row stride cout + 4 puts those 32 lanes on 32 distinct banks (4 ci + co mod 32)
  const int ldw = cout + 4;
  static_assert(CIN % 8 == 0, "CIN");
  for (int i = threadIdx.x; i < 9 * CIN * cout; i += blockDim.x) {
    const int lo = i & 31, rest = i >> 5;
    const int ci_lo = lo & 7, co_lo = lo >> 3;
    const int cib = rest % (CIN / 8), rest2 = rest / (CIN / 8);
    const int tap = rest2 % 9, co = (rest2 / 9) * 4 + co_lo, ci = cib * 8 + ci_lo;
    sw[(tap * CIN + ci) * ldw + co] = w[((int64_t)co * 9 + tap) * CIN + ci];
  }
  float* stb = sw + 9 * CIN * ldw;
  if constexpr (PAR)
    for (int i = threadIdx.x; i < 9 * cout; i += blockDim.x) stb[i] = tap_bias ? tap_bias[i] : 0.f;
  __syncthreads();
  const int groups = cout / 4;
  const int64_t total = B * H * W * groups;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
    const int cg = (int)(idx % groups);
    const int64_t pixg = idx / groups;
    const int64_t b = pixg / (H * W);
    const int pix = (int)(pixg % (H * W));
    const int y = pix / W, x = pix % W;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      const bf16* src = g + ((b * H + yy) * W + xx) * CIN;
      uint4 u[CIN / 8];
#pragma unroll
      for (int v = 0; v < CIN / 8; ++v) u[v] = ld16(src + 8 * v);
      const bf16* e = reinterpret_cast<const bf16*>(u);
      const float* wt = sw + tap * CIN * ldw + cg * 4;
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci) {
        const float v = bf2f(e[ci]);
        const float4 ww = *reinterpret_cast<const float4*>(wt + ci * ldw);
        a0 += v * ww.x; a1 += v * ww.y; a2 += v * ww.z; a3 += v * ww.w;
      }
    }
    if constexpr (PAR) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
        if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
        const float4 tb = *reinterpret_cast<const float4*>(stb + tap * cout + cg * 4);
        a0 += tb.x; a1 += tb.y; a2 += tb.z; a3 += tb.w;
      }
      const int64_t o = ((b * (H / 2) + y / 2) * (W / 2) + x / 2) * 4 * cout + ((y & 1) * 2 + (x & 1)) * cout + cg * 4;
      *reinterpret_cast<float4*>(out + o) = make_float4(a0, a1, a2, a3);
    } else {
      *reinterpret_cast<float4*>(out + pixg * cout + cg * 4) = make_float4(a0, a1, a2, a3);
    }
  }
}

// The same per-image partial conv on the MFMA (g_partial_mfma, default): an im2col GEMM over
// k = tap * CIN + ci, D^T = W . X^T per 16-pixel tile (a lane ends with 4 consecutive output channels
// of one pixel: float4 stores).  The guidance is bf16 (exact as an MFMA operand); the fp32 weights
// enter as two bf16 pieces w = w_hi + w_lo (w_lo = bf16(w - w_hi)), two MFMAs per k-step, so the
// weights keep ~16 mantissa bits (relative 2^-17) instead of bf16's 8.  CIN = 32: one tap per 32-deep
// k-step (9 steps); CIN = 16: taps 2s (lanes q < 2) and 2s + 1 (q >= 2) share step s (5 steps, tap 9
// zero).  Each wave walks 16-pixel tiles with its 9 / 5 guidance fragment loads issued before the
// MFMAs; the weight pieces are staged once per workgroup in LDS ([co][k] rows padded by 16 bytes).
template <int CIN, bool PAR = false>
__global__ __launch_bounds__(256) void conv_partial_mfma_kernel(const bf16* __restrict__ g, int64_t B, int H, int W,
                                                               const float* __restrict__ w, int cout, float* out,
                                                               const float* __restrict__ tap_bias, int64_t ntiles) {
  static_assert(CIN == 16 || CIN == 32, "CIN");
  constexpr int KS = CIN == 32 ? 9 : 5;            // 32-deep k-steps
  constexpr int LDR = KS * 32 + 8;                 // LDS row (one output channel), elements
  extern __shared__ __attribute__((aligned(16))) char smem_p[];
  bf16* whi = reinterpret_cast<bf16*>(smem_p);     // [cout][LDR]
  bf16* wlo = whi + cout * LDR;
  float* stb = reinterpret_cast<float*>(wlo + cout * LDR);   // PAR: [9][cout]
  // k = tap * CIN + ci is also the order of a weight row w[co][tap][ci]: 16-byte loads, k >= 9 CIN zero
  for (int i = threadIdx.x; i < cout * KS * 8; i += blockDim.x) {
    const int co = i / (KS * 8), k4 = (i % (KS * 8)) * 4;
    const float4 v = k4 < 9 * CIN ? *reinterpret_cast<const float4*>(w + (int64_t)co * 9 * CIN + k4) : make_float4(0.f, 0.f, 0.f, 0.f);
    const unsigned h0 = f2bf2(v.x, v.y), h1 = f2bf2(v.z, v.w);
    const unsigned l0 = f2bf2(v.x - __uint_as_float(h0 << 16), v.y - __uint_as_float(h0 & 0xffff0000u));
    const unsigned l1 = f2bf2(v.z - __uint_as_float(h1 << 16), v.w - __uint_as_float(h1 & 0xffff0000u));
    *reinterpret_cast<uint2*>(whi + co * LDR + k4) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(wlo + co * LDR + k4) = make_uint2(l0, l1);
  }
  if constexpr (PAR)
    for (int i = threadIdx.x; i < 9 * cout; i += blockDim.x) stb[i] = tap_bias ? tap_bias[i] : 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int HW = H * W;
  const int nt = cout / 16;
  // guidance fragments of a tile: lane (pixel r16, q) holds k = 32 s + 8 q .. +7; the next tile's are
  // requested before this tile's MFMAs
  auto gather = [&](int64_t tile, s16x8 (&xf)[KS]) {
    const int64_t pixg = tile * 16 + r16;
    const int64_t b = pixg / HW;
    const int pix = (int)(pixg - b * HW), y = pix / W, x = pix - y * W;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int tap = CIN == 32 ? st : 2 * st + (q >> 1), ci = CIN == 32 ? 8 * q : 8 * (q & 1);
      const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
      const bool ok = tile < ntiles && tap < 9 && yy >= 0 && yy < H && xx >= 0 && xx < W;
      const uint4 u = ok ? ld16(g + ((b * H + yy) * W + xx) * CIN + ci) : make_uint4(0, 0, 0, 0);
      xf[st] = __builtin_bit_cast(s16x8, u);
    }
  };
  const int64_t tstride = (int64_t)gridDim.x * 4;
  s16x8 xn[KS];
  gather((int64_t)blockIdx.x * 4 + wave, xn);
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles; tile += tstride) {
    const int64_t pixg = tile * 16 + r16;          // this lane's pixel (the second operand's column)
    const int64_t b = pixg / HW;
    const int pix = (int)(pixg - b * HW), y = pix / W, x = pix - y * W;
    s16x8 xf[KS];
#pragma unroll
    for (int st = 0; st < KS; ++st) xf[st] = xn[st];
    gather(tile + tstride, xn);
    for (int n = 0; n < nt; ++n) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const bf16* rh = whi + (n * 16 + r16) * LDR + 8 * q;
      const bf16* rl = wlo + (n * 16 + r16) * LDR + 8 * q;
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        acc = mfma_bf16(*reinterpret_cast<const s16x8*>(rl + st * 32), xf[st], acc);
        acc = mfma_bf16(*reinterpret_cast<const s16x8*>(rh + st * 32), xf[st], acc);
      }
      // lane: output channels 16 n + 4 q .. +3 of pixel r16
      const int co = n * 16 + 4 * q;
      if constexpr (PAR) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
          if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
          acc += *reinterpret_cast<const f32x4*>(stb + tap * cout + co);
        }
        const int64_t o = ((b * (H / 2) + y / 2) * (W / 2) + x / 2) * 4 * cout + ((y & 1) * 2 + (x & 1)) * cout + co;
        *reinterpret_cast<f32x4*>(out + o) = acc;
      } else {
        *reinterpret_cast<f32x4*>(out + pixg * cout + co) = acc;
      }
    }
  }
}

int g_partial_mfma = 1;   // 1 = conv_partial_mfma_kernel, 0 = the VALU kernel (conv_partial_vec_kernel)

template <int CIN, bool PAR>
void launch_partial_mfma(const bf16* g, int64_t B, int H, int W, const float* w, int cout, float* out,
                         const float* tap_bias, hipStream_t st) {
  constexpr int KS = CIN == 32 ? 9 : 5, LDR = KS * 32 + 8;
  const size_t sh = (size_t)2 * cout * LDR * 2 + (PAR ? (size_t)9 * cout * 4 : 0);
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_partial_mfma_kernel<CIN, PAR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    configured = true;
  }
  const int64_t ntiles = B * H * W / 16;
  // two workgroups per CU (the weight pieces are staged once per workgroup, 16-byte loads)
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ntiles + 3) / 4, 2LL * catseg_device_cus()));
  hipLaunchKernelGGL((conv_partial_mfma_kernel<CIN, PAR>), dim3(grid), dim3(256), sh, st, g, B, H, W, w, cout, out,
                     tap_bias, ntiles);
}

}  // namespace

// Variant table of the ring kernel: 0 = not applicable, else an id; *tile = pixels per
// GroupNorm partial (the wave pixel block PXW = CH / WPX).
static int ring_variant(const CatsegConvArgs* a, int* tile) {
  if (a->dtype != CATSEG_BF16) return 0;
  const int C = a->c1 + a->c2;
  const int64_t HW = (int64_t)a->H * a->W;
  if (HW % 128 != 0 || a->W < 48 || a->W > 96) return 0;
  if (a->s1_offset != 0 || a->s2_offset != 0) return 0;
  if (a->stats && a->stats_cpg != 16) return 0;
  if (a->gn_mean && (a->c1 % 8 != 0)) return 0;
  if (a->addend && ((uintptr_t)a->addend % 16 != 0 || a->addend_slice_stride % 4 != 0)) return 0;
  const bool narrow = a->W < 64;      // CH = 128 spans <= 3 rows only from W >= 64 on
  int v = 0, t = 0;
  if (C == 64 && a->c_out == 32) { v = narrow ? 1 : 2; t = 32; }
  else if (C == 48 && a->c_out == 32) {
    v = narrow ? 3 : 9;
    t = 32;
  } else if (C == 32 && a->c_out == 32) {
    v = narrow ? 5 : 6;
    t = 32;
  }
  else if (C == 64 && a->c_out == 64 && a->W <= 50) { v = 7; t = 128; }
  else if (C == 96 && a->c_out == 64 && a->W <= 50) { v = 8; t = 64; }
  if (tile) *tile = t;
  return v;
}

int g_ring_store = 0;   // conv ring output stores: 0 = plain, 1 = sc1 write-through (A/B knob; same box, whole step 9.251 -> 9.375 ms: slower)
CATSEG_KNOB(g_ring_store, "ring_store");

// Pixels per GroupNorm partial ("tile") of the conv catseg_conv3x3 would run for these args.
int catseg_conv3x3_ring_tile(const CatsegConvArgs* a) {
  int t = 0;
  return ring_variant(a, &t) ? t : 0;
}

// bf16 fast path of catseg_conv3x3 (conv.hip): 0 = launched, 1 = not applicable.
int catseg_conv3x3_ring(const CatsegConvArgs* a, hipStream_t st) {
  const int v = ring_variant(a, nullptr);
  if (!v) return 1;
  RingP p;
  p.s1 = (const bf16*)a->src1; p.s1_ss = a->s1_slice_stride; p.c1 = a->c1;
  p.s2 = (const bf16*)a->src2; p.s2_ss = a->s2_slice_stride; p.c2 = a->c2; p.s2_div = a->src2_div > 0 ? a->src2_div : 1;
  p.S = a->S; p.H = a->H; p.W = a->W;
  p.up_split = 1;
  p.w = (const bf16*)a->weight; p.bias = a->bias; p.act = a->act;
  p.gmean = a->gn_mean; p.grstd = a->gn_rstd; p.ggamma = a->gn_gamma; p.gbeta = a->gn_beta; p.gcpg = a->gn_cpg;
  p.add = a->addend; p.add_ss = a->addend_slice_stride; p.add_div = a->addend_div > 0 ? a->addend_div : 1;
  p.out = (bf16*)a->out; p.stats = a->stats;
  p.wt = g_ring_store && (int64_t)a->S * a->H * a->W * a->c_out * 2 < 0x7fffffffLL;
  // weights in registers: 9 taps x C/16 half-steps x COUT/WCO/16 fragments
  switch (v) {
    case 1: return launch_ring<64, 32, 4, 1, 156>(p, st);
    case 2: return launch_ring<64, 32, 4, 1, 198, 128, 2, 5>(p, st);
    case 3: return launch_ring<48, 32, 4, 1, 156>(p, st);
    case 5: return launch_ring<32, 32, 4, 1, 156>(p, st);
    case 6:
      // one barrier per chunk: a 128-pixel chunk spans <= 3 rows of 96 (+2 halo), the next adds <= 2
      if (g_ring_onebar) return launch_ring<32, 32, 4, 1, 198, 128, 2, 7, true>(p, st);
      return launch_ring<32, 32, 4, 1, 198, 128, 2, 5>(p, st);
    case 7:
      // 128 pixels of 48: <= 4 rows (+2), the next adds <= 3
      if (g_ring_onebar) return launch_ring<64, 64, 1, 4, 156, 128, 2, 9, true>(p, st);
      return launch_ring<64, 64, 1, 4, 156>(p, st);
    case 8: return launch_ring<96, 64, 1, 4, 104, 64, 2, 5>(p, st);
    case 9: return launch_ring<48, 32, 4, 1, 198, 128, 2, 5>(p, st);
    default: return 1;
  }
}

extern "C" int catseg_conv3x3_partial(const void* g, int64_t B, int H, int W, int cin, const float* weight, int cout,
                                      float* out, int dtype, void* stream) {
  CATSEG_CHECK(g && weight && out && B > 0 && H > 0 && W > 0 && cin > 0, "conv3x3_partial: bad args");
  CATSEG_CHECK(cout % 4 == 0 && (size_t)9 * cin * cout * 4 <= 128 * 1024, "conv3x3_partial: cout % 4, weights <= 128 KB");
  const size_t sh = (size_t)9 * cin * cout * 4;
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_partial_kernel<bf16>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_partial_kernel<float>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    configured = true;
  }
  const int64_t total = B * H * W * (cout / 4);
  const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
  const bool vec = dtype == CATSEG_BF16 && ((uintptr_t)g % 16) == 0 && (cin == 16 || cin == 32);
  if (vec) {
    // grid-stride over the pixels with ~2 workgroups per CU: the [9][cin][cout + 4] weight image
    // (up to 78 KB) is staged once per workgroup, not once per 256 pixels
    const unsigned vgrid = (unsigned)std::min<int64_t>((total + 255) / 256, 512);
    static bool vconfigured = false;
    if (!vconfigured) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_partial_vec_kernel<16>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_partial_vec_kernel<32>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      vconfigured = true;
    }
    const size_t shv = (size_t)9 * cin * (cout + 4) * 4;   // padded LDS rows (conv_partial_vec_kernel)
    CATSEG_CHECK(shv <= 128 * 1024, "conv3x3_partial: weights <= 128 KB");
    if (g_partial_mfma && cout % 16 == 0 && (H * W) % 16 == 0 && cout <= 128) {
      if (cin == 16) launch_partial_mfma<16, false>((const bf16*)g, B, H, W, weight, cout, out, nullptr, (hipStream_t)stream);
      else launch_partial_mfma<32, false>((const bf16*)g, B, H, W, weight, cout, out, nullptr, (hipStream_t)stream);
    } else if (cin == 16)
      hipLaunchKernelGGL(conv_partial_vec_kernel<16>, dim3(vgrid), dim3(256), shv, (hipStream_t)stream, (const bf16*)g,
                         B, H, W, weight, cout, out);
    else
      hipLaunchKernelGGL(conv_partial_vec_kernel<32>, dim3(vgrid), dim3(256), shv, (hipStream_t)stream, (const bf16*)g,
                         B, H, W, weight, cout, out);
  } else if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL(conv_partial_kernel<bf16>, dim3(grid), dim3(256), sh, (hipStream_t)stream, (const bf16*)g, B, H,
                       W, cin, weight, cout, out);
  else
    hipLaunchKernelGGL(conv_partial_kernel<float>, dim3(grid), dim3(256), sh, (hipStream_t)stream, (const float*)g, B,
                       H, W, cin, weight, cout, out);
  return catseg_launch_status("conv3x3_partial");
}

CATSEG_KNOB(g_ring_persist, "ring_persist");
CATSEG_KNOB(g_partial_mfma, "partial_mfma");
CATSEG_KNOB(g_ring_onebar, "ring_onebar");

// ---- ConvTranspose2d(k=2, s=2) folded into the following conv3x3 (Up, model.py:546-555) ----
// The conv over the ConvTranspose output y (2H x 2W, no nonlinearity between them) equals, per
// output parity (a, b), a 2x2-tap conv over the ConvTranspose INPUT with composite weights
// W_c(a,b)[co][tap][ci] = sum over the conv taps that land on source tap `tap` of
// W_conv[co][.][m] W_convT[ci][m][py][px] (built by the caller), plus the ConvTranspose bias
// pushed through the conv taps that fall inside the image (the addend, catseg_upconv_addend).
// The 2H x 2W ConvTranspose output is never materialised.
extern "C" int catseg_upconv_addend(const void* g, int64_t B, int H2, int W2, int cin, const float* weight,
                                    const float* tap_bias, int cout, float* out, int dtype, void* stream) {
  CATSEG_CHECK(g && weight && out && B > 0 && H2 > 0 && W2 > 0 && H2 % 2 == 0 && W2 % 2 == 0, "upconv_addend: bad args");
  CATSEG_CHECK(dtype == CATSEG_BF16 && (cin == 16 || cin == 32) && ((uintptr_t)g % 16) == 0,
               "upconv_addend: bf16 guidance with 16 or 32 channels, 16B aligned");
  CATSEG_CHECK(cout % 4 == 0 && (size_t)(9 * cin * (cout + 4) + 9 * cout) * 4 <= 128 * 1024 && ((uintptr_t)out % 16) == 0 &&
                   (!tap_bias || ((uintptr_t)tap_bias % 16) == 0),
               "upconv_addend: cout % 4, weights <= 128 KB, 16B aligned out / tap_bias");
  const size_t sh = (size_t)(9 * cin * (cout + 4) + 9 * cout) * 4;   // padded weight rows + tap bias
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_partial_vec_kernel<16, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_partial_vec_kernel<32, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    configured = true;
  }
  const int64_t total = B * H2 * W2 * (cout / 4);
  const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 512);
  if (g_partial_mfma && cout % 16 == 0 && (H2 * W2) % 16 == 0 && cout <= 128) {
    if (cin == 16) launch_partial_mfma<16, true>((const bf16*)g, B, H2, W2, weight, cout, out, tap_bias, (hipStream_t)stream);
    else launch_partial_mfma<32, true>((const bf16*)g, B, H2, W2, weight, cout, out, tap_bias, (hipStream_t)stream);
  } else if (cin == 16)
    hipLaunchKernelGGL((conv_partial_vec_kernel<16, true>), dim3(grid), dim3(256), sh, (hipStream_t)stream,
                       (const bf16*)g, B, H2, W2, weight, cout, out, tap_bias);
  else
    hipLaunchKernelGGL((conv_partial_vec_kernel<32, true>), dim3(grid), dim3(256), sh, (hipStream_t)stream,
                       (const bf16*)g, B, H2, W2, weight, cout, out, tap_bias);
  return catseg_launch_status("upconv_addend");
}

// Pixels per GroupNorm partial of catseg_upconv3x3 on the SOURCE grid; its stats hold
// [S][4 * H*W / tile][c_out/4/16][2] (parity-major partials).
extern "C" int catseg_upconv3x3_stats_tile(void) { return 64; }

extern "C" int catseg_upconv3x3(const CatsegConvArgs* a, void* stream) {
  CATSEG_CHECK(a && a->src1 && a->weight && a->out, "upconv3x3: null pointer");
  CATSEG_CHECK(a->dtype == CATSEG_BF16 && a->c2 == 0 && !a->src2, "upconv3x3: bf16, one source");
  const bool up2 = a->c1 == 64 && a->c_out == 128 && a->W == 48;
  const bool up1 = a->c1 == 128 && a->c_out == 256 && a->W == 24;
  CATSEG_CHECK((up1 || up2) && ((int64_t)a->H * a->W) % 64 == 0,
               "upconv3x3: instantiated for 64 source channels -> 4 x 32 outputs on a 48-wide source grid "
               "and 128 -> 4 x 64 on a 24-wide one (H*W % 64 == 0)");
  CATSEG_CHECK(a->s1_offset == 0 && a->s1_slice_stride % 8 == 0, "upconv3x3: src stride alignment");
  CATSEG_CHECK(!a->stats || a->stats_cpg == 16, "upconv3x3: GN stats in 16-channel groups");
  CATSEG_CHECK(!a->gn_mean || (a->gn_rstd && a->gn_gamma && a->gn_beta && a->gn_cpg > 0 && a->c1 % a->gn_cpg == 0),
               "upconv3x3: bad GroupNorm prologue");
  CATSEG_CHECK(!a->addend || (((uintptr_t)a->addend % 16) == 0 && a->addend_slice_stride % 4 == 0),
               "upconv3x3: addend alignment");
  RingP p;
  p.s1 = (const bf16*)a->src1; p.s1_ss = a->s1_slice_stride; p.c1 = a->c1;
  p.s2 = nullptr; p.s2_ss = 0; p.c2 = 0; p.s2_div = 1;
  p.S = a->S; p.H = a->H; p.W = a->W;
  p.w = (const bf16*)a->weight; p.bias = a->bias; p.act = a->act;
  p.gmean = a->gn_mean; p.grstd = a->gn_rstd; p.ggamma = a->gn_gamma; p.gbeta = a->gn_beta; p.gcpg = a->gn_cpg;
  p.add = a->addend; p.add_ss = a->addend_slice_stride; p.add_div = a->addend_div > 0 ? a->addend_div : 1;
  p.out = (bf16*)a->out; p.stats = a->stats;
  p.wt = g_ring_store && (int64_t)a->S * a->H * a->W * a->c_out * 2 < 0x7fffffffLL;
  p.up_split = 1;
  hipStream_t st = (hipStream_t)stream;
  // 64-pixel chunks (a 48-wide chunk spans <= 3 rows: 5-row ring, <= 2 new rows = 104 positions):
  // 128-pixel chunks spilled ~100 VGPRs with the addend (one 512-register workgroup per CU measured
  // slower, as did 96-pixel chunks and four 16-channel workgroups per parity for the first block)
  int rc;
  if (up2) {
    // one barrier per chunk: 64 pixels of 48 span <= 3 rows (+2), the next chunk adds <= 2
    if (g_ring_onebar) {
      if (p.add) rc = launch_ring_t<64, 128, 1, 4, 104, 64, 2, 7, true, true, 48, true>(p, st);
      else rc = launch_ring_t<64, 128, 1, 4, 104, 64, 2, 7, false, true, 48, true>(p, st);
    } else if (p.add) rc = launch_ring_t<64, 128, 1, 4, 104, 64, 2, 5, true, true, 48>(p, st);
    else rc = launch_ring_t<64, 128, 1, 4, 104, 64, 2, 5, false, true, 48>(p, st);
  } else {
    // first Up block (24-wide source, 128 channels): a parity's 64 outputs x 4 taps x 4 k-steps would
    // be 256 weight VGPRs per wave, so two workgroups split them (32 each, the source ring read by
    // both); a 64-pixel chunk spans <= 4 rows (6-row ring) and adds <= 3 (78 positions)
    p.up_split = 2;
    // one barrier per chunk: 64 pixels of 24 span <= 4 rows (+2), the next chunk adds <= 3
    if (g_ring_onebar) {
      if (p.add) rc = launch_ring_t<128, 128, 1, 4, 78, 64, 1, 9, true, true, 24, true>(p, st);
      else rc = launch_ring_t<128, 128, 1, 4, 78, 64, 1, 9, false, true, 24, true>(p, st);
    } else if (p.add) rc = launch_ring_t<128, 128, 1, 4, 78, 64, 1, 6, true, true, 24>(p, st);
    else rc = launch_ring_t<128, 128, 1, 4, 78, 64, 1, 6, false, true, 24>(p, st);
  }
  if (rc != 0) return rc;
  return catseg_launch_status("upconv3x3");
}
