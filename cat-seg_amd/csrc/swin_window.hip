// Swin window attention (bf16): the kernels behind catseg_swin_window_attention (swin_fused.hip
// holds the argument checks, the variant switch and the older row-tile-wave form).
// Reference: SwinTransformerBlock.forward model.py:191-199 (norm1, concat guidance, roll,
// window_partition) and WindowAttention.forward model.py:86-114 up to the output projection;
// the -100 region mask of model.py:161-183.
//
// A window is 144 tokens = 9 row tiles of 16, 4 heads of 32.  Two forms cut the work by HEAD:
//
// swin_win5 (default, swin_variant 0; below): two 4-wave workgroups per CU, wave h = head h of its
// workgroup's window for all 9 tiles.  LayerNorm by the 4 waves into Xn (LDS), then the projection
// leaves k^T / q^T / v of the head in the wave's own registers in exactly the MFMA operand layouts the
// attention needs (108 VGPRs), so no K / V image goes through LDS and there is no barrier between
// projection and attention; the two workgroups of a CU interleave their MFMA and softmax phases.
//
// swin_win3 (swin_variant 3; other guidance row maps): one 8-wave workgroup per CU, waves w and w + 4 share head
// w % 4 (every SIMD does one head), K and V^T of each head staged in LDS:
//   P1  LayerNorm(norm1) of the 144 rows in place in Xn (bf16, chunk-major XOR-swizzled), 16
//       lanes per row.  The raw rows were brought in by LDS-DMA during the previous window's P3.
//   --  barrier
//   P2  wave (h, sub) projects row tiles sub, sub + 2, ... of head h against W_q / W_k of the head
//       held in REGISTERS (64 x 128 rows as MFMA fragments, loaded once) and W_v from LDS:
//         q^T = W_q Xn^T + b + guidance   -> registers (already the B operand of S^T = K Q^T)
//         k^T = W_k Xn^T + b + guidance   -> LDS K_h [key][32] (same permuted d order as q)
//         v   = Xn W_v^T + b              -> LDS V_h^T [d][key] (operands swapped: 4 keys per lane)
//       (the region one-hot of the shifted windows is written here too)
//   --  barrier
//   P3  the same row tiles as queries: S^T = K Q^T (+ the -100 region mask as a second MFMA on
//       one-hot key dims, skipped for the window location with a single region), softmax over
//       the 144 keys of the window in registers, O^T = V^T P^T and the row sums on the MFMA,
//       8-byte stores of the head's 32 output channels.  The next window's rows are requested
//       (LDS-DMA into Xn, free once P2 is done everywhere).
//   --  counted vmcnt + barrier (the DMA is visible; every wave is past P3)
// HBM traffic per window: the 144 input rows, the 144 output rows, the guidance rows (shared by
// every class of an image: L2-resident).
#include "common.h"
#include <type_traits>
#include "capi.h"

namespace {

constexpr int IMG = 24, WS = 12, NWIN = 4, L = WS * WS;    // 144 tokens per window
constexpr int C = 128, D = 32, NH = 4;
constexpr int NW = 8, NT = NW * 64;
constexpr int NTILE = L / 16;                              // 9 row tiles
constexpr int MYT = (NTILE + 1) / 2;                       // row tiles of a wave (5 / 4)
constexpr int KBV = 160;                                   // keys of V^T (5 x 32-key MFMA steps)
constexpr int VP = KBV + 4;                                // V^T row stride (elements)
constexpr int LNS = (L + 4 * NW - 1) / (4 * NW);           // LayerNorm steps (4 rows per wave each)

struct Swin3P {
  const bf16* x; int64_t ld_x;
  const float* ln_g; const float* ln_b; float eps;
  const bf16* w; const float* bias;
  const bf16* g; int64_t ld_g; RowMap gmap;
  bf16* out; int64_t ld_out;
  int shift; float scale;
  int glin;     // gmap restricted to a slice is rowmap(slice * 576) + pixel
  int wt;       // swin_win5: launch the sc1 write-through instance (swin_store knob)
};

// 16-byte chunk c of row r of a chunk-major image with ROWS rows, row XOR swizzle in the low 4 bits
template <int ROWS>
DEV int cs(int c, int r) { return (c * ROWS + (r ^ (c & 15))) * 8; }

DEV int win_row3(int slice, int wloc, int i, int shift) {     // roll(-shift) + window_partition
  const int Y = (wloc >> 1) * WS + i / WS, X = (wloc & 1) * WS + i % WS;
  const int y = Y + shift < IMG ? Y + shift : Y + shift - IMG;
  const int x = X + shift < IMG ? X + shift : X + shift - IMG;
  return slice * IMG * IMG + y * IMG + x;
}

DEV int region3(int wloc, int i, int shift) {                  // model.py:161-176 label
  const int Y = (wloc >> 1) * WS + i / WS, X = (wloc & 1) * WS + i % WS;
  const int hb = Y < IMG - WS ? 0 : (Y < IMG - shift ? 1 : 2);
  const int wb = X < IMG - WS ? 0 : (X < IMG - shift ? 1 : 2);
  return hb * 3 + wb;
}

DEV s16x8 pk8(const f32x4& a, const f32x4& b) {
  return __builtin_bit_cast(s16x8, make_uint4(f2bf2(a[0], a[1]), f2bf2(a[2], a[3]), f2bf2(b[0], b[1]), f2bf2(b[2], b[3])));
}
DEV f32x4 unpack4(uint2 u) {
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}

// LDS-DMA issued from inline asm: the compiler does not see it, so it does not make every later LDS
// read wait (s_waitcnt vmcnt(0)) for the next window's rows in flight -- with the builtin, P3's first
// K-fragment read waited for the whole prefetch, and the window start for every P3 store.  The
// kernel retires the DMA itself (counted vmcnt at the window start).
DEV void dma16_opaque(const void* src, unsigned lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr) : "memory", "m0");
}

template <bool SWM>
__global__ __launch_bounds__(NT) void swin_win3_kernel(Swin3P p, int nwin_total) {
  __shared__ __attribute__((aligned(16))) bf16 Xn[L * C];               // LayerNorm'd window rows
  __shared__ __attribute__((aligned(16))) bf16 Ks[NH][4 * L * 8];       // [head][chunk][key] (chunk-major)
  __shared__ __attribute__((aligned(16))) bf16 Oh[SWM ? 4 * L * 8 : 8]; // region one-hot of the keys
  __shared__ __attribute__((aligned(16))) bf16 Vt[NH][D * VP];          // [head][d][key]
  __shared__ __attribute__((aligned(16))) bf16 sWv[C * C];              // W_v (every head), chunk-major
  __shared__ __attribute__((aligned(16))) float sP[2 * C + 3 * C];      // LN gamma | beta | qkv bias

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = wave & 3, sub = wave >> 2;
  const int r16 = lane & 15, g = lane >> 4;
  for (int i = tid; i < 5 * C; i += NT) sP[i] = i < C ? p.ln_g[i] : i < 2 * C ? p.ln_b[i - C] : p.bias[i - 2 * C];
  for (int i = tid; i < NH * D * (KBV - L); i += NT) {       // V^T key columns 144..159 stay zero
    const int hh = i / (D * (KBV - L)), j = i % (D * (KBV - L));
    Vt[hh][(j / (KBV - L)) * VP + L + j % (KBV - L)] = 0;
  }
  for (int c = tid; c < C * 16; c += NT) {                  // W_v rows -> LDS (read as B fragments)
    const int lr = c >> 4, ch = c & 15;
    st16(&sWv[cs<C>(ch, lr)], ld16(p.w + (int64_t)(2 * C + lr) * C + ch * 8));
  }
  // head h's q / k weight rows as MFMA fragments: wf[part][dt][ks] = W[part*C + h*D + 16dt + r16][32ks + 8g ..]
  s16x8 wf[2][2][4];
#pragma unroll
  for (int part = 0; part < 2; ++part)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        wf[part][dt][ks] = __builtin_bit_cast(
            s16x8, ld16(p.w + (int64_t)(part * C + h * D + dt * 16 + r16) * C + ks * 32 + 8 * g));
  __syncthreads();
  s16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)0x3F80;
  const float sl2 = p.scale * 1.4426950408889634f;

  // LayerNorm rows: step s, row s*32 + 4*wave + (lane >> 4), 16-byte chunk lane & 15
  const int lc = lane & 15, lrow0 = 4 * wave + (lane >> 4);
  // raw rows of a window -> Xn by LDS-DMA (no VGPRs held across the attention phase): the image
  // is lane-linear per wave-instruction, so slot s (16 bytes) of the chunk-major swizzled Xn
  // receives chunk c = s / L of token row (s % L) ^ (c & 15), and the LayerNorm then runs in place
  constexpr int NDMA = L * 16 / 64;                       // 36 wave-instructions per window
  auto fetch = [&](int win) {
    const int slice = win / NWIN, wloc = win % NWIN;
    for (int k = wave; k < NDMA; k += NW) {
      const int sl = k * 64 + lane, c = sl / L, i = (sl % L) ^ (c & 15);
      const bf16* src = p.x + (int64_t)win_row3(slice, wloc, i, p.shift) * p.ld_x + c * 8;
      dma16_opaque(src, __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(Xn + k * 64 * 8)));
    }
  };
  int win = blockIdx.x;
  if (win < nwin_total) fetch(win);
  // the first window's rows: retired here, outside the window loop, so that the counted wait at
  // the loop top is only ever reached from the previous window's P3 (tools/isa_lint.py R3)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (; win < nwin_total; win += gridDim.x) {
    const int slice = win / NWIN, wloc = win % NWIN;
    // this wave's DMA of the window landed: only the previous window's P3 stores (2 per row tile,
    // >= 8 per wave) were issued behind it, and those may stay in flight (the first window's DMA
    // was retired before the loop)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __syncthreads();                                       // every wave's DMA visible; P3 done
    // guidance row of token rb + r16 of this window: rowmap(slice*576) + pixel when the host
    // found the map linear in the pixel (CAT-Seg's (b, t, p) -> (b, p)), else the general map
    const int64_t gbase = p.glin ? rowmap(p.gmap, (int64_t)slice * (IMG * IMG)) : 0;
    auto fetch_g = [&](int t, uint2 (&gd)[2][2]) {
      const int row = win_row3(slice, wloc, 16 * t + r16, p.shift);
      const int64_t grow = p.glin ? gbase + (row - slice * (IMG * IMG)) : rowmap(p.gmap, row);
      const bf16* gp = p.g + grow * p.ld_g + h * D + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        gd[0][dt] = *reinterpret_cast<const uint2*>(gp + dt * 16);
        gd[1][dt] = *reinterpret_cast<const uint2*>(gp + C + dt * 16);
      }
    };
    uint2 gc[2][2];
    fetch_g(sub, gc);
    // ---------------- P1: LayerNorm of Xn in place ----------------
    {
      const float4 g0 = *reinterpret_cast<const float4*>(&sP[lc * 8]), g1 = *reinterpret_cast<const float4*>(&sP[lc * 8 + 4]);
      const float4 b0 = *reinterpret_cast<const float4*>(&sP[C + lc * 8]), b1 = *reinterpret_cast<const float4*>(&sP[C + lc * 8 + 4]);
      const float lg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float lb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int s = 0; s < LNS; ++s) {
        const int i = min(s * 32 + lrow0, L - 1);
        const uint4 raw = *reinterpret_cast<const uint4*>(&Xn[cs<L>(lc, i)]);
        const bf16* e = reinterpret_cast<const bf16*>(&raw);
        float v[8], sum = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[j] = bf2f(e[j]); sum += v[j]; }
        sum = row16_sum(sum);
        const float mean = sum * (1.f / C);
        float qs = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[j] -= mean; qs += v[j] * v[j]; }
        qs = row16_sum(qs);
        const float rstd = __builtin_amdgcn_rsqf(qs * (1.f / C) + p.eps);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] * rstd * lg[j] + lb[j];
        if (s * 32 + 4 * NW <= L || s * 32 + lrow0 < L)
          st16(&Xn[cs<L>(lc, i)], make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7])));
      }
    }
    __syncthreads();
    // ---------------- P2: q / k / v of head h for row tiles sub, sub + 2, ... ----------------
    if constexpr (SWM) {   // region one-hot of the keys (P3 of the previous window has retired its reads)
      if (gridDim.x % NWIN != 0 || win == (int)blockIdx.x) {
        for (int key = tid; key < L; key += NT) {
          const int reg = region3(wloc, key, p.shift);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            unsigned w4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int e0 = c * 8 + 2 * j;
              w4[j] = (e0 == reg ? 0x3F80u : 0u) | (e0 + 1 == reg ? 0x3F800000u : 0u);
            }
            st16(&Oh[(c * L + key) * 8], make_uint4(w4[0], w4[1], w4[2], w4[3]));
          }
        }
      }
    }
    s16x8 qf[MYT];
    // guidance rows of row tile sub + 2j (q, k halves of head h): tile j+1's are in flight during
    // tile j, tile 0's were requested before P1
#pragma unroll
    for (int j = 0; j < MYT; ++j) {
      const int t = sub + 2 * j;
      if (t < NTILE) {
        const int rb = 16 * t;
        uint2 gn[2][2];
        if (j + 1 < MYT && t + 2 < NTILE) fetch_g(t + 2, gn);
        s16x8 xb[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) xb[ks] = *reinterpret_cast<const s16x8*>(&Xn[(( (ks * 4 + g) * L) + rb + (r16 ^ ((ks * 4 + g) & 15))) * 8]);
        f32x4 dq[2], dk[2], dv[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          // accumulators start at bias + guidance (q, k: features 16dt + 4g + r of token r16) / bias (v)
          dq[dt] = *reinterpret_cast<const f32x4*>(&sP[2 * C + h * D + dt * 16 + 4 * g]) + unpack4(gc[0][dt]);
          dk[dt] = *reinterpret_cast<const f32x4*>(&sP[3 * C + h * D + dt * 16 + 4 * g]) + unpack4(gc[1][dt]);
          const float bvv = sP[4 * C + h * D + dt * 16 + r16];
          dv[dt] = f32x4{bvv, bvv, bvv, bvv};
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            dq[dt] = mfma_bf16(wf[0][dt][ks], xb[ks], dq[dt]);
            dk[dt] = mfma_bf16(wf[1][dt][ks], xb[ks], dk[dt]);
            dv[dt] = mfma_bf16(xb[ks], *reinterpret_cast<const s16x8*>(&sWv[cs<C>(ks * 4 + g, h * D + dt * 16 + r16)]),
                               dv[dt]);                   // D[token 4g + r][feature 16dt + r16]
          }
        qf[j] = pk8(dq[0], dq[1]);              // q features {4g..4g+3, 16+4g..16+4g+3} of token r16
        st16(&Ks[h][(g * L + rb + r16) * 8], __builtin_bit_cast(uint4, pk8(dk[0], dk[1])));
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          *reinterpret_cast<uint2*>(&Vt[h][(dt * 16 + r16) * VP + rb + 4 * g]) =
              make_uint2(f2bf2(dv[dt][0], dv[dt][1]), f2bf2(dv[dt][2], dv[dt][3]));
#pragma unroll
        for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) gc[a2][dt] = gn[a2][dt];
      }
      __builtin_amdgcn_sched_barrier(0);        // no cross-tile hoisting (register pressure)
    }
    __syncthreads();
    // ---------------- P3: attention of head h for the same row tiles ----------------
    if (win + (int)gridDim.x < nwin_total) fetch(win + gridDim.x);   // Xn is free: P2 is done everywhere
    const bool masked = SWM && wloc != 0;       // window location 0 holds a single region
#pragma unroll
    for (int j = 0; j < MYT; ++j) {
      const int t = sub + 2 * j;
      if (t >= NTILE) break;
      const int rb = 16 * t;
      s16x8 qmask;
      if (masked) {
        const int qreg = region3(wloc, rb + r16, p.shift);
        const short neg = (short)f2bf(-100.f / p.scale);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int dim = 8 * g + e;
          qmask[e] = dim < 9 && dim != qreg ? neg : (short)0;
        }
      }
      f32x4 st[NTILE + 1];
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt) {
        f32x4 a = mfma_bf16(*reinterpret_cast<const s16x8*>(&Ks[h][(g * L + kt * 16 + r16) * 8]), qf[j],
                            f32x4{0.f, 0.f, 0.f, 0.f});
        if (masked) a = mfma_bf16(*reinterpret_cast<const s16x8*>(&Oh[(g * L + kt * 16 + r16) * 8]), qmask, a);
        st[kt] = a;
      }
      float mx = fmaxf(fmaxf(st[0][0], st[0][1]), fmaxf(st[0][2], st[0][3]));
#pragma unroll
      for (int kt = 1; kt < NTILE; ++kt) mx = fmaxf(mx, fmaxf(fmaxf(st[kt][0], st[kt][1]), fmaxf(st[kt][2], st[kt][3])));
      mx = xrow4_max(mx);
      const float nb = -mx * sl2;
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[kt][r] = __builtin_amdgcn_exp2f(fmaf(st[kt][r], sl2, nb));
      st[NTILE] = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, osum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < KBV / 32; ++u) {
        const s16x8 pb = pk8(st[2 * u], st[2 * u + 1]);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16* vr = &Vt[h][(dt * 16 + r16) * VP + 32 * u + 4 * g];
          const uint2 lo = *reinterpret_cast<const uint2*>(vr);
          const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16);
          o[dt] = mfma_bf16(__builtin_bit_cast(s16x8, make_uint4(lo.x, lo.y, hi.x, hi.y)), pb, o[dt]);
        }
        osum = mfma_bf16(ones, pb, osum);
      }
      const float inv = 1.f / osum[0];
      bf16* O = p.out + (int64_t)win_row3(slice, wloc, rb + r16, p.shift) * p.ld_out + h * D;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
        *reinterpret_cast<uint2*>(O + dt * 16 + 4 * g) =
            make_uint2(f2bf2(o[dt][0] * inv, o[dt][1] * inv), f2bf2(o[dt][2] * inv, o[dt][3] * inv));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Register-resident form (win5): 4-wave workgroups, TWO per CU (75 KB of LDS each), wave h owns
// head h of the workgroup's window for all 9 row tiles.  The projection leaves every operand the
// attention needs in the lane that needs it: an MFMA output k^T tile (lane: features 16dt + 4g + r
// of token r16) is already the A fragment of S^T = K Q^T for that key tile, q^T the B fragment, and
// v (lane: tokens 4g + r, feature 16dt + r16) is the V^T A fragment of O^T = V^T P^T when two key
// tiles are paired.  So K, V^T and Q stay in registers (108 VGPRs), no K / V image goes through LDS,
// and there is no barrier between projection and attention.  The LayerNorm'd rows (Xn, filled by
// LDS-DMA and normalised by the 4 waves together) and W_v stay in LDS; W_q / W_k are re-read (L2) at
// each window start so they are dead during the attention.  The two workgroups of a CU run different
// windows, so one's projection MFMAs sit beside the other's softmax VALU on every SIMD.
constexpr int NW5 = 4, NT5 = NW5 * 64;
constexpr int LNS5 = (L + 4 * NW5 - 1) / (4 * NW5);          // LayerNorm steps (4 rows per wave each)

DEV int local_region5(int wloc, int i, int shift) {   // region3 renumbered within the window: 0..3
  const int wy = wloc >> 1, wx = wloc & 1;
  const int Y = wy * WS + i / WS, X = wx * WS + i % WS;
  const int lh = wy ? (Y < IMG - shift ? 0 : 1) : 0;
  const int lw = wx ? (X < IMG - shift ? 0 : 1) : 0;
  return lh * 2 + lw;
}

// swin_win5's window image Xn: row-major 256-byte rows, 16-byte chunk c of row r at slot c ^ (r & 15):
// the LDS-DMA fills whole rows (16 lanes per row), a fragment read (16 rows x one chunk) and a
// LayerNorm row read (one row x 16 chunks) touch 16 distinct 16-byte bank slots
DEV int xs5(int c, int r) { return (r * 16 + (c ^ (r & 15))) * 8; }

template <bool SWM, bool GLIN, bool WT = false>
__global__ __launch_bounds__(NT5, 2) void swin_win5_kernel(Swin3P p, int nwin_total) {
  __shared__ __attribute__((aligned(16))) bf16 Xn[L * C];               // LayerNorm'd window rows
  __shared__ __attribute__((aligned(16))) bf16 sWv[C * C];              // W_v (every head), chunk-major
  // local region one-hot per key (regions 0..3 of 8 bf16): the A operand of the 16x16x32 mask product
  // for every k group -- the B operand (qmask) is zero outside k 0..3, so lanes g > 0 may read it too
  __shared__ __attribute__((aligned(16))) bf16 Oh[SWM ? L * 8 : 8];
  __shared__ __attribute__((aligned(16))) float sP[5 * C];              // LN gamma | beta | qkv bias

  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int wloc = (int)(blockIdx.x % NWIN);                 // the grid is a multiple of 4 (host)
  for (int i = tid; i < 5 * C; i += NT5) sP[i] = i < C ? p.ln_g[i] : i < 2 * C ? p.ln_b[i - C] : p.bias[i - 2 * C];
  for (int c = tid; c < C * 16; c += NT5) {
    const int lr = c >> 4, ch = c & 15;
    st16(&sWv[cs<C>(ch, lr)], ld16(p.w + (int64_t)(2 * C + lr) * C + ch * 8));
  }
  if constexpr (SWM) {
    for (int key = tid; key < L; key += NT5) {
      const int reg = local_region5(wloc, key, p.shift);
      st16(&Oh[key * 8], make_uint4(reg == 0 ? 0x3F80u : reg == 1 ? 0x3F800000u : 0u,
                                    reg == 2 ? 0x3F80u : reg == 3 ? 0x3F800000u : 0u, 0u, 0u));
    }
  }
  s16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)0x3F80;
  const float sl2 = p.scale * 1.4426950408889634f;
  const bool masked = SWM && wloc != 0;                      // window location 0 holds a single region
  const short neg = (short)f2bf(-100.f / p.scale);
  constexpr int NDMA = L * 16 / 64;                          // 36 wave-instructions per window
  auto fetch = [&](int win) {
    const int slice = win / NWIN;
    for (int k = h; k < NDMA; k += NW5) {
      // row-major image, chunk XOR-swizzled by the row (xs5): the 16 lanes of a row fetch its 16 chunks,
      // so a wave-instruction reads 4 whole 256-byte rows (the chunk-major image it replaces read one
      // 16-byte chunk of 64 rows)
      const int sl = k * 64 + lane, i = sl >> 4, c = (sl & 15) ^ (i & 15);
      const bf16* src = p.x + (int64_t)win_row3(slice, wloc, i, p.shift) * p.ld_x + c * 8;
      dma16_opaque(src, __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(Xn + k * 64 * 8)));
    }
  };
  int win = blockIdx.x;
  if (win < nwin_total) fetch(win);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the first window's rows, retired outside the loop
  __syncthreads();
  for (; win < nwin_total; win += gridDim.x) {
    const int slice = win / NWIN;
    // lane-derived offsets recomputed per window from an opaque copy: hoisted out of the window loop
    // they would hold ~100 VGPRs for the whole kernel
    int lane_w = lane;
    asm volatile("" : "+v"(lane_w));
    const int r16 = lane_w & 15, g = lane_w >> 4, lc = lane_w & 15, lrow0 = 4 * h + (lane_w >> 4);
    // this wave's DMA of the window landed: only the previous window's 18 output stores were
    // issued behind it and may stay in flight (the first window's DMA was retired before the loop;
    // tools/isa_lint.py R3 checks the count on every path of the shipped code object)
    asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    __syncthreads();
    // W_q / W_k of head h (A fragments: rows 16dt + r16 of the head, k = 32ks + 8g ..), L2-resident
    s16x8 wf[2][2][4];
#pragma unroll
    for (int part = 0; part < 2; ++part)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          wf[part][dt][ks] = __builtin_bit_cast(
              s16x8, ld16(p.w + (int64_t)(part * C + h * D + dt * 16 + r16) * C + ks * 32 + 8 * g));
    const int64_t gbase = GLIN ? rowmap(p.gmap, (int64_t)slice * (IMG * IMG)) : 0;
    auto fetch_g = [&](int t, int part, uint2 (&gd)[2]) {     // guidance of the q (0) or k (1) half
      const int row = win_row3(slice, wloc, 16 * t + r16, p.shift);
      const int64_t grow = GLIN ? gbase + (row - slice * (IMG * IMG)) : rowmap(p.gmap, row);
      const bf16* gp = p.g + grow * p.ld_g + part * C + h * D + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) gd[dt] = *reinterpret_cast<const uint2*>(gp + dt * 16);
    };
    uint2 gc[2];
    fetch_g(0, 1, gc);
    // ---------------- P1: LayerNorm of Xn in place, the 4 waves together ----------------
    {
      const float4 g0 = *reinterpret_cast<const float4*>(&sP[lc * 8]), g1 = *reinterpret_cast<const float4*>(&sP[lc * 8 + 4]);
      const float4 b0 = *reinterpret_cast<const float4*>(&sP[C + lc * 8]), b1 = *reinterpret_cast<const float4*>(&sP[C + lc * 8 + 4]);
      const float lg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float lb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int st_ = 0; st_ < LNS5; ++st_) {
        const int i = min(st_ * 16 + lrow0, L - 1);
        const uint4 raw = *reinterpret_cast<const uint4*>(&Xn[xs5(lc, i)]);
        const bf16* e = reinterpret_cast<const bf16*>(&raw);
        float v[8], sum = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[j] = bf2f(e[j]); sum += v[j]; }
        sum = row16_sum(sum);
        const float mean = sum * (1.f / C);
        float qs = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[j] -= mean; qs += v[j] * v[j]; }
        qs = row16_sum(qs);
        const float rstd = __builtin_amdgcn_rsqf(qs * (1.f / C) + p.eps);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] * rstd * lg[j] + lb[j];
        if (st_ * 16 + 4 * NW5 <= L || st_ * 16 + lrow0 < L)
          st16(&Xn[xs5(lc, i)], make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7])));
      }
    }
    __syncthreads();
    // ---------------- P2: k / v of head h for all 9 row tiles, then q, kept in registers ----------------
    // (two passes over Xn so that W_k is dead before q's pass and q's guidance is not held during k's)
    s16x8 qf[NTILE], kf[NTILE];
    uint2 vv[NTILE][2];                       // v of tokens 16t + 4g + r, feature 16dt + r16 (bf16 x 4)
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      uint2 gn[2];
      fetch_g(t + 1 < NTILE ? t + 1 : 0, t + 1 < NTILE ? 1 : 0, gn);   // the last prefetches q's tile 0
      __builtin_amdgcn_sched_barrier(0);      // keep the prefetch at the tile start
      asm volatile("" ::: "memory");          // W_v / bias fragments re-read per tile, not held across tiles
      const int rb = 16 * t;
      s16x8 xb[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) xb[ks] = *reinterpret_cast<const s16x8*>(&Xn[xs5(ks * 4 + g, rb + r16)]);
      f32x4 dk[2], dv[2];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        dk[dt] = *reinterpret_cast<const f32x4*>(&sP[3 * C + h * D + dt * 16 + 4 * g]) + unpack4(gc[dt]);
        const float bvv = sP[4 * C + h * D + dt * 16 + r16];
        dv[dt] = f32x4{bvv, bvv, bvv, bvv};
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dk[dt] = mfma_bf16(wf[1][dt][ks], xb[ks], dk[dt]);
          dv[dt] = mfma_bf16(xb[ks], *reinterpret_cast<const s16x8*>(&sWv[cs<C>(ks * 4 + g, h * D + dt * 16 + r16)]),
                             dv[dt]);
        }
      kf[t] = pk8(dk[0], dk[1]);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) vv[t][dt] = make_uint2(f2bf2(dv[dt][0], dv[dt][1]), f2bf2(dv[dt][2], dv[dt][3]));
      // pin the packed bf16 forms: left alone the conversions sink to the use in P3 and the f32
      // accumulators (twice the registers) stay live across the tiles
      asm volatile("" : "+v"(kf[t]), "+v"(vv[t][0]), "+v"(vv[t][1]));
      gc[0] = gn[0]; gc[1] = gn[1];
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      uint2 gn[2];
      if (t + 1 < NTILE) fetch_g(t + 1, 0, gn);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");          // W_v / bias fragments re-read per tile, not held across tiles
      const int rb = 16 * t;
      s16x8 xb[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) xb[ks] = *reinterpret_cast<const s16x8*>(&Xn[xs5(ks * 4 + g, rb + r16)]);
      f32x4 dq[2];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
        dq[dt] = *reinterpret_cast<const f32x4*>(&sP[2 * C + h * D + dt * 16 + 4 * g]) + unpack4(gc[dt]);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) dq[dt] = mfma_bf16(wf[0][dt][ks], xb[ks], dq[dt]);
      qf[t] = pk8(dq[0], dq[1]);
      asm volatile("" : "+v"(qf[t]));
      if (t + 1 < NTILE) { gc[0] = gn[0]; gc[1] = gn[1]; }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();                          // every wave is done with Xn
    if (win + (int)gridDim.x < nwin_total) fetch(win + gridDim.x);
    // ---------------- P3: attention of head h, 9 query tiles, K / V^T / Q from registers ----------------
    // (one instance per kernel: a hoisted per-window choice between a masked and an unmasked instance
    // produced wrong shifted-window outputs on the box and was not kept)
    auto attend = [&](auto mk) {
    constexpr bool MK = decltype(mk)::value;
#pragma unroll
    for (int j = 0; j < NTILE; ++j) {
      const int rb = 16 * j;
      asm volatile("" ::: "memory");          // the region one-hots are re-read per query tile
      // an opaque window location per tile: otherwise the output rows are CSE'd with P2's guidance rows
      // and carried (spilled) across P2, and the per-tile masks are hoisted out of the loop
      int wl = wloc;
      asm volatile("" : "+s"(wl));
      // B of the mask product: -100/scale at the regions other than the query's (k 0..3, lanes g = 0).
      // (The 16x16x16 form with 2-VGPR operands was intermittently wrong -- one wave's tile in ~1
      // launch of 5, tools/debug_swin_diff.py; hipcc allocated its destination over its A operand,
      // the K=16 bf16 MFMA defect DESIGN.md section 8 records for the ring conv.)
      s16x8 qmask;
      // window location 0 holds one region: its mask operand is zero (S + 0 is exact), which keeps
      // the tile free of a branch per key tile (branches split the MFMA / softmax schedule)
      if constexpr (MK) {
        const int qreg = local_region5(wl, rb + r16, p.shift);
#pragma unroll
        for (int e = 0; e < 8; ++e) qmask[e] = masked && g == 0 && e < 4 && e != qreg ? neg : (short)0;
      }
      f32x4 st[NTILE + 1];
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt) {
        f32x4 a = mfma_bf16(kf[kt], qf[j], f32x4{0.f, 0.f, 0.f, 0.f});
        if constexpr (MK)
          a = mfma_bf16(*reinterpret_cast<const s16x8*>(&Oh[(kt * 16 + r16) * 8]), qmask, a);
        st[kt] = a;
      }
      float mx = fmaxf(fmaxf(st[0][0], st[0][1]), fmaxf(st[0][2], st[0][3]));
#pragma unroll
      for (int kt = 1; kt < NTILE; ++kt) mx = fmaxf(mx, fmaxf(fmaxf(st[kt][0], st[kt][1]), fmaxf(st[kt][2], st[kt][3])));
      mx = xrow4_max(mx);
      const float nb = -mx * sl2;
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[kt][r] = __builtin_amdgcn_exp2f(fmaf(st[kt][r], sl2, nb));
      st[NTILE] = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, osum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < KBV / 32; ++u) {
        const s16x8 pb = pk8(st[2 * u], st[2 * u + 1]);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          // V^T fragment: keys 32u + 4g .. +3 (tile 2u) and 32u + 16 + 4g .. +3 (tile 2u + 1), feature 16dt + r16
          const uint2 lo = vv[2 * u][dt];
          const uint2 hi = 2 * u + 1 < NTILE ? vv[2 * u + 1][dt] : make_uint2(0u, 0u);
          o[dt] = mfma_bf16(__builtin_bit_cast(s16x8, make_uint4(lo.x, lo.y, hi.x, hi.y)), pb, o[dt]);
        }
        osum = mfma_bf16(ones, pb, osum);
      }
      const float inv = 1.f / osum[0];
      const int64_t oe = (int64_t)win_row3(slice, wl, rb + r16, p.shift) * p.ld_out + h * D;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const uint2 val = make_uint2(f2bf2(o[dt][0] * inv, o[dt][1] * inv), f2bf2(o[dt][2] * inv, o[dt][3] * inv));
        if constexpr (WT) st8_wt(p.out, (oe + dt * 16 + 4 * g) * 2, val);
        else *reinterpret_cast<uint2*>(p.out + oe + dt * 16 + 4 * g) = val;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    };
    attend(std::integral_constant<bool, SWM>{});
  }
}

}  // namespace

int g_swin_store = 0;   // swin_win5 output stores: 0 = plain, 1 = sc1 write-through (A/B knob; same box, whole step 9.251 -> 9.356 ms: slower)
CATSEG_KNOB(g_swin_store, "swin_store");

// launched by catseg_swin_window_attention (swin_fused.hip) after its argument checks
int swin_win3_launch(const CatsegSwinAttnArgs* a, int n_cu, hipStream_t st, bool glin) {
  Swin3P p;
  p.glin = glin ? 1 : 0;
  p.x = (const bf16*)a->x; p.ld_x = a->ld_x;
  p.ln_g = a->ln_g; p.ln_b = a->ln_b; p.eps = a->eps;
  p.w = (const bf16*)a->w_qkv; p.bias = a->b_qkv;
  p.g = (const bf16*)a->gqk; p.ld_g = a->ld_g;
  p.gmap = RowMap{a->gmap.d1, a->gmap.m1, a->gmap.s1, a->gmap.d2, a->gmap.m2, a->gmap.s2, a->gmap.off};
  p.out = (bf16*)a->out; p.ld_out = a->ld_out;
  p.shift = a->shift; p.scale = a->scale;
  p.wt = 0;
  const int nwin_total = (int)(a->S * NWIN);
  const dim3 grid((unsigned)std::min(nwin_total, n_cu));
  if (a->shift > 0) hipLaunchKernelGGL((swin_win3_kernel<true>), grid, dim3(NT), 0, st, p, nwin_total);
  else hipLaunchKernelGGL((swin_win3_kernel<false>), grid, dim3(NT), 0, st, p, nwin_total);
  return 0;
}

// two 4-wave workgroups per CU, the grid a multiple of the 4 window locations
int swin_win5_launch(const CatsegSwinAttnArgs* a, int n_cu, hipStream_t st, bool glin) {
  Swin3P p;
  p.glin = glin ? 1 : 0;
  p.x = (const bf16*)a->x; p.ld_x = a->ld_x;
  p.ln_g = a->ln_g; p.ln_b = a->ln_b; p.eps = a->eps;
  p.w = (const bf16*)a->w_qkv; p.bias = a->b_qkv;
  p.g = (const bf16*)a->gqk; p.ld_g = a->ld_g;
  p.gmap = RowMap{a->gmap.d1, a->gmap.m1, a->gmap.s1, a->gmap.d2, a->gmap.m2, a->gmap.s2, a->gmap.off};
  p.out = (bf16*)a->out; p.ld_out = a->ld_out;
  p.shift = a->shift; p.scale = a->scale;
  p.wt = g_swin_store && a->S * 576 * a->ld_out * 2 < 0x7fffffffLL;
  const int nwin_total = (int)(a->S * NWIN);
  const dim3 grid((unsigned)std::min(nwin_total, (2 * n_cu) / NWIN * NWIN));
  // only for guidance rows that are one base + the pixel per slice (every engine call; the caller
  // sends other row maps to swin_win3).  The general-row-map instance spilled 19-23 VGPRs and gave
  // wrong shifted-window outputs on the box, so it is not instantiated.
  if (!glin) return -1;
  if (p.wt) {
    if (a->shift > 0) hipLaunchKernelGGL((swin_win5_kernel<true, true, true>), grid, dim3(NT5), 0, st, p, nwin_total);
    else hipLaunchKernelGGL((swin_win5_kernel<false, true, true>), grid, dim3(NT5), 0, st, p, nwin_total);
    return 0;
  }
  if (a->shift > 0) hipLaunchKernelGGL((swin_win5_kernel<true, true>), grid, dim3(NT5), 0, st, p, nwin_total);
  else hipLaunchKernelGGL((swin_win5_kernel<false, true>), grid, dim3(NT5), 0, st, p, nwin_total);
  return 0;
}
