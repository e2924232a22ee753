// Class attention, register-resident form (bf16): one pixel per 4-wave workgroup at a time,
// one wave per head, two workgroups per CU (catseg_class_attention): norm1 + [q|k|v] projection (+ the per-class text-guidance half
// of q, k) + linear attention over the T classes of a pixel + the attention residual.
// Reference: ClassTransformerLayer.forward model.py:387-413, AttentionLayer.forward
// model.py:338-354, LinearAttention.forward model.py:256-286 (phi = elu + 1, V / S, KV, Z, * S).
//
// Per pixel:
//   LN    all 4 waves: the pixel's T class rows (16 lanes per 256-byte row) -> LayerNorm ->
//         bf16 rows in LDS, XOR-swizzled 16-byte chunks (conflict-free fragment reads);
//         rows T..Tpad-1 are zero.
//   A     wave h, per pair of 16-row class tiles:
//           D_k[t][i] = xn W_k^T, D_v[t][j] = xn W_v^T (W_k, W_v rows of head h held in
//           registers), + bias, + guidance (k); phi(k) (rows >= T -> 0)
//           KV_h[i][j] += phi(K)^T V and ksum_h[i] += phi(K)^T 1 on the MFMA with the MFMA
//           output tiles used directly as operands: a lane holds rows t = 4q..4q+3 of both
//           tiles for one column, which is an 8-deep k-slice of the next MFMA (the k order
//           inside an MFMA is free when both operands share it) -- no LDS transpose.
//         + the learned padding term n_pad * phi(k_pad) (x) [v_pad | 1], KV / S, then KV as
//         bf16 hi + lo operands (~16-bit mantissa).
//   B     wave h, per 16-row class tile: D_q^T[i][t] = W_q xn^T + bias + guidance -> phi;
//         z[t] = phi(q) . ksum (fp32, 4-lane reduction); O^T[j][t] = KV^T phi(q)^T (hi + lo);
//         y = x + O * S / (z + eps), 8-byte stores of the head's 32 channels.
// q, k, v, KV never leave the CU; HBM traffic per pixel: its rows read once (+ the residual
// re-read of the same rows, L2-hot) and written once, plus guidance rows (L2-resident).
#include "common.h"
#include "capi.h"

namespace {

constexpr int C = 128, D = 32, NH = 4;
constexpr int NT = NH * 64;                 // 4 waves, one per head
constexpr int TMAX = 256;                   // class rows per pixel (pad_len bounds T)

struct Cls2P {
  const bf16* x; int64_t ld_x;
  const float* ln_g; const float* ln_b; float eps;
  const bf16* w; const float* bias;         // [384][128] (q, k, v rows), [384]
  const bf16* tg; int64_t ld_tg; int64_t tg_bstride;   // [.][256]: q half | k half
  const bf16* tgkT; int ld_tgkT; int64_t tgkT_bstride;  // k half transposed [128][ld] per image
  const float* k_pad; const float* v_pad; int n_pad; float attn_eps;
  bf16* y; int64_t ld_y;
  int64_t B; int T; int HW;
  int wt;        // output rows through sc1 write-through stores (cls_store knob)
  int dbg;       // diagnostics (catseg_set_classattn_variant(16 + bits)): 1 = LN rows all row 0, 2 = stage-B rows all row 0
};

DEV float phi(float v) { return v > 0.f ? v + 1.f : __expf(v); }   // elu(v) + 1
DEV int xoff(int t, int ch) { return (t * 16 + (ch ^ (t & 15))) * 8; }   // xn element offset of 16-B chunk ch
DEV s16x8 pack8(const f32x4& a, const f32x4& b) {
  const unsigned u0 = f2bf2(a[0], a[1]), u1 = f2bf2(a[2], a[3]), u2 = f2bf2(b[0], b[1]), u3 = f2bf2(b[2], b[3]);
  return __builtin_bit_cast(s16x8, make_uint4(u0, u1, u2, u3));
}
DEV float ushort_f(const bf16* p) { return bf2f(*p); }

// LNB: LayerNorm row steps (16 rows each) loaded per batch
// SB: the q / k / v biases read from LDS where used instead of held in 12 VGPRs (the kernel sits at
// 256 VGPRs; its spill reloads, counted in vmcnt, drained the in-flight prefetches)
template <int LNB, bool SB = true>
__global__ __launch_bounds__(NT, 2) void classattn2_kernel(Cls2P a) {
  __shared__ __attribute__((aligned(16))) bf16 xn[TMAX * C];
  __shared__ __attribute__((aligned(16))) float sbias[SB ? 3 * C : 4];   // q | k | v bias
  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;

  // ---- head h's weights as MFMA fragments (lane: row r16 of a 16-row block, k 8q..8q+7) ----
  s16x8 wq[2][4], wk[2][4], wv[2][4];
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int64_t col = ks * 32 + 8 * q, row = h * D + ib * 16 + r16;
      wq[ib][ks] = *reinterpret_cast<const s16x8*>(a.w + row * C + col);
      wk[ib][ks] = *reinterpret_cast<const s16x8*>(a.w + (C + row) * C + col);
      wv[ib][ks] = *reinterpret_cast<const s16x8*>(a.w + (2 * C + row) * C + col);
    }
  // biases in registers (a load inside the tile loops would wait, in vmcnt order, for the
  // prefetches issued before it); LayerNorm affine and padding projections are read where used
  float bk[2], bv[2];
  f32x4 bq[2];
  if constexpr (SB) {
    for (int i = tid; i < 3 * C; i += NT) sbias[i] = a.bias[i];   // first read after the LN barrier
  } else {
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      bk[ib] = a.bias[C + h * D + ib * 16 + r16];
      bv[ib] = a.bias[2 * C + h * D + ib * 16 + r16];
      bq[ib] = *reinterpret_cast<const f32x4*>(a.bias + h * D + ib * 16 + 4 * q);
    }
  }
  const float S = (float)(a.T + a.n_pad), invS = 1.f / S;

  const int T = a.T, HW = a.HW;
  const int ntile = (T + 15) >> 4;
  const int npix = (int)(a.B * HW);          // < 2^31 (host-checked)
  const int lr = tid >> 4, lc = tid & 15;    // LN: row within a 16-row step, 16-byte chunk
  uint64_t* stamps = reinterpret_cast<uint64_t*>(a.y) + (int64_t)blockIdx.x * 64;   // dbg & 4 only
  const bool stamp = (a.dbg & 4) && tid == 0;
  int it = 0;
  for (int pix = blockIdx.x; pix < npix; pix += gridDim.x, ++it) {
    const int b = (unsigned)pix / (unsigned)HW, p = pix - b * HW;
    if (stamp && it < 8) stamps[it * 4 + 0] = __builtin_amdgcn_s_memtime();
    const bf16* xrow0 = a.x + ((int64_t)b * T * HW + p) * a.ld_x;          // row t at + t*HW*ld_x
    bf16* yrow0 = a.y + ((int64_t)b * T * HW + p) * a.ld_y;
    const int xs = HW * (int)a.ld_x, ys = HW * (int)a.ld_y, ldg = (int)a.ld_tg;   // 32-bit offsets (host-checked)
    const bf16* tgb = a.tg + (int64_t)b * a.tg_bstride * a.ld_tg;
    const bf16* tkb = a.tgkT + (int64_t)b * a.tgkT_bstride;

    // ---------------- LN: rows -> xn (8 steps of 16 rows in flight per batch) ----------------
    // loads are unconditional (rows past T re-read row T-1, values dropped): a per-row
    // conditional load makes hipcc wait for each load in turn
    for (int t0 = 0; t0 < ntile * 16; t0 += LNB * 16) {
      uint4 u[LNB];
#pragma unroll
      for (int s = 0; s < LNB; ++s) {
        const int t = (a.dbg & 1) ? 0 : min(t0 + 16 * s + lr, T - 1);
        u[s] = ld16(xrow0 + t * xs + lc * 8);
      }
      const float4 g0 = *reinterpret_cast<const float4*>(a.ln_g + lc * 8), g1 = *reinterpret_cast<const float4*>(a.ln_g + lc * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(a.ln_b + lc * 8), b1 = *reinterpret_cast<const float4*>(a.ln_b + lc * 8 + 4);
      const float lg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float lb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int s = 0; s < LNB; ++s) {
        const int t = t0 + 16 * s + lr;
        // rows T..Tpad-1 hold the LayerNorm of row T-1 (finite); stage A zeroes their phi(k)
        // and v, stage B does not store them
        const bf16* e = reinterpret_cast<const bf16*>(&u[s]);
        float v[8], sum = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[j] = bf2f(e[j]); sum += v[j]; }
        sum = row16_sum(sum);
        const float mean = sum * (1.f / C);
        float qs = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[j] -= mean; qs += v[j] * v[j]; }
        qs = row16_sum(qs);
        const float rstd = __builtin_amdgcn_rsqf(qs * (1.f / C) + a.eps);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] * rstd * lg[j] + lb[j];
        if (t0 + 16 * s < ntile * 16)                 // uniform: steps past the last tile are dropped
          st16(&xn[xoff(t, lc)], make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7])));
      }
    }
    __syncthreads();
    if (stamp && it < 8) stamps[it * 4 + 1] = __builtin_amdgcn_s_memtime();

    // ---------------- A: KV_h, ksum_h over the class tiles ----------------
    // ksum_h[i] = sum_t phi(k)[t][i] in fp32 on the VALU: each lane sums its rows of column
    // i = ib*16 + r16, the 4 row groups q are folded once per pixel
    f32x4 kv[2][2];
    float kcol[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) kv[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto fetchk = [&](int tp, uint2 (*gk)[2]) {
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        const bf16* gcol = tkb + (h * D + ib * 16 + r16) * a.ld_tgkT + 16 * tp + 4 * q;
        gk[ib][0] = *reinterpret_cast<const uint2*>(gcol);
        gk[ib][1] = *reinterpret_cast<const uint2*>(gcol + (tp + 1 < ntile ? 16 : 0));
      }
    };
    // one pair of 16-row class tiles; g = its guidance, fetched one pair ahead into the other
    // of two register buffers (unrolled by two: no register copy waits for a prefetch)
    auto pair = [&](int tp, const uint2 (&g)[2][2]) {
      const bool two = tp + 1 < ntile;
      // accumulators start at bias + guidance: k rows t = 16(tp+tt) + 4q + r of column
      // i = h*32 + ib*16 + r16 (4 consecutive t in the transposed guidance: one 8-byte load)
      f32x4 dk[2][2], dv[2][2];
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const float bkk = SB ? sbias[C + h * D + ib * 16 + r16] : bk[ib];
          const float bvv = SB ? sbias[2 * C + h * D + ib * 16 + r16] : bv[ib];
          dk[tt][ib] = f32x4{__uint_as_float(g[ib][tt].x << 16) + bkk, __uint_as_float(g[ib][tt].x & 0xffff0000u) + bkk,
                             __uint_as_float(g[ib][tt].y << 16) + bkk, __uint_as_float(g[ib][tt].y & 0xffff0000u) + bkk};
          dv[tt][ib] = f32x4{bvv, bvv, bvv, bvv};
        }
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) {
        s16x8 xa[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
          xa[tt] = two || tt == 0 ? *reinterpret_cast<const s16x8*>(&xn[xoff(16 * (tp + tt) + r16, kq * 4 + q)])
                                  : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int ib = 0; ib < 2; ++ib) {
            dk[tt][ib] = mfma_bf16(xa[tt], wk[ib][kq], dk[tt][ib]);
            dv[tt][ib] = mfma_bf16(xa[tt], wv[ib][kq], dv[tt][ib]);
          }
      }
      // phi(k) with rows >= T zeroed; v + bias.  Operand k-slot 8q+r <-> t = 16tp + 4q + r,
      // 8q+4+r <-> t = 16(tp+1) + 4q + r (the same map for the K and V operands)
      s16x8 ak[2], bvv[2];
      const bool full = 16 * tp + 32 <= T;     // uniform: only the last pair has rows past T
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        f32x4 k0, k1, v0 = dv[0][ib], v1 = dv[1][ib];
#pragma unroll
        for (int r = 0; r < 4; ++r) { k0[r] = phi(dk[0][ib][r]); k1[r] = phi(dk[1][ib][r]); }
        if (!full) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t0 = 16 * tp + 4 * q + r, t1 = t0 + 16;
            k0[r] = t0 < T ? k0[r] : 0.f;
            k1[r] = t1 < T ? k1[r] : 0.f;
            v1[r] = t1 < T ? v1[r] : 0.f;
          }
        }
        kcol[ib] += (k0[0] + k0[1]) + (k0[2] + k0[3]) + ((k1[0] + k1[1]) + (k1[2] + k1[3]));
        ak[ib] = pack8(k0, k1);
        bvv[ib] = pack8(v0, v1);
      }
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) kv[ib][jb] = mfma_bf16(ak[ib], bvv[jb], kv[ib][jb]);
      }
    };
    uint2 gA[2][2], gB[2][2];
    fetchk(0, gA);
    for (int tp = 0; tp < ntile; tp += 4) {
      if (tp + 2 < ntile) fetchk(tp + 2, gB);
      pair(tp, gA);
      if (tp + 2 < ntile) {
        if (tp + 4 < ntile) fetchk(tp + 4, gA);
        pair(tp + 2, gB);
      }
    }
    // padding tokens, V / S, KV^T operands hi + lo: A-operand slot 8q+r <-> key row 4q + r of
    // block 0, 8q+4+r <-> block 1; lane row = value channel jb*16 + r16
    // (model.py:397-410): key rows i = ib*16 + 4q + r, value column j = jb*16 + r16
    f32x4 kp[2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        kp[ib][r] = a.n_pad > 0 ? (float)a.n_pad * phi(a.k_pad[h * D + ib * 16 + 4 * q + r]) : 0.f;
    s16x8 khi[2], klo[2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      const float vp = a.n_pad > 0 ? a.v_pad[h * D + jb * 16 + r16] : 0.f;
      f32x4 hv[2], lv[2];
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = (kv[ib][jb][r] + kp[ib][r] * vp) * invS;
          hv[ib][r] = bf2f(f2bf(x));
          lv[ib][r] = x - hv[ib][r];
        }
      khi[jb] = pack8(hv[0], hv[1]);
      klo[jb] = pack8(lv[0], lv[1]);
    }
    // ksum in the KV row layout (rows i = ib*16 + 4q + r per lane) + the padding term
    f32x4 ks[2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const float col = xrow4_sum(kcol[ib]);          // ksum[ib*16 + r16] in every lane of column r16
#pragma unroll
      for (int r = 0; r < 4; ++r) ks[ib][r] = __shfl(col, 4 * q + r, 64) + kp[ib][r];
    }

    if (stamp && it < 8) stamps[it * 4 + 2] = __builtin_amdgcn_s_memtime();
    // ---------------- B: queries, output, residual ----------------
    // the next tile's q-guidance and residual rows are fetched one tile ahead (rows past T clamp)
    // the residual rows as 16-byte loads: lane pair (q, q ^ 1) of a row reads the head's channels
    // 8 (q & 2) + 16 (q & 1) .. +7 (the 4 + 4 that the even lane's jb = 0 and the odd lane's jb = 1
    // need, plus their partner's) and swaps halves; 64-byte segments per row instead of 32
    const int xcol = (q & 1) ? 12 + 4 * q : 4 * q;       // q = 0, 1, 2, 3 -> channels 0, 16, 8, 24
    auto fetch = [&](int tt, uint2* g, uint2* xr) {
      const int t = (a.dbg & 2) ? 0 : min(16 * tt + r16, T - 1);
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
        g[ib] = *reinterpret_cast<const uint2*>(tgb + t * ldg + h * D + ib * 16 + 4 * q);
      const uint4 w = *reinterpret_cast<const uint4*>(xrow0 + t * xs + h * D + xcol);
      // even q holds channels 4q .. 4q+7 (its jb = 0 half, then the odd partner's); odd q holds
      // 16 + 4(q-1) .. +7 (the even partner's jb = 1 half, then its own)
      const uint2 mine = (q & 1) ? make_uint2(w.z, w.w) : make_uint2(w.x, w.y);
      const uint2 give = (q & 1) ? make_uint2(w.x, w.y) : make_uint2(w.z, w.w);
      const uint2 got = make_uint2((unsigned)__shfl_xor((int)give.x, 16, 64), (unsigned)__shfl_xor((int)give.y, 16, 64));
      xr[0] = (q & 1) ? got : mine;
      xr[1] = (q & 1) ? mine : got;
    };
    auto tile = [&](int tt, const uint2 (&gq)[2], const uint2 (&xr)[2]) {
      const int t = 16 * tt + r16;            // this lane's class row
      // q^T accumulators start at bias + guidance: lane rows i = ib*16 + 4q + r of column t
      f32x4 dq[2];
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
        dq[ib] = f32x4{__uint_as_float(gq[ib].x << 16), __uint_as_float(gq[ib].x & 0xffff0000u),
                       __uint_as_float(gq[ib].y << 16), __uint_as_float(gq[ib].y & 0xffff0000u)} +
                (SB ? *reinterpret_cast<const f32x4*>(&sbias[h * D + ib * 16 + 4 * q]) : bq[ib]);
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) {
        const s16x8 xb = *reinterpret_cast<const s16x8*>(&xn[xoff(t, kq * 4 + q)]);
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) dq[ib] = mfma_bf16(wq[ib][kq], xb, dq[ib]);
      }
      f32x4 pq[2];
      float zp = 0.f;
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pq[ib][r] = phi(dq[ib][r]);
          zp += pq[ib][r] * ks[ib][r];
        }
      const float z = xrow4_sum(zp);
      const s16x8 bq8 = pack8(pq[0], pq[1]);
      const float sc = S * __builtin_amdgcn_rcpf(z + a.attn_eps);
      f32x4 o[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {        // full-wave MFMAs; only the stores are masked
        o[jb] = mfma_bf16(khi[jb], bq8, f32x4{0.f, 0.f, 0.f, 0.f});
        o[jb] = mfma_bf16(klo[jb], bq8, o[jb]);
      }
      uint2 yv[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        // o[jb][r] = O[t][j = jb*16 + 4q + r]
        const float xv[4] = {__uint_as_float(xr[jb].x << 16), __uint_as_float(xr[jb].x & 0xffff0000u),
                             __uint_as_float(xr[jb].y << 16), __uint_as_float(xr[jb].y & 0xffff0000u)};
        yv[jb] = make_uint2(f2bf2(xv[0] + o[jb][0] * sc, xv[1] + o[jb][1] * sc),
                            f2bf2(xv[2] + o[jb][2] * sc, xv[3] + o[jb][3] * sc));
      }
      // one 16-byte store per lane: the pair (q, q ^ 1) swaps halves so that it holds 8 consecutive
      // channels (the same layout as the residual load above); the swap runs on every lane
      const uint2 give = (q & 1) ? yv[0] : yv[1];
      const uint2 got = make_uint2((unsigned)__shfl_xor((int)give.x, 16, 64), (unsigned)__shfl_xor((int)give.y, 16, 64));
      if (t < T) {
        const uint4 w = (q & 1) ? make_uint4(got.x, got.y, yv[1].x, yv[1].y) : make_uint4(yv[0].x, yv[0].y, got.x, got.y);
        bf16* dst = yrow0 + ((a.dbg & 2) ? 0 : t) * ys + h * D + xcol;
        if (a.wt) st16_wt(a.y, (dst - a.y) * 2, w);
        else *reinterpret_cast<uint4*>(dst) = w;
      }
    };
    uint2 gqA[2], xrA[2], gqB[2], xrB[2];
    fetch(0, gqA, xrA);
    for (int tt = 0; tt < ntile; tt += 2) {
      if (tt + 1 < ntile) fetch(tt + 1, gqB, xrB);
      tile(tt, gqA, xrA);
      if (tt + 1 < ntile) {
        if (tt + 2 < ntile) fetch(tt + 2, gqA, xrA);
        tile(tt + 1, gqB, xrB);
      }
    }
    if (stamp && it < 8) stamps[it * 4 + 3] = __builtin_amdgcn_s_memtime();
    __syncthreads();                          // xn is rewritten for the next pixel
  }
}

}  // namespace

// >= 16: diagnostics (dbg = v - 16: LN / stage-B rows all row 0, phase stamps); 0 = default
int g_classattn_variant = 0;
CATSEG_KNOB(g_classattn_variant, "classattn_variant");
int g_cls_store = 0;   // class attention output stores: 0 = plain, 1 = sc1 write-through (A/B knob; same box, whole step 9.250 -> 9.280 ms)
CATSEG_KNOB(g_cls_store, "cls_store");

extern "C" int catseg_class_attention(const CatsegClassAttnArgs* a, void* stream) {
  CATSEG_CHECK(a && a->x && a->w_qkv && a->b_qkv && a->ln_g && a->ln_b && a->tg && a->y && a->tgk_t,
               "class_attention: null pointer");
  CATSEG_CHECK(a->dtype == CATSEG_BF16, "class_attention: bf16 only");
  CATSEG_CHECK(a->n_heads == NH && a->head_dim == D, "class_attention: needs 4 heads x 32");
  CATSEG_CHECK(a->B > 0 && a->T > 0 && a->HW > 0, "class_attention: empty shape");
  CATSEG_CHECK(a->T <= TMAX, "class_attention: T must be <= 256 (the class padding length)");
  CATSEG_CHECK(a->n_pad >= 0 && (a->n_pad == 0 || (a->k_pad && a->v_pad)), "class_attention: padding projections missing");
  CATSEG_CHECK(a->ld_x % 8 == 0 && a->ld_y % 8 == 0 && a->ld_tg % 8 == 0 && a->ld_x >= C && a->ld_y >= C &&
               a->ld_tg >= 2 * C, "class_attention: row strides must be multiples of 8 elements");
  CATSEG_CHECK(a->tg_bstride >= 0, "class_attention: bad guidance image stride");
  CATSEG_CHECK(a->x != a->y, "class_attention: y must not alias x");
  CATSEG_CHECK(a->B * a->T * (int64_t)a->HW * std::max(a->ld_x, a->ld_y) < (1LL << 31) &&
               (int64_t)a->T * a->ld_tg < (1LL << 31), "class_attention: element offsets must fit 31 bits");
  CATSEG_CHECK(a->ld_tgk_t >= (a->T + 15) / 16 * 16 && a->ld_tgk_t % 4 == 0 && ((uintptr_t)a->tgk_t % 8) == 0,
               "class_attention: tgk_t rows must hold round_up(T, 16) entries, 8-byte aligned");
  Cls2P p;
  p.x = (const bf16*)a->x; p.ld_x = a->ld_x;
  p.ln_g = a->ln_g; p.ln_b = a->ln_b; p.eps = a->eps;
  p.w = (const bf16*)a->w_qkv; p.bias = a->b_qkv;
  p.tg = (const bf16*)a->tg; p.ld_tg = a->ld_tg; p.tg_bstride = a->tg_bstride;
  p.tgkT = (const bf16*)a->tgk_t; p.ld_tgkT = (int)a->ld_tgk_t; p.tgkT_bstride = a->tgk_t_bstride;
  p.k_pad = a->k_pad; p.v_pad = a->v_pad; p.n_pad = a->n_pad; p.attn_eps = a->attn_eps;
  p.y = (bf16*)a->y; p.ld_y = a->ld_y;
  p.B = a->B; p.T = a->T; p.HW = a->HW;
  p.dbg = g_classattn_variant >= 16 ? g_classattn_variant - 16 : 0;
  p.wt = g_cls_store && a->B * a->T * (int64_t)a->HW * a->ld_y * 2 < 0x7fffffffLL;
  const int cus = catseg_device_cus();
  const int64_t npix = a->B * a->HW;
  const unsigned grid = (unsigned)std::min<int64_t>(npix, 2LL * cus);
  hipStream_t st = (hipStream_t)stream;
  // LayerNorm batch = the pixel's class tiles when they fit one batch of <= 10 (T = 150: one HBM round
  // trip per pixel instead of 8 + 2 steps: 271 -> 258 us, same box), else 8 per batch
  const int ntile = (a->T + 15) / 16;
  if (ntile <= 4) hipLaunchKernelGGL(classattn2_kernel<4>, dim3(grid), dim3(NT), 0, st, p);
  else if (ntile <= 10) hipLaunchKernelGGL(classattn2_kernel<10>, dim3(grid), dim3(NT), 0, st, p);
  else hipLaunchKernelGGL(classattn2_kernel<8>, dim3(grid), dim3(NT), 0, st, p);
  return catseg_launch_status("class_attention");
}
