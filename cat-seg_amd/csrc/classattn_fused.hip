// Fused class attention for the CAT-Seg class aggregation (bf16):
//   LayerNorm(norm1) + [q|k|v] projection (+ the per-class text-guidance half of q, k)
//   + linear attention over the T classes of a pixel + the attention residual.
// Reference: ClassTransformerLayer.forward model.py:387-413 (norm1, padding, guidance
// repeat, x_pool + attention), AttentionLayer.forward model.py:338-354 (q, k from
// [x | guidance], v from x, no output projection) and LinearAttention.forward
// model.py:256-286 (phi = elu + 1, V / S, KV, Z, * S).
//
// One persistent 8-wave workgroup per CU walks pixels.  A pixel's sequence is its T
// class rows (b*T + t)*HW + p, taken in 32-row chunks, in two passes:
//   pass 1  LN -> [k | v] by MFMA -> phi(k), v transposed into LDS -> KV_h += phi(K_h)^T V_h
//           on the MFMA, with a ones column appended to V so the same MFMA yields
//           ksum_h = sum_t phi(k_t,h) (KV accumulators stay in registers over the chunks);
//           then the learned-padding term n_pad * phi(k_pad) (x) [v_pad | 1] and the 1/S
//           scale, and KV_h goes to LDS as a bf16 hi + lo pair (~16-bit mantissa).
//   pass 2  LN -> q by MFMA -> phi(q) -> [num | z] = phi(q_h) . [KV_h | ksum_h] on the MFMA
//           -> y = x + num * S / (z + eps), 16-byte row stores.
// q/k/v never reach HBM: traffic per pixel is its rows read twice (the second pass from
// L2) and written once, plus the per-class guidance rows (L2-resident).
#include "common.h"
#include "capi.h"

namespace {

constexpr int C = 128, D = 32, NH = 4;
constexpr int NW = 8, NT = NW * 64;
constexpr int BM = 32;                 // class rows per chunk
constexpr int LDT = BM + 8;            // transposed phi(K) / V rows [channel][t]
constexpr int LDG = C + 8;             // guidance rows [t][128]
constexpr int LDQ = C + 8;             // phi(Q) rows [t][128]
constexpr int LDO = C + 4;             // fp32 attention output rows [t][128]
constexpr int KVR = D + 1;             // KV^T rows per head: 32 value channels + ksum
constexpr int LDK = D + 8;             // KV^T row stride (i = key channel contiguous)

struct ClsP {
  const bf16* x; int64_t ld_x;
  const float* ln_g; const float* ln_b; float eps;
  const bf16* w; const float* bias;      // [384][128] bf16, [384]
  const bf16* tg; int64_t ld_tg; int64_t tg_bstride;
  const float* k_pad; const float* v_pad; int n_pad; float attn_eps;
  bf16* y; int64_t ld_y;
  int64_t B; int T; int HW;
};

template <int ROWS>
DEV int cslot(int c, int r) { return (c * ROWS + (r ^ (c & 15))) * 8; }

DEV float phi(float v) { return v > 0.f ? v + 1.f : __expf(v); }   // elu(v) + 1

struct __attribute__((aligned(16))) Smem {
  bf16 xn[BM * C];                     // LayerNorm'd chunk rows (chunk-major, swizzled)
  bf16 tg[BM * LDG];                   // guidance half of this pass for the chunk rows
  union {
    struct { bf16 kt[C * LDT]; bf16 vt[C * LDT]; } p1;   // pass 1: phi(K)^T, V^T
    struct { bf16 q[BM * LDQ]; float o[BM * LDO]; } p2;  // pass 2: phi(Q), output
  } u;
  bf16 kv[2][NH * KVR * LDK];          // KV^T (+ ksum row) hi / lo
};

__global__ __launch_bounds__(NT, 2) void classattn_kernel(ClsP a) {
  __shared__ Smem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int lr = tid >> 4, lc = tid & 15;          // loader: chunk row, 16-byte column chunk

  // ---- weights in registers (MFMA operand fragments), loaded once ----
  // pass 1: wave w owns k/v output columns 128 + 32w .. +32 (waves 0-3: k, 4-7: v)
  // pass 2: wave w owns q output columns 16w .. +16
  s16x8 wkv[2][4], wq[4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      wkv[i][ks] = *reinterpret_cast<const s16x8*>(a.w + (int64_t)(C + 32 * wave + 16 * i + r16) * C + ks * 32 + 8 * q);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    wq[ks] = *reinterpret_cast<const s16x8*>(a.w + (int64_t)(16 * wave + r16) * C + ks * 32 + 8 * q);
  float bkv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) bkv[i] = a.bias[C + 32 * wave + 16 * i + r16];
  const float4 bq = *reinterpret_cast<const float4*>(a.bias + 16 * wave + 4 * q);

  const int T = a.T, HW = a.HW;
  const int nc = (T + BM - 1) / BM;
  const int npix = (int)(a.B * HW);                    // < 2^31 (host-checked)
  const int G = gridDim.x;
  const float S = (float)(T + a.n_pad);
  const bool kwave = wave < 4;

  // chunk walk: pixel blockIdx.x + k*G; pass 0 chunks 0..nc-1, then pass 1 chunks 0..nc-1.
  // The loader runs one step ahead on its own cursor (no divisions in the loop).
  struct Cursor { int pix, pass, c; };
  auto advance = [&](Cursor& u) {
    if (++u.c == nc) { u.c = 0; if (++u.pass == 2) { u.pass = 0; u.pix += G; } }
  };
  auto load = [&](const Cursor& u, uint4& ux, uint4& ug) {
    const int b = (unsigned)u.pix / (unsigned)HW, p = u.pix - b * HW;
    const int t = u.c * BM + lr;
    if (u.pix < npix && t < T) {
      ux = ld16(a.x + ((int64_t)(b * T + t) * HW + p) * a.ld_x + lc * 8);
      ug = ld16(a.tg + ((int64_t)b * a.tg_bstride + t) * a.ld_tg + (u.pass ? 0 : C) + lc * 8);
    } else {
      ux = make_uint4(0, 0, 0, 0);
      ug = make_uint4(0, 0, 0, 0);
    }
  };

  Cursor cur{(int)blockIdx.x, 0, 0}, nxt = cur;
  uint4 nx = make_uint4(0, 0, 0, 0), ng = nx;
  load(nxt, nx, ng);
  advance(nxt);
  f32x4 kvacc[3];
  for (; cur.pix < npix; advance(cur)) {
    const int pass = cur.pass, c = cur.c, pix = cur.pix;
    const uint4 xc = nx;
    {
      // LayerNorm of the chunk rows (16 lanes per row) into the MFMA image; guidance rows
      uint4 u = xc;
      bf16* e = reinterpret_cast<bf16*>(&u);
      float v[8], sum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[j] = bf2f(e[j]); sum += v[j]; }
      sum = row16_sum(sum);
      const float mean = sum * (1.f / C);
      float qs = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[j] -= mean; qs += v[j] * v[j]; }
      qs = row16_sum(qs);
      const float rstd = rsqrtf(qs * (1.f / C) + a.eps);
      {
        const float4 g0 = *reinterpret_cast<const float4*>(a.ln_g + lc * 8), g1 = *reinterpret_cast<const float4*>(a.ln_g + lc * 8 + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(a.ln_b + lc * 8), b1 = *reinterpret_cast<const float4*>(a.ln_b + lc * 8 + 4);
        const float lg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        const float lb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] * rstd * lg[j] + lb[j];
      }
      st16(&sm.xn[cslot<BM>(lc, lr)], make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]),
                                                  f2bf2(v[6], v[7])));
      st16(&sm.tg[lr * LDG + lc * 8], ng);
    }
    if (pass == 0 && c == 0) {
#pragma unroll
      for (int f = 0; f < 3; ++f) kvacc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();                                                           // B1
    load(nxt, nx, ng);                                                         // prefetch the next chunk
    advance(nxt);

    if (pass == 0) {
      // ---- [k | v] = LN(x) W^T + b (+ guidance on k): D[t][n], lane = 4 rows t of one column n
      f32x4 acc[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s16x8 xf[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) xf[j] = *reinterpret_cast<const s16x8*>(&sm.xn[cslot<BM>(ks * 4 + q, 16 * j + r16)]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(xf[j], wkv[i][ks], acc[i][j]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int cc = 32 * (wave & 3) + 16 * i + r16;          // channel within k or v
        bf16* dst = kwave ? sm.u.p1.kt : sm.u.p1.vt;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t = 16 * j + 4 * q + r;
            float x = acc[i][j][r] + bkv[i];
            if (kwave) x = phi(x + bf2f(sm.tg[t * LDG + cc]));
            v[r] = c * BM + t < T ? x : 0.f;                    // chunk rows past T add nothing
          }
          *reinterpret_cast<uint2*>(&dst[cc * LDT + 16 * j + 4 * q]) = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
        }
      }
      __syncthreads();                                                         // B2
      // ---- KV_h [+ ksum_h] += phi(K_h)^T [V_h | 1]: wave w -> head w/2, key rows 16*(w&1)
      {
        const int h = wave >> 1, fi = wave & 1;
        const s16x8 ka = *reinterpret_cast<const s16x8*>(&sm.u.p1.kt[(h * D + 16 * fi + r16) * LDT + 8 * q]);
#pragma unroll
        for (int fj = 0; fj < 2; ++fj) {
          const s16x8 vb = *reinterpret_cast<const s16x8*>(&sm.u.p1.vt[(h * D + 16 * fj + r16) * LDT + 8 * q]);
          kvacc[fj] = mfma_bf16(ka, vb, kvacc[fj]);
        }
        const short one = r16 == 0 ? (short)0x3F80 : (short)0;   // bf16 1.0 in column 0 only
        const s16x8 ones = {one, one, one, one, one, one, one, one};
        kvacc[2] = mfma_bf16(ka, ones, kvacc[2]);
      }
      if (c == nc - 1) {
        // padding tokens (model.py:397-410): n_pad * phi(k_pad) (x) [v_pad | 1]; V / S
        const int h = wave >> 1, fi = wave & 1;
        const float invS = 1.f / S;
#pragma unroll
        for (int fj = 0; fj < 3; ++fj) {
          if (fj == 2 && r16 != 0) continue;
          const int j = 16 * fj + r16;                             // value channel (32 = ksum)
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * fi + 4 * q + r;                     // key channel within the head
            float x = kvacc[fj][r];
            if (a.n_pad > 0) {
              const float kp = (float)a.n_pad * phi(a.k_pad[h * D + i]);
              x += fj < 2 ? kp * a.v_pad[h * D + j] : kp;
            }
            v[r] = fj < 2 ? x * invS : x;
          }
          float lo[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) lo[r] = v[r] - bf2f(f2bf(v[r]));
          const int off = (h * KVR + j) * LDK + 16 * fi + 4 * q;
          *reinterpret_cast<uint2*>(&sm.kv[0][off]) = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
          *reinterpret_cast<uint2*>(&sm.kv[1][off]) = make_uint2(f2bf2(lo[0], lo[1]), f2bf2(lo[2], lo[3]));
        }
      }
    } else {
      // ---- q = LN(x) W_q^T + b (+ guidance): D[n][t], lane = 4 columns n of one row t
      f32x4 acc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[j] = mfma_bf16(wq[ks], *reinterpret_cast<const s16x8*>(&sm.xn[cslot<BM>(ks * 4 + q, 16 * j + r16)]), acc[j]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int t = 16 * j + r16, n = 16 * wave + 4 * q;
        const uint2 gu = *reinterpret_cast<const uint2*>(&sm.tg[t * LDG + n]);
        const float g[4] = {__uint_as_float(gu.x << 16), __uint_as_float(gu.x & 0xffff0000u),
                            __uint_as_float(gu.y << 16), __uint_as_float(gu.y & 0xffff0000u)};
        const float bb[4] = {bq.x, bq.y, bq.z, bq.w};
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = phi(acc[j][r] + bb[r] + g[r]);
        *reinterpret_cast<uint2*>(&sm.u.p2.q[t * LDQ + n]) = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
      }
      __syncthreads();                                                         // B2
      // ---- [num | z] = [KV_h | ksum_h]^T phi(q_h): D[j][t]; wave w -> head w/2, rows 16*(w&1)
      {
        const int h = wave >> 1, jt = wave & 1;
        const s16x8 qb = *reinterpret_cast<const s16x8*>(&sm.u.p2.q[(16 * jt + r16) * LDQ + h * D + 8 * q]);
        f32x4 o[3];
#pragma unroll
        for (int fj = 0; fj < 3; ++fj) {
          o[fj] = f32x4{0.f, 0.f, 0.f, 0.f};
          const int j = 16 * fj + r16;
#pragma unroll
          for (int hl = 0; hl < 2; ++hl) {
            s16x8 ka = {0, 0, 0, 0, 0, 0, 0, 0};
            if (j < KVR) ka = *reinterpret_cast<const s16x8*>(&sm.kv[hl][(h * KVR + j) * LDK + 8 * q]);
            o[fj] = mfma_bf16(ka, qb, o[fj]);
          }
        }
        const float z = __shfl(o[2][0], r16, 64);                  // D[32][t] sits in lane t, reg 0
        const float sc = S / (z + a.attn_eps);
        const int t = 16 * jt + r16;
#pragma unroll
        for (int fj = 0; fj < 2; ++fj) {
          const f32x4 w = o[fj] * sc;
          *reinterpret_cast<f32x4*>(&sm.u.p2.o[t * LDO + h * D + 16 * fj + 4 * q]) = w;
        }
      }
      __syncthreads();                                                         // B3
      // ---- y = x + attention, full-row 16-byte stores
      const int t = c * BM + lr;
      if (t < T) {
        const int b = (unsigned)pix / (unsigned)HW, p = pix - b * HW;
        float v[8];
        *reinterpret_cast<f32x4*>(&v[0]) = *reinterpret_cast<const f32x4*>(&sm.u.p2.o[lr * LDO + lc * 8]);
        *reinterpret_cast<f32x4*>(&v[4]) = *reinterpret_cast<const f32x4*>(&sm.u.p2.o[lr * LDO + lc * 8 + 4]);
        const bf16* e = reinterpret_cast<const bf16*>(&xc);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += bf2f(e[j]);
        st16(a.y + ((int64_t)(b * T + t) * HW + p) * a.ld_y + lc * 8,
             make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7])));
      }
    }
  }
}

}  // namespace

int classattn2_launch(const CatsegClassAttnArgs* a, hipStream_t st);   // classattn2.hip (default kernel)

extern "C" int catseg_class_attention(const CatsegClassAttnArgs* a, void* stream) {
  CATSEG_CHECK(a && a->x && a->w_qkv && a->b_qkv && a->ln_g && a->ln_b && a->tg && a->y,
               "class_attention: null pointer");
  CATSEG_CHECK(a->dtype == CATSEG_BF16, "class_attention: bf16 only");
  CATSEG_CHECK(a->n_heads == NH && a->head_dim == D, "class_attention: needs 4 heads x 32");
  CATSEG_CHECK(a->B > 0 && a->T > 0 && a->HW > 0, "class_attention: empty shape");
  CATSEG_CHECK(a->n_pad >= 0 && (a->n_pad == 0 || (a->k_pad && a->v_pad)), "class_attention: padding projections missing");
  CATSEG_CHECK(a->ld_x % 8 == 0 && a->ld_y % 8 == 0 && a->ld_tg % 8 == 0 && a->ld_x >= C && a->ld_y >= C &&
               a->ld_tg >= 2 * C, "class_attention: row strides must be multiples of 8 elements");
  CATSEG_CHECK(a->tg_bstride >= 0, "class_attention: bad guidance image stride");
  CATSEG_CHECK(a->x != a->y, "class_attention: y must not alias x");
  CATSEG_CHECK(a->B * a->T * (int64_t)a->HW < (1LL << 31), "class_attention: row count must fit 31 bits");
  ClsP p;
  p.x = (const bf16*)a->x; p.ld_x = a->ld_x;
  p.ln_g = a->ln_g; p.ln_b = a->ln_b; p.eps = a->eps;
  p.w = (const bf16*)a->w_qkv; p.bias = a->b_qkv;
  p.tg = (const bf16*)a->tg; p.ld_tg = a->ld_tg; p.tg_bstride = a->tg_bstride;
  p.k_pad = a->k_pad; p.v_pad = a->v_pad; p.n_pad = a->n_pad; p.attn_eps = a->attn_eps;
  p.y = (bf16*)a->y; p.ld_y = a->ld_y;
  p.B = a->B; p.T = a->T; p.HW = a->HW;
  const int rc2 = classattn2_launch(a, (hipStream_t)stream);
  if (rc2 == 0) return catseg_launch_status("class_attention");
  if (rc2 < 0) return rc2;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int64_t npix = a->B * a->HW;
  const unsigned grid = (unsigned)std::min<int64_t>(npix, (int64_t)cus);
  hipLaunchKernelGGL(classattn_kernel, dim3(grid), dim3(NT), 0, (hipStream_t)stream, p);
  return catseg_launch_status("class_attention");
}
