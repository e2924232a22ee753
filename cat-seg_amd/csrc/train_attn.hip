// Attention backward kernels of the aggregation head, fp32.
//
// catseg_window_attention_backward — WindowAttention (model.py:86-114) with the cyclic shift and
//   the -100 region mask (model.py:161-216): given the forward q/k/v rows, the forward attention
//   output o and its gradient do, returns dq, dk, dv in the same row layout.  One workgroup per
//   (slice, window, head); the window's Q, K, V, dO stay in LDS and P is recomputed (never in HBM):
//     pass 0  per query: softmax max / sum over the window (online, per lane, then across the
//             4 lanes that share an MFMA column), and D_q = dO_q . O_q
//     pass A  waves own KEY tiles:   dV += P^T dO,  dK += scale dS^T Q    (dS = P (dP - D))
//     pass B  waves own QUERY tiles: dQ += scale dS K
//   Every product is an exact-f32 MFMA (16x16x4).  An accumulator tile is used directly as the next
//   MFMA's A operand (its 4 registers = the 4 k-steps of one 16-deep reduction, k order permuted
//   inside the step; the matching B rows are read from LDS in the same permuted order).  Each dK / dV
//   / dQ element is owned by one wave: no atomics, deterministic.
//
// catseg_linear_attention_backward — LinearAttention (model.py:256-286) inside AttentionLayer
//   (model.py:338-354) with the learned padding tokens (model.py:397-410): one workgroup per pixel,
//   one wave per head (head_dim 32), VALU with the 32x32 KV / dKV states in LDS.  The padding
//   tokens' k / v gradients are summed over their n_pad copies per pixel into a workspace and then
//   over pixels in a fixed order.
#include "common.h"
#include "capi.h"
#include "catseg_hip_train.h"

namespace {

// ------------------------------------------------------------------------------ window attention
constexpr int WD = 32;          // head_dim
constexpr int WNMAX = 144;      // tokens per window (12 x 12)
constexpr int WP = 34;          // LDS row pitch (floats)

struct WinGeo {
  int H, W, ws, shift, nwx, nwin;
};

DEV int64_t win_row(const WinGeo& g, int64_t slice, int w, int i) {
  const int Y = (w / g.nwx) * g.ws + i / g.ws, X = (w % g.nwx) * g.ws + i % g.ws;
  const int y = (Y + g.shift) % g.H, x = (X + g.shift) % g.W;
  return slice * g.H * g.W + y * g.W + x;
}
DEV int win_region(const WinGeo& g, int w, int i) {
  const int Y = (w / g.nwx) * g.ws + i / g.ws, X = (w % g.nwx) * g.ws + i % g.ws;
  const int hb = Y < g.H - g.ws ? 0 : (Y < g.H - g.shift ? 1 : 2);
  const int wb = X < g.W - g.ws ? 0 : (X < g.W - g.shift ? 1 : 2);
  return hb * 3 + wb;
}

__global__ __launch_bounds__(256) void win_attn_bwd_kernel(CatsegWinAttnBwdArgs a, WinGeo geo, int N) {
  __shared__ float Qs[WNMAX * WP], Ks[WNMAX * WP], Vs[WNMAX * WP], Os[WNMAX * WP];   // Os holds dO
  __shared__ float mst[WNMAX], lst[WNMAX], Dst[WNMAX];
  __shared__ int reg[WNMAX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int H = a.n_heads;
  const int64_t wid = blockIdx.x / H;
  const int h = (int)(blockIdx.x % H);
  const int64_t slice = wid / geo.nwin;
  const int w = (int)(wid % geo.nwin);
  const float* q = (const float*)a.q;
  const float* k = (const float*)a.k;
  const float* v = (const float*)a.v;
  const float* o = (const float*)a.o;
  const float* dout = (const float*)a.dout;
  const int col = h * WD;
  const bool masked = geo.shift > 0;
  const float scale = a.scale;
  const int NT = N / 16;

  // ---- stage Q, K, V, dO of the window (rows gathered through the roll / partition) ----
  for (int e = tid; e < N * (WD / 4); e += 256) {
    const int i = e / (WD / 4), c = (e % (WD / 4)) * 4;
    const int64_t row = win_row(geo, slice, w, i);
    const float4 qv = *reinterpret_cast<const float4*>(q + row * a.ld_qkv + col + c);
    const float4 kv = *reinterpret_cast<const float4*>(k + row * a.ld_qkv + col + c);
    const float4 vv = *reinterpret_cast<const float4*>(v + row * a.ld_qkv + col + c);
    const float4 dv = *reinterpret_cast<const float4*>(dout + row * a.ld_dout + col + c);
    float* qd = Qs + i * WP + c; qd[0] = qv.x; qd[1] = qv.y; qd[2] = qv.z; qd[3] = qv.w;
    float* kd = Ks + i * WP + c; kd[0] = kv.x; kd[1] = kv.y; kd[2] = kv.z; kd[3] = kv.w;
    float* vd = Vs + i * WP + c; vd[0] = vv.x; vd[1] = vv.y; vd[2] = vv.z; vd[3] = vv.w;
    float* od = Os + i * WP + c; od[0] = dv.x; od[1] = dv.y; od[2] = dv.z; od[3] = dv.w;
  }
  for (int i = tid; i < N; i += 256) reg[i] = masked ? win_region(geo, w, i) : 0;
  __syncthreads();
  // D_q = dO_q . O_q (O from the forward output rows)
  for (int i = tid; i < N; i += 256) {
    const float* orow = o + win_row(geo, slice, w, i) * a.ld_o + col;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < WD; c += 4) {
      const float4 ov = *reinterpret_cast<const float4*>(orow + c);
      const float* d = Os + i * WP + c;
      s += ov.x * d[0] + ov.y * d[1] + ov.z * d[2] + ov.w * d[3];
    }
    Dst[i] = s;
  }

  // ---- pass 0: softmax statistics per query (S^T tiles: lane column = query) ----
  for (int qt = wave; qt < NT; qt += 4) {
    const int qi = qt * 16 + r;
    const int rq = reg[qi];
    float m_l = -INFINITY, l_l = 0.f;
    for (int kt = 0; kt < NT; ++kt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < WD / 4; ++s)
        acc = mfma_f32(Ks[(kt * 16 + r) * WP + 4 * s + g], Qs[qi * WP + 4 * s + g], acc);
      float sc[4];
      float tm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = kt * 16 + 4 * g + j;
        sc[j] = scale * acc[j] + ((masked && reg[key] != rq) ? -100.f : 0.f);
        tm = fmaxf(tm, sc[j]);
      }
      const float mn = fmaxf(m_l, tm);
      float add = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) add += __expf(sc[j] - mn);
      l_l = l_l * __expf(m_l - mn) + add;
      m_l = mn;
    }
    const float M = xrow4_max(m_l);
    const float Lsum = xrow4_sum(l_l * __expf(m_l - M));
    if (g == 0) { mst[qi] = M; lst[qi] = 1.f / Lsum; }
  }
  __syncthreads();

  // ---- passes A and B as one list of 2 NT items dealt round-robin over the waves (item < NT: pass A
  // for key tile item, else pass B for query tile item - NT): with NT = 9 the longest wave does 3 A +
  // 2 B items instead of 3 A + 3 B when each pass is dealt on its own ----
  // pass A: the wave owns a key tile; dV = P^T dO, dK = scale dS^T Q
  auto pass_a = [&](int kt) {
    f32x4 dV[2], dK[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) { dV[e] = f32x4{0.f, 0.f, 0.f, 0.f}; dK[e] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    const int key = kt * 16 + r;
    const int rk = reg[key];
    for (int qt = 0; qt < NT; ++qt) {
      f32x4 sa = f32x4{0.f, 0.f, 0.f, 0.f}, pa = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < WD / 4; ++s) {
        sa = mfma_f32(Qs[(qt * 16 + r) * WP + 4 * s + g], Ks[key * WP + 4 * s + g], sa);   // S[q][key]
        pa = mfma_f32(Os[(qt * 16 + r) * WP + 4 * s + g], Vs[key * WP + 4 * s + g], pa);   // dP[q][key]
      }
      float P[4], dS[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qj = qt * 16 + 4 * g + j;
        const float sc = scale * sa[j] + ((masked && reg[qj] != rk) ? -100.f : 0.f);
        P[j] = __expf(sc - mst[qj]) * lst[qj];
        dS[j] = P[j] * (pa[j] - Dst[qj]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qj = qt * 16 + 4 * g + j;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          dV[e] = mfma_f32(P[j], Os[qj * WP + 16 * e + r], dV[e]);
          dK[e] = mfma_f32(dS[j], Qs[qj * WP + 16 * e + r], dK[e]);
        }
      }
    }
    // lane holds rows key = kt*16 + 4g + j, column d = 16e + r
    float* dk = (float*)a.dk;
    float* dv = (float*)a.dv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t row = win_row(geo, slice, w, kt * 16 + 4 * g + j);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        dv[row * a.ld_dqkv + col + 16 * e + r] = dV[e][j];
        dk[row * a.ld_dqkv + col + 16 * e + r] = scale * dK[e][j];
      }
    }
  };

  // pass B: the wave owns a query tile; dQ = scale dS K
  auto pass_b = [&](int qt) {
    f32x4 dQ[2];
    dQ[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    dQ[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int qi = qt * 16 + r;
    const int rq = reg[qi];
    const float mq = mst[qi], lq = lst[qi], Dq = Dst[qi];
    for (int kt = 0; kt < NT; ++kt) {
      f32x4 sa = f32x4{0.f, 0.f, 0.f, 0.f}, pa = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < WD / 4; ++s) {
        sa = mfma_f32(Ks[(kt * 16 + r) * WP + 4 * s + g], Qs[qi * WP + 4 * s + g], sa);   // S^T[key][q]
        pa = mfma_f32(Vs[(kt * 16 + r) * WP + 4 * s + g], Os[qi * WP + 4 * s + g], pa);   // dP^T[key][q]
      }
      float dS[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kj = kt * 16 + 4 * g + j;
        const float sc = scale * sa[j] + ((masked && reg[kj] != rq) ? -100.f : 0.f);
        dS[j] = __expf(sc - mq) * lq * (pa[j] - Dq);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kj = kt * 16 + 4 * g + j;
#pragma unroll
        for (int e = 0; e < 2; ++e) dQ[e] = mfma_f32(dS[j], Ks[kj * WP + 16 * e + r], dQ[e]);
      }
    }
    float* dq = (float*)a.dq;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t row = win_row(geo, slice, w, qt * 16 + 4 * g + j);
#pragma unroll
      for (int e = 0; e < 2; ++e) dq[row * a.ld_dqkv + col + 16 * e + r] = scale * dQ[e][j];
    }
  };

  for (int it = wave; it < 2 * NT; it += 4) {
    if (it < NT) pass_a(it);
    else pass_b(it - NT);
  }
}

// ------------------------------------------------------------------------------ dense attention
// nn.MultiheadAttention of the CLIP blocks (model_vpt.py:169-182,202-206; causal text encoder
// model_vpt.py:400-406), head_dim 64, fp32.  Three kernels, each one workgroup of 4 waves per
// (sequence, head, 64-row block):
//   dense_stats  per query: softmax max m, 1/sum l over the keys, D = dO . O
//   dense_dkv    waves own 16-key tiles (K, V rows in registers), the query blocks stream through LDS:
//                dV += P^T dO, dK += scale dS^T Q
//   dense_dq     waves own 16-query tiles (Q, dO rows in registers), the key blocks stream through LDS:
//                dQ += scale dS K
// No atomics: every output element is owned by one wave.  Rows past L are staged as zeros and masked.
constexpr int HD = 64;          // head_dim
constexpr int DP = HD + 4;      // LDS pitch: a fragment read's 16 rows x 4 k on 64 distinct banks

struct DenseP {
  const float* q; const float* k; const float* v; int64_t ld_qkv;
  const float* o; int64_t ld_o;
  const float* dout; int64_t ld_dout;
  float* dq; float* dk; float* dv; int64_t ld_dqkv;
  float* stats;                  // [n_seq * H * L][3]: m, 1/l, D
  int64_t n_seq; int L; int H; float scale; int causal;
};

DEV bool dense_mask_ok(const DenseP& p, int q, int key) {
  return q < p.L && key < p.L && (!p.causal || key <= q);
}

// stage rows [r0, r0 + 64) x head columns of `src` into an LDS tile [64][DP] (zeros past L)
DEV void stage64(float* tile, const float* src, int64_t ld, int64_t row0, int r0, int L, int col) {
  for (int e = threadIdx.x; e < 64 * (HD / 4); e += 256) {
    const int i = e / (HD / 4), c = (e % (HD / 4)) * 4;
    float4 v = make_float4(0, 0, 0, 0);
    if (r0 + i < L) v = *reinterpret_cast<const float4*>(src + (row0 + r0 + i) * ld + col + c);
    float* d = tile + i * DP + c;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
}

__global__ __launch_bounds__(256) void dense_stats_kernel(DenseP p) {
  __shared__ float Kt[64 * DP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const int64_t sh = blockIdx.y;
  const int64_t s = sh / p.H;
  const int h = (int)(sh % p.H), col = h * HD;
  const int64_t row0 = s * p.L;
  const int qi = (blockIdx.x * 4 + wave) * 16 + r;
  // the lane's query as the B operand: Q[qi][4 t + g], t = 0..15
  float qf[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) qf[t] = qi < p.L ? p.q[(row0 + qi) * p.ld_qkv + col + 4 * t + g] : 0.f;
  float m_l = -INFINITY, l_l = 0.f;
  const int kmax = p.causal ? (blockIdx.x * 4 + 4) * 16 : p.L;   // keys past the block's last query are masked
  for (int kb = 0; kb < p.L && kb < kmax; kb += 64) {
    __syncthreads();
    stage64(Kt, p.k, p.ld_qkv, row0, kb, p.L, col);
    __syncthreads();
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 16; ++t) acc = mfma_f32(Kt[(kt * 16 + r) * DP + 4 * t + g], qf[t], acc);
      float sc[4], tm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = kb + kt * 16 + 4 * g + j;
        sc[j] = dense_mask_ok(p, qi, key) ? p.scale * acc[j] : -INFINITY;
        tm = fmaxf(tm, sc[j]);
      }
      const float mn = fmaxf(m_l, tm);
      if (mn != -INFINITY) {
        float add = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) add += __expf(sc[j] - mn);
        l_l = l_l * __expf(m_l - mn) + add;
        m_l = mn;
      }
    }
  }
  const float M = xrow4_max(m_l);
  const float Lsum = xrow4_sum(M == -INFINITY ? 0.f : l_l * __expf(m_l - M));
  // D = dO . O over the lane's 16 columns g*16 .. g*16+15, then across the 4 lanes of the query
  float d = 0.f;
  if (qi < p.L) {
#pragma unroll
    for (int c = 0; c < 16; c += 4) {
      const float4 a = *reinterpret_cast<const float4*>(p.dout + (row0 + qi) * p.ld_dout + col + g * 16 + c);
      const float4 b = *reinterpret_cast<const float4*>(p.o + (row0 + qi) * p.ld_o + col + g * 16 + c);
      d += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
    }
  }
  d = xrow4_sum(d);
  if (g == 0 && qi < p.L) {
    float* st = p.stats + ((sh * p.L) + qi) * 3;
    st[0] = M;
    st[1] = Lsum > 0.f ? 1.f / Lsum : 0.f;
    st[2] = d;
  }
}

__global__ __launch_bounds__(256) void dense_dkv_kernel(DenseP p) {
  __shared__ float Qt[64 * DP], Ot[64 * DP];    // Ot holds dO
  __shared__ float st[64 * 3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const int64_t sh = blockIdx.y;
  const int64_t s = sh / p.H;
  const int h = (int)(sh % p.H), col = h * HD;
  const int64_t row0 = s * p.L;
  const int kt0 = (blockIdx.x * 4 + wave) * 16;
  const int key = kt0 + r;
  float kf[16], vf[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    kf[t] = key < p.L ? p.k[(row0 + key) * p.ld_qkv + col + 4 * t + g] : 0.f;
    vf[t] = key < p.L ? p.v[(row0 + key) * p.ld_qkv + col + 4 * t + g] : 0.f;
  }
  f32x4 dV[4], dK[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) { dV[e] = f32x4{0.f, 0.f, 0.f, 0.f}; dK[e] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  const int qstart = p.causal ? (blockIdx.x * 64) / 64 * 64 : 0;   // queries before the block see none of its keys
  for (int qb = qstart; qb < p.L; qb += 64) {
    __syncthreads();
    stage64(Qt, p.q, p.ld_qkv, row0, qb, p.L, col);
    stage64(Ot, p.dout, p.ld_dout, row0, qb, p.L, col);
    for (int i = threadIdx.x; i < 64 * 3; i += 256) {
      const int qq = qb + i / 3;
      st[i] = qq < p.L ? p.stats[(sh * p.L + qq) * 3 + i % 3] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      f32x4 sa = f32x4{0.f, 0.f, 0.f, 0.f}, pa = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        sa = mfma_f32(Qt[(qs * 16 + r) * DP + 4 * t + g], kf[t], sa);   // S[q][key]
        pa = mfma_f32(Ot[(qs * 16 + r) * DP + 4 * t + g], vf[t], pa);   // dP[q][key]
      }
      float P[4], dS[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ql = qs * 16 + 4 * g + j, qq = qb + ql;
        const float* sq = st + ql * 3;
        P[j] = dense_mask_ok(p, qq, key) ? __expf(p.scale * sa[j] - sq[0]) * sq[1] : 0.f;
        dS[j] = P[j] * (pa[j] - sq[2]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ql = qs * 16 + 4 * g + j;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dV[e] = mfma_f32(P[j], Ot[ql * DP + 16 * e + r], dV[e]);
          dK[e] = mfma_f32(dS[j], Qt[ql * DP + 16 * e + r], dK[e]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kk = kt0 + 4 * g + j;
    if (kk >= p.L) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      p.dv[(row0 + kk) * p.ld_dqkv + col + 16 * e + r] = dV[e][j];
      p.dk[(row0 + kk) * p.ld_dqkv + col + 16 * e + r] = p.scale * dK[e][j];
    }
  }
}

__global__ __launch_bounds__(256) void dense_dq_kernel(DenseP p) {
  __shared__ float Kt[64 * DP], Vt[64 * DP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const int64_t sh = blockIdx.y;
  const int64_t s = sh / p.H;
  const int h = (int)(sh % p.H), col = h * HD;
  const int64_t row0 = s * p.L;
  const int qt0 = (blockIdx.x * 4 + wave) * 16;
  const int qi = qt0 + r;
  float qf[16], of[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    qf[t] = qi < p.L ? p.q[(row0 + qi) * p.ld_qkv + col + 4 * t + g] : 0.f;
    of[t] = qi < p.L ? p.dout[(row0 + qi) * p.ld_dout + col + 4 * t + g] : 0.f;
  }
  float mq = 0.f, lq = 0.f, Dq = 0.f;
  if (qi < p.L) {
    const float* sq = p.stats + (sh * p.L + qi) * 3;
    mq = sq[0]; lq = sq[1]; Dq = sq[2];
  }
  f32x4 dQ[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) dQ[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kend = p.causal ? (blockIdx.x * 4 + 4) * 16 : p.L;
  for (int kb = 0; kb < p.L && kb < kend; kb += 64) {
    __syncthreads();
    stage64(Kt, p.k, p.ld_qkv, row0, kb, p.L, col);
    stage64(Vt, p.v, p.ld_qkv, row0, kb, p.L, col);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      f32x4 sa = f32x4{0.f, 0.f, 0.f, 0.f}, pa = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        sa = mfma_f32(Kt[(ks * 16 + r) * DP + 4 * t + g], qf[t], sa);   // S^T[key][q]
        pa = mfma_f32(Vt[(ks * 16 + r) * DP + 4 * t + g], of[t], pa);   // dP^T[key][q]
      }
      float dS[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = kb + ks * 16 + 4 * g + j;
        dS[j] = dense_mask_ok(p, qi, kk) ? __expf(p.scale * sa[j] - mq) * lq * (pa[j] - Dq) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kl = ks * 16 + 4 * g + j;
#pragma unroll
        for (int e = 0; e < 4; ++e) dQ[e] = mfma_f32(dS[j], Kt[kl * DP + 16 * e + r], dQ[e]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int qq = qt0 + 4 * g + j;
    if (qq >= p.L) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) p.dq[(row0 + qq) * p.ld_dqkv + col + 16 * e + r] = p.scale * dQ[e][j];
  }
}

// ------------------------------------------------------------------------------ linear attention
constexpr int LD = 32;     // head_dim
constexpr int LCH = 32;    // tokens staged per chunk
constexpr int KVP = 33;    // LDS pitch of the 32x32 states

DEV float phi(float x) { return x > 0.f ? x + 1.f : __expf(x); }       // elu(x) + 1
DEV float dphi(float x) { return x > 0.f ? 1.f : __expf(x); }

struct LinWave {
  float kv[LD * KVP];     // KV (phase 1-2), then dKV (phase 3)
  float ks[LD];           // ksum, then dksum
  float a[LCH * LD];      // staged token vectors
  float b[LCH * LD];
  float c[LCH];
};

__global__ __launch_bounds__(256) void lin_attn_bwd_kernel(CatsegLinAttnBwdArgs p, float* __restrict__ padpart) {
  __shared__ LinWave sw[4];
  const int lane = threadIdx.x & 63, h = threadIdx.x >> 6;
  LinWave& S = sw[h];
  const int64_t pix = blockIdx.x;              // (b, p)
  const int64_t b = pix / p.HW, pp = pix % p.HW;
  const int T = p.T, L = p.T + p.n_pad;
  const float invL = 1.f / (float)L, fL = (float)L;
  const float* q = (const float*)p.q;
  const float* k = (const float*)p.k;
  const float* v = (const float*)p.v;
  const float* dy = (const float*)p.dy;
  const int col = h * LD;
  auto row_of = [&](int t) -> int64_t { return ((b * T + t) * p.HW + pp); };
  const int i = lane >> 1, j0 = (lane & 1) * 16;   // lane-owned state entries [i][j0 .. j0+16)

  // ---- phase 1: KV = sum_s phi(k_s) v_s^T / L, ksum = sum_s phi(k_s) (+ the padding copies) ----
  float kv[16], ks = 0.f;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) kv[jj] = 0.f;
  for (int t0 = 0; t0 < T; t0 += LCH) {
    const int nt = T - t0 < LCH ? T - t0 : LCH;
    for (int e = lane; e < nt * (LD / 4); e += 64) {
      const int tt = e / (LD / 4), c = (e % (LD / 4)) * 4;
      const int64_t row = row_of(t0 + tt);
      const float4 kk = *reinterpret_cast<const float4*>(k + row * p.ld_qkv + col + c);
      const float4 vv = *reinterpret_cast<const float4*>(v + row * p.ld_qkv + col + c);
      float* ad = S.a + tt * LD + c; ad[0] = phi(kk.x); ad[1] = phi(kk.y); ad[2] = phi(kk.z); ad[3] = phi(kk.w);
      float* bd = S.b + tt * LD + c; bd[0] = vv.x * invL; bd[1] = vv.y * invL; bd[2] = vv.z * invL; bd[3] = vv.w * invL;
    }
    __syncthreads();
    for (int tt = 0; tt < nt; ++tt) {
      const float f = S.a[tt * LD + i];
      ks += f;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) kv[jj] += f * S.b[tt * LD + j0 + jj];
    }
    __syncthreads();
  }
  const float fpad = (float)p.n_pad;
  float kpad_i = 0.f, phikp_i = 0.f;
  if (p.n_pad > 0) {
    kpad_i = p.k_pad[col + i];
    phikp_i = phi(kpad_i);
    ks += fpad * phikp_i;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) kv[jj] += fpad * phikp_i * p.v_pad[col + j0 + jj] * invL;
  }
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) S.kv[i * KVP + j0 + jj] = kv[jj];
  if ((lane & 1) == 0) S.ks[i] = ks;
  __syncthreads();

  // ---- phase 2: per query row: dq; accumulate dKV = sum_l phi(q_l) dn_l^T, dksum = sum_l dden_l phi(q_l) ----
  float dkv[16], dks = 0.f;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) dkv[jj] = 0.f;
  float* dq = (float*)p.dq;
  for (int t0 = 0; t0 < T; t0 += LCH) {
    const int nt = T - t0 < LCH ? T - t0 : LCH;
    if (lane < nt) {
      const int64_t row = row_of(t0 + lane);
      float qv[LD], fq[LD], g[LD];
#pragma unroll
      for (int c = 0; c < LD; c += 4) {
        const float4 a4 = *reinterpret_cast<const float4*>(q + row * p.ld_qkv + col + c);
        const float4 d4 = *reinterpret_cast<const float4*>(dy + row * p.ld_dy + col + c);
        qv[c] = a4.x; qv[c + 1] = a4.y; qv[c + 2] = a4.z; qv[c + 3] = a4.w;
        g[c] = d4.x; g[c + 1] = d4.y; g[c + 2] = d4.z; g[c + 3] = d4.w;
      }
      float den = p.eps;
#pragma unroll
      for (int c = 0; c < LD; ++c) { fq[c] = phi(qv[c]); den += fq[c] * S.ks[c]; }
      // n = phi(q)^T KV ; dn = L dy / den ; dden = -L (dy . n) / den^2
      float dyn = 0.f;
#pragma unroll
      for (int jj = 0; jj < LD; ++jj) {
        float n = 0.f;
#pragma unroll
        for (int c = 0; c < LD; ++c) n += fq[c] * S.kv[c * KVP + jj];
        dyn += g[jj] * n;
      }
      const float rden = 1.f / den;
      const float dden = -fL * dyn * rden * rden;
#pragma unroll
      for (int jj = 0; jj < LD; ++jj) g[jj] *= fL * rden;     // dn
      // dphi(q) = KV dn + dden ksum
      float* dqr = dq + row * p.ld_dqkv + col;
#pragma unroll
      for (int c = 0; c < LD; c += 4) {
        float o4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float s = dden * S.ks[c + u];
#pragma unroll
          for (int jj = 0; jj < LD; ++jj) s += S.kv[(c + u) * KVP + jj] * g[jj];
          o4[u] = s * dphi(qv[c + u]);
        }
        *reinterpret_cast<float4*>(dqr + c) = make_float4(o4[0], o4[1], o4[2], o4[3]);
      }
#pragma unroll
      for (int c = 0; c < LD; ++c) { S.a[lane * LD + c] = fq[c]; S.b[lane * LD + c] = g[c]; }
      S.c[lane] = dden;
    }
    __syncthreads();
    for (int tt = 0; tt < nt; ++tt) {
      const float f = S.a[tt * LD + i];
      dks += S.c[tt] * f;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) dkv[jj] += f * S.b[tt * LD + j0 + jj];
    }
    __syncthreads();
  }
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) S.kv[i * KVP + j0 + jj] = dkv[jj];
  if ((lane & 1) == 0) S.ks[i] = dks;
  __syncthreads();

  // ---- phase 3: per key row: dk = (dKV v'_s + dksum) * phi'(k), dv = dKV^T phi(k) / L ----
  float* dk = (float*)p.dk;
  float* dv = (float*)p.dv;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    if (t < T) {
      const int64_t row = row_of(t);
      float kr[LD], fk[LD], vv[LD];
#pragma unroll
      for (int c = 0; c < LD; c += 4) {
        const float4 a4 = *reinterpret_cast<const float4*>(k + row * p.ld_qkv + col + c);
        const float4 b4 = *reinterpret_cast<const float4*>(v + row * p.ld_qkv + col + c);
        kr[c] = a4.x; kr[c + 1] = a4.y; kr[c + 2] = a4.z; kr[c + 3] = a4.w;
        vv[c] = b4.x * invL; vv[c + 1] = b4.y * invL; vv[c + 2] = b4.z * invL; vv[c + 3] = b4.w * invL;
      }
#pragma unroll
      for (int c = 0; c < LD; ++c) fk[c] = phi(kr[c]);
      float* dkr = dk + row * p.ld_dqkv + col;
      float* dvr = dv + row * p.ld_dqkv + col;
#pragma unroll
      for (int c = 0; c < LD; c += 4) {
        float o4[4], w4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float s = S.ks[c + u], s2 = 0.f;
#pragma unroll
          for (int jj = 0; jj < LD; ++jj) {
            s += S.kv[(c + u) * KVP + jj] * vv[jj];
            s2 += S.kv[jj * KVP + c + u] * fk[jj];
          }
          o4[u] = s * dphi(kr[c + u]);
          w4[u] = s2 * invL;
        }
        *reinterpret_cast<float4*>(dkr + c) = make_float4(o4[0], o4[1], o4[2], o4[3]);
        *reinterpret_cast<float4*>(dvr + c) = make_float4(w4[0], w4[1], w4[2], w4[3]);
      }
    }
  }
  // the padding copies: d k_pad = n_pad (dKV v'_pad + dksum) phi'(k_pad), d v_pad = n_pad dKV^T phi(k_pad) / L
  if (p.n_pad > 0 && lane < LD) {
    const int c = lane;
    float s = S.ks[c], s2 = 0.f;
    for (int jj = 0; jj < LD; ++jj) {
      s += S.kv[c * KVP + jj] * p.v_pad[col + jj] * invL;
      s2 += S.kv[jj * KVP + c] * phi(p.k_pad[col + jj]);
    }
    padpart[pix * 256 + col + c] = fpad * s * dphi(p.k_pad[col + c]);
    padpart[pix * 256 + 128 + col + c] = fpad * s2 * invL;
  }
}

// d k_pad / d v_pad = sum over pixels (fixed order)
__global__ __launch_bounds__(256) void lin_pad_reduce_kernel(const float* __restrict__ part, int64_t npix,
                                                             float* __restrict__ dk_pad, float* __restrict__ dv_pad) {
  const int c = threadIdx.x;
  float s = 0.f;
  for (int64_t i = 0; i < npix; ++i) s += part[i * 256 + c];
  if (c < 128) dk_pad[c] = s;
  else dv_pad[c - 128] = s;
}

}  // namespace

extern "C" int catseg_window_attention_backward(const CatsegWinAttnBwdArgs* a, void* stream) {
  CATSEG_CHECK(a && a->q && a->k && a->v && a->o && a->dout && a->dq && a->dk && a->dv, "window_attention_backward: null");
  CATSEG_CHECK(a->head_dim == WD, "window_attention_backward: head_dim must be 32");
  CATSEG_CHECK(a->n_heads > 0 && a->S > 0 && a->img_h > 0 && a->img_w > 0 && a->window > 0,
               "window_attention_backward: bad shape");
  CATSEG_CHECK(a->img_h % a->window == 0 && a->img_w % a->window == 0, "window_attention_backward: window must tile the map");
  CATSEG_CHECK(a->shift >= 0 && a->shift < a->window, "window_attention_backward: bad shift");
  const int N = a->window * a->window;
  CATSEG_CHECK(N % 16 == 0 && N <= WNMAX, "window_attention_backward: window^2 must be a multiple of 16, <= 144");
  CATSEG_CHECK(a->ld_qkv % 4 == 0 && a->ld_o % 4 == 0 && a->ld_dout % 4 == 0, "window_attention_backward: strides % 4");
  WinGeo geo;
  geo.H = a->img_h; geo.W = a->img_w; geo.ws = a->window; geo.shift = a->shift;
  geo.nwx = a->img_w / a->window;
  geo.nwin = (a->img_h / a->window) * geo.nwx;
  const int64_t nwg = a->S * geo.nwin * a->n_heads;
  CATSEG_CHECK(nwg < (1LL << 31), "window_attention_backward: too many windows");
  hipLaunchKernelGGL(win_attn_bwd_kernel, dim3((unsigned)nwg), dim3(256), 0, (hipStream_t)stream, *a, geo, N);
  return catseg_launch_status("window_attention_backward");
}

extern "C" int64_t catseg_linear_attention_backward_workspace(int64_t B, int HW) {
  return B > 0 && HW > 0 ? B * HW * 256 * (int64_t)sizeof(float) : 0;
}

extern "C" int catseg_linear_attention_backward(const CatsegLinAttnBwdArgs* p, void* stream) {
  CATSEG_CHECK(p && p->q && p->k && p->v && p->dy && p->dq && p->dk && p->dv, "linear_attention_backward: null");
  CATSEG_CHECK(p->n_heads == 4 && p->head_dim == LD, "linear_attention_backward: 4 heads x 32 only");
  CATSEG_CHECK(p->B > 0 && p->T > 0 && p->HW > 0 && p->n_pad >= 0, "linear_attention_backward: bad shape");
  CATSEG_CHECK(p->ld_qkv % 4 == 0 && p->ld_dy % 4 == 0 && p->ld_dqkv % 4 == 0, "linear_attention_backward: strides % 4");
  CATSEG_CHECK(p->n_pad == 0 || (p->k_pad && p->v_pad && p->dk_pad && p->dv_pad), "linear_attention_backward: pad args");
  const int64_t npix = p->B * p->HW;
  CATSEG_CHECK(npix < (1LL << 31), "linear_attention_backward: too many pixels");
  if (p->n_pad > 0)
    CATSEG_CHECK(p->workspace && p->workspace_bytes >= npix * 256 * (int64_t)sizeof(float),
                 "linear_attention_backward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(lin_attn_bwd_kernel, dim3((unsigned)npix), dim3(256), 0, st, *p, (float*)p->workspace);
  if (p->n_pad > 0)
    hipLaunchKernelGGL(lin_pad_reduce_kernel, dim3(1), dim3(256), 0, st, (const float*)p->workspace, npix, p->dk_pad,
                       p->dv_pad);
  return catseg_launch_status("linear_attention_backward");
}

extern "C" int64_t catseg_attention_backward_workspace(int64_t n_seq, int seq_len, int n_heads) {
  return n_seq > 0 && seq_len > 0 && n_heads > 0 ? n_seq * n_heads * seq_len * 3 * (int64_t)sizeof(float) : 0;
}

extern "C" int catseg_attention_backward(const CatsegAttnBwdArgs* a, void* stream) {
  CATSEG_CHECK(a && a->q && a->k && a->v && a->o && a->dout && a->dq && a->dk && a->dv, "attention_backward: null");
  CATSEG_CHECK(a->head_dim == HD, "attention_backward: head_dim must be 64");
  CATSEG_CHECK(a->n_seq > 0 && a->seq_len > 0 && a->n_heads > 0, "attention_backward: bad shape");
  CATSEG_CHECK(a->ld_qkv % 4 == 0 && a->ld_o % 4 == 0 && a->ld_dout % 4 == 0 && a->ld_dqkv % 4 == 0,
               "attention_backward: strides % 4");
  CATSEG_CHECK(a->n_seq * a->n_heads < 65536, "attention_backward: at most 65535 (sequence, head) pairs");
  const int64_t need = a->n_seq * a->n_heads * a->seq_len * 3 * (int64_t)sizeof(float);
  CATSEG_CHECK(a->workspace && a->workspace_bytes >= need, "attention_backward: workspace too small");
  DenseP p;
  p.q = (const float*)a->q; p.k = (const float*)a->k; p.v = (const float*)a->v; p.ld_qkv = a->ld_qkv;
  p.o = (const float*)a->o; p.ld_o = a->ld_o;
  p.dout = (const float*)a->dout; p.ld_dout = a->ld_dout;
  p.dq = (float*)a->dq; p.dk = (float*)a->dk; p.dv = (float*)a->dv; p.ld_dqkv = a->ld_dqkv;
  p.stats = (float*)a->workspace;
  p.n_seq = a->n_seq; p.L = a->seq_len; p.H = a->n_heads; p.scale = a->scale; p.causal = a->causal;
  const dim3 grid((unsigned)((a->seq_len + 63) / 64), (unsigned)(a->n_seq * a->n_heads));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dense_stats_kernel, grid, dim3(256), 0, st, p);
  hipLaunchKernelGGL(dense_dkv_kernel, grid, dim3(256), 0, st, p);
  hipLaunchKernelGGL(dense_dq_kernel, grid, dim3(256), 0, st, p);
  return catseg_launch_status("attention_backward");
}
