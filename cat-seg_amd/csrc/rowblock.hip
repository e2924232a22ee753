// Row-block kernels for the 128-channel cost-embedding stream of the aggregation
// (reference model.py:117-225 Swin blocks, :357-424 class layers, :540-555 ConvT):
//
//   catseg_rows_gemm  out = epi(LN?(X) . W^T)            K = 128 (the hidden width)
//   catseg_rows_mlp   out = R + fc2(act(fc1(LN(Y)))) (+ R2)  the whole token MLP
//
// One workgroup owns BM rows.  The rows are loaded ONCE (16 B per lane, 16 lanes per
// row), LayerNorm'd in registers (xor-shuffle row reduction) and parked in LDS as the
// MFMA B operand; the weights are staged to LDS; the fp32 accumulators are staged back
// through LDS so that bias / broadcast-add / activation / residual run on full rows
// with 16-byte loads and stores (the plain GEMM's per-lane 8-byte column stores cost
// ~5x at these 256-512 B rows).  The MLP keeps its 512-wide hidden activations on chip:
// per 128-wide hidden chunk, H = act(Xn . W1c^T + b1c) goes to LDS and is immediately
// contracted with W2c into the output accumulators, so neither the hidden tensor nor
// the LayerNorm output ever touch HBM.
#include "common.h"
#include "capi.h"

namespace {

constexpr int KD = 128;    // feature width of the rows
constexpr int NT = 256;    // 4 waves

// fp32 LDS images (row pitch 132 / 68 floats = 4 mod 32 dwords): rows with bit 3 set hold each
// 4-float chunk rotated by two (halves swapped), and fragment reads use k-lane q ^ 2 there, so the
// 16 rows x 2 k of a ds_read_b32 lane group fall on 32 distinct banks (rows r and r + 8 shared a
// bank pair); bf16 images are untouched
template <typename T>
DEV uint4 rot_row(uint4 u, int row) {
  if constexpr (sizeof(T) == 4) return ((row >> 3) & 1) ? make_uint4(u.z, u.w, u.x, u.y) : u;
  else return u;
}
DEV int rot_q(int q, int r) { return q ^ (((r >> 3) & 1) << 1); }

template <typename T> struct RB;
template <> struct RB<bf16> { static constexpr int BM = 128, PAD = 8, HC = 128; };
template <> struct RB<float> { static constexpr int BM = 64, PAD = 4, HC = 64; };

// ---- load BM rows of X (K = 128) into LDS, optionally LayerNorm'd ----------------------
template <typename T, int BM>
DEV void load_rows(const T* __restrict__ X, int64_t ldx, int64_t m0, int64_t M, const float* g, const float* b,
                   float eps, T* sX, int ld) {
  constexpr int VN = Vec16<T>::N, LPR = KD / VN, RPI = 64 / LPR;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = (lane % LPR) * VN;
  float gg[VN], bb[VN];
  if (g) {
#pragma unroll
    for (int j = 0; j < VN; ++j) { gg[j] = g[c + j]; bb[j] = b[c + j]; }
  }
  for (int r0 = wave * RPI; r0 < BM; r0 += 4 * RPI) {
    const int r = r0 + lane / LPR;
    const int64_t m = m0 + r;
    uint4 u = m < M ? ld16(X + m * ldx + c) : make_uint4(0, 0, 0, 0);
    if (g) {
      T* e = reinterpret_cast<T*>(&u);
      float v[VN], s = 0.f;
#pragma unroll
      for (int j = 0; j < VN; ++j) { v[j] = to_f<T>(e[j]); s += v[j]; }
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      const float mean = s * (1.f / KD);
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < VN; ++j) { v[j] -= mean; q += v[j] * v[j]; }
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
      const float rstd = rsqrtf(q * (1.f / KD) + eps);
#pragma unroll
      for (int j = 0; j < VN; ++j) e[j] = from_f<T>(v[j] * rstd * gg[j] + bb[j]);
    }
    st16(&sX[r * ld + c], rot_row<T>(u, r));
  }
}

// ---- stage a [ROWS][128] weight slab (row stride ldw) into LDS ------------------------
template <typename T, int ROWS>
DEV void load_w(const T* __restrict__ W, int64_t ldw, int rows_valid, T* sW, int ld) {
  constexpr int VN = Vec16<T>::N, CPR = KD / VN;
  for (int i = threadIdx.x; i < ROWS * CPR; i += NT) {
    const int r = i / CPR, c = (i % CPR) * VN;
    st16(&sW[r * ld + c], rot_row<T>(r < rows_valid ? ld16(W + (int64_t)r * ldw + c) : make_uint4(0, 0, 0, 0), r));
  }
}

// ---- acc[FN][FM] += sW[wn.., k] . sA[wm.., k]^T over K = 128 ---------------------------
template <typename T, int FN, int FM>
DEV void tile_mma(const T* sW, int ldw, const T* sA, int lda, int wn, int wm, f32x4 (&acc)[FN][FM]) {
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int ks = 0; ks < KD / 32; ++ks) {
      s16x8 bf[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) bf[j] = *reinterpret_cast<const s16x8*>(&sA[(wm + 16 * j + r) * lda + ks * 32 + 8 * q]);
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const s16x8 af = *reinterpret_cast<const s16x8*>(&sW[(wn + 16 * i + r) * ldw + ks * 32 + 8 * q]);
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(af, bf[j], acc[i][j]);
      }
    }
  } else {
    const int qr = rot_q(q, r);
#pragma unroll 4
    for (int s = 0; s < KD / 4; ++s) {
      float bv[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) bv[j] = sA[(wm + 16 * j + r) * lda + 4 * s + qr];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const float av = sW[(wn + 16 * i + r) * ldw + 4 * s + qr];
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_f32(av, bv[j], acc[i][j]);
      }
    }
  }
}

template <int FN, int FM>
DEV void zero(f32x4 (&acc)[FN][FM]) {
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// accumulators -> fp32 stage [m][n] (row stride sld)
template <int FN, int FM>
DEV void stage_acc(float* st, int sld, int wn, int wm, const f32x4 (&acc)[FN][FM]) {
  const int lane = threadIdx.x & 63, col = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j)
      *reinterpret_cast<f32x4*>(&st[(wm + 16 * j + col) * sld + wn + 16 * i + rq]) = acc[i][j];
}

struct Epi {
  const float* bias;
  const void* add; int64_t ld_add; RowMap addmap; int add_ncols;
  int act;
  const void* res; int64_t ld_res;
  const void* res2; int64_t ld_res2;
  void* out; int64_t ldo;
  int store_mode, cvt_k, cvt_hin, cvt_win, cvt_cout;
};

// fp32 stage [BM][BN] -> epilogue -> global, 8 consecutive columns per thread
template <typename T, int BM, int BN>
DEV void store_rows(const float* st, int sld, int64_t m0, int64_t M, int n0, const Epi& e) {
  constexpr int CH = BN / 8;
  for (int i = threadIdx.x; i < BM * CH; i += NT) {
    const int r = i / CH, c = (i % CH) * 8;
    const int64_t m = m0 + r;
    if (m >= M) continue;
    const int n = n0 + c;
    float v[8];
    *reinterpret_cast<f32x4*>(&v[0]) = *reinterpret_cast<const f32x4*>(&st[r * sld + c]);
    *reinterpret_cast<f32x4*>(&v[4]) = *reinterpret_cast<const f32x4*>(&st[r * sld + c + 4]);
    if (e.bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += e.bias[n + j];
    }
    if (e.add && n < e.add_ncols) {
      const T* a = reinterpret_cast<const T*>(e.add) + rowmap(e.addmap, m) * e.ld_add + n;
      float t[8];
      load4<T>(a, t); load4<T>(a + 4, t + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t[j];
    }
    if (e.act != ACT_NONE) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = apply_act(v[j], e.act);
    }
    if (e.res) {
      const T* a = reinterpret_cast<const T*>(e.res) + m * e.ld_res + n;
      float t[8];
      load4<T>(a, t); load4<T>(a + 4, t + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t[j];
    }
    if (e.res2) {
      const T* a = reinterpret_cast<const T*>(e.res2) + m * e.ld_res2 + n;
      float t[8];
      load4<T>(a, t); load4<T>(a + 4, t + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t[j];
    }
    int64_t off;
    if (e.store_mode == 0) {
      off = m * e.ldo + n;
    } else {
      off = convt_offset(m, n, e.cvt_k, e.cvt_hin, e.cvt_win, e.cvt_cout);
    }
    T* o = reinterpret_cast<T*>(e.out) + off;
    store4<T>(o, v);
    store4<T>(o + 4, v + 4);
  }
}

// ============================ rows_gemm =============================================
template <typename T>
__global__ __launch_bounds__(NT) void rows_gemm_kernel(const T* __restrict__ X, int64_t ldx, int64_t M,
                                                       const float* ln_g, const float* ln_b, float eps,
                                                       const T* __restrict__ W, int N, Epi e) {
  constexpr int BM = RB<T>::BM, BN = sizeof(T) == 2 ? 128 : 64;
  constexpr int LD = KD + RB<T>::PAD;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int SLD = BN + 4;
  constexpr int AB = BM * LD * sizeof(T), WB = BN * LD * sizeof(T), SB = BM * SLD * 4;
  constexpr int LDS = (AB + WB) > SB ? (AB + WB) : SB;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  T* sA = reinterpret_cast<T*>(smem);
  T* sW = reinterpret_cast<T*>(smem + AB);
  float* st = reinterpret_cast<float*>(smem);

  const int wave = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  if constexpr (sizeof(T) == 4) {
    // fp32: one workgroup walks every BN-column block of its rows (grid.y = 1), so the rows are
    // loaded and LayerNorm'd once instead of once per block (6x for the 384-wide q|k|v GEMM); the
    // accumulator stage reuses the weight slab's LDS, the rows stay put
    static_assert(BM * SLD * 4 <= WB, "fp32 stage must fit in the weight slab");
    float* st4 = reinterpret_cast<float*>(smem + AB);
    load_rows<T, BM>(X, ldx, m0, M, ln_g, ln_b, eps, sA, LD);
    const int wm = (wave & 1) * WM, wn = (wave >> 1) * WN;
    for (int n0 = 0; n0 < N; n0 += BN) {
      load_w<T, BN>(W + (int64_t)n0 * KD, KD, min(BN, N - n0), sW, LD);
      __syncthreads();
      f32x4 acc[FN][FM];
      zero(acc);
      tile_mma<T, FN, FM>(sW, LD, sA, LD, wn, wm, acc);
      __syncthreads();
      stage_acc(st4, SLD, wn, wm, acc);
      __syncthreads();
      store_rows<T, BM, BN>(st4, SLD, m0, M, n0, e);
      __syncthreads();
    }
    return;
  }
  const int n0 = blockIdx.y * BN;
  load_rows<T, BM>(X, ldx, m0, M, ln_g, ln_b, eps, sA, LD);
  load_w<T, BN>(W + (int64_t)n0 * KD, KD, min(BN, N - n0), sW, LD);
  __syncthreads();
  const int wm = (wave & 1) * WM, wn = (wave >> 1) * WN;
  f32x4 acc[FN][FM];
  zero(acc);
  tile_mma<T, FN, FM>(sW, LD, sA, LD, wn, wm, acc);
  __syncthreads();
  stage_acc(st, SLD, wn, wm, acc);
  __syncthreads();
  store_rows<T, BM, BN>(st, SLD, m0, M, n0, e);
}

// ============================ rows_mlp ==============================================
template <typename T>
__global__ __launch_bounds__(NT) void rows_mlp_kernel(const T* __restrict__ Y, int64_t ldy, int64_t M,
                                                      const float* ln_g, const float* ln_b, float eps,
                                                      const T* __restrict__ W1, const float* b1, int hidden, int act,
                                                      const T* __restrict__ W2, Epi e) {
  constexpr int BM = RB<T>::BM, HC = RB<T>::HC;
  constexpr int LD = KD + RB<T>::PAD, LDH = HC + RB<T>::PAD;
  constexpr int XB = BM * LD * sizeof(T), HB = BM * LDH * sizeof(T), W1B = HC * LD * sizeof(T),
                W2B = KD * LDH * sizeof(T);
  constexpr int SLD = KD + 4, SB = BM * SLD * 4;
  constexpr int LDS = (XB + HB + W1B + W2B) > SB ? (XB + HB + W1B + W2B) : SB;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  T* sX = reinterpret_cast<T*>(smem);
  T* sH = reinterpret_cast<T*>(smem + XB);
  T* sW1 = reinterpret_cast<T*>(smem + XB + HB);
  T* sW2 = reinterpret_cast<T*>(smem + XB + HB + W1B);
  float* st = reinterpret_cast<float*>(smem);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  load_rows<T, BM>(Y, ldy, m0, M, ln_g, ln_b, eps, sX, LD);

  // GEMM1 tile: (HC hidden) x (BM rows); GEMM2 tile: (128 out) x (BM rows); 2x2 waves each
  constexpr int W1N = HC / 2, W1M = BM / 2, F1N = W1N / 16, F1M = W1M / 16;
  constexpr int W2N = KD / 2, W2M = BM / 2, F2N = W2N / 16, F2M = W2M / 16;
  const int wm = (wave & 1) * (BM / 2);
  const int wn1 = (wave >> 1) * W1N, wn2 = (wave >> 1) * W2N;
  f32x4 acc2[F2N][F2M];
  zero(acc2);
  const int col = lane & 15, rq = (lane >> 4) * 4;
  for (int h0 = 0; h0 < hidden; h0 += HC) {
    // stage W1[h0:h0+HC, :] as [hid][k] and W2[:, h0:h0+HC] as [out][hid]
    load_w<T, HC>(W1 + (int64_t)h0 * KD, KD, HC, sW1, LD);
    {
      constexpr int VN = Vec16<T>::N, CPR = HC / VN;
      for (int i = threadIdx.x; i < KD * CPR; i += NT) {
        const int r = i / CPR, c = (i % CPR) * VN;
        st16(&sW2[r * LDH + c], rot_row<T>(ld16(W2 + (int64_t)r * hidden + h0 + c), r));
      }
    }
    __syncthreads();
    f32x4 acc1[F1N][F1M];
    zero(acc1);
    tile_mma<T, F1N, F1M>(sW1, LD, sX, LD, wn1, wm, acc1);
    // h = act(acc1 + b1) -> sH[m][hid]
#pragma unroll
    for (int i = 0; i < F1N; ++i) {
      const int hh = wn1 + 16 * i + rq;
      const float4 bv = *reinterpret_cast<const float4*>(b1 + h0 + hh);
      const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int j = 0; j < F1M; ++j) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(acc1[i][j][r] + bb[r], act);
        if constexpr (sizeof(T) == 4) {
          if ((col >> 3) & 1) {               // rot_row's layout for the fp32 hidden tile
            const float t0 = v[0], t1 = v[1];
            v[0] = v[2]; v[1] = v[3]; v[2] = t0; v[3] = t1;
          }
        }
        store4<T>(&sH[(wm + 16 * j + col) * LDH + hh], v);
      }
    }
    __syncthreads();
    // acc2 += sH . W2c^T   (K = HC)
    if constexpr (sizeof(T) == 2) {
      const int r = lane & 15, q = lane >> 4;
#pragma unroll
      for (int ks = 0; ks < HC / 32; ++ks) {
        s16x8 bf[F2M];
#pragma unroll
        for (int j = 0; j < F2M; ++j) bf[j] = *reinterpret_cast<const s16x8*>(&sH[(wm + 16 * j + r) * LDH + ks * 32 + 8 * q]);
#pragma unroll
        for (int i = 0; i < F2N; ++i) {
          const s16x8 af = *reinterpret_cast<const s16x8*>(&sW2[(wn2 + 16 * i + r) * LDH + ks * 32 + 8 * q]);
#pragma unroll
          for (int j = 0; j < F2M; ++j) acc2[i][j] = mfma_bf16(af, bf[j], acc2[i][j]);
        }
      }
    } else {
      const int r = lane & 15, q = rot_q(lane >> 4, lane & 15);
#pragma unroll 4
      for (int s = 0; s < HC / 4; ++s) {
        float bv[F2M];
#pragma unroll
        for (int j = 0; j < F2M; ++j) bv[j] = sH[(wm + 16 * j + r) * LDH + 4 * s + q];
#pragma unroll
        for (int i = 0; i < F2N; ++i) {
          const float av = sW2[(wn2 + 16 * i + r) * LDH + 4 * s + q];
#pragma unroll
          for (int j = 0; j < F2M; ++j) acc2[i][j] = mfma_f32(av, bv[j], acc2[i][j]);
        }
      }
    }
    __syncthreads();
  }
  stage_acc(st, SLD, wn2, wm, acc2);
  __syncthreads();
  store_rows<T, BM, KD>(st, SLD, m0, M, 0, e);
}

Epi make_epi(const CatsegRowsEpi* p) {
  Epi e;
  e.bias = p->bias;
  e.add = p->add; e.ld_add = p->ld_add; e.add_ncols = (int)p->add_ncols;
  e.addmap = RowMap{p->addmap.d1, p->addmap.m1, p->addmap.s1, p->addmap.d2, p->addmap.m2, p->addmap.s2, p->addmap.off};
  e.act = p->act;
  e.res = p->res; e.ld_res = p->ld_res; e.res2 = p->res2; e.ld_res2 = p->ld_res2;
  e.out = p->out; e.ldo = p->ldo;
  e.store_mode = p->store_mode; e.cvt_k = p->cvt_k; e.cvt_hin = p->cvt_hin; e.cvt_win = p->cvt_win;
  e.cvt_cout = p->cvt_cout;
  return e;
}

int check_epi(const CatsegRowsEpi* p, int n_total) {
  CATSEG_CHECK(p->out, "rows: out missing");
  CATSEG_CHECK(p->store_mode != 0 || p->ldo % 8 == 0, "rows: ldo must be a multiple of 8");
  CATSEG_CHECK(!p->add || (p->ld_add % 8 == 0 && p->add_ncols % 8 == 0 && p->addmap.d1 > 0 && p->addmap.m1 > 0 &&
                           p->addmap.d2 > 0 && p->addmap.m2 > 0), "rows: bad add operand");
  CATSEG_CHECK(!p->res || p->ld_res % 8 == 0, "rows: ld_res must be a multiple of 8");
  CATSEG_CHECK(!p->res2 || p->ld_res2 % 8 == 0, "rows: ld_res2 must be a multiple of 8");
  CATSEG_CHECK(p->store_mode == 0 || (p->cvt_cout % 8 == 0 && n_total == p->cvt_k * p->cvt_k * p->cvt_cout),
               "rows: bad ConvTranspose scatter geometry");
  return 0;
}

}  // namespace

// persistent register-weight variants (rowpersist.hip); 0 = launched, 1 = not applicable
int catseg_rows_gemm_persistent(const void* x, int64_t ld_x, int64_t M, const float* g, const float* b, float eps,
                                const void* w, int64_t N, const CatsegRowsEpi* epi, hipStream_t st);
int catseg_rows_mlp_persistent(const void* y, int64_t ld_y, int64_t M, const float* g, const float* b, float eps,
                               const void* w1, const float* b1, int64_t hidden, int act, const void* w2,
                               const CatsegRowsEpi* epi, hipStream_t st);

int g_persistent = 1;
CATSEG_KNOB(g_persistent, "persistent");

extern "C" int catseg_rows_gemm(const void* x, int64_t ld_x, int64_t M, const float* ln_gamma, const float* ln_beta,
                                float eps, const void* w, int64_t N, const CatsegRowsEpi* epi, int dtype,
                                void* stream) {
  CATSEG_CHECK(x && w && epi && M > 0 && N > 0, "rows_gemm: bad args");
  const int bn = dtype == CATSEG_BF16 ? 128 : 64;
  CATSEG_CHECK(N % bn == 0, "rows_gemm: N must be a multiple of 128 (bf16) / 64 (f32)");
  CATSEG_CHECK(ld_x % 8 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0, "rows_gemm: alignment");
  CATSEG_CHECK(!ln_gamma || ln_beta, "rows_gemm: ln_beta missing");
  if (int rc = check_epi(epi, (int)N)) return rc;
  CATSEG_CHECK(epi->store_mode == 0 || M < (1LL << 31), "rows_gemm: ConvTranspose row count must fit 31 bits");
  Epi e = make_epi(epi);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CATSEG_BF16 && g_persistent &&
      catseg_rows_gemm_persistent(x, ld_x, M, ln_gamma, ln_beta, eps, w, N, epi, st) == 0)
    return catseg_launch_status("rows_gemm");
  if (dtype == CATSEG_BF16) {
    dim3 grid((unsigned)((M + RB<bf16>::BM - 1) / RB<bf16>::BM), (unsigned)(N / 128));
    hipLaunchKernelGGL(rows_gemm_kernel<bf16>, grid, dim3(NT), 0, st, (const bf16*)x, ld_x, M, ln_gamma, ln_beta, eps,
                       (const bf16*)w, (int)N, e);
  } else {
    dim3 grid((unsigned)((M + RB<float>::BM - 1) / RB<float>::BM), 1u);   // the kernel walks the N / 64 blocks
    hipLaunchKernelGGL(rows_gemm_kernel<float>, grid, dim3(NT), 0, st, (const float*)x, ld_x, M, ln_gamma, ln_beta,
                       eps, (const float*)w, (int)N, e);
  }
  return catseg_launch_status("rows_gemm");
}

extern "C" int catseg_rows_mlp(const void* y, int64_t ld_y, int64_t M, const float* ln_gamma, const float* ln_beta,
                               float eps, const void* w1, const float* b1, int64_t hidden, int act, const void* w2,
                               const CatsegRowsEpi* epi, int dtype, void* stream) {
  CATSEG_CHECK(y && w1 && b1 && w2 && epi && ln_gamma && ln_beta && M > 0, "rows_mlp: bad args");
  CATSEG_CHECK(hidden > 0 && hidden % 128 == 0, "rows_mlp: hidden must be a multiple of 128");
  CATSEG_CHECK(ld_y % 8 == 0 && epi->store_mode == 0, "rows_mlp: alignment / store mode");
  if (int rc = check_epi(epi, KD)) return rc;
  Epi e = make_epi(epi);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CATSEG_BF16 && g_persistent &&
      catseg_rows_mlp_persistent(y, ld_y, M, ln_gamma, ln_beta, eps, w1, b1, hidden, act, w2, epi, st) == 0)
    return catseg_launch_status("rows_mlp");
  if (dtype == CATSEG_BF16) {
    hipLaunchKernelGGL(rows_mlp_kernel<bf16>, dim3((unsigned)((M + RB<bf16>::BM - 1) / RB<bf16>::BM)), dim3(NT), 0, st,
                       (const bf16*)y, ld_y, M, ln_gamma, ln_beta, eps, (const bf16*)w1, b1, (int)hidden, act,
                       (const bf16*)w2, e);
  } else {
    hipLaunchKernelGGL(rows_mlp_kernel<float>, dim3((unsigned)((M + RB<float>::BM - 1) / RB<float>::BM)), dim3(NT), 0,
                       st, (const float*)y, ld_y, M, ln_gamma, ln_beta, eps, (const float*)w1, b1, (int)hidden, act,
                       (const float*)w2, e);
  }
  return catseg_launch_status("rows_mlp");
}
