// Training-side GEMMs (the network's backward).
//
// catseg_gemm_ex: the general fp32 contraction the backward needs in every operand layout
//   C[m][n] = alpha * sum_k A(m,k) B(k,n) + beta * C[m][n]
//   A(m,k) = A[m*a_sm + k*a_sk],  B(k,n) = B[k*b_sk + n*b_sn]
// with one unit stride per operand (the contiguous dimension is read in 16-byte vectors):
//   dX = dY . W          (A = dY rows, k-contiguous;   B = W [N_out][K_in], n-contiguous)
//   dW = dY^T . X        (A = dY^T,    m-contiguous;   B = X rows, n-contiguous; K = rows)
//   cost-volume grads    (model.py:648-652 einsum backward)
// so no operand is ever transposed in HBM.  Exact-f32 MFMA (v_mfma_f32_16x16x4_f32, fp32
// accumulate).  Tall reductions (K = the row count of a weight gradient) split K over
// grid.y into fp32 partials summed in a fixed order by a second kernel: deterministic,
// no atomics.
//
// catseg_colsum: out[c] = alpha * sum_r x[r][c] (+ beta * out[c]), the bias gradients,
// two-stage fixed-order reduction.
#include "common.h"
#include "capi.h"
#include "catseg_hip_train.h"

namespace {

constexpr int TBM = 128, TBN = 128, TBK = 16, TNT = 256;
// catseg_gemm_ex's product form (gemm_ex_kernel TERMS): -1 = automatic (6 for the tall reductions,
// K >= 8192 -- the weight gradients, K = the row count -- else 0), 0 = exact-f32 MFMA, 6 / 3 = split-bf16
// MFMA.  tools/micro_gemm_ex.py at the training shapes (4 x 171 x 576 rows of 128 / 512 channels):
// dW 484 -> 395 us (128 -> 512), 454 -> 402 (512 -> 128), 134 -> 123 (128 -> 128), 350 -> 310 (128 -> 384)
// at the f32 form's error (rel 7-10e-7 vs 6-8e-7); dX (K = 128 / 512) 446-509 vs 487-496 us, so it keeps
// the f32 form; TERMS 3 runs dW in 290-294 us at ~5e-6 (not used).
int g_gemm_ex_terms = -1;

// d act / d u in the GEMM epilogue.  GELU' = Phi(u) + u phi(u) with erf by Abramowitz & Stegun 7.1.26
// (|error| <= 1.5e-7) sharing its exp(-u^2 / 2) with phi: one exp + one rcp per value, where
// ocml erff + expf cost ~40 VALU (the epilogue runs once per output, outside the MFMA loop).
DEV float act_grad(float v, int act) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? 1.f : 0.f;
    case ACT_GELU: {
      const float z = fabsf(v) * 0.70710678118654752f;
      const float e = __expf(-z * z);                     // exp(-u^2 / 2)
      const float t = __frcp_rn(fmaf(0.3275911f, z, 1.f));
      float p = fmaf(1.061405429f, t, -1.453152027f);
      p = fmaf(p, t, 1.421413741f);
      p = fmaf(p, t, -0.284496736f);
      p = fmaf(p, t, 0.254829592f);
      const float erf_z = copysignf(1.f - p * t * e, v);
      return fmaf(0.5f, erf_z, 0.5f) + v * 0.39894228040143268f * e;
    }
    case ACT_QUICKGELU: {
      const float s = __frcp_rn(1.f + __expf(-1.702f * v));
      return s + 1.702f * v * s * (1.f - s);
    }
    default: return 1.f;
  }
}

constexpr int LP = TBM + 16;  // LDS row (one k) of a tile: 144 floats, the 4 k rows of a fragment read on
                               // disjoint 16-bank groups

// fp32 x -> the bf16 pieces x = p0 + p1 (+ p2) + (error <= 2^-24 |x| with three pieces): each piece is
// the round-to-nearest-even bf16 of what the previous ones left (v_cvt_pk_bf16_f32 per pair), and
// every residual x - p is exact in fp32.  Products of pieces are exact in the MFMA's fp32 accumulator.
template <int NP>
DEV void split_bf16(const float (&x)[8], s16x8 (&piece)[NP]) {
  float r[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = x[e];
#pragma unroll
  for (int pi = 0; pi < NP; ++pi) {
    unsigned w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      w[e] = f2bf2(r[2 * e], r[2 * e + 1]);
      if (pi + 1 < NP) {
        r[2 * e] -= __uint_as_float(w[e] << 16);
        r[2 * e + 1] -= __uint_as_float(w[e] & 0xffff0000u);
      }
    }
    uint4 u = make_uint4(w[0], w[1], w[2], w[3]);
    piece[pi] = *reinterpret_cast<s16x8*>(&u);
  }
}

// AM: A is m-contiguous (a_sm == 1) else k-contiguous (a_sk == 1).
// BN: B is n-contiguous (b_sn == 1) else k-contiguous (b_sk == 1).
// KS: k depth of one LDS slab (16, or 32 for the bf16 MFMA).
// TERMS: 0 = exact-f32 MFMA (v_mfma_f32_16x16x4_f32); 6 = the fp32 products from bf16 pieces
//   (3 per operand, split at fragment load): a b = sum over the 6 piece pairs (i, j) with i + j <= 2
//   of a_i b_j, smallest first, each one v_mfma_f32_16x16x32_bf16 (16 issue cycles for 32 k vs 8 x 32
//   for the f32 form); the dropped pairs are below 2^-24 |a b|, so the result is an fp32 GEMM's up
//   to accumulation order; 3 = pieces 0-1 only (a0 b0 + a0 b1 + a1 b0, ~2^-17 relative).
template <bool AM, bool BNC, int KS = TBK, int TERMS = 0>
__global__ __launch_bounds__(TNT) void gemm_ex_kernel(const float* __restrict__ A, int64_t a_sm, int64_t a_sk,
                                                      const float* __restrict__ B, int64_t b_sk, int64_t b_sn,
                                                      int64_t M, int64_t N, int64_t K, int64_t k_chunk,
                                                      float* __restrict__ C, int64_t ldc, float alpha, int beta,
                                                      float* __restrict__ part, int tiles_n,
                                                      const float* __restrict__ act_u, int64_t ld_u, int act) {
  static_assert(TERMS == 0 ? KS % 4 == 0 : KS % 32 == 0, "k slab");
  constexpr int CH = TBM * KS / 4 / TNT;        // 16-byte chunks per operand per thread per slab
  constexpr int CPK = KS / 4;                    // chunks per k-contiguous row of a slab
  __shared__ __attribute__((aligned(16))) float As[2][KS * LP];
  __shared__ __attribute__((aligned(16))) float Bs[2][KS * LP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntiles = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, ntiles);
  const int64_t m0 = (int64_t)(lin / tiles_n) * TBM, n0 = (int64_t)(lin % tiles_n) * TBN;
  const int64_t kb = (int64_t)blockIdx.y * k_chunk;
  const int64_t ke = kb + k_chunk < K ? kb + k_chunk : K;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;

  // staging: CH x 16-byte chunks per operand per thread per k-slab
  float4 ra[CH], rb[CH];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = tid + i * TNT;
      if constexpr (AM) {                      // chunk = 4 consecutive m at one k
        const int k = c >> 5, m4 = (c & 31) * 4;
        const int64_t gm = m0 + m4, gk = k0 + k;
        ra[i] = (gm < M && gk < ke) ? *reinterpret_cast<const float4*>(A + gm + gk * a_sk) : make_float4(0, 0, 0, 0);
      } else {                                 // chunk = 4 consecutive k at one m
        const int m = c / CPK, k4 = (c % CPK) * 4;
        const int64_t gm = m0 + m, gk = k0 + k4;
        ra[i] = (gm < M && gk < ke) ? *reinterpret_cast<const float4*>(A + gm * a_sm + gk) : make_float4(0, 0, 0, 0);
      }
      if constexpr (BNC) {
        const int k = c >> 5, n4 = (c & 31) * 4;
        const int64_t gn = n0 + n4, gk = k0 + k;
        rb[i] = (gn < N && gk < ke) ? *reinterpret_cast<const float4*>(B + gn + gk * b_sk) : make_float4(0, 0, 0, 0);
      } else {
        const int n = c / CPK, k4 = (c % CPK) * 4;
        const int64_t gn = n0 + n, gk = k0 + k4;
        rb[i] = (gn < N && gk < ke) ? *reinterpret_cast<const float4*>(B + gn * b_sn + gk) : make_float4(0, 0, 0, 0);
      }
    }
  };
  // LDS image [k][m] / [k][n] with the m (n) index XOR-swizzled by bits 2-3 of k:  element (k, m) at
  // k * LP + (m ^ swz(k)).  The k-contiguous operand's transposing stores (lanes: 8 m x 4 k-quads)
  // then hit 32 distinct banks per 32-lane group instead of 8 (4-way), and a fragment read (16 m x
  // lanes g = k & 3) keeps its 16 + 16 banks (swz is uniform over the 4 k of a read).
  auto swz = [](int k) { return ((k >> 2) & 3) << 3; };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = tid + i * TNT;
      if constexpr (AM) {
        const int k = c >> 5;
        *reinterpret_cast<float4*>(&As[buf][k * LP + (((c & 31) * 4) ^ swz(k))]) = ra[i];
      } else {
        const int m = c / CPK, k4 = (c % CPK) * 4, mm = m ^ swz(k4);
        As[buf][(k4 + 0) * LP + mm] = ra[i].x; As[buf][(k4 + 1) * LP + mm] = ra[i].y;
        As[buf][(k4 + 2) * LP + mm] = ra[i].z; As[buf][(k4 + 3) * LP + mm] = ra[i].w;
      }
      if constexpr (BNC) {
        const int k = c >> 5;
        *reinterpret_cast<float4*>(&Bs[buf][k * LP + (((c & 31) * 4) ^ swz(k))]) = rb[i];
      } else {
        const int n = c / CPK, k4 = (c % CPK) * 4, nn = n ^ swz(k4);
        Bs[buf][(k4 + 0) * LP + nn] = rb[i].x; Bs[buf][(k4 + 1) * LP + nn] = rb[i].y;
        Bs[buf][(k4 + 2) * LP + nn] = rb[i].z; Bs[buf][(k4 + 3) * LP + nn] = rb[i].w;
      }
    }
  };

  // D^T = B^T . A^T: the first MFMA operand is B^T (rows n), the second A^T (columns m), so a
  // lane ends with 4 consecutive n of one m (16-byte stores)
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((ke - kb + KS - 1) / KS);
  const int r = lane & 15, g = lane >> 4;
  if (nk > 0) {
    gload(kb);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kb + (int64_t)(kt + 1) * KS);
    const float* as = As[buf];
    const float* bs = Bs[buf];
    if constexpr (TERMS == 0) {
#pragma unroll
      for (int kk = 0; kk < KS; kk += 4) {
        float av[4], bv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) av[j] = as[(kk + g) * LP + ((wm + 16 * j + r) ^ swz(kk))];
#pragma unroll
        for (int i = 0; i < 4; ++i) bv[i] = bs[(kk + g) * LP + ((wn + 16 * i + r) ^ swz(kk))];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma_f32(bv[i], av[j], acc[i][j]);
      }
    } else {
      constexpr int NP = TERMS == 6 ? 3 : 2;
#pragma unroll
      for (int kk = 0; kk < KS; kk += 32) {
        // lane (r, g) holds k = kk + 8g .. +7 of its row (the 16x16x32 bf16 operand layout); the
        // swizzle of k is ((2g + e / 4) & 3) << 3 for element e
        const int k0 = kk + 8 * g;
        const int s0 = swz(k0), s1 = swz(k0 + 4);
        // the A pieces of all four m-fragments stay live; each n-fragment's pieces are made just
        // before its 4 x TERMS MFMAs (register pressure: two waves per SIMD)
        s16x8 ap[4][NP];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = wm + 16 * j + r;
          float x[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = as[(k0 + e) * LP + (m ^ (e < 4 ? s0 : s1))];
          split_bf16<NP>(x, ap[j]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = wn + 16 * i + r;
          float x[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = bs[(k0 + e) * LP + (n ^ (e < 4 ? s0 : s1))];
          s16x8 bp[NP];
          split_bf16<NP>(x, bp);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f32x4 c = acc[i][j];
            if constexpr (NP == 3) {
              c = mfma_bf16(bp[2], ap[j][0], c);
              c = mfma_bf16(bp[1], ap[j][1], c);
              c = mfma_bf16(bp[0], ap[j][2], c);
            }
            c = mfma_bf16(bp[1], ap[j][0], c);
            c = mfma_bf16(bp[0], ap[j][1], c);
            acc[i][j] = mfma_bf16(bp[0], ap[j][0], c);
          }
        }
      }
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds C[m = .. + r][n = .. + 4g .. 4g+3]
  float* dst = part ? part + (int64_t)blockIdx.y * M * N : C;
  const int64_t ld = part ? N : ldc;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t n = n0 + wn + 16 * i + 4 * g;
    if (n >= N) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = m0 + wm + 16 * j + r;
      if (m >= M) continue;
      float4* p = reinterpret_cast<float4*>(dst + m * ld + n);
      float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      if (!part) {
        v.x *= alpha; v.y *= alpha; v.z *= alpha; v.w *= alpha;
        if (act) {
          const float4 u = *reinterpret_cast<const float4*>(act_u + m * ld_u + n);
          v.x *= act_grad(u.x, act); v.y *= act_grad(u.y, act); v.z *= act_grad(u.z, act); v.w *= act_grad(u.w, act);
        }
        if (beta) { const float4 o = *p; v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w; }
      }
      *p = v;
    }
  }
}

// C[m][n] = alpha * sum_s part[s][m][n] + beta * C[m][n]: 16 float4 outputs x 16 split lanes per
// workgroup (lane z takes splits z, z + 16, ...), then a fixed tree over the lanes
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int splits, int64_t M,
                                                            int64_t N, float* __restrict__ C, int64_t ldc, float alpha,
                                                            int beta) {
  __shared__ float4 red[256];
  const int64_t n4 = N / 4, total = M * n4;
  const int ci = threadIdx.x & 15, zl = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + ci;
  float4 s = make_float4(0, 0, 0, 0);
  if (i < total) {
    const float4* p4 = reinterpret_cast<const float4*>(part) + i;
#pragma unroll 4
    for (int z = zl; z < splits; z += 16) {
      const float4 v = p4[(int64_t)z * total];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off >= 16; off >>= 1) {
    if ((int)threadIdx.x < off) {
      const float4 o = red[threadIdx.x + off];
      float4& r = red[threadIdx.x];
      r.x += o.x; r.y += o.y; r.z += o.z; r.w += o.w;
    }
    __syncthreads();
  }
  if (threadIdx.x < 16 && i < total) {
    const int64_t m = i / n4, n = (i % n4) * 4;
    float4 v = red[threadIdx.x];
    float4* p = reinterpret_cast<float4*>(C + m * ldc + n);
    v.x *= alpha; v.y *= alpha; v.z *= alpha; v.w *= alpha;
    if (beta) { const float4 o = *p; v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w; }
    *p = v;
  }
}

// Split count: only when the tiles alone leave CUs idle (< 256 tiles), then ~4 workgroups per CU
// (1024) of tiles x splits, each split at least 8 k-slabs (128 k), at most 512 splits.  Measured on
// the training step's shapes (tools/micro_gemm_ex_splits.py): 456 tiles x 3 splits of K 768 took
// 192 us against 119 unsplit (the partials' traffic), 16 tiles of K 2052 25 us at 16 splits against
// 34 at 8.  Depends on the shape only (never the device), so results are reproducible across parts.
int g_gemm_ex_splits = 0;   // tuning: > 0 forces the split count (capped by K / 16 and 512)
int gemm_ex_splits(int64_t M, int64_t N, int64_t K) {
  if (g_gemm_ex_splits > 0) {
    int64_t f = g_gemm_ex_splits, kmax = (K + TBK - 1) / TBK;
    if (f > kmax) f = kmax;
    return (int)(f > 512 ? 512 : f);
  }
  const int64_t tiles = ((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN);
  if (tiles >= 256) return 1;
  int64_t s = 1024 / tiles;                 // floor: tiles x splits <= 1024 resident slots (no tail round)
  const int64_t kmax = K / (TBK * 8);
  if (s > kmax) s = kmax;
  if (s > 512) s = 512;
  return s < 1 ? 1 : (int)s;
}

// column sums.  The rows are cut into `chunks` ranges of cr rows; one 256-thread workgroup per (column
// block, chunk): QW consecutive column vectors (V floats: 16-byte loads when the layout allows) x
// 256/QW row lanes, so a wave reads whole row segments; the row lanes reduce by a fixed tree and
// write part[chunk][col].  The final pass sums the chunks per column with 16 lanes and a fixed tree.
// chunks and cr depend on (rows, cols) only: deterministic.
constexpr int COLSUM_MAX_CHUNKS = 2048;
struct ColsumPlan {
  int v, qw, gx;
  int64_t chunks, cr;
};
ColsumPlan colsum_plan(int64_t rows, int64_t cols, int64_t ld, uintptr_t x) {
  ColsumPlan p;
  p.v = (cols % 4 == 0 && ld % 4 == 0 && x % 16 == 0) ? 4 : 1;
  const int64_t nv = cols / p.v;
  int qw = 1;
  while (qw < nv && qw < 64) qw <<= 1;
  p.qw = qw;
  p.gx = (int)((nv + qw - 1) / qw);
  int64_t ch = (rows + 63) / 64;
  const int64_t cap = (COLSUM_MAX_CHUNKS + p.gx - 1) / p.gx;
  if (ch > cap) ch = cap;
  if (ch < 1) ch = 1;
  p.cr = (rows + ch - 1) / ch;
  p.chunks = (rows + p.cr - 1) / p.cr;
  return p;
}

template <int V>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x, int64_t ld, int64_t rows,
                                                             int64_t cols, int qw, int64_t cr, float* __restrict__ part) {
  __shared__ float red[V][256];
  const int qi = threadIdx.x & (qw - 1), rl = threadIdx.x / qw, nrl = 256 / qw;
  const int64_t vec = (int64_t)blockIdx.x * qw + qi;
  const int64_t r0 = (int64_t)blockIdx.y * cr;
  const int64_t r1 = r0 + cr < rows ? r0 + cr : rows;
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  if (vec * V < cols) {
    if constexpr (V == 4) {
      const float4* xv = reinterpret_cast<const float4*>(x) + vec;
      const int64_t ldv = ld / 4;
#pragma unroll 4
      for (int64_t r = r0 + rl; r < r1; r += nrl) {
        const float4 t = xv[r * ldv];
        acc[0] += t.x; acc[1] += t.y; acc[2] += t.z; acc[3] += t.w;
      }
    } else {
#pragma unroll 4
      for (int64_t r = r0 + rl; r < r1; r += nrl) acc[0] += x[r * ld + vec];
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) red[j][threadIdx.x] = acc[j];
  __syncthreads();
  for (int off = 128; off >= qw; off >>= 1) {
    if ((int)threadIdx.x < off) {
#pragma unroll
      for (int j = 0; j < V; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + off];
    }
    __syncthreads();
  }
  if ((int)threadIdx.x < qw && vec * V < cols) {
#pragma unroll
    for (int j = 0; j < V; ++j) part[(int64_t)blockIdx.y * cols + vec * V + j] = red[j][threadIdx.x];
  }
}

// out[c] = alpha * sum_z part[z][c] (+ beta * out[c]); 16 columns x 16 chunk lanes per workgroup
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int64_t chunks, int64_t cols,
                                                           float* __restrict__ out, float alpha, int beta) {
  __shared__ float red[256];
  const int ci = threadIdx.x & 15, zl = threadIdx.x >> 4;
  const int64_t c = (int64_t)blockIdx.x * 16 + ci;
  float s = 0.f;
  if (c < cols) {
#pragma unroll 8
    for (int64_t z = zl; z < chunks; z += 16) s += part[z * cols + c];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off >= 16; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x < 16 && c < cols) out[c] = alpha * red[threadIdx.x] + (beta ? out[c] : 0.f);
}

}  // namespace

CATSEG_KNOB(g_gemm_ex_splits, "gemm_ex_splits");
CATSEG_KNOB(g_gemm_ex_terms, "gemm_ex_terms");

extern "C" int64_t catseg_gemm_ex_workspace(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int s = gemm_ex_splits(M, N, K);
  return s > 1 ? (int64_t)s * M * N * (int64_t)sizeof(float) : 0;
}

extern "C" int catseg_gemm_ex(const CatsegGemmExArgs* g, void* stream) {
  CATSEG_CHECK(g && g->A && g->B && g->C, "gemm_ex: null pointer");
  CATSEG_CHECK(g->M > 0 && g->N > 0 && g->K > 0, "gemm_ex: empty shape");
  const bool am = g->a_sm == 1, ak = g->a_sk == 1, bn = g->b_sn == 1, bk = g->b_sk == 1;
  CATSEG_CHECK(am || ak, "gemm_ex: A needs a unit stride (a_sm or a_sk == 1)");
  CATSEG_CHECK(bn || bk, "gemm_ex: B needs a unit stride (b_sn or b_sk == 1)");
  const bool AM = am && (!ak || (g->M % 4 == 0 && g->a_sk % 4 == 0));
  const bool BNC = bn && (!bk || (g->N % 4 == 0 && g->b_sk % 4 == 0));
  // the contiguous extent and the other stride must keep 16-byte vectors aligned
  if (AM) CATSEG_CHECK(g->M % 4 == 0 && g->a_sk % 4 == 0, "gemm_ex: m-contiguous A needs M % 4 == 0, a_sk % 4 == 0");
  else CATSEG_CHECK(g->K % 4 == 0 && g->a_sm % 4 == 0, "gemm_ex: k-contiguous A needs K % 4 == 0, a_sm % 4 == 0");
  if (BNC) CATSEG_CHECK(g->N % 4 == 0 && g->b_sk % 4 == 0, "gemm_ex: n-contiguous B needs N % 4 == 0, b_sk % 4 == 0");
  else CATSEG_CHECK(g->K % 4 == 0 && g->b_sn % 4 == 0, "gemm_ex: k-contiguous B needs K % 4 == 0, b_sn % 4 == 0");
  CATSEG_CHECK(g->N % 4 == 0 && g->ldc % 4 == 0 && g->ldc >= g->N, "gemm_ex: C needs N % 4 == 0, ldc % 4 == 0, ldc >= N");
  CATSEG_CHECK(((uintptr_t)g->A % 16) == 0 && ((uintptr_t)g->B % 16) == 0 && ((uintptr_t)g->C % 16) == 0,
               "gemm_ex: A, B, C must be 16-byte aligned");
  const int64_t tm = (g->M + TBM - 1) / TBM, tn = (g->N + TBN - 1) / TBN;
  CATSEG_CHECK(tm * tn < (1LL << 31), "gemm_ex: too many tiles");
  const int act = g->act;
  CATSEG_CHECK(act == ACT_NONE || act == ACT_RELU || act == ACT_GELU || act == ACT_QUICKGELU, "gemm_ex: bad act");
  if (act) {
    CATSEG_CHECK(g->act_u && g->ld_u >= g->N && g->ld_u % 4 == 0 && ((uintptr_t)g->act_u % 16) == 0 && !g->beta,
                 "gemm_ex: the act epilogue needs 16-byte aligned act_u rows (ld_u % 4 == 0) and beta == 0");
  }
  const int splits = act ? 1 : gemm_ex_splits(g->M, g->N, g->K);   // the epilogue runs unsplit
  const int64_t ws_need = splits > 1 ? (int64_t)splits * g->M * g->N * (int64_t)sizeof(float) : 0;
  if (splits > 1) CATSEG_CHECK(g->workspace && g->workspace_bytes >= ws_need, "gemm_ex: workspace too small");
  int64_t kc = (g->K + splits - 1) / splits;
  const int terms = g_gemm_ex_terms >= 0 ? g_gemm_ex_terms : (g->K >= 8192 ? 6 : 0);
  const int ks = terms ? 32 : TBK;
  kc = (kc + ks - 1) / ks * ks;
  hipStream_t st = (hipStream_t)stream;
  float* part = splits > 1 ? (float*)g->workspace : nullptr;
  dim3 grid((unsigned)(tm * tn), (unsigned)splits);
#define GEX(a_, b_, ks_, t_) hipLaunchKernelGGL((gemm_ex_kernel<a_, b_, ks_, t_>), grid, dim3(TNT), 0, st, (const float*)g->A, \
                                       g->a_sm, g->a_sk, (const float*)g->B, g->b_sk, g->b_sn, g->M, g->N, g->K, kc, \
                                       (float*)g->C, g->ldc, g->alpha, g->beta, part, (int)tn, (const float*)g->act_u, \
                                       g->ld_u, act)
#define GEX4(ks_, t_)                      \
  if (AM && BNC) GEX(true, true, ks_, t_); \
  else if (AM) GEX(true, false, ks_, t_);  \
  else if (BNC) GEX(false, true, ks_, t_); \
  else GEX(false, false, ks_, t_);
  if (terms == 6) { GEX4(32, 6) }
  else if (terms == 3) { GEX4(32, 3) }
  else { GEX4(TBK, 0) }
#undef GEX4
#undef GEX
  if (splits > 1) {
    const int64_t n = g->M * (g->N / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, st, part, splits, g->M,
                       g->N, (float*)g->C, g->ldc, g->alpha, g->beta);
  }
  return catseg_launch_status("gemm_ex");
}

extern "C" int64_t catseg_colsum_workspace(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  // the larger of the 16-byte-load plan and the scalar plan (the launch picks one by ld / alignment)
  const int64_t a = colsum_plan(rows, cols, cols, 0).chunks, b = colsum_plan(rows, cols, cols, 1).chunks;
  return (a > b ? a : b) * cols * (int64_t)sizeof(float);
}

extern "C" int catseg_colsum(const float* x, int64_t ld, int64_t rows, int64_t cols, float* out, float alpha, int beta,
                             void* workspace, int64_t workspace_bytes, void* stream) {
  CATSEG_CHECK(x && out && rows > 0 && cols > 0 && ld >= cols, "colsum: bad args");
  const ColsumPlan p = colsum_plan(rows, cols, ld, (uintptr_t)x);
  CATSEG_CHECK(workspace && workspace_bytes >= p.chunks * cols * (int64_t)sizeof(float), "colsum: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)p.gx, (unsigned)p.chunks);
  if (p.v == 4)
    hipLaunchKernelGGL(colsum_partial_kernel<4>, grid, dim3(256), 0, st, x, ld, rows, cols, p.qw, p.cr, (float*)workspace);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<1>, grid, dim3(256), 0, st, x, ld, rows, cols, p.qw, p.cr, (float*)workspace);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)((cols + 15) / 16)), dim3(256), 0, st, (const float*)workspace,
                     p.chunks, cols, out, alpha, beta);
  return catseg_launch_status("colsum");
}
