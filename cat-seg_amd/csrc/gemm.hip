// MFMA GEMM with fused epilogue:  out[m, n] = act(alpha-free) ...
//
//   v = sum_k A[amap(m), k] * W[n, k]            (fp32 accumulate)
//   v += bias[n]                                 (optional, fp32)
//   v += add[addmap(m), n]   for n < add_ncols   (optional: per-image / per-class
//                                                 guidance terms, CLS broadcast)
//   v = act(v) * alpha
//   v += res[m, n] + res2[m, n]                  (optional residual streams)
//   out[store(m, n)] = v                          (row-major or ConvTranspose scatter)
//
// W is in nn.Linear layout [N, K] (K contiguous), as are A's rows, so both MFMA
// operands are K-contiguous 16-byte fragments.  The product is computed as
// D = W_tile . A_tile^T, so each lane ends with 4 CONSECUTIVE output columns of one
// row (C/D layout row = 4*(lane>>4)+r -> n, col = lane&15 -> m): one 8/16-byte
// vector store per fragment, and bias/residual loads are vectors too.
//
// This serves every GEMM-shaped op on the path: ViT QKV / out-proj / MLP,
// ln_post@proj, patch-embed (im2col), Swin and class-attention projections and
// MLPs, the cost volume, ConvTranspose2d (store mode 1) and the guidance terms.
#include "common.h"
#include "capi.h"

namespace {

constexpr int BK = 32;
constexpr int NT = 256;   // 4 waves

template <typename TA> struct Lds;
template <> struct Lds<bf16> { static constexpr int PAD = 8; };   // row = 40 bf16 = 80 B
template <> struct Lds<float> { static constexpr int PAD = 4; };  // row = 36 f32 = 144 B

struct EpiArgs {
  const float* bias;
  const void* add; int64_t ld_add; RowMap addmap; int64_t add_ncols;
  int act; float alpha;
  const void* res; int64_t ld_res;
  const void* res2; int64_t ld_res2;
  void* out; int64_t ldo;
  int store_mode; int cvt_k, cvt_hin, cvt_win, cvt_cout;
  const float* sa; const float* sw;   // fp8 path: per-row scales of A and W (dequant in the epilogue)
  int pf;                             // gemm3 lean epilogue: next round's residual in flight (g_epi_prefetch)
};

template <typename TO>
DEV void epilogue4(const EpiArgs& e, int64_t m, int64_t n, f32x4 acc) {
  float v[4] = {acc[0], acc[1], acc[2], acc[3]};
  if (e.bias) {
    float4 b = *reinterpret_cast<const float4*>(e.bias + n);
    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
  }
  if (e.add && n < e.add_ncols) {
    float a[4];
    load4<TO>(reinterpret_cast<const TO*>(e.add) + rowmap(e.addmap, m) * e.ld_add + n, a);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += a[r];
  }
  if (e.act != ACT_NONE || e.alpha != 1.f) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], e.act) * e.alpha;
  }
  if (e.res) {
    float a[4];
    load4<TO>(reinterpret_cast<const TO*>(e.res) + m * e.ld_res + n, a);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += a[r];
  }
  if (e.res2) {
    float a[4];
    load4<TO>(reinterpret_cast<const TO*>(e.res2) + m * e.ld_res2 + n, a);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += a[r];
  }
  int64_t off;
  if (e.store_mode == 0) {
    off = m * e.ldo + n;
  } else {   // ConvTranspose2d(k, stride k) scatter: m = (s, y, x), n = (ky, kx, co)
    off = convt_offset(m, n, e.cvt_k, e.cvt_hin, e.cvt_win, e.cvt_cout);
  }
  store4<TO>(reinterpret_cast<TO*>(e.out) + off, v);
}

// 8 consecutive output columns of one row (row-major store only): 16-byte bf16 stores,
// the form the LDS-staged epilogues use (an 8-byte store per lane halves the per-CU
// store rate, MI355X_MICROARCH.md "attention epilogue store tail").
DEV void load8f(const float* p, float v[8]) { load4<float>(p, v); load4<float>(p + 4, v + 4); }
DEV void load8f(const bf16* p, float v[8]) {
  const uint4 u = ld16(p);
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
}
DEV void store8f(float* p, const float v[8]) { store4<float>(p, v); store4<float>(p + 4, v + 4); }
DEV void store8f(bf16* p, const float v[8]) {
  st16(p, make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7])));
}

// EPI selects a compile-time epilogue: 0 = general (every runtime option), 1 = bias (+ res),
// 2 = bias + QuickGELU.  The lean forms drop the unused paths' code and registers, which the
// epilogue-heavy ViT GEMMs measurably feel (a dead scatter branch alone cost QKV 2.5 us).
template <typename TO, bool SC = false, int EPI = 0>
DEV void epilogue8(const EpiArgs& e, int64_t m, int64_t n, f32x4 lo, f32x4 hi) {
  float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  if constexpr (EPI != 0) {
    if (e.bias) {
      float b[8];
      load8f(e.bias + n, b);
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] += b[r];
    }
    if constexpr (EPI == 2) {
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = apply_act(v[r], ACT_QUICKGELU);
    }
    if constexpr (EPI == 1) {
      if (e.res) {
        float a[8];
        load8f(reinterpret_cast<const TO*>(e.res) + m * e.ld_res + n, a);
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] += a[r];
      }
    }
    store8f(reinterpret_cast<TO*>(e.out) + m * e.ldo + n, v);
    return;
  }
  if (e.bias) {
    float b[8];
    load8f(e.bias + n, b);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += b[r];
  }
  if (e.add && n < e.add_ncols) {     // add_ncols is a multiple of 8 on the 8-wide path
    float a[8];
    load8f(reinterpret_cast<const TO*>(e.add) + rowmap(e.addmap, m) * e.ld_add + n, a);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += a[r];
  }
  if (e.act != ACT_NONE || e.alpha != 1.f) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = apply_act(v[r], e.act) * e.alpha;
  }
  if (e.res) {
    float a[8];
    load8f(reinterpret_cast<const TO*>(e.res) + m * e.ld_res + n, a);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += a[r];
  }
  if (e.res2) {
    float a[8];
    load8f(reinterpret_cast<const TO*>(e.res2) + m * e.ld_res2 + n, a);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += a[r];
  }
  int64_t off = m * e.ldo + n;
  if constexpr (SC) {   // ConvTranspose2d scatter (as epilogue4); cout % 8 == 0 keeps the 8 columns together
    off = convt_offset(m, n, e.cvt_k, e.cvt_hin, e.cvt_win, e.cvt_cout);
  }
  store8f(reinterpret_cast<TO*>(e.out) + off, v);
}

template <typename TA, typename TO, int BM, int BN>
__global__ __launch_bounds__(NT) void gemm_kernel(const TA* __restrict__ A, int64_t lda, RowMap amap,
                                                  const TA* __restrict__ W, int64_t ldw,
                                                  int64_t M, int64_t N, int64_t K, EpiArgs e) {
  constexpr int VN = Vec16<TA>::N;           // elements per 16-byte chunk
  // fp32 K-tile 16 (bf16: 32): 37 KB of LDS per 128 x 128 workgroup, four workgroups per CU
  constexpr int BKT = sizeof(TA) == 4 ? 16 : BK;
  constexpr int CPR = BKT / VN;              // chunks per tile row
  constexpr int LDR = BKT + Lds<TA>::PAD;    // LDS row stride (elements)
  constexpr int A_CH = BM * CPR / NT;        // chunks per thread
  constexpr int W_CH = BN * CPR / NT;
  static_assert(A_CH >= 1 && W_CH >= 1, "tile too small");
  constexpr int WM = BM / 2, WN = BN / 2;    // wave tile (2x2 waves)
  constexpr int FM = WM / 16, FN = WN / 16;

  __shared__ __attribute__((aligned(16))) TA sA[2][BM * LDR];
  __shared__ __attribute__((aligned(16))) TA sW[2][BN * LDR];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  const int wm = (wave & 1) * WM, wn = (wave >> 1) * WN;

  // per-thread staging rows (fixed over the K loop)
  const TA* a_ptr[A_CH]; int a_lrow[A_CH], a_col[A_CH]; bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    int c = tid + i * NT;
    a_lrow[i] = c / CPR; a_col[i] = (c % CPR) * VN;
    int64_t m = m0 + a_lrow[i];
    a_ok[i] = m < M;
    a_ptr[i] = A + (a_ok[i] ? rowmap(amap, m) : 0) * lda;
  }
  const TA* w_ptr[W_CH]; int w_lrow[W_CH], w_col[W_CH]; bool w_ok[W_CH];
#pragma unroll
  for (int i = 0; i < W_CH; ++i) {
    int c = tid + i * NT;
    w_lrow[i] = c / CPR; w_col[i] = (c % CPR) * VN;
    int64_t n = n0 + w_lrow[i];
    w_ok[i] = n < N;
    w_ptr[i] = W + (w_ok[i] ? n : 0) * ldw;
  }

  uint4 ra[A_CH], rw[W_CH];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int64_t k = k0 + a_col[i];
      ra[i] = (a_ok[i] && k < K) ? ld16(a_ptr[i] + k) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      int64_t k = k0 + w_col[i];
      rw[i] = (w_ok[i] && k < K) ? ld16(w_ptr[i] + k) : make_uint4(0, 0, 0, 0);
    }
  };
  // fp32: rows 8..15 of every 16-row group hold each 4-float chunk rotated by two (halves swapped),
  // so the 16 rows x 2 k of a ds_read_b32 lane group (bank = (36 row + k) mod 32) fall on 32
  // distinct banks instead of two rows per bank; the read index is k ^ 2 on those rows
  auto rot = [](uint4 u, int row) {
    if constexpr (sizeof(TA) == 4) return ((row >> 3) & 1) ? make_uint4(u.z, u.w, u.x, u.y) : u;
    else return u;
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) st16(&sA[buf][a_lrow[i] * LDR + a_col[i]], rot(ra[i], a_lrow[i]));
#pragma unroll
    for (int i = 0; i < W_CH; ++i) st16(&sW[buf][w_lrow[i] * LDR + w_col[i]], rot(rw[i], w_lrow[i]));
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ktiles = (int)((K + BKT - 1) / BKT);
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < ktiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ktiles) gload((int64_t)(kt + 1) * BKT);
    const TA* As = sA[buf];
    const TA* Ws = sW[buf];
    if constexpr (sizeof(TA) == 2) {
      const int r = lane & 15, kc = (lane >> 4) * 8;
      s16x8 bfrag[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j)
        bfrag[j] = *reinterpret_cast<const s16x8*>(&As[(wm + 16 * j + r) * LDR + kc]);
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        s16x8 afrag = *reinterpret_cast<const s16x8*>(&Ws[(wn + 16 * i + r) * LDR + kc]);
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(afrag, bfrag[j], acc[i][j]);
      }
    } else {
      const int r = lane & 15, kq = (lane >> 4) ^ (((lane >> 3) & 1) << 1);   // rot() above
#pragma unroll
      for (int s = 0; s < BKT / 4; ++s) {
        float bv[FM];
#pragma unroll
        for (int j = 0; j < FM; ++j) bv[j] = As[(wm + 16 * j + r) * LDR + 4 * s + kq];
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          float av = Ws[(wn + 16 * i + r) * LDR + 4 * s + kq];
#pragma unroll
          for (int j = 0; j < FM; ++j) acc[i][j] = mfma_f32(av, bv[j], acc[i][j]);
        }
      }
    }
    if (kt + 1 < ktiles) {
      sstore(buf ^ 1);
    }
    __syncthreads();
  }

  // epilogue
  const int col = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int64_t n = n0 + wn + 16 * i + rq;
    if (n >= N) continue;
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int64_t m = m0 + wm + 16 * j + col;
      if (m < M) epilogue4<TO>(e, m, n, acc[i][j]);
    }
  }
}

// ------------------------------------------------------------------------------------
// bf16 main GEMM: BK = 64, 16-byte chunks XOR-swizzled in LDS (chunk' = chunk ^ (row & 7))
// so the 16 rows a fragment read touches spread over the bank row; register-staged
// double buffer (next tile's global loads issued before the MFMAs of this one);
// 1-D grid remapped so consecutive tiles (same A row panel) land on one XCD's L2.
// ------------------------------------------------------------------------------------
constexpr int BK2 = 64;

template <typename TO, int BM, int BN>
__global__ __launch_bounds__(NT) void gemm2_kernel(const bf16* __restrict__ A, int64_t lda, RowMap amap,
                                                   const bf16* __restrict__ W, int64_t ldw, int64_t M, int64_t N,
                                                   int64_t K, int tiles_n, EpiArgs e) {
  constexpr int CPR = BK2 / 8;               // 8 chunks of 16 B per tile row
  constexpr int A_CH = BM * CPR / NT, W_CH = BN * CPR / NT;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  __shared__ __attribute__((aligned(16))) bf16 sA[2][BM * BK2];
  __shared__ __attribute__((aligned(16))) bf16 sW[2][BN * BK2];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
  const int wm = (wave & 1) * WM, wn = (wave >> 1) * WN;

  const bf16* a_ptr[A_CH]; int a_off[A_CH], a_col[A_CH]; bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int c = tid + i * NT, row = c / CPR, ch = c % CPR;
    a_col[i] = ch * 8;
    a_off[i] = (row * CPR + (ch ^ (row & 7))) * 8;
    const int64_t m = m0 + row;
    a_ok[i] = m < M;
    a_ptr[i] = A + (a_ok[i] ? rowmap(amap, m) : 0) * lda;
  }
  const bf16* w_ptr[W_CH]; int w_off[W_CH], w_col[W_CH]; bool w_ok[W_CH];
#pragma unroll
  for (int i = 0; i < W_CH; ++i) {
    const int c = tid + i * NT, row = c / CPR, ch = c % CPR;
    w_col[i] = ch * 8;
    w_off[i] = (row * CPR + (ch ^ (row & 7))) * 8;
    const int64_t n = n0 + row;
    w_ok[i] = n < N;
    w_ptr[i] = W + (w_ok[i] ? n : 0) * ldw;
  }
  uint4 ra[A_CH], rw[W_CH];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int64_t k = k0 + a_col[i];
      ra[i] = (a_ok[i] && k < K) ? ld16(a_ptr[i] + k) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int64_t k = k0 + w_col[i];
      rw[i] = (w_ok[i] && k < K) ? ld16(w_ptr[i] + k) : make_uint4(0, 0, 0, 0);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) st16(&sA[buf][a_off[i]], ra[i]);
#pragma unroll
    for (int i = 0; i < W_CH; ++i) st16(&sW[buf][w_off[i]], rw[i]);
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r = lane & 15, q = lane >> 4;
  const int ktiles = (int)((K + BK2 - 1) / BK2);
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < ktiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ktiles) gload((int64_t)(kt + 1) * BK2);
    const bf16* As = sA[buf];
    const bf16* Ws = sW[buf];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + q;
      s16x8 bfrag[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int row = wm + 16 * j + r;
        bfrag[j] = *reinterpret_cast<const s16x8*>(&As[(row * CPR + (ch ^ (row & 7))) * 8]);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int row = wn + 16 * i + r;
        const s16x8 afrag = *reinterpret_cast<const s16x8*>(&Ws[(row * CPR + (ch ^ (row & 7))) * 8]);
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(afrag, bfrag[j], acc[i][j]);
      }
    }
    if (kt + 1 < ktiles) sstore(buf ^ 1);
    __syncthreads();
  }
  const int col = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int64_t n = n0 + wn + 16 * i + rq;
    if (n >= N) continue;
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int64_t m = m0 + wm + 16 * j + col;
      if (m < M) epilogue4<TO>(e, m, n, acc[i][j]);
    }
  }
}

// ------------------------------------------------------------------------------------
// bf16 large GEMM (ViT QKV / out-proj / MLP): LDS-DMA staging (global_load_lds 16 B,
// no VGPR round trip) into an S-stage ring of BK-deep K-tiles, with a counted `vmcnt` so
// S-2 tiles stay in flight across the single raw barrier of each K-step.  The LDS image
// of a tile is lane-linear per wave-instruction (64 x 16 B); the XOR swizzle
// slot = chunk ^ ((row / RPB) % BKC) (RPB = rows per 256-byte bank row) is applied on the
// per-lane GLOBAL source address and again on the fragment reads (the same involution
// on both sides), which makes the 16 rows of a ds_read_b128 fragment read hit 16
// distinct 16-byte bank slots.  WGM x WGN waves, each owning a (BM/WGM) x (BN/WGN)
// sub-tile of D = W . A^T (4 consecutive output columns per lane).  Needs K % BK == 0 and
// N % BN == 0 (host-checked); rows >= M read row M-1 and are masked in the epilogue.
// ------------------------------------------------------------------------------------

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
DEV i32x8 cat8(i32x4 a, i32x4 b) { return i32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }
// 16x16x128 e4m3 x e4m3 MFMA, unit block scales (E8M0 127 = 2^0)
DEV f32x4 mfma_fp8x128(i32x8 a, i32x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

template <int BK>
struct Swz {
  static constexpr int BKC = BK / 8;            // 16-byte chunks per tile row
  static constexpr int RPB = 256 / (BK * 2);    // tile rows per 256-byte bank row
  static DEV int slot(int row, int ch) { return ch ^ ((row / RPB) % BKC); }
};

// F8: A and W hold OCP e4m3 bytes, addressed here in 2-byte units (K, lda, ldw, BK halved),
// so staging, swizzle and LDS-DMA are byte-identical to bf16.  One K=128 block-scaled MFMA
// (unit scales; fp8 rate = 2x bf16) consumes two 16-byte chunks per lane; A and W fragments
// read the same chunks, so the k order inside the instruction does not matter.  The
// epilogue multiplies by sa[m] * sw[n] (per-row dequant scales) before bias / act / residual.
// 1 (default) = the lean one-item-per-thread epilogue with the next round's residual in flight and the
// bias loaded once (same box, M = 4616: out-proj 20.8 -> 19.9 us, fc1 55.1 -> 52.7, fc2 48.3 -> 47.1;
// bit-identical); 0 = one residual round trip per epilogue round
int g_epi_prefetch = 1;
int g_gemm3_store = 0;  // gemm3 lean fp32 epilogue stores: 0 = plain, 1 = nt (A/B knob)
// gemm6 bf16 epilogue stores: 0 = plain, 1 = nt, 2 = sc1 write-through (default: the output leaves the
// XCD's L2 as it is written instead of as dirty lines at the kernel boundary; same box, whole step,
// tools/ab_knob.py: 9.309 / 9.286 / 9.234 ms)
int g_wide_store = 2;
int g_wide_epi = 1;   // gemm6 bf16 outputs: 1 = register-side epilogue (wide_epilogue_bf16), 0 = fp32 LDS staging
template <typename TO, int BM, int BN, int WGM, int WGN, int S, int BK, bool F8 = false, bool SC = false,
          int EPI = 0>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm3_kernel(const bf16* __restrict__ A, int64_t lda, RowMap amap,
                                                            const bf16* __restrict__ W, int64_t ldw, int64_t M,
                                                            int64_t K, int tiles_n, EpiArgs e, int group_m) {
  constexpr int NT3 = 64 * WGM * WGN;
  using SW = Swz<BK>;
  constexpr int BKC = SW::BKC;
  // A chunks may leave a partial last group (160 / 224-row tiles at 8 waves): every wave still
  // issues it (uniform counted vmcnt), the waves past AREM re-loading the chunks of wave
  // (wave mod AREM/64) into the same LDS slots -- identical bytes, a benign duplicate write
  constexpr int AG = (BM * BKC + NT3 - 1) / NT3, WG = BN * BKC / NT3, G = AG + WG;
  constexpr int AREM = BM * BKC - (AG - 1) * NT3;      // chunks of the last A group
  static_assert(WG * NT3 == BN * BKC, "tile / thread mismatch");
  static_assert(AREM % 64 == 0, "partial A group must be whole waves");
  constexpr int WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
  constexpr int STAGE = (BM + BN) * BK;           // elements per stage
  __shared__ __attribute__((aligned(16))) bf16 smem[S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  // tile order: row-major, or grouped (group_m m-tiles swept across all n-tiles) so that each
  // XCD's contiguous range of tiles covers a 2-D block: fewer A / W bytes per XCD L2
  int tm_i, tn_i;
  if (group_m > 0) {
    const int tiles_m = (int)((M + BM - 1) / BM);
    const int per = group_m * tiles_n, g = wg / per, r = wg - g * per;
    const int gs = min(group_m, tiles_m - g * group_m);
    tm_i = g * group_m + r % gs;
    tn_i = r / gs;
  } else {
    tm_i = wg / tiles_n;
    tn_i = wg % tiles_n;
  }
  const int64_t m0 = (int64_t)tm_i * BM, n0 = (int64_t)tn_i * BN;
  const int wm = (wave % WGM) * WM, wn = (wave / WGM) * WN;
  const bool ident = amap.d1 == 1 && amap.m1 >= M && amap.s1 == 1 && amap.m2 == 1 && amap.off == 0;

  // per-instruction source pointers: chunk c = g*NT3 + tid -> LDS row c/BKC, slot c%BKC,
  // which holds the global chunk slot(row, c%BKC)
  const bf16* asrc[AG];
#pragma unroll
  for (int g = 0; g < AG; ++g) {
    const int c = g * NT3 + (g == AG - 1 ? tid % AREM : tid), row = c / BKC, ch = SW::slot(row, c % BKC);
    int64_t m = m0 + row;
    if (m >= M) m = M - 1;
    asrc[g] = A + (ident ? m : rowmap(amap, m)) * lda + ch * 8;
  }
  const bf16* wsrc[WG];
#pragma unroll
  for (int g = 0; g < WG; ++g) {
    const int c = g * NT3 + tid, row = c / BKC, ch = SW::slot(row, c % BKC);
    wsrc[g] = W + (n0 + row) * ldw + ch * 8;
  }
  auto issue = [&](int kt) {
    bf16* sa = smem + (kt % S) * STAGE;
    bf16* sw = sa + BM * BK;
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int g = 0; g < AG; ++g) {
      const int wv = g == AG - 1 ? wave % (AREM / 64) : wave;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(asrc[g] + k0), (lds_void_t*)(sa + (g * NT3 + wv * 64) * 8), 16, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < WG; ++g)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(wsrc[g] + k0), (lds_void_t*)(sw + (g * NT3 + wave * 64) * 8), 16, 0, 0);
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r = lane & 15, q = lane >> 4;
  const int ktiles = (int)(K / BK);
#pragma unroll
  for (int t = 0; t < S - 1; ++t)
    if (t < ktiles) issue(t);
  for (int kt = 0; kt < ktiles; ++kt) {
    // tiles kt .. min(kt+S-2, ktiles-1) are in flight; retire tile kt
    if (kt + S - 2 < ktiles) wait_vmcnt<(S - 2) * G>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();                 // tile kt visible; stage (kt-1)%S free
    __builtin_amdgcn_sched_barrier(0);
    if (kt + S - 1 < ktiles) issue(kt + S - 1);
    const bf16* As = smem + (kt % S) * STAGE;
    const bf16* Ws = As + BM * BK;
    if constexpr (F8) {
      static_assert(BK % 64 == 0, "fp8 K-step is 128 bytes");
#pragma unroll
      for (int ks = 0; ks < BK / 64; ++ks) {
        const int ch = ks * 8 + 2 * q;
        i32x8 bfrag[FM], afrag[FN];
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int row = wm + 16 * j + r;
          bfrag[j] = cat8(*reinterpret_cast<const i32x4*>(&As[(row * BKC + SW::slot(row, ch)) * 8]),
                          *reinterpret_cast<const i32x4*>(&As[(row * BKC + SW::slot(row, ch + 1)) * 8]));
        }
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int row = wn + 16 * i + r;
          afrag[i] = cat8(*reinterpret_cast<const i32x4*>(&Ws[(row * BKC + SW::slot(row, ch)) * 8]),
                          *reinterpret_cast<const i32x4*>(&Ws[(row * BKC + SW::slot(row, ch + 1)) * 8]));
        }
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc[i][j] = mfma_fp8x128(afrag[i], bfrag[j], acc[i][j]);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        const int ch = ks * 4 + q;
        s16x8 bfrag[FM], afrag[FN];
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int row = wm + 16 * j + r;
          bfrag[j] = *reinterpret_cast<const s16x8*>(&As[(row * BKC + SW::slot(row, ch)) * 8]);
        }
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int row = wn + 16 * i + r;
          afrag[i] = *reinterpret_cast<const s16x8*>(&Ws[(row * BKC + SW::slot(row, ch)) * 8]);
        }
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(afrag[i], bfrag[j], acc[i][j]);
      }
    }
  }
  // ---- epilogue through LDS: rounds of 64 tile rows (JR m-fragments per wave row) are
  // staged as fp32, then every thread walks whole output rows (coalesced stores); the
  // accumulator indices stay compile-time constants (no scratch) ----
  // JR = the largest divisor of FM that keeps a round <= 64 rows (FM = 5 for 160-row tiles)
  constexpr int JR0 = 4 / WGM, JR = FM % JR0 == 0 ? JR0 : (JR0 >= 2 && FM % 2 == 0 ? 2 : 1);
  constexpr int ROWS = WGM * JR * 16, SLD = BN + 4;
  static_assert(JR >= 1 && FM % JR == 0, "epilogue rounds");
  static_assert(ROWS * SLD * 4 <= S * STAGE * 2, "epilogue stage exceeds LDS");
  float* stg = reinterpret_cast<float*>(smem);
  const int col = lane & 15, rq = (lane >> 4) * 4;
  const int wmi = wave % WGM;
  // lean epilogues with one or two output items per thread per round (160 x 128, 96 x 128, 224 x 256): the
  // bias of the thread's 8 columns is loaded once, and the residual rows of round h + 1 are
  // requested before round h's barrier, so no round waits for its own global loads (the loop
  // below issues them inside each round: one HBM round trip per round, ~5 rounds per tile)
  // IPT = output items per thread per round; every item of a thread has the same 8 columns
  constexpr int IPT = ROWS * (BN / 8) / NT3;
  constexpr bool ONE = IPT >= 1 && IPT <= 2 && ROWS * (BN / 8) == IPT * NT3 && NT3 % (BN / 8) == 0 && EPI != 0 &&
                       !SC;
  if constexpr (ONE) {
    if (e.pf & 1) {
      const int c8 = (tid % (BN / 8)) * 8;
      const int64_t n = n0 + c8;
      float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (e.bias) load8f(e.bias + n, b);
      auto lrow_of = [&](int k) { return (tid + k * NT3) / (BN / 8); };
      auto mrow = [&](int h, int k) {
        const int lrow = lrow_of(k);
        const int wi = lrow / (JR * 16), jj = (lrow / 16) % JR, rr = lrow % 16;
        return m0 + wi * WM + (h * JR + jj) * 16 + rr;
      };
      const bool res = EPI == 1 && e.res;
      float rc[IPT][8], rn[IPT][8];
      // F8: the per-column dequant scales once, the per-row scale of each item with its residual
      float wsc[8];
      float sc[IPT], sn[IPT];
      if constexpr (F8) load8f(e.sw + n, wsc);
      auto ldres = [&](int h, float (&r)[IPT][8], float (&sr)[IPT]) {
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
          const int64_t m = std::min<int64_t>(mrow(h, k), M - 1);
          if (res) load8f(reinterpret_cast<const TO*>(e.res) + m * e.ld_res + n, r[k]);
          if constexpr (F8) sr[k] = e.sa[ident ? m : rowmap(amap, m)];
        }
      };
      ldres(0, rc, sc);
#pragma unroll
      for (int h = 0; h < FM / JR; ++h) {
        if (h + 1 < FM / JR) ldres(h + 1, rn, sn);
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int j2 = 0; j2 < JR; ++j2)
#pragma unroll
          for (int i = 0; i < FN; ++i)
            *reinterpret_cast<f32x4*>(&stg[((wmi * JR + j2) * 16 + col) * SLD + wn + 16 * i + rq]) = acc[i][h * JR + j2];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
          const int lrow = lrow_of(k);
          const int64_t m = mrow(h, k);
          if (m < M) {
            const f32x4 lo = *reinterpret_cast<const f32x4*>(&stg[lrow * SLD + c8]);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(&stg[lrow * SLD + c8 + 4]);
            float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            if constexpr (F8) {
#pragma unroll
              for (int r = 0; r < 8; ++r) v[r] = v[r] * (wsc[r] * sc[k]);
            }
            if (e.bias) {
#pragma unroll
              for (int r = 0; r < 8; ++r) v[r] += b[r];
            }
            if constexpr (EPI == 2) {
#pragma unroll
              for (int r = 0; r < 8; ++r) v[r] = apply_act(v[r], ACT_QUICKGELU);
            }
            if (res) {
#pragma unroll
              for (int r = 0; r < 8; ++r) v[r] += rc[k][r];
            }
            if constexpr (sizeof(TO) == 4) {
              if (e.pf & 16) {          // A/B knob gemm3_store 1: nt stores of the fp32 rows
                float* p = reinterpret_cast<float*>(e.out) + m * e.ldo + n;
                __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(p));
                __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, reinterpret_cast<f32x4*>(p + 4));
                continue;
              }
              if (e.pf & 32) {          // gemm3_store 2: sc1 write-through
                const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(e.out, (short)0, 0x7fffffff, 0x00020000);
                const int off = (int)((m * e.ldo + n) * 4);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, f32x4{v[0], v[1], v[2], v[3]}), r, off, 0, 16);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, f32x4{v[4], v[5], v[6], v[7]}), r, off + 16, 0, 16);
                continue;
              }
            }
            store8f(reinterpret_cast<TO*>(e.out) + m * e.ldo + n, v);
          }
        }
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
#pragma unroll
          for (int r = 0; r < 8; ++r) rc[k][r] = rn[k][r];
          sc[k] = sn[k];
        }
      }
      return;
    }
  }
#pragma unroll
  for (int h = 0; h < FM / JR; ++h) {
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int jj = 0; jj < JR; ++jj)
#pragma unroll
      for (int i = 0; i < FN; ++i)
        *reinterpret_cast<f32x4*>(&stg[((wmi * JR + jj) * 16 + col) * SLD + wn + 16 * i + rq]) = acc[i][h * JR + jj];
    __syncthreads();
    for (int idx = tid; idx < ROWS * (BN / 8); idx += NT3) {
      const int lrow = idx / (BN / 8), c8 = (idx % (BN / 8)) * 8;
      const int wi = lrow / (JR * 16), jj = (lrow / 16) % JR, rr = lrow % 16;
      const int64_t m = m0 + wi * WM + (h * JR + jj) * 16 + rr;
      if (m < M) {
        f32x4 lo = *reinterpret_cast<const f32x4*>(&stg[lrow * SLD + c8]);
        f32x4 hi = *reinterpret_cast<const f32x4*>(&stg[lrow * SLD + c8 + 4]);
        if constexpr (F8) {
          const float s = e.sa[ident ? m : rowmap(amap, m)];   // scale of the A row read for m
          const f32x4 w0 = *reinterpret_cast<const f32x4*>(e.sw + n0 + c8);
          const f32x4 w1 = *reinterpret_cast<const f32x4*>(e.sw + n0 + c8 + 4);
          lo = lo * (w0 * s);
          hi = hi * (w1 * s);
        }
        epilogue8<TO, SC, EPI>(e, m, n0 + c8, lo, hi);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Wide tiles for the ViT GEMMs (gemm6): BM = 320 rows x BN = 256 / 192 columns, one 8-wave
// workgroup per CU.  At M = 4616 the 320-row tiles make ONE round on 240 CUs for fc1 (15 x 16 at
// BN 256) and QKV (15 x 16 at BN 192), with half of gemm3's L2 -> LDS bytes per FLOP (142 FLOP per
// byte at 320 x 256 vs 71 at 160 x 128): 8 waves as 2 (m) x 4 (n), a 160 x 64 (48) wave tile = 14
// (13) fragment reads per 40 (30) MFMAs per k32, 160 (120) accumulator VGPRs.  Arithmetic per
// output = gemm3's (the same MFMA over the same k order, the same epilogue expression), so the tile
// choice never changes a bit (batch invariance).  Round-6 forms measured and removed (DESIGN.md
// §11): BK = 32 stages (16 rows x 64 B per DMA instruction), in step or ping-pong; a register-
// prefetched 160 x 128 tile for the narrow-N GEMMs.
// ------------------------------------------------------------------------------------
// 16-byte LDS-DMA through a buffer resource (buffer_load_dwordx4 ... lds): base and size are wave-
// uniform, the lane's part is a 32-bit byte offset, `soff` a uniform byte offset (SGPR)
DEV void dma_buf16(const void* base, int bytes, void* lds, int voff, int soff) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, voff, soff, 0, 0);
}

DEV int swz4(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }   // g = {0, 2, 3, 1} as 2-bit fields

// Tile origin for the wide kernels: after the XCD remap, groups of `group_m` m-tiles sweep the
// n-tiles, so an XCD's contiguous range of workgroups covers a compact block of A and W panels.
DEV void wide_tile(int wg, int64_t M, int BM, int tiles_n, int group_m, int& tm_i, int& tn_i) {
  const int tiles_m = (int)((M + BM - 1) / BM);
  const int per = group_m * tiles_n, g = wg / per, r = wg - g * per;
  const int gs = min(group_m, tiles_m - g * group_m);
  tm_i = g * group_m + r % gs;
  tn_i = r / gs;
}

// LDS-staged epilogue shared by gemm4 / gemm5: rounds of 64 tile rows (2 m-fragments per wave
// row) staged as fp32, each thread then stores 8 consecutive columns of whole rows; the bias of a
// thread's items is loaded once, a round's residual rows are all requested before the round's
// first barrier.
template <typename TO, int BM, int BN, int EPI, int FM, int FN>
DEV void wide_epilogue(const EpiArgs& e, f32x4 (&acc)[FN][FM], bf16* smem, int64_t M, int64_t m0, int64_t n0) {
  constexpr int NT4 = 512, WGM = 2, WM = BM / WGM, WN = BN / 4;
  constexpr int JR = FM % 2 == 0 ? 2 : 1, ROWS = WGM * JR * 16, SLD = BN + 4;
  static_assert(FM % JR == 0, "epilogue rounds");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wmi = wave / 4, wn = (wave % 4) * WN;
  float* stg = reinterpret_cast<float*>(smem);
  const int col = lane & 15, rq = (lane >> 4) * 4;
  constexpr int CG = BN / 8, ITEMS = ROWS * CG, IPT = (ITEMS + NT4 - 1) / NT4;
  static_assert(ITEMS % 64 == 0, "whole waves per epilogue item slot");
  // when 512 is a multiple of the column groups every item of a thread has the same 8 columns
  constexpr bool SAMEC = NT4 % CG == 0;
  constexpr int NB = SAMEC ? 1 : IPT;
  int lr[IPT], c8[IPT];
  float bias[NB][8];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int idx = min(tid + k * NT4, ITEMS - 1);
    lr[k] = idx / CG;
    c8[k] = (idx % CG) * 8;
  }
#pragma unroll
  for (int k = 0; k < NB; ++k) {
#pragma unroll
    for (int r = 0; r < 8; ++r) bias[k][r] = 0.f;
    if (e.bias) load8f(e.bias + n0 + c8[k], bias[k]);
  }
  const bool res = EPI == 1 && e.res;
#pragma unroll
  for (int h = 0; h < FM / JR; ++h) {
    int64_t mk[IPT];
    float rv[IPT][8];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int lrow = lr[k], wi = lrow / (JR * 16), jj = (lrow / 16) % JR, rr = lrow % 16;
      mk[k] = m0 + wi * WM + (h * JR + jj) * 16 + rr;
      if (res) load8f(reinterpret_cast<const TO*>(e.res) + min<int64_t>(mk[k], M - 1) * e.ld_res + n0 + c8[k], rv[k]);
    }
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < JR; ++jj)
#pragma unroll
      for (int i = 0; i < FN; ++i)
        *reinterpret_cast<f32x4*>(&stg[((wmi * JR + jj) * 16 + col) * SLD + wn + 16 * i + rq]) = acc[i][h * JR + jj];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      if (tid + k * NT4 < ITEMS && mk[k] < M) {
        const f32x4 lo = *reinterpret_cast<const f32x4*>(&stg[lr[k] * SLD + c8[k]]);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(&stg[lr[k] * SLD + c8[k] + 4]);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] += bias[SAMEC ? 0 : k][r];
        if constexpr (EPI == 2) {
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = apply_act(v[r], ACT_QUICKGELU);
        }
        if (res) {
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] += rv[k][r];
        }
        store8f(reinterpret_cast<TO*>(e.out) + mk[k] * e.ldo + n0 + c8[k], v);
      }
    }
  }
}

// Register-side epilogue of the wide kernels for bf16 outputs without a residual (QKV: bias; fc1:
// bias + QuickGELU).  The bias (4 columns per n-fragment, fixed per lane) and the activation are
// applied on the accumulators in registers; the bf16 values go through LDS in TWO rounds of half the
// tile's rows (both wave rows' m-fragments 0..FM/2-1, then the rest), 8-byte writes into rows of
// BN + 8 elements (a row stride = 16 B mod 256: the 16 rows of a write group hit 16 distinct 16-B
// slots), and leave as whole-row 16-byte stores.  Against wide_epilogue: 4 instead of 10 barriers and
// half the LDS bytes (bf16 instead of fp32 staging); the arithmetic of an output is the same
// expression (acc + bias, then the activation, then one rounding).
template <int BM, int BN, int EPI, int FM, int FN>
DEV void wide_epilogue_bf16(const EpiArgs& e, f32x4 (&acc)[FN][FM], bf16* smem, int64_t M, int64_t m0, int64_t n0) {
  constexpr int NT4 = 512, WM = BM / 2, WN = BN / 4, SR = BN + 8;
  constexpr int FH = FM / 2, ROWS = 2 * FH * 16;                 // rows staged per round
  static_assert(FM % 2 == 0, "two rounds");
  static_assert(ROWS * SR * 2 <= 160 * 1024, "staging exceeds LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wmi = wave / 4, wn = (wave % 4) * WN;
  const int col = lane & 15, q = lane >> 4;
  float bias[FN][4];
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    if (e.bias) {
      const float4 b = *reinterpret_cast<const float4*>(e.bias + n0 + wn + 16 * i + 4 * q);
      bias[i][0] = b.x; bias[i][1] = b.y; bias[i][2] = b.z; bias[i][3] = b.w;
    } else {
      bias[i][0] = bias[i][1] = bias[i][2] = bias[i][3] = 0.f;
    }
  }
  constexpr int CG = BN / 8, ITEMS = ROWS * CG, IPT = (ITEMS + NT4 - 1) / NT4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < FH; ++jj)
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const f32x4 a = acc[i][h * FH + jj];
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = a[r] + bias[i][r];
          if constexpr (EPI == 2) v[r] = apply_act(v[r], ACT_QUICKGELU);
        }
        const int lrow = (wmi * FH + jj) * 16 + col;
        *reinterpret_cast<uint2*>(&smem[lrow * SR + wn + 16 * i + 4 * q]) = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
      }
    __syncthreads();
    uint4 val[IPT];
    int64_t mr[IPT];
    int cc[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int idx = min(tid + k * NT4, ITEMS - 1);
      const int lrow = idx / CG, c8 = (idx % CG) * 8;
      const int wi = lrow / (FH * 16), rr = lrow % (FH * 16);
      mr[k] = m0 + wi * WM + h * FH * 16 + rr;
      cc[k] = c8;
      val[k] = *reinterpret_cast<const uint4*>(&smem[lrow * SR + c8]);
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k)
      if (tid + k * NT4 < ITEMS && mr[k] < M) {
        bf16* p = reinterpret_cast<bf16*>(e.out) + mr[k] * e.ldo + n0 + cc[k];
        if (e.pf & 4) __builtin_nontemporal_store(__builtin_bit_cast(i32x4, val[k]), reinterpret_cast<i32x4*>(p));
        else if (e.pf & 8) {
          const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(e.out, (short)0, 0x7fffffff, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, val[k]), r,
                                                 (int)((mr[k] * e.ldo + n0 + cc[k]) * 2), 0, 16);   // sc1 write-through
        } else st16(p, val[k]);
      }
  }
}

// gemm6: the wide tile as a PING-PONG loop (cdna_hip_programming.md §5, the staggered 8-wave
// template) with FULL-LINE staging.  Waves w and w + 4 share a SIMD; the waves of the second m-half
// (group 1 = waves 4-7) run one barrier behind group 0, so between any two barriers one group issues
// its fragment reads, LDS-DMA and counted waits (LOAD) while the other issues MFMAs (COMPUTE): each
// SIMD's matrix pipe is fed by one wave while its partner loads.  The stages are BK = 64 (each DMA
// wave-instruction moves 8 rows x 128 B, whole lines; the BK = 32 form's 16 rows x 64 B measured
// 724 vs 683 us of fill alone at 8192^3) in S = 2 slots (2 x (BM + BN) x 128 B of LDS), each K64
// tile run as two k32 phases so the per-wave fragment registers stay those of one k32 step.  The
// DMA is buffer_load ... lds (one 32-bit lane offset, the K offset in soffset: no per-issue VALU).
// Schedule (interval = the span between two barriers; group 1 one interval behind group 0):
//   group 0: L(t,0) @4t, C(t,0) @4t+1, L(t,1) @4t+2, C(t,1) @4t+3;  group 1: each one later.
//   L(t,0) issues the wave's share of tile t + 1's DMA (slot (t + 1) % 2 = (t - 1) % 2, whose last
//   reads -- group 1's L(t - 1, 1) @4t-1 -- retired before the barrier that opened @4t);
//   tile t + 1 is read from @4t+4 (group 0) / @4t+5 (group 1), so every wave waits its own DMA of
//   t + 1 before the barrier closing @4t+3: group 0 at the end of C(t,1), group 1 at the end of L(t,1).
// Swizzle: the 16-byte chunk c of row r sits at slot c ^ ((r / 2) % 8) (Swz<64>, as gemm3).
template <typename TO, int BM, int BN, int EPI, int ABL = 0>
__global__ __launch_bounds__(512) void gemm6_kernel(const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ W,
                                                    int64_t ldw, int64_t M, int64_t K, int tiles_n, EpiArgs e,
                                                    int group_m) {
  constexpr int BK = 64, BKC = 8, WM = BM / 2, WN = BN / 4, FM = WM / 16, FN = WN / 16;
  constexpr int STAGE = (BM + BN) * BK, NI = (BM + BN) / 8, JMAX = (NI + 7) / 8;
  static_assert(BM % 16 == 0 && BN % 16 == 0, "rows per fragment");
  using SW = Swz<64>;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wave) >> 2;
  int tm_i, tn_i;
  wide_tile(xcd_remap(blockIdx.x, gridDim.x), M, BM, tiles_n, group_m, tm_i, tn_i);
  const int64_t m0 = (int64_t)tm_i * BM, n0 = (int64_t)tn_i * BN;
  const int wm = grp * WM, wn = (wave % 4) * WN;

  // DMA plan: instruction i = wave + 8 j covers stage rows 8 i .. 8 i + 7 (A rows, then W rows);
  // lane -> row 8 i + lane / 8, physical slot lane % 8 = logical chunk SW::slot(row, lane % 8).
  // Buffer loads (buffer_load_dwordx4 ... lds): whether instruction j reads A or W is wave-uniform,
  // the lane's part is one 32-bit byte offset, the K offset goes in soffset (no per-issue VALU).
  const int64_t abytes = M * lda * 2, wbytes = (int64_t)tiles_n * BN * ldw * 2;
  const int anr = abytes < 0x7fffffff ? (int)abytes : 0x7fffffff, wnr = wbytes < 0x7fffffff ? (int)wbytes : 0x7fffffff;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const bool full = (wave + 8 * (JMAX - 1)) < NI;
  int voff[JMAX];
#pragma unroll
  for (int j = 0; j < JMAX; ++j) {
    const int i = min(wave + 8 * j, NI - 1);
    const int row = 8 * i + (lane >> 3), ch = SW::slot(row, lane & 7);
    if (row < BM) {
      const int64_t m = min<int64_t>(m0 + row, M - 1);
      voff[j] = (int)((m * lda + ch * 8) * 2);
    } else {
      voff[j] = (int)(((n0 + row - BM) * ldw + ch * 8) * 2);
    }
  }
  auto issue = [&](int kt) {
    bf16* st = smem + (kt & 1) * STAGE;
    const int kb = kt * BK * 2;
#pragma unroll
    for (int j = 0; j < JMAX; ++j) {
      if (j < JMAX - 1 || full) {
        if ((wv + 8 * j) * 8 < BM) dma_buf16(A, anr, st + (wv + 8 * j) * 512, voff[j], kb);   // wave-uniform choice
        else dma_buf16(W, wnr, st + (wv + 8 * j) * 512, voff[j], kb);
      }
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, q = lane >> 4;
  // fragment address of row base rb (a multiple of 16), k32 half h: rows rb + r16, chunk 4 h + q,
  // whose slot (4 h + q) ^ ((r16 / 2) % 8) depends on the lane only
  const int fo0 = r16 * BK + ((q ^ ((r16 >> 1) & 7)) * 8), fo1 = r16 * BK + (((4 + q) ^ ((r16 >> 1) & 7)) * 8);
  auto fptr = [&](const bf16* base, int rb, int h) {
    return reinterpret_cast<const s16x8*>(&base[rb * BK + (h ? fo1 : fo0)]);
  };
  const int ktiles = (int)(K / BK);
  issue(0);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();                        // tile 0 visible
  if (grp == 1) __builtin_amdgcn_s_barrier();          // the stagger
  __builtin_amdgcn_sched_barrier(0);
  for (int kt = 0; kt < ktiles; ++kt) {
    const bf16* As = smem + (kt & 1) * STAGE;
    const bf16* Ws = As + BM * BK;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // ---- LOAD(kt, h) ----
      s16x8 bfrag[FM], afrag[FN];
#pragma unroll
      for (int i = 0; i < FN; ++i) afrag[i] = *fptr(Ws, wn + 16 * i, h);
#pragma unroll
      for (int j = 0; j < FM; ++j) bfrag[j] = *fptr(As, wm + 16 * j, h);
      if (ABL != 1 && h == 0 && kt + 1 < ktiles) issue(kt + 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (ABL != 1 && h == 1 && grp == 1) wait_vmcnt<0>();     // group 1: own DMA of kt + 1 landed
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- COMPUTE(kt, h) ----
      __builtin_amdgcn_s_setprio(1);
      if constexpr (ABL == 2) {
#pragma unroll
        for (int j = 0; j < FM; ++j) asm volatile("" :: "v"(bfrag[j]));
#pragma unroll
        for (int i = 0; i < FN; ++i) asm volatile("" :: "v"(afrag[i]));
      } else {
#pragma unroll
        for (int j = 0; j < FM; ++j)
#pragma unroll
          for (int i = 0; i < FN; ++i) acc[i][j] = mfma_bf16(afrag[i], bfrag[j], acc[i][j]);
      }
      __builtin_amdgcn_s_setprio(0);
      if (ABL != 1 && h == 1 && grp == 0) wait_vmcnt<0>();     // group 0: own DMA of kt + 1 landed
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();          // re-align the groups' barrier counts
  if constexpr (ABL == 3) {   // ablation: no epilogue (the accumulators kept live)
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  if constexpr (sizeof(TO) == 2 && FM % 2 == 0) {
    if ((e.pf & 2) && !(EPI == 1 && e.res)) {
      wide_epilogue_bf16<BM, BN, EPI, FM, FN>(e, acc, smem, M, m0, n0);
      return;
    }
  }
  wide_epilogue<TO, BM, BN, EPI, FM, FN>(e, acc, smem, M, m0, n0);
}

int g_gemm_group = 4;   // gemm3 tile order: 0 = row-major, G > 0 = G m-tiles per group (catseg_set_gemm_group); 4 measured best (fc2 48.6 -> 47.4 us)

EpiArgs make_epi(const CatsegGemmArgs* g) {
  EpiArgs e;
  e.bias = g->bias;
  e.add = g->add; e.ld_add = g->ld_add; e.add_ncols = g->add_ncols;
  e.addmap = RowMap{g->addmap.d1, g->addmap.m1, g->addmap.s1, g->addmap.d2, g->addmap.m2, g->addmap.s2, g->addmap.off};
  e.act = g->act; e.alpha = g->alpha;
  e.res = g->res; e.ld_res = g->ld_res; e.res2 = g->res2; e.ld_res2 = g->ld_res2;
  e.out = g->out; e.ldo = g->ldo;
  e.store_mode = g->store_mode; e.cvt_k = g->cvt_k; e.cvt_hin = g->cvt_hin; e.cvt_win = g->cvt_win;
  e.cvt_cout = g->cvt_cout;
  e.sa = nullptr; e.sw = nullptr;
  e.pf = g_epi_prefetch | (g_wide_epi ? 2 : 0) | (g_wide_store == 1 ? 4 : g_wide_store == 2 ? 8 : 0) |
         (g_gemm3_store == 1 ? 16 : g_gemm3_store == 2 ? 32 : 0);
  return e;
}

int g_gemm4_group = 5;   // gemm6 tile order: G m-tiles per group (catseg_set_gemm4_group)

// the wide ping-pong tiles (gemm6); ABL > 0: timing ablations (tools/micro_gemm.py 56-60, wrong outputs)
template <typename TO, int BM, int BN, int EPI, int ABL = 0>
bool launch6(const CatsegGemmArgs* g, hipStream_t st) {
  if (g->N % BN != 0 || g->K % 64 != 0) return false;
  const bool ident = g->amap.d1 == 1 && g->amap.m1 >= g->M && g->amap.s1 == 1 && g->amap.m2 == 1 && g->amap.off == 0;
  if (!ident) return false;
  const EpiArgs e = make_epi(g);
  const int tm = (int)((g->M + BM - 1) / BM), tn = (int)(g->N / BN);
  auto kern = gemm6_kernel<TO, BM, BN, EPI, ABL>;
  hipLaunchKernelGGL(kern, dim3((unsigned)(tm * tn)), dim3(512), 0, st, (const bf16*)g->A, g->lda, (const bf16*)g->W,
                     g->ldw, g->M, g->K, tn, e, std::max(1, g_gemm4_group));
  return true;
}

template <typename TO, int BM, int BN, int WGM, int WGN, int S, int BK, bool SC = false, int EPI = 0>
bool launch3(const CatsegGemmArgs* g, hipStream_t st) {
  if (g->N % BN != 0 || g->K % BK != 0) return false;
  const EpiArgs e = make_epi(g);
  RowMap am{g->amap.d1, g->amap.m1, g->amap.s1, g->amap.d2, g->amap.m2, g->amap.s2, g->amap.off};
  const int tm = (int)((g->M + BM - 1) / BM), tn = (int)(g->N / BN);
  hipLaunchKernelGGL((gemm3_kernel<TO, BM, BN, WGM, WGN, S, BK, false, SC, EPI>), dim3((unsigned)(tm * tn)), dim3(64 * WGM * WGN), 0,
                     st, (const bf16*)g->A, g->lda, am, (const bf16*)g->W, g->ldw, g->M, g->K, tn, e, g_gemm_group);
  return true;
}

// fp8: g's K / lda / ldw are in fp8 elements (bytes); the kernel sees 2-byte units
template <typename TO, int BM, int BN, int WGM, int WGN, int S, int BK, int EPI = 0>
bool launch3f8(const CatsegGemmArgs* g, const float* sa, const float* sw, hipStream_t st) {
  if (g->N % BN != 0 || (g->K / 2) % BK != 0) return false;
  EpiArgs e = make_epi(g);
  e.sa = sa; e.sw = sw;
  RowMap am{g->amap.d1, g->amap.m1, g->amap.s1, g->amap.d2, g->amap.m2, g->amap.s2, g->amap.off};
  const int tm = (int)((g->M + BM - 1) / BM), tn = (int)(g->N / BN);
  hipLaunchKernelGGL((gemm3_kernel<TO, BM, BN, WGM, WGN, S, BK, true, false, EPI>), dim3((unsigned)(tm * tn)), dim3(64 * WGM * WGN),
                     0, st, (const bf16*)g->A, g->lda / 2, am, (const bf16*)g->W, g->ldw / 2, g->M, g->K / 2, tn, e,
                     g_gemm_group);
  return true;
}

int g_gemm_wide = 1;      // 1 = the automatic choice includes the wide ping-pong tiles (gemm6); 0 = round-5 candidates
int g_gemm_variant = 0;   // 0 = automatic; >0 forces one of the automatic gemm3 tiles (tests / tuning)

// returns true when a gemm3 variant was launched
template <typename TO>
bool try_gemm3(const CatsegGemmArgs* g, hipStream_t st) {
  if (g->K % 32 != 0 || g->lda % 8 != 0 || g->ldw % 8 != 0) return false;
  // 8-wide epilogue: 16-byte aligned output / residual / add rows
  const int vo = sizeof(TO) == 2 ? 8 : 4;
  if (g->ldo % 8 != 0 || ((uintptr_t)g->out % 16) != 0) return false;
  if (g->res && (g->ld_res % 8 != 0 || ((uintptr_t)g->res % 16) != 0)) return false;
  if (g->res2 && (g->ld_res2 % 8 != 0 || ((uintptr_t)g->res2 % 16) != 0)) return false;
  if (g->add && (g->add_ncols % 8 != 0 || g->ld_add % vo != 0 || ((uintptr_t)g->add % 16) != 0)) return false;
  int v = g_gemm_variant;
  if (v < 0) return false;
  if (v == 0) {
    if (g->M < 1024 || g->K < 256) return false;
    // Tile choice by wave quantization over the 256 CUs (tools/micro_gemm.py, MG_M for other M):
    // score = fill x w / (1 + 0.15 (rounds - 1)), fill = tiles / (rounds x slots), slots = 256
    // or 512 (two workgroups per CU), w = the tile's measured per-CU efficiency.  Picks, e.g.:
    //  M = 4616 (bs 8): QKV 224x256 (35.1 us; hipBLASLt 32.3), fc1 160x128 two per CU (54.2 vs
    //    71.3 for 256x256), out-proj / fc2 160x128 BK=128 (19.8 / 47.9 us);
    //  M = 2308 (bs 4, config 4): QKV 128x128 8-wave two per CU (22.9 vs 24.2 us), fc1 160x128
    //    two per CU (31.4 vs 47.6 for 256x256), out-proj / fc2 96x128 BK=128 (13.9 / 35.2 vs
    //    18.8 / 50.9 us).
    // (Earlier measurements: deeper rings S = 3 / 4 slower on fc2; a one-round 320x256 fc1 tile
    // 58.4 us vs 54.5; 288x256 102 us.)  The tile never changes the arithmetic: every variant
    // accumulates the full K of an output in the same k order.
    // The ping-pong wide tiles (gemm6, v 50 / 51) need an identity A map and 32-bit buffer offsets.
    // (round 6, tools/micro_gemm.py, one box: fc1 41.2 us vs 47.3 for 160x128 two per CU, QKV 31.4
    // vs 33.3 for 224x256; weights from those ratios)
    struct Cand { int v, bm, bn, slots, bk; float w; };
    static const Cand cands[] = {{20, 224, 256, 1, 64, 1.0f}, {1, 256, 256, 1, 64, 0.95f}, {15, 160, 128, 1, 128, 0.95f},
                                 {17, 160, 128, 2, 64, 0.9f}, {19, 128, 128, 2, 64, 0.85f}, {24, 96, 128, 1, 128, 0.85f},
                                 {50, 320, 256, 1, 64, 1.1f}, {51, 320, 192, 1, 64, 1.1f}};
    const bool ident = g->amap.d1 == 1 && g->amap.m1 >= g->M && g->amap.s1 == 1 && g->amap.m2 == 1 && g->amap.off == 0;
    const bool lean = !g->add && !g->res2 && g->alpha == 1.f &&
                      (g->act == ACT_NONE || (g->act == ACT_QUICKGELU && !g->res)) && g->store_mode == 0;
    const bool wide_ok = g_gemm_wide && ident && lean && g->M * g->lda * 2 < 0x7fffffffLL && g->N * g->ldw * 2 < 0x7fffffffLL;
    float best = 0.f;
    for (const Cand& c : cands) {
      if (g->N % c.bn != 0 || g->K % c.bk != 0) continue;
      if (c.v >= 50 && !wide_ok) continue;
      const int64_t tiles = ((g->M + c.bm - 1) / c.bm) * (g->N / c.bn), slots = 256LL * c.slots;
      const int64_t rounds = (tiles + slots - 1) / slots;
      const float score = (float)tiles / (float)(rounds * slots) * c.w / (1.f + 0.15f * (float)(rounds - 1));
      if (score > best) { best = score; v = c.v; }
    }
    if (v == 0) return false;
  }
  if (g->store_mode != 0) {   // ConvTranspose scatter epilogue: instantiated for the 160x128 tiles only
    int sv = v;
    if (g_gemm_variant == 0 && sv != 15 && sv != 17) sv = g->K % 128 == 0 ? 15 : 17;
    if (sv == 15) return launch3<TO, 160, 128, 2, 4, 2, 128, true>(g, st);
    if (sv == 17) return launch3<TO, 160, 128, 2, 4, 2, 64, true>(g, st);
    return false;
  }
  // lean epilogues for the automatic ViT tiles
  const bool plain = !g->add && !g->res2 && g->alpha == 1.f;
  const int epi = plain && g->act == ACT_NONE ? 1 : plain && g->act == ACT_QUICKGELU && !g->res ? 2 : 0;
  if (epi == 1 && v == 15) return launch3<TO, 160, 128, 2, 4, 2, 128, false, 1>(g, st);
  if (epi == 1 && v == 17) return launch3<TO, 160, 128, 2, 4, 2, 64, false, 1>(g, st);
  if (epi == 1 && v == 20) return launch3<TO, 224, 256, 2, 4, 2, 64, false, 1>(g, st);
  if (epi == 2 && v == 15) return launch3<TO, 160, 128, 2, 4, 2, 128, false, 2>(g, st);
  if (epi == 2 && v == 17) return launch3<TO, 160, 128, 2, 4, 2, 64, false, 2>(g, st);
  if (epi == 2 && v == 20) return launch3<TO, 224, 256, 2, 4, 2, 64, false, 2>(g, st);
  if (epi == 1 && v == 19) return launch3<TO, 128, 128, 2, 4, 2, 64, false, 1>(g, st);
  if (epi == 2 && v == 19) return launch3<TO, 128, 128, 2, 4, 2, 64, false, 2>(g, st);
  if (epi == 1 && v == 24) return launch3<TO, 96, 128, 2, 4, 2, 128, false, 1>(g, st);
  if (epi == 1 && v == 21) return launch3<TO, 160, 128, 2, 4, 3, 64, false, 1>(g, st);
  if (epi == 2 && v == 21) return launch3<TO, 160, 128, 2, 4, 3, 64, false, 2>(g, st);
  if (epi == 1 && v == 22) return launch3<TO, 160, 128, 2, 4, 4, 64, false, 1>(g, st);
  if (epi == 2 && v == 22) return launch3<TO, 160, 128, 2, 4, 4, 64, false, 2>(g, st);
  if (epi == 2 && v == 24) return launch3<TO, 96, 128, 2, 4, 2, 128, false, 2>(g, st);
  // wide ping-pong tiles (gemm6, lean epilogues only); 56-60: timing ablations (wrong outputs)
  if (v >= 50 && v < 70 && (epi == 1 || epi == 2)) {
    const bool e1 = epi == 1;
    switch (v) {
      case 50: return e1 ? launch6<TO, 320, 256, 1>(g, st) : launch6<TO, 320, 256, 2>(g, st);
      case 51: return e1 ? launch6<TO, 320, 192, 1>(g, st) : launch6<TO, 320, 192, 2>(g, st);
      case 52: return e1 ? launch6<TO, 256, 256, 1>(g, st) : launch6<TO, 256, 256, 2>(g, st);
      case 56: return launch6<TO, 256, 256, 1, 1>(g, st);   // no LDS-DMA
      case 57: return launch6<TO, 256, 256, 1, 2>(g, st);   // no MFMA
      case 58: return launch6<TO, 320, 256, 2, 1>(g, st);   // the fc1 tile: no LDS-DMA
      case 59: return launch6<TO, 320, 256, 2, 2>(g, st);   //                no MFMA
      case 60: return launch6<TO, 320, 256, 2, 3>(g, st);   //                no epilogue
      default: return false;
    }
  }
  // forced tiles (gemm_variant, tests / tools/micro_gemm.py): the automatic candidates only
  switch (v) {
    case 1: return launch3<TO, 256, 256, 2, 4, 2, 64>(g, st);
    case 15: return launch3<TO, 160, 128, 2, 4, 2, 128>(g, st);
    case 17: return launch3<TO, 160, 128, 2, 4, 2, 64>(g, st);
    case 19: return launch3<TO, 128, 128, 2, 4, 2, 64>(g, st);
    case 20: return launch3<TO, 224, 256, 2, 4, 2, 64>(g, st);
    case 24: return launch3<TO, 96, 128, 2, 4, 2, 128>(g, st);
    default: return false;
  }
}

template <typename TA, typename TO, int BM, int BN>
void launch(const CatsegGemmArgs* g, hipStream_t st) {
  EpiArgs e;
  e.bias = g->bias;
  e.add = g->add; e.ld_add = g->ld_add; e.add_ncols = g->add_ncols;
  e.addmap = RowMap{g->addmap.d1, g->addmap.m1, g->addmap.s1, g->addmap.d2, g->addmap.m2, g->addmap.s2, g->addmap.off};
  e.act = g->act; e.alpha = g->alpha;
  e.res = g->res; e.ld_res = g->ld_res; e.res2 = g->res2; e.ld_res2 = g->ld_res2;
  e.out = g->out; e.ldo = g->ldo;
  e.store_mode = g->store_mode; e.cvt_k = g->cvt_k; e.cvt_hin = g->cvt_hin; e.cvt_win = g->cvt_win;
  e.cvt_cout = g->cvt_cout;
  RowMap am{g->amap.d1, g->amap.m1, g->amap.s1, g->amap.d2, g->amap.m2, g->amap.s2, g->amap.off};
  dim3 grid((unsigned)((g->M + BM - 1) / BM), (unsigned)((g->N + BN - 1) / BN));
  hipLaunchKernelGGL((gemm_kernel<TA, TO, BM, BN>), grid, dim3(NT), 0, st,
                     (const TA*)g->A, g->lda, am, (const TA*)g->W, g->ldw, g->M, g->N, g->K, e);
}

template <typename TO, int BM, int BN>
void launch2(const CatsegGemmArgs* g, hipStream_t st) {
  EpiArgs e;
  e.bias = g->bias;
  e.add = g->add; e.ld_add = g->ld_add; e.add_ncols = g->add_ncols;
  e.addmap = RowMap{g->addmap.d1, g->addmap.m1, g->addmap.s1, g->addmap.d2, g->addmap.m2, g->addmap.s2, g->addmap.off};
  e.act = g->act; e.alpha = g->alpha;
  e.res = g->res; e.ld_res = g->ld_res; e.res2 = g->res2; e.ld_res2 = g->ld_res2;
  e.out = g->out; e.ldo = g->ldo;
  e.store_mode = g->store_mode; e.cvt_k = g->cvt_k; e.cvt_hin = g->cvt_hin; e.cvt_win = g->cvt_win;
  e.cvt_cout = g->cvt_cout;
  RowMap am{g->amap.d1, g->amap.m1, g->amap.s1, g->amap.d2, g->amap.m2, g->amap.s2, g->amap.off};
  const int tm = (int)((g->M + BM - 1) / BM), tn = (int)((g->N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm2_kernel<TO, BM, BN>), dim3((unsigned)(tm * tn)), dim3(NT), 0, st, (const bf16*)g->A,
                     g->lda, am, (const bf16*)g->W, g->ldw, g->M, g->N, g->K, tn, e);
}

template <typename TA, typename TO>
void launch_tiles(const CatsegGemmArgs* g, hipStream_t st) {
  if constexpr (sizeof(TA) == 2) {
    if ((g->store_mode == 0 || g->cvt_cout % 8 == 0) && try_gemm3<TO>(g, st)) return;
    const int64_t t128 = ((g->M + 127) / 128) * ((g->N + 127) / 128);
    if (g->N <= 64) launch2<TO, 128, 64>(g, st);
    else if (t128 < 512) launch2<TO, 64, 128>(g, st);     // fill 256 CUs x 2 slots
    else launch2<TO, 128, 128>(g, st);
  } else {
    // fp32: 64 x 64 tiles when 128 x 128 would leave most CUs idle (the CLIP GEMMs of the training
    // step at M = 4 x 577 / 171 x 12 rows: 68-114 tiles)
    const int64_t t128 = ((g->M + 127) / 128) * ((g->N + 127) / 128);
    if (t128 < 256) launch<TA, TO, 64, 64>(g, st);
    else if (g->N <= 64) launch<TA, TO, 128, 64>(g, st);
    else launch<TA, TO, 128, 128>(g, st);
  }
}

int g_gemm_f8_variant = 0;   // 0 = automatic

// fp8 tiles (sizes in output rows x cols; BK in 2-byte units, i.e. 2x the fp8 K depth)
template <typename TO>
bool launch_f8(const CatsegGemmArgs* g, const float* sa, const float* sw, hipStream_t st) {
  int v = g_gemm_f8_variant;
  if (v == 0) {
    // same wave-quantization rule as the bf16 tiles (one round of <= 256 tiles)
    const int64_t t224 = ((g->M + 223) / 224) * (g->N / 256);
    const int64_t t160 = ((g->M + 159) / 160) * (g->N / 128);
    if (g->N % 256 == 0 && g->K % 128 == 0 && t224 >= 200 && t224 <= 256) v = 20;
    else if (g->N % 128 == 0 && g->K % 256 == 0 && t160 >= 160 && t160 <= 256) v = 15;
    else if (g->N % 128 == 0 && g->K % 128 == 0 && t160 > 256) v = 17;
    else if (g->N % 128 == 0 && g->K % 128 == 0) v = 19;
    else return false;
  }
  // lean epilogues (bias / bias + residual, bias + QuickGELU) for the automatic tiles, as in try_gemm3
  const bool plain = !g->add && !g->res2 && g->alpha == 1.f;
  const int epi = plain && g->act == ACT_NONE ? 1 : plain && g->act == ACT_QUICKGELU && !g->res ? 2 : 0;
  if (epi == 1 && v == 15) return launch3f8<TO, 160, 128, 2, 4, 2, 128, 1>(g, sa, sw, st);
  if (epi == 1 && v == 17) return launch3f8<TO, 160, 128, 2, 4, 2, 64, 1>(g, sa, sw, st);
  if (epi == 1 && v == 20) return launch3f8<TO, 224, 256, 2, 4, 2, 64, 1>(g, sa, sw, st);
  if (epi == 2 && v == 15) return launch3f8<TO, 160, 128, 2, 4, 2, 128, 2>(g, sa, sw, st);
  if (epi == 2 && v == 17) return launch3f8<TO, 160, 128, 2, 4, 2, 64, 2>(g, sa, sw, st);
  if (epi == 2 && v == 20) return launch3f8<TO, 224, 256, 2, 4, 2, 64, 2>(g, sa, sw, st);
  switch (v) {
    case 1: return launch3f8<TO, 256, 256, 2, 4, 2, 64>(g, sa, sw, st);
    case 15: return launch3f8<TO, 160, 128, 2, 4, 2, 128>(g, sa, sw, st);
    case 17: return launch3f8<TO, 160, 128, 2, 4, 2, 64>(g, sa, sw, st);
    case 19: return launch3f8<TO, 128, 128, 2, 4, 2, 64>(g, sa, sw, st);
    case 20: return launch3f8<TO, 224, 256, 2, 4, 2, 64>(g, sa, sw, st);
    case 21: return launch3f8<TO, 160, 128, 2, 4, 3, 64>(g, sa, sw, st);
    case 23: return launch3f8<TO, 160, 256, 2, 4, 3, 64>(g, sa, sw, st);
    case 24: return launch3f8<TO, 160, 256, 2, 4, 2, 64>(g, sa, sw, st);
    default: return false;
  }
}

}  // namespace

CATSEG_KNOB(g_gemm_variant, "gemm_variant");
CATSEG_KNOB(g_gemm_wide, "gemm_wide");
CATSEG_KNOB(g_gemm_group, "gemm_group");
CATSEG_KNOB(g_gemm4_group, "gemm4_group");
CATSEG_KNOB(g_epi_prefetch, "epi_prefetch");
CATSEG_KNOB(g_wide_epi, "wide_epi");
CATSEG_KNOB(g_wide_store, "wide_store");
CATSEG_KNOB(g_gemm3_store, "gemm3_store");
CATSEG_KNOB(g_gemm_f8_variant, "gemm_fp8_variant");

extern "C" int catseg_gemm_fp8(const CatsegGemmArgs* g, const float* scale_a, const float* scale_w, void* stream) {
  CATSEG_CHECK(g && g->A && g->W && g->out && scale_a && scale_w, "gemm_fp8: null pointer");
  CATSEG_CHECK(g->dtype_a == CATSEG_FP8, "gemm_fp8: dtype_a must be CATSEG_FP8");
  CATSEG_CHECK(g->M > 0 && g->N > 0 && g->K > 0, "gemm_fp8: empty shape");
  CATSEG_CHECK(g->K % 128 == 0 && g->lda % 16 == 0 && g->ldw % 16 == 0, "gemm_fp8: K must be a multiple of 128, lda/ldw of 16");
  CATSEG_CHECK(g->N % 128 == 0, "gemm_fp8: N must be a multiple of 128");
  CATSEG_CHECK(((uintptr_t)g->A % 16) == 0 && ((uintptr_t)g->W % 16) == 0 && ((uintptr_t)scale_w % 16) == 0,
               "gemm_fp8: A/W/scale_w must be 16B aligned");
  CATSEG_CHECK(g->store_mode == 0, "gemm_fp8: row-major store only");
  CATSEG_CHECK(g->ldo % 8 == 0 && ((uintptr_t)g->out % 16) == 0, "gemm_fp8: out rows must be 16B aligned");
  CATSEG_CHECK(!g->res || (g->ld_res % 8 == 0 && ((uintptr_t)g->res % 16) == 0), "gemm_fp8: res rows must be 16B aligned");
  CATSEG_CHECK(!g->res2 || (g->ld_res2 % 8 == 0 && ((uintptr_t)g->res2 % 16) == 0), "gemm_fp8: res2 rows must be 16B aligned");
  CATSEG_CHECK(!g->add || (g->add_ncols % 8 == 0 && g->ld_add % 8 == 0 && ((uintptr_t)g->add % 16) == 0),
               "gemm_fp8: add rows must be 16B aligned");
  CATSEG_CHECK(g->amap.d1 > 0 && g->amap.m1 > 0 && g->amap.d2 > 0 && g->amap.m2 > 0, "gemm_fp8: bad amap");
  CATSEG_CHECK(!g->add || (g->addmap.d1 > 0 && g->addmap.m1 > 0 && g->addmap.d2 > 0 && g->addmap.m2 > 0),
               "gemm_fp8: bad addmap");
  hipStream_t st = (hipStream_t)stream;
  bool ok;
  if (g->dtype_out == CATSEG_BF16) ok = launch_f8<bf16>(g, scale_a, scale_w, st);
  else if (g->dtype_out == CATSEG_F32) ok = launch_f8<float>(g, scale_a, scale_w, st);
  else CATSEG_FAIL("gemm_fp8: dtype_out must be f32 or bf16");
  CATSEG_CHECK(ok, "gemm_fp8: no tile fits this shape / variant");
  return catseg_launch_status("gemm_fp8");
}

extern "C" int catseg_gemm(const CatsegGemmArgs* g, void* stream) {
  CATSEG_CHECK(g && g->A && g->W && g->out, "gemm: null pointer");
  CATSEG_CHECK(g->M > 0 && g->N > 0 && g->K > 0, "gemm: empty shape");
  CATSEG_CHECK(g->N % 4 == 0, "gemm: N must be a multiple of 4");
  const int va = g->dtype_a == CATSEG_BF16 ? 8 : 4;
  CATSEG_CHECK(g->K % va == 0 && g->lda % va == 0 && g->ldw % va == 0,
               "gemm: K/lda/ldw must be multiples of 16 bytes");
  CATSEG_CHECK(((uintptr_t)g->A % 16) == 0 && ((uintptr_t)g->W % 16) == 0, "gemm: A/W must be 16B aligned");
  CATSEG_CHECK(g->ldo % 4 == 0, "gemm: ldo must be a multiple of 4");
  CATSEG_CHECK(!g->add || g->ld_add % 4 == 0, "gemm: ld_add must be a multiple of 4");
  CATSEG_CHECK(g->store_mode == 0 || (g->cvt_cout % 4 == 0 && g->cvt_k > 0 && g->cvt_hin > 0 && g->cvt_win > 0),
               "gemm: bad ConvTranspose scatter geometry");
  CATSEG_CHECK(g->store_mode == 0 || g->N == (int64_t)g->cvt_k * g->cvt_k * g->cvt_cout,
               "gemm: ConvTranspose N must be k*k*cout");
  CATSEG_CHECK(g->store_mode == 0 || g->M < (1LL << 31), "gemm: ConvTranspose row count must fit 31 bits");
  CATSEG_CHECK(g->amap.d1 > 0 && g->amap.m1 > 0 && g->amap.d2 > 0 && g->amap.m2 > 0, "gemm: bad amap");
  CATSEG_CHECK(!g->add || (g->addmap.d1 > 0 && g->addmap.m1 > 0 && g->addmap.d2 > 0 && g->addmap.m2 > 0),
               "gemm: bad addmap");
  hipStream_t st = (hipStream_t)stream;
  if (g->dtype_a == CATSEG_BF16 && g->dtype_out == CATSEG_BF16) launch_tiles<bf16, bf16>(g, st);
  else if (g->dtype_a == CATSEG_BF16 && g->dtype_out == CATSEG_F32) launch_tiles<bf16, float>(g, st);
  else if (g->dtype_a == CATSEG_F32 && g->dtype_out == CATSEG_F32) launch_tiles<float, float>(g, st);
  else if (g->dtype_a == CATSEG_F32 && g->dtype_out == CATSEG_BF16) launch_tiles<float, bf16>(g, st);
  else CATSEG_FAIL("gemm: unsupported dtype combination");
  return catseg_launch_status("gemm");
}
