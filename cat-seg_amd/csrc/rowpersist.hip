// Persistent bf16 row-block kernels for the 128-channel aggregation stream
// (reference model.py:117-225 Swin blocks, :357-424 class layers, :546 ConvTranspose).
//
// The whole weight matrix lives in REGISTERS as MFMA A-operand fragments for the life
// of the workgroup (one 8-wave workgroup per CU walks 32-row tiles), so the only
// HBM traffic is the compulsory row read and write.  Per tile:
//   rows (prefetched one tile ahead, with any residual rows) -> LayerNorm in registers
//   -> LDS -> MFMA against the register weights -> fp32 stage in LDS -> epilogue on
//   full rows with 16-byte stores.
// The MLP variant keeps the 512-wide hidden tile in LDS (H never touches HBM) and reads
// its residual (= its own input rows) from an LDS copy.  Epilogue options are template
// parameters so each variant compiles to one straight-line loop.
#include "common.h"
#include "capi.h"

namespace {

constexpr int KD = 128;          // row width
constexpr int NW = 8, NT = NW * 64;
constexpr int BM = 32;           // rows per tile
// LDS images of bf16 row tiles are chunk-major with a row XOR swizzle: 16-byte chunk c of
// tile row r lives at 16-byte slot  c * BM + (r ^ (c & 15)).  An MFMA fragment read (16
// rows x one chunk per 16 lanes, chunks 4ks+q) and a row-chunk write (8 lanes = 8 chunks
// of one row) then touch 16 (8) distinct bank slots: conflict-free (a padded row-major
// image left ~45 % of the LDS cycles of these kernels as bank conflicts, rocprofv3
// SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
template <int ROWS>
DEV int cslot(int c, int r) { return (c * ROWS + (r ^ (c & 15))) * 8; }   // element offset
constexpr int LDX = KD;          // sX holds BM rows x 16 chunks (no padding)
constexpr int CPT = BM * 16 / NT; // 16-byte chunks of a tile per thread (= 1)
constexpr int DEPTH = 3;          // tiles of input rows in flight per workgroup
constexpr int DEPTH_MLP = 1;      // (the MLP holds both weight matrices in registers: no room)
static_assert(CPT == 1, "one chunk per thread");

struct PEpi {
  const float* bias;
  const bf16* add; int64_t ld_add; RowMap addmap; int add_ncols;
  const bf16* res; int64_t ld_res;
  const bf16* res2; int64_t ld_res2;
  bf16* out; int64_t ldo;
  int cvt_k, cvt_hin, cvt_win, cvt_cout;
  int wt;                        // 1: output rows leave through sc1 write-through stores (rows_store knob)
};

// one 16-byte output chunk at element offset `idx` of e.out: plain, or sc1 write-through (the rows
// leave the XCD's L2 as they are written; the launch sets wt only when every byte offset fits 31 bits)
DEV void st_out(const PEpi& e, int64_t idx, uint4 v) {
  if (e.wt) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(e.out, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, v), r, (int)(idx * 2), 0, 16);
  } else {
    st16(e.out + idx, v);
  }
}

// thread t holds chunk t of the tile: row t/16, columns (t%16)*8 .. +8
DEV uint4 fetch_chunk(const bf16* X, int64_t ldx, int64_t m0, int64_t M) {
  const int r = threadIdx.x >> 4, ch = threadIdx.x & 15;
  const int64_t m = m0 + r;
  return m < M ? ld16(X + m * ldx + ch * 8) : make_uint4(0, 0, 0, 0);
}

// LayerNorm one chunk (16 lanes per row) and store it to LDS
DEV void put_chunk(uint4 u, const float* g, const float* b, float eps, bf16* sX) {
  const int r = threadIdx.x >> 4, ch = threadIdx.x & 15;
  if (g) {
    bf16* e = reinterpret_cast<bf16*>(&u);
    float v[8], s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { v[j] = bf2f(e[j]); s += v[j]; }
    s = row16_sum(s);
    const float mean = s * (1.f / KD);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { v[j] -= mean; q += v[j] * v[j]; }
    q = row16_sum(q);
    const float rstd = rsqrtf(q * (1.f / KD) + eps);
    const float4 g0 = *reinterpret_cast<const float4*>(g + ch * 8), g1 = *reinterpret_cast<const float4*>(g + ch * 8 + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(b + ch * 8), b1 = *reinterpret_cast<const float4*>(b + ch * 8 + 4);
    const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = f2bf(v[j] * rstd * gg[j] + bb[j]);
  }
  st16(&sX[cslot<BM>(ch, r)], u);
}

DEV void add8(float* v, uint4 u) {
  const bf16* e = reinterpret_cast<const bf16*>(&u);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] += bf2f(e[j]);
}

DEV uint4 pack8(const float* v) {
  return make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7]));
}

// ============================ persistent GEMM: out = epi(LN?(X) . W^T) =================
// wave w owns output columns [w*NOUT/8, (w+1)*NOUT/8).  Epilogue: + bias (+ add on the
// first add_ncols columns) (+ residual rows, prefetched with the input rows), row-major
// or ConvTranspose-scattered store.
template <int NOUT, bool ADD, bool RES, bool SCATTER>
__global__ __launch_bounds__(NT, 2) void pgemm_kernel(const bf16* __restrict__ X, int64_t ldx, int64_t M,
                                                      const float* ln_g, const float* ln_b, float eps,
                                                      const bf16* __restrict__ W, PEpi e) {
  static_assert(!(ADD && RES), "the add rows use the residual ring slots");
  constexpr int WN = NOUT / NW, FN = WN / 16, FM = BM / 16;
  constexpr int SLD = NOUT + 4;
  constexpr int CH = NOUT / 8;                    // 8-column items per row
  constexpr int ITEMS = BM * CH, PER = ITEMS / NT;
  static_assert(ITEMS % NT == 0, "");
  __shared__ __attribute__((aligned(16))) bf16 sX[BM * LDX];
  __shared__ __attribute__((aligned(16))) float st[BM * SLD];
  // LayerNorm gamma / beta and the bias live in LDS: a global load of them inside the tile
  // loop would be younger than the row prefetch (and the previous tile's stores), and
  // vmcnt retires in issue order, so waiting for it would expose the prefetch latency
  __shared__ __attribute__((aligned(16))) float sPar[2 * KD + NOUT];
  for (int i = threadIdx.x; i < 2 * KD + NOUT; i += NT)
    sPar[i] = i < KD ? (ln_g ? ln_g[i] : 0.f) : i < 2 * KD ? (ln_b ? ln_b[i - KD] : 0.f) : e.bias[i - 2 * KD];
  __syncthreads();
  const float* lg = ln_g ? sPar : nullptr;
  const float* lb = sPar + KD;
  const float* bias = sPar + 2 * KD;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int wn = wave * WN;
  s16x8 wf[FN][4];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      uint4 u = ld16(W + (int64_t)(wn + 16 * i + r16) * KD + ks * 32 + 8 * q);
      wf[i][ks] = *reinterpret_cast<s16x8*>(&u);
    }
  const int64_t ntiles = (M + BM - 1) / BM;
  const int64_t G = gridDim.x;
  // register ring: the rows (and residual rows) of the next DEPTH tiles are in flight
  // while this one computes (one tile per CU in flight left the loop latency-bound)
  uint4 rx[DEPTH];
  uint4 rres[DEPTH][PER];
  auto fetch = [&](uint4& x, uint4* rr, int64_t t) {
    x = fetch_chunk(X, ldx, t * BM, M);
    if constexpr (ADD) {       // the gathered guidance rows ride in the residual ring slots
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = threadIdx.x + k * NT, r = i / CH, c = (i % CH) * 8;
        const int64_t m = t * BM + r;
        rr[k] = (c < e.add_ncols && m < M) ? ld16(e.add + rowmap(e.addmap, m) * e.ld_add + c) : make_uint4(0, 0, 0, 0);
      }
    }
    if constexpr (RES) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = threadIdx.x + k * NT, r = i / CH, c = (i % CH) * 8;
        const int64_t m = t * BM + r;
        rr[k] = m < M ? ld16(e.res + m * e.ld_res + c) : make_uint4(0, 0, 0, 0);
      }
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (blockIdx.x + d * G < ntiles) fetch(rx[d], rres[d], blockIdx.x + d * G);
  for (int64_t base = blockIdx.x; base < ntiles; base += DEPTH * G)
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const int64_t tile = base + d * G;
    if (tile >= ntiles) break;
    const int64_t m0 = tile * BM;
    put_chunk(rx[d], lg, lb, eps, sX);
    uint4 res_cur[PER];
    if constexpr (RES || ADD) {
#pragma unroll
      for (int k = 0; k < PER; ++k) res_cur[k] = rres[d][k];
    }
    __syncthreads();
    if (tile + DEPTH * G < ntiles) fetch(rx[d], rres[d], tile + DEPTH * G);   // refill this ring slot
    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      s16x8 xf[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) xf[j] = *reinterpret_cast<const s16x8*>(&sX[cslot<BM>(ks * 4 + q, 16 * j + r16)]);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(wf[i][ks], xf[j], acc[i][j]);
    }
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
        *reinterpret_cast<f32x4*>(&st[(16 * j + r16) * SLD + wn + 16 * i + 4 * q]) = acc[i][j];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * NT, r = i / CH, c = (i % CH) * 8;
      const int64_t m = m0 + r;
      const bool do_add = ADD && c < e.add_ncols && m < M;
      float v[8];
      *reinterpret_cast<f32x4*>(&v[0]) = *reinterpret_cast<const f32x4*>(&st[r * SLD + c]);
      *reinterpret_cast<f32x4*>(&v[4]) = *reinterpret_cast<const f32x4*>(&st[r * SLD + c + 4]);
      const float4 b0 = *reinterpret_cast<const float4*>(bias + c), b1 = *reinterpret_cast<const float4*>(bias + c + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
      if (do_add) add8(v, res_cur[k]);
      if constexpr (RES) add8(v, res_cur[k]);
      if (m < M) {
        int64_t off;
        if constexpr (SCATTER) {
          off = convt_offset(m, c, e.cvt_k, e.cvt_hin, e.cvt_win, e.cvt_cout);
        } else {
          off = m * e.ldo + c;
        }
        st_out(e, off, pack8(v));
      }
    }
    __syncthreads();
  }
}

// ============================ persistent MLP ===========================================
// out = Y + act(LN(Y) . W1^T + b1) . W2^T + b2 (+ R2), hidden = 512.
// wave w: GEMM1 hidden rows [64w, 64w+64) (W1 fragments in registers),
//         GEMM2 output rows [16w, 16w+16) over all 512 hidden (W2 fragments in registers).
// sH: 528-element rows (66 16-byte slots), 16-byte chunk c of row r at slot c ^ ((r >> 2) & 1).
// The GEMM1 output writes (8 lanes = rows r..r+7 of one chunk) and the GEMM2 fragment reads (lanes
// r16, q: chunk 4 ks + q of row r16) then hit distinct bank slots in every lane group
// (tools/lds_bank_model.py), and the swizzle only flips the q part of a chunk index, so a lane's
// 16 GEMM2 reads stay one base + immediate offsets.  Round 3's unswizzled 528 read conflict-free
// but wrote 2-way conflicted (rows r and r + 4 on one slot; ~14 % of the kernel's LDS cycles,
// SQ_LDS_BANK_CONFLICT); 520 had the reverse (42 %); a full 4-bit row XOR on unpadded rows is
// conflict-free too but its per-k-step addresses pushed the projection + MLP kernel to 256 VGPRs
// and a spill (488 vs 398 us).
constexpr int HID = 512, LDH = HID + 16;
DEV int hoff(int r, int e) { return r * LDH + ((((e >> 3) ^ ((r >> 2) & 1))) << 3) + (e & 7); }

// PROJ (catseg_swin_proj_mlp): the Swin block's output projection + residual runs first, per
// tile: x1 = bf16(x + attn . Wp^T + bp) (model.py:112 proj, :222 shortcut), then the MLP above
// on x1 (Y = the attention rows, res2 slot = the x rows); x1 never reaches HBM, and the
// arithmetic (MFMA order, bias then residual, one bf16 rounding) is the separate
// pgemm_kernel<128, false, true> + pmlp_kernel pair's, bit for bit.
// PAIR: fragments 2hf and 2hf+1 of wave w take the 32 hidden units 64w + 32hf + [0, 32) in
// the order  row r of fragment i -> unit 8 (r / 4) + 4 i + r % 4,  so lane quad q ends GEMM1
// holding units 8q .. 8q+7 of the pair: one 16-byte ds_write_b128 per row instead of two
// 8-byte stores 16 units apart (whose 16 lanes sat 4-way on one bank pair at the 264-dword
// row stride).  Every hidden unit is still one MFMA chain over the same k order: bit-identical.
// GELU of the persistent MLPs as a segment table (tools/gelu_table_fit.py): Phi on [-5, 5] as 32 cubics
// in the in-segment position, GELU(x) = x * P_seg(f).  Per value: fma + med3 (segment coordinate),
// cvt + fract, one 16-byte LDS read of the segment's coefficients (512-byte table: at most two
// segments per bank group), 3 fma + mul: 9 single-rate VALU against 2 med3 + 12 packed ops per value
// pair for the degree-8 polynomial (gelu1, 3.0e-5), at a max GELU error of 4.3e-6.  Same box
// (tools/micro_mlp.py): Swin proj + MLP 390 -> 379 us (the file built without SLP, Makefile); in the
// step the two forms take the same time (363 vs 364 us), so the gain is the 7x smaller error.
// GELU_SEG=0 builds the polynomial form (A/B).
#ifndef GELU_SEG
#define GELU_SEG 1
#endif
constexpr int GSEG = 32;
__device__ const float kGeluSeg[GSEG][4] = {
    {2.857138099e-07f, 4.937455742e-07f, 2.254223403e-07f, 3.768647900e-07f},
    {1.379555215e-06f, 2.212427944e-06f, 1.064327307e-06f, 1.411648441e-06f},
    {6.061552995e-06f, 9.013059753e-06f, 4.444804745e-06f, 4.744361377e-06f},
    {2.424740342e-05f, 3.337237649e-05f, 1.648918806e-05f, 1.427804364e-05f},
    {8.835084009e-05f, 1.122780523e-04f, 5.447883814e-05f, 3.837561962e-05f},
    {2.934156510e-04f, 3.431500809e-04f, 1.605219877e-04f, 9.178832261e-05f},
    {8.887727745e-04f, 9.524713387e-04f, 4.219991388e-04f, 1.943924581e-04f},
    {2.457518829e-03f, 2.400514437e-03f, 9.894206887e-04f, 3.618174233e-04f},
    {6.209207233e-03f, 5.492324010e-03f, 2.066157293e-03f, 5.848744768e-04f},
    {1.435265690e-02f, 1.140593924e-02f, 3.833262948e-03f, 8.041608962e-04f},
    {3.039636090e-02f, 2.149616554e-02f, 6.291609723e-03f, 9.010374779e-04f},
    {5.908574536e-02f, 3.676088154e-02f, 9.071586654e-03f, 7.322515594e-04f},
    {1.056510732e-01f, 5.703652650e-02f, 1.135013346e-02f, 2.143343008e-04f},
    {1.742523909e-01f, 8.028168976e-02f, 1.203648932e-02f, -5.833524046e-04f},
    {2.659869790e-01f, 1.025029495e-01f, 1.025549136e-02f, -1.413749764e-03f},
    {3.773308992e-01f, 1.187075824e-01f, 5.908886902e-03f, -1.946855802e-03f},
    {4.999994934e-01f, 1.246847883e-01f, -6.831953942e-05f, -1.946855802e-03f},
    {6.226683259e-01f, 1.187726855e-01f, -6.014242303e-03f, -1.413749764e-03f},
    {7.340127826e-01f, 1.026046127e-01f, -1.028643269e-02f, -5.833524046e-04f},
    {8.257479072e-01f, 8.037979901e-02f, -1.199313626e-02f, 2.143343008e-04f},
    {8.943495154e-01f, 5.710081011e-02f, -1.126834191e-02f, 7.322515594e-04f},
    {9.409148097e-01f, 3.678249940e-02f, -8.994722739e-03f, 9.010374779e-04f},
    {9.696039557e-01f, 2.148494869e-02f, -6.245745812e-03f, 8.041608962e-04f},
    {9.856474400e-01f, 1.137926243e-02f, -3.820780898e-03f, 5.848744768e-04f},
    {9.937907457e-01f, 5.464808084e-03f, -2.074873075e-03f, 3.618174233e-04f},
    {9.975423813e-01f, 2.379646990e-03f, -1.005176571e-03f, 1.943924581e-04f},
    {9.991111159e-01f, 9.395590168e-04f, -4.358869628e-04f, 9.178832261e-05f},
    {9.997065067e-01f, 3.363625729e-04f, -1.696057006e-04f, 3.837561962e-05f},
    {9.999116063e-01f, 1.091848826e-04f, -5.932331987e-05f, 1.427804364e-05f},
    {9.999757409e-01f, 3.213575474e-05f, -1.867788887e-05f, 4.744361377e-06f},
    {9.999939203e-01f, 8.576027540e-06f, -5.299272743e-06f, 1.411648441e-06f},
    {9.999986291e-01f, 2.075184739e-06f, -1.356016696e-06f, 3.768647900e-07f},
};
// (fit: R = 5, 32 cubic segments; max |GELU error| 4.3e-6 on [-12, 12], 1.7e-6 on [-4, 4])
//
// ACT_GELU7 (gelu_form knob 1): the same idea in 7 VALU per value (tools/gelu_x7_fit.py).  The segment
// k = round(3.2 x + 16), clamped to [0, 32], comes without a float->int conversion: t = fma(x, 3.2,
// 2^23 + 16) rounds to an integer whose fp32 bits are 0x4B000000 + k, med3 clamps it, and the bits
// shifted left by 4 address the 16-byte coefficient row (one v_lshl_add_u32); the cubic is in x itself
// (no in-segment coordinate, so no fract), the edge segments are the constants 0 and 1, so x * P stays
// bounded for any x.  fma + med3 + lshl_add + LDS read + 3 fma + mul against gelu_seg's 9 VALU.
constexpr int ACT_GELU7 = 91;      // internal activation id (not in the C ABI)
constexpr int GSEG7 = 33;
// 33 segments (k = round(3.2 x + 16), edges 0 / 1), cubic in x: max |GELU error| 3.287e-06 on [-12, 12] (1.547e-06 on [-4, 4])
__device__ const float kGeluX7[GSEG7][4] = {
    {0.000000000e+00f, 0.000000000e+00f, 0.000000000e+00f, 0.000000000e+00f},
    {2.882618923e-03f, 1.753379707e-03f, 3.561640915e-04f, 2.415746530e-05f},
    {8.511394262e-03f, 5.501359701e-03f, 1.188187511e-03f, 8.573576633e-05f},
    {2.231834829e-02f, 1.537315361e-02f, 3.541412065e-03f, 2.727602259e-04f},
    {5.184482783e-02f, 3.816473484e-02f, 9.407166392e-03f, 7.760967128e-04f},
    {1.064083949e-01f, 8.392206579e-02f, 2.220178954e-02f, 1.968990080e-03f},
    {1.924447566e-01f, 1.628885567e-01f, 4.636982083e-02f, 4.435458686e-03f},
    {3.059913516e-01f, 2.779548168e-01f, 8.525618166e-02f, 8.817944676e-03f},
    {4.273824394e-01f, 4.152130187e-01f, 1.370187402e-01f, 1.532850228e-02f},
    {5.257804394e-01f, 5.409126878e-01f, 1.905829757e-01f, 2.294243686e-02f},
    {5.756489635e-01f, 6.137913465e-01f, 2.261149138e-01f, 2.872194536e-02f},
    {5.745609403e-01f, 6.108088493e-01f, 2.237454057e-01f, 2.813855931e-02f},
    {5.451580286e-01f, 5.472433567e-01f, 1.778536141e-01f, 1.707486995e-02f},
    {5.165857673e-01f, 4.688404500e-01f, 1.059021130e-01f, -5.007953849e-03f},
    {5.029187202e-01f, 4.172078967e-01f, 4.047473893e-02f, -3.282082453e-02f},
    {5.001025200e-01f, 4.003199339e-01f, 6.250044797e-03f, -5.630261824e-02f},
    {5.000000000e-01f, 3.989397287e-01f, -2.000167085e-15f, -6.615200639e-02f},
    {4.998974502e-01f, 4.003199339e-01f, -6.250044797e-03f, -5.630261824e-02f},
    {4.970813096e-01f, 4.172078967e-01f, -4.047473893e-02f, -3.282082453e-02f},
    {4.834142625e-01f, 4.688404500e-01f, -1.059021130e-01f, -5.007953849e-03f},
    {4.548419714e-01f, 5.472433567e-01f, -1.778536141e-01f, 1.707486995e-02f},
    {4.254390597e-01f, 6.108088493e-01f, -2.237454057e-01f, 2.813855931e-02f},
    {4.243510365e-01f, 6.137913465e-01f, -2.261149138e-01f, 2.872194536e-02f},
    {4.742195904e-01f, 5.409126878e-01f, -1.905829757e-01f, 2.294243686e-02f},
    {5.726175308e-01f, 4.152130187e-01f, -1.370187402e-01f, 1.532850228e-02f},
    {6.940086484e-01f, 2.779548168e-01f, -8.525618166e-02f, 8.817944676e-03f},
    {8.075552583e-01f, 1.628885567e-01f, -4.636982083e-02f, 4.435458686e-03f},
    {8.935915828e-01f, 8.392206579e-02f, -2.220178954e-02f, 1.968990080e-03f},
    {9.481551647e-01f, 3.816473484e-02f, -9.407166392e-03f, 7.760967128e-04f},
    {9.776816368e-01f, 1.537315361e-02f, -3.541412065e-03f, 2.727602259e-04f},
    {9.914885759e-01f, 5.501359701e-03f, -1.188187511e-03f, 8.573576633e-05f},
    {9.971174002e-01f, 1.753379707e-03f, -3.561640915e-04f, 2.415746530e-05f},
    {1.000000000e+00f, 0.000000000e+00f, 0.000000000e+00f, 0.000000000e+00f},
};
constexpr int GTAB = GSEG7;        // float4 rows of the LDS table (either form)
template <int ACT>
DEV void stage_gelu_table(float4* sG) {
  if constexpr (ACT == ACT_GELU7) {
    if (threadIdx.x < GSEG7) sG[threadIdx.x] = *reinterpret_cast<const float4*>(kGeluX7[threadIdx.x]);
  } else {
    if (threadIdx.x < GSEG) sG[threadIdx.x] = *reinterpret_cast<const float4*>(kGeluSeg[threadIdx.x]);
  }
}
DEV float gelu_x7(float x, const float4* sG) {
  const float t = __builtin_amdgcn_fmed3f(__builtin_fmaf(x, 3.2f, 8388624.0f), 8388608.0f, 8388640.0f);
  const unsigned off = (__builtin_bit_cast(unsigned, t) << 4) - (0x4B000000u << 4);
  const float4 c = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(sG) + off);
  return x * __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(c.w, x, c.z), x, c.y), x, c.x);
}
DEV float gelu_seg(float x, const float4* sG) {
  const float u = __builtin_amdgcn_fmed3f(__builtin_fmaf(x, GSEG / 10.f, GSEG / 2.f), 0.f, GSEG - 0x1p-18f);
  const float4 c = sG[(int)u];
  const float f = __builtin_amdgcn_fractf(u);
  return x * __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(c.w, f, c.z), f, c.y), f, c.x);
}
template <int ACT>
DEV float mlp_act(float v, const float4* sG) {
  if constexpr (ACT == ACT_GELU7) return gelu_x7(v, sG);
  else if constexpr (ACT == ACT_GELU) return GELU_SEG ? gelu_seg(v, sG) : gelu1(v);
  else return act_t<ACT>(v);
}

template <int ACT, bool RES2, bool PROJ = false, bool PAIR = true>
__global__ __launch_bounds__(NT, 2) void pmlp_kernel(const bf16* __restrict__ Y, int64_t ldy, int64_t M,
                                                     const float* ln_g, const float* ln_b, float eps,
                                                     const bf16* __restrict__ W1, const float* __restrict__ b1,
                                                     const bf16* __restrict__ W2, PEpi e,
                                                     const bf16* __restrict__ Xr = nullptr, int64_t ldxr = 0,
                                                     const bf16* __restrict__ Wp = nullptr,
                                                     const float* __restrict__ bp = nullptr) {
  static_assert(!(PROJ && RES2), "PROJ carries the x rows in the res2 slot");
  constexpr int FM = BM / 16, SLD = KD + 4;
  constexpr int NPAR = 2 * KD + HID + KD + (PROJ ? KD : 0);
  __shared__ __attribute__((aligned(16))) bf16 sX[BM * LDX];
  __shared__ __attribute__((aligned(16))) bf16 sH[BM * LDH];
  __shared__ __attribute__((aligned(16))) float st[BM * SLD];
  // gamma / beta / b1 / b2 (/ bp) in LDS (see pgemm_kernel: no global loads behind the prefetch)
  __shared__ __attribute__((aligned(16))) float sPar[NPAR];
  __shared__ __attribute__((aligned(16))) float4 sG[GTAB];
  for (int i = threadIdx.x; i < NPAR; i += NT)
    sPar[i] = i < KD ? ln_g[i] : i < 2 * KD ? ln_b[i - KD] : i < 2 * KD + HID ? b1[i - 2 * KD]
            : i < 3 * KD + HID ? e.bias[i - 2 * KD - HID] : bp[i - 3 * KD - HID];
  stage_gelu_table<ACT>(sG);
  __syncthreads();
  const float* sb1 = sPar + 2 * KD;
  const float* sb2 = sPar + 2 * KD + HID;
  const float* sbp = sPar + 3 * KD + HID;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  // the hidden tile's chunk swizzle (hoff) as per-lane offsets: GEMM1 stores at column hh + hsw,
  // GEMM2 fragment reads at ks * 32 + hq
  const int hsw = (((q ^ ((r16 >> 2) & 1)) - q) << 3), hq = (q ^ ((r16 >> 2) & 1)) << 3;
  s16x8 wpf[PROJ ? 4 : 1];           // PROJ: Wp rows 16*wave .. +15 (this wave's proj columns)
  if constexpr (PROJ) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      uint4 u = ld16(Wp + (int64_t)(16 * wave + r16) * KD + ks * 32 + 8 * q);
      wpf[ks] = *reinterpret_cast<s16x8*>(&u);
    }
  }
  s16x8 w1f[4][4], w2f[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int unit = PAIR ? 64 * wave + 32 * (i >> 1) + 8 * (r16 >> 2) + 4 * (i & 1) + (r16 & 3)
                            : 64 * wave + 16 * i + r16;
      uint4 u = ld16(W1 + (int64_t)unit * KD + ks * 32 + 8 * q);
      w1f[i][ks] = *reinterpret_cast<s16x8*>(&u);
    }
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    uint4 u = ld16(W2 + (int64_t)(16 * wave + r16) * HID + ks * 32 + 8 * q);
    w2f[ks] = *reinterpret_cast<s16x8*>(&u);
  }
  const int64_t ntiles = (M + BM - 1) / BM;
  const int64_t G = gridDim.x;
  const int er = threadIdx.x >> 4, ec = (threadIdx.x & 15) * 8;   // epilogue item = the thread's input chunk
  uint4 ry[DEPTH_MLP] = {}, rr2[DEPTH_MLP] = {};
  auto fetch = [&](uint4& y, uint4& r2, int64_t t) {
    y = fetch_chunk(Y, ldy, t * BM, M);
    if constexpr (RES2) r2 = fetch_chunk(e.res2, e.ld_res2, t * BM, M);
    if constexpr (PROJ) r2 = fetch_chunk(Xr, ldxr, t * BM, M);
  };
#pragma unroll
  for (int d = 0; d < DEPTH_MLP; ++d)
    if (blockIdx.x + d * G < ntiles) fetch(ry[d], rr2[d], blockIdx.x + d * G);
  for (int64_t base = blockIdx.x; base < ntiles; base += DEPTH_MLP * G)
#pragma unroll
  for (int d = 0; d < DEPTH_MLP; ++d) {
    const int64_t tile = base + d * G;
    if (tile >= ntiles) break;
    const int64_t m0 = tile * BM;
    uint4 y_raw = ry[d];                            // residuals of this tile stay in registers
    const uint4 r2_cur = rr2[d];
    if constexpr (PROJ) {
      put_chunk(ry[d], nullptr, nullptr, eps, sX);  // the attention rows, as they are
      __syncthreads();
      f32x4 ap[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) ap[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
        for (int j = 0; j < FM; ++j)
          ap[j] = mfma_bf16(wpf[ks], *reinterpret_cast<const s16x8*>(&sX[cslot<BM>(ks * 4 + q, 16 * j + r16)]), ap[j]);
      }
#pragma unroll
      for (int j = 0; j < FM; ++j)
        *reinterpret_cast<f32x4*>(&st[(16 * j + r16) * SLD + 16 * wave + 4 * q]) = ap[j];
      __syncthreads();
      float v[8];
      *reinterpret_cast<f32x4*>(&v[0]) = *reinterpret_cast<const f32x4*>(&st[er * SLD + ec]);
      *reinterpret_cast<f32x4*>(&v[4]) = *reinterpret_cast<const f32x4*>(&st[er * SLD + ec + 4]);
      const float4 p0 = *reinterpret_cast<const float4*>(sbp + ec), p1 = *reinterpret_cast<const float4*>(sbp + ec + 4);
      v[0] += p0.x; v[1] += p0.y; v[2] += p0.z; v[3] += p0.w;
      v[4] += p1.x; v[5] += p1.y; v[6] += p1.z; v[7] += p1.w;
      add8(v, r2_cur);
      y_raw = pack8(v);                             // x1 = bf16(attn . Wp^T + bp + x)
    }
    put_chunk(y_raw, sPar, sPar + KD, eps, sX);
    __syncthreads();
    if (tile + DEPTH_MLP * G < ntiles) fetch(ry[d], rr2[d], tile + DEPTH_MLP * G);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      // the accumulators start from the fc1 bias (no per-element add after the MFMAs)
      f32x4 acc1[2][FM];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int u0 = PAIR ? 64 * wave + 32 * hf + 8 * q + 4 * i : 64 * wave + 16 * (2 * hf + i) + 4 * q;
        const float4 bv = *reinterpret_cast<const float4*>(sb1 + u0);
#pragma unroll
        for (int j = 0; j < FM; ++j) acc1[i][j] = f32x4{bv.x, bv.y, bv.z, bv.w};
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s16x8 xf[FM];
#pragma unroll
        for (int j = 0; j < FM; ++j) xf[j] = *reinterpret_cast<const s16x8*>(&sX[cslot<BM>(ks * 4 + q, 16 * j + r16)]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc1[i][j] = mfma_bf16(w1f[2 * hf + i][ks], xf[j], acc1[i][j]);
      }
      if constexpr (PAIR) {
        const int hh = 64 * wave + 32 * hf + 8 * q;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          float v[8];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[4 * i + r] = mlp_act<ACT>(acc1[i][j][r], sG);
            }
          st16(&sH[(16 * j + r16) * LDH + hh + hsw], pack8(v));
        }
      } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int hh = 64 * wave + 16 * (2 * hf + i) + 4 * q;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = mlp_act<ACT>(acc1[i][j][r], sG);
          store4<bf16>(&sH[hoff(16 * j + r16, hh)], v);
        }
      }
      }
    }
    __syncthreads();
    f32x4 acc2[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const s16x8 hf = *reinterpret_cast<const s16x8*>(&sH[(16 * j + r16) * LDH + ks * 32 + hq]);
        acc2[j] = mfma_bf16(w2f[ks], hf, acc2[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < FM; ++j)
      *reinterpret_cast<f32x4*>(&st[(16 * j + r16) * SLD + 16 * wave + 4 * q]) = acc2[j];
    __syncthreads();
    {
      const int64_t m = m0 + er;
      float v[8];
      *reinterpret_cast<f32x4*>(&v[0]) = *reinterpret_cast<const f32x4*>(&st[er * SLD + ec]);
      *reinterpret_cast<f32x4*>(&v[4]) = *reinterpret_cast<const f32x4*>(&st[er * SLD + ec + 4]);
      const float4 c0 = *reinterpret_cast<const float4*>(sb2 + ec), c1 = *reinterpret_cast<const float4*>(sb2 + ec + 4);
      v[0] += c0.x; v[1] += c0.y; v[2] += c0.z; v[3] += c0.w;
      v[4] += c1.x; v[5] += c1.y; v[6] += c1.z; v[7] += c1.w;
      add8(v, y_raw);
      if constexpr (RES2) add8(v, r2_cur);
      if (m < M) st_out(e, m * e.ldo + ec, pack8(v));
    }
    __syncthreads();
  }
}

// ---- barrier-lean form (default): the epilogue of tile t runs in the same barrier interval as
// the first GEMM (MLP) / the projection (PROJ) of tile t+1, and the next tile's rows are put into
// LDS beside GEMM2 of this one; the residual rows (x1 / the raw input rows, res2) wait in LDS,
// double-buffered by tile parity, instead of registers.  Barriers per 32-row tile: 2 (MLP) /
// 4 (PROJ) instead of 4 / 6 -- one workgroup per CU (the weights fill the registers), so every
// barrier stalls all of the CU's waves.  Same arithmetic in the same order as pmlp_kernel
// (PAIR order): bit-identical.
template <int ACT, bool RES2, bool PROJ>
__global__ __launch_bounds__(NT, 2) void pmlp2_kernel(const bf16* __restrict__ Y, int64_t ldy, int64_t M,
                                                      const float* ln_g, const float* ln_b, float eps,
                                                      const bf16* __restrict__ W1, const float* __restrict__ b1,
                                                      const bf16* __restrict__ W2, PEpi e,
                                                      const bf16* __restrict__ Xr = nullptr, int64_t ldxr = 0,
                                                      const bf16* __restrict__ Wp = nullptr,
                                                      const float* __restrict__ bp = nullptr) {
  static_assert(!(PROJ && RES2), "PROJ carries the x rows in the res2 slot");
  constexpr int FM = BM / 16, SLD = KD + 4;
  constexpr int NPAR = 2 * KD + HID + KD + (PROJ ? KD : 0);
  __shared__ __attribute__((aligned(16))) bf16 sX[BM * LDX];
  __shared__ __attribute__((aligned(16))) bf16 sH[BM * LDH];
  __shared__ __attribute__((aligned(16))) float stA[PROJ ? BM * SLD : 4];      // projection output
  __shared__ __attribute__((aligned(16))) float stB[BM * SLD];                 // GEMM2 output
  __shared__ __attribute__((aligned(16))) bf16 yres[2][BM * KD];               // x1 / raw rows, by tile parity
  __shared__ __attribute__((aligned(16))) bf16 r2res[RES2 ? 2 : 1][RES2 ? BM * KD : 8];
  __shared__ __attribute__((aligned(16))) bf16 xres[PROJ ? BM * KD : 8];       // PROJ: the x rows
  __shared__ __attribute__((aligned(16))) float sPar[NPAR];
  __shared__ __attribute__((aligned(16))) float4 sG[GTAB];
  for (int i = threadIdx.x; i < NPAR; i += NT)
    sPar[i] = i < KD ? ln_g[i] : i < 2 * KD ? ln_b[i - KD] : i < 2 * KD + HID ? b1[i - 2 * KD]
            : i < 3 * KD + HID ? e.bias[i - 2 * KD - HID] : bp[i - 3 * KD - HID];
  stage_gelu_table<ACT>(sG);
  const float* sb1 = sPar + 2 * KD;
  const float* sb2 = sPar + 2 * KD + HID;
  const float* sbp = sPar + 3 * KD + HID;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  // the hidden tile's chunk swizzle (hoff) as per-lane offsets: GEMM1 stores at column hh + hsw,
  // GEMM2 fragment reads at ks * 32 + hq
  const int hsw = (((q ^ ((r16 >> 2) & 1)) - q) << 3), hq = (q ^ ((r16 >> 2) & 1)) << 3;
  s16x8 wpf[PROJ ? 4 : 1];
  if constexpr (PROJ) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) wpf[ks] = __builtin_bit_cast(s16x8, ld16(Wp + (int64_t)(16 * wave + r16) * KD + ks * 32 + 8 * q));
  }
  s16x8 w1f[4][4], w2f[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int unit = 64 * wave + 32 * (i >> 1) + 8 * (r16 >> 2) + 4 * (i & 1) + (r16 & 3);
      w1f[i][ks] = __builtin_bit_cast(s16x8, ld16(W1 + (int64_t)unit * KD + ks * 32 + 8 * q));
    }
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) w2f[ks] = __builtin_bit_cast(s16x8, ld16(W2 + (int64_t)(16 * wave + r16) * HID + ks * 32 + 8 * q));
  const int64_t ntiles = (M + BM - 1) / BM;
  const int64_t G = gridDim.x;
  const int er = threadIdx.x >> 4, ec = (threadIdx.x & 15) * 8;   // this thread's chunk of a tile
  const int rofs = er * KD + ec;
  uint4 ry = {}, rr2 = {};                        // rows of the next tile, in flight
  auto fetch = [&](int64_t t) {
    ry = fetch_chunk(Y, ldy, t * BM, M);
    if constexpr (RES2) rr2 = fetch_chunk(e.res2, e.ld_res2, t * BM, M);
    if constexpr (PROJ) rr2 = fetch_chunk(Xr, ldxr, t * BM, M);
  };
  auto put = [&](int par) {                       // the fetched tile -> LDS
    if constexpr (PROJ) {
      put_chunk(ry, nullptr, nullptr, eps, sX);   // the attention rows, as they are
      st16(&xres[rofs], rr2);
    } else {
      st16(&yres[par][rofs], ry);
      if constexpr (RES2) st16(&r2res[par][rofs], rr2);
      put_chunk(ry, sPar, sPar + KD, eps, sX);
    }
  };
  auto gemm1 = [&]() {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      f32x4 acc1[2][FM];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float4 bv = *reinterpret_cast<const float4*>(sb1 + 64 * wave + 32 * hf + 8 * q + 4 * i);
#pragma unroll
        for (int j = 0; j < FM; ++j) acc1[i][j] = f32x4{bv.x, bv.y, bv.z, bv.w};
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s16x8 xf[FM];
#pragma unroll
        for (int j = 0; j < FM; ++j) xf[j] = *reinterpret_cast<const s16x8*>(&sX[cslot<BM>(ks * 4 + q, 16 * j + r16)]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc1[i][j] = mfma_bf16(w1f[2 * hf + i][ks], xf[j], acc1[i][j]);
      }
      const int hh = 64 * wave + 32 * hf + 8 * q;
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[4 * i + r] = mlp_act<ACT>(acc1[i][j][r], sG);
          }
        st16(&sH[(16 * j + r16) * LDH + hh + hsw], pack8(v));
      }
    }
  };
  auto epilogue = [&](int64_t t, int par) {
    const int64_t m = t * BM + er;
    float v[8];
    *reinterpret_cast<f32x4*>(&v[0]) = *reinterpret_cast<const f32x4*>(&stB[er * SLD + ec]);
    *reinterpret_cast<f32x4*>(&v[4]) = *reinterpret_cast<const f32x4*>(&stB[er * SLD + ec + 4]);
    const float4 c0 = *reinterpret_cast<const float4*>(sb2 + ec), c1 = *reinterpret_cast<const float4*>(sb2 + ec + 4);
    v[0] += c0.x; v[1] += c0.y; v[2] += c0.z; v[3] += c0.w;
    v[4] += c1.x; v[5] += c1.y; v[6] += c1.z; v[7] += c1.w;
    add8(v, *reinterpret_cast<const uint4*>(&yres[par][rofs]));
    if constexpr (RES2) add8(v, *reinterpret_cast<const uint4*>(&r2res[par][rofs]));
    if (m < M) st_out(e, m * e.ldo + ec, pack8(v));
  };

  int64_t t = blockIdx.x;
  if (t < ntiles) fetch(t);
  __syncthreads();                                // sPar
  if (t < ntiles) put(0);
  if (t + G < ntiles) fetch(t + G);
  __syncthreads();
  int it = 0;
  for (; t < ntiles; t += G, ++it) {
    const int par = it & 1;
    // [A] projection (PROJ) / GEMM1 of tile t beside the epilogue of tile t - G
    if constexpr (PROJ) {
      f32x4 ap[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) ap[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          ap[j] = mfma_bf16(wpf[ks], *reinterpret_cast<const s16x8*>(&sX[cslot<BM>(ks * 4 + q, 16 * j + r16)]), ap[j]);
#pragma unroll
      for (int j = 0; j < FM; ++j)
        *reinterpret_cast<f32x4*>(&stA[(16 * j + r16) * SLD + 16 * wave + 4 * q]) = ap[j];
    } else {
      gemm1();
    }
    if (it > 0) epilogue(t - G, par ^ 1);
    __syncthreads();
    if constexpr (PROJ) {
      // [B] x1 = bf16(attn . Wp^T + bp + x) -> residual slot; LayerNorm(x1) -> sX
      float v[8];
      *reinterpret_cast<f32x4*>(&v[0]) = *reinterpret_cast<const f32x4*>(&stA[er * SLD + ec]);
      *reinterpret_cast<f32x4*>(&v[4]) = *reinterpret_cast<const f32x4*>(&stA[er * SLD + ec + 4]);
      const float4 p0 = *reinterpret_cast<const float4*>(sbp + ec), p1 = *reinterpret_cast<const float4*>(sbp + ec + 4);
      v[0] += p0.x; v[1] += p0.y; v[2] += p0.z; v[3] += p0.w;
      v[4] += p1.x; v[5] += p1.y; v[6] += p1.z; v[7] += p1.w;
      add8(v, *reinterpret_cast<const uint4*>(&xres[rofs]));
      const uint4 x1 = pack8(v);
      st16(&yres[par][rofs], x1);
      put_chunk(x1, sPar, sPar + KD, eps, sX);
      __syncthreads();
      // [C] GEMM1
      gemm1();
      __syncthreads();
    }
    // [D] GEMM2 -> stB; the next tile's rows -> LDS; the one after that requested
    f32x4 acc2[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const s16x8 hf = *reinterpret_cast<const s16x8*>(&sH[(16 * j + r16) * LDH + ks * 32 + hq]);
        acc2[j] = mfma_bf16(w2f[ks], hf, acc2[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < FM; ++j)
      *reinterpret_cast<f32x4*>(&stB[(16 * j + r16) * SLD + 16 * wave + 4 * q]) = acc2[j];
    if (t + G < ntiles) {
      put(par ^ 1);
      if (t + 2 * G < ntiles) fetch(t + 2 * G);
    }
    __syncthreads();
  }
  if (it > 0) epilogue(t - G, (it - 1) & 1);
}

// ============================ decoder ConvTranspose over 64-channel rows ================
// out = scatter_k2(relu(GN(X)) . W^T + bias): the second Up block's ConvTranspose2d
// (model.py:546) fused with the preceding GroupNorm+ReLU of DoubleConv (model.py:532-533).
// X: [M][64] NHWC rows, slice = row / HW (HW % 64 == 0), W: [NOUT][64] in registers.
constexpr int K64 = 64, NW4 = 4, NT4 = NW4 * 64, BM64 = 64, LDX64 = K64 + 8;

template <int NOUT>
__global__ __launch_bounds__(NT4, 2) void pconvt64_kernel(const bf16* __restrict__ X, int64_t M, int64_t HW,
                                                          const float* mean, const float* rstd, const float* gamma,
                                                          const float* beta, int cpg, const bf16* __restrict__ W,
                                                          PEpi e) {
  constexpr int WN = NOUT / NW4, FN = WN / 16, FM = BM64 / 16;
  constexpr int SLD = NOUT + 4, CH = NOUT / 8, ITEMS = BM64 * CH, PER = ITEMS / NT4;
  static_assert(WN % 16 == 0 && ITEMS % NT4 == 0, "");
  __shared__ __attribute__((aligned(16))) bf16 sX[BM64 * LDX64];
  __shared__ __attribute__((aligned(16))) float st[BM64 * SLD];
  __shared__ float ssc[K64], ssh[K64];
  // bias / gamma / beta in LDS once, and the next tile's rows + GroupNorm statistics
  // prefetched right after this tile's rows reach LDS: no global load is issued behind the
  // previous tile's stores (vmcnt retires in order)
  __shared__ __attribute__((aligned(16))) float sPar[NOUT + 2 * K64];
  for (int i = threadIdx.x; i < NOUT + 2 * K64; i += NT4)
    sPar[i] = i < NOUT ? e.bias[i] : i < NOUT + K64 ? gamma[i - NOUT] : beta[i - NOUT - K64];
  __syncthreads();
  const float* sbias = sPar;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int wn = wave * WN;
  s16x8 wf[FN][2];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 u = ld16(W + (int64_t)(wn + 16 * i + r16) * K64 + ks * 32 + 8 * q);
      wf[i][ks] = *reinterpret_cast<s16x8*>(&u);
    }
  const int groups = K64 / cpg;
  const int64_t ntiles = (M + BM64 - 1) / BM64;
  uint4 u[2];
  float pm = 0.f, pr = 0.f;
  auto fetch = [&](int64_t t) {
    const int64_t m0 = t * BM64;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = threadIdx.x + k * NT4, r = c >> 3, ch = c & 7;
      u[k] = m0 + r < M ? ld16(X + (m0 + r) * K64 + ch * 8) : make_uint4(0, 0, 0, 0);
    }
    if (threadIdx.x < K64) {
      const int64_t gi = (m0 / HW) * groups + threadIdx.x / cpg;
      pm = mean[gi];
      pr = rstd[gi];
    }
  };
  if (blockIdx.x < ntiles) fetch(blockIdx.x);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t m0 = tile * BM64;
    if (threadIdx.x < K64) {
      const int c = threadIdx.x;
      const float sc = pr * sPar[NOUT + c];
      ssc[c] = sc;
      ssh[c] = sPar[NOUT + K64 + c] - pm * sc;
    }
    __syncthreads();                  // ssc ready; the previous tile's MFMA / epilogue reads are done
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = threadIdx.x + k * NT4, r = c >> 3, ch = c & 7;
      bf16* ev = reinterpret_cast<bf16*>(&u[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ev[j] = f2bf(fmaxf(fmaf(bf2f(ev[j]), ssc[ch * 8 + j], ssh[ch * 8 + j]), 0.f));
      st16(&sX[r * LDX64 + ch * 8], u[k]);
    }
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);
    __syncthreads();
    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s16x8 xf[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) xf[j] = *reinterpret_cast<const s16x8*>(&sX[(16 * j + r16) * LDX64 + ks * 32 + 8 * q]);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(wf[i][ks], xf[j], acc[i][j]);
    }
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
        *reinterpret_cast<f32x4*>(&st[(16 * j + r16) * SLD + wn + 16 * i + 4 * q]) = acc[i][j];
    __syncthreads();
    const uint32_t hin = e.cvt_hin, win = e.cvt_win, cout = e.cvt_cout;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * NT4, r = i / CH, c = (i % CH) * 8;
      const int64_t m = m0 + r;
      if (m >= M) continue;
      float v[8];
      *reinterpret_cast<f32x4*>(&v[0]) = *reinterpret_cast<const f32x4*>(&st[r * SLD + c]);
      *reinterpret_cast<f32x4*>(&v[4]) = *reinterpret_cast<const f32x4*>(&st[r * SLD + c + 4]);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += sbias[c + j];
      // ConvTranspose scatter, 32-bit index math (m < 2^31, host-checked): kk = 2
      const uint32_t mu = (uint32_t)m, mw = mu / win, x = mu - mw * win;
      const uint32_t sl = mw / hin, y = mw - sl * hin;
      const uint32_t ky = (uint32_t)c / (2 * cout), rem = (uint32_t)c - ky * 2 * cout;
      const uint32_t kx = rem / cout, co = rem - kx * cout;
      const int64_t orow = ((int64_t)(sl * hin + y) * 2 + ky) * (2 * win) + x * 2 + kx;
      st_out(e, orow * cout + co, pack8(v));
    }
  }
}

PEpi make_pepi(const CatsegRowsEpi* p) {
  PEpi e;
  e.bias = p->bias;
  e.add = (const bf16*)p->add; e.ld_add = p->ld_add; e.add_ncols = (int)p->add_ncols;
  e.addmap = RowMap{p->addmap.d1, p->addmap.m1, p->addmap.s1, p->addmap.d2, p->addmap.m2, p->addmap.s2, p->addmap.off};
  e.res = (const bf16*)p->res; e.ld_res = p->ld_res; e.res2 = (const bf16*)p->res2; e.ld_res2 = p->ld_res2;
  e.out = (bf16*)p->out; e.ldo = p->ldo;
  e.cvt_k = p->cvt_k; e.cvt_hin = p->cvt_hin; e.cvt_win = p->cvt_win; e.cvt_cout = p->cvt_cout;
  e.wt = 0;
  return e;
}

int g_rows_store = 0;   // output stores of the persistent row kernels: 0 = plain, 1 = sc1 write-through (A/B knob; same box, whole step 9.249 vs 9.249 ms: neutral)
CATSEG_KNOB(g_rows_store, "rows_store");
// e with the write-through flag of the rows_store knob, for an output spanning `out_elems` bf16
PEpi with_wt(PEpi e, int64_t out_elems) {
  e.wt = g_rows_store && out_elems * 2 < 0x7fffffffLL;
  return e;
}

unsigned persist_grid(int64_t M, int per_cu = 1) {
  const int cus = catseg_device_cus();
  const int64_t tiles = (M + BM - 1) / BM;
  return (unsigned)std::min<int64_t>(tiles, (int64_t)cus * per_cu);
}

template <int NOUT, bool ADD, bool RES, bool SCATTER>
void launch_pgemm(const void* x, int64_t ld_x, int64_t M, const float* g, const float* b, float eps, const void* w,
                  const PEpi& e, hipStream_t st) {
  // NOUT=128 variants fit 3 workgroups per CU (<= 96 VGPRs, 25 KB LDS): more rows in flight
  hipLaunchKernelGGL((pgemm_kernel<NOUT, ADD, RES, SCATTER>), dim3(persist_grid(M, NOUT == 128 ? 3 : 1)), dim3(NT), 0, st,
                     (const bf16*)x, ld_x, M, g, b, eps, (const bf16*)w,
                     with_wt(e, SCATTER ? M * e.cvt_k * e.cvt_k * e.cvt_cout : M * e.ldo));
}

}  // namespace

// bf16 fast paths used by catseg_rows_gemm / catseg_rows_mlp (rowblock.hip) when the
// shapes and epilogue fit; return 1 if not applicable (the caller then uses the tiled kernels).
int catseg_rows_gemm_persistent(const void* x, int64_t ld_x, int64_t M, const float* g, const float* b, float eps,
                                const void* w, int64_t N, const CatsegRowsEpi* epi, hipStream_t st) {
  if (!epi->bias || epi->act != 0 || epi->res2) return 1;
  const bool add = epi->add != nullptr, res = epi->res != nullptr, sc = epi->store_mode == 1;
  const PEpi e = make_pepi(epi);
  if (N == 384 && add && !res && !sc) launch_pgemm<384, true, false, false>(x, ld_x, M, g, b, eps, w, e, st);
  else if (N == 384 && !add && !res && sc) launch_pgemm<384, false, false, true>(x, ld_x, M, g, b, eps, w, e, st);
  else if (N == 384 && !add && !res && !sc) launch_pgemm<384, false, false, false>(x, ld_x, M, g, b, eps, w, e, st);
  else if (N == 128 && !add && res && !sc) launch_pgemm<128, false, true, false>(x, ld_x, M, g, b, eps, w, e, st);
  else if (N == 128 && !add && !res && !sc) launch_pgemm<128, false, false, false>(x, ld_x, M, g, b, eps, w, e, st);
  else return 1;
  return 0;
}

extern "C" int catseg_convt64_gn(const void* x, int64_t M, int64_t HW, const float* mean, const float* rstd,
                                 const float* gamma, const float* beta, int cpg, const void* w, int64_t N,
                                 const CatsegRowsEpi* epi, void* stream) {
  CATSEG_CHECK(x && w && epi && epi->out && epi->bias && mean && rstd && gamma && beta, "convt64_gn: null pointer");
  CATSEG_CHECK(M > 0 && HW > 0 && HW % BM64 == 0 && M % HW == 0, "convt64_gn: rows must tile slices of HW % 64 == 0");
  CATSEG_CHECK(cpg > 0 && K64 % cpg == 0, "convt64_gn: bad GroupNorm grouping");
  CATSEG_CHECK(epi->store_mode == 1 && epi->cvt_cout % 8 == 0 && N == (int64_t)epi->cvt_k * epi->cvt_k * epi->cvt_cout,
               "convt64_gn: needs the ConvTranspose scatter store");
  CATSEG_CHECK(N == 192 && epi->cvt_k == 2, "convt64_gn: N = 192 (k=2, 48 channels) only");
  CATSEG_CHECK(M < (1LL << 31), "convt64_gn: row count must fit 31 bits");
  const PEpi e = make_pepi(epi);
  hipLaunchKernelGGL((pconvt64_kernel<192>), dim3(persist_grid((M + 1) / 2, 2)), dim3(NT4), 0, (hipStream_t)stream,
                     (const bf16*)x, M, HW, mean, rstd, gamma, beta, cpg, (const bf16*)w, with_wt(e, M * 192));
  return catseg_launch_status("convt64_gn");
}

int g_mlp_variant = 0;   // 0 = barrier-lean pmlp2_kernel (default), 1 = pmlp_kernel (A/B; bit-identical)
CATSEG_KNOB(g_mlp_variant, "mlp_variant");
int g_gelu_form = 1;     // GELU of pmlp2_kernel: 0 = gelu_seg (9 VALU), 1 = gelu_x7 (7 VALU; same box, whole step 9.675 -> 9.608 ms)
CATSEG_KNOB(g_gelu_form, "gelu_form");

int rows_mlp_persistent(const bf16* Yb, int64_t ld_y, int64_t M, const float* g, const float* b, float eps,
                        const bf16* w1, const float* b1, int act, const bf16* w2, const PEpi& e0, bool res2,
                        hipStream_t st) {
  const dim3 grid(persist_grid(M)), blk(NT);
  const PEpi e = with_wt(e0, M * e0.ldo);
  if (g_mlp_variant == 0) {
    if (act == ACT_GELU && g_gelu_form == 1 && !res2)
      hipLaunchKernelGGL((pmlp2_kernel<ACT_GELU7, false, false>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
    else if (act == ACT_GELU && g_gelu_form == 1 && res2)
      hipLaunchKernelGGL((pmlp2_kernel<ACT_GELU7, true, false>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
    else if (act == ACT_GELU && !res2)
      hipLaunchKernelGGL((pmlp2_kernel<ACT_GELU, false, false>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
    else if (act == ACT_RELU && res2)
      hipLaunchKernelGGL((pmlp2_kernel<ACT_RELU, true, false>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
    else if (act == ACT_RELU && !res2)
      hipLaunchKernelGGL((pmlp2_kernel<ACT_RELU, false, false>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
    else if (act == ACT_GELU && res2)
      hipLaunchKernelGGL((pmlp2_kernel<ACT_GELU, true, false>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
    else return 1;
    return 0;
  }
  if (act == ACT_GELU && !res2)
    hipLaunchKernelGGL((pmlp_kernel<ACT_GELU, false, false, true>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
  else if (act == ACT_RELU && res2)
    hipLaunchKernelGGL((pmlp_kernel<ACT_RELU, true, false, true>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
  else if (act == ACT_RELU && !res2)
    hipLaunchKernelGGL((pmlp_kernel<ACT_RELU, false, false, true>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
  else if (act == ACT_GELU && res2)
    hipLaunchKernelGGL((pmlp_kernel<ACT_GELU, true, false, true>), grid, blk, 0, st, Yb, ld_y, M, g, b, eps, w1, b1, w2, e);
  else return 1;
  return 0;
}

int catseg_rows_mlp_persistent(const void* y, int64_t ld_y, int64_t M, const float* g, const float* b, float eps,
                               const void* w1, const float* b1, int64_t hidden, int act, const void* w2,
                               const CatsegRowsEpi* epi, hipStream_t st) {
  // residual must be the input rows themselves (both reference MLPs: model.py:223, :413)
  if (hidden != HID || !epi->bias || epi->res != y || epi->ld_res != ld_y || epi->add || epi->store_mode) return 1;
  const PEpi e = make_pepi(epi);
  const bool r2 = epi->res2 != nullptr;
  return rows_mlp_persistent((const bf16*)y, ld_y, M, g, b, eps, (const bf16*)w1, b1, act, (const bf16*)w2, e, r2, st);
}

extern "C" int catseg_swin_proj_mlp(const void* attn, int64_t ld_attn, const void* x, int64_t ld_x, int64_t M,
                                    const void* w_proj, const float* b_proj, const float* ln_gamma,
                                    const float* ln_beta, float eps, const void* w1, const float* b1, int64_t hidden,
                                    const void* w2, const float* b2, void* out, int64_t ld_out, void* stream) {
  CATSEG_CHECK(attn && x && w_proj && b_proj && ln_gamma && ln_beta && w1 && b1 && w2 && b2 && out,
               "swin_proj_mlp: null pointer");
  CATSEG_CHECK(M > 0 && hidden == HID, "swin_proj_mlp: hidden must be 512");
  CATSEG_CHECK(ld_attn % 8 == 0 && ld_x % 8 == 0 && ld_out % 8 == 0 && ((uintptr_t)attn % 16) == 0 &&
                   ((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 16) == 0,
               "swin_proj_mlp: 16-byte aligned rows");
  CATSEG_CHECK(out == x ? ld_out == ld_x : true, "swin_proj_mlp: in place needs ld_out == ld_x");
  PEpi e{};
  e.bias = b2; e.out = (bf16*)out; e.ldo = ld_out;
  e = with_wt(e, M * ld_out);
  if (g_mlp_variant == 0 && g_gelu_form == 1)
    hipLaunchKernelGGL((pmlp2_kernel<ACT_GELU7, false, true>), dim3(persist_grid(M)), dim3(NT), 0, (hipStream_t)stream,
                       (const bf16*)attn, ld_attn, M, ln_gamma, ln_beta, eps, (const bf16*)w1, b1, (const bf16*)w2, e,
                       (const bf16*)x, ld_x, (const bf16*)w_proj, b_proj);
  else if (g_mlp_variant == 0)
    hipLaunchKernelGGL((pmlp2_kernel<ACT_GELU, false, true>), dim3(persist_grid(M)), dim3(NT), 0, (hipStream_t)stream,
                       (const bf16*)attn, ld_attn, M, ln_gamma, ln_beta, eps, (const bf16*)w1, b1, (const bf16*)w2, e,
                       (const bf16*)x, ld_x, (const bf16*)w_proj, b_proj);
  else
    hipLaunchKernelGGL((pmlp_kernel<ACT_GELU, false, true, true>), dim3(persist_grid(M)), dim3(NT), 0, (hipStream_t)stream,
                       (const bf16*)attn, ld_attn, M, ln_gamma, ln_beta, eps, (const bf16*)w1, b1, (const bf16*)w2, e,
                       (const bf16*)x, ld_x, (const bf16*)w_proj, b_proj);
  return catseg_launch_status("swin_proj_mlp");
}
