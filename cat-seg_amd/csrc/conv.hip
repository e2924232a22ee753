// 3x3 / pad 1 convolution over NHWC as an MFMA implicit GEMM (gfx950), plus the
// GroupNorm statistics / apply kernels and the 1-channel head conv of the guided
// upsampler (reference cat_seg/modeling/transformer/model.py:520-555,616,627,634).
//
// GEMM view: D[co][m] = sum_k Wt[co][k] * A[m][k], m = (slice, y, x), k = (ky, kx, ci).
// The A loader gathers 16-byte channel chunks of the 3x3 neighbourhood straight from
// the NHWC sources (zero outside the image), reading channels [0, c1) from the per-
// slice tensor and [c1, c1+c2) from the per-image guidance tensor, so the channel
// concatenation of Up.forward (model.py:551-554) and its repeat over classes are
// never materialised.  An optional GroupNorm+ReLU prologue normalises src1 on load
// (DoubleConv's second conv consumes relu(GN(conv1))).  The epilogue adds bias,
// applies the activation and, for GroupNorm consumers, emits per-(tile, group)
// mean/M2 partials that catseg_groupnorm_stats combines deterministically.
#include "common.h"
#include "capi.h"

namespace {

constexpr int BK = 32, NT = 256, BM = 128;

struct ConvP {
  const void* s1; int64_t s1_ss, s1_off; int c1;
  const void* s2; int64_t s2_ss, s2_off; int c2; int64_t s2_div;
  int64_t S; int H, W;
  const void* w; int cout;
  const float* bias; int act;
  const float* gmean; const float* grstd; const float* ggamma; const float* gbeta; int gcpg;
  void* out; float* stats; int scpg;
  const float* add; int64_t add_ss, add_div;
  float* ws; int ksplit;       // split-K: fp32 partials [ksplit][M][cout], reduced by conv_splitk_reduce
};

// GroupNorm + ReLU on a loaded chunk with the block's per-channel scale/shift (LDS):
// relu(x * rstd*gamma + (beta - mean*rstd*gamma)).  A conv tile never spans two slices
// when GN is on (host-checked H*W % BM == 0), so one table per block suffices.
template <typename T>
DEV uint4 gn_chunk(uint4 u, const float* gsc, const float* gsh, int ci) {
  constexpr int VN = Vec16<T>::N;
  T* e = reinterpret_cast<T*>(&u);
#pragma unroll
  for (int j = 0; j < VN; ++j) e[j] = from_f<T>(fmaxf(fmaf(to_f<T>(e[j]), gsc[ci + j], gsh[ci + j]), 0.f));
  return u;
}

template <typename T, int BN>
__global__ __launch_bounds__(NT) void conv3x3_kernel(ConvP p) {
  constexpr int VN = Vec16<T>::N;
  constexpr int CPR = BK / VN;
  // bf16 tiles: unpadded 64-byte rows, 16-byte chunk ch of row r stored at slot ch ^ g[(r >> 2) & 3]
  // with g = {0, 2, 3, 1}: the 16 (row, chunk) pairs of every ds_read_b128 lane group of a fragment
  // read land in 16 distinct bank slots, and each ds_write_b128 group of the staging store writes
  // two whole rows (was: +8-element pad, 2-way conflicts on both, ~50 % SQ_LDS_BANK_CONFLICT)
  constexpr int LDR = BK + (sizeof(T) == 2 ? 0 : 4);
  static_assert(sizeof(T) != 2 || BK == 32, "bf16 swizzle assumes 4 chunks per row");
  auto soff = [](int row, int col) {       // element offset of (row, col), col a multiple of VN
    if constexpr (sizeof(T) == 2) return row * LDR + ((((col >> 3) ^ (0x1320 >> (4 * ((row >> 2) & 3)))) & 3) << 3);
    else return row * LDR + col;
  };
  constexpr int A_CH = BM * CPR / NT;
  constexpr int W_TOT = BN * CPR, W_CH = (W_TOT + NT - 1) / NT;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  __shared__ __attribute__((aligned(16))) T sA[2][BM * LDR];
  __shared__ __attribute__((aligned(16))) T sW[2][BN * LDR];
  __shared__ float red[4][8];
  __shared__ float gsc[128], gsh[128];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t HW = (int64_t)p.H * p.W;
  const int64_t M = p.S * HW;
  const int cin = p.c1 + p.c2;
  const int64_t K = 9LL * cin;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int wm = (wave & 1) * WM, wn = (wave >> 1) * WN;

  int a_lrow[A_CH], a_col[A_CH], a_y[A_CH], a_x[A_CH];
  int64_t a_s[A_CH]; bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    int c = tid + i * NT;
    a_lrow[i] = c / CPR; a_col[i] = (c % CPR) * VN;
    int64_t m = m0 + a_lrow[i];
    a_ok[i] = m < M;
    int64_t mm = a_ok[i] ? m : 0;
    a_s[i] = mm / HW;
    int pix = (int)(mm % HW);
    a_y[i] = pix / p.W; a_x[i] = pix % p.W;
  }
  const T* S1 = reinterpret_cast<const T*>(p.s1);
  const T* S2 = reinterpret_cast<const T*>(p.s2);
  const T* Wt = reinterpret_cast<const T*>(p.w);

  // gload issues every chunk's load unconditionally (out-of-image / past-K / past-cout chunks read
  // a clamped in-bounds address) and records what sstore must do with it (zero it, or apply the
  // GroupNorm prologue): a load inside a per-lane branch, or a GroupNorm applied right after it,
  // made the compiler retire each load before issuing the next (s_waitcnt vmcnt(0) between them),
  // so a K-step paid two or three serial memory latencies.  Same values reach LDS as before.
  uint4 ra[A_CH], rw[W_CH];
  bool a_zero[A_CH], w_zero[W_CH];
  int a_gci[A_CH];                      // >= 0: GroupNorm+ReLU on load, channel base
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int64_t k = k0 + a_col[i];
      const int64_t kc = k < K ? k : K - VN;
      const int tap = (int)(kc / cin), ci = (int)(kc % cin);
      const int yy = a_y[i] + tap / 3 - 1, xx = a_x[i] + tap % 3 - 1;
      const bool inside = yy >= 0 && yy < p.H && xx >= 0 && xx < p.W;
      a_zero[i] = !(a_ok[i] && k < K && inside);
      const int64_t pix = (int64_t)min(max(yy, 0), p.H - 1) * p.W + min(max(xx, 0), p.W - 1);
      const bool first = ci < p.c1;
      const T* base = first ? S1 : S2;   // S2 is only selected when c2 > 0 (then it is set)
      const int64_t off = first ? a_s[i] * p.s1_ss + p.s1_off + pix * p.c1 + ci
                                : (a_s[i] / p.s2_div) * p.s2_ss + p.s2_off + pix * p.c2 + (ci - p.c1);
      const T* src = base + off;
      a_gci[i] = (first && p.gmean) ? ci : -1;
      ra[i] = ld16(src);
    }
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int c = min(tid + i * NT, W_TOT - 1);
      const int n = n0 + c / CPR;
      const int64_t k = k0 + (c % CPR) * VN;
      w_zero[i] = !(n < p.cout && k < K);
      rw[i] = ld16(Wt + (int64_t)min(n, p.cout - 1) * K + (k < K ? k : K - VN));
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      uint4 u = ra[i];
      if (a_zero[i]) u = make_uint4(0, 0, 0, 0);
      else if (a_gci[i] >= 0) u = gn_chunk<T>(u, gsc, gsh, a_gci[i]);
      st16(&sA[buf][soff(a_lrow[i], a_col[i])], u);
    }
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int c = tid + i * NT;
      if (c < W_TOT) st16(&sW[buf][soff(c / CPR, (c % CPR) * VN)], w_zero[i] ? make_uint4(0, 0, 0, 0) : rw[i]);
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ktiles_all = (int)((K + BK - 1) / BK);
  const int kper = (ktiles_all + p.ksplit - 1) / p.ksplit;
  const int kt0 = blockIdx.z * kper;
  const int ktiles = max(0, min(ktiles_all - kt0, kper));
  if (p.gmean) {
    const int64_t s0 = (m0 < M ? m0 : 0) / HW;
    const int ngroups = p.c1 / p.gcpg;
    for (int c = tid; c < p.c1; c += NT) {
      const float rs = p.grstd[s0 * ngroups + c / p.gcpg], mu = p.gmean[s0 * ngroups + c / p.gcpg];
      const float sc = rs * p.ggamma[c];
      gsc[c] = sc;
      gsh[c] = p.gbeta[c] - mu * sc;
    }
    __syncthreads();
  }
  gload((int64_t)kt0 * BK);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < ktiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ktiles) gload((int64_t)(kt0 + kt + 1) * BK);
    const T* As = sA[buf];
    const T* Ws = sW[buf];
    if constexpr (sizeof(T) == 2) {
      const int r = lane & 15, kc = (lane >> 4) * 8;
      s16x8 bfrag[FM];
#pragma unroll
      for (int j = 0; j < FM; ++j) bfrag[j] = *reinterpret_cast<const s16x8*>(&As[soff(wm + 16 * j + r, kc)]);
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        s16x8 afrag = *reinterpret_cast<const s16x8*>(&Ws[soff(wn + 16 * i + r, kc)]);
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma_bf16(afrag, bfrag[j], acc[i][j]);
      }
    } else {
      const int r = lane & 15, kq = lane >> 4;
#pragma unroll
      for (int s = 0; s < BK / 4; ++s) {
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
    if (kt + 1 < ktiles) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: bias, act, store, GroupNorm partials ----
  const int col = lane & 15, rq = (lane >> 4) * 4;
  if (p.ksplit > 1) {          // raw fp32 partial of this K slice (bias / act in the reduce)
    float* Wp = p.ws + (int64_t)blockIdx.z * M * p.cout;
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = n0 + wn + 16 * i + rq;
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int64_t m = m0 + wm + 16 * j + col;
        if (m < M && n < p.cout) {
          const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          store4<float>(Wp + m * p.cout + n, v);
        }
      }
    }
    return;
  }
  T* O = reinterpret_cast<T*>(p.out);
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn + 16 * i + rq;
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int64_t m = m0 + wm + 16 * j + col;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[i][j][r] + ((p.bias && n + r < p.cout) ? p.bias[n + r] : 0.f);
        if (p.add && m < M && n + r < p.cout)
          v += p.add[(m / HW / p.add_div) * p.add_ss + (m % HW) * p.cout + n + r];
        acc[i][j][r] = apply_act(v, p.act);
      }
      if (m < M && n < p.cout) {
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        store4<T>(O + m * p.cout + n, v);
      }
    }
  }
  if (p.stats) {
    // tile = BM rows of ONE slice (host checks HW % BM == 0), columns = all groups
    // (host checks BN >= cout, scpg == 16).  Two passes: tile mean, then M2.
    const int64_t s = m0 / HW;
    const int tile = (int)((m0 % HW) / BM);
    const int ntiles = (int)(HW / BM);
    const int ngroups = p.cout / p.scpg;
    float gsum[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) a += acc[i][j][r];
      gsum[i] = warp_sum(a);
    }
    // each wave covers groups (wn/16 + i) over its WM rows; combine the two row-halves
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < FN; ++i) red[wave][i] = gsum[i];
    __syncthreads();
    float gmean[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int wpair = wave ^ 1;   // same wn, other wm
      gmean[i] = (red[wave][i] + red[wpair][i]) / (float)(BM * 16);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[i][j][r] - gmean[i];
          a += d * d;
        }
      gsum[i] = warp_sum(a);
    }
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < FN; ++i) red[wave][i] = gsum[i];
    __syncthreads();
    if ((wave & 1) == 0 && lane == 0) {
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int grp = (n0 + wn) / 16 + i;
        if (grp < ngroups) {
          float* o = p.stats + ((s * ntiles + tile) * ngroups + grp) * 2;
          o[0] = gmean[i];
          o[1] = red[wave][i] + red[wave ^ 1][i];
        }
      }
    }
  }
}

// split-K factor for the im2col kernel: grids far below the CU count (the per-image guidance
// projections: 36-144 tiles over K = 9 x 256..768) split K so >= ~512 workgroups run;
// never with GroupNorm statistics (partials are per output tile).  Sized on ONE slice
// (S = 1), never on the batch: the K partition, hence every output bit, must not depend on
// how many images share the launch (batch invariance, the multi-GPU bit-identity gate).
int conv_ksplit(const CatsegConvArgs* a) {
  if (a->stats) return 1;
  const int64_t M = (int64_t)a->H * a->W;
  const int64_t tiles = ((M + BM - 1) / BM) * ((a->c_out + 127) / 128);
  const int64_t ktiles = (9LL * (a->c1 + a->c2) + BK - 1) / BK;
  int ks = 1;
  while (tiles * ks < 512 && ktiles / (2 * ks) >= 8 && ks < 16) ks *= 2;
  return ks;
}

template <typename T>
__global__ void conv_splitk_reduce(const float* ws, int ksplit, int64_t total4, int cout, const float* bias, int act,
                                   const float* add, int64_t add_ss, int64_t add_div, int64_t HW, T* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    float4 a = *reinterpret_cast<const float4*>(ws + e);
    for (int z = 1; z < ksplit; ++z) {
      const float4 b = *reinterpret_cast<const float4*>(ws + (int64_t)z * total4 * 4 + e);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float v[4] = {a.x, a.y, a.z, a.w};
    const int n = (int)(e % cout);
    const int64_t m = e / cout;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (bias) v[r] += bias[n + r];
      if (add) v[r] += add[(m / HW / add_div) * add_ss + (m % HW) * cout + n + r];
      v[r] = apply_act(v[r], act);
    }
    store4<T>(out + e, v);
  }
}

template <typename T>
int launch_conv(const ConvP& p, hipStream_t st) {
  const int64_t M = p.S * p.H * p.W;
  const unsigned gx = (unsigned)((M + BM - 1) / BM);
  const unsigned gz = (unsigned)p.ksplit;
  if (p.cout <= 32) {
    hipLaunchKernelGGL((conv3x3_kernel<T, 32>), dim3(gx, 1, gz), dim3(NT), 0, st, p);
  } else if (p.cout <= 64) {
    hipLaunchKernelGGL((conv3x3_kernel<T, 64>), dim3(gx, 1, gz), dim3(NT), 0, st, p);
  } else {
    hipLaunchKernelGGL((conv3x3_kernel<T, 128>), dim3(gx, (unsigned)((p.cout + 127) / 128), gz), dim3(NT), 0, st, p);
  }
  if (p.ksplit > 1) {
    const int64_t total4 = M * p.cout / 4;
    const unsigned grid = (unsigned)std::min<int64_t>((total4 + 255) / 256, 4096);
    hipLaunchKernelGGL(conv_splitk_reduce<T>, dim3(grid), dim3(256), 0, st, p.ws, p.ksplit, total4, p.cout, p.bias,
                       p.act, p.add, p.add_ss, p.add_div, (int64_t)p.H * p.W, reinterpret_cast<T*>(p.out));
  }
  return 0;
}

// ---------------- GroupNorm stats combine (Chan et al. pairwise, fixed order) ----
// One wave per (slice, group).  Every partial covers the same tile_n values, so the
// combined mean is the mean of the tile means and M2 = sum M2_t + tile_n * sum (mean_t -
// mean)^2 (exact two-pass form); lane sums reduce in a fixed butterfly order (deterministic).
DEV double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void gn_stats_kernel(const float* part, int64_t S, int tiles, int groups,
                                                       float tile_n, float eps, float* mean, float* rstd) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= S * groups) return;
  const int64_t s = i / groups;
  const int g = (int)(i % groups);
  const float* q = part + (s * tiles * groups + g) * 2;
  double sm = 0;
  for (int t = lane; t < tiles; t += 64) sm += q[(int64_t)t * groups * 2];
  const double mu = wave_sum_f64(sm) / tiles;
  double sd = 0, s2 = 0;
  for (int t = lane; t < tiles; t += 64) {
    const double d = q[(int64_t)t * groups * 2] - mu;
    sd += d * d;
    s2 += q[(int64_t)t * groups * 2 + 1];
  }
  const double m2 = wave_sum_f64(s2) + (double)tile_n * wave_sum_f64(sd);
  if (lane == 0) {
    mean[i] = (float)mu;
    rstd[i] = (float)(1.0 / sqrt(m2 / ((double)tile_n * tiles) + (double)eps));
  }
}

template <typename T>
__global__ void gn_relu_kernel(const T* x, T* y, int64_t total4, int C, int cpg, int64_t HW,
                               const float* mean, const float* rstd, const float* gamma, const float* beta) {
  const int groups = C / cpg;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    const int c = (int)(e % C);
    const int64_t s = e / ((int64_t)C * HW);
    const int g = c / cpg;
    const float mu = mean[s * groups + g], rs = rstd[s * groups + g];
    float v[4];
    load4<T>(x + e, v);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf((v[r] - mu) * rs * gamma[c + r] + beta[c + r], 0.f);
    store4<T>(y + e, v);
  }
}

// ---------------- head conv3x3 C -> 1 (+bias), GN+ReLU applied on load -----------
template <typename T>
__global__ void head_kernel(const T* x, int64_t B, int Tn, int H, int W, int C, const float* w, float bias,
                            const float* mean, const float* rstd, const float* gamma, const float* beta, int cpg,
                            const int32_t* classes, int Tout, float* out) {
  // grid: (pixel blocks, slices).  Per block: weights [9][C] and the slice's GroupNorm
  // scale/shift per channel in LDS; one output pixel per thread, 16-byte channel loads.
  extern __shared__ float sw[];   // [9][C] weights | scale[C] | shift[C]
  float* ssc = sw + 9 * C;
  float* ssh = ssc + C;
  const int64_t s = blockIdx.y;
  const int groups = C / cpg;
  for (int i = threadIdx.x; i < 9 * C; i += blockDim.x) sw[i] = w[i];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    if (mean) {
      const float sc = rstd[s * groups + c / cpg] * gamma[c];
      ssc[c] = sc;
      ssh[c] = beta[c] - mean[s * groups + c / cpg] * sc;
    } else {
      ssc[c] = 1.f;
      ssh[c] = 0.f;
    }
  }
  __syncthreads();
  const int HW = H * W;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= HW) return;
  const int y = pix / W, xx = pix % W;
  const bool relu = mean != nullptr;
  float acc = bias;
  for (int tap = 0; tap < 9; ++tap) {
    const int yy = y + tap / 3 - 1, x2 = xx + tap % 3 - 1;
    if (yy < 0 || yy >= H || x2 < 0 || x2 >= W) continue;
    const T* src = x + (s * HW + (int64_t)yy * W + x2) * C;
    const float* wt = sw + tap * C;
    for (int c = 0; c < C; c += 8) {
      float v[8];
      load4<T>(src + c, v);
      load4<T>(src + c + 4, v + 4);
      // weights / GroupNorm terms as 16-byte LDS broadcasts (a ds_read_b32 per element and term was
      // the fp32 head's limit: 3 LDS reads per multiply-add)
      const float4 w0 = *reinterpret_cast<const float4*>(wt + c), w1 = *reinterpret_cast<const float4*>(wt + c + 4);
      const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      if (relu) {
        const float4 a0 = *reinterpret_cast<const float4*>(ssc + c), a1 = *reinterpret_cast<const float4*>(ssc + c + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(ssh + c), b1 = *reinterpret_cast<const float4*>(ssh + c + 4);
        const float aa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int r = 0; r < 8; ++r) acc = fmaf(fmaxf(fmaf(v[r], aa[r], bb[r]), 0.f), ww[r], acc);
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) acc = fmaf(v[r], ww[r], acc);   // no GroupNorm: scale 1, shift 0
      }
    }
  }
  const int64_t b = s / Tn;
  const int t = (int)(s % Tn);
  const int cls = classes ? classes[b * Tn + t] : t;
  out[(b * Tout + cls) * (int64_t)HW + pix] = acc;
}

// ---------------- head conv C -> 1, fp32 input: C/4 lanes per pixel ---------------------
// The fp32 (training / config 2) head: lane l of a pixel's LPP = C/4 lanes loads channels 4l..4l+3 of
// each tap, so one load instruction covers LPP-lane groups of whole 128-byte pixel rows (the
// one-pixel-per-thread form touched 64 lines per instruction, 16 bytes each); the LPP partial sums
// meet by xor shuffles.  GroupNorm + ReLU on load as head_kernel.
template <int LPP>
__global__ __launch_bounds__(256) void head_vec_kernel(const float* __restrict__ x, int Tn, int H, int W,
                                                       const float* __restrict__ w, float bias,
                                                       const float* mean, const float* rstd, const float* gamma,
                                                       const float* beta, int cpg, const int32_t* classes, int Tout,
                                                       float* __restrict__ out) {
  constexpr int C = 4 * LPP, PPB = 256 / LPP;              // pixels per block pass
  const int64_t s = blockIdx.y;
  const int l = threadIdx.x % LPP, pl = threadIdx.x / LPP;
  const int c = 4 * l;
  float4 wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wv[t] = *reinterpret_cast<const float4*>(w + t * C + c);
  float sc[4] = {1.f, 1.f, 1.f, 1.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
  const bool gn = mean != nullptr;
  if (gn) {
    const int groups = C / cpg;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a = rstd[s * groups + (c + r) / cpg] * gamma[c + r];
      sc[r] = a;
      sh[r] = beta[c + r] - mean[s * groups + (c + r) / cpg] * a;
    }
  }
  const int HW = H * W;
  const int64_t b = s / Tn;
  const int t0 = (int)(s % Tn);
  const int cls = classes ? classes[b * Tn + t0] : t0;
  float* o = out + (b * Tout + cls) * (int64_t)HW;
  const float* xs = x + s * (int64_t)HW * C + c;
  for (int pix = blockIdx.x * PPB + pl; pix < HW; pix += gridDim.x * PPB) {
    const int y = pix / W, xx = pix - y * W;
    float acc = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int yy = y + tap / 3 - 1, x2 = xx + tap % 3 - 1;
      if (yy < 0 || yy >= H || x2 < 0 || x2 >= W) continue;
      const float4 v = *reinterpret_cast<const float4*>(xs + ((int64_t)yy * W + x2) * C);
      const float vv[4] = {v.x, v.y, v.z, v.w}, ww[4] = {wv[tap].x, wv[tap].y, wv[tap].z, wv[tap].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float u = gn ? fmaxf(fmaf(vv[r], sc[r], sh[r]), 0.f) : vv[r];
        acc = fmaf(u, ww[r], acc);
      }
    }
#pragma unroll
    for (int off = LPP / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (l == 0) o[pix] = acc + bias;
  }
}

// ---------------- head conv, banded (bf16 input) ---------------------------------------
// One workgroup = BR output rows of one slice.  The BR + 2 input rows (+ zero halo) are
// staged ONCE into LDS with GroupNorm+ReLU applied in fp32 and stored as fp16 (10-bit
// mantissa: the head's 288-term dot product then carries ~4x less input rounding than a
// bf16 stage would), pixel stride C + 8 halves (conflict-free 16-byte reads across
// consecutive pixels); the weights sit in LDS as fp16 pairs (broadcast reads).  Each
// output is 9 x C/2 v_dot2c_f32_f16 (fp32 accumulate).  Replaces the per-tap global
// gathers of head_kernel (every input element was re-read and re-normalised 9 times).
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
constexpr int HBR = 8;            // output rows per workgroup

// WC != 0: the map width is compile-time (96 at both CAT-Seg geometries), so the staging loop's
// per-chunk (row, column) split and the output loop's are multiplies, not integer divisions.
template <int C, int WC = 0>
__global__ __launch_bounds__(256) void head_band_kernel(const bf16* __restrict__ x, int Tn, int H, int W_,
                                                        const float* __restrict__ w, float bias, const float* mean,
                                                        const float* rstd, const float* gamma, const float* beta,
                                                        int cpg, const int32_t* classes, int Tout, float* out) {
  constexpr int CPX = C / 8, CP = C + 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* wl = reinterpret_cast<_Float16*>(smem);                    // [9][C]
  float* ssc = reinterpret_cast<float*>(smem + 9 * C * 2);              // [C]
  float* ssh = ssc + C;                                                 // [C]
  _Float16* tile = reinterpret_cast<_Float16*>(smem + 9 * C * 2 + 2 * C * 4);   // [HBR+2][W+2][CP]
  const int64_t s = blockIdx.y;
  const int y0 = blockIdx.x * HBR;
  const int rows = min(HBR, H - y0);
  const int W = WC ? WC : W_;
  const int WP = W + 2;
  const int tid = threadIdx.x;
  for (int i = tid; i < 9 * C; i += 256) wl[i] = (_Float16)w[i];
  const int groups = C / cpg;
  for (int c = tid; c < C; c += 256) {
    if (mean) {
      const float sc = rstd[s * groups + c / cpg] * gamma[c];
      ssc[c] = sc;
      ssh[c] = beta[c] - mean[s * groups + c / cpg] * sc;
    } else {
      ssc[c] = 1.f;
      ssh[c] = 0.f;
    }
  }
  __syncthreads();
  const bool relu = mean != nullptr;
  const int64_t HW = (int64_t)H * W;
  const bf16* xs = x + s * HW * C;
  const int total = (rows + 2) * WP * CPX;
  // all of the band's loads in flight at once (<= 16 per thread for W <= 100): one memory
  // round trip per workgroup instead of one per 4 loads (two workgroups per CU by LDS)
  constexpr int NL = 16;
  for (int i0 = 0; i0 < total; i0 += 256 * NL) {
    uint4 u[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = i0 + j * 256 + tid;
      const int ch = i % CPX, pos = i / CPX, r = pos / WP, xc = pos - r * WP;
      const int yy = y0 - 1 + r, xx = xc - 1;
      u[j] = (i < total && yy >= 0 && yy < H && xx >= 0 && xx < W) ? ld16(xs + ((int64_t)yy * W + xx) * C + ch * 8)
                                                                   : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = i0 + j * 256 + tid;
      if (i >= total) continue;
      const int ch = i % CPX, pos = i / CPX, r = pos / WP, xc = pos - r * WP;
      const int yy = y0 - 1 + r, xx = xc - 1;
      const bool inside = yy >= 0 && yy < H && xx >= 0 && xx < W;
      const bf16* e = reinterpret_cast<const bf16*>(&u[j]);
      _Float16 hv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = fmaf(bf2f(e[k]), ssc[ch * 8 + k], ssh[ch * 8 + k]);
        if (relu) v = fmaxf(v, 0.f);
        hv[k] = (_Float16)(inside ? v : 0.f);
      }
      st16(&tile[pos * CP + ch * 8], *reinterpret_cast<uint4*>(hv));
    }
  }
  __syncthreads();
  const int b = (int)(s / Tn), t = (int)(s % Tn);
  const int cls = classes ? classes[(int64_t)b * Tn + t] : t;
  float* o = out + ((int64_t)b * Tout + cls) * HW + (int64_t)y0 * W;
  for (int idx = tid; idx < rows * W; idx += 256) {
    const int yy = idx / W, xx = idx - yy * W;
    float acc = bias;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const _Float16* px = &tile[((yy + dy) * WP + xx + dx) * CP];
        const _Float16* wt = &wl[(dy * 3 + dx) * C];
#pragma unroll
        for (int k = 0; k < CPX; ++k) {
          const uint4 a = ld16(px + k * 8), bw = ld16(wt + k * 8);
          const h2* ah = reinterpret_cast<const h2*>(&a);
          const h2* bh = reinterpret_cast<const h2*>(&bw);
#pragma unroll
          for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_fdot2(ah[m], bh[m], acc, false);
        }
      }
    o[idx] = acc;
  }
}

// ---------------- head conv, MFMA tap products (bf16 input, C = 32, W = 96) ---------------
// out[y][x] = bias + sum_{dy,dx} D[y+dy-1][x+dx-1][3 dy + dx],  D[p][tap] = relu(GN(x[p])) . w[tap]:
// one v_mfma_f32_16x16x32_f16 per 16 input pixels computes all 9 tap products of every pixel
// (A = the 16 pixels' 32 channels straight from a 16-byte load per lane, GroupNorm+ReLU applied
// in fp32 and rounded to fp16 as the band kernel does; B = the 9 weight rows, zero columns 9-15),
// and each input element is read ONCE per band (no per-tap re-reads, no fp16 staging image).  A
// workgroup walks the input rows of one band (RB output rows of a slice + 2 halo rows) two rows
// per step; the D rows go to a 6-row LDS ring [row][tap][x] (4 zero columns each side) and the
// output rows whose three D rows are complete are summed there (9 LDS reads per output).  Loads
// of step k+1 are in flight during step k (registers); one barrier per step.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
constexpr int HT_W = 96, HT_TPR = HT_W / 16, HT_NR = 6, HT_WP = HT_W + 8;
constexpr int HT_TPS = 2 * HT_TPR / 4;      // 16-pixel tiles per wave per step (two rows, 4 waves)

// PD: input steps in flight (registers) ahead of the one being computed
template <int PD>
__global__ __launch_bounds__(256) void head_tap_kernel(const bf16* __restrict__ x, int Tn, int H, const float* __restrict__ w,
                                                       float bias, const float* mean, const float* rstd,
                                                       const float* gamma, const float* beta, int cpg,
                                                       const int32_t* classes, int Tout, float* out, int RB,
                                                       int ups, int nunits) {
  constexpr int C = 32;
  __shared__ __attribute__((aligned(16))) float ring[HT_NR][9][HT_WP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  for (int i = tid; i < HT_NR * 9 * HT_WP; i += 256) (&ring[0][0][0])[i] = 0.f;   // pad columns stay zero
  // B operand: W[tap r16][channels 8g .. 8g+7] (taps 9..15 zero)
  h8 wb;
#pragma unroll
  for (int j = 0; j < 8; ++j) wb[j] = r16 < 9 ? (_Float16)w[r16 * C + 8 * g + j] : (_Float16)0.f;
  const int groups = C / cpg;
  const int64_t HW = (int64_t)H * HT_W;
  __syncthreads();
  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    const int s = u / ups, y0 = (u - s * ups) * RB, y1 = min(H, y0 + RB);
    const int nin = y1 - y0 + 2;                     // input rows y0 - 1 .. y1
    const int nsteps = (nin + 1) >> 1;
    // GroupNorm affine of this lane's channels 8g .. 8g+7 (slice s)
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 8 * g + j;
      if (mean) {
        const float a = rstd[(int64_t)s * groups + c / cpg] * gamma[c];
        sc[j] = a;
        sh[j] = beta[c] - mean[(int64_t)s * groups + c / cpg] * a;
      } else {
        sc[j] = 1.f;
        sh[j] = 0.f;
      }
    }
    const bf16* xs = x + (int64_t)s * HW * C;
    // tile j of step k: input row i = 2k + (tile / TPR), pixels 16 (tile % TPR) + r16
    auto load = [&](int k, uint4 (&v)[HT_TPS]) {
#pragma unroll
      for (int j = 0; j < HT_TPS; ++j) {
        const int tile = wave * HT_TPS + j, i = 2 * k + tile / HT_TPR, yy = y0 - 1 + i;
        const int xx = (tile % HT_TPR) * 16 + r16;
        const bool in = i < nin && yy >= 0 && yy < H;
        v[j] = ld16(xs + ((int64_t)(in ? yy : 0) * HT_W + xx) * C + 8 * g);
      }
    };
    uint4 cur[HT_TPS], nxt[HT_TPS], nn[HT_TPS];
    load(0, cur);
    if (PD > 1 && 1 < nsteps) load(1, nxt);
    const int b = s / Tn, t = s - b * Tn;
    const int cls = classes ? classes[(int64_t)b * Tn + t] : t;
    float* o = out + ((int64_t)b * Tout + cls) * HW;
    for (int k = 0; k < nsteps; ++k) {
      if (PD == 1 && k + 1 < nsteps) load(k + 1, nxt);
      if (PD > 1 && k + 2 < nsteps) load(k + 2, nn);
#pragma unroll
      for (int j = 0; j < HT_TPS; ++j) {
        const int tile = wave * HT_TPS + j, i = 2 * k + tile / HT_TPR, yy = y0 - 1 + i;
        const int x0 = (tile % HT_TPR) * 16;
        const bool in = i < nin && yy >= 0 && yy < H;       // wave-uniform
        // GroupNorm affine on bf16 pairs, rounded to f16 pairs (v_cvt_pk_f16_f32), ReLU in f16
        // (v_pk_max_f16: the same values as rounding the ReLU'd floats)
        const unsigned wv[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
        h8 a;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 y = {fmaf(__uint_as_float(wv[q] << 16), sc[2 * q], sh[2 * q]),
                           fmaf(__uint_as_float(wv[q] & 0xffff0000u), sc[2 * q + 1], sh[2 * q + 1])};
          const h2 hh = __builtin_elementwise_max(__builtin_convertvector(y, h2), (h2){(_Float16)0.f, (_Float16)0.f});
          a[2 * q] = in ? hh[0] : (_Float16)0.f;
          a[2 * q + 1] = in ? hh[1] : (_Float16)0.f;
        }
        const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, wb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        // D[pixel x0 + 4g + r][tap r16]
        if (r16 < 9) *reinterpret_cast<f32x4*>(&ring[(i % HT_NR)][r16][4 + x0 + 4 * g]) = d;
      }
      __syncthreads();
      // outputs whose rows y-1, y, y+1 are in: y - y0 + 2 <= 2k + 1
      const int ylo = max(y0, y0 + 2 * k - 2), yhi = min(y1, y0 + 2 * k);
      for (int idx = tid; idx < (yhi - ylo) * HT_W; idx += 256) {
        const int yy = ylo + idx / HT_W, xx = idx % HT_W, i0 = yy - y0;   // rows i0, i0+1, i0+2
        float acc = bias;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const float* rr = &ring[(i0 + dy) % HT_NR][3 * dy][3 + xx];
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) acc += rr[dx * HT_WP + dx];
        }
        o[(int64_t)yy * HT_W + xx] = acc;
      }
#pragma unroll
      for (int j = 0; j < HT_TPS; ++j) {
        cur[j] = nxt[j];
        if (PD > 1) nxt[j] = nn[j];
      }
    }
    __syncthreads();                                 // the ring is rewritten by the next unit
  }
}

// 0 = MFMA tap-product kernel at W = 96 (head_tap_kernel, two input steps in flight), 1 = the v_dot2c
// band kernel with the compile-time width 96, 2 = the band kernel with a runtime width, 3 = the tap
// kernel with one input step in flight
int g_head_variant = 0;

}  // namespace

extern "C" int catseg_conv_tile_rows(void) { return BM; }

int catseg_conv3x3_ring(const CatsegConvArgs* a, hipStream_t st);   // conv_ring.hip
int g_conv_mode = 2;   // 2 = row-ring kernel where it applies, 0 = im2col only
CATSEG_KNOB(g_conv_mode, "conv_mode");
CATSEG_KNOB(g_head_variant, "head_variant");

int catseg_conv3x3_ring_tile(const CatsegConvArgs* a);   // conv_ring.hip
// fp32 workspace the im2col kernel would use for split-K on these args (0 = none needed)
extern "C" int64_t catseg_conv3x3_workspace(const CatsegConvArgs* a) {
  if (!a) return 0;
  if (g_conv_mode >= 2 && catseg_conv3x3_ring_tile(a)) return 0;
  const int ks = conv_ksplit(a);
  return ks > 1 ? (int64_t)ks * a->S * a->H * a->W * a->c_out * 4 : 0;
}

extern "C" int catseg_conv3x3_stats_tile(const CatsegConvArgs* a) {
  if (!a) return 0;
  if (g_conv_mode >= 2) {
    const int t = catseg_conv3x3_ring_tile(a);
    if (t) return t;
  }
  return BM;   // the im2col kernel emits 128-pixel partials
}

extern "C" int catseg_conv3x3(const CatsegConvArgs* a, void* stream) {
  CATSEG_CHECK(a && a->src1 && a->weight && a->out, "conv3x3: null pointer");
  CATSEG_CHECK(a->S > 0 && a->H > 0 && a->W > 0 && a->c1 > 0 && a->c_out > 0, "conv3x3: empty shape");
  const int vn = a->dtype == CATSEG_BF16 ? 8 : 4;
  CATSEG_CHECK(a->c1 % vn == 0 && a->c2 % vn == 0, "conv3x3: channel counts must be multiples of 16 bytes");
  CATSEG_CHECK(a->c2 == 0 || (a->src2 && a->src2_div > 0), "conv3x3: src2 missing");
  CATSEG_CHECK(a->c_out % 4 == 0, "conv3x3: c_out must be a multiple of 4");
  CATSEG_CHECK(a->s1_slice_stride % vn == 0 && a->s1_offset % vn == 0, "conv3x3: src1 stride alignment");
  CATSEG_CHECK(!a->gn_mean || (a->gn_rstd && a->gn_gamma && a->gn_beta && a->gn_cpg > 0 && a->c1 % a->gn_cpg == 0 &&
                               a->gn_cpg % vn == 0 && a->c1 <= 128 && ((int64_t)a->H * a->W) % BM == 0),
               "conv3x3: bad GroupNorm prologue (needs c1 <= 128, H*W % 128 == 0)");
  if (a->stats) {
    CATSEG_CHECK(((int64_t)a->H * a->W) % BM == 0, "conv3x3: GN stats need H*W % 128 == 0");
    CATSEG_CHECK(a->c_out <= 64 && a->stats_cpg == 16 && a->c_out % 16 == 0, "conv3x3: GN stats need cout<=64, 16/group");
  }
  ConvP p;
  p.s1 = a->src1; p.s1_ss = a->s1_slice_stride; p.s1_off = a->s1_offset; p.c1 = a->c1;
  p.s2 = a->src2; p.s2_ss = a->s2_slice_stride; p.s2_off = a->s2_offset; p.c2 = a->c2; p.s2_div = a->src2_div > 0 ? a->src2_div : 1;
  p.S = a->S; p.H = a->H; p.W = a->W; p.w = a->weight; p.cout = a->c_out; p.bias = a->bias; p.act = a->act;
  p.gmean = a->gn_mean; p.grstd = a->gn_rstd; p.ggamma = a->gn_gamma; p.gbeta = a->gn_beta; p.gcpg = a->gn_cpg;
  p.out = a->out; p.stats = a->stats; p.scpg = a->stats_cpg;
  p.add = a->addend; p.add_ss = a->addend_slice_stride; p.add_div = a->addend_div > 0 ? a->addend_div : 1;
  p.ksplit = 1; p.ws = nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (g_conv_mode >= 2 && catseg_conv3x3_ring(a, st) == 0) return catseg_launch_status("conv3x3_ring");
  const int ks = conv_ksplit(a);
  const int64_t Mtot = a->S * (int64_t)a->H * a->W;
  if (ks > 1 && a->workspace && a->workspace_bytes >= (int64_t)ks * Mtot * a->c_out * 4 && a->c_out % 4 == 0) {
    p.ksplit = ks;
    p.ws = (float*)a->workspace;
  }
  if (a->dtype == CATSEG_BF16) launch_conv<bf16>(p, st);
  else launch_conv<float>(p, st);
  return catseg_launch_status("conv3x3");
}

extern "C" int catseg_groupnorm_stats(const float* partials, int64_t S, int tiles, int groups, int64_t tile_count,
                                      float eps, float* mean, float* rstd, void* stream) {
  CATSEG_CHECK(partials && mean && rstd && S > 0 && tiles > 0 && groups > 0, "groupnorm_stats: bad args");
  const int64_t n = S * groups;
  hipLaunchKernelGGL(gn_stats_kernel, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     partials, S, tiles, groups, (float)tile_count, eps, mean, rstd);
  return catseg_launch_status("groupnorm_stats");
}

extern "C" int catseg_groupnorm_relu(const void* x, void* y, int64_t S, int64_t HW, int C, int cpg,
                                     const float* mean, const float* rstd, const float* gamma,
                                     const float* beta, int dtype, void* stream) {
  CATSEG_CHECK(x && y && mean && rstd && gamma && beta && C % 4 == 0 && cpg > 0 && C % cpg == 0 && cpg % 4 == 0,
               "groupnorm_relu: bad args");
  const int64_t total4 = S * HW * C / 4;
  const unsigned grid = (unsigned)std::min<int64_t>((total4 + 255) / 256, 8192);
  if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL(gn_relu_kernel<bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (bf16*)y,
                       total4, C, cpg, HW, mean, rstd, gamma, beta);
  else
    hipLaunchKernelGGL(gn_relu_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)x,
                       (float*)y, total4, C, cpg, HW, mean, rstd, gamma, beta);
  return catseg_launch_status("groupnorm_relu");
}

extern "C" int catseg_conv3x3_head_gn(const void* x, int64_t B, int T, int H, int W, int C, const float* weight,
                                      float bias, const float* mean, const float* rstd, const float* gamma,
                                      const float* beta, int cpg, const int32_t* classes, int T_out, float* out,
                                      int dtype, void* stream) {
  CATSEG_CHECK(x && weight && out && C % 8 == 0 && C <= 256 && B > 0 && T > 0, "conv3x3_head: bad args");
  CATSEG_CHECK(!mean || (rstd && gamma && beta && cpg > 0 && C % cpg == 0), "conv3x3_head: bad GN args");
  if (dtype == CATSEG_BF16 && C == 32 && W <= 128) {
    const size_t shb = 9 * C * 2 + 2 * C * 4 + (size_t)(HBR + 2) * (W + 2) * (C + 8) * 2;
    static bool configured = false;
    if (!configured) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&head_band_kernel<32>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      configured = true;
    }
    if (W == 96 && (g_head_variant == 0 || g_head_variant == 3)) {
      const int n_cu = catseg_device_cus();
      const int RB = 24, ups = (H + RB - 1) / RB;
      const int64_t nunits = B * (int64_t)T * ups;
      CATSEG_CHECK(nunits < (1LL << 31), "conv3x3_head: too many bands");
      // four workgroups per CU (six measured slower: 189-193 vs 171 us); two input steps in flight
      // (one: 178-180 us, variant 3)
      const unsigned grid = (unsigned)std::min<int64_t>(nunits, 4LL * n_cu);
      if (g_head_variant == 3)
        hipLaunchKernelGGL(head_tap_kernel<1>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, T, H, weight,
                           bias, mean, rstd, gamma, beta, cpg, classes, T_out, out, RB, ups, (int)nunits);
      else
        hipLaunchKernelGGL(head_tap_kernel<2>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, T, H, weight,
                           bias, mean, rstd, gamma, beta, cpg, classes, T_out, out, RB, ups, (int)nunits);
    } else if (W == 96 && g_head_variant != 2) {
      static bool configured96 = false;
      if (!configured96) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&head_band_kernel<32, 96>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        configured96 = true;
      }
      hipLaunchKernelGGL((head_band_kernel<32, 96>), dim3((unsigned)((H + HBR - 1) / HBR), (unsigned)(B * T)), dim3(256),
                         shb, (hipStream_t)stream, (const bf16*)x, T, H, W, weight, bias, mean, rstd, gamma, beta, cpg,
                         classes, T_out, out);
    } else {
      hipLaunchKernelGGL(head_band_kernel<32>, dim3((unsigned)((H + HBR - 1) / HBR), (unsigned)(B * T)), dim3(256), shb,
                         (hipStream_t)stream, (const bf16*)x, T, H, W, weight, bias, mean, rstd, gamma, beta, cpg,
                         classes, T_out, out);
    }
    return catseg_launch_status("conv3x3_head");
  }
  const dim3 grid((unsigned)(((int64_t)H * W + 255) / 256), (unsigned)(B * T));
  const size_t sh = 11 * C * sizeof(float);
  if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL(head_kernel<bf16>, grid, dim3(256), sh, (hipStream_t)stream, (const bf16*)x, B, T, H, W,
                       C, weight, bias, mean, rstd, gamma, beta, cpg, classes, T_out, out);
  else if (C == 32 && ((uintptr_t)x % 16) == 0) {
    // fp32, 32 channels (the decoder's last width): 8 lanes per pixel, 32 pixels per block pass
    const unsigned gx = (unsigned)std::min<int64_t>(((int64_t)H * W + 31) / 32, 64);
    hipLaunchKernelGGL(head_vec_kernel<8>, dim3(gx, (unsigned)(B * T)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)x, T, H, W, weight, bias, mean, rstd, gamma, beta, cpg, classes, T_out, out);
  } else
    hipLaunchKernelGGL(head_kernel<float>, grid, dim3(256), sh, (hipStream_t)stream, (const float*)x, B, T, H,
                       W, C, weight, bias, mean, rstd, gamma, beta, cpg, classes, T_out, out);
  return catseg_launch_status("conv3x3_head");
}

extern "C" int catseg_conv3x3_head(const void* x, int64_t B, int T, int H, int W, int C, const float* weight,
                                   float bias, const int32_t* classes, int T_out, float* out, int dtype,
                                   void* stream) {
  return catseg_conv3x3_head_gn(x, B, T, H, W, C, weight, bias, nullptr, nullptr, nullptr, nullptr, 1, classes,
                                T_out, out, dtype, stream);
}
