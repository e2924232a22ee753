// Resampling kernels around the aggregation and the sliding-window branch (HBM-bound,
// 16-byte channel vectors, no reductions beyond a pooling window):
//   catseg_avgpool_rows       ClassTransformerLayer.pool_features   (model.py:374-385)
//   catseg_upsample_add_rows  x + interpolate(x_pool, align_corners=True) (model.py:415-423)
//   catseg_sliding_crops      640² resize + Unfold(384, 256) + global 384² (cat_seg_model.py:158-168)
//   catseg_sliding_merge      interp 384 + sigmoid + Fold/count + global avg (cat_seg_model.py:204-213)
#include <type_traits>
#include "common.h"
#include "capi.h"

namespace {

inline unsigned grid_of(int64_t n, int64_t cap = 65536) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  return (unsigned)(g < cap ? g : cap);
}

// PyTorch bilinear source index, align_corners=False (area_pixel_compute_source_index)
DEV void lin_src(int dst, int in_size, float scale, int& i0, int& i1, float& l1) {
  float src = fmaxf(scale * ((float)dst + 0.5f) - 0.5f, 0.f);
  i0 = (int)src;
  i1 = i0 + ((i0 < in_size - 1) ? 1 : 0);
  l1 = src - (float)i0;
}
// align_corners=True: src = scale * dst, scale = (in - 1) / (out - 1)
DEV void lin_src_ac(int dst, int in_size, float scale, int& i0, int& i1, float& l1) {
  const float src = scale * (float)dst;
  i0 = (int)src;
  i1 = i0 + ((i0 < in_size - 1) ? 1 : 0);
  l1 = src - (float)i0;
}
// PyTorch's blend order: h0l * (w0l * v00 + w1l * v01) + h1l * (w0l * v10 + w1l * v11)
DEV float blend(float v00, float v01, float v10, float v11, float ly, float lx) {
  return (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
}

// ---------------- class-attention pooling (rows layout [S][H][W][C]) -----------------
template <typename T>
__global__ void avgpool_rows_kernel(const T* __restrict__ in, int64_t S, int H, int W, int C, int ph, int pw,
                                    T* __restrict__ out) {
  const int Hp = H / ph, Wp = W / pw, C4 = C / 4;
  const int64_t total = S * Hp * Wp * C4;
  const float inv = 1.f / (float)(ph * pw);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const int64_t p = i / C4;
    const int x = (int)(p % Wp), y = (int)((p / Wp) % Hp);
    const int64_t s = p / ((int64_t)Wp * Hp);
    const T* src = in + ((s * H + (int64_t)y * ph) * W + (int64_t)x * pw) * C + c;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int dy = 0; dy < ph; ++dy)
      for (int dx = 0; dx < pw; ++dx) {
        float v[4];
        load4<T>(src + ((int64_t)dy * W + dx) * C, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += v[r];
      }
    // avg_pool2d divides the window sum by the window size (no padding, count_include_pad moot)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = acc[r] * inv;
    store4<T>(out + p * C + c, acc);
  }
}

template <typename T>
__global__ void upsample_add_rows_kernel(const T* __restrict__ xp, int64_t S, int Hp, int Wp, int C, T* __restrict__ x,
                                         int H, int W) {
  const int C4 = C / 4;
  const int64_t total = S * H * W * C4;
  const float sy = H > 1 ? (float)(Hp - 1) / (float)(H - 1) : 0.f;
  const float sx = W > 1 ? (float)(Wp - 1) / (float)(W - 1) : 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const int64_t p = i / C4;
    const int xx = (int)(p % W), yy = (int)((p / W) % H);
    const int64_t s = p / ((int64_t)W * H);
    int y0, y1, x0, x1;
    float ly, lx;
    lin_src_ac(yy, Hp, sy, y0, y1, ly);
    lin_src_ac(xx, Wp, sx, x0, x1, lx);
    const T* base = xp + s * Hp * Wp * (int64_t)C + c;
    float a[4], b[4], d[4], e[4], o[4];
    load4<T>(base + ((int64_t)y0 * Wp + x0) * C, a);
    load4<T>(base + ((int64_t)y0 * Wp + x1) * C, b);
    load4<T>(base + ((int64_t)y1 * Wp + x0) * C, d);
    load4<T>(base + ((int64_t)y1 * Wp + x1) * C, e);
    T* dst = x + p * C + c;
    load4<T>(dst, o);
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] += blend(a[r], b[r], d[r], e[r], ly, lx);
    store4<T>(dst, o);
  }
}

// ---------------- sliding window ---------------------------------------------------------
// crops[n*(nb*nb+1) + l][c][y][x], k x k, unnormalised 0-255: l < nb*nb is the Unfold block
// (bi, bj) = (l / nb, l % nb) of the out_res x out_res bilinear resize; the last is the
// k x k bilinear resize of the whole image (the "global" crop).
__global__ void sliding_crops_kernel(const float* __restrict__ raw, const int32_t* __restrict__ sizes, int64_t N,
                                     int Hc, int Wc, int out_res, int k, int stride, int nb, float* __restrict__ crops) {
  const int L = nb * nb + 1;
  const int64_t total = N * L * 3 * (int64_t)k * k;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % k), y = (int)((i / k) % k);
    const int c = (int)((i / ((int64_t)k * k)) % 3);
    const int64_t nl = i / (3 * (int64_t)k * k);
    const int l = (int)(nl % L);
    const int64_t n = nl / L;
    const int h = sizes[2 * n], w = sizes[2 * n + 1];
    int Y = y, X = x, R = k;
    if (l < L - 1) {
      Y = y + stride * (l / nb);
      X = x + stride * (l % nb);
      R = out_res;
    }
    int y0, y1, x0, x1;
    float ly, lx;
    lin_src(Y, h, (float)h / (float)R, y0, y1, ly);
    lin_src(X, w, (float)w / (float)R, x0, x1, lx);
    const float* src = raw + (n * 3 + c) * (int64_t)Hc * Wc;
    crops[i] = blend(src[(int64_t)y0 * Wc + x0], src[(int64_t)y0 * Wc + x1], src[(int64_t)y1 * Wc + x0],
                     src[(int64_t)y1 * Wc + x1], ly, lx);
  }
}

DEV float sigm(float v) { return 1.f / (1.f + expf(-v)); }

// sigmoid(bilinear(plane h x w -> k x k))(y, x)
DEV float up_sig(const float* __restrict__ pl, int h, int w, int k, int y, int x) {
  int y0, y1, x0, x1;
  float ly, lx;
  lin_src(y, h, (float)h / (float)k, y0, y1, ly);
  lin_src(x, w, (float)w / (float)k, x0, x1, lx);
  return sigm(blend(pl[y0 * w + x0], pl[y0 * w + x1], pl[y1 * w + x0], pl[y1 * w + x1], ly, lx));
}

// out[n][t][Y][X] (out_res²) = (Fold(tiles)/count + bilinear(global -> out_res)) / 2
__global__ void sliding_merge_kernel(const float* __restrict__ lg, int64_t N, int T, int h, int w, int k, int stride,
                                     int nb, int out_res, float* __restrict__ out) {
  const int L = nb * nb + 1;
  const int64_t total = N * T * (int64_t)out_res * out_res;
  const float sg = (float)k / (float)out_res;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int X = (int)(i % out_res), Y = (int)((i / out_res) % out_res);
    const int64_t nt = i / ((int64_t)out_res * out_res);
    const int t = (int)(nt % T);
    const int64_t n = nt / T;
    const int64_t plane = (int64_t)h * w;
    // global crop: sigmoid(interp 96 -> k), then interp k -> out_res
    const float* gp = lg + ((n * L + L - 1) * T + t) * plane;
    int y0, y1, x0, x1;
    float ly, lx;
    lin_src(Y, k, sg, y0, y1, ly);
    lin_src(X, k, sg, x0, x1, lx);
    const float glob = blend(up_sig(gp, h, w, k, y0, x0), up_sig(gp, h, w, k, y0, x1), up_sig(gp, h, w, k, y1, x0),
                             up_sig(gp, h, w, k, y1, x1), ly, lx);
    float sum = 0.f, cnt = 0.f;
    for (int bi = 0; bi < nb; ++bi) {
      const int yy = Y - stride * bi;
      if (yy < 0 || yy >= k) continue;
      for (int bj = 0; bj < nb; ++bj) {
        const int xx = X - stride * bj;
        if (xx < 0 || xx >= k) continue;
        sum += up_sig(lg + ((n * L + bi * nb + bj) * T + t) * plane, h, w, k, yy, xx);
        cnt += 1.f;
      }
    }
    out[i] = (sum / cnt + glob) / 2.f;
  }
}

// Banded form of the same merge: one workgroup per (image, class) plane and BY output rows.
// The global crop's sigmoid(interp 96 -> k) values under the band (<= BY + 2 rows of k) are
// formed once into LDS, so each output pixel blends 4 LDS values instead of re-deriving 4
// sigmoids from the 96² plane (the k-res map is 2.8x oversampled at out_res = 640, k = 384);
// the tile terms (1-4 per pixel, at native resolution) come straight from the L2-resident
// planes.  Sigmoid and the Fold average use the hardware exp / reciprocal (~1e-7 relative).
constexpr int MERGE_BY = 16, MERGE_KMAX = 512;

// hardware exp / reciprocal (~1 ulp each): the merge is VALU-bound on ~3 sigmoids per pixel
DEV float sigm_fast(float v) { return __builtin_amdgcn_rcpf(1.f + __expf(-v)); }
DEV float up_sig_fast(const float* __restrict__ pl, int h, int w, int k, int y, int x) {
  int y0, y1, x0, x1;
  float ly, lx;
  lin_src(y, h, (float)h / (float)k, y0, y1, ly);
  lin_src(x, w, (float)w / (float)k, x0, x1, lx);
  return sigm_fast(blend(pl[y0 * w + x0], pl[y0 * w + x1], pl[y1 * w + x0], pl[y1 * w + x1], ly, lx));
}

__global__ __launch_bounds__(256) void sliding_merge_band_kernel(const float* __restrict__ lg, int T, int h, int w,
                                                                 int k, int stride, int nb, int out_res, int bands,
                                                                 float* __restrict__ out) {
  extern __shared__ float gsig[];     // (rows of the global k-res map under the band) x k
  const int L = nb * nb + 1;
  const int64_t nt = blockIdx.x / bands;
  const int band = blockIdx.x % bands;
  const int t = (int)(nt % T);
  const int64_t n = nt / T;
  const int Y0 = band * MERGE_BY, Y1 = min(Y0 + MERGE_BY, out_res);
  const float sg = (float)k / (float)out_res;
  int r_lo, r_hi, tmp;
  float tl;
  lin_src(Y0, k, sg, r_lo, tmp, tl);
  lin_src(Y1 - 1, k, sg, tmp, r_hi, tl);
  const int nr = r_hi - r_lo + 1;
  const int64_t plane = (int64_t)h * w;
  const float* gp = lg + ((n * L + L - 1) * T + t) * plane;
#pragma unroll 4
  for (int idx = threadIdx.x; idx < nr * k; idx += blockDim.x) {
    const int r = r_lo + idx / k, x = idx % k;
    gsig[idx] = up_sig_fast(gp, h, w, k, r, x);
  }
  __syncthreads();
  // each thread owns output columns X = tid + 256 j; the column terms (global-map taps, the
  // tile columns covering X and their 96-res taps) are derived once and reused down the band
  float* ob = out + nt * (int64_t)out_res * out_res;
  for (int X = threadIdx.x; X < out_res; X += blockDim.x) {
    int gx0, gx1;
    float glx;
    lin_src(X, k, sg, gx0, gx1, glx);
    int tx0[4], tx1[4], tbj[4];
    float tlx[4];
    int ncol = 0;
    for (int bj = 0; bj < nb && ncol < 4; ++bj) {
      const int xx = X - stride * bj;
      if (xx < 0 || xx >= k) continue;
      lin_src(xx, w, (float)w / (float)k, tx0[ncol], tx1[ncol], tlx[ncol]);
      tbj[ncol++] = bj;
    }
#pragma unroll 4
    for (int Y = Y0; Y < Y1; ++Y) {       // unrolled: several rows' tile loads in flight
      int y0, y1;
      float ly;
      lin_src(Y, k, sg, y0, y1, ly);
      const float* g0 = gsig + (y0 - r_lo) * k;
      const float* g1 = gsig + (y1 - r_lo) * k;
      const float glob = blend(g0[gx0], g0[gx1], g1[gx0], g1[gx1], ly, glx);
      float sum = 0.f, cnt = 0.f;
      for (int bi = 0; bi < nb; ++bi) {
        const int yy = Y - stride * bi;
        if (yy < 0 || yy >= k) continue;
        int ty0, ty1;
        float tly;
        lin_src(yy, h, (float)h / (float)k, ty0, ty1, tly);
        for (int c = 0; c < ncol; ++c) {
          const float* pl = lg + ((n * L + bi * nb + tbj[c]) * T + t) * plane;
          sum += sigm_fast(blend(pl[ty0 * w + tx0[c]], pl[ty0 * w + tx1[c]], pl[ty1 * w + tx0[c]],
                                 pl[ty1 * w + tx1[c]], tly, tlx[c]));
          cnt += 1.f;
        }
      }
      ob[(int64_t)Y * out_res + X] = (sum * __builtin_amdgcn_rcpf(cnt) + glob) * 0.5f;
    }
  }
}

// The banded merge with the tile planes' source rows staged in LDS (nb <= 2: every X is covered
// by at most two tile columns, every band by at most two tile rows): the <= (BY-1) h/k + 3 source
// rows of each covering tile plane that the band's output rows interpolate from are copied once per
// workgroup (coalesced), so each tile term blends 4 LDS values with 32-bit offsets instead of 4
// gathers through L1 with 64-bit plane addressing.  Same taps, same blend / sigmoid / Fold order as
// sliding_merge_band_kernel: bit-identical.
__global__ __launch_bounds__(256) void sliding_merge_stage_kernel(const float* __restrict__ lg, int T, int h, int w,
                                                                  int k, int stride, int nb, int out_res, int bands,
                                                                  int grows, int trows, float* __restrict__ out) {
  extern __shared__ float smem_m[];
  float* gsig = smem_m;                        // [grows][k]: sigmoid of the global k-res map rows
  float* tsl = smem_m + grows * k;             // [2 tile rows][2 tile cols][trows][w]
  const int L = nb * nb + 1;
  const int64_t nt = blockIdx.x / bands;
  const int band = blockIdx.x % bands;
  const int t = (int)(nt % T);
  const int64_t n = nt / T;
  const int Y0 = band * MERGE_BY, Y1 = min(Y0 + MERGE_BY, out_res);
  const float sg = (float)k / (float)out_res, st_ = (float)h / (float)k;
  int r_lo, r_hi, tmp;
  float tl;
  lin_src(Y0, k, sg, r_lo, tmp, tl);
  lin_src(Y1 - 1, k, sg, tmp, r_hi, tl);
  const int nr = r_hi - r_lo + 1;
  const int64_t plane = (int64_t)h * w;
  const float* gp = lg + ((n * L + L - 1) * T + t) * plane;
  for (int idx = threadIdx.x; idx < nr * k; idx += blockDim.x) {
    const int r = r_lo + idx / k, x = idx % k;
    gsig[idx] = up_sig_fast(gp, h, w, k, r, x);
  }
  // tile rows bi covering the band: source rows [tlo[bi], thi[bi]] of planes (bi, 0..nb-1)
  int tlo[2] = {0, 0};
#pragma unroll
  for (int bi = 0; bi < 2; ++bi) {
    if (bi >= nb) break;
    const int ya = max(Y0, stride * bi), yb = min(Y1, stride * bi + k) - 1;
    if (ya > yb) continue;
    int a0, a1, b0, b1;
    float la;
    lin_src(ya - stride * bi, h, st_, a0, a1, la);
    lin_src(yb - stride * bi, h, st_, b0, b1, la);
    tlo[bi] = a0;
    const int rows = b1 - a0 + 1;
    for (int bj = 0; bj < nb; ++bj) {
      const float* pl = lg + ((n * L + bi * nb + bj) * T + t) * plane + (int64_t)a0 * w;
      float* dst = tsl + (bi * 2 + bj) * trows * w;
      for (int i = threadIdx.x; i < rows * w; i += blockDim.x) dst[i] = pl[i];
    }
  }
  __syncthreads();
  float* ob = out + nt * (int64_t)out_res * out_res;
  for (int X = threadIdx.x; X < out_res; X += blockDim.x) {
    int gx0, gx1;
    float glx;
    lin_src(X, k, sg, gx0, gx1, glx);
    int tx0[2], tx1[2], tbj[2];
    float tlx[2];
    int ncol = 0;
    for (int bj = 0; bj < nb && ncol < 2; ++bj) {
      const int xx = X - stride * bj;
      if (xx < 0 || xx >= k) continue;
      lin_src(xx, w, (float)w / (float)k, tx0[ncol], tx1[ncol], tlx[ncol]);
      tbj[ncol++] = bj;
    }
#pragma unroll 4
    for (int Y = Y0; Y < Y1; ++Y) {
      int y0, y1;
      float ly;
      lin_src(Y, k, sg, y0, y1, ly);
      const float* g0 = gsig + (y0 - r_lo) * k;
      const float* g1 = gsig + (y1 - r_lo) * k;
      const float glob = blend(g0[gx0], g0[gx1], g1[gx0], g1[gx1], ly, glx);
      float sum = 0.f, cnt = 0.f;
      for (int bi = 0; bi < nb; ++bi) {
        const int yy = Y - stride * bi;
        if (yy < 0 || yy >= k) continue;
        int ty0, ty1;
        float tly;
        lin_src(yy, h, (float)h / (float)k, ty0, ty1, tly);
        for (int c = 0; c < ncol; ++c) {
          const float* pl = tsl + (bi * 2 + tbj[c]) * trows * w - tlo[bi] * w;
          sum += sigm_fast(blend(pl[ty0 * w + tx0[c]], pl[ty0 * w + tx1[c]], pl[ty1 * w + tx0[c]],
                                 pl[ty1 * w + tx1[c]], tly, tlx[c]));
          cnt += 1.f;
        }
      }
      ob[(int64_t)Y * out_res + X] = (sum * __builtin_amdgcn_rcpf(cnt) + glob) * 0.5f;
    }
  }
}

// The staged merge with the per-row interpolation terms tabulated once per workgroup (the row-side
// lin_src of the global map and of both tile rows is uniform over a band row: computed per output
// by every thread it was ~25 VALU of ~70) and the band's 16 x 640 outputs split evenly over the
// threads (columns t and t + 256 for all rows, column 512 + t % 128 for half the rows: 40 each;
// the column-per-thread walk gave 128 threads 48 outputs and 128 threads 32).  Same taps, blend,
// sigmoid and Fold order as sliding_merge_stage_kernel (the blends' FMA contraction may differ by
// an ulp).  nb == 2, out_res <= 768.
// The global plane's source rows are staged in LDS with the tile rows, all of a band's source
// loads issued before the first LDS write (one HBM round trip instead of one per loop trip), and
// the k-res global sigmoid rows are blended from LDS instead of four global loads per element
// (3.84 -> 3.59 ms per merge of 8 x 459 planes, same box).  The output terms are branch-light (see
// below): 3.63 -> 3.38 ms, bit-identical.
__global__ __launch_bounds__(256) void sliding_merge_tab_kernel(const float* __restrict__ lg, int T, int h, int w,
                                                                int k, int stride, int out_res, int bands, int grows,
                                                                int trows, float* __restrict__ out) {
  extern __shared__ float smem_m[];
  float* gsig = smem_m;                        // [grows][k]
  float* tsl = smem_m + grows * k;             // [2 tile rows][2 tile cols][trows][w]
  float* gsrc = tsl + 4 * trows * w;           // [rows of the global plane under the band][w]
  __shared__ int ti[MERGE_BY][6];              // gy0, gy1 (rel. r_lo); per tile row bi: ty0, ty1 (rel.), or -1
  __shared__ float tf[MERGE_BY][3];            // gly, tly[0], tly[1]
  constexpr int nb = 2, L = nb * nb + 1;
  const int64_t nt = blockIdx.x / bands;
  const int band = blockIdx.x % bands;
  const int t = (int)(nt % T);
  const int64_t n = nt / T;
  const int Y0 = band * MERGE_BY, Y1 = min(Y0 + MERGE_BY, out_res);
  const float sg = (float)k / (float)out_res, st_ = (float)h / (float)k;
  int r_lo, r_hi, tmp;
  float tl;
  lin_src(Y0, k, sg, r_lo, tmp, tl);
  lin_src(Y1 - 1, k, sg, tmp, r_hi, tl);
  const int nr = r_hi - r_lo + 1;
  const int64_t plane = (int64_t)h * w;
  const float* gp = lg + ((n * L + L - 1) * T + t) * plane;
  int tlo[2] = {0, 0};
  {
    int gs_lo, gs_hi;
    lin_src(r_lo, h, st_, gs_lo, tmp, tl);
    lin_src(r_hi, h, st_, tmp, gs_hi, tl);
    const float* sp[5];
    float* sd[5];
    int se[5];                                 // cumulative segment ends of the flat copy list
    sp[0] = gp + (int64_t)gs_lo * w;
    sd[0] = gsrc;
    se[0] = (gs_hi - gs_lo + 1) * w;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
      const int ya = max(Y0, stride * bi), yb = min(Y1, stride * bi + k) - 1;
      int rows = 0;
      if (ya <= yb) {
        int a0, a1, b0, b1;
        float la;
        lin_src(ya - stride * bi, h, st_, a0, a1, la);
        lin_src(yb - stride * bi, h, st_, b0, b1, la);
        tlo[bi] = a0;
        rows = b1 - a0 + 1;
      }
#pragma unroll
      for (int bj = 0; bj < nb; ++bj) {
        const int sg_ = 1 + bi * 2 + bj;
        sp[sg_] = lg + ((n * L + bi * nb + bj) * T + t) * plane + (int64_t)tlo[bi] * w;
        sd[sg_] = tsl + (bi * 2 + bj) * trows * w;
        se[sg_] = se[sg_ - 1] + rows * w;
      }
    }
    constexpr int NLD = 8;
    for (int base = 0; base < se[4]; base += NLD * 256) {
      float v[NLD];
      int sgm[NLD], off[NLD];
#pragma unroll
      for (int m = 0; m < NLD; ++m) {
        const int i = min(base + (int)threadIdx.x + 256 * m, se[4] - 1);
        const int g = (i >= se[0]) + (i >= se[1]) + (i >= se[2]) + (i >= se[3]);
        sgm[m] = g;
        off[m] = i - (g ? se[g - 1] : 0);
        v[m] = sp[g][off[m]];
      }
#pragma unroll
      for (int m = 0; m < NLD; ++m)
        if (base + (int)threadIdx.x + 256 * m < se[4]) sd[sgm[m]][off[m]] = v[m];
    }
    __syncthreads();
    const float sx = (float)w / (float)k;
#pragma unroll
    for (int m = 0; m < 2; ++m) {                // k <= 512: two k-res columns per thread
      const int x = threadIdx.x + 256 * m;
      if (x < k) {
        int x0, x1;
        float lx;
        lin_src(x, w, sx, x0, x1, lx);
        for (int i = 0; i < nr; ++i) {
          int y0, y1;
          float ly;
          lin_src(r_lo + i, h, st_, y0, y1, ly);
          const float* g0 = gsrc + (y0 - gs_lo) * w;
          const float* g1 = gsrc + (y1 - gs_lo) * w;
          gsig[i * k + x] = sigm_fast(blend(g0[x0], g0[x1], g1[x0], g1[x1], ly, lx));
        }
      }
    }
  }
  if (threadIdx.x < Y1 - Y0) {
    const int Y = Y0 + threadIdx.x;
    int y0, y1;
    float ly;
    lin_src(Y, k, sg, y0, y1, ly);
    ti[threadIdx.x][0] = (y0 - r_lo) * k;
    ti[threadIdx.x][1] = (y1 - r_lo) * k;
    tf[threadIdx.x][0] = ly;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
      const int yy = Y - stride * bi;
      if (yy < 0 || yy >= k) {
        ti[threadIdx.x][2 + 2 * bi] = -1;
        ti[threadIdx.x][3 + 2 * bi] = -1;
        tf[threadIdx.x][1 + bi] = 0.f;
      } else {
        int ty0, ty1;
        float tly;
        lin_src(yy, h, st_, ty0, ty1, tly);
        ti[threadIdx.x][2 + 2 * bi] = (ty0 - tlo[bi]) * w;
        ti[threadIdx.x][3 + 2 * bi] = (ty1 - tlo[bi]) * w;
        tf[threadIdx.x][1 + bi] = tly;
      }
    }
  }
  __syncthreads();
  float* ob = out + nt * (int64_t)out_res * out_res;
  // this thread's columns: X = tid + 256 c for c < C0 over every band row, then one more column
  // of the remainder over half the rows when out_res % 256 != 0
  const int full = out_res / 256, rem = out_res % 256;
  const int nrow = Y1 - Y0;
  const int ncols = full + (rem ? 1 : 0);
  bool cov_all[2], cov_none[2];                 // tile row bi covers every / no row of the band
#pragma unroll
  for (int bi = 0; bi < 2; ++bi) {
    cov_all[bi] = Y0 - stride * bi >= 0 && Y1 - 1 - stride * bi < k;
    cov_none[bi] = Y1 - 1 - stride * bi < 0 || Y0 - stride * bi >= k;
  }
  for (int c = 0; c < ncols; ++c) {
    int X, ya, yb;
    if (c < full) {
      X = threadIdx.x + 256 * c; ya = 0; yb = nrow;
    } else {
      // rem columns x (256 / rem) row groups share the 256 threads
      const int groups = 256 / rem, gi = threadIdx.x / rem;
      if (gi >= groups) break;
      X = 256 * full + threadIdx.x % rem;
      const int per = (nrow + groups - 1) / groups;
      ya = gi * per; yb = min(nrow, ya + per);
    }
    int gx0, gx1;
    float glx;
    lin_src(X, k, sg, gx0, gx1, glx);
    int tx0[2], tx1[2], tbj[2];
    float tlx[2];
    int ncol = 0;
#pragma unroll
    for (int bj = 0; bj < nb; ++bj) {
      const int xx = X - stride * bj;
      if (xx < 0 || xx >= k) continue;
      lin_src(xx, w, (float)w / (float)k, tx0[ncol], tx1[ncol], tlx[ncol]);
      tbj[ncol++] = bj;
    }
    // branch-light form: the second tile column duplicates the first's taps with weight 0 where
    // only one covers X, and a term is skipped only by wave-uniform tests (no lane covers it), so
    // no exec-masked branch separates a term's LDS reads from the next term's; x + 0 * s = x
    // keeps the sum bit-identical
    if (ncol == 1) { tx0[1] = tx0[0]; tx1[1] = tx1[0]; tlx[1] = tlx[0]; tbj[1] = tbj[0]; }
    const float cw1 = ncol == 2 ? 1.f : 0.f;
    const bool two = __builtin_amdgcn_ballot_w64(ncol == 2) != 0;
    auto term = [&](int yi, int bi, int cc) {
      const int o0 = max(ti[yi][2 + 2 * bi], 0), o1 = max(ti[yi][3 + 2 * bi], 0);
      const float tly = tf[yi][1 + bi];
      const float* p = tsl + (bi * 2 + tbj[cc]) * trows * w;
      return sigm_fast(blend(p[o0 + tx0[cc]], p[o0 + tx1[cc]], p[o1 + tx0[cc]], p[o1 + tx1[cc]], tly, tlx[cc]));
    };
    auto global = [&](int yi) {
      const float* g0 = gsig + ti[yi][0];
      const float* g1 = gsig + ti[yi][1];
      return blend(g0[gx0], g0[gx1], g1[gx0], g1[gx1], tf[yi][0], glx);
    };
    // bands whose rows all share one tile-row coverage (every band at 640 / 384 / 256: the
    // coverage edges are multiples of the 16-row band) run a row loop with no coverage test;
    // the others test each row (wave-uniform ballots)
    auto rows_uniform = [&](auto C0, auto C1, auto TWO) {
      constexpr bool c0 = decltype(C0)::value, c1 = decltype(C1)::value, tw = decltype(TWO)::value;
      const float cnt = (float)((c0 ? 1 : 0) + (c1 ? 1 : 0)) * (1.f + (tw ? cw1 : 0.f));
      const float rc = __builtin_amdgcn_rcpf(cnt);
#pragma unroll 4
      for (int yi = ya; yi < yb; ++yi) {
        const float glob = global(yi);
        float sum = 0.f;
        if constexpr (c0) {
          sum += term(yi, 0, 0);
          if constexpr (tw) sum += cw1 * term(yi, 0, 1);
        }
        if constexpr (c1) {
          sum += term(yi, 1, 0);
          if constexpr (tw) sum += cw1 * term(yi, 1, 1);
        }
        ob[(int64_t)(Y0 + yi) * out_res + X] = (sum * rc + glob) * 0.5f;
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    if (cov_all[0] && cov_all[1]) {
      if (two) rows_uniform(T_{}, T_{}, T_{}); else rows_uniform(T_{}, T_{}, F_{});
      continue;
    }
    if (cov_all[0] && cov_none[1]) {
      if (two) rows_uniform(T_{}, F_{}, T_{}); else rows_uniform(T_{}, F_{}, F_{});
      continue;
    }
    if (cov_none[0] && cov_all[1]) {
      if (two) rows_uniform(F_{}, T_{}, T_{}); else rows_uniform(F_{}, T_{}, F_{});
      continue;
    }
    for (int yi = ya; yi < yb; ++yi) {
      const float* g0 = gsig + ti[yi][0];
      const float* g1 = gsig + ti[yi][1];
      const float glob = blend(g0[gx0], g0[gx1], g1[gx0], g1[gx1], tf[yi][0], glx);
      float sum = 0.f, cnt = 0.f;
#pragma unroll
      for (int bi = 0; bi < nb; ++bi) {
        const int o0r = ti[yi][2 + 2 * bi];
        if (__builtin_amdgcn_ballot_w64(o0r >= 0) == 0) continue;
        const float rw = o0r >= 0 ? 1.f : 0.f;
        const int o0 = max(o0r, 0), o1 = max(ti[yi][3 + 2 * bi], 0);
        const float tly = tf[yi][1 + bi];
        const float* p0 = tsl + (bi * 2 + tbj[0]) * trows * w;
        sum += rw * sigm_fast(blend(p0[o0 + tx0[0]], p0[o0 + tx1[0]], p0[o1 + tx0[0]], p0[o1 + tx1[0]], tly, tlx[0]));
        cnt += rw;
        if (two) {
          const float* p1 = tsl + (bi * 2 + tbj[1]) * trows * w;
          sum += rw * cw1 *
                 sigm_fast(blend(p1[o0 + tx0[1]], p1[o0 + tx1[1]], p1[o1 + tx0[1]], p1[o1 + tx1[1]], tly, tlx[1]));
          cnt += rw * cw1;
        }
      }
      ob[(int64_t)(Y0 + yi) * out_res + X] = (sum * __builtin_amdgcn_rcpf(cnt) + glob) * 0.5f;
    }
  }
}

// 0 = staged merge with tabulated row terms (sliding_merge_tab_kernel, nb == 2), 1 = band kernel,
// 2 = staged merge (sliding_merge_stage_kernel); a variant whose shape limits are not met falls
// through in the order 0 -> 2 -> 1
int g_merge_variant = 0;

}  // namespace

extern "C" int catseg_avgpool_rows(const void* in, int64_t S, int H, int W, int C, int ph, int pw, void* out,
                                   int dtype, void* stream) {
  CATSEG_CHECK(in && out && S > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0, "avgpool_rows: bad args");
  CATSEG_CHECK(ph > 0 && pw > 0 && H >= ph && W >= pw, "avgpool_rows: bad pooling window");
  const int64_t total = S * (H / ph) * (W / pw) * (C / 4);
  if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL(avgpool_rows_kernel<bf16>, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)in, S, H, W, C, ph, pw, (bf16*)out);
  else
    hipLaunchKernelGGL(avgpool_rows_kernel<float>, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)in, S, H, W, C, ph, pw, (float*)out);
  return catseg_launch_status("avgpool_rows");
}

extern "C" int catseg_upsample_add_rows(const void* xp, int64_t S, int Hp, int Wp, int C, void* x, int H, int W,
                                        int dtype, void* stream) {
  CATSEG_CHECK(xp && x && S > 0 && Hp > 0 && Wp > 0 && H > 0 && W > 0, "upsample_add_rows: bad args");
  CATSEG_CHECK(C > 0 && C % 4 == 0, "upsample_add_rows: C must be a multiple of 4");
  const int64_t total = S * H * W * (C / 4);
  if (dtype == CATSEG_BF16)
    hipLaunchKernelGGL(upsample_add_rows_kernel<bf16>, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)xp, S, Hp, Wp, C, (bf16*)x, H, W);
  else
    hipLaunchKernelGGL(upsample_add_rows_kernel<float>, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)xp, S, Hp, Wp, C, (float*)x, H, W);
  return catseg_launch_status("upsample_add_rows");
}

extern "C" int catseg_sliding_crops(const float* raw, const int32_t* sizes, int64_t N, int Hc, int Wc, int out_res,
                                    int kernel, int stride, float* crops, void* stream) {
  CATSEG_CHECK(raw && sizes && crops && N > 0 && Hc > 0 && Wc > 0, "sliding_crops: bad args");
  CATSEG_CHECK(kernel > 0 && stride > 0 && out_res >= kernel, "sliding_crops: bad window geometry");
  const int nb = (out_res - kernel) / stride + 1;
  const int64_t total = N * (nb * nb + 1) * 3 * (int64_t)kernel * kernel;
  hipLaunchKernelGGL(sliding_crops_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, raw, sizes, N, Hc,
                     Wc, out_res, kernel, stride, nb, crops);
  return catseg_launch_status("sliding_crops");
}

CATSEG_KNOB(g_merge_variant, "merge_variant");

extern "C" int catseg_sliding_merge(const float* logits, int64_t N, int T, int h, int w, int kernel, int stride,
                                    int out_res, float* out, void* stream) {
  CATSEG_CHECK(logits && out && N > 0 && T > 0 && h > 0 && w > 0, "sliding_merge: bad args");
  CATSEG_CHECK(kernel > 0 && stride > 0 && out_res >= kernel, "sliding_merge: bad window geometry");
  // every output pixel must be covered by at least one tile (Fold count > 0)
  const int nb = (out_res - kernel) / stride + 1;
  CATSEG_CHECK(stride * (nb - 1) + kernel == out_res && stride <= kernel, "sliding_merge: tiles must cover out_res");
  if (kernel <= MERGE_KMAX && (kernel + stride - 1) / stride <= 4) {   // <= 4 tile columns cover any X
    const int bands = (out_res + MERGE_BY - 1) / MERGE_BY;
    const int64_t blocks = N * T * (int64_t)bands;
    CATSEG_CHECK(blocks < ((int64_t)1 << 31), "sliding_merge: grid too large");
    // LDS rows: the k-res rows under MERGE_BY output rows, + 2 for the bilinear taps
    const int rows = (int)((int64_t)(MERGE_BY - 1) * kernel / out_res) + 3;
    // tile-plane rows under one band: (MERGE_BY - 1) output rows span (MERGE_BY - 1) h / k source rows
    const int trows = (int)((int64_t)(MERGE_BY - 1) * h / kernel) + 3;
    const size_t sh2 = ((size_t)rows * kernel + (size_t)4 * trows * w) * sizeof(float);
    // the global plane's source rows under a band's k-res rows
    const int gsrows = (int)((int64_t)(rows - 1) * h / kernel) + 3;
    const size_t sh3 = sh2 + (size_t)gsrows * w * sizeof(float);
    if (g_merge_variant == 0 && nb == 2 && sh3 <= 64 * 1024 && out_res <= 768 && kernel <= 512) {
      hipLaunchKernelGGL(sliding_merge_tab_kernel, dim3((unsigned)blocks), dim3(256), sh3, (hipStream_t)stream, logits,
                         T, h, w, kernel, stride, out_res, bands, rows, trows, out);
      return catseg_launch_status("sliding_merge");
    }
    if (g_merge_variant != 1 && nb <= 2 && sh2 <= 64 * 1024) {
      hipLaunchKernelGGL(sliding_merge_stage_kernel, dim3((unsigned)blocks), dim3(256), sh2, (hipStream_t)stream, logits,
                         T, h, w, kernel, stride, nb, out_res, bands, rows, trows, out);
      return catseg_launch_status("sliding_merge");
    }
    hipLaunchKernelGGL(sliding_merge_band_kernel, dim3((unsigned)blocks), dim3(256), rows * kernel * sizeof(float),
                       (hipStream_t)stream, logits, T, h, w, kernel, stride, nb, out_res, bands, out);
  } else {
    const int64_t total = N * T * (int64_t)out_res * out_res;
    hipLaunchKernelGGL(sliding_merge_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, logits, N, T, h,
                       w, kernel, stride, nb, out_res, out);
  }
  return catseg_launch_status("sliding_merge");
}
