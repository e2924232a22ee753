// catseg_swin_window_attention: argument checks and dispatch of the fused bf16 Swin window
// attention (LayerNorm(norm1) + [q|k|v] projection (+ the per-image guidance half of q, k) +
// shifted-window multi-head attention; the kernels are in swin_window.hip).
// Reference: SwinTransformerBlock.forward model.py:191-199 (norm1, concat guidance,
// roll, window_partition) and WindowAttention.forward model.py:86-114 up to (and not
// including) the output projection; the -100 region mask of model.py:161-183.
//   swin_win5 (default): register-resident, two 4-wave workgroups per CU; guidance rows that are
//     one base + the pixel per slice (every engine call).
//   swin_win3 (swin_variant 3, and any other guidance row map): head-per-SIMD, K / V^T in LDS.
// Window geometry is compile-time (24 x 24 feature map, 12 x 12 windows: CAT-Seg's
// FEATURE_RESOLUTION / window_size, host-checked).
#include "common.h"
#include "capi.h"

namespace {

constexpr int IMG = 24, WS = 12, NWIN = 4;
constexpr int D = 32, NH = 4;
int g_swin_variant = 0;   // 0 = default, 3 = swin_win3 (tests / tools)

}  // namespace

CATSEG_KNOB(g_swin_variant, "swin_variant");

int swin_win3_launch(const CatsegSwinAttnArgs* a, int n_cu, hipStream_t st, bool glin);   // swin_window.hip
int swin_win5_launch(const CatsegSwinAttnArgs* a, int n_cu, hipStream_t st, bool glin);

// the guidance row map restricted to one slice is rowmap(slice * 576) + pixel (swin_win3 then adds the pixel)
static bool gmap_linear_in_pixel(const CatsegRowMap& m) {
  const int64_t P = IMG * IMG;
  return (m.d2 == 1 && m.s2 == 1 && m.m2 % P == 0 && m.d1 % P == 0) ||
         (m.d1 == 1 && m.s1 == 1 && m.m1 % P == 0 && m.d2 % P == 0);
}

extern "C" int catseg_swin_window_attention(const CatsegSwinAttnArgs* a, void* stream) {
  CATSEG_CHECK(a && a->x && a->ln_g && a->ln_b && a->w_qkv && a->b_qkv && a->gqk && a->out,
               "swin_window_attention: null pointer");
  CATSEG_CHECK(a->dtype == CATSEG_BF16, "swin_window_attention: bf16 only");
  CATSEG_CHECK(a->img_h == IMG && a->img_w == IMG && a->window == WS, "swin_window_attention: 24x24 map, 12x12 windows");
  CATSEG_CHECK(a->n_heads == NH && a->head_dim == D, "swin_window_attention: 4 heads x 32");
  CATSEG_CHECK(a->shift >= 0 && a->shift < WS, "swin_window_attention: bad shift");
  CATSEG_CHECK(a->S > 0 && a->S * NWIN < (1LL << 31), "swin_window_attention: bad slice count");
  CATSEG_CHECK(a->ld_x % 8 == 0 && a->ld_g % 4 == 0 && a->ld_out % 4 == 0, "swin_window_attention: row alignment");
  CATSEG_CHECK(a->gmap.d1 > 0 && a->gmap.m1 > 0 && a->gmap.d2 > 0 && a->gmap.m2 > 0, "swin_window_attention: bad gmap");
  const int n_cu = catseg_device_cus();
  const bool glin = gmap_linear_in_pixel(a->gmap);
  if (glin && g_swin_variant == 0) swin_win5_launch(a, n_cu, (hipStream_t)stream, true);
  else swin_win3_launch(a, n_cu, (hipStream_t)stream, glin);
  return catseg_launch_status("swin_window_attention");
}
