// Optimizer step of the training loop: torch.optim.AdamW wrapped by the reference's
// FullModelGradientClippingOptimizer (train_net.py:228-253: clip_grad_norm_ over every parameter, then
// the AdamW step), for all parameters of all groups in one multi-tensor pass.
//
//   catseg_adamw_step: (1) per 4096-element chunk, sum of squared gradients -> partials (fixed order);
//   (2) one workgroup: total = sqrt(sum of partials), coef = min(1, max_norm / (total + 1e-6)) -> device
//   scalar (no host sync); (3) per chunk: g = grad * coef (written back, as clip_grad_norm_ scales
//   .grad in place); p *= 1 - lr * wd; m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g^2;
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps).  Deterministic; no atomics.
#include "common.h"
#include "capi.h"
#include "catseg_hip_train.h"

namespace {

constexpr int CHUNK = 4096;

__global__ __launch_bounds__(256) void sumsq_kernel(const CatsegAdamWTensor* __restrict__ ts,
                                                    const int64_t* __restrict__ chunks, float* __restrict__ part) {
  __shared__ float red[4];
  const int64_t c = chunks[blockIdx.x];
  const int t = (int)(c >> 40);
  const int64_t off = (c & ((1LL << 40) - 1)) * CHUNK;
  const CatsegAdamWTensor d = ts[t];
  const int64_t end = off + CHUNK < d.numel ? off + CHUNK : d.numel;
  float s = 0.f;
  for (int64_t i = off + threadIdx.x; i < end; i += 256) {
    const float gv = d.grad[i];
    s += gv * gv;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(256) void clip_coef_kernel(const float* __restrict__ part, int64_t n, float max_norm,
                                                        float* __restrict__ out) {
  __shared__ float red[4];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += part[i];
  // fixed-order tree over the 256 lanes' partials (double)
  __shared__ double sd[256];
  sd[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) sd[threadIdx.x] += sd[threadIdx.x + w];
    __syncthreads();
  }
  (void)red;
  if (threadIdx.x == 0) {
    const float total = (float)sqrt(sd[0]);
    out[0] = total;
    out[1] = max_norm > 0.f ? fminf(max_norm / (total + 1e-6f), 1.f) : 1.f;
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(const CatsegAdamWTensor* __restrict__ ts,
                                                    const int64_t* __restrict__ chunks, const float* __restrict__ coef,
                                                    float beta1, float beta2, float eps, int clip) {
  const int64_t c = chunks[blockIdx.x];
  const int t = (int)(c >> 40);
  const int64_t off = (c & ((1LL << 40) - 1)) * CHUNK;
  const CatsegAdamWTensor d = ts[t];
  const int64_t end = off + CHUNK < d.numel ? off + CHUNK : d.numel;
  const float k = clip ? coef[1] : 1.f;
  const float decay = 1.f - d.lr * d.weight_decay;
  const float step_size = d.lr / d.bias_correction1;
  const float rbc2 = 1.f / sqrtf(d.bias_correction2);
  for (int64_t i = off + threadIdx.x; i < end; i += 256) {
    float gv = d.grad[i];
    if (clip) {
      gv *= k;
      d.grad[i] = gv;
    }
    float p = d.param[i] * decay;
    float m = d.exp_avg[i];
    m = m + (1.f - beta1) * (gv - m);
    float v = d.exp_avg_sq[i] * beta2 + (1.f - beta2) * gv * gv;
    p -= step_size * m / (sqrtf(v) * rbc2 + eps);
    d.param[i] = p;
    d.exp_avg[i] = m;
    d.exp_avg_sq[i] = v;
  }
}

}  // namespace

extern "C" int64_t catseg_adamw_chunks(const int64_t* numels, int n_tensors) {
  int64_t n = 0;
  for (int i = 0; i < n_tensors; ++i) n += (numels[i] + CHUNK - 1) / CHUNK;
  return n;
}

extern "C" int catseg_adamw_chunk_table(const int64_t* numels, int n_tensors, int64_t* table) {
  CATSEG_CHECK(numels && table && n_tensors > 0 && n_tensors < (1 << 23), "adamw_chunk_table: bad args");
  int64_t k = 0;
  for (int i = 0; i < n_tensors; ++i) {
    CATSEG_CHECK(numels[i] > 0 && numels[i] < (1LL << 40), "adamw_chunk_table: bad tensor size");
    for (int64_t c = 0; c < (numels[i] + CHUNK - 1) / CHUNK; ++c) table[k++] = ((int64_t)i << 40) | c;
  }
  return CATSEG_OK;
}

extern "C" int catseg_adamw_step(const CatsegAdamWTensor* tensors, const int64_t* chunk_table, int64_t n_chunks,
                                 float beta1, float beta2, float eps, float max_grad_norm, float* norm_out,
                                 void* workspace, int64_t workspace_bytes, void* stream) {
  CATSEG_CHECK(tensors && chunk_table && n_chunks > 0 && n_chunks < (1LL << 31), "adamw_step: bad args");
  const bool clip = max_grad_norm > 0.f;
  if (clip) {
    CATSEG_CHECK(norm_out, "adamw_step: norm_out (2 device floats) required with clipping");
    CATSEG_CHECK(workspace && workspace_bytes >= n_chunks * (int64_t)sizeof(float), "adamw_step: workspace too small");
  }
  hipStream_t st = (hipStream_t)stream;
  if (clip) {
    hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)n_chunks), dim3(256), 0, st, tensors, chunk_table, (float*)workspace);
    hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, st, (const float*)workspace, n_chunks, max_grad_norm,
                       norm_out);
  }
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)n_chunks), dim3(256), 0, st, tensors, chunk_table,
                     (const float*)norm_out, beta1, beta2, eps, (int)clip);
  return catseg_launch_status("adamw_step");
}
