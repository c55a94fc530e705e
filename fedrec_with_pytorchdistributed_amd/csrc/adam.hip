// Fused Adam over the flat trainable buffer (reference model.py:22-23,89,93: two
// torch.optim.Adam(lr=5e-5) that always step together).
//
//   g' = g * grad_scale        (grad_scale = 1/W folds the all-reduce average in)
//   m = b1 m + (1-b1) g' ;  v = b2 v + (1-b2) g'^2
//   p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)          (torch.optim.Adam, no weight decay)
//
// One streaming pass, float4 vectorised; optionally writes a bf16 copy of p (unfrozen
// backbone: the compute weights are refreshed in the same pass).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void adam_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                   float4* __restrict__ m, float4* __restrict__ v,
                                                   bf16x4* __restrict__ plow, long n4, float lr, float b1, float b2,
                                                   float eps, float step_size, float inv_sqrt_bc2, float gs) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    float* pa = (float*)&pp;
    float* ga = (float*)&gg;
    float* ma = (float*)&mm;
    float* va = (float*)&vv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x = ga[k] * gs;
      ma[k] = b1 * ma[k] + (1.f - b1) * x;
      va[k] = b2 * va[k] + (1.f - b2) * x * x;
      const float denom = sqrtf(va[k]) * inv_sqrt_bc2 + eps;
      pa[k] -= step_size * ma[k] / denom;
    }
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
    if (plow) plow[i] = bf16x4{f2bf(pa[0]), f2bf(pa[1]), f2bf(pa[2]), f2bf(pa[3])};
  }
}

}  // namespace

extern "C" int fr_adam_flat(float* p, const float* g, float* m, float* v, void* plow, long n, float lr, float b1,
                            float b2, float eps, float bc1, float bc2, float grad_scale, hipStream_t s) {
  if (n % 4 != 0) return 1;
  const long n4 = n / 4;
  if (n4 == 0) return 0;
  long blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (float4*)p, (const float4*)g, (float4*)m,
                     (float4*)v, (bf16x4*)plow, n4, lr, b1, b2, eps, lr / bc1, 1.0f / sqrtf(bc2), grad_scale);
  return 0;
}
