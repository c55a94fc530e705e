// Additive attention pooling (reference attention.py:8-26):
//
//   a_t   = w2 . e_t + b2               e = tanh(W1 x + b1) comes from the GEMM epilogue
//   alpha = exp(a) / (sum_t exp(a) + 1e-8)   -- evaluated as exp(a-m) / (sum exp(a-m) + 1e-8 exp(-m))
//   out   = sum_t alpha_t x_t
//
// and its backward:
//   dalpha_t = x_t . g ;  da_t = alpha_t (dalpha_t - sum_k alpha_k dalpha_k)
//   dpre_t   = da_t w2 (1 - e_t^2)      (tanh folded in: the caller's GEMMs give dW1, dx)
//   dw2     += sum_t da_t e_t ;  db2 += sum_t da_t ;  dx_direct_t = alpha_t g
//
// One 256-thread block per sequence (a title for the text head: T=50, D=768, Q=384; an
// impression for the user encoder: H=50, D=400, Q=200).  x/e are bf16 (text path) or
// fp32 (user path); statistics and outputs are fp32.  dw2/db2 are reduced in LDS per
// block, then one float atomic per element per block.
#include "common.h"

namespace {

constexpr int MAXT = 128;

template <typename T>
__device__ __forceinline__ float ld(const T* p) { return (float)*p; }

template <typename TX>
__global__ __launch_bounds__(256) void pool_fwd_kernel(const TX* __restrict__ x, const TX* __restrict__ e,
                                                       const float* __restrict__ w2, const float* __restrict__ b2,
                                                       float* __restrict__ out, float* __restrict__ alpha_out, int T,
                                                       int D, int Q) {
  __shared__ float a_s[MAXT];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const TX* xe = x + (size_t)n * T * D;
  const TX* ee = e + (size_t)n * T * Q;
  for (int t = wave; t < T; t += 4) {
    float s = 0.f;
    for (int q = lane; q < Q; q += 64) s += ld(ee + (size_t)t * Q + q) * w2[q];
    s = wave_sum(s);
    if (lane == 0) a_s[t] = s + b2[0];
  }
  __syncthreads();
  if (wave == 0) {
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, a_s[t]);
    m = wave_max(m);
    float l = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float p = __expf(a_s[t] - m);
      a_s[t] = p;
      l += p;
    }
    l = wave_sum(l) + 1e-8f * __expf(-m);
    const float inv = 1.0f / l;
    for (int t = lane; t < T; t += 64) {
      const float al = a_s[t] * inv;
      a_s[t] = al;
      alpha_out[(size_t)n * T + t] = al;
    }
  }
  __syncthreads();
  for (int d = tid; d < D; d += 256) {
    float acc = 0.f;
    for (int t = 0; t < T; ++t) acc += a_s[t] * ld(xe + (size_t)t * D + d);
    out[(size_t)n * D + d] = acc;
  }
}

template <typename TX>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const TX* __restrict__ x, const TX* __restrict__ e,
                                                       const float* __restrict__ alpha, const float* __restrict__ w2,
                                                       const float* __restrict__ g, float* __restrict__ dx,
                                                       TX* __restrict__ dpre, float* __restrict__ dw2,
                                                       float* __restrict__ db2, int T, int D, int Q) {
  __shared__ float da_s[MAXT];
  __shared__ float al_s[MAXT];
  __shared__ float red[4];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const TX* xe = x + (size_t)n * T * D;
  const TX* ee = e + (size_t)n * T * Q;
  const float* gn = g + (size_t)n * D;
  for (int t = tid; t < T; t += 256) al_s[t] = alpha[(size_t)n * T + t];
  // dalpha_t = x_t . g
  for (int t = wave; t < T; t += 4) {
    float s = 0.f;
    for (int d = lane; d < D; d += 64) s += ld(xe + (size_t)t * D + d) * gn[d];
    s = wave_sum(s);
    if (lane == 0) da_s[t] = s;
  }
  __syncthreads();
  if (wave == 0) {
    float s = 0.f;
    for (int t = lane; t < T; t += 64) s += al_s[t] * da_s[t];
    s = wave_sum(s);
    float sd = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float v = al_s[t] * (da_s[t] - s);
      da_s[t] = v;
      sd += v;
    }
    sd = wave_sum(sd);
    if (lane == 0) red[0] = sd;
  }
  __syncthreads();
  if (tid == 0) atomicAdd(db2, red[0]);
  // dpre and dw2
  for (int q = tid; q < Q; q += 256) {
    const float wq = w2[q];
    float acc = 0.f;
    for (int t = 0; t < T; ++t) {
      const float ev = ld(ee + (size_t)t * Q + q);
      const float da = da_s[t];
      acc += da * ev;
      dpre[((size_t)n * T + t) * Q + q] = (TX)(da * wq * (1.0f - ev * ev));
    }
    atomicAdd(dw2 + q, acc);
  }
  if (dx != nullptr) {
    for (int d = tid; d < D; d += 256) {
      const float gd = gn[d];
      for (int t = 0; t < T; ++t) dx[((size_t)n * T + t) * D + d] = al_s[t] * gd;
    }
  }
}

}  // namespace

extern "C" int fr_additive_pool_fwd(const void* x, const void* e, const float* w2, const float* b2, float* out,
                                    float* alpha, int n, int T, int D, int Q, int is_bf16, hipStream_t s) {
  if (T > MAXT) return 1;
  if (n == 0) return 0;
  if (is_bf16)
    hipLaunchKernelGGL(pool_fwd_kernel<bf16>, dim3(n), dim3(256), 0, s, (const bf16*)x, (const bf16*)e, w2, b2, out,
                       alpha, T, D, Q);
  else
    hipLaunchKernelGGL(pool_fwd_kernel<float>, dim3(n), dim3(256), 0, s, (const float*)x, (const float*)e, w2, b2,
                       out, alpha, T, D, Q);
  return 0;
}

extern "C" int fr_additive_pool_bwd(const void* x, const void* e, const float* alpha, const float* w2, const float* g,
                                    float* dx, void* dpre, float* dw2, float* db2, int n, int T, int D, int Q,
                                    int is_bf16, hipStream_t s) {
  if (T > MAXT) return 1;
  if (n == 0) return 0;
  if (is_bf16)
    hipLaunchKernelGGL(pool_bwd_kernel<bf16>, dim3(n), dim3(256), 0, s, (const bf16*)x, (const bf16*)e, alpha, w2, g,
                       dx, (bf16*)dpre, dw2, db2, T, D, Q);
  else
    hipLaunchKernelGGL(pool_bwd_kernel<float>, dim3(n), dim3(256), 0, s, (const float*)x, (const float*)e, alpha, w2,
                       g, dx, (float*)dpre, dw2, db2, T, D, Q);
  return 0;
}
