// Pairwise-mask secure aggregation (described in the reference README.md:56,65 but never
// implemented there; BASELINE config 5).
//
// Client i uploads   y_i = Q(x_i) + sum_{j != i} sign_ij * PRG(seed_ij, round)   (mod 2^32)
// with Q(x) = round(clamp(x, -c, c) * 2^f) as a two's-complement int32 and sign_ij = +1 for
// i < j, -1 for i > j.  The pairwise masks cancel exactly in the wrap-around int32 sum, so
// the all-reduce (RCCL int32 SUM over xGMI) yields sum_i Q(x_i) bit-exactly while no
// single upload reveals x_i.  Fixed point (not float) masking is what makes cancellation
// exact.  PRG = Philox-4x32-10 keyed by the pair seed, counter =
// (round, element).
#include "common.h"

namespace {

constexpr int MAXP = 64;

__global__ __launch_bounds__(256) void mask_kernel(const float* __restrict__ x, int* __restrict__ out, long n,
                                                   float scale, float clipv, const unsigned long long* __restrict__ seeds,
                                                   const int* __restrict__ signs, int npeers, unsigned long long round) {
  __shared__ unsigned long long sd[MAXP];
  __shared__ int sg[MAXP];
  for (int i = threadIdx.x; i < npeers; i += blockDim.x) {
    sd[i] = seeds[i];
    sg[i] = signs[i];
  }
  __syncthreads();
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = fminf(fmaxf(x[i], -clipv), clipv);
    uint32_t acc = (uint32_t)(int32_t)rintf(v * scale);
    for (int p = 0; p < npeers; ++p) {
      const uint32_t r = Philox::gen(sd[p], round, (unsigned long long)i).x;
      acc += sg[p] > 0 ? r : (uint32_t)(0u - r);
    }
    out[i] = (int32_t)acc;
  }
}

__global__ __launch_bounds__(256) void unmask_kernel(const int* __restrict__ x, float* __restrict__ out, long n,
                                                     float inv_scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (float)x[i] * inv_scale;
}

// ---- device-scale variants (bucketed gradient averaging, no host sync) ---------------------
// The fixed-point exponent comes from m = max_k max|x_k| (a device scalar, MAX all-reduced
// over the clients): f = clamp(floor(log2(2^30 / (W m))), 0, 56) so the W-client sum of
// |Q(x)| <= 2^30 fits int32.  Every client derives the same f from the same bits of m.  One
// Philox call masks 4 consecutive elements (counter = element / 4, word = element % 4).
__device__ __forceinline__ float frac_exp2(const float* __restrict__ mdev, int W, float sign) {
  float m = mdev[0];
  if (!(m > 1e-30f)) m = 1e-30f;  // also NaN
  if (!(m < 3.0e38f)) m = 3.0e38f;
  float f = floorf(log2f(1073741824.0f / ((float)W * m)));
  f = fminf(fmaxf(f, 0.f), 56.f);
  return exp2f(sign * f);
}

__global__ __launch_bounds__(256) void mask_dev_kernel(const float* __restrict__ x, int* __restrict__ out, long n,
                                                       const float* __restrict__ mdev, int W,
                                                       const unsigned long long* __restrict__ seeds,
                                                       const int* __restrict__ signs, int npeers,
                                                       unsigned long long round) {
  __shared__ unsigned long long sd[MAXP];
  __shared__ int sg[MAXP];
  for (int i = threadIdx.x; i < npeers; i += blockDim.x) {
    sd[i] = seeds[i];
    sg[i] = signs[i];
  }
  __syncthreads();
  const float scale = frac_exp2(mdev, W, 1.f);
  float clipv = mdev[0];
  if (!(clipv >= 0.f)) clipv = 0.f;
  const long n4 = (n + 3) >> 2;
  for (long g = blockIdx.x * (long)blockDim.x + threadIdx.x; g < n4; g += (long)gridDim.x * blockDim.x) {
    uint32_t acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long i = g * 4 + j;
      const float v = i < n ? fminf(fmaxf(x[i], -clipv), clipv) : 0.f;
      acc[j] = (uint32_t)(int32_t)rintf(v * scale);
    }
    for (int p = 0; p < npeers; ++p) {
      const uint4 r = Philox::gen(sd[p], round, (unsigned long long)g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t rr = u4_get(r, j);
        acc[j] += sg[p] > 0 ? rr : (uint32_t)(0u - rr);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (g * 4 + j < n) out[g * 4 + j] = (int32_t)acc[j];
  }
}

__global__ __launch_bounds__(256) void unmask_dev_kernel(const int* __restrict__ x, float* __restrict__ out, long n,
                                                         const float* __restrict__ mdev, int W) {
  const float inv = frac_exp2(mdev, W, -1.f);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (float)x[i] * inv;
}

unsigned grid_for(long n) {
  long b = (n + 255) / 256;
  return (unsigned)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" int fr_secagg_mask(const float* x, int* out, long n, float scale, float clipv, const unsigned long long* seeds,
                              const int* signs, int npeers, unsigned long long round, hipStream_t s) {
  if (npeers > MAXP) return 1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(mask_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, out, n, scale, clipv, seeds, signs, npeers,
                     round);
  return 0;
}

extern "C" int fr_secagg_unmask(const int* x, float* out, long n, float inv_scale, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(unmask_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, out, n, inv_scale);
  return 0;
}

extern "C" int fr_secagg_mask_dev(const float* x, int* out, long n, const float* mdev, int W,
                                  const unsigned long long* seeds, const int* signs, int npeers,
                                  unsigned long long round, hipStream_t s) {
  if (npeers > MAXP || W < 1) return 1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(mask_dev_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, x, out, n, mdev, W, seeds, signs,
                     npeers, round);
  return 0;
}

extern "C" int fr_secagg_unmask_dev(const int* x, float* out, long n, const float* mdev, int W, hipStream_t s) {
  if (W < 1) return 1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(unmask_dev_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, out, n, mdev, W);
  return 0;
}
