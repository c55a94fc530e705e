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

// ---- exact device variants (bucketed gradient averaging, no host sync) ----------------------
// Per sum, a PRE-PASS agrees on a bound every client's values fit: each client adds a one-hot of
// the binary exponent of its own max|x| (plus its count of non-finite coordinates) into a masked
// int32 histogram of HB slots, one tiny SUM all-reduce of it, and every client reads the largest
// occupied slot: m = 2^E >= max_k max|x_k|.  Nothing is ever clamped, so the fixed-point sum is
// the plain sum to within the grid; the histogram discloses only how many clients have their
// maximum in each power-of-two range (the masks hide whose).
//   slot 0: max|x| = 0;  slot 1: non-finite count;  slot s >= 2: max|x| in [2^(s-128), 2^(s-127))
//   (exponent field e of the fp32 max -> s = max(e, 1) + 1; subnormals share slot 2).
// f = 30 - ceil(log2 W) - E (W m 2^f <= 2^30: the W-client int32 sum cannot wrap), clamped to
// [-120, 60].  One Philox call masks 4 consecutive elements (counter = element / 4).
constexpr int HB = 256;

__device__ __forceinline__ int ceil_log2(int W) {
  int c = 0;
  while ((1 << c) < W) ++c;
  return c;
}

// every thread of the block (blockDim >= HB) returns 2^f (sign > 0) or 2^-f; *bad = non-finite seen
__device__ float hist_scale(const int* __restrict__ H, int W, float sign, bool* bad) {
  __shared__ int smax, snf;
  if (threadIdx.x == 0) {
    smax = 0;
    snf = 0;
  }
  __syncthreads();
  if (threadIdx.x < HB) {
    const int h = H[threadIdx.x];
    if (threadIdx.x >= 2 && h != 0) atomicMax(&smax, (int)threadIdx.x);
    if (threadIdx.x == 1 && h != 0) snf = 1;
  }
  __syncthreads();
  *bad = snf != 0;
  if (smax == 0) return 1.f;  // every coordinate of every client is 0
  int f = 30 - ceil_log2(W) - (smax - 127);
  f = f < -120 ? -120 : (f > 60 ? 60 : f);
  return ldexpf(1.f, sign > 0.f ? f : -f);
}

// scratch[0] |= max over finite |x| (fp32 bits: ordered as unsigned), scratch[1] += non-finite count
__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, long n, unsigned* __restrict__ scratch) {
  unsigned mx = 0, nf = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = fabsf(x[i]);
    if (v <= 3.4028234663852886e38f)
      mx = mx > __float_as_uint(v) ? mx : __float_as_uint(v);
    else
      ++nf;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned m2 = __shfl_xor(mx, o, 64);
    mx = mx > m2 ? mx : m2;
    nf += __shfl_xor(nf, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (mx) atomicMax(&scratch[0], mx);
    if (nf) atomicAdd(&scratch[1], nf);
  }
}

// one block of HB / 4 threads: this client's masked histogram
__global__ __launch_bounds__(64) void hist_kernel(const unsigned* __restrict__ scratch, int* __restrict__ out,
                                                  const unsigned long long* __restrict__ seeds,
                                                  const int* __restrict__ signs, int npeers,
                                                  unsigned long long round) {
  const unsigned bits = scratch[0], nf = scratch[1];
  const int e = (int)(bits >> 23);
  const int slot = bits == 0 ? 0 : (e > 1 ? e : 1) + 1;
  const int g = threadIdx.x;
  uint32_t acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int s = 4 * g + j;
    acc[j] = (s == slot ? 1u : 0u) + (s == 1 ? nf : 0u);
  }
  for (int p = 0; p < npeers; ++p) {
    const uint4 r = Philox::gen(seeds[p], round, (unsigned long long)g);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t rr = u4_get(r, j);
      acc[j] += signs[p] > 0 ? rr : (uint32_t)(0u - rr);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) out[4 * g + j] = (int32_t)acc[j];
}

__global__ __launch_bounds__(256) void mask_exact_kernel(const float* __restrict__ x, int* __restrict__ out, long n,
                                                         const int* __restrict__ H, int W,
                                                         const unsigned long long* __restrict__ seeds,
                                                         const int* __restrict__ signs, int npeers,
                                                         unsigned long long round) {
  __shared__ unsigned long long sd[MAXP];
  __shared__ int sg[MAXP];
  for (int i = threadIdx.x; i < npeers; i += blockDim.x) {
    sd[i] = seeds[i];
    sg[i] = signs[i];
  }
  bool bad;
  const float scale = hist_scale(H, W, 1.f, &bad);  // (its barriers also cover sd / sg)
  const long n4 = (n + 3) >> 2;
  for (long g = blockIdx.x * (long)blockDim.x + threadIdx.x; g < n4; g += (long)gridDim.x * blockDim.x) {
    uint32_t acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long i = g * 4 + j;
      float v = i < n ? x[i] : 0.f;
      if (!(fabsf(v) <= 3.4028234663852886e38f)) v = 0.f;  // counted in the histogram instead
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

// the sum, dequantised; NaN everywhere if any client had a non-finite coordinate (as the plain
// sum would have been non-finite)
__global__ __launch_bounds__(256) void unmask_exact_kernel(const int* __restrict__ x, float* __restrict__ out, long n,
                                                           const int* __restrict__ H, int W) {
  bool bad;
  const float inv = hist_scale(H, W, -1.f, &bad);
  const float nan = __builtin_nanf("");
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = bad ? nan : (float)x[i] * inv;
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

// x [n] fp32 -> masked histogram out [HB] int32 (scratch: 2 zeroed uint32)
extern "C" int fr_secagg_hist(const float* x, long n, unsigned* scratch, int* out, const unsigned long long* seeds,
                              const int* signs, int npeers, unsigned long long round, hipStream_t s) {
  if (npeers > MAXP) return 1;
  if (n > 0) hipLaunchKernelGGL(amax_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, n, scratch);
  hipLaunchKernelGGL(hist_kernel, dim3(1), dim3(HB / 4), 0, s, scratch, out, seeds, signs, npeers, round);
  return 0;
}

extern "C" int fr_secagg_mask_exact(const float* x, int* out, long n, const int* H, int W,
                                    const unsigned long long* seeds, const int* signs, int npeers,
                                    unsigned long long round, hipStream_t s) {
  if (npeers > MAXP || W < 1) return 1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(mask_exact_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, x, out, n, H, W, seeds, signs,
                     npeers, round);
  return 0;
}

extern "C" int fr_secagg_unmask_exact(const int* x, float* out, long n, const int* H, int W, hipStream_t s) {
  if (W < 1) return 1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(unmask_exact_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, out, n, H, W);
  return 0;
}
