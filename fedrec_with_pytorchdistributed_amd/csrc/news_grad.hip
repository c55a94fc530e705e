// Per-news gradient reduction with fused local differential privacy
// (reference client.py:26-48 process_news_grad, client.py:87-89 noise, model.py:105-109;
// SURVEY §2.3 K16/K17):
//
//   out[u] = sum_{r in segment u} ( clip_C(g_r) + N(0, std) )
//
// g_r is one occurrence's gradient w.r.t. a candidate/history news vector (400 floats).
// Rows are grouped by output id (perm/seg_ptr from the dedup kernel), so each output row
// is summed by ONE wave in a fixed order: deterministic, no float atomics.
//
// LDP: per-occurrence L2 clip to C (clip > 0), then Gaussian noise N(0, std) with
// std = sigma * C (default) or sigma (reference quirk Q10: no clip, std = sigma).  Noise
// comes from Philox-4x32-10 keyed by (seed, offset=step) with counter = occurrence*D + d,
// so a row's noise does not depend on which wave processes it.
#include "common.h"

namespace {

constexpr int MAXV = 8;  // D <= 512

__global__ __launch_bounds__(256) void segsum_kernel(const float* __restrict__ rows, const int* __restrict__ perm,
                                                     const int* __restrict__ seg_ptr, float* __restrict__ out, int U,
                                                     int D, float clip, float noise_std, unsigned long long seed,
                                                     unsigned long long offset) {
  const int lane = threadIdx.x & 63;
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= U) return;
  float acc[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) acc[k] = 0.f;
  const int beg = seg_ptr[u], end = seg_ptr[u + 1];
  for (int i = beg; i < end; ++i) {
    const int r = perm[i];
    const float* g = rows + (size_t)r * D;
    float v[MAXV];
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int d = lane + 64 * k;
      v[k] = d < D ? g[d] : 0.f;
      sq += v[k] * v[k];
    }
    float f = 1.0f;
    if (clip > 0.f) {
      const float nrm = sqrtf(wave_sum(sq));
      f = fminf(1.0f, clip / (nrm + 1e-12f));
    }
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int d = lane + 64 * k;
      if (d < D) {
        float x = v[k] * f;
        if (noise_std > 0.f) {
          const uint4 rnd = Philox::gen(seed, offset, (unsigned long long)r * D + d);
          x += noise_std * box_muller(rnd.x, rnd.y).x;
        }
        acc[k] += x;
      }
    }
  }
  float* o = out + (size_t)u * D;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int d = lane + 64 * k;
    if (d < D) o[d] = acc[k];
  }
}

}  // namespace

extern "C" int fr_segment_sum_rows(const float* rows, const int* perm, const int* seg_ptr, float* out, int U, int D,
                                   float clip, float noise_std, unsigned long long seed, unsigned long long offset,
                                   hipStream_t s) {
  if (D > 64 * MAXV) return 1;
  if (U == 0) return 0;
  hipLaunchKernelGGL(segsum_kernel, dim3((U + 3) / 4), dim3(256), 0, s, rows, perm, seg_ptr, out, U, D, clip,
                     noise_std, seed, offset);
  return 0;
}
