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

constexpr int MAXV = 8;   // D <= 512
constexpr int NW = 4;     // waves per segment
constexpr int UNR = 4;    // rows in flight per wave

// one row's (clipped, noised) contribution added into acc
__device__ __forceinline__ void add_row(float (&acc)[MAXV], const float (&v)[MAXV], int r, int D, int lane, float clip,
                                        float noise_std, unsigned long long seed, unsigned long long offset) {
  float f = 1.0f;
  if (clip > 0.f) {
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) sq += v[k] * v[k];
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

// One 256-thread block per output row (segment).  Wave w takes occurrences beg+w, beg+w+4,
// ... with UNR independent row loads in flight (popular news -- and the <unk>/pad row 0 that
// every short history points at -- have hundreds of occurrences per batch); the 4 wave
// partials are combined in LDS in a fixed order, so the result is deterministic.
__global__ __launch_bounds__(256) void segsum_kernel(const float* __restrict__ rows, const int* __restrict__ perm,
                                                     const int* __restrict__ seg_ptr, float* __restrict__ out, int U,
                                                     int D, float clip, float noise_std, unsigned long long seed,
                                                     unsigned long long offset) {
  __shared__ float part[NW][64 * MAXV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = blockIdx.x;
  float acc[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) acc[k] = 0.f;
  const int beg = seg_ptr[u], end = seg_ptr[u + 1];
  for (int i0 = beg + w; i0 < end; i0 += NW * UNR) {
    float v[UNR][MAXV];
    int rr[UNR];
#pragma unroll
    for (int j = 0; j < UNR; ++j) {
      const int i = i0 + j * NW;
      rr[j] = i < end ? perm[i] : -1;
    }
#pragma unroll
    for (int j = 0; j < UNR; ++j) {
      const float* g = rows + (size_t)(rr[j] < 0 ? 0 : rr[j]) * D;
#pragma unroll
      for (int k = 0; k < MAXV; ++k) {
        const int d = lane + 64 * k;
        v[j][k] = (rr[j] >= 0 && d < D) ? g[d] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < UNR; ++j)
      if (rr[j] >= 0) add_row(acc, v[j], rr[j], D, lane, clip, noise_std, seed, offset);
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) part[w][lane + 64 * k] = acc[k];
  __syncthreads();
  float* o = out + (size_t)u * D;
  for (int d = threadIdx.x; d < D; d += 256) o[d] = ((part[0][d] + part[1][d]) + part[2][d]) + part[3][d];
}

}  // namespace

extern "C" int fr_segment_sum_rows(const float* rows, const int* perm, const int* seg_ptr, float* out, int U, int D,
                                   float clip, float noise_std, unsigned long long seed, unsigned long long offset,
                                   hipStream_t s) {
  if (D > 64 * MAXV) return 1;
  if (U == 0) return 0;
  hipLaunchKernelGGL(segsum_kernel, dim3(U), dim3(256), 0, s, rows, perm, seg_ptr, out, U, D, clip,
                     noise_std, seed, offset);
  return 0;
}
