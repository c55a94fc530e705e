// Fused scoring + loss + gradients (reference model.py:121-126):
//
//   z_c = cand_c . u,  s = sigmoid(z),  loss = mean_b [ logsumexp_c s_c - s_0 ]   (label 0)
//   ds_c = (softmax(s)_c - [c = 0]) / B,  dz = ds s (1 - s)
//   dcand_c = dz_c u,  du = sum_c dz_c cand_c
//
// One wave per impression; the forward and the backward are one pass, so autograd's
// backward is a scale by the incoming loss gradient.  Also used for validation scores.
#include "common.h"

namespace {

constexpr int MAXC = 16;

__global__ __launch_bounds__(256) void score_ce_kernel(const float* __restrict__ cand, const float* __restrict__ user,
                                                       float* __restrict__ loss, float* __restrict__ scores,
                                                       float* __restrict__ dcand, float* __restrict__ duser, int B,
                                                       int C, int D, int sigm) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* cb = cand + (size_t)b * C * D;
  const float* ub = user + (size_t)b * D;
  float z[MAXC];
  for (int c = 0; c < C; ++c) {
    float s = 0.f;
    for (int d = lane; d < D; d += 64) s += cb[(size_t)c * D + d] * ub[d];
    z[c] = wave_sum(s);
  }
  float s[MAXC], mx = -INFINITY;
  for (int c = 0; c < C; ++c) {
    s[c] = sigm ? 1.0f / (1.0f + __expf(-z[c])) : z[c];
    mx = fmaxf(mx, s[c]);
  }
  float se = 0.f;
  for (int c = 0; c < C; ++c) se += __expf(s[c] - mx);
  const float lse = mx + __logf(se);
  if (lane == 0) {
    loss[b] = (lse - s[0]) / (float)B;  // per-impression share; the caller sums in a fixed order
    for (int c = 0; c < C; ++c) scores[(size_t)b * C + c] = s[c];
  }
  float dz[MAXC];
  const float invB = 1.0f / (float)B;
  for (int c = 0; c < C; ++c) {
    float ds = (__expf(s[c] - mx) / se - (c == 0 ? 1.f : 0.f)) * invB;
    dz[c] = sigm ? ds * s[c] * (1.f - s[c]) : ds;
  }
  for (int d = lane; d < D; d += 64) {
    const float ud = ub[d];
    float du = 0.f;
    for (int c = 0; c < C; ++c) {
      du += dz[c] * cb[(size_t)c * D + d];
      dcand[((size_t)b * C + c) * D + d] = dz[c] * ud;
    }
    duser[(size_t)b * D + d] = du;
  }
}

// Block-per-impression form (default): one wave per candidate computes its score, so the C
// dot products run side by side instead of one after another in a single wave (that chain of
// load -> reduce rounds made the wave-per-impression kernel ~18 us for B = 64).  The softmax /
// loss / dz of the impression come from wave 0's first C lanes; dcand rows are written by
// their own wave, du by all threads over the D columns.  ci (optional): candidate (b, c) is
// row ci[b C + c] of a news-vector table (the training step's rows, no gathered copy).
__global__ __launch_bounds__(64 * MAXC) void score_ce_block_kernel(const float* __restrict__ cand,
                                                                   const float* __restrict__ user,
                                                                   float* __restrict__ loss,
                                                                   float* __restrict__ scores,
                                                                   float* __restrict__ dcand,
                                                                   float* __restrict__ duser, int B, int C, int D,
                                                                   int sigm, const int* __restrict__ ci,
                                                                   float* __restrict__ loss_total,
                                                                   unsigned* __restrict__ cnt) {
  __shared__ float zs[MAXC], dzs[MAXC];
  __shared__ const float* rowp[MAXC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x;
  if (threadIdx.x < C)
    rowp[threadIdx.x] = cand + (size_t)(ci ? ci[(size_t)b * C + threadIdx.x] : b * C + threadIdx.x) * D;
  __syncthreads();
  const float* ub = user + (size_t)b * D;
  float a = 0.f;
  const float* cw = rowp[w];
  for (int d = lane; d < D; d += 64) a += cw[d] * ub[d];
  a = wave_sum(a);
  if (lane == 0) zs[w] = a;
  __syncthreads();
  if (w == 0) {
    const bool on = lane < C;
    const float z = on ? zs[lane] : 0.f;
    const float sc = sigm ? 1.0f / (1.0f + __expf(-z)) : z;
    const float mx = wave_max(on ? sc : -INFINITY);
    const float se = wave_sum(on ? __expf(sc - mx) : 0.f);
    if (on) {
      scores[(size_t)b * C + lane] = sc;
      const float ds = (__expf(sc - mx) / se - (lane == 0 ? 1.f : 0.f)) / (float)B;
      dzs[lane] = sigm ? ds * sc * (1.f - sc) : ds;
      if (lane == 0) {  // per-impression share
        const float lb = (mx + __logf(se) - sc) / (float)B;
        if (cnt != nullptr) st_sc1(loss + b, lb);
        else loss[b] = lb;
      }
    }
  }
  __syncthreads();
  const float dzw = dzs[w];
  for (int d = lane; d < D; d += 64) dcand[((size_t)b * C + w) * D + d] = dzw * ub[d];
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float du = 0.f;
    for (int c = 0; c < C; ++c) du += dzs[c] * rowp[c][d];
    duser[(size_t)b * D + d] = du;
  }
  // the batch loss: the last impression block to finish sums the shares -- wave 0, every lane's
  // loads in flight at once (a one-lane loop pays a memory round trip per impression), then a
  // fixed-order shuffle tree (deterministic)
  if (cnt != nullptr && last_arrival(cnt, gridDim.x) && threadIdx.x < 64) {
    float t = 0.f;
    for (int i = threadIdx.x; i < B; i += 64) t += ld_sc1(loss + i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (threadIdx.x == 0) loss_total[0] = t;
  }
}

__device__ unsigned g_score_cnt[1];  // zero-initialised; every launch leaves it zero

int g_score_variant = 1;  // 1: block per impression (default), 0: wave per impression

}  // namespace

extern "C" void fr_score_set_variant(int v) { g_score_variant = v; }

// loss_total (optional): the batch loss sum_b loss[b], formed by the last block (block form only;
// else the caller sums loss[])
extern "C" int fr_score_ce(const float* cand, const float* user, float* loss, float* scores, float* dcand,
                           float* duser, int B, int C, int D, int sigm, const int* ci, float* loss_total,
                           hipStream_t s) {
  if (C > MAXC) return 1;
  if (B == 0) return 0;
  if (ci != nullptr || (g_score_variant == 1 && C <= MAXC)) {
    static unsigned* cnt = [] {
      unsigned* p = nullptr;
      (void)hipGetSymbolAddress((void**)&p, HIP_SYMBOL(g_score_cnt));
      return p;
    }();
    hipLaunchKernelGGL(score_ce_block_kernel, dim3(B), dim3(64 * C), 0, s, cand, user, loss, scores, dcand, duser, B,
                       C, D, sigm, ci, loss_total, loss_total != nullptr ? cnt : nullptr);
    return 0;
  }
  if (loss_total != nullptr) return 2;
  else
    hipLaunchKernelGGL(score_ce_kernel, dim3((B + 3) / 4), dim3(256), 0, s, cand, user, loss, scores, dcand, duser, B,
                       C, D, sigm);
  return 0;
}
