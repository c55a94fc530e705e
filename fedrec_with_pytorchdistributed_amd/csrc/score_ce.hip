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

}  // namespace

extern "C" int fr_score_ce(const float* cand, const float* user, float* loss, float* scores, float* dcand,
                           float* duser, int B, int C, int D, int sigm, hipStream_t s) {
  if (C > MAXC) return 1;
  if (B == 0) return 0;
  hipLaunchKernelGGL(score_ce_kernel, dim3((B + 3) / 4), dim3(256), 0, s, cand, user, loss, scores, dcand, duser, B,
                     C, D, sigm);
  return 0;
}
