// User-encoder multi-head self-attention core (reference attention.py:32-82):
//
//   S = Q K^T / sqrt(d_k),  A = exp(S) / (rowsum exp(S) + 1e-8),  ctx = A V
//
// 20 heads x d_k 20 over H <= 64 clicked news, fp32 (the user side is tiny: ~0.5 MFLOP per
// impression and head; it is latency-, not FLOP-bound, so it runs on the VALU with K/V
// broadcast from LDS).  The eps softmax is evaluated stably:
// A = exp(S - m) / (sum exp(S - m) + 1e-8 exp(-m)).  No mask (Q7), like the reference.
//
// Forward: one wave per (impression, head), lane = query row; saves (m, l) per row.
// Backward: lane = query row for dQ and the row term D_t = sum_s A_ts dA_ts, then
// lane = key row for dK = sum_t dS_ts q_t and dV = sum_t A_ts dctx_t (no cross-lane sums).
//
// qkv: [B, H, 3*NH*DK] fp32 (q | k | v; head h at columns h*DK); ctx/dctx: [B, H, NH*DK].
#include "common.h"

namespace {

constexpr int DK = 20;
constexpr int MAXH = 64;

__global__ __launch_bounds__(128) void user_attn_fwd_kernel(const float* __restrict__ qkv, float* __restrict__ ctx,
                                                            float* __restrict__ stats, int B, int H, int NH) {
  __shared__ float ks[2][MAXH][DK + 1];
  __shared__ float vs[2][MAXH][DK + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pair = blockIdx.x * 2 + wave;
  const bool active = pair < B * NH;
  const int b = active ? pair / NH : 0, h = active ? pair - b * NH : 0;
  const int ld = 3 * NH * DK, D = NH * DK;
  const float* base = qkv + (size_t)b * H * ld + h * DK;
  for (int i = lane; i < H * DK; i += 64) {
    const int r = i / DK, c = i - r * DK;
    ks[wave][r][c] = base[(size_t)r * ld + D + c];
    vs[wave][r][c] = base[(size_t)r * ld + 2 * D + c];
  }
  __syncthreads();
  if (!active || lane >= H) return;
  float q[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) q[c] = base[(size_t)lane * ld + c];
  const float scale = rsqrtf((float)DK);
  float m = -INFINITY;
  for (int s = 0; s < H; ++s) {
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < DK; ++c) d += q[c] * ks[wave][s][c];
    m = fmaxf(m, d * scale);
  }
  float acc[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) acc[c] = 0.f;
  float l = 0.f;
  for (int s = 0; s < H; ++s) {
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < DK; ++c) d += q[c] * ks[wave][s][c];
    const float p = __expf(d * scale - m);
    l += p;
#pragma unroll
    for (int c = 0; c < DK; ++c) acc[c] += p * vs[wave][s][c];
  }
  l += 1e-8f * __expf(-m);
  const float inv = 1.0f / l;
  float* o = ctx + ((size_t)b * H + lane) * D + h * DK;
#pragma unroll
  for (int c = 0; c < DK; ++c) o[c] = acc[c] * inv;
  float* st = stats + (((size_t)b * NH + h) * H + lane) * 2;
  st[0] = m;
  st[1] = inv;
}

__global__ __launch_bounds__(64) void user_attn_bwd_kernel(const float* __restrict__ qkv, const float* __restrict__ stats,
                                                           const float* __restrict__ dctx, float* __restrict__ dqkv,
                                                           int B, int H, int NH) {
  __shared__ float qs[MAXH][DK + 1];
  __shared__ float ks[MAXH][DK + 1];
  __shared__ float vs[MAXH][DK + 1];
  __shared__ float gs[MAXH][DK + 1];
  __shared__ float ms[MAXH], is_[MAXH], Ds[MAXH];
  const int lane = threadIdx.x;
  const int pair = blockIdx.x;
  const int b = pair / NH, h = pair - b * NH;
  const int ld = 3 * NH * DK, D = NH * DK;
  const float* base = qkv + (size_t)b * H * ld + h * DK;
  const float* gb = dctx + (size_t)b * H * D + h * DK;
  for (int i = lane; i < H * DK; i += 64) {
    const int r = i / DK, c = i - r * DK;
    qs[r][c] = base[(size_t)r * ld + c];
    ks[r][c] = base[(size_t)r * ld + D + c];
    vs[r][c] = base[(size_t)r * ld + 2 * D + c];
    gs[r][c] = gb[(size_t)r * D + c];
  }
  const float* st = stats + ((size_t)b * NH + h) * H * 2;
  for (int t = lane; t < H; t += 64) {
    ms[t] = st[2 * t];
    is_[t] = st[2 * t + 1];
  }
  __syncthreads();
  const float scale = rsqrtf((float)DK);
  float* dbase = dqkv + (size_t)b * H * ld + h * DK;
  // pass 1: lane = query t -> D_t, dq_t
  if (lane < H) {
    const int t = lane;
    const float m = ms[t], inv = is_[t];
    float Dt = 0.f;
    for (int s = 0; s < H; ++s) {
      float d = 0.f, dA = 0.f;
#pragma unroll
      for (int c = 0; c < DK; ++c) {
        d += qs[t][c] * ks[s][c];
        dA += gs[t][c] * vs[s][c];
      }
      Dt += __expf(d * scale - m) * inv * dA;
    }
    Ds[t] = Dt;
    float dq[DK];
#pragma unroll
    for (int c = 0; c < DK; ++c) dq[c] = 0.f;
    for (int s = 0; s < H; ++s) {
      float d = 0.f, dA = 0.f;
#pragma unroll
      for (int c = 0; c < DK; ++c) {
        d += qs[t][c] * ks[s][c];
        dA += gs[t][c] * vs[s][c];
      }
      const float A = __expf(d * scale - m) * inv;
      const float dS = A * (dA - Dt) * scale;
#pragma unroll
      for (int c = 0; c < DK; ++c) dq[c] += dS * ks[s][c];
    }
    float* o = dbase + (size_t)t * ld;
#pragma unroll
    for (int c = 0; c < DK; ++c) o[c] = dq[c];
  }
  __syncthreads();
  // pass 2: lane = key s -> dk_s, dv_s
  if (lane < H) {
    const int s = lane;
    float dk[DK], dv[DK];
#pragma unroll
    for (int c = 0; c < DK; ++c) dk[c] = dv[c] = 0.f;
    for (int t = 0; t < H; ++t) {
      float d = 0.f, dA = 0.f;
#pragma unroll
      for (int c = 0; c < DK; ++c) {
        d += qs[t][c] * ks[s][c];
        dA += gs[t][c] * vs[s][c];
      }
      const float A = __expf(d * scale - ms[t]) * is_[t];
      const float dS = A * (dA - Ds[t]) * scale;
#pragma unroll
      for (int c = 0; c < DK; ++c) {
        dk[c] += dS * qs[t][c];
        dv[c] += A * gs[t][c];
      }
    }
    float* o = dbase + (size_t)s * ld;
#pragma unroll
    for (int c = 0; c < DK; ++c) {
      o[D + c] = dk[c];
      o[2 * D + c] = dv[c];
    }
  }
}

}  // namespace

extern "C" int fr_user_attn_fwd(const float* qkv, float* ctx, float* stats, int B, int H, int NH, int dk,
                                hipStream_t s) {
  if (dk != DK || H > MAXH || H < 1) return 1;
  const int pairs = B * NH;
  if (pairs == 0) return 0;
  hipLaunchKernelGGL(user_attn_fwd_kernel, dim3((pairs + 1) / 2), dim3(128), 0, s, qkv, ctx, stats, B, H, NH);
  return 0;
}

extern "C" int fr_user_attn_bwd(const float* qkv, const float* stats, const float* dctx, float* dqkv, int B, int H,
                                int NH, int dk, hipStream_t s) {
  if (dk != DK || H > MAXH || H < 1) return 1;
  const int pairs = B * NH;
  if (pairs == 0) return 0;
  hipLaunchKernelGGL(user_attn_bwd_kernel, dim3(pairs), dim3(64), 0, s, qkv, stats, dctx, dqkv, B, H, NH);
  return 0;
}
