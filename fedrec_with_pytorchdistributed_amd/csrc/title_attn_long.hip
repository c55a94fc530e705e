// Title self-attention for long sequences, T in (64, 512] (DistilBERT's position table caps
// T at 512; MIND titles are 50, so the hot path is title_attn.hip's T <= 64 MFMA kernels).
// SURVEY §5.7 / §7.5 ask for T limited only by memory; this is that path, forward and
// backward, with the exact HF eager semantics of ops/reference.py:title_attention: a masked
// key scores finfo(f32).min (so an all-masked <unk> title attends uniformly), softmax over
// all T keys, no gradient through masked scores.
//
// One wave per (title, head, 64-row query chunk), lane = query row, fp32 on the VALU with
// K/V streamed through LDS in 64-row chunks (online softmax).  Backward per (title, head):
// pass A (lane = query) recomputes (m, l), then dq = scale (u - D w) with
// u = sum_unmasked A dA k, w = sum_unmasked A k, D = sum_all A dA (dA = dO . v), keeping
// (m, l, D) per row in LDS; pass B (lane = key) streams Q / dO chunks for dk, dv.
#include "common.h"

namespace {

constexpr int DHL = 64;   // head dim (DistilBERT / BERT-base)
constexpr int CHL = 64;   // rows per LDS chunk
constexpr int MAXTL = 512;
constexpr float MASKED = -3.402823466e38f;  // torch.finfo(torch.float32).min

__device__ __forceinline__ void stage_bf16(float (*dst)[DHL + 4], const bf16* __restrict__ src, size_t ld, int r0,
                                           int n, int lane) {
  // rows r0..r0+n-1, DHL bf16 each (8 per 16-B load) -> fp32 LDS rows (padded: 4-float skew)
  for (int i = lane; i < n * (DHL / 8); i += 64) {
    const int r = i / (DHL / 8), c = (i - r * (DHL / 8)) * 8;
    const bf16x8 v = *(const bf16x8*)(src + (size_t)(r0 + r) * ld + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[r][c + k] = (float)v[k];
  }
}

__device__ __forceinline__ void load_row64(float (&x)[DHL], const bf16* __restrict__ p, float s) {
#pragma unroll
  for (int c = 0; c < DHL; c += 8) {
    const bf16x8 v = *(const bf16x8*)(p + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[c + k] = (float)v[k] * s;
  }
}

__device__ __forceinline__ float dot64(const float (&q)[DHL], const float* __restrict__ row) {
  float d = 0.f;
#pragma unroll
  for (int c = 0; c < DHL; c += 4) {
    const float4 k = *(const float4*)(row + c);
    d += q[c] * k.x + q[c + 1] * k.y + q[c + 2] * k.z + q[c + 3] * k.w;
  }
  return d;
}

__device__ __forceinline__ void axpy64(float (&acc)[DHL], float a, const float* __restrict__ row) {
#pragma unroll
  for (int c = 0; c < DHL; c += 4) {
    const float4 v = *(const float4*)(row + c);
    acc[c] += a * v.x;
    acc[c + 1] += a * v.y;
    acc[c + 2] += a * v.z;
    acc[c + 3] += a * v.w;
  }
}

__device__ __forceinline__ void store_row64(bf16* __restrict__ p, const float (&x)[DHL], float s) {
#pragma unroll
  for (int c = 0; c < DHL; c += 8) {
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = f2bf(x[c + k] * s);
    *(bf16x8*)(p + c) = o;
  }
}

// qkv [n*T, 3D] (q | k | v, head h at columns h*64), mask [n, T] (nonzero = keep), out [n*T, D]
__global__ __launch_bounds__(64) void title_attn_long_kernel(const bf16* __restrict__ qkv, const int* __restrict__ mask,
                                                             bf16* __restrict__ out, int T, int H, int D, int nch) {
  __shared__ __attribute__((aligned(16))) float ks[CHL][DHL + 4];
  __shared__ __attribute__((aligned(16))) float vs[CHL][DHL + 4];
  __shared__ float kp[CHL];  // 1 = keep
  const int lane = threadIdx.x;
  const int chunk = blockIdx.x % nch, pair = blockIdx.x / nch;
  const int title = pair / H, h = pair - title * H;
  const size_t ld = 3 * (size_t)D;
  const bf16* base = qkv + (size_t)title * T * ld + h * DHL;
  const int* mk = mask + (size_t)title * T;
  const int t = chunk * CHL + lane;
  const bool valid = t < T;
  float q[DHL], acc[DHL];
  load_row64(q, base + (size_t)(valid ? t : 0) * ld, 0.125f);  // 1/sqrt(64)
#pragma unroll
  for (int c = 0; c < DHL; ++c) acc[c] = 0.f;
  float m = -INFINITY, l = 0.f;
  for (int s0 = 0; s0 < T; s0 += CHL) {
    const int n = min(CHL, T - s0);
    __syncthreads();
    stage_bf16(ks, base + D, ld, s0, n, lane);
    stage_bf16(vs, base + 2 * D, ld, s0, n, lane);
    if (lane < n) kp[lane] = mk[s0 + lane] != 0 ? 1.f : 0.f;
    __syncthreads();
    float mc = m;
    for (int s = 0; s < n; ++s) mc = fmaxf(mc, kp[s] != 0.f ? dot64(q, &ks[s][0]) : MASKED);
    const float alpha = __expf(m - mc);
    l *= alpha;
#pragma unroll
    for (int c = 0; c < DHL; ++c) acc[c] *= alpha;
    for (int s = 0; s < n; ++s) {
      const float p = __expf((kp[s] != 0.f ? dot64(q, &ks[s][0]) : MASKED) - mc);
      l += p;
      axpy64(acc, p, &vs[s][0]);
    }
    m = mc;
  }
  if (valid) store_row64(out + ((size_t)title * T + t) * D + h * DHL, acc, 1.0f / l);
}

__global__ __launch_bounds__(64) void title_attn_bwd_long_kernel(const bf16* __restrict__ qkv,
                                                                 const bf16* __restrict__ dout,
                                                                 const int* __restrict__ mask,
                                                                 bf16* __restrict__ dqkv, int T, int H, int D) {
  __shared__ __attribute__((aligned(16))) float xs[CHL][DHL + 4];  // K (pass A) / Q (pass B)
  __shared__ __attribute__((aligned(16))) float ys[CHL][DHL + 4];  // V (pass A) / dO (pass B)
  __shared__ float ms[MAXTL], ls[MAXTL], Ds[MAXTL], kps[MAXTL];
  const int lane = threadIdx.x;
  const int title = blockIdx.x / H, h = blockIdx.x - title * H;
  const size_t ld = 3 * (size_t)D;
  const bf16* base = qkv + (size_t)title * T * ld + h * DHL;
  const bf16* gb = dout + (size_t)title * T * D + h * DHL;
  bf16* dbase = dqkv + (size_t)title * T * ld + h * DHL;
  const int* mk = mask + (size_t)title * T;
  for (int s = lane; s < T; s += 64) kps[s] = mk[s] != 0 ? 1.f : 0.f;
  const float scale = 0.125f;
  // pass A: lane = query t
  for (int t0 = 0; t0 < T; t0 += CHL) {
    const int t = t0 + lane;
    const bool valid = t < T;
    const int tc = valid ? t : 0;
    float q[DHL], g[DHL];
    load_row64(q, base + (size_t)tc * ld, scale);
    load_row64(g, gb + (size_t)tc * D, 1.f);
    float m = -INFINITY, l = 0.f;
    for (int s0 = 0; s0 < T; s0 += CHL) {  // (m, l) of row t
      const int n = min(CHL, T - s0);
      __syncthreads();
      stage_bf16(xs, base + D, ld, s0, n, lane);
      __syncthreads();
      float mc = m;
      for (int s = 0; s < n; ++s) mc = fmaxf(mc, kps[s0 + s] != 0.f ? dot64(q, &xs[s][0]) : MASKED);
      float lc = 0.f;
      for (int s = 0; s < n; ++s) lc += __expf((kps[s0 + s] != 0.f ? dot64(q, &xs[s][0]) : MASKED) - mc);
      l = l * __expf(m - mc) + lc;
      m = mc;
    }
    const float inv = 1.0f / l;
    float u[DHL], w[DHL];
#pragma unroll
    for (int c = 0; c < DHL; ++c) u[c] = w[c] = 0.f;
    float Dt = 0.f;
    for (int s0 = 0; s0 < T; s0 += CHL) {
      const int n = min(CHL, T - s0);
      __syncthreads();
      stage_bf16(xs, base + D, ld, s0, n, lane);
      stage_bf16(ys, base + 2 * D, ld, s0, n, lane);
      __syncthreads();
      for (int s = 0; s < n; ++s) {
        const bool keep = kps[s0 + s] != 0.f;
        const float A = __expf((keep ? dot64(q, &xs[s][0]) : MASKED) - m) * inv;
        const float dA = dot64(g, &ys[s][0]);
        Dt += A * dA;
        if (keep) {
          axpy64(u, A * dA, &xs[s][0]);
          axpy64(w, A, &xs[s][0]);
        }
      }
    }
    if (!valid) continue;
    ms[t] = m;
    ls[t] = inv;
    Ds[t] = Dt;
#pragma unroll
    for (int c = 0; c < DHL; ++c) u[c] = u[c] - Dt * w[c];
    store_row64(dbase + (size_t)t * ld, u, scale);
  }
  // pass B: lane = key s
  for (int s0 = 0; s0 < T; s0 += CHL) {
    const int s = s0 + lane;
    const bool valid = s < T;
    const int sc = valid ? s : 0;
    const bool keep = kps[sc] != 0.f;
    float k[DHL], v[DHL], dk[DHL], dv[DHL];
    load_row64(k, base + (size_t)sc * ld + D, scale);
    load_row64(v, base + (size_t)sc * ld + 2 * D, 1.f);
#pragma unroll
    for (int c = 0; c < DHL; ++c) dk[c] = dv[c] = 0.f;
    for (int t0 = 0; t0 < T; t0 += CHL) {
      const int n = min(CHL, T - t0);
      __syncthreads();  // also orders pass A's ms / ls / Ds writes before these reads
      stage_bf16(xs, base, ld, t0, n, lane);
      stage_bf16(ys, gb, D, t0, n, lane);
      __syncthreads();
      for (int j = 0; j < n; ++j) {
        const int t = t0 + j;
        const float A = __expf((keep ? dot64(k, &xs[j][0]) : MASKED) - ms[t]) * ls[t];
        const float dA = dot64(v, &ys[j][0]);
        if (keep) axpy64(dk, A * (dA - Ds[t]), &xs[j][0]);
        axpy64(dv, A, &ys[j][0]);
      }
    }
    if (!valid) continue;
    store_row64(dbase + (size_t)s * ld + D, dk, scale);
    store_row64(dbase + (size_t)s * ld + 2 * D, dv, 1.f);
  }
}

}  // namespace

extern "C" int fr_title_attention_long_bf16(const void* qkv, const int* mask, void* out, int n_titles, int T, int H,
                                            int D, hipStream_t s) {
  if (T < 1 || T > MAXTL || D != H * DHL) return 1;
  const int nch = (T + CHL - 1) / CHL, pairs = n_titles * H;
  if (pairs == 0) return 0;
  hipLaunchKernelGGL(title_attn_long_kernel, dim3(pairs * nch), dim3(64), 0, s, (const bf16*)qkv, mask, (bf16*)out, T,
                     H, D, nch);
  return 0;
}

extern "C" int fr_title_attention_bwd_long_bf16(const void* qkv, const void* dout, const int* mask, void* dqkv,
                                                int n_titles, int T, int H, int D, hipStream_t s) {
  if (T < 1 || T > MAXTL || D != H * DHL) return 1;
  const int pairs = n_titles * H;
  if (pairs == 0) return 0;
  hipLaunchKernelGGL(title_attn_bwd_long_kernel, dim3(pairs), dim3(64), 0, s, (const bf16*)qkv, (const bf16*)dout, mask,
                     (bf16*)dqkv, T, H, D);
  return 0;
}
