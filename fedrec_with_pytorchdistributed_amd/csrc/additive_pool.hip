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
// fp32 (user path); statistics and outputs are fp32.  dw2/db2 (and the text kernel's dpre
// column sums) are reduced in LDS per block and stored to the block's own partial row; the
// caller sums the rows with the deterministic colsum kernel (no float atomics).
#include "common.h"

namespace {

constexpr int MAXT = 128;    // vectorised text-head kernels (titles: T = 50)
constexpr int MAXT_G = 2048;  // generic kernels: long user histories (Q6: never truncated)

template <typename T>
__device__ __forceinline__ float ld(const T* p) { return (float)*p; }

// keep (optional, [n, T] int32): position t of sequence n is pooled iff keep[n T + t] != 0 (the
// mask_padding option): its score becomes -inf, so its weight is exactly 0; a sequence with every
// position masked pools to 0 (m := 0), as the torch oracle's masked eps-softmax.  The backward
// needs no mask: it reads the (zero) weights.
template <typename TX>
__global__ __launch_bounds__(256) void pool_fwd_kernel(const TX* __restrict__ x, const TX* __restrict__ e,
                                                       const float* __restrict__ w2, const float* __restrict__ b2,
                                                       float* __restrict__ out, float* __restrict__ alpha_out, int T,
                                                       int D, int Q, const int* __restrict__ keep) {
  __shared__ float a_s[MAXT_G];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const TX* xe = x + (size_t)n * T * D;
  const TX* ee = e + (size_t)n * T * Q;
  // rows interleaved 4 at a time and the t loops unrolled: these kernels are latency-bound
  // (one block per impression, 64 blocks at B = 64), so independent loads must be in flight
#pragma unroll 4
  for (int t = wave; t < T; t += 4) {
    float s = 0.f;
    for (int q = lane; q < Q; q += 64) s += ld(ee + (size_t)t * Q + q) * w2[q];
    s = wave_sum(s);
    if (lane == 0) a_s[t] = (keep == nullptr || keep[(size_t)n * T + t] != 0) ? s + b2[0] : -INFINITY;
  }
  __syncthreads();
  if (wave == 0) {
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, a_s[t]);
    m = wave_max(m);
    if (m == -INFINITY) m = 0.f;
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
      if (blockIdx.y == 0) alpha_out[(size_t)n * T + t] = al;
    }
  }
  __syncthreads();
  // gridDim.y blocks share a sequence (few sequences, e.g. B = 64 impressions): each recomputes
  // the T scores (cheap) and writes its own slice of the D output columns
  const int dspan = (D + gridDim.y - 1) / gridDim.y;
  const int dlo = blockIdx.y * dspan, dhi = min(D, dlo + dspan);
  for (int d = dlo + tid; d < dhi; d += 256) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int t = 0;
#pragma unroll 2
    for (; t + 4 <= T; t += 4)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += a_s[t + j] * ld(xe + (size_t)(t + j) * D + d);
    for (; t < T; ++t) acc[0] += a_s[t] * ld(xe + (size_t)t * D + d);
    out[(size_t)n * D + d] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
}

template <typename TX>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const TX* __restrict__ x, const TX* __restrict__ e,
                                                       const float* __restrict__ alpha, const float* __restrict__ w2,
                                                       const float* __restrict__ g, float* __restrict__ dx,
                                                       TX* __restrict__ dpre, float* __restrict__ dw2,
                                                       float* __restrict__ db2, int T, int D, int Q, int R) {
  __shared__ float da_s[MAXT_G];
  __shared__ float al_s[MAXT_G];
  __shared__ float red[4];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  dw2 += (size_t)(n % R) * Q;  // this block's partial row (R == n)
  db2 += n % R;
  const TX* xe = x + (size_t)n * T * D;
  const TX* ee = e + (size_t)n * T * Q;
  const float* gn = g + (size_t)n * D;
  for (int t = tid; t < T; t += 256) al_s[t] = alpha[(size_t)n * T + t];
  // dalpha_t = x_t . g
#pragma unroll 4
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
  if (tid == 0) *db2 = red[0];
  // dpre and dw2
  for (int q = tid; q < Q; q += 256) {
    const float wq = w2[q];
    float acc = 0.f;
#pragma unroll 8
    for (int t = 0; t < T; ++t) {
      const float ev = ld(ee + (size_t)t * Q + q);
      const float da = da_s[t];
      acc += da * ev;
      dpre[((size_t)n * T + t) * Q + q] = (TX)(da * wq * (1.0f - ev * ev));
    }
    dw2[q] = acc;
  }
  if (dx != nullptr) {
    for (int d = tid; d < D; d += 256) {
      const float gd = gn[d];
#pragma unroll 8
      for (int t = 0; t < T; ++t) dx[((size_t)n * T + t) * D + d] = al_s[t] * gd;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Text-head (bf16) forms with 16-byte accesses: every x / e / dpre access is one bf16x8 per
// lane.  Requires D % 8 == 0, Q % 8 == 0, D/8 <= 128, Q/8 <= 256.
__device__ __forceinline__ void unpack8(const bf16x8 v, float (&f)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = (float)v[k];
}

__global__ __launch_bounds__(256) void pool_fwd16_kernel(const bf16* __restrict__ x, const bf16* __restrict__ e,
                                                         const float* __restrict__ w2, const float* __restrict__ b2,
                                                         float* __restrict__ out, float* __restrict__ alpha_out, int T,
                                                         int D, int Q, const int* __restrict__ keep) {
  __shared__ float a_s[MAXT];
  __shared__ float part[2][1024];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16* xe = x + (size_t)n * T * D;
  const bf16* ee = e + (size_t)n * T * Q;
  const int QC = Q >> 3, DC = D >> 3;
  // a_t = w2 . e_t + b2: one wave per t, lanes over 8-wide q chunks (w2 chunk kept in registers)
  float wq[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int qc = lane + 64 * c;
#pragma unroll
    for (int k = 0; k < 8; ++k) wq[c][k] = qc < QC ? w2[qc * 8 + k] : 0.f;
  }
  for (int t = wave; t < T; t += 4) {
    float sacc = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int qc = lane + 64 * c;
      if (qc < QC) {
        float f[8];
        unpack8(*(const bf16x8*)(ee + (size_t)t * Q + qc * 8), f);
#pragma unroll
        for (int k = 0; k < 8; ++k) sacc += f[k] * wq[c][k];
      }
    }
    sacc = wave_sum(sacc);
    if (lane == 0) a_s[t] = (keep == nullptr || keep[(size_t)n * T + t] != 0) ? sacc + b2[0] : -INFINITY;
  }
  __syncthreads();
  if (wave == 0) {
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, a_s[t]);
    m = wave_max(m);
    if (m == -INFINITY) m = 0.f;
    float l = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float p = __expf(a_s[t] - m);
      a_s[t] = p;
      l += p;
    }
    const float inv = 1.0f / (wave_sum(l) + 1e-8f * __expf(-m));
    for (int t = lane; t < T; t += 64) {
      const float al = a_s[t] * inv;
      a_s[t] = al;
      alpha_out[(size_t)n * T + t] = al;
    }
  }
  __syncthreads();
  // out = sum_t alpha_t x_t: thread (t-group tg of 2, chunk dc) accumulates 8 columns
  const int dc = tid % DC, tg = tid / DC;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (tg < 2) {
    for (int t = tg; t < T; t += 2) {
      float f[8];
      unpack8(*(const bf16x8*)(xe + (size_t)t * D + dc * 8), f);
      const float al = a_s[t];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += al * f[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) part[tg][dc * 8 + k] = acc[k];
  }
  __syncthreads();
  for (int d = tid; d < D; d += 256) out[(size_t)n * D + d] = part[0][d] + part[1][d];
}

__global__ __launch_bounds__(256) void pool_bwd16_kernel(const bf16* __restrict__ x, const bf16* __restrict__ e,
                                                         const float* __restrict__ alpha, const float* __restrict__ w2,
                                                         const float* __restrict__ g, bf16* __restrict__ dpre,
                                                         float* __restrict__ dw2, float* __restrict__ db2,
                                                         float* __restrict__ dsum, int T, int D, int Q, int R) {
  __shared__ float da_s[MAXT];
  __shared__ float al_s[MAXT];
  __shared__ float part[8][256 * 8 / 4];  // per t-group dw2 partials (Q <= 512 for TG >= 4)
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  dw2 += (size_t)(n % R) * Q;  // this block's partial row (R == n)
  db2 += n % R;
  dsum += (size_t)(n % R) * Q;  // column sums of dpre (= the att_fc1 bias gradient)
  const bf16* xe = x + (size_t)n * T * D;
  const bf16* ee = e + (size_t)n * T * Q;
  const float* gn = g + (size_t)n * D;
  const int QC = Q >> 3, DC = D >> 3;
  for (int t = tid; t < T; t += 256) al_s[t] = alpha[(size_t)n * T + t];
  // dalpha_t = x_t . g (g chunks in registers)
  float gv[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int dcc = lane + 64 * c;
#pragma unroll
    for (int k = 0; k < 8; ++k) gv[c][k] = dcc < DC ? gn[dcc * 8 + k] : 0.f;
  }
  for (int t = wave; t < T; t += 4) {
    float sacc = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int dcc = lane + 64 * c;
      if (dcc < DC) {
        float f[8];
        unpack8(*(const bf16x8*)(xe + (size_t)t * D + dcc * 8), f);
#pragma unroll
        for (int k = 0; k < 8; ++k) sacc += f[k] * gv[c][k];
      }
    }
    sacc = wave_sum(sacc);
    if (lane == 0) da_s[t] = sacc;
  }
  __syncthreads();
  if (wave == 0) {
    float sacc = 0.f;
    for (int t = lane; t < T; t += 64) sacc += al_s[t] * da_s[t];
    sacc = wave_sum(sacc);
    float sd = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float v = al_s[t] * (da_s[t] - sacc);
      da_s[t] = v;
      sd += v;
    }
    sd = wave_sum(sd);
    if (lane == 0) *db2 = sd;
  }
  __syncthreads();
  // dpre_t = da_t w2 (1 - e_t^2) (bf16x8 stores); dw2 += sum_t da_t e_t
  const int TG = 256 / QC;
  const int qc = tid % QC, tg = tid / QC;
  float bs[8];
  if (tg < TG) {
    float wv[8], acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      wv[k] = w2[qc * 8 + k];
      acc[k] = 0.f;
      bs[k] = 0.f;
    }
    for (int t = tg; t < T; t += TG) {
      float f[8];
      unpack8(*(const bf16x8*)(ee + (size_t)t * Q + qc * 8), f);
      const float da = da_s[t];
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc[k] += da * f[k];
        o[k] = f2bf(da * wv[k] * (1.0f - f[k] * f[k]));
        bs[k] += (float)o[k];  // the rounded value the dW1 GEMM consumes
      }
      *(bf16x8*)(dpre + ((size_t)n * T + t) * Q + qc * 8) = o;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) part[tg][qc * 8 + k] = acc[k];
  }
  __syncthreads();
  for (int q = tid; q < Q; q += 256) {
    float sacc = 0.f;
    for (int j = 0; j < TG; ++j) sacc += part[j][q];
    dw2[q] = sacc;
  }
  __syncthreads();
  if (tg < TG) {
#pragma unroll
    for (int k = 0; k < 8; ++k) part[tg][qc * 8 + k] = bs[k];
  }
  __syncthreads();
  for (int q = tid; q < Q; q += 256) {
    float sacc = 0.f;
    for (int j = 0; j < TG; ++j) sacc += part[j][q];
    dsum[q] = sacc;
  }
}

// ---------------------------------------------------------------------------------------
// fp32 short-sequence forms (the user encoder's pool: n = B impressions, T = H <= 64, D = 400,
// Q = 200).  The generic kernels above run one block per impression -- 64 blocks at B = 64 --
// and walk rows with a wave-sum per row: ~13 dependent load + reduce rounds per wave, 20 us
// (fwd) / 24 us (bwd) for 7.7 MB.  Here each impression gets US blocks (column / row slices)
// and every phase issues all of a lane's loads at once: row-parallel partial dots (lane =
// (row, quarter of the row)) reduced through LDS, then the weighted sums over t-groups.
constexpr int UT = 64;  // max T
constexpr int US = 4;   // blocks per sequence

// a_t = w2 . e_t + b2 for t < T -> a_s (masked: -inf); lane (t = tid / 4, part = tid % 4)
__device__ __forceinline__ void upool_scores(const float* __restrict__ ee, const float* __restrict__ w2, float b2,
                                             const int* __restrict__ keep_n, int T, int Q, float* a_s,
                                             float (*part)[4]) {
  const int tid = threadIdx.x, t = tid >> 2, pq = tid & 3;
  const int Q4 = Q >> 2, per = (Q4 + 3) >> 2;
  float acc = 0.f;
  if (t < T) {
    const float4* er = (const float4*)(ee + (size_t)t * Q);
    const float4* wr = (const float4*)w2;
#pragma unroll 7
    for (int c = pq * per; c < min(Q4, (pq + 1) * per); ++c) {
      const float4 v = er[c], w = wr[c];
      acc += v.x * w.x + v.y * w.y + v.z * w.z + v.w * w.w;
    }
  }
  part[t][pq] = acc;
  __syncthreads();
  if (tid < T) {
    const float a = (part[tid][0] + part[tid][1]) + (part[tid][2] + part[tid][3]) + b2;
    a_s[tid] = (keep_n == nullptr || keep_n[tid] != 0) ? a : -INFINITY;
  }
  __syncthreads();
}

// in wave 0: a_s -> alpha (eps-softmax, stable form; every position masked -> all 0)
__device__ __forceinline__ void upool_softmax(float* a_s, int T) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x >= 64) return;
  const float a = lane < T ? a_s[lane] : -INFINITY;
  float m = wave_max(a);
  if (m == -INFINITY) m = 0.f;
  const float p = lane < T ? __expf(a - m) : 0.f;
  const float inv = 1.0f / (wave_sum(p) + 1e-8f * __expf(-m));
  if (lane < T) a_s[lane] = p * inv;
}

__global__ __launch_bounds__(256) void upool_fwd_kernel(const float* __restrict__ x, const float* __restrict__ e,
                                                        const float* __restrict__ w2, const float* __restrict__ b2,
                                                        float* __restrict__ out, float* __restrict__ alpha_out, int T,
                                                        int D, int Q, const int* __restrict__ keep) {
  __shared__ float a_s[UT];
  __shared__ float part[UT][4];
  __shared__ float4 red[10][32];
  const int n = blockIdx.x, y = blockIdx.y, tid = threadIdx.x;
  upool_scores(e + (size_t)n * T * Q, w2, b2[0], keep ? keep + (size_t)n * T : nullptr, T, Q, a_s, part);
  upool_softmax(a_s, T);
  __syncthreads();
  if (y == 0 && tid < T) alpha_out[(size_t)n * T + tid] = a_s[tid];
  // out[d] for this block's slice of float4 columns: lane (t-group tg of 10, column c)
  const int D4 = D >> 2, span = (D4 + US - 1) / US, c0 = y * span, nc = min(span, D4 - c0);
  const int tg = tid / 32, c = tid % 32;  // 8 t-groups x 32 columns (span <= 32)
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < nc) {
    const float4* xr = (const float4*)(x + (size_t)n * T * D) + c0 + c;
#pragma unroll 4
    for (int t = tg; t < T; t += 8) {
      const float4 v = xr[(size_t)t * D4];
      const float al = a_s[t];
      acc.x += al * v.x; acc.y += al * v.y; acc.z += al * v.z; acc.w += al * v.w;
    }
  }
  red[tg][c] = acc;
  __syncthreads();
  if (tid < 32 && c < nc) {
    float4 s = red[0][c];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      s.x += red[j][c].x; s.y += red[j][c].y; s.z += red[j][c].z; s.w += red[j][c].w;
    }
    ((float4*)(out + (size_t)n * D))[c0 + c] = s;
  }
}

// grid (n, US): every block forms da (full x . g dots), then its quarter of the rows: dpre,
// the dw2 partial of those rows (partial row n US + y), dx_direct; db2 from block 0 (others 0)
// dpre_b (optional): dpre rounded to bf16 as well -- the operand of the bf16 input-gradient GEMM
// dctx += dpre W1 (the weight gradient keeps the fp32 dpre: its column sums are att_fc1's bias
// gradient, which cancels to a few per cent of the terms' size -- bf16 terms measured 6 % off)
template <bool BF = false>
__global__ __launch_bounds__(256) void upool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ e,
                                                        const float* __restrict__ alpha, const float* __restrict__ w2,
                                                        const float* __restrict__ g, float* __restrict__ dx,
                                                        void* __restrict__ dpre_, float* __restrict__ dw2,
                                                        float* __restrict__ db2, int T, int D, int Q,
                                                        float* __restrict__ da8, bf16* __restrict__ dpre_b = nullptr) {
  float* const dpre = (float*)dpre_;
  __shared__ float da_s[UT], al_s[UT];
  __shared__ float part[UT][4];
  __shared__ float4 red[4][64];
  const int n = blockIdx.x, y = blockIdx.y, tid = threadIdx.x;
  const float* xe = x + (size_t)n * T * D;
  const float* gn = g + (size_t)n * D;
  if (tid < T) al_s[tid] = alpha[(size_t)n * T + tid];
  {  // dalpha_t = x_t . g: lane (t, quarter)
    const int t = tid >> 2, pq = tid & 3, D4 = D >> 2, per = (D4 + 3) >> 2;
    float acc = 0.f;
    if (t < T) {
      const float4* xr = (const float4*)(xe + (size_t)t * D);
      const float4* gr = (const float4*)gn;
#pragma unroll 5
      for (int c = pq * per; c < min(D4, (pq + 1) * per); ++c) {
        const float4 v = xr[c], w = gr[c];
        acc += v.x * w.x + v.y * w.y + v.z * w.z + v.w * w.w;
      }
    }
    part[t][pq] = acc;
  }
  __syncthreads();
  if (tid < 64) {  // wave 0: da_t = alpha_t (dalpha_t - sum alpha dalpha); db2
    const int lane = tid;
    const float dal = lane < T ? (part[lane][0] + part[lane][1]) + (part[lane][2] + part[lane][3]) : 0.f;
    const float al = lane < T ? al_s[lane] : 0.f;
    const float s = wave_sum(al * dal);
    const float da = al * (dal - s);
    if (lane < T) da_s[lane] = da;
    if (da8 != nullptr) {  // da as column 0 of [n T, 8] (the weight-gradient launch reduces it)
      if (y == 0 && lane < T) {
        float4* o = (float4*)(da8 + ((size_t)n * T + lane) * 8);
        o[0] = make_float4(da, 0.f, 0.f, 0.f);
        o[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
      const float sd = wave_sum(da);
      if (lane == 0) db2[(size_t)n * US + y] = y == 0 ? sd : 0.f;
    }
  }
  __syncthreads();
  const int rspan = (T + US - 1) / US, r0 = y * rspan, r1 = min(T, r0 + rspan);
  {  // dpre rows [r0, r1) and their dw2 partial: lane (t-group of 4, float4 column q)
    const int Q4 = Q >> 2, tg = tid >> 6, qc = tid & 63;  // Q4 <= 64
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (qc < Q4) {
      const float4 w = ((const float4*)w2)[qc];
      for (int t = r0 + tg; t < r1; t += 4) {
        const float4 v = ((const float4*)(e + ((size_t)n * T + t) * Q))[qc];
        const float da = da_s[t];
        acc.x += da * v.x; acc.y += da * v.y; acc.z += da * v.z; acc.w += da * v.w;
        const float4 dp = make_float4(da * w.x * (1.f - v.x * v.x), da * w.y * (1.f - v.y * v.y),
                                      da * w.z * (1.f - v.z * v.z), da * w.w * (1.f - v.w * v.w));
        ((float4*)(dpre + ((size_t)n * T + t) * Q))[qc] = dp;
        if constexpr (BF)
          *(bf16x4*)(dpre_b + ((size_t)n * T + t) * Q + 4 * qc) = bf16x4{f2bf(dp.x), f2bf(dp.y), f2bf(dp.z), f2bf(dp.w)};
      }
    }
    if (dw2 != nullptr) {  // block-uniform
      red[tg][qc] = acc;
      __syncthreads();
      if (tid < Q4) {
        float4 s = red[0][tid];
#pragma unroll
        for (int j = 1; j < 4; ++j) {
          s.x += red[j][tid].x; s.y += red[j][tid].y; s.z += red[j][tid].z; s.w += red[j][tid].w;
        }
        ((float4*)(dw2 + ((size_t)n * US + y) * Q))[tid] = s;
      }
    }
  }
  if (dx != nullptr) {  // dx_direct rows [r0, r1) = alpha_t g
    const int D4 = D >> 2;
    const float4* gr = (const float4*)gn;
    for (int i = tid; i < (r1 - r0) * D4; i += 256) {
      const int t = r0 + i / D4, c = i % D4;
      const float4 gv = gr[c];
      const float al = al_s[t];
      ((float4*)(dx + ((size_t)n * T + t) * D))[c] = make_float4(al * gv.x, al * gv.y, al * gv.z, al * gv.w);
    }
  }
}

// the fp32 short-sequence kernels apply (16-byte rows, T <= 64, a block's column slice <= 32
// float4, Q / 4 <= 64)
__host__ __device__ inline bool upool_ok(int T, int D, int Q, int is_bf16) {
  return !is_bf16 && T >= 1 && T <= UT && D % 4 == 0 && Q % 4 == 0 && (D / 4 + US - 1) / US <= 32 && Q / 4 <= 64;
}

}  // namespace

extern "C" int fr_additive_pool_fwd(const void* x, const void* e, const float* w2, const float* b2, float* out,
                                    float* alpha, int n, int T, int D, int Q, int is_bf16, const int* keep,
                                    hipStream_t s) {
  if (T > MAXT_G) return 1;
  if (n == 0) return 0;
  if (upool_ok(T, D, Q, is_bf16) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)e & 15) == 0 && ((uintptr_t)w2 & 15) == 0 &&
      ((uintptr_t)out & 15) == 0)
    hipLaunchKernelGGL(upool_fwd_kernel, dim3(n, US), dim3(256), 0, s, (const float*)x, (const float*)e, w2, b2, out,
                       alpha, T, D, Q, keep);
  else if (is_bf16 && T <= MAXT && D % 8 == 0 && Q % 8 == 0 && D <= 1024 && Q <= 512 && Q >= 256)
    hipLaunchKernelGGL(pool_fwd16_kernel, dim3(n), dim3(256), 0, s, (const bf16*)x, (const bf16*)e, w2, b2, out, alpha,
                       T, D, Q, keep);
  else if (is_bf16)
    hipLaunchKernelGGL(pool_fwd_kernel<bf16>, dim3(n), dim3(256), 0, s, (const bf16*)x, (const bf16*)e, w2, b2, out,
                       alpha, T, D, Q, keep);
  else
    hipLaunchKernelGGL(pool_fwd_kernel<float>, dim3(n, n < 128 ? 4 : (n < 256 ? 2 : 1)), dim3(256), 0, s,
                       (const float*)x, (const float*)e, w2, b2, out, alpha, T, D, Q, keep);
  return 0;
}

// dw2 / db2 point at n partial rows ([n, Q] / [n], R must equal n); the caller sums them.
// dsum ([n, Q]): column sums of dpre, produced only by the vectorised text-head kernel.
// Returns 0 when dsum was produced, -1 when the generic kernel ran (caller reduces dpre),
// > 0 on argument errors.
// partial rows of dw2 / db2 per sequence the backward writes (the caller sizes R = n * this)
extern "C" int fr_additive_pool_rows(int T, int D, int Q, int is_bf16) { return upool_ok(T, D, Q, is_bf16) ? US : 1; }

extern "C" int fr_additive_pool_bwd(const void* x, const void* e, const float* alpha, const float* w2, const float* g,
                                    float* dx, void* dpre, float* dw2, float* db2, float* dsum, int n, int T, int D,
                                    int Q, int R, int is_bf16, hipStream_t s) {
  if (T > MAXT_G) return 1;
  if (n == 0) return -1;
  if (upool_ok(T, D, Q, is_bf16)) {
    if (R != n * US) return 1;
    const uintptr_t al = (uintptr_t)x | (uintptr_t)e | (uintptr_t)w2 | (uintptr_t)g | (uintptr_t)dpre |
                         (uintptr_t)(dx ? dx : g);
    if (al & 15) return 3;  // 16-byte rows (fresh tensors and 256-B aligned parameter views)
    hipLaunchKernelGGL(upool_bwd_kernel<false>, dim3(n, US), dim3(256), 0, s, (const float*)x, (const float*)e, alpha, w2,
                       g, dx, dpre, dw2, db2, T, D, Q, nullptr, nullptr);
    return -1;
  }
  if (R != n) return 1;
  if (is_bf16 && T <= MAXT && dx == nullptr && D % 8 == 0 && Q % 8 == 0 && D <= 1024 && Q <= 512 && Q >= 256) {
    hipLaunchKernelGGL(pool_bwd16_kernel, dim3(n), dim3(256), 0, s, (const bf16*)x, (const bf16*)e, alpha, w2, g,
                       (bf16*)dpre, dw2, db2, dsum, T, D, Q, R);
    return 0;
  }
  if (is_bf16)
    hipLaunchKernelGGL(pool_bwd_kernel<bf16>, dim3(n), dim3(256), 0, s, (const bf16*)x, (const bf16*)e, alpha, w2, g,
                       dx, (bf16*)dpre, dw2, db2, T, D, Q, R);
  else
    hipLaunchKernelGGL(pool_bwd_kernel<float>, dim3(n), dim3(256), 0, s, (const float*)x, (const float*)e, alpha, w2,
                       g, dx, (float*)dpre, dw2, db2, T, D, Q, R);
  return -1;
}

// The user pool's backward without the dw2 / db2 partial rows: da goes out as column 0 of
// da8 [n T, 8] (zeros elsewhere) and the caller adds dw2 = e^T da, db2 = sum da to its weight-
// gradient launch (a small-GEMM desc with M = 8; db2 from that desc's column sums) -- two
// deterministic colsum launches fewer per step.  fp32 short-sequence shapes only (upool_ok).
// dpre_b != nullptr: dpre rounded to bf16 as well (8-byte aligned rows: Q % 4 == 0)
extern "C" int fr_upool_bwd_da(const float* x, const float* e, const float* alpha, const float* w2, const float* g,
                               float* dx, float* dpre, float* da8, int n, int T, int D, int Q, hipStream_t s,
                               void* dpre_b) {
  if (!upool_ok(T, D, Q, 0)) return 1;
  const uintptr_t al = (uintptr_t)x | (uintptr_t)e | (uintptr_t)w2 | (uintptr_t)g | (uintptr_t)dpre |
                       (uintptr_t)(dx ? dx : g) | (uintptr_t)da8 | (uintptr_t)(dpre_b ? dpre_b : dpre);
  if (al & 15) return 3;
  if (n == 0) return 0;
  if (dpre_b != nullptr)
    hipLaunchKernelGGL(upool_bwd_kernel<true>, dim3(n, US), dim3(256), 0, s, x, e, alpha, w2, g, dx, dpre, nullptr,
                       nullptr, T, D, Q, da8, (bf16*)dpre_b);
  else
    hipLaunchKernelGGL(upool_bwd_kernel<false>, dim3(n, US), dim3(256), 0, s, x, e, alpha, w2, g, dx, dpre, nullptr,
                       nullptr, T, D, Q, da8, nullptr);
  return 0;
}
