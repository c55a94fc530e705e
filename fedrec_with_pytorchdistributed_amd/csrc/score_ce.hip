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

// ---------------------------------------------------------------------------------------
// The user side's tail in one launch (reference attention.py:14-26 + model.py:121-126): one
// block per impression b --
//   additive pool   a_t = w2 . e_t + b2 (masked -> -inf), alpha = eps-softmax(a),
//                   u = sum_t alpha_t x_t                       (x = the MHSA context [T, D])
//   score + CE      as score_ce_block_kernel (candidate rows of the news-vector table by index,
//                   their gradients into dcand, du = sum_c dz_c cand_c, the batch loss by the
//                   last block)
//   pool backward   for du (dctx != null): dalpha_t = x_t . du, da = alpha (dalpha - sum alpha
//                   dalpha), dctx = alpha_t du, dpre = da w2 (1 - e^2) (fp32 + bf16), da as
//                   column 0 of da8 [T B, 8]
// -- three launches (pool forward US blocks per impression, score, pool backward) were 25 us of
// chained latency per config-2 step.  1,024 threads: T <= 64 rows x 16 lanes in the row dots,
// 16 t-groups of the D / 4 float4 columns in the weighted sum (D in [256, 512], Q % 4 == 0),
// C <= 16 candidates (a wave each).
template <int NW>
__global__ __launch_bounds__(NW * 64) void user_pool_score_kernel(
    const float* __restrict__ x, const float* __restrict__ e, const float* __restrict__ w2,
    const float* __restrict__ b2p, const int* __restrict__ keep, const float* __restrict__ cand,
    const int* __restrict__ ci, int B, int T, int D, int Q, int C, int sigm, float* __restrict__ lossb,
    float* __restrict__ scores, float* __restrict__ dcand, float* __restrict__ loss_total,
    unsigned* __restrict__ cnt, float* __restrict__ dctx, float* __restrict__ dpre, bf16* __restrict__ dpre_b,
    float* __restrict__ da8) {
  constexpr int NT = NW * 64, RP = NT / 64;  // RP threads per row in the row-dot phases (T <= 64)
  __shared__ float a_s[64], dal_s[64], part[64];
  __shared__ __attribute__((aligned(16))) float us[512], dus[512];
  __shared__ float4 red[NT / 64][128];  // t-groups x float4 columns (host: NT / 64 <= D / 4 <= 128)
  __shared__ float zs[NW], dzs[NW];
  __shared__ const float* rowp[NW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x;
  const float* xb = x + (size_t)b * T * D;
  const float* eb = e + (size_t)b * T * Q;
  const int D4 = D >> 2, Q4 = Q >> 2;
  if (tid < C) rowp[tid] = cand + (size_t)ci[(size_t)b * C + tid] * D;
  {  // scores a_t: RP lanes per row (float4 columns c = pq, pq + RP, ...), then a 16-lane sum
    const int t = tid / RP, pq = tid % RP;
    float acc = 0.f;
    if (t < T) {
      const float4* er = (const float4*)(eb + (size_t)t * Q);
      const float4* wr = (const float4*)w2;
#pragma unroll 4
      for (int c = pq; c < Q4; c += RP) {
        const float4 v = er[c], ww = wr[c];
        acc += v.x * ww.x + v.y * ww.y + v.z * ww.z + v.w * ww.w;
      }
    }
#pragma unroll
    for (int o = RP / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (pq == 0 && t < 64) part[t] = acc;
  }
  __syncthreads();
  if (w == 0) {  // alpha (stable eps-softmax; every position masked -> all 0)
    float a = -INFINITY;
    if (lane < T) {
      const float v = part[lane] + b2p[0];
      a = (keep == nullptr || keep[(size_t)b * T + lane] != 0) ? v : -INFINITY;
    }
    float m = wave_max(a);
    if (m == -INFINITY) m = 0.f;
    const float p = lane < T ? __expf(a - m) : 0.f;
    const float inv = 1.0f / (wave_sum(p) + 1e-8f * __expf(-m));
    a_s[lane] = p * inv;
  }
  __syncthreads();
  {  // u = sum_t alpha_t x_t: t-groups of D4 float4 columns
    const int G = NT / D4, g = tid / D4, c = tid - g * D4;
    if (g < G) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int t = g; t < T; t += G) {
        const float4 v = ((const float4*)(xb + (size_t)t * D))[c];
        const float al = a_s[t];
        acc.x += al * v.x; acc.y += al * v.y; acc.z += al * v.z; acc.w += al * v.w;
      }
      red[g][c] = acc;
    }
    __syncthreads();
    if (tid < D4) {
      float4 sm = red[0][tid];
      for (int j = 1; j < G; ++j) {
        sm.x += red[j][tid].x; sm.y += red[j][tid].y; sm.z += red[j][tid].z; sm.w += red[j][tid].w;
      }
      ((float4*)us)[tid] = sm;
    }
  }
  __syncthreads();
  if (w < C) {  // z_c = cand_c . u
    float a = 0.f;
    const float* cw = rowp[w];
    for (int d = lane; d < D; d += 64) a += cw[d] * us[d];
    a = wave_sum(a);
    if (lane == 0) zs[w] = a;
  }
  __syncthreads();
  if (w == 0) {  // CE over the C candidates (label 0), as score_ce_block_kernel
    const bool on = lane < C;
    const float z = on ? zs[lane] : 0.f;
    const float sc = sigm ? 1.0f / (1.0f + __expf(-z)) : z;
    const float mx = wave_max(on ? sc : -INFINITY);
    const float se = wave_sum(on ? __expf(sc - mx) : 0.f);
    if (on) {
      scores[(size_t)b * C + lane] = sc;
      const float ds = (__expf(sc - mx) / se - (lane == 0 ? 1.f : 0.f)) / (float)B;
      dzs[lane] = sigm ? ds * sc * (1.f - sc) : ds;
      if (lane == 0) {
        const float lb = (mx + __logf(se) - sc) / (float)B;
        if (cnt != nullptr) st_sc1(lossb + b, lb);
        else lossb[b] = lb;
      }
    }
  }
  __syncthreads();
  if (w < C) {
    const float dzw = dzs[w];
    for (int d = lane; d < D; d += 64) dcand[((size_t)b * C + w) * D + d] = dzw * us[d];
  }
  for (int d = tid; d < D; d += NT) {
    float du = 0.f;
    for (int c = 0; c < C; ++c) du += dzs[c] * rowp[c][d];
    dus[d] = du;
  }
  if (dctx != nullptr) {  // block-uniform: the pool's backward for du
    __syncthreads();
    {  // dalpha_t = x_t . du: RP lanes per row
      const int t = tid / RP, pq = tid % RP;
      float acc = 0.f;
      if (t < T) {
        const float4* xr = (const float4*)(xb + (size_t)t * D);
#pragma unroll 4
        for (int c = pq; c < D4; c += RP) {
          const float4 v = xr[c], g4 = ((const float4*)dus)[c];
          acc += v.x * g4.x + v.y * g4.y + v.z * g4.z + v.w * g4.w;
        }
      }
#pragma unroll
      for (int o = RP / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (pq == 0 && t < 64) part[t] = acc;
    }
    __syncthreads();
    if (w == 0) {
      const float dal = lane < T ? part[lane] : 0.f;
      const float al = lane < T ? a_s[lane] : 0.f;
      const float sdot = wave_sum(al * dal);
      const float da = al * (dal - sdot);
      dal_s[lane] = da;
      if (lane < T) {
        float4* o = (float4*)(da8 + ((size_t)b * T + lane) * 8);
        o[0] = make_float4(da, 0.f, 0.f, 0.f);
        o[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    __syncthreads();
    for (int i = tid; i < T * D4; i += NT) {  // dctx = alpha_t du
      const int t = i / D4, c = i - t * D4;
      const float al = a_s[t];
      const float4 g4 = ((const float4*)dus)[c];
      ((float4*)(dctx + ((size_t)b * T + t) * D))[c] = make_float4(al * g4.x, al * g4.y, al * g4.z, al * g4.w);
    }
    for (int i = tid; i < T * Q4; i += NT) {  // dpre = da w2 (1 - e^2), fp32 and bf16
      const int t = i / Q4, c = i - t * Q4;
      const float da = dal_s[t];
      const float4 v = ((const float4*)(eb + (size_t)t * Q))[c], ww = ((const float4*)w2)[c];
      const float4 dp = make_float4(da * ww.x * (1.f - v.x * v.x), da * ww.y * (1.f - v.y * v.y),
                                    da * ww.z * (1.f - v.z * v.z), da * ww.w * (1.f - v.w * v.w));
      const size_t o = ((size_t)b * T + t) * Q + 4 * c;
      *(float4*)(dpre + o) = dp;
      *(bf16x4*)(dpre_b + o) = bf16x4{f2bf(dp.x), f2bf(dp.y), f2bf(dp.z), f2bf(dp.w)};
    }
  }
  if (cnt != nullptr && last_arrival(cnt, gridDim.x) && tid < 64) {  // the batch loss, impression order
    float tt = 0.f;
    for (int i = tid; i < B; i += 64) tt += ld_sc1(lossb + i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tt += __shfl_xor(tt, o, 64);
    if (tid == 0) loss_total[0] = tt;
  }
}

__device__ unsigned g_ups_cnt[1];  // the fused tail's own ticket (zero between launches)

__device__ unsigned g_score_cnt[1];  // zero-initialised; every launch leaves it zero

int g_score_variant = 1;  // 1: block per impression (default), 0: wave per impression

// The last-arriver tickets above are process-wide __device__ symbols: their address is per
// DEVICE, so it is looked up for the launch's current device (a process that launches on two
// devices gets each one's own counter).  Launches that share one device's counter must not
// overlap (two streams of one device): each launch re-arms it to zero only when its last block
// arrives, so interleaved tickets would hand the sum to the wrong block.  The engine issues
// these launches on one stream per device.
constexpr int MAXDEV = 64;
unsigned* ticket_addr(const void* sym, unsigned* (&cache)[MAXDEV]) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= MAXDEV) dev = 0;
  if (cache[dev] == nullptr) {
    unsigned* p = nullptr;
    (void)hipGetSymbolAddress((void**)&p, sym);
    cache[dev] = p;
  }
  return cache[dev];
}
unsigned* g_score_cnt_addr[MAXDEV] = {};
unsigned* g_ups_cnt_addr[MAXDEV] = {};

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
    unsigned* cnt = ticket_addr(HIP_SYMBOL(g_score_cnt), g_score_cnt_addr);
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

// the user side's tail (user_pool_score_kernel); dctx == null: forward only (validation).
// Returns 1 when the shape is outside the kernel's domain (nothing launched).
extern "C" int fr_user_pool_score(const float* x, const float* e, const float* w2, const float* b2, const int* keep,
                                  const float* cand, const int* ci, int B, int T, int D, int Q, int C, int sigm,
                                  float* lossb, float* scores, float* dcand, float* loss_total, float* dctx,
                                  float* dpre, void* dpre_b, float* da8, hipStream_t s) {
  if (T < 1 || T > 64 || D % 4 || Q % 4 || D < 256 || D > 512 || Q / 4 > 512 || C < 1 || C > 16 ||
      ((uintptr_t)x | (uintptr_t)e | (uintptr_t)w2 | (uintptr_t)(dctx ? dctx : x) | (uintptr_t)(dpre ? dpre : x) |
       (uintptr_t)(da8 ? da8 : x)) & 15 || (dpre_b != nullptr && ((uintptr_t)dpre_b & 7)))
    return 1;
  if (B == 0) return 0;
  unsigned* cnt = ticket_addr(HIP_SYMBOL(g_ups_cnt), g_ups_cnt_addr);
  hipLaunchKernelGGL(user_pool_score_kernel<16>, dim3(B), dim3(1024), 0, s, x, e, w2, b2, keep, cand, ci, B, T, D, Q,
                     C, sigm, lossb, scores, dcand, loss_total, cnt, dctx, dpre, (bf16*)dpre_b, da8);
  return 0;
}
