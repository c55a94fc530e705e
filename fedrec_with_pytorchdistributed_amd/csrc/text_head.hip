// The text head of the news encoder, fused over gathered backbone hidden states (gfx950).
//
// Reference (encoder.py:27-29, attention.py:14-26): for a title's
// last hidden state x [T, D] (D = 768, T = 50)
//     e_t = tanh(W1 x_t + b1)          W1 [Q, D], Q = 384
//     a_t = w2 . e_t + b2              alpha = exp(a) / (sum_t exp(a) + 1e-8)
//     pooled = sum_t alpha_t x_t       -> fc [400, D] (small_gemm.hip, not here)
//
// The frozen backbone's hidden states sit in an HBM cache [N, T, D] bf16 (train/news_cache.py)
// and a step needs the U ~ 1.6k unique titles of its batch.  Round 2 materialised them with a
// gather (128 MB), ran att_fc1 as a plain GEMM that wrote e (64 MB), re-read x and e in the pool,
// wrote dpre = da w2 (1 - e^2) (64 MB) in the pool backward and re-read dpre and x in the weight
// gradient: ~290 us of the 0.8 ms step was the same rows going through HBM five times.  Here:
//
//   head_score   A rows loaded straight from the cache by title index (row m -> cache row
//                ids[m / T] * T + m % T, per-lane glds source address), the whole Q = 384 in
//                one block (128 x 384 tile, 8 waves) so the epilogue forms the score
//                a_m = w2 . tanh(acc + b1) + b2 in registers (cross-lane + LDS reduction);
//                e is stored once in bf16 for the backward.
//   head_pool    per title: eps-softmax of a (optional token mask) and pooled = sum alpha x
//                (x read through the same index).
//   head_pool_bwd  per title: dalpha_t = g . x_t, da_t = alpha_t (dalpha_t - sum alpha dalpha).
//   head_wgrad   dW1[q][k] = w2[q] sum_m da_m (1 - e_mq^2) x_mk: a split-K TN MFMA GEMM whose
//                dY operand is FORMED IN ITS LDS PIPELINE -- the raw e tile and the da values
//                arrive by glds, one pass per stage rewrites the e tile in place as
//                g = da (1 - e^2) (bf16) while accumulating the dw2 = sum da e and
//                db1 = w2 sum g column sums; no dpre tensor exists.  w2[q] is applied to the
//                fp32 result in the split-K reduction.
//
// Requirements (host-checked in binding.cpp): D % 256 == 0, Q in {128, 256, 384}, T <= 128 (T <= 96
// at D = 1024).  Q = 384 (DistilBERT) takes the G path below; Q = 128 / 256 the round-4 head_wgrad.
#include "common.h"
#include "gemm_batch.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace {

constexpr int MAXT = 128;

__device__ __forceinline__ float tanh_fast(float x) {  // 1 - 2 / (1 + e^{2x}), as gemm_bf16.hip
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + e);
}

__device__ __attribute__((aligned(16))) bf16 g_zero_row[512];  // zero-initialised (bss)
__device__ float g_zero_f32[64];

// cache row of logical row m (title slot m / T, token m % T)
__device__ __forceinline__ const bf16* hrow(const bf16* __restrict__ table, const int* __restrict__ ids, int m, int T,
                                            int D) {
  const int u = m / T;
  const int t = m - u * T;
  const int id = ids != nullptr ? ids[u] : u;
  return table + ((size_t)id * T + t) * D;
}

// LDS accesses as opaque asm: a builtin LDS access after a glds into the same LDS object makes
// the compiler drain vmcnt -- every in-flight stage (gemm_wgrad.hip); completion is ours to wait
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4_t lds_read128(uint32_t addr) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

// -----------------------------------------------------------------------------------------
// head_score2: e = tanh(X W1^T + b1) (bf16, optional), a = e . w2 + b2 (fp32, from the fp32 e).
// The A rows come straight from the cache by title index (row m -> cache row ids[m / T] * T +
// m % T, per-lane glds source addresses); the whole Q sits in one block, so the epilogue forms
// the score in registers (cross-lane + LDS reduction).  512 threads = 8 waves as WMN (rows) x
// WQ (columns), v_mfma_f32_16x16x32_bf16 with W1 as the A operand (a lane ends with 4
// consecutive columns of one row).  The row tile (32 RF rows), the k-tile (BK) and the depth
// of the LDS pipeline (NST stages, NST - 2 in flight while the MFMAs read one) are parameters.
// A stage is XP + WP "pieces" of one wave-instruction each (64 lanes x 16 B = RPP rows of BK
// bf16); wave w issues pieces w, w + 8, ... and pads to PPW pieces with duplicates of the
// first ones (identical bytes to the same LDS address), so every wave counts the same glds per
// stage and the waits are counted (vmcnt) rather than drains.  LDS reads are opaque asm (a
// builtin LDS read after a glds makes the compiler drain vmcnt).  Rows of BK = 32 stages are
// 64 B: chunk c of row r at c ^ ((r >> 2) & 3) keeps a 16-lane ds_read_b128 group on 64
// distinct banks; BK = 64 rows are 128 B with chunk c of row r at c ^ (r & 7) (conflict-free
// ds_read_b128; glds images are lane-linear so the XOR goes on the source).
// -----------------------------------------------------------------------------------------
template <int BK>
__device__ __forceinline__ int hs_swz(int r) {
  return BK == 64 ? (r & 7) : ((r >> 2) & 3);
}

template <int N>
__device__ __forceinline__ void hs_wait_sync() {  // this wave's stage landed except N younger glds, then barrier
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

//
// Q slices (gridDim.y > 1): block (x, y) computes columns [y Q, (y + 1) Q) of e (row stride ldq)
// and the partial score sum_{q in slice} w2_q tanh(.) into a_out[y M + m] (b2 in slice 0); the
// pool adds the slices.  Halving the W1 panel per block (192 of 384 columns) frees the LDS for a
// third stage: two stages in flight while the MFMAs read one.
// SW: staged LDS waits -- the X fragments first, then the W1 fragments in MFMA-row order, and
// row i of the MFMAs waits only for W1 fragment i (lgkmcnt QFW - 1 - i), as head_wgrad's SW.
template <int N>
__device__ __forceinline__ void lgkm_tie(u32x4_t& r) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(r) : "n"(N));
}
__device__ __forceinline__ void lgkm_tie_rt(int n, u32x4_t& r) {  // n folds to a constant once unrolled
  switch (n) {
    case 0: lgkm_tie<0>(r); break;
    case 1: lgkm_tie<1>(r); break;
    case 2: lgkm_tie<2>(r); break;
    case 3: lgkm_tie<3>(r); break;
    case 4: lgkm_tie<4>(r); break;
    case 5: lgkm_tie<5>(r); break;
    case 6: lgkm_tie<6>(r); break;
    default: lgkm_tie<7>(r); break;
  }
}

// ILV (with SW): the next stage's PPW glds pieces are issued between the MFMA rows of this
// stage (one per row) instead of all at once after the barrier -- an LDS-DMA piece costs ~60-185
// issue cycles (MI355X_MICROARCH.md, per-instruction table), ~1,000 per wave per stage that
// otherwise sit between the barrier and the first MFMA.  Standalone (benchmarks/head_bench.py,
// 1600 titles): 192-row tiles 78.0 -> 67.4 us, 160-row tiles 64.8 -> 61.1 us; inside the step
// graph neutral (0.4414 vs 0.4414 ms, profiles/r6_ab_head_ilv.jsonl).  The default; the plain
// form stays for the bitwise test (head_score_set_ilv(0)).
template <int QF, int RF, int BK, int NST, int WQ = 4, bool SW = false, bool ILV = false>
__global__ __launch_bounds__(512, 1) void head_score2_kernel(const bf16* __restrict__ table, const int* __restrict__ ids,
                                                             int M, int T, int D, const bf16* __restrict__ W1,
                                                             const float* __restrict__ b1, const float* __restrict__ w2,
                                                             const float* __restrict__ b2, bf16* __restrict__ e_out,
                                                             float* __restrict__ a_out, int ldq,
                                                             const int* __restrict__ nreal) {
  constexpr int Q = QF * 64;
  {
    const int qs = blockIdx.y;
    W1 += (size_t)qs * Q * D;
    b1 += qs * Q;
    w2 += qs * Q;
    if (e_out != nullptr) e_out += qs * Q;
    a_out += (size_t)qs * M;
  }
  const float b2v = blockIdx.y == 0 ? b2[0] : 0.f;
  constexpr int MR = 32 * RF;       // rows per block
  constexpr int RB = BK * 2;        // LDS row bytes
  constexpr int CPR = BK / 8;       // 16-B chunks per row
  constexpr int RPP = 64 / CPR;     // rows per piece
  constexpr int XP = MR / RPP, PT = XP + Q / RPP;
  constexpr int PPW = (PT + 7) / 8;
  constexpr int ST = (MR + Q) * RB;
  constexpr int KS = BK / 32;       // MFMA k-steps per stage
  constexpr int WMN = 8 / WQ;       // waves along the rows
  constexpr int QFW = Q / 16 / WQ;  // 16-column fragments per wave
  constexpr int RFW = MR / 16 / WMN;  // 16-row fragments per wave
  static_assert(QFW % 2 == 0 && QFW * 16 * WQ == Q && RFW * 16 * WMN == MR, "wave tiling");
  static_assert(MR % RPP == 0 && Q % RPP == 0 && PT >= 8, "piece tiling");
  __shared__ __attribute__((aligned(16))) char smem[NST * ST];
  const int m0 = blockIdx.x * MR;
  if (nreal != nullptr && m0 >= min(M, nreal[0] * T)) return;  // only padded titles' rows (never read)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WQ, wq = wave % WQ;
  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);

  const bf16* src[PPW];
  uint32_t dst[PPW];
  {
    const int lr = lane / CPR, pc = lane % CPR;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      int p = wave + 8 * i;
      p = p < PT ? p : p - PT;
      if (p < XP) {
        const int r = p * RPP + lr;
        int gm = m0 + r;
        gm = gm < M ? gm : M - 1;  // rows past M: any valid row (outputs masked)
        src[i] = hrow(table, ids, gm, T, D) + (pc ^ hs_swz<BK>(r)) * 8;
        dst[i] = (uint32_t)(p * RPP * RB);
      } else {
        const int r = (p - XP) * RPP + lr;
        src[i] = W1 + (size_t)r * D + (pc ^ hs_swz<BK>(r)) * 8;
        dst[i] = (uint32_t)((MR + (p - XP) * RPP) * RB);
      }
    }
  }
  auto issue = [&](int stage, int k0) {
#pragma unroll
    for (int i = 0; i < PPW; ++i)
      __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, src[i] + k0),
                                       LDS_PTR(void, smem + stage * ST + dst[i]), 16, 0, 0);
  };
  auto issue_one = [&](int i, int stage, int k0) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, src[i] + k0),
                                     LDS_PTR(void, smem + stage * ST + dst[i]), 16, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  static_assert(!ILV || (SW && PPW <= KS * QFW), "interleaved issue: one piece per MFMA row");

  f32x4 acc[QFW][RFW];
#pragma unroll
  for (int i = 0; i < QFW; ++i)
#pragma unroll
    for (int j = 0; j < RFW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = D / BK;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s, s * BK);
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (every wave), every wave done with stage kt - 1
    const int younger = nk - 1 - kt;  // stages issued after kt, at most NST - 2
    if (NST >= 4 && younger >= 2) hs_wait_sync<(NST >= 4 ? 2 * PPW : 0)>();
    else if (NST >= 3 && younger >= 1) hs_wait_sync<(NST >= 3 ? PPW : 0)>();
    else hs_wait_sync<0>();
    const bool nxt = kt + NST - 1 < nk;
    const int nst = (kt + NST - 1) % NST, nk0 = (kt + NST - 1) * BK;
    if (!ILV && nxt) issue(nst, nk0);
    const uint32_t As = lds0 + (kt % NST) * ST, Ws = As + MR * RB;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int lc = kk * 4 + fq;
      u32x4_t xr[RFW], wr[QFW];
#pragma unroll
      for (int j = 0; j < RFW; ++j) {
        const int r = wm * 16 * RFW + j * 16 + fr;
        xr[j] = lds_read128(As + r * RB + ((lc ^ hs_swz<BK>(r)) << 4));
      }
#pragma unroll
      for (int i = 0; i < QFW; ++i) {
        const int r = wq * QFW * 16 + i * 16 + fr;
        wr[i] = lds_read128(Ws + r * RB + ((lc ^ hs_swz<BK>(r)) << 4));
      }
      if constexpr (SW) {
        static_assert(QFW <= 8, "lgkmcnt staging");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < QFW; ++i) {
          lgkm_tie_rt(QFW - 1 - i, wr[i]);  // X fragments (issued first) and W1 fragment i landed
          if (i == 0) {
#pragma unroll
            for (int j = 0; j < RFW; ++j) asm volatile("" : "+v"(xr[j]));
          }
#pragma unroll
          for (int j = 0; j < RFW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wr[i]),
                                                                __builtin_bit_cast(bf16x8, xr[j]), acc[i][j], 0, 0, 0);
          if constexpr (ILV) {
            const int pc_ = kk * QFW + i;
            if (pc_ < PPW && nxt) issue_one(pc_, nst, nk0);
          }
        }
        __builtin_amdgcn_s_setprio(0);
        continue;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < RFW; ++j) asm volatile("" : "+v"(xr[j]));  // uses stay after the wait
#pragma unroll
      for (int i = 0; i < QFW; ++i) asm volatile("" : "+v"(wr[i]));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < QFW; ++i)
#pragma unroll
        for (int j = 0; j < RFW; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wr[i]),
                                                              __builtin_bit_cast(bf16x8, xr[j]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  __syncthreads();  // every wave done reading the last stage before the reduction buffer reuses it

  float part[RFW];
#pragma unroll
  for (int j = 0; j < RFW; ++j) part[j] = 0.f;
#pragma unroll
  for (int i = 0; i < QFW; i += 2) {
    float v[2][RFW][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int qb = wq * QFW * 16 + (i + h) * 16 + fq * 4;
      const float4 bb = *(const float4*)(b1 + qb);
      const float4 ww = *(const float4*)(w2 + qb);
#pragma unroll
      for (int j = 0; j < RFW; ++j) {
        v[h][j][0] = tanh_fast(acc[i + h][j][0] + bb.x);
        v[h][j][1] = tanh_fast(acc[i + h][j][1] + bb.y);
        v[h][j][2] = tanh_fast(acc[i + h][j][2] + bb.z);
        v[h][j][3] = tanh_fast(acc[i + h][j][3] + bb.w);
        part[j] += v[h][j][0] * ww.x + v[h][j][1] * ww.y + v[h][j][2] * ww.z + v[h][j][3] * ww.w;
      }
    }
    if (e_out != nullptr) {
#pragma unroll
      for (int j = 0; j < RFW; ++j) {
        const int m = m0 + wm * 16 * RFW + j * 16 + fr;
        store_pair16_if(e_out + (size_t)(m < M ? m : 0) * ldq + wq * QFW * 16 + i * 16, v[0][j], v[1][j], fq, m < M);
      }
    }
  }
  float* red = (float*)smem;
#pragma unroll
  for (int j = 0; j < RFW; ++j) {
    const float s = group4_sum(part[j]);
    if (fq == 0) red[wq * MR + wm * 16 * RFW + j * 16 + fr] = s;
  }
  __syncthreads();
  if (tid < MR && m0 + tid < M) {
    float sa;
    if constexpr (WQ == 4) sa = (red[tid] + red[MR + tid]) + (red[2 * MR + tid] + red[3 * MR + tid]);
    else sa = red[tid] + red[MR + tid];
    a_out[m0 + tid] = sa + b2v;
  }
}

// -----------------------------------------------------------------------------------------
// The pools, load-first (round 3; the first forms that streamed a title's 76.8 KB after a serial
// prologue -- 26 and 31 us per step -- were removed in round 6).  Every thread issues ALL of its X
// chunks first (TPT / TPW registers of 16 B), then works on them:
//   head_pool2      per title u: alpha = eps-softmax(a) (stable form exp(a - m) / (sum + 1e-8
//                   e^-m), masked tokens weight 0) in every wave (no barrier before the weights;
//                   a token's weight reaches the lanes by shuffle), pooled = sum_t alpha_t x_t
//                   (fp32) by TG t-groups x D / 8 column chunks, the t-group sums via LDS.
//   head_pool_bwd2  per title: dalpha_t = g . x_t, da_t = alpha_t (dalpha_t - sum alpha dalpha),
//                   db2 partial = sum_t da_t; six waves over tokens t = w, w + 6, ..., the
//                   per-token wave sums independent chains the compiler interleaves.
// -----------------------------------------------------------------------------------------
template <int TPT>
__global__ __launch_bounds__(384) void head_pool2_kernel(const bf16* __restrict__ table, const int* __restrict__ ids,
                                                         const float* __restrict__ a, const float* __restrict__ a2,
                                                         const int* __restrict__ tokens,
                                                         int T, int D, float* __restrict__ pooled,
                                                         float* __restrict__ alpha, const int* __restrict__ nreal,
                                                         bf16* __restrict__ pooled_b) {
  __shared__ float part[3072];
  const int u = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (nreal != nullptr && u >= nreal[0]) {  // a padded title of a step graph: exact zeros
    for (int d = tid; d < D; d += blockDim.x) {
      pooled[(size_t)u * D + d] = 0.f;
      if (pooled_b != nullptr) pooled_b[(size_t)u * D + d] = f2bf(0.f);
    }
    for (int t = tid; t < T; t += blockDim.x) alpha[(size_t)u * T + t] = 0.f;
    return;
  }
  const int id = ids != nullptr ? ids[u] : u;
  const bf16* xe = table + (size_t)id * T * D;
  const int DC = D >> 3, TG = 384 / DC;
  const int dc = tid % DC, tgr = tid / DC;
  const int tg = tgr < TG ? tgr : TG - 1;  // spare threads (384 % DC != 0) load a valid row, store nothing
  bf16x8 v[TPT];
#pragma unroll
  for (int i = 0; i < TPT; ++i) {
    const int t = tg + TG * i;
    v[i] = *(const bf16x8*)(xe + (size_t)(t < T ? t : T - 1) * D + dc * 8);
  }
  float av[2], m = -INFINITY;
  bool keep[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int t = lane + 64 * c;
    keep[c] = t < T && (tokens == nullptr || tokens[((size_t)id * 2 + 1) * T + t] != 0);
    av[c] = keep[c] ? (a2 != nullptr ? a[(size_t)u * T + t] + a2[(size_t)u * T + t] : a[(size_t)u * T + t]) : -INFINITY;
    m = fmaxf(m, av[c]);
  }
  m = wave_max(m);
  if (!(m > -INFINITY)) m = 0.f;
  float p[2], l = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    p[c] = keep[c] ? __expf(av[c] - m) : 0.f;
    l += p[c];
  }
  const float inv = 1.0f / (wave_sum(l) + 1e-8f * __expf(-m));
  const float al0 = p[0] * inv, al1 = p[1] * inv;
  if (wave == 0) {
    if (lane < T) alpha[(size_t)u * T + lane] = al0;
    if (lane + 64 < T) alpha[(size_t)u * T + lane + 64] = al1;
  }
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < TPT; ++i) {
    const int t = tg + TG * i;
    const float w0 = __shfl(al0, t & 63, 64), w1 = __shfl(al1, t & 63, 64);
    const float w = t < T ? (t < 64 ? w0 : w1) : 0.f;
    if (t < T) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += w * (float)v[i][k];
    }
  }
  if (tgr < TG) {
#pragma unroll
    for (int k = 0; k < 8; ++k) part[tg * D + dc * 8 + k] = acc[k];
  }
  __syncthreads();
  for (int d = tid; d < D; d += 384) {
    float s = 0.f;
    for (int j = 0; j < TG; ++j) s += part[j * D + d];
    pooled[(size_t)u * D + d] = s;
    if (pooled_b != nullptr) pooled_b[(size_t)u * D + d] = f2bf(s);  // the fc GEMM's operand rounding
  }
}

template <int TPW>
__global__ __launch_bounds__(384) void head_pool_bwd2_kernel(const bf16* __restrict__ table,
                                                             const int* __restrict__ ids,
                                                             const float* __restrict__ alpha,
                                                             const float* __restrict__ g, int T, int D,
                                                             float* __restrict__ da, float* __restrict__ db2p,
                                                             const int* __restrict__ nreal) {
  __shared__ float dal[MAXT];
  const int u = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (nreal != nullptr && u >= nreal[0]) {  // a padded title: no gradient
    for (int t = tid; t < T; t += blockDim.x) da[(size_t)u * T + t] = 0.f;
    if (tid == 0) db2p[u] = 0.f;
    return;
  }
  const int id = ids != nullptr ? ids[u] : u;
  const bf16* xe = table + (size_t)id * T * D;
  const float* gu = g + (size_t)u * D;
  const int DC = D >> 3;
  bf16x8 v[TPW][2];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wave + 6 * i;
    const bf16* row = xe + (size_t)(t < T ? t : T - 1) * D;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int dc = lane + 64 * c;
      v[i][c] = *(const bf16x8*)(row + (dc < DC ? dc : 0) * 8);
    }
  }
  float gv[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int dc = lane + 64 * c;
    const float4 g0 = dc < DC ? *(const float4*)(gu + dc * 8) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 g1 = dc < DC ? *(const float4*)(gu + dc * 8 + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    gv[c][0] = g0.x; gv[c][1] = g0.y; gv[c][2] = g0.z; gv[c][3] = g0.w;
    gv[c][4] = g1.x; gv[c][5] = g1.y; gv[c][6] = g1.z; gv[c][7] = g1.w;
  }
  float s[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    s[i] = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (lane + 64 * c < DC) {
#pragma unroll
        for (int k = 0; k < 8; ++k) s[i] += (float)v[i][c][k] * gv[c][k];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TPW; ++i) s[i] = wave_sum(s[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < TPW; ++i)
      if (wave + 6 * i < T) dal[wave + 6 * i] = s[i];
  }
  __syncthreads();
  if (wave == 0) {
    float al[2], dv[2], sm = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int t = lane + 64 * c;
      al[c] = t < T ? alpha[(size_t)u * T + t] : 0.f;
      dv[c] = t < T ? dal[t] : 0.f;
      sm += al[c] * dv[c];
    }
    sm = wave_sum(sm);
    float sd = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int t = lane + 64 * c;
      const float val = al[c] * (dv[c] - sm);
      if (t < T) da[(size_t)u * T + t] = val;
      sd += val;
    }
    sd = wave_sum(sd);
    if (lane == 0) db2p[u] = sd;
  }
}

// =========================================================================================
// head_wgrad: P[s][q][k] = sum_{m in split s} g_mq x_mk with g = da_m (1 - e_mq^2), formed in
// the LDS pipeline; dw2 / dsum partials [s][q] from blocks of the first k tile.
//
// Tile 128 (q) x 256 (k), 512 threads = 8 waves as 2 (q) x 4 (k), 64 x 64 per wave (4 x 4 MFMA
// tiles; operands are M-major, so fragments are read with ds_read_b64_tr_b16 exactly as
// gemm_wgrad.hip).  Stage = 32 rows: E [32 x 256 B] (raw e, then g), X [32 x 512 B] (cache rows
// by index), DA [8 waves x 64 floats] (each wave stages the 32 da values its transform threads
// read, so every wave issues the same 4 glds per stage and counted vmcnt waits hold).
// Four stages: in iteration st the MFMAs read stage st, stage st+1 is rewritten (e -> g), st+2
// is in flight and st+3 is issued.  One barrier per iteration.
// =========================================================================================
constexpr int WQT = 128, WKT = 256, WTM = 32;
constexpr int E_BYTES = WTM * WQT * 2;         // 8 KB
constexpr int X_BYTES = WTM * WKT * 2;         // 16 KB
constexpr int DA_BYTES = 8 * 64 * 4;           // 2 KB
constexpr int WSTAGE = E_BYTES + X_BYTES + DA_BYTES;
constexpr int MAX_SPLIT_TITLES = 1024;  // title ids of one split, staged in LDS up front

// (more opaque LDS accesses, see lds_read128)
__device__ __forceinline__ s16x4 tr_read(uint32_t addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ float lds_read32(uint32_t addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ int lds_read32i(uint32_t addr) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ void lds_write128(uint32_t addr, u32x4_t v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

__device__ __forceinline__ int swz(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }

// ids_lds: LDS byte address of the split's title ids (title u at ids_lds + 4 (u - u_lo)): a
// global load of ids[] here would be an ordinary load whose use makes the compiler wait
// vmcnt(0) -- draining every glds stage in flight
__device__ __forceinline__ void wg_stage(char* base, const bf16* __restrict__ e, const bf16* __restrict__ table,
                                         uint32_t ids_lds, int u_lo, const float* __restrict__ da, int T, int D,
                                         int Q, int q0, int k0, int m, int me, int wave, int lane) {
  // E: 8 pieces of 4 rows x 16 chunks (one per wave)
  {
    const int row = wave * 4 + (lane >> 4), pc = lane & 15;
    const int c = pc ^ swz(row);
    const int gm = m + row;
    const bf16* p = gm < me ? e + (size_t)gm * Q + q0 + 8 * c : g_zero_row + 8 * c;
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, p), LDS_PTR(void, base + wave * 1024), 16, 0, 0);
  }
  // X: 16 pieces of 2 rows x 32 chunks (two per wave), rows from the cache by title index
  const int rsub = lane >> 5, pc = lane & 31;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = wave * 2 + i;
    const int row = 2 * blk + rsub;
    const int c = pc ^ swz(row);
    const int gm = m + row;
    const bf16* p = g_zero_row + 8 * c;
    if (gm < me) {
      const int u = gm / T;
      const int id = lds_read32i(ids_lds + 4 * (u - u_lo));
      p = table + ((size_t)id * T + (gm - u * T)) * D + k0 + 8 * c;
    }
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, p), LDS_PTR(void, base + E_BYTES + blk * 1024), 16, 0,
                                     0);
  }
  // DA: this wave's copy (lanes 0..31 = rows; lanes 32..63 duplicate)
  {
    const int gm = m + (lane & 31);
    const float* p = gm < me ? da + gm : g_zero_f32;
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, p), LDS_PTR(void, base + E_BYTES + X_BYTES + wave * 256), 4,
                                     0, 0);
  }
}

__device__ __forceinline__ uint32_t tr_off_e(int r0, int col0, int q, int p) {  // 256-B rows
  const int c = (col0 >> 3) + (p >> 1);
  const int r = r0 + q;
  return (uint32_t)(r * 256 + ((c ^ swz(r)) << 4) + (p & 1) * 8);
}
__device__ __forceinline__ uint32_t tr_off_x(int r0, int col0, int q, int p) {  // 512-B rows
  const int c = (col0 >> 3) + (p >> 1);
  const int r = r0 + q;
  return (uint32_t)(r * 512 + ((c ^ swz(r)) << 4) + (p & 1) * 8);
}

#define LGKM_TIE8(r)                                                                                  \
  asm volatile("s_waitcnt lgkmcnt(0)"                                                                 \
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), \
                 "+v"(r[7]))

__device__ __forceinline__ bf16x8 join(s16x4 a, s16x4 b) {
  bf16x4 x = __builtin_bit_cast(bf16x4, a), y = __builtin_bit_cast(bf16x4, b);
  return bf16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

// stage landed for this wave except `inflight` younger stages (4 glds each), then barrier
__device__ __forceinline__ void wg_sync(int inflight) {
  __builtin_amdgcn_sched_barrier(0);
  if (inflight >= 4) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if (inflight == 3) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if (inflight == 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if (inflight == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// rewrite this thread's 16-B chunk of a stage's E tile: e -> g = da (1 - e^2) (bf16); STATS:
// accumulate dw2 += da e and dsum += g (the rounded g the GEMM consumes) for its 8 columns
template <bool STATS>
__device__ __forceinline__ void wg_transform(uint32_t base, int tid, int wave, float (&dw2)[8], float (&dsum)[8]) {
  const int r = tid >> 4, pc = tid & 15;
  const uint32_t ea = base + r * 256 + pc * 16;
  u32x4_t v = lds_read128(ea);
  float dav = lds_read32(base + E_BYTES + X_BYTES + wave * 256 + r * 4);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v), "+v"(dav));
  const bf16x8 ev = __builtin_bit_cast(bf16x8, v);
  bf16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float f = (float)ev[k];
    o[k] = f2bf(dav * (1.0f - f * f));
    if constexpr (STATS) {
      dw2[k] += dav * f;
      dsum[k] += (float)o[k];
    }
  }
  lds_write128(ea, __builtin_bit_cast(u32x4_t, o));
}

// IL (the default): the e -> g rewrite of stage st+1 no longer runs as its own LDS round trip
// in front of stage st's MFMAs (25 us of the 128 in isolation: the in-LDS-pass form measured 104);
// its two LDS reads join the fragment reads, one wait covers both, and its VALU work is spread
// between the MFMA groups (the MFMAs do not depend on it), its write after them.  The column
// sums dw2 / db1 accumulate in every block (a few FMAs) and only the k-tile-0 blocks store them.
//
// SW (staged waits, with IL; the default): the stage's LDS reads go out in the order the MFMA groups consume
// them -- the transform's e chunk and da first, the 8 X fragment halves, then g fragment i --
// and each group waits only for its own reads (lgkmcnt 6 / 4 / 2 / 0: LDS reads retire in
// order), so group 0's MFMAs start while the reads of groups 1-3 are still in the LDS queue
// (the 8 waves leave one barrier together and all want the LDS at once).
template <int NSTAGE, bool IL = false, bool SW = false>
__global__ __launch_bounds__(512, 1) void head_wgrad_kernel(const bf16* __restrict__ e, const bf16* __restrict__ table,
                                                            const int* __restrict__ ids, const float* __restrict__ da,
                                                            int M, int T, int D, int Q, float* __restrict__ P,
                                                            float* __restrict__ dw2p, float* __restrict__ dsump,
                                                            int tiles_k, int ntiles, int mchunk, int no_transform,
                                                            const int* __restrict__ nreal) {
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * WSTAGE + 4 * MAX_SPLIT_TITLES];
  // XCD-aware order: all tiles of one split (same e / x row panel) on one XCD's L2
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, qq = nwg >> 3, rmd = nwg & 7;
  const int t = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (bid >> 3);
  const int s = t / ntiles, tile = t - s * ntiles;
  const int qt = tile / tiles_k, kt = tile - qt * tiles_k;
  const int q0 = qt * WQT, k0 = kt * WKT;
  // a padded step graph: rows past the real titles' carry no gradient -- re-split the real rows
  // over the same grid (no split grows past the host's chunk, so the LDS id table still fits)
  if (nreal != nullptr) {
    M = min(M, nreal[0] * T);
    const int S = nwg / ntiles;
    const int c = ((M + S - 1) / S + WTM - 1) / WTM * WTM;
    mchunk = max(WTM, min(mchunk, c));
  }
  const int mb = s * mchunk;
  const int me = min(M, mb + mchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 2, wk = wave & 3;
  const bool stats = kt == 0 && !no_transform;  // block-uniform
  const bool xform = !no_transform;  // diagnostic A/B: raw e as the dY operand

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float sw2[8], ssum[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sw2[k] = ssum[k] = 0.f;

  const int nsteps = me > mb ? (me - mb + WTM - 1) / WTM : 0;
  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
  // the split's title ids into LDS before any glds is in flight (host guarantees the count fits)
  const int u_lo = mb / T;
  const int u_hi = me > mb ? (me - 1) / T : u_lo;
  int* ids_s = (int*)(smem + NSTAGE * WSTAGE);
  for (int u = u_lo + tid; u <= u_hi; u += 512) ids_s[u - u_lo] = ids != nullptr ? ids[u] : u;
  __syncthreads();
  const uint32_t ids_lds = lds0 + NSTAGE * WSTAGE;
  // NSTAGE buffers: MFMAs read stage st, stage st+1 is being rewritten, NSTAGE-2 are in flight
#pragma unroll
  for (int i = 0; i < NSTAGE - 1; ++i)
    if (i < nsteps)
      wg_stage(smem + i * WSTAGE, e, table, ids_lds, u_lo, da, T, D, Q, q0, k0, mb + i * WTM, me, wave, lane);
  if (nsteps > 0) {
    wg_sync(nsteps - 1 < NSTAGE - 2 ? nsteps - 1 : NSTAGE - 2);  // stage 0 landed
    if (stats || (IL && xform)) wg_transform<true>(lds0, tid, wave, sw2, ssum);
    else if (xform) wg_transform<false>(lds0, tid, wave, sw2, ssum);
  }
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = g * 8;
  uint32_t xo[4][2], yo[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    xo[j][0] = E_BYTES + tr_off_x(r0, wk * 64 + j * 16, q, p);
    xo[j][1] = E_BYTES + tr_off_x(r0 + 4, wk * 64 + j * 16, q, p);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    yo[i][0] = tr_off_e(r0, wn * 64 + i * 16, q, p);
    yo[i][1] = tr_off_e(r0 + 4, wn * 64 + i * 16, q, p);
  }
  for (int st = 0; st < nsteps; ++st) {
    // stage st+1 landed (all waves), stage st fully rewritten (all waves' transform writes,
    // lgkmcnt(0) before the barrier), every wave done reading stage st-1
    const int left = nsteps - 2 - st;  // stages issued beyond st+1
    wg_sync(left < 0 ? 0 : (left > NSTAGE - 3 ? NSTAGE - 3 : left));
    if (st + NSTAGE - 1 < nsteps)
      wg_stage(smem + ((st + NSTAGE - 1) % NSTAGE) * WSTAGE, e, table, ids_lds, u_lo, da, T, D, Q, q0, k0,
               mb + (st + NSTAGE - 1) * WTM, me, wave, lane);
    if constexpr (IL && SW) {
      const bool tr = st + 1 < nsteps && xform;  // block-uniform
      const uint32_t base = lds0 + (st % NSTAGE) * WSTAGE;
      const uint32_t nb = lds0 + ((st + 1) % NSTAGE) * WSTAGE;
      const uint32_t ea = nb + (tid >> 4) * 256 + (tid & 15) * 16;
      // 18 reads whatever tr is (stage st+1's buffer is always a valid LDS address), so the
      // counted waits are immediates
      u32x4_t ev4 = lds_read128(ea);
      float dav = lds_read32(nb + E_BYTES + X_BYTES + wave * 256 + (tid >> 4) * 4);
      s16x4 xr[8], yr[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xr[2 * j] = tr_read(base + xo[j][0]);
        xr[2 * j + 1] = tr_read(base + xo[j][1]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        yr[2 * i] = tr_read(base + yo[i][0]);
        yr[2 * i + 1] = tr_read(base + yo[i][1]);
      }
      asm volatile("s_waitcnt lgkmcnt(6)"
                   : "+v"(ev4), "+v"(dav), "+v"(xr[0]), "+v"(xr[1]), "+v"(xr[2]), "+v"(xr[3]), "+v"(xr[4]),
                     "+v"(xr[5]), "+v"(xr[6]), "+v"(xr[7]), "+v"(yr[0]), "+v"(yr[1]));
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 ev = __builtin_bit_cast(bf16x8, ev4);
      bf16x8 o;
      bf16x8 xb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) xb[j] = join(xr[2 * j], xr[2 * j + 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i == 1) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(yr[2]), "+v"(yr[3]));
        if (i == 2) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(yr[4]), "+v"(yr[5]));
        if (i == 3) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(yr[6]), "+v"(yr[7]));
        const bf16x8 ya = join(yr[2 * i], yr[2 * i + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[j], ya, acc[i][j], 0, 0, 0);
        if (tr) {
#pragma unroll
          for (int k = 2 * i; k < 2 * i + 2; ++k) {
            const float f = (float)ev[k];
            o[k] = f2bf(dav * (1.0f - f * f));
            sw2[k] += dav * f;
            ssum[k] += (float)o[k];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (tr) lds_write128(ea, __builtin_bit_cast(u32x4_t, o));
      __builtin_amdgcn_sched_barrier(0);
      continue;
    }
    if constexpr (IL) {
      const bool tr = st + 1 < nsteps && xform;  // block-uniform
      const uint32_t base = lds0 + (st % NSTAGE) * WSTAGE;
      const uint32_t nb = lds0 + ((st + 1) % NSTAGE) * WSTAGE;
      const uint32_t ea = nb + (tid >> 4) * 256 + (tid & 15) * 16;
      s16x4 xr[8], yr[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xr[2 * j] = tr_read(base + xo[j][0]);
        xr[2 * j + 1] = tr_read(base + xo[j][1]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        yr[2 * i] = tr_read(base + yo[i][0]);
        yr[2 * i + 1] = tr_read(base + yo[i][1]);
      }
      u32x4_t ev4 = u32x4_t{0u, 0u, 0u, 0u};
      float dav = 0.f;
      if (tr) {
        ev4 = lds_read128(ea);
        dav = lds_read32(nb + E_BYTES + X_BYTES + wave * 256 + (tid >> 4) * 4);
      }
      LGKM_TIE8(xr);
      LGKM_TIE8(yr);
      asm volatile("" : "+v"(ev4), "+v"(dav));
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 ev = __builtin_bit_cast(bf16x8, ev4);
      bf16x8 o;
      bf16x8 xb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) xb[j] = join(xr[2 * j], xr[2 * j + 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 ya = join(yr[2 * i], yr[2 * i + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[j], ya, acc[i][j], 0, 0, 0);
#pragma unroll
        for (int k = 2 * i; k < 2 * i + 2; ++k) {  // two of the eight transform elements per MFMA group
          const float f = (float)ev[k];
          o[k] = f2bf(dav * (1.0f - f * f));
          sw2[k] += dav * f;
          ssum[k] += (float)o[k];
        }
      }
      if (tr) lds_write128(ea, __builtin_bit_cast(u32x4_t, o));
      __builtin_amdgcn_sched_barrier(0);
      continue;
    }
    if (st + 1 < nsteps) {
      const uint32_t nb = lds0 + ((st + 1) % NSTAGE) * WSTAGE;
      if (stats) wg_transform<true>(nb, tid, wave, sw2, ssum);
      else if (xform) wg_transform<false>(nb, tid, wave, sw2, ssum);
    }
    const uint32_t base = lds0 + (st % NSTAGE) * WSTAGE;
    s16x4 xr[8], yr[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xr[2 * j] = tr_read(base + xo[j][0]);
      xr[2 * j + 1] = tr_read(base + xo[j][1]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      yr[2 * i] = tr_read(base + yo[i][0]);
      yr[2 * i + 1] = tr_read(base + yo[i][1]);
    }
    LGKM_TIE8(xr);
    LGKM_TIE8(yr);
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 xb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xb[j] = join(xr[2 * j], xr[2 * j + 1]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16x8 ya = join(yr[2 * i], yr[2 * i + 1]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[j], ya, acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  // lane holds P[q][k .. k+3]: q = tile column (lane % 16), k = 4 consecutive (lane / 16)
  float* out = P + (size_t)s * Q * D;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qq2 = q0 + wn * 64 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wk * 64 + j * 16 + 4 * g;
      *(f32x4*)(out + (size_t)qq2 * D + k) = acc[i][j];
    }
  }
  if (stats) {  // column sums over the split's rows: 32 row-threads per 8-column chunk
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float* red = (float*)smem;  // [32 rows][128 q] x 2
    const int r = tid >> 4, lc = (tid & 15) ^ swz(r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[r * WQT + lc * 8 + k] = sw2[k];
      red[WTM * WQT + r * WQT + lc * 8 + k] = ssum[k];
    }
    __syncthreads();
    if (tid < 2 * WQT) {
      const int which = tid / WQT, c = tid % WQT;
      float acc2 = 0.f;
      for (int rr = 0; rr < WTM; ++rr) acc2 += red[which * WTM * WQT + rr * WQT + c];
      (which == 0 ? dw2p : dsump)[(size_t)s * Q + q0 + c] = acc2;
    }
  }
}

// dW1 = w2 (.) sum_s P[s] ; db1 = w2 (.) sum_s dsum[s] ; dw2 = sum_s dw2p[s] ; db2 = sum_u db2p[u]
// (fixed summation order: deterministic).  A block owns 64 float4 of dW1: its 4 waves sum the
// split partials s = w, w+4, ... (independent 16-B loads in flight per lane), then wave 0 adds
// the 4 wave sums in order.  Then Q/64 blocks do dw2 / db1 the same way, the last block db2.
// PB: blocks from head_blocks on run a deferred small-GEMM split-K reduction (gemm_batch.h) --
// the text FC backward's weight gradients, which nothing reads before the optimizer -- so that
// reduction costs no launch of its own
template <bool PB = false>
__global__ __launch_bounds__(256) void head_reduce_kernel(const f32x4* __restrict__ P, const float* __restrict__ dw2p,
                                                          const float* __restrict__ dsump,
                                                          const float* __restrict__ db2p, const float* __restrict__ w2,
                                                          f32x4* __restrict__ dW1, float* __restrict__ db1,
                                                          float* __restrict__ dw2, float* __restrict__ db2, int S, int Q,
                                                          int D, int U, const fr_sg::GemmBatch pb = {},
                                                          int pb_cblocks = 0, int head_blocks = 0) {
  if constexpr (PB) {
    if ((int)blockIdx.x >= head_blocks) {
      fr_sg::splitk_reduce_block(pb, pb_cblocks, (int)blockIdx.x - head_blocks);
      return;
    }
  }
  __shared__ f32x4 part[4][64];
  __shared__ float red[4];
  const long n4 = (long)Q * D / 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if ((long)blockIdx.x * 64 < n4) {
    const long i = (long)blockIdx.x * 64 + lane;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
      int s = wave;
#pragma unroll 4
      for (; s + 12 < S; s += 16) {
        const f32x4 a0 = P[(size_t)s * n4 + i], a1 = P[(size_t)(s + 4) * n4 + i];
        const f32x4 a2 = P[(size_t)(s + 8) * n4 + i], a3 = P[(size_t)(s + 12) * n4 + i];
        v += ((a0 + a1) + (a2 + a3));
      }
      for (; s < S; s += 4) v += P[(size_t)s * n4 + i];
    }
    part[wave][lane] = v;
    __syncthreads();
    if (wave == 0 && i < n4) dW1[i] = ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane])) * w2[(i * 4) / D];
    return;
  }
  const int nmain = (int)((n4 + 63) / 64), nvec = (Q + 63) / 64;
  if ((int)blockIdx.x < nmain + nvec) {  // 64 columns of dw2 / db1, the splits over 4 waves
    const int q = ((int)blockIdx.x - nmain) * 64 + lane;
    float a = 0.f, b = 0.f;
    if (q < Q)
#pragma unroll 4
      for (int s = wave; s < S; s += 4) {
        a += dw2p[(size_t)s * Q + q];
        b += dsump[(size_t)s * Q + q];
      }
    float* pa = (float*)&part[0][0];
    pa[wave * 64 + lane] = a;
    pa[256 + wave * 64 + lane] = b;
    __syncthreads();
    if (wave == 0 && q < Q) {
      dw2[q] = (pa[lane] + pa[64 + lane]) + (pa[128 + lane] + pa[192 + lane]);
      db1[q] = ((pa[256 + lane] + pa[320 + lane]) + (pa[384 + lane] + pa[448 + lane])) * w2[q];
    }
    return;
  }
  float c = 0.f;
  for (int u = threadIdx.x; u < U; u += blockDim.x) c += db2p[u];
  c = wave_sum(c);
  if (lane == 0) red[wave] = c;
  __syncthreads();
  if (threadIdx.x == 0) db2[0] = (red[0] + red[1]) + (red[2] + red[3]);
}

// =========================================================================================
// The G path (round 5): the e -> g = da (1 - e^2) rewrite leaves the weight-gradient GEMM.
// head_wgrad rewrote each E tile in all three K-tile blocks of a split (10 VALU instructions per
// MFMA, 26 % of its wave time; profiles/r4_pmc_stalls_cfg2.json).  Here the pool backward, which
// forms da, also reads the title's e rows once, writes g (bf16, in place over e) and the title's
// column partials dw2_u = sum_t da_t e_tq and dsum_u = sum_t g_tq (the rounded g the GEMM
// consumes); the weight gradient is then a pure TN MFMA stream over G and the cached X rows.
// =========================================================================================

// head_pool_bwd3: head_pool_bwd2 + the g rewrite of title u's e rows + its column partials
// cs[0][u][q] (dw2) and cs[1][u][q] (dsum).  e chunks: Q/8 16-B chunks per row, 384 / (Q/8)
// row groups, ETP rows per thread (loaded first: in flight with the X rows).
template <int TPW, int ETP>
__global__ __launch_bounds__(384) void head_pool_bwd3_kernel(const bf16* __restrict__ table, const int* __restrict__ ids,
                                                             const float* __restrict__ alpha,
                                                             const float* __restrict__ g, int T, int D, int Q,
                                                             float* __restrict__ da, float* __restrict__ db2p,
                                                             bf16* __restrict__ e, float* __restrict__ cs, int U,
                                                             const int* __restrict__ nreal) {
  __shared__ float dal[MAXT];
  __shared__ float dat[MAXT];
  __shared__ float red[2][3072];
  const int u = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* cs0 = cs + (size_t)u * Q;
  float* cs1 = cs + ((size_t)U + u) * Q;
  if (nreal != nullptr && u >= nreal[0]) {  // a padded title: no gradient (its rows are never read)
    for (int t = tid; t < T; t += blockDim.x) da[(size_t)u * T + t] = 0.f;
    for (int q = tid; q < Q; q += blockDim.x) {
      cs0[q] = 0.f;
      cs1[q] = 0.f;
    }
    if (tid == 0) db2p[u] = 0.f;
    return;
  }
  // e rows of this title: loaded once the X rows are consumed (their registers are dead by then;
  // loading both at once took 141 VGPRs and halved the blocks in flight), in flight through the
  // wave sums and the softmax backward
  const int EC = Q >> 3, EG = 384 / EC;
  const int ec = tid % EC, egr = tid / EC;
  const bool eact = egr < EG;
  const int eg = eact ? egr : 0;
  bf16* eu = e + (size_t)u * T * Q;
  bf16x8 ev[ETP];
  const int id = ids != nullptr ? ids[u] : u;
  const bf16* xe = table + (size_t)id * T * D;
  const float* gu = g + (size_t)u * D;
  const int DC = D >> 3;
  bf16x8 v[TPW][2];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wave + 6 * i;
    const bf16* row = xe + (size_t)(t < T ? t : T - 1) * D;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int dc = lane + 64 * c;
      v[i][c] = *(const bf16x8*)(row + (dc < DC ? dc : 0) * 8);
    }
  }
  float gv[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int dc = lane + 64 * c;
    const float4 g0 = dc < DC ? *(const float4*)(gu + dc * 8) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 g1 = dc < DC ? *(const float4*)(gu + dc * 8 + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    gv[c][0] = g0.x; gv[c][1] = g0.y; gv[c][2] = g0.z; gv[c][3] = g0.w;
    gv[c][4] = g1.x; gv[c][5] = g1.y; gv[c][6] = g1.z; gv[c][7] = g1.w;
  }
  float s[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    s[i] = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (lane + 64 * c < DC) {
#pragma unroll
        for (int k = 0; k < 8; ++k) s[i] += (float)v[i][c][k] * gv[c][k];
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < ETP; ++i) {
    const int t = eg + EG * i;
    ev[i] = *(const bf16x8*)(eu + (size_t)(t < T ? t : T - 1) * Q + ec * 8);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < TPW; ++i) s[i] = wave_sum(s[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < TPW; ++i)
      if (wave + 6 * i < T) dal[wave + 6 * i] = s[i];
  }
  __syncthreads();
  if (wave == 0) {
    float al[2], dv[2], sm = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int t = lane + 64 * c;
      al[c] = t < T ? alpha[(size_t)u * T + t] : 0.f;
      dv[c] = t < T ? dal[t] : 0.f;
      sm += al[c] * dv[c];
    }
    sm = wave_sum(sm);
    float sd = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int t = lane + 64 * c;
      const float val = al[c] * (dv[c] - sm);
      if (t < T) {
        da[(size_t)u * T + t] = val;
        dat[t] = val;
      }
      sd += val;
    }
    sd = wave_sum(sd);
    if (lane == 0) db2p[u] = sd;
  }
  __syncthreads();
  // g = da (1 - e^2) in place, column partials over this thread's rows
  float sw2[8], ssum[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sw2[k] = ssum[k] = 0.f;
#pragma unroll
  for (int i = 0; i < ETP; ++i) {
    const int t = eg + EG * i;
    if (eact && t < T) {
      const float dav = dat[t];
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float f = (float)ev[i][k];
        o[k] = f2bf(dav * (1.0f - f * f));
        sw2[k] += dav * f;
        ssum[k] += (float)o[k];
      }
      *(bf16x8*)(eu + (size_t)t * Q + ec * 8) = o;
    }
  }
  if (eact) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[0][eg * Q + ec * 8 + k] = sw2[k];
      red[1][eg * Q + ec * 8 + k] = ssum[k];
    }
  }
  __syncthreads();
  for (int q = tid; q < Q; q += blockDim.x) {
    float a0 = 0.f, a1 = 0.f;
    for (int j = 0; j < EG; ++j) {
      a0 += red[0][j * Q + q];
      a1 += red[1][j * Q + q];
    }
    cs0[q] = a0;
    cs1[q] = a1;
  }
}

// head_wgrad_g: P[s][q][k] = sum_{m in split s} g_mq x_mk -- a plain TN MFMA GEMM (the g tile
// arrives ready in bf16).  Tile 384 (q: the whole head width) x 128 (k), 512 threads = 8 waves
// as 4 (q) x 2 (k) of 96 x 64 (6 x 4 MFMA tiles, 96 accumulators), 4 LDS stages of 32 rows:
// G [32 x 768 B] (3 glds per wave), X [32 x 256 B] (cache rows by title index, 1 glds per wave);
// both read back with ds_read_b64_tr_b16 (M-major operands), 16-B chunks swizzled by swz(row)
// within aligned 16-chunk groups (gemm_wgrad.hip's bank pattern).
//
// The issue budget is the point of this form: at two waves per SIMD a stage is 48 MFMAs (768
// cycles) per SIMD, and the first form spent ~76 VALU instructions per wave per stage on
// addresses (64-bit multiplies, a division by T, 26 LDS address adds) -- more vector issue
// than the MFMAs leave free (profiles/r5_pmc_stalls_head.json: 4.5 VALU per MFMA, 19 % of wave
// time).  Here every per-lane offset is computed once: G sources are a uniform row pointer +
// a 32-bit lane offset, the X row's (title, token) advances by 32 rows per stage with one
// compare, the second read of a fragment is +4 rows (same swizzle) as an immediate offset.
// The G fragments are read a pair at a time, one pair ahead of the MFMAs that use it.
// Splits are whole titles (the column partials are per title): the k-tile blocks of split s
// each sum a 1 / tiles_k share of the 2 Q columns of cs over the split's titles into dw2p /
// dsump[s] after their GEMM.
constexpr int GQT = 384, GKT = 128;
constexpr int G_BYTES = WTM * GQT * 2;  // 24 KB
constexpr int GX_BYTES = WTM * GKT * 2;  // 8 KB
constexpr int GSTB = G_BYTES + GX_BYTES;  // 32 KB

__device__ __forceinline__ uint32_t tr_off_pitch(int pitch, int r0, int col0, int q, int p) {
  const int c = (col0 >> 3) + (p >> 1);
  const int r = r0 + q;
  return (uint32_t)(r * pitch + ((c ^ swz(r)) << 4) + (p & 1) * 8);
}

// a fragment = two ds_read_b64_tr_b16 four rows apart: the second at an immediate offset.
// `a` is early-clobber: the first read's destination must not be the address register the
// second read still needs (the return can land before a queued second read issues).
template <int OFF>
__device__ __forceinline__ void tr_read2(uint32_t addr, s16x4& a, s16x4& b) {
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:%3"
               : "=&v"(a), "=v"(b)
               : "v"(addr), "n"(OFF));
}

template <int N>
__device__ __forceinline__ void lgkm_tie4(s16x4 (&r)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]) : "n"(N));
}

template <int NSTAGE>
__global__ __launch_bounds__(512, 1) void head_wgrad_g_kernel(const bf16* __restrict__ G, const bf16* __restrict__ table,
                                                              const int* __restrict__ ids, const float* __restrict__ cs,
                                                              int U, int T, int D, float* __restrict__ P,
                                                              float* __restrict__ dw2p, float* __restrict__ dsump,
                                                              int tiles_k, int tps, const int* __restrict__ nreal) {
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * GSTB + 4 * MAX_SPLIT_TITLES];
  constexpr int Q = GQT, QF = 6;
  // XCD-aware order: the k-tiles of one split (same G / X row panel) on one XCD's L2
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, qq = nwg >> 3, rmd = nwg & 7;
  const int t = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (bid >> 3);
  const int s = t / tiles_k, kt = t - s * tiles_k;
  const int k0 = kt * GKT;
  int Ur = U;
  if (nreal != nullptr) {  // a padded step graph: the real titles re-split over the same grid
    Ur = min(U, nreal[0]);
    const int S = nwg / tiles_k;
    tps = max(1, min(tps, (Ur + S - 1) / S));
  }
  const int u_lo = min(Ur, s * tps), u_hi = min(Ur, u_lo + tps);  // titles [u_lo, u_hi)
  const int mb = u_lo * T, me = u_hi * T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: LDS destinations in SGPRs
  const int wq = wave >> 1, wk = wave & 1;

  f32x4 acc[QF][4];
#pragma unroll
  for (int i = 0; i < QF; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = me > mb ? (me - mb + WTM - 1) / WTM : 0;
  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
  int* ids_s = (int*)(smem + NSTAGE * GSTB);
  for (int u = u_lo + tid; u < u_hi; u += 512) ids_s[u - u_lo] = ids != nullptr ? ids[u] : u;
  __syncthreads();
  const uint32_t ids_lds = lds0 + NSTAGE * GSTB;

  // ---- per-lane staging constants ----
  // G: 3 pieces per wave, lane-linear LDS; source = row pointer of the stage + lane offset
  int g_row[3];
  uint32_t g_off[3], g_zoff[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int off = (wave * 3 + i) * 1024 + lane * 16;
    const int row = off / 768, c = ((off % 768) >> 4) ^ swz(row);
    g_row[i] = row;
    g_off[i] = (uint32_t)(row * (GQT * 2) + c * 16);
    g_zoff[i] = (uint32_t)(c * 16);
  }
  // X: 1 piece per wave = 4 rows x 16 chunks; the lane's row advances 32 per stage
  const int x_row = wave * 4 + (lane >> 4);
  const int x_c = (lane & 15) ^ swz(x_row);
  const uint32_t x_coff = (uint32_t)(k0 + 8 * x_c);  // bf16 elements within the row
  int x_t = (mb + x_row) % T, x_u = (mb + x_row) / T;  // once per block
  const size_t DD = (size_t)D;
  auto stage = [&](int buf, int m) __attribute__((always_inline)) {
    char* base = smem + buf * GSTB;
    const char* gm_ptr = (const char*)(G + (size_t)m * GQT);  // uniform
    if (m + WTM <= me) {  // every row of the stage is real (uniform): no per-lane select
#pragma unroll
      for (int i = 0; i < 3; ++i)
        __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, gm_ptr + g_off[i]),
                                         LDS_PTR(void, base + (wave * 3 + i) * 1024), 16, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const char* src = (m + g_row[i] < me) ? gm_ptr + g_off[i] : (const char*)g_zero_row + g_zoff[i];
        __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, src), LDS_PTR(void, base + (wave * 3 + i) * 1024), 16,
                                         0, 0);
      }
    }
    const bf16* xs = g_zero_row + 8 * x_c;
    if (m + x_row < me) {
      const int id = lds_read32i(ids_lds + 4 * (x_u - u_lo));
      xs = table + ((size_t)id * T + x_t) * DD + x_coff;
    }
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, xs), LDS_PTR(void, base + G_BYTES + wave * 1024), 16, 0,
                                     0);
    // next stage of this lane's row: 32 rows on
    x_t += WTM;
    while (x_t >= T) {
      x_t -= T;
      ++x_u;
    }
  };
#pragma unroll
  for (int i = 0; i < NSTAGE - 1; ++i)
    if (i < nsteps) stage(i, mb + i * WTM);
  // ---- per-lane fragment offsets (row r0 + q; the +4-row half is an immediate) ----
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = g * 8;
  uint32_t xo[4], yo[QF];
#pragma unroll
  for (int j = 0; j < 4; ++j) xo[j] = G_BYTES + tr_off_pitch(2 * GKT, r0, wk * 64 + j * 16, q, p);
#pragma unroll
  for (int i = 0; i < QF; ++i) yo[i] = tr_off_pitch(2 * GQT, r0, wq * QF * 16 + i * 16, q, p);
  for (int st = 0; st < nsteps; ++st) {
    // stage st landed (this wave's 4 glds, then every wave's); every wave is done with st - 1
    const int left = nsteps - 1 - st;
    const int inflight = left < NSTAGE - 2 ? left : NSTAGE - 2;
    __builtin_amdgcn_sched_barrier(0);
    if (inflight >= 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if (inflight == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const bool nxt = st + NSTAGE - 1 < nsteps;
    const int nbuf = (st + NSTAGE - 1) % NSTAGE;
    if (nxt) stage(nbuf, mb + (st + NSTAGE - 1) * WTM);
    const uint32_t base = lds0 + (st % NSTAGE) * GSTB;
    s16x4 xr[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) tr_read2<4 * 2 * GKT>(base + xo[j], xr[2 * j], xr[2 * j + 1]);
    s16x4 yr[2][4];  // a pair of G fragments (2 reads each), one pair ahead
    tr_read2<4 * 2 * GQT>(base + yo[0], yr[0][0], yr[0][1]);
    tr_read2<4 * 2 * GQT>(base + yo[1], yr[0][2], yr[0][3]);
    bf16x8 xb[4];
#pragma unroll
    for (int ip = 0; ip < QF / 2; ++ip) {
      const int cur = ip & 1;
      if (ip + 1 < QF / 2) {
        tr_read2<4 * 2 * GQT>(base + yo[2 * ip + 2], yr[cur ^ 1][0], yr[cur ^ 1][1]);
        tr_read2<4 * 2 * GQT>(base + yo[2 * ip + 3], yr[cur ^ 1][2], yr[cur ^ 1][3]);
        lgkm_tie4<4>(yr[cur]);
      } else {
        lgkm_tie4<0>(yr[cur]);
      }
      if (ip == 0) {
        asm volatile("" : "+v"(xr[0]), "+v"(xr[1]), "+v"(xr[2]), "+v"(xr[3]), "+v"(xr[4]), "+v"(xr[5]), "+v"(xr[6]),
                     "+v"(xr[7]));
#pragma unroll
        for (int j = 0; j < 4; ++j) xb[j] = join(xr[2 * j], xr[2 * j + 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const bf16x8 ya = join(yr[cur][2 * f], yr[cur][2 * f + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[2 * ip + f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[j], ya, acc[2 * ip + f][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float* out = P + (size_t)s * Q * D;
#pragma unroll
  for (int i = 0; i < QF; ++i) {
    const int qq2 = wq * QF * 16 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wk * 64 + j * 16 + 4 * g;
      *(f32x4*)(out + (size_t)qq2 * D + k) = acc[i][j];
    }
  }
  // column partials: this k-tile's slice of the 2 Q columns (dw2 | dsum) over the split's titles
  const int per = (2 * Q + tiles_k - 1) / tiles_k;
  const int c = kt * per + tid;
  if (tid < per && c < 2 * Q) {
    const int which = c / Q, qc = c - which * Q;
    const float* src = cs + ((size_t)which * U) * Q + qc;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int u = u_lo;
    for (; u + 3 < u_hi; u += 4) {
      a0 += src[(size_t)u * Q];
      a1 += src[(size_t)(u + 1) * Q];
      a2 += src[(size_t)(u + 2) * Q];
      a3 += src[(size_t)(u + 3) * Q];
    }
    for (; u < u_hi; ++u) a0 += src[(size_t)u * Q];
    (which == 0 ? dw2p : dsump)[(size_t)s * Q + qc] = (a0 + a1) + (a2 + a3);
  }
}

int g_cus = 0;
int g_score_ilv = 1;  // head_score2: next stage's pieces interleaved with the MFMA rows
int g_score_rows = 0;  // head_score2 row tile: 0 = by the rounds rule, 160 / 192 forced (benchmarks)

}  // namespace

extern "C" void fr_head_score_set_rows(int r) { g_score_rows = r; }
extern "C" void fr_head_score_set_ilv(int v) { g_score_ilv = v; }

extern "C" int fr_head_supported(int D, int Q, int T) {
  // (head_pool2 holds ceil(T / (384 / (D / 8))) <= 32 rows per thread: D = 1024 up to T = 96)
  return D % 256 == 0 && D <= 1024 && (Q == 128 || Q == 256 || Q == 384) && T >= 1 && T <= MAXT &&
         (T + 384 / (D / 8) - 1) / (384 / (D / 8)) <= 32;
}

extern "C" int fr_head_score(const void* table, const int* ids, int U, int T, int D, int Q, const void* W1,
                             const float* b1, const float* w2, const float* b2, void* e_out, float* a_out,
                             const int* nreal, hipStream_t s) {
  if (!fr_head_supported(D, Q, T)) return 1;
  const int M = U * T;
  if (M == 0) return 0;
  // Q = 384 (the DistilBERT head): 192-row tiles, BK 64, 2 stages, staged LDS waits (steady step
  // 0.5452-0.5473 vs 0.5477-0.5520 ms for one wait, profiles/r3_ab_score_sw.txt; the X-only
  // LDS ring with W1 fragments from L2 ran 100 vs 75 us, profiles/r4_ab_head_score3.txt)
  // Row tile: one block per CU, so the grid runs in ceil(blocks / CUs) rounds, each as long as
  // its block's stages ((rows + 384) x 128 B per k-tile): 160-row tiles when that gives fewer
  // stage bytes over the rounds than 192 (M = 80,000 on 256 CUs: 500 blocks in 2 rounds of 544
  // vs 417 in 2 rounds of 576)
  if (Q == 384) {
    if (g_cus == 0) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (g_cus <= 0) g_cus = 256;
    }
    // a padded step graph (nreal given): blocks past the real titles exit at once, and the real
    // count is the padded one less up to a bucket (128 titles) -- judge the rounds at mid-bucket
    const long Me = nreal != nullptr ? std::max<long>((long)M - 64L * T, (long)T) : (long)M;
    const long rounds192 = ((Me + 191) / 192 + g_cus - 1) / g_cus, rounds160 = ((Me + 159) / 160 + g_cus - 1) / g_cus;
    const bool r160 = g_score_rows == 160 || (g_score_rows == 0 && rounds160 * (160 + 384) < rounds192 * (192 + 384));
#define LAUNCH_S2(RF_, IL_)                                                                                  \
  hipLaunchKernelGGL((head_score2_kernel<6, RF_, 64, 2, 4, true, IL_>), dim3((M + 32 * RF_ - 1) / (32 * RF_)),     \
                     dim3(512), 0, s, (const bf16*)table, ids, M, T, D, (const bf16*)W1, b1, w2, b2, (bf16*)e_out, \
                     a_out, Q, nreal)
    if (r160) {
      if (g_score_ilv) LAUNCH_S2(5, true);
      else LAUNCH_S2(5, false);
    } else {
      if (g_score_ilv) LAUNCH_S2(6, true);
      else LAUNCH_S2(6, false);
    }
#undef LAUNCH_S2
    return 0;
  }
  // Q = 128 / 256 (the tiny test backbones): 128-row tiles, the same pipeline
  if (Q == 256)
    hipLaunchKernelGGL((head_score2_kernel<4, 4, 64, 2, 4, true>), dim3((M + 127) / 128), dim3(512), 0, s,
                       (const bf16*)table, ids, M, T, D, (const bf16*)W1, b1, w2, b2, (bf16*)e_out, a_out, Q, nreal);
  else
    hipLaunchKernelGGL((head_score2_kernel<2, 4, 64, 2, 4, true>), dim3((M + 127) / 128), dim3(512), 0, s,
                       (const bf16*)table, ids, M, T, D, (const bf16*)W1, b1, w2, b2, (bf16*)e_out, a_out, Q, nreal);
  return 0;
}

// score partials per row: head_score writes a[slices][M] (the pool sums the slices); every
// current tiling writes whole scores
extern "C" int fr_head_score_slices(int Q) {
  (void)Q;
  return 1;
}

extern "C" int fr_head_pool(const void* table, const int* ids, const float* a, int slices, const int* tokens, int U,
                            int T, int D, float* pooled, float* alpha, const int* nreal, hipStream_t s,
                            void* pooled_b) {
  const float* a2 = slices == 2 ? a + (size_t)U * T : nullptr;
  if (T > MAXT || D % 8 != 0 || D / 8 > 384) return 1;
  if (U == 0) return 0;
  const int TG = 384 / (D / 8), tpt = (T + TG - 1) / TG;
  if (tpt > 32) return 1;  // (fr_head_supported excludes these shapes)
  {
#define LAUNCH_POOL2(N)                                                                                          \
  hipLaunchKernelGGL(head_pool2_kernel<N>, dim3(U), dim3(384), 0, s, (const bf16*)table, ids, a, a2, tokens, T, D, \
                     pooled, alpha, nreal, (bf16*)pooled_b)
    if (tpt <= 13) LAUNCH_POOL2(13);
    else if (tpt <= 16) LAUNCH_POOL2(16);
    else LAUNCH_POOL2(32);
#undef LAUNCH_POOL2
    return 0;
  }
  return 0;
}

extern "C" int fr_head_pool_bwd(const void* table, const int* ids, const float* alpha, const float* g, int U, int T,
                                int D, float* da, float* db2p, const int* nreal, hipStream_t s) {
  if (T > MAXT || D % 8 != 0 || D / 8 > 128) return 1;
  if (U == 0) return 0;
  const int tpw = (T + 5) / 6;  // <= 22 at T <= MAXT
  {
#define LAUNCH_PBWD2(N)                                                                                           \
  hipLaunchKernelGGL(head_pool_bwd2_kernel<N>, dim3(U), dim3(384), 0, s, (const bf16*)table, ids, alpha, g, T, D, \
                     da, db2p, nreal)
    if (tpw <= 9) LAUNCH_PBWD2(9);
    else if (tpw <= 11) LAUNCH_PBWD2(11);
    else LAUNCH_PBWD2(22);
#undef LAUNCH_PBWD2
    return 0;
  }
  return 0;
}

// scratch = null: returns the fp32 scratch element count needed; else launches.
extern "C" long fr_head_wgrad(const void* e, const void* table, const int* ids, const float* da, const float* db2p,
                              const float* w2, int U, int T, int D, int Q, float* dW1, float* db1, float* dw2,
                              float* db2, float* scratch, const int* nreal, hipStream_t s) {
  if (!fr_head_supported(D, Q, T)) return -1;
  const int M = U * T;
  if (g_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 256;
  }
  const int tiles_k = D / WKT, ntiles = (Q / WQT) * tiles_k;
  // one wave of blocks (one per CU), each split >= 8 stages of 32 rows.  The first form left
  // 16 CUs out for the lookahead stream's sampler / dedup, which then still ran beside this
  // kernel (a block that could not be placed beside them started a wave late: 168 vs 117 us).
  // The register-bitonic dedup (30 us) finishes before this kernel starts, so every CU gets a
  // block: 28 splits vs 26 measured 0.5709 / 0.5707 vs 0.5780 / 0.5791 ms per step (A/B/A/B,
  // profiles/r3_ab_wgrad_splits.txt)
  int S = g_cus / ntiles;
  const int smax = (M + 8 * WTM - 1) / (8 * WTM);
  S = S < 1 ? 1 : (S > smax ? smax : S);
  if (S < 1) S = 1;
  int mchunk = ((M + S - 1) / S + WTM - 1) / WTM * WTM;
  if (mchunk < WTM) mchunk = WTM;
  // a split's title ids (32-row forms) / cache-row table (64-row form) must fit in LDS
  const int cap = (MAX_SPLIT_TITLES - 2) * T / WTM * WTM;
  if (mchunk > cap) mchunk = cap < 64 ? 64 : cap / 64 * 64;
  S = (M + mchunk - 1) / mchunk;
  if (S < 1) S = 1;
  const long need = (long)S * Q * D + 2L * S * Q;
  if (scratch == nullptr) return need;
  float* P = scratch;
  float* dw2p = scratch + (long)S * Q * D;
  float* dsump = dw2p + (long)S * Q;
  // 32-row stages x4 with staged LDS waits: 139 us at U = 1600 vs 146 / 149 for x5 / x6 and
  // 183 for a 64-row form (benchmarks/head_bench.py); staged waits: steady step 0.5498-0.5529
  // vs 0.5509-0.5534 ms over two calls (profiles/r3_ab_wgrad_sw_bump.txt)
  if (M > 0) {
    hipLaunchKernelGGL((head_wgrad_kernel<4, true, true>), dim3(S * ntiles), dim3(512), 0, s, (const bf16*)e,
                       (const bf16*)table, ids, da, M, T, D, Q, P, dw2p, dsump, tiles_k, ntiles, mchunk, 0, nreal);
  } else {
    (void)hipMemsetAsync(scratch, 0, need * sizeof(float), s);
  }
  const long n4 = (long)Q * D / 4;
  const long blocks = (n4 + 63) / 64 + (Q + 63) / 64 + 1;  // dW1 | dw2, db1 | db2
  hipLaunchKernelGGL(head_reduce_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, (const f32x4*)P, dw2p,
                     dsump, db2p, w2, (f32x4*)dW1, db1, dw2, db2, S, Q, D, U, fr_sg::GemmBatch{}, 0, 0);
  return 0;
}

extern "C" int fr_small_gemm_batch_bytes();  // small_gemm.hip

// ---- the G path (round 5) -------------------------------------------------------------------
extern "C" int fr_head_g_supported(int D, int Q, int T) {
  return Q == GQT && D % GKT == 0 && D <= 1024 && T >= 1 && T <= MAXT && fr_head_supported(D, Q, T);
}

// pool backward + g rewrite (e in place) + per-title column partials cs [2][U][Q]
extern "C" int fr_head_pool_bwd_g(const void* table, const int* ids, const float* alpha, const float* g, int U, int T,
                                  int D, int Q, float* da, float* db2p, void* e, float* cs, const int* nreal,
                                  hipStream_t s) {
  if (!fr_head_g_supported(D, Q, T) || D / 8 > 128) return 1;
  if (U == 0) return 0;
  const int tpw = (T + 5) / 6;
  const int EG = 384 / (Q / 8), etp = (T + EG - 1) / EG;
  if (tpw > 22 || etp > 16) return 1;
#define LAUNCH_PBWD3(N, E)                                                                                         \
  hipLaunchKernelGGL((head_pool_bwd3_kernel<N, E>), dim3(U), dim3(384), 0, s, (const bf16*)table, ids, alpha, g, T, \
                     D, Q, da, db2p, (bf16*)e, cs, U, nreal)
  if (tpw <= 9 && etp <= 7) LAUNCH_PBWD3(9, 7);
  else if (tpw <= 11 && etp <= 8) LAUNCH_PBWD3(11, 8);
  else LAUNCH_PBWD3(22, 16);
#undef LAUNCH_PBWD3
  return 0;
}

extern "C" void fr_head_wgrad_g_set_kt(int kt) { (void)kt; }  // one form left (the benchmarks' knob)

// scratch = null: returns the fp32 scratch element count needed; else launches.  G = the g rows
// (the e buffer after the rewrite), cs its column partials.
extern "C" long fr_head_wgrad_g(const void* G, const void* table, const int* ids, const float* cs, const float* db2p,
                                const float* w2, int U, int T, int D, int Q, float* dW1, float* db1, float* dw2,
                                float* db2, float* scratch, const int* nreal, hipStream_t s,
                                const void* pend, int pend_cblocks, int pend_total) {
  // pend (optional): a deferred small-GEMM split-K reduction (fr_small_gemm_take_pending), run
  // in pend_total extra blocks of the reduce launch
  if (!fr_head_g_supported(D, Q, T)) return -1;
  if (g_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 256;
  }
  const int KT = GKT;
  const int tiles_k = D / KT;
  // one block per CU: S splits of whole titles
  int S = g_cus / tiles_k;
  if (S < 1) S = 1;
  int tps = (U + S - 1) / S;
  if (tps < 1) tps = 1;
  if (tps > MAX_SPLIT_TITLES - 2) tps = MAX_SPLIT_TITLES - 2;
  S = U > 0 ? (U + tps - 1) / tps : 1;
  const long need = (long)S * Q * D + 2L * S * Q;
  if (scratch == nullptr) return need;
  float* P = scratch;
  float* dw2p = scratch + (long)S * Q * D;
  float* dsump = dw2p + (long)S * Q;
  if (U > 0) {
    hipLaunchKernelGGL((head_wgrad_g_kernel<4>), dim3(S * tiles_k), dim3(512), 0, s, (const bf16*)G,
                       (const bf16*)table, ids, cs, U, T, D, P, dw2p, dsump, tiles_k, tps, nreal);
  } else {
    (void)hipMemsetAsync(scratch, 0, need * sizeof(float), s);
  }
  const long n4 = (long)Q * D / 4;
  const long blocks = (n4 + 63) / 64 + (Q + 63) / 64 + 1;
  if (pend != nullptr && pend_total > 0) {
    // the descriptor was laid out by small_gemm.o: both objects must agree on GemmBatch
    if (fr_small_gemm_batch_bytes() != (int)sizeof(fr_sg::GemmBatch)) return -2;
    fr_sg::GemmBatch pb;
    memcpy(&pb, pend, sizeof(pb));
    hipLaunchKernelGGL(head_reduce_kernel<true>, dim3((unsigned)(blocks + pend_total)), dim3(256), 0, s,
                       (const f32x4*)P, dw2p, dsump, db2p, w2, (f32x4*)dW1, db1, dw2, db2, S, Q, D, U, pb,
                       pend_cblocks, (int)blocks);
  } else {
    hipLaunchKernelGGL(head_reduce_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, (const f32x4*)P, dw2p,
                       dsump, db2p, w2, (f32x4*)dW1, db1, dw2, db2, S, Q, D, U, fr_sg::GemmBatch{}, 0, 0);
  }
  return 0;
}
