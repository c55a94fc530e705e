// bf16 "NT" GEMM with fused epilogues on MFMA (gfx950):
//   C[M,N] = act(A[M,K] . W[N,K]^T + bias[N]) + R[M,N]      (bf16 in/out, fp32 accumulate)
//
// Every DistilBERT linear (fused Q|K|V N=2304, out-proj N=768, FFN1 N=3072 + GELU,
// FFN2 N=768 + residual) and the text head's att_fc1 (N=384 + tanh) run here
// (SURVEY §2.3 K02/K05/K06).  Both operands are K-contiguous, which is the natural
// layout for v_mfma_f32_16x16x32_bf16: each lane's A and B fragments are 16 contiguous
// bytes of one row.
//
// Structure (cdna_hip_programming.md §5, "minimum 2-phase"):
//   * 128x128x64 block tile, 256 threads = 4 waves in 2x2, 64x64 per wave
//     (4x4 MFMA tiles -> 64 accumulator VGPRs);
//   * global -> LDS by global_load_lds_dwordx4 (16 B per lane, no VGPR round trip),
//     two LDS stages (64 KB -> 2 blocks per CU), next tile issued before the MFMAs;
//   * LDS image is lane-linear (a glds constraint), so the bank-conflict XOR swizzle
//     (16-B chunk c of row r stored at chunk c ^ (r & 7)) is applied to the per-lane
//     SOURCE address and undone on the ds_read_b128 address (§5.4 rule 21);
//   * operands swapped (W as the MFMA A operand) so each lane ends with 4 consecutive
//     output columns -> one 8-byte bias load / residual load / store per 4 outputs;
//   * XCD-aware tile order: consecutive tiles (which share the A row panel) land on one
//     XCD's L2 (bijective remap, §5.5 T1).
// Requirements (checked on the host): N % 128 == 0, K % 64 == 0; any M (rows clamped on
// load, masked on store).
//
// Variants (fr_gemm_set_variant; -1 = auto): 0 the 128x128 kernel above; 6 the persistent
// 256x256 ping-pong (two wave rows half a phase apart, row-predicated stores); 9 the ping-pong
// with a store-tolerant stage schedule (padded C rows; also the residual / GELU-backward /
// dual-output epilogues); 12 = 9 with bias-armed accumulators; 13 = 12 with non-temporal
// stores.  Auto: 13 for no-residual N % 256 == 0 shapes with padded C, K < 2048 and M < 256k,
// 9 for the residual forms, K >= 2048 and M >= 256k (the cache build), 6 outside the padded-C
// domain, 0 otherwise
// (benchmarks/gemm_bench.py, profiles/r4_gemm_bench.json).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;  // 32 KB

// GELU(erf) with erf from Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16 output
// rounding): one rcp + one exp + 6 FMA, no range branches (ocml erff costs ~3x in the epilogue).
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __frcp_rn(1.0f + 0.3275911f * ax);
  const float y = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float r = 1.0f - y * __expf(-ax * ax);
  return copysignf(r, x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

// tanh(x) = 1 - 2 / (1 + e^{2x}): one exp2 + one rcp (ocml tanhf is a ~40-instruction
// branchy routine in an epilogue that runs once per output element); saturates cleanly
// (e^{2x} = inf -> 1, 0 -> -1); absolute error ~1e-7, far below the bf16 output rounding
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // 2 log2(e)
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + e);
}

template <int ACT>
__device__ __forceinline__ float act_fn(float x) {
  if constexpr (ACT == 1) return gelu_erf(x);
  else if constexpr (ACT == 2) return tanh_fast(x);
  else return x;
}

// GELU(erf) on a pair, written so the polynomial and scalings lower to packed f32 VALU
// (v_pk_fma_f32 / v_pk_mul_f32: two elements per instruction); only v_rcp / v_exp stay
// per element.  Same A&S 7.1.26 erf as gelu_erf, algebra folded:
//   Phi(x) = 1 - h (x >= 0), h (x < 0),  h = 0.5 * P(t) * exp(-z^2),  z = |x| / sqrt(2),
//   t = 1 / (1 + p z)  ->  GELU = x >= 0 ? x - x h : x h.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_pair(f32x2 x) {
  const f32x2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f32x2 d = z * 0.3275911f + 1.0f;
  f32x2 t;
  t.x = __builtin_amdgcn_rcpf(d.x);
  t.y = __builtin_amdgcn_rcpf(d.y);
  const f32x2 P = t * (0.127414796f + t * (-0.142248368f + t * (0.7107068705f + t * (-0.7265760135f + t * 0.5307027145f))));
  const f32x2 q = z * z * -1.44269504088896341f;
  f32x2 e;
  e.x = __builtin_amdgcn_exp2f(q.x);
  e.y = __builtin_amdgcn_exp2f(q.y);
  const f32x2 r = x * (P * e);
  f32x2 o;
  o.x = x.x >= 0.f ? x.x - r.x : r.x;
  o.y = x.y >= 0.f ? x.y - r.y : r.y;
  return o;
}

template <int ACT>
__device__ __forceinline__ void act4(float& v0, float& v1, float& v2, float& v3) {
  if constexpr (ACT == 1) {
    const f32x2 a = gelu_pair(f32x2{v0, v1}), b = gelu_pair(f32x2{v2, v3});
    v0 = a.x; v1 = a.y; v2 = b.x; v3 = b.y;
  } else {
    v0 = act_fn<ACT>(v0); v1 = act_fn<ACT>(v1); v2 = act_fn<ACT>(v2); v3 = act_fn<ACT>(v3);
  }
}

// residual combine: ACT 0-2 add R; ACT 3 (training FFN2 dgrad, dz = dF * GELU'(z)) multiplies
// by GELU'(R) with R = the saved pre-activation z -- the GELU backward rides in the epilogue
// of the GEMM that produces dF instead of a separate pass over dF and z
__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.0f + erf_fast(x * 0.70710678118654752f));
  return cdf + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}
// GELU'(x) = Phi(x) + x phi(x) on a pair, packed like gelu_pair: Phi from the same A&S erf
// (hardware rcp, one exp2), and phi(x) = exp(-x^2/2) / sqrt(2 pi) reuses that exp2 -- the
// IEEE-rounded __frcp_rn + two exps of the scalar gelu_grad made the FFN2 dgrad epilogue
// (ACT 3) cost ~40 % over the same GEMM without it
__device__ __forceinline__ f32x2 gelu_grad_pair(f32x2 x) {
  const f32x2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f32x2 d = z * 0.3275911f + 1.0f;
  f32x2 t;
  t.x = __builtin_amdgcn_rcpf(d.x);
  t.y = __builtin_amdgcn_rcpf(d.y);
  const f32x2 P = t * (0.127414796f + t * (-0.142248368f + t * (0.7107068705f + t * (-0.7265760135f + t * 0.5307027145f))));
  const f32x2 q = z * z * -1.44269504088896341f;
  f32x2 e;
  e.x = __builtin_amdgcn_exp2f(q.x);
  e.y = __builtin_amdgcn_exp2f(q.y);
  const f32x2 h = P * e;  // = 1 - Phi(|x|)
  const f32x2 g = x * e * 0.3989422804014327f;
  f32x2 o;
  o.x = (x.x >= 0.f ? 1.0f - h.x : h.x) + g.x;
  o.y = (x.y >= 0.f ? 1.0f - h.y : h.y) + g.y;
  return o;
}

template <int ACT>
__device__ __forceinline__ void res4(float& v0, float& v1, float& v2, float& v3, float r0, float r1, float r2,
                                     float r3) {
  if constexpr (ACT == 3) {
    const f32x2 a = gelu_grad_pair(f32x2{r0, r1}), b = gelu_grad_pair(f32x2{r2, r3});
    v0 *= a.x; v1 *= a.y; v2 *= b.x; v3 *= b.y;
  } else {
    v0 += r0; v1 += r1; v2 += r2; v3 += r3;
  }
}

// issue the glds for one K-tile into stage `st`
__device__ __forceinline__ void stage_tile(char* smem, int st, const bf16* __restrict__ A, const bf16* __restrict__ W,
                                           int M, int K, int m0, int n0, int k0, int wave, int lane) {
  char* base = smem + st * STAGE_BYTES;
  const int rsub = lane >> 3;                    // row within the 8-row piece
  const int chunk = (lane & 7) ^ rsub;           // logical 16-B chunk this lane fetches
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 32 + i * 8 + rsub;    // 0..127
    int gm = m0 + row;
    gm = gm < M ? gm : M - 1;
    const bf16* src = A + (size_t)gm * K + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, src), LDS_PTR(void, base + (wave * 32 + i * 8) * 128),
                                     16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 32 + i * 8 + rsub;
    const bf16* src = W + (size_t)(n0 + row) * K + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, src),
                                     LDS_PTR(void, base + BM * 128 + (wave * 32 + i * 8) * 128), 16, 0, 0);
  }
}

template <int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                         const float* __restrict__ bias, const bf16* __restrict__ R,
                                                         bf16* __restrict__ C, int M, int N, int K, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  // bijective XCD remap: blocks b, b+8, ... share an XCD -> give each XCD a contiguous tile range
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, q = nwg >> 3, rmd = nwg & 7;
  const int tile = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + (bid >> 3);
  const int mt = tile / tiles_n, nt = tile - mt * tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage_tile(smem, 0, A, W, M, K, m0, n0, 0, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15;         // fragment row
  const int fq = lane >> 4;         // k quarter
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage_tile(smem, cur ^ 1, A, W, M, K, m0, n0, (kt + 1) * BK, wave, lane);
    const char* As = smem + cur * STAGE_BYTES;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int phys = ((kk * 4 + fq) ^ (fr & 7)) * 16;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *(const bf16x8*)(As + (wm * 64 + i * 16 + fr) * 128 + phys);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *(const bf16x8*)(Bs + (wn * 64 + j * 16 + fr) * 128 + phys);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane holds C[m][nb..nb+3]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wn * 64 + j * 16 + fq * 4;
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      if constexpr (HAS_BIAS) {
        const float4 bb = *(const float4*)(bias + nb);
        v0 += bb.x; v1 += bb.y; v2 += bb.z; v3 += bb.w;
      }
      act4<ACT>(v0, v1, v2, v3);
      if constexpr (HAS_RES) {
        const bf16x4 rr = *(const bf16x4*)(R + (size_t)m * N + nb);
        res4<ACT>(v0, v1, v2, v3, (float)rr[0], (float)rr[1], (float)rr[2], (float)rr[3]);
      }
      bf16x4 o = {f2bf(v0), f2bf(v1), f2bf(v2), f2bf(v3)};
      *(bf16x4*)(C + (size_t)m * N + nb) = o;
    }
  }
}

// ---------------------------------------------------------------------------------------
// 256x256x64 block tile, 512 threads = 8 waves (2 along M x 4 along N), 128x64 per wave
// (8x4 MFMA tiles -> 128 accumulator VGPRs), 64 KB per LDS stage, two stages, one block
// per CU.  Twice the FLOP per staged byte of the 128x128 tile (128 vs 64 FLOP/B), which is
// what the L2 can feed at MFMA rate (~34 TB/s aggregate L2 vs ~39 TB/s the small tile needs).
constexpr int BM2 = 256, BN2 = 256;
// ---------------------------------------------------------------------------------------
// Variant 6: 256x256x64 persistent "ping-pong" GEMM (cdna_hip_programming.md §5, 256² 8-phase
// template), 512 threads = 8 waves (2 along M x 4 along N), 128x64 outputs per wave.
//
// * LDS = 2 K-buffers x 4 half-tiles x 16 KB = 128 KB (one block per CU).  A half-tile is
//   128 rows x 64 K of ONE operand: A_h0 = the rows of output quadrant qm = 0 of both wave
//   rows, A_h1 = qm = 1; B_h0 = columns of quadrant qn = 0 of all four wave columns, B_h1 =
//   qn = 1.  Each half is staged by all 512 threads with 2 global_load_lds x 16 B.
// * A K-step is 4 phases; phase = [ds_read fragments + stage one half-tile] s_barrier
//   [16 MFMAs of one 64x32 quadrant] s_barrier.  Quadrant order (0,0) (0,1) (1,1) (1,0)
//   keeps one operand in registers between phases (24 ds_read_b128 per K-step per wave).
// * Waves of M-row 1 execute one extra s_barrier up front, so the two wave rows run half a
//   phase apart: on every SIMD one wave issues MFMAs while its partner reads LDS/stages.
// * Stage schedule (step s, phase j): j0 -> A_h1 of s+1; j1 -> A_h0 of s+2; j2 -> B_h0 of
//   s+2; j3 -> B_h1 of s+2, then s_waitcnt vmcnt(6) retires everything of step s+1 (the
//   three younger half-tiles stay in flight across the barrier).  Every half is restaged
//   >= 1 phase after its last ds_read (whose lgkmcnt(0) precedes that phase's barrier)
//   and read >= 1 phase after the wait that retires it.
// * The K-step stream runs across output tiles (persistent, one block per CU, XCD-aware
//   tile walk): the next tile's first half-tiles are in flight during the current tile's
//   last phases; each wave row stores its tile while the other row is still on MFMAs.
constexpr int PP_HALF = 16384;
constexpr int PP2_MAXN = 3072;  // bias staged in LDS by variant 9

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __launch_bounds__(512, 1) void gemm_nt_pp_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                            const float* __restrict__ bias,
                                                            const bf16* __restrict__ R, bf16* __restrict__ C, int M,
                                                            int N, int K, int tiles_n, int ntiles) {
  __shared__ __attribute__((aligned(16))) char smem[8 * PP_HALF];
  const int G = gridDim.x, b = blockIdx.x;
  const int c = (G % 8 == 0) ? (b & 7) * (G >> 3) + (b >> 3) : b;
  if (c >= ntiles) return;
  const int nk = K >> 6;
  const int S = ((ntiles - c + G - 1) / G) * nk;  // K-steps of this block's stream
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int rsub = lane >> 3, schunk = (lane & 7) ^ rsub;

  // Per-thread source offsets (elements, < 2^31: checked on the host) of the 8 rows this
  // thread stages per K-step -- 2 per half-tile -- for the current tile and the next one.
  // Computed once per tile, so a phase's staging is 2 adds + 2 glds (no index math).
  int ocur[4][2], onxt[4][2];
  auto tile_offs = [&](int itile, int (&o)[4][2]) {
    int t = itile * G + c;
    t = t < ntiles ? t : c;
    const int mt = t / tiles_n;
    const int m0 = mt * 256, n0 = (t - mt * tiles_n) * 256;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rho = wave * 16 + i * 8 + rsub;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        int gm = m0 + (rho >> 6) * 128 + h * 64 + (rho & 63);
        gm = gm < M ? gm : M - 1;
        o[h][i] = gm * K + schunk * 8;
        o[2 + h][i] = (n0 + (rho >> 5) * 64 + h * 32 + (rho & 31)) * K + schunk * 8;
      }
    }
  };
  // stage half h of K-step g (tile-relative K index kts; `nx` = g lies in the next tile)
  auto stage = [&](int g, int h, int kts, bool nx) {
    if (g >= S) return;
    char* dst = smem + ((g & 1) * 4 + h) * PP_HALF;
    const bf16* base = (h < 2 ? A : W) + kts * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int off = nx ? onxt[h][i] : ocur[h][i];
      __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, base + off),
                                       LDS_PTR(void, dst + (wave * 16 + i * 8) * 128), 16, 0, 0);
    }
  };

  // prologue: step 0 (all four halves) + step 1's A_h0, B_h0, B_h1; retire step 0
  tile_offs(0, ocur);
  tile_offs(1, onxt);
  stage(0, 0, 0, false); stage(0, 2, 0, false); stage(0, 3, 0, false); stage(0, 1, 0, false);
  stage(1, 0, 1, false); stage(1, 2, 1, false); stage(1, 3, 1, false);
  if (S > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  if (wr == 1) pp_barrier();

  f32x4 acc[2][4][2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[q][i][p][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  const int arow = (wr * 64 + fr) * 128, brow = (wc * 32 + fr) * 128;
  const int ph0 = ((0 * 4 + fq) ^ (fr & 7)) * 16, ph1 = ((1 * 4 + fq) ^ (fr & 7)) * 16;
  auto read_a = [&](const char* hb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *(const bf16x8*)(hb + arow + i * 16 * 128 + ph0);
      af[i][1] = *(const bf16x8*)(hb + arow + i * 16 * 128 + ph1);
    }
  };
  auto read_b = [&](const char* hb, bf16x8 (&bf)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf[j][0] = *(const bf16x8*)(hb + brow + j * 16 * 128 + ph0);
      bf[j][1] = *(const bf16x8*)(hb + brow + j * 16 * 128 + ph1);
    }
  };
#define PP_MFMA(QM, QN, BF)                                                                             \
  {                                                                                                     \
    pp_barrier();                                                                                       \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                \
    __builtin_amdgcn_s_setprio(1);                                                                      \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) _Pragma("unroll") for (int i = 0; i < 4; ++i)      \
        _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[QM][i][QN][j] =                               \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(BF[j][kk], af[i][kk], acc[QM][i][QN][j], 0, 0, 0);  \
    __builtin_amdgcn_s_setprio(0);                                                                      \
    pp_barrier();                                                                                       \
  }

  int kt = 0, it = 0;
  for (int g = 0; g < S; ++g) {
    const char* buf = smem + (g & 1) * 4 * PP_HALF;
    const bool nx1 = kt + 1 >= nk, nx2 = kt + 2 >= nk;  // nk >= 2 (host): g+2 is at most one tile ahead
    const int k1 = nx1 ? kt + 1 - nk : kt + 1, k2 = nx2 ? kt + 2 - nk : kt + 2;
    // phase 0: quadrant (0,0)
    read_a(buf);
    read_b(buf + 2 * PP_HALF, b0);
    stage(g + 1, 1, k1, nx1);
    PP_MFMA(0, 0, b0)
    // phase 1: quadrant (0,1)
    read_b(buf + 3 * PP_HALF, b1);
    stage(g + 2, 0, k2, nx2);
    PP_MFMA(0, 1, b1)
    // phase 2: quadrant (1,1)
    read_a(buf + PP_HALF);
    stage(g + 2, 2, k2, nx2);
    PP_MFMA(1, 1, b1)
    // phase 3: quadrant (1,0); retire step g+1
    stage(g + 2, 3, k2, nx2);
    if (g + 2 < S) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PP_MFMA(1, 0, b0)
    if (++kt == nk) {
      // epilogue: this wave row's 128 x 64 of the finished tile.  Bias once per tile; the
      // residual rows of one 64-row quadrant are all loaded before any is consumed (one
      // memory round trip per quadrant instead of one per row).
      const int t = it * G + c;
      const int mt = t / tiles_n;
      const int m0 = mt * 256, n0 = (t - mt * tiles_n) * 256;
      const int nb0 = n0 + wc * 64 + fq * 4;
      float4 bb[2][2];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bb[p][j] = HAS_BIAS ? *(const float4*)(bias + nb0 + p * 32 + j * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        bf16x4 rr[4][2][2];
        if constexpr (HAS_RES) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            int m = m0 + wr * 128 + q * 64 + i * 16 + fr;
            m = m < M ? m : M - 1;
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
              for (int j = 0; j < 2; ++j) rr[i][p][j] = *(const bf16x4*)(R + (size_t)m * N + nb0 + p * 32 + j * 16);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wr * 128 + q * 64 + i * 16 + fr;
#pragma unroll
          for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              f32x4& a4 = acc[q][i][p][j];
              float v0 = a4[0] + bb[p][j].x, v1 = a4[1] + bb[p][j].y;
              float v2 = a4[2] + bb[p][j].z, v3 = a4[3] + bb[p][j].w;
              act4<ACT>(v0, v1, v2, v3);
              if constexpr (HAS_RES) {
                res4<ACT>(v0, v1, v2, v3, (float)rr[i][p][j][0], (float)rr[i][p][j][1], (float)rr[i][p][j][2],
                          (float)rr[i][p][j][3]);
              }
              if (m < M) {
                bf16x4 o = {f2bf(v0), f2bf(v1), f2bf(v2), f2bf(v3)};
                *(bf16x4*)(C + (size_t)m * N + nb0 + p * 32 + j * 16) = o;
              }
              a4 = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
      }
      kt = 0;
      ++it;
#pragma unroll
      for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) ocur[h][i] = onxt[h][i];
      tile_offs(it + 1, onxt);
    }
  }
#undef PP_MFMA
  if (wr == 0) pp_barrier();  // balance the staggered row's extra barrier
}

// Store one 32-column group of a 16x16 MFMA row block: lane (fr, fq) holds columns
// [4fq, 4fq+4) of frag j = 0 (v0) and of frag j = 1 (v1, +16).  One v_permlane16_swap per
// dword pair gives every lane 8 contiguous columns -- fq 0: 0-7, 1: 16-23, 2: 8-15,
// 3: 24-31 -- so the group goes out as ONE 16-byte store per lane instead of two 8-byte
// ones (cdna_hip_programming.md T21).
template <bool NT = false>
__device__ __forceinline__ void store_pair16(bf16* __restrict__ crow, const float (&v0)[4], const float (&v1)[4],
                                             int fq) {
  const bf16x4 o0 = {f2bf(v0[0]), f2bf(v0[1]), f2bf(v0[2]), f2bf(v0[3])};
  const bf16x4 o1 = {f2bf(v1[0]), f2bf(v1[1]), f2bf(v1[2]), f2bf(v1[3])};
  uint2 a = __builtin_bit_cast(uint2, o0), b = __builtin_bit_cast(uint2, o1);
  auto r = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  a.x = r[0];
  b.x = r[1];
  r = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  a.y = r[0];
  b.y = r[1];
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  if constexpr (NT)  // streaming store: the output is not re-read by this kernel
    __builtin_nontemporal_store(u32x4{a.x, a.y, b.x, b.y}, GLOBAL_PTR(u32x4, crow + (fq & 1) * 16 + (fq >> 1) * 8));
  else
    *GLOBAL_PTR(u32x4, crow + (fq & 1) * 16 + (fq >> 1) * 8) = u32x4{a.x, a.y, b.x, b.y};
}

// ---------------------------------------------------------------------------------------
// Variant 9: the ping-pong kernel with a store-tolerant stage schedule.  Profiling variant 6
// (scripts/gpu_gemm_pmc.sh) showed the epilogue stores cost +81 % SQ_WAIT_ANY: vmcnt retires
// in issue order, so the next K-step's counted wait -- which needs a half-tile staged AFTER
// the stores -- also waits for every store to be acknowledged.  Here all four half-tiles of
// step g+2 are staged during step g (A_h0 @ phase 1, B_h0 @ 2, B_h1 + A_h1 @ 3), so the
// half-tiles that the wait after an epilogue needs were issued BEFORE its stores and the wait
// can leave them outstanding: vmcnt(8) normally, vmcnt(8 + 16) in the step after a tile's
// epilogue (exactly 16 unconditional dwordx4 stores per wave: C has round_up(M, 256) rows,
// so no row predicate; bias comes from LDS, so the epilogue issues no loads; with a residual
// its loads would break the count, so HAS_RES keeps vmcnt(8)).  One more half-tile is in
// flight per wait than in variant 6.  WAR: every half is restaged >= 1 phase after its last
// read (A_h1 is read in phase 2 and restaged in phase 3).
// (Spreading a tile's epilogue over the load sections of the next tile's first K-step measured
// slower: 815 vs 964 TF on QKV, profiles/r4_gemm_bench_base.json.)
template <int ACT, bool HAS_BIAS, bool HAS_RES, bool DUAL = false>
__global__ __launch_bounds__(512, 1) void gemm_nt_pp2_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                             const float* __restrict__ bias,
                                                             const bf16* __restrict__ R, bf16* __restrict__ C, int M,
                                                             int N, int K, int tiles_n, int ntiles,
                                                             const int* __restrict__ full_rows = nullptr,
                                                             int tiles_np = 0, bf16* __restrict__ Z = nullptr,
                                                             float* __restrict__ colpart = nullptr) {
  // colpart (ACT 3, training FFN2 dgrad): per-(row tile, wave row) column sums of the dz the
  // epilogue writes, [tiles_m * 2, N] -- the FFN1 bias gradient without a pass over dz
  // DUAL (training FFN1): the epilogue also stores the pre-activation z = acc + bias to Z
  // (the GELU backward needs it), so no separate activation pass reads z back
  // ONE __shared__ object (staging halves + the bias vector): a second one makes hipcc drain
  // vmcnt(0) before every fragment read (cdna_hip_programming.md §5 "Three .s-level traps")
  __shared__ __attribute__((aligned(16))) char smem[8 * PP_HALF + (HAS_BIAS ? PP2_MAXN * 4 : 0)];
  float* bias_s = (float*)(smem + 8 * PP_HALF);
  const int G = gridDim.x, b = blockIdx.x;
  const int c = (G % 8 == 0) ? (b & 7) * (G >> 3) + (b >> 3) : b;
  // row-split tile list (packed title rows, fr_gemm_nt_bf16_split): row tiles below
  // *full_rows (a device count: no host sync) take all tiles_n column tiles, the rest only
  // the first tiles_np (the Q columns); without full_rows the map is the plain one
  int full_t = ntiles;
  if (full_rows != nullptr) {
    const int tiles_m = (M + 255) >> 8;
    int fm = (*full_rows + 255) >> 8;
    fm = fm < tiles_m ? fm : tiles_m;
    full_t = fm * tiles_n;
    ntiles = full_t + (tiles_m - fm) * tiles_np;
  }
  auto tile_mn = [&](int t, int& m0_, int& n0_) {
    int mt_, nt_;
    if (t < full_t) {
      mt_ = t / tiles_n;
      nt_ = t - mt_ * tiles_n;
    } else {
      const int u = t - full_t, q = u / tiles_np;
      mt_ = full_t / tiles_n + q;
      nt_ = u - q * tiles_np;
    }
    m0_ = mt_ * 256;
    n0_ = nt_ * 256;
  };
  if (c >= ntiles) return;
  const int nk = K >> 6;
  const int S = ((ntiles - c + G - 1) / G) * nk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int rsub = lane >> 3, schunk = (lane & 7) ^ rsub;
  if constexpr (HAS_BIAS) {
    for (int i = tid; i < N; i += 512) bias_s[i] = bias[i];
  }
  int ocur[4][2], onxt[4][2];
  auto tile_offs = [&](int itile, int (&o)[4][2]) {
    int t = itile * G + c;
    t = t < ntiles ? t : c;
    int m0, n0;
    tile_mn(t, m0, n0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rho = wave * 16 + i * 8 + rsub;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        int gm = m0 + (rho >> 6) * 128 + h * 64 + (rho & 63);
        gm = gm < M ? gm : M - 1;
        o[h][i] = gm * K + schunk * 8;
        int wrow = n0 + (rho >> 5) * 64 + h * 32 + (rho & 31);
        wrow = wrow < N ? wrow : N - 1;  // partial last column tile (N % 256 != 0): clamped, never stored
        o[2 + h][i] = wrow * K + schunk * 8;
      }
    }
  };
  auto stage = [&](int g, int h, int kts, bool nx) {
    if (g >= S) return;
    char* dst = smem + ((g & 1) * 4 + h) * PP_HALF;
    const bf16* base = (h < 2 ? A : W) + kts * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int off = nx ? onxt[h][i] : ocur[h][i];
      __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, base + off),
                                       LDS_PTR(void, dst + (wave * 16 + i * 8) * 128), 16, 0, 0);
    }
  };
  // prologue: steps 0 and 1 (all halves); retire step 0 (bias loads are older: retired too)
  tile_offs(0, ocur);
  tile_offs(1, onxt);
  const bool nx_1 = nk < 2;  // nk >= 2 on the host path: step 1 is in tile 0
  stage(0, 0, 0, false); stage(0, 2, 0, false); stage(0, 3, 0, false); stage(0, 1, 0, false);
  stage(1, 0, 1, nx_1); stage(1, 2, 1, nx_1); stage(1, 3, 1, nx_1); stage(1, 1, 1, nx_1);
  if (S > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  if (wr == 1) pp_barrier();

  f32x4 acc[2][4][2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[q][i][p][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  const int arow = (wr * 64 + fr) * 128, brow = (wc * 32 + fr) * 128;
  const int ph0 = ((0 * 4 + fq) ^ (fr & 7)) * 16, ph1 = ((1 * 4 + fq) ^ (fr & 7)) * 16;
  auto read_a = [&](const char* hb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *(const bf16x8*)(hb + arow + i * 16 * 128 + ph0);
      af[i][1] = *(const bf16x8*)(hb + arow + i * 16 * 128 + ph1);
    }
  };
  auto read_b = [&](const char* hb, bf16x8 (&bf)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf[j][0] = *(const bf16x8*)(hb + brow + j * 16 * 128 + ph0);
      bf[j][1] = *(const bf16x8*)(hb + brow + j * 16 * 128 + ph1);
    }
  };
#define PP_MFMA(QM, QN, BF)                                                                             \
  {                                                                                                     \
    pp_barrier();                                                                                       \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                \
    __builtin_amdgcn_s_setprio(1);                                                                      \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) _Pragma("unroll") for (int i = 0; i < 4; ++i)      \
        _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[QM][i][QN][j] =                               \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(BF[j][kk], af[i][kk], acc[QM][i][QN][j], 0, 0, 0);  \
    __builtin_amdgcn_s_setprio(0);                                                                      \
    pp_barrier();                                                                                       \
  }

  int kt = 0, it = 0;
  bool after_epi = false;  // the previous step ended with a tile epilogue (its 16 stores in flight)
  bool epi_stored = true;  // ... and this wave issued them (false: columns past a partial tile)
  for (int g = 0; g < S; ++g) {
    const char* buf = smem + (g & 1) * 4 * PP_HALF;
    const bool nx2 = kt + 2 >= nk;
    const int k2 = nx2 ? kt + 2 - nk : kt + 2;
    // phase 0: quadrant (0,0)
    read_a(buf);
    read_b(buf + 2 * PP_HALF, b0);
    PP_MFMA(0, 0, b0)
    // phase 1: quadrant (0,1)
    read_b(buf + 3 * PP_HALF, b1);
    stage(g + 2, 0, k2, nx2);
    PP_MFMA(0, 1, b1)
    // phase 2: quadrant (1,1)
    read_a(buf + PP_HALF);
    stage(g + 2, 2, k2, nx2);
    PP_MFMA(1, 1, b1)
    // phase 3: quadrant (1,0); stage the rest of g+2, retire step g+1 (issued during step g-1,
    // so everything of this step may stay in flight: its 8 loads and, deferred, 16 stores)
    stage(g + 2, 3, k2, nx2);
    stage(g + 2, 1, k2, nx2);
    if (g + 2 >= S) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (a wave whose columns lay outside a partial last tile issued no stores: plain wait)
    else if (!HAS_RES && after_epi && epi_stored && DUAL) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");  // 8 + 32 stores
    else if (!HAS_RES && after_epi && epi_stored) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // 8 + 16 stores
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    after_epi = false;
    PP_MFMA(1, 0, b0)
    if (++kt == nk) {
      int m0, n0;
      tile_mn(it * G + c, m0, n0);
      const int nb0 = n0 + wc * 64 + fq * 4;
      // partial last column tile (N % 256 == 64/128/192, no residual / dual / colsum: host
      // checked): this wave's 64 columns are either all inside N or all outside
      const bool col_ok = n0 + wc * 64 < N;
      epi_stored = col_ok;
      f32x4 bb[2][2];
      if constexpr (HAS_BIAS) {
        // bias via opaque ds_reads (a plain read of the staging object would also drain vmcnt)
        const uint32_t ba = (uint32_t)(uintptr_t)LDS_PTR(char, smem) + 8 * PP_HALF + nb0 * 4;
        asm volatile("ds_read_b128 %0, %1" : "=v"(bb[0][0]) : "v"(ba));
        asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(bb[0][1]) : "v"(ba));
        asm volatile("ds_read_b128 %0, %1 offset:128" : "=v"(bb[1][0]) : "v"(ba));
        asm volatile("ds_read_b128 %0, %1 offset:192" : "=v"(bb[1][1]) : "v"(ba));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bb[0][0]), "+v"(bb[0][1]), "+v"(bb[1][0]), "+v"(bb[1][1]));
      } else {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int j = 0; j < 2; ++j) bb[p][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      float csum[2][2][4];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) csum[p][j][e] = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        bf16x4 rr[4][2][2];
        if constexpr (HAS_RES) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            int m = m0 + wr * 128 + q * 64 + i * 16 + fr;
            m = m < M ? m : M - 1;
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
              for (int j = 0; j < 2; ++j) rr[i][p][j] = *(const bf16x4*)(R + (size_t)m * N + nb0 + p * 32 + j * 16);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wr * 128 + q * 64 + i * 16 + fr;  // < round_up(M, 256): C is padded
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            float v[2][4], zv[2][4];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              f32x4& a4 = acc[q][i][p][j];
#pragma unroll
              for (int e = 0; e < 4; ++e) v[j][e] = a4[e] + bb[p][j][e];
              if constexpr (DUAL) {
#pragma unroll
                for (int e = 0; e < 4; ++e) zv[j][e] = v[j][e];
              }
              act4<ACT>(v[j][0], v[j][1], v[j][2], v[j][3]);
              if constexpr (HAS_RES) {
                res4<ACT>(v[j][0], v[j][1], v[j][2], v[j][3], (float)rr[i][p][j][0], (float)rr[i][p][j][1],
                          (float)rr[i][p][j][2], (float)rr[i][p][j][3]);
              }
              if constexpr (ACT == 3) {
                if (colpart != nullptr && m < M) {  // padded rows (m >= M) hold duplicates: excluded
#pragma unroll
                  for (int e = 0; e < 4; ++e) csum[p][j][e] += v[j][e];
                }
              }
              a4 = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            if (col_ok) store_pair16(C + (size_t)m * N + n0 + wc * 64 + p * 32, v[0], v[1], fq);
            if constexpr (DUAL) {
              if (col_ok) store_pair16(Z + (size_t)m * N + n0 + wc * 64 + p * 32, zv[0], zv[1], fq);
            }
          }
        }
      }
      if constexpr (ACT == 3) {
        if (colpart != nullptr) {
          // rows of this wave are (fr, i, q): sum the 16 fr lanes; lane fr == 0 of each fq
          // group then holds 16 column sums -> 4 x 16-byte stores
#pragma unroll
          for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float x = csum[p][j][e];
                x += __shfl_xor(x, 1, 64);
                x += __shfl_xor(x, 2, 64);
                x += __shfl_xor(x, 4, 64);
                x += __shfl_xor(x, 8, 64);
                csum[p][j][e] = x;
              }
          if (fr == 0) {
            float* cp = colpart + (size_t)((m0 >> 8) * 2 + wr) * N + n0 + wc * 64 + fq * 4;
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
              for (int j = 0; j < 2; ++j)
                *(float4*)(cp + p * 32 + j * 16) = make_float4(csum[p][j][0], csum[p][j][1], csum[p][j][2], csum[p][j][3]);
          }
        }
      }
      after_epi = true;
      kt = 0;
      ++it;
#pragma unroll
      for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) ocur[h][i] = onxt[h][i];
      tile_offs(it + 1, onxt);
    }
  }
#undef PP_MFMA
  if (wr == 0) pp_barrier();
}

// ---------------------------------------------------------------------------------------
// Variants 12 / 13 (13 = auto on no-residual shapes with N % 256 == 0 and K < 2048): the variant-9 ping-pong
// schedule with bias-armed accumulators -- once the tile epilogue has stored a quadrant, its
// accumulators are set to the NEXT tile's bias (0 without a bias) instead of zero, so the
// epilogue has no bias add and no separate zeroing.  (Storing each quadrant inside the next
// phase's MFMA section instead -- 4 stores per phase -- needs ~40 more VGPRs than 2 waves / SIMD
// leave: it spilled, and re-reading B_h0 to free them races its restaging in phase 2.)
// NT (variant 13): non-temporal output stores (the C tile is not re-read by this launch).
template <int ACT, bool HAS_BIAS, bool DUAL, bool NT = false>
__global__ __launch_bounds__(512, 1) void gemm_nt_pp3_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                             const float* __restrict__ bias, bf16* __restrict__ C,
                                                             int M, int N, int K, int tiles_n, int ntiles,
                                                             const int* __restrict__ full_rows = nullptr,
                                                             int tiles_np = 0, bf16* __restrict__ Z = nullptr) {
  // ONE __shared__ object (staging halves + the bias vector), as variant 9
  __shared__ __attribute__((aligned(16))) char smem[8 * PP_HALF + (HAS_BIAS ? PP2_MAXN * 4 : 0)];
  float* bias_s = (float*)(smem + 8 * PP_HALF);
  const int G = gridDim.x, b = blockIdx.x;
  const int c = (G % 8 == 0) ? (b & 7) * (G >> 3) + (b >> 3) : b;
  int full_t = ntiles;
  if (full_rows != nullptr) {  // row-split tile list (fr_gemm_nt_bf16_split), as variant 9
    const int tiles_m = (M + 255) >> 8;
    int fm = (*full_rows + 255) >> 8;
    fm = fm < tiles_m ? fm : tiles_m;
    full_t = fm * tiles_n;
    ntiles = full_t + (tiles_m - fm) * tiles_np;
  }
  auto tile_mn = [&](int t, int& m0_, int& n0_) {
    int mt_, nt_;
    if (t < full_t) {
      mt_ = t / tiles_n;
      nt_ = t - mt_ * tiles_n;
    } else {
      const int u = t - full_t, q = u / tiles_np;
      mt_ = full_t / tiles_n + q;
      nt_ = u - q * tiles_np;
    }
    m0_ = mt_ * 256;
    n0_ = nt_ * 256;
  };
  if (c >= ntiles) return;
  const int nk = K >> 6;
  const int S = ((ntiles - c + G - 1) / G) * nk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int rsub = lane >> 3, schunk = (lane & 7) ^ rsub;
  if constexpr (HAS_BIAS) {  // complete before the first tile's accumulators read it
    for (int i = tid; i < N; i += 512) bias_s[i] = bias[i];
    __syncthreads();
  }
  // staging addresses from the (scalar) tile origins: row r0 + 8 i + rsub of half h, r0
  // wave-uniform; A rows past M clamp to M - 1 (their products land in C's padding rows)
  int cm0, cn0, nm0, nn0;  // current / next tile of this block's stream
  auto tile_at = [&](int itile, int& m0_, int& n0_) {
    int t = itile * G + c;
    tile_mn(t < ntiles ? t : c, m0_, n0_);
  };
  auto stage = [&](int g, int h, int kts, bool nx) {
    if (g >= S) return;
    char* dst = smem + ((g & 1) * 4 + h) * PP_HALF;
    const int r0 = h < 2 ? (nx ? nm0 : cm0) + (wave >> 2) * 128 + h * 64 + (wave & 3) * 16
                         : (nx ? nn0 : cn0) + (wave >> 1) * 64 + (h - 2) * 32 + (wave & 1) * 16;
    const bf16* base = (h < 2 ? A : W) + kts * 64 + schunk * 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int row = r0 + i * 8 + rsub;
      if (h < 2) row = row < M ? row : M - 1;
      __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, base + row * K),
                                       LDS_PTR(void, dst + (wave * 16 + i * 8) * 128), 16, 0, 0);
    }
  };
  tile_at(0, cm0, cn0);
  tile_at(1, nm0, nn0);
  const bool nx_1 = nk < 2;
  stage(0, 0, 0, false); stage(0, 2, 0, false); stage(0, 3, 0, false); stage(0, 1, 0, false);
  stage(1, 0, 1, nx_1); stage(1, 2, 1, nx_1); stage(1, 3, 1, nx_1); stage(1, 1, 1, nx_1);
  if (S > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  if (wr == 1) pp_barrier();

  f32x4 acc[2][4][2][2];
  bf16x8 af[4][2], b0[2][2], b1[2][2];
  const int arow = (wr * 64 + fr) * 128, brow = (wc * 32 + fr) * 128;
  const int ph0 = ((0 * 4 + fq) ^ (fr & 7)) * 16, ph1 = ((1 * 4 + fq) ^ (fr & 7)) * 16;
  auto read_a = [&](const char* hb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *(const bf16x8*)(hb + arow + i * 16 * 128 + ph0);
      af[i][1] = *(const bf16x8*)(hb + arow + i * 16 * 128 + ph1);
    }
  };
  auto read_b = [&](const char* hb, bf16x8 (&bf)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf[j][0] = *(const bf16x8*)(hb + brow + j * 16 * 128 + ph0);
      bf[j][1] = *(const bf16x8*)(hb + brow + j * 16 * 128 + ph1);
    }
  };
  const uint32_t bias_lds = (uint32_t)(uintptr_t)LDS_PTR(char, smem) + 8 * PP_HALF;
  // bias of columns n0 + wc*64 + qn*32 + j*16 + 4fq + e (j = 0, 1) via opaque ds_reads (a plain
  // read of the staging object would also drain vmcnt); tie_bias waits for them
  auto read_bias = [&](int n0, int qn, f32x4 (&bv)[2]) {
    if constexpr (HAS_BIAS) {
      const uint32_t ba = bias_lds + (n0 + wc * 64 + qn * 32 + fq * 4) * 4;
      asm volatile("ds_read_b128 %0, %1" : "=v"(bv[0]) : "v"(ba));
      asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(bv[1]) : "v"(ba));
    } else {
      bv[0] = f32x4{0.f, 0.f, 0.f, 0.f};
      bv[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto tie_bias = [&](f32x4 (&bv)[2]) {
    if constexpr (HAS_BIAS) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bv[0]), "+v"(bv[1]));
  };
  {  // the first tile's accumulators start at its bias
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      f32x4 bv[2];
      read_bias(cn0, p, bv);
      tie_bias(bv);
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[q][i][p][j] = bv[j];
    }
  }
  f32x4 bn[2];  // the bias that re-arms the quadrant an epilogue phase stores
#define PP3_MF(QM, QN, BF)                                                                              \
  {                                                                                                     \
    pp_barrier();                                                                                       \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                \
    __builtin_amdgcn_s_setprio(1);                                                                      \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) _Pragma("unroll") for (int i = 0; i < 4; ++i)      \
        _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[QM][i][QN][j] =                               \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(BF[j][kk], af[i][kk], acc[QM][i][QN][j], 0, 0, 0);  \
    __builtin_amdgcn_s_setprio(0);                                                                      \
    pp_barrier();                                                                                       \
  }
#define PP3_EPI(QM, QN)                                                                                 \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                      \
    float v0[4], v1[4];                                                                                 \
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                    \
      v0[e] = acc[QM][i][QN][0][e];                                                                     \
      v1[e] = acc[QM][i][QN][1][e];                                                                     \
    }                                                                                                   \
    const size_t o_ = (size_t)(pm0 + wr * 128 + QM * 64 + i * 16 + fr) * N + pn0 + wc * 64 + QN * 32;  \
    if constexpr (DUAL) store_pair16<NT>(Z + o_, v0, v1, fq);                                           \
    act4<ACT>(v0[0], v0[1], v0[2], v0[3]);                                                              \
    act4<ACT>(v1[0], v1[1], v1[2], v1[3]);                                                              \
    store_pair16<NT>(C + o_, v0, v1, fq);                                                               \
    acc[QM][i][QN][0] = bn[0];                                                                          \
    acc[QM][i][QN][1] = bn[1];                                                                          \
  }
  int kt = 0, it = 0, pm0 = 0, pn0 = 0;
  for (int g = 0; g < S; ++g) {
    const char* buf = smem + (g & 1) * 4 * PP_HALF;
    const bool nx2 = kt + 2 >= nk;
    const int k2 = nx2 ? kt + 2 - nk : kt + 2;
    const bool last = kt == nk - 1;
    const bool epi0 = kt == 0 && it > 0;  // the step after a tile epilogue
    if (last) {  // the tile this step's epilogue stores
      pm0 = cm0;
      pn0 = cn0;
    }
    // phase 0: quadrant (0,0)
    read_a(buf);
    read_b(buf + 2 * PP_HALF, b0);
    PP3_MF(0, 0, b0)
    // phase 1: quadrant (0,1)
    read_b(buf + 3 * PP_HALF, b1);
    stage(g + 2, 0, k2, nx2);
    PP3_MF(0, 1, b1)
    // phase 2: quadrant (1,1)
    read_a(buf + PP_HALF);
    stage(g + 2, 2, k2, nx2);
    PP3_MF(1, 1, b1)
    // phase 3: quadrant (1,0); stage the rest of g+2, retire step g+1 (after a tile epilogue its
    // stores are younger than step g+1's loads and may stay in flight)
    stage(g + 2, 3, k2, nx2);
    stage(g + 2, 1, k2, nx2);
    if (g + 2 >= S) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (epi0 && DUAL) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");  // 8 loads + 32 stores
    else if (epi0) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");          // 8 loads + 16 stores
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    PP3_MF(1, 0, b0)
    if (last) {  // the tile epilogue; the quadrants are re-armed with the next tile's bias
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      read_bias(nn0, 0, bn);
      tie_bias(bn);
      PP3_EPI(0, 0) PP3_EPI(1, 0)
      read_bias(nn0, 1, bn);
      tie_bias(bn);
      PP3_EPI(0, 1) PP3_EPI(1, 1)
    }
    if (last) {
      kt = 0;
      ++it;
      cm0 = nm0;
      cn0 = nn0;
      tile_at(it + 1, nm0, nn0);
    } else {
      ++kt;
    }
  }
#undef PP3_MF
#undef PP3_EPI
  if (wr == 0) pp_barrier();
}

int g_num_cus = 0;

int g_gemm_variant = -1;  // -1 auto; 0 = 128x128, 6 / 9 / 12 / 13 = the ping-pong forms (A/B runs)

static int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_num_cus <= 0) g_num_cus = 256;
  }
  return g_num_cus;
}

// the ping-pong kernels' domain: 256x256 tiles (a partial last column tile only in variant 9),
// C rows padded to a multiple of 256 (unpredicated stores), 32-bit operand offsets
static bool pp_domain(int M, int N, int K, int c_rows) {
  return K >= 128 && N <= PP2_MAXN && c_rows >= ((M + 255) / 256) * 256 && (long long)M * K < (1ll << 31) &&
         (long long)N * K < (1ll << 31);
}

template <int ACT>
void launch_act(const bf16* A, const bf16* W, const float* bias, const bf16* R, bf16* C, int M, int N, int K,
                int c_rows, hipStream_t s) {
  // N % 256 != 0 (the text head's N = 384): the ping-pong kernel with a partial last column
  // tile (plain / bias / act epilogue only) -- opt-in (variant 9) only: at M = 80k, N = 384
  // with tanh it measured 133 us vs 102 us for the 128x128 kernel (2.45 waves of 256-row
  // tiles, a third of the MFMA work wasted on the clamped columns, tanh in the exposed epilogue)
  const bool auto_v = g_gemm_variant < 0;
  // (at M >= 256k rows the partial tile wins: 770 vs 612 TF for N = 384 + tanh at M = 409,600,
  // profiles/r4_gemm_bench_M409600.json)
  const bool part_n = N % BN2 != 0 && N % 64 == 0 && R == nullptr && ACT != 3 &&
                      (g_gemm_variant == 9 || (auto_v && M >= (1 << 18)));
  const bool big = (auto_v && (N % BN2 == 0 || part_n) && M >= 4096) || (g_gemm_variant >= 6 && (N % BN2 == 0 || part_n));
  if (big && (auto_v || g_gemm_variant == 9 || g_gemm_variant >= 12) && pp_domain(M, N, K, c_rows)) {
    const int tiles_n = (N + BN2 - 1) / BN2, tiles_m = (M + BM2 - 1) / BM2, ntiles = tiles_m * tiles_n;
    const int G = ntiles < num_cus() ? ntiles : num_cus();
    // auto: variant 13 (bias-armed accumulators, non-temporal stores) on the no-residual shapes
    // with K < 2048; variant 9 for the rest (residual / GELU-backward epilogues, FFN2)
    if constexpr (ACT != 3) {
      if (R == nullptr && N % BN2 == 0 && g_gemm_variant != 9) {
        // variant 13 (non-temporal stores) by default where K < 2048 and M < 256k: at M = 78,850
        // QKV 1029 vs 952 TF (v9), FFN1 + GELU 867 vs 842; FFN2 (K = 3072) 1070 vs 1150; at the
        // cache build's M = 409,600 variant 9 wins every shape (QKV 1007 vs 948, out-proj 979 vs
        // 929, FFN1 871 vs 842): profiles/r4_gemm_bench.json, r4_gemm_bench_M409600.json
        if (auto_v && (K >= 2048 || M >= (1 << 18))) {
          if (bias) hipLaunchKernelGGL((gemm_nt_pp2_kernel<ACT, true, false>), dim3(G), dim3(512), 0, s, A, W, bias, R, C,
                                       M, N, K, tiles_n, ntiles);
          else hipLaunchKernelGGL((gemm_nt_pp2_kernel<ACT, false, false>), dim3(G), dim3(512), 0, s, A, W, bias, R, C,
                                  M, N, K, tiles_n, ntiles);
          return;
        }
        const bool nt = g_gemm_variant == 13 || auto_v;
#define LPP3(HB, NT)                                                                                               \
  hipLaunchKernelGGL((gemm_nt_pp3_kernel<ACT, HB, false, NT>), dim3(G), dim3(512), 0, s, A, W, bias, C, M, N, K, tiles_n, \
                     ntiles)
        if (bias && nt) LPP3(true, true);
        else if (bias) LPP3(true, false);
        else if (nt) LPP3(false, true);
        else LPP3(false, false);
#undef LPP3
        return;
      }
    }
#define LPP2(HB, HR)                                                                                          \
  hipLaunchKernelGGL((gemm_nt_pp2_kernel<ACT, HB, HR>), dim3(G), dim3(512), 0, s, A, W, bias, R, C, M, N, K, tiles_n, \
                     ntiles)
    if (bias && R) LPP2(true, true);
    else if (bias) LPP2(true, false);
    else if (R) LPP2(false, true);
    else LPP2(false, false);
#undef LPP2
    return;
  }
  // outside that domain (unpadded C, offsets past 2^31 elements): variant 6 (row-predicated
  // stores) while the 32-bit offsets hold, else the 128x128 kernel (64-bit addressing)
  if (big && N % BN2 == 0 && K >= 128 && (long long)M * K < (1ll << 31) && (long long)N * K < (1ll << 31)) {
    const int tiles_n = N / BN2, tiles_m = (M + BM2 - 1) / BM2, ntiles = tiles_m * tiles_n;
    const int G = ntiles < num_cus() ? ntiles : num_cus();
#define LPP(HB, HR)                                                                                        \
  hipLaunchKernelGGL((gemm_nt_pp_kernel<ACT, HB, HR>), dim3(G), dim3(512), 0, s, A, W, bias, R, C, M, N, K, tiles_n, \
                     ntiles)
    if (bias && R) LPP(true, true);
    else if (bias) LPP(true, false);
    else if (R) LPP(false, true);
    else LPP(false, false);
#undef LPP
    return;
  }
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  dim3 grid(tiles_m * tiles_n), block(256);
  if (bias && R) hipLaunchKernelGGL((gemm_nt_kernel<ACT, true, true>), grid, block, 0, s, A, W, bias, R, C, M, N, K, tiles_n);
  else if (bias) hipLaunchKernelGGL((gemm_nt_kernel<ACT, true, false>), grid, block, 0, s, A, W, bias, R, C, M, N, K, tiles_n);
  else if (R) hipLaunchKernelGGL((gemm_nt_kernel<ACT, false, true>), grid, block, 0, s, A, W, bias, R, C, M, N, K, tiles_n);
  else hipLaunchKernelGGL((gemm_nt_kernel<ACT, false, false>), grid, block, 0, s, A, W, bias, R, C, M, N, K, tiles_n);
}

}  // namespace

extern "C" void fr_gemm_set_variant(int v) { g_gemm_variant = v; }

// c_rows: rows allocated in C (>= M); round_up(M, 256) lets variant 9 store without a row predicate
extern "C" int fr_gemm_nt_bf16(const void* A, const void* W, const float* bias, const void* R, void* C, int M, int N,
                               int K, int act, int c_rows, hipStream_t s) {
  if (N % BN != 0 || K % BK != 0 || M <= 0) return 1;
  const bf16* a = (const bf16*)A;
  const bf16* w = (const bf16*)W;
  const bf16* r = (const bf16*)R;
  bf16* c = (bf16*)C;
  switch (act) {
    case 0: launch_act<0>(a, w, bias, r, c, M, N, K, c_rows, s); break;
    case 1: launch_act<1>(a, w, bias, r, c, M, N, K, c_rows, s); break;
    case 2: launch_act<2>(a, w, bias, r, c, M, N, K, c_rows, s); break;
    case 3:  // C = (A W^T) * GELU'(R): needs R, no bias
      if (r == nullptr || bias != nullptr) return 2;
      launch_act<3>(a, w, bias, r, c, M, N, K, c_rows, s);
      break;
    default: return 2;
  }
  return 0;
}

// Row-split GEMM for the packed title layout: rows [0, *full_rows) get all N columns, the
// remaining rows only the first n_partial (the Q third of the fused QKV weight: padding
// tokens are never read as keys or values).  full_rows stays on the device (the count comes
// from the row-plan kernel of the same step), so no host synchronisation.  Shapes outside
// the ping-pong kernel's domain fall back to the full product (same values in the columns
// that are read).
extern "C" int fr_gemm_nt_bf16_split(const void* A, const void* W, const float* bias, void* C, int M, int N, int K,
                                     int c_rows, const int* full_rows, int n_partial, hipStream_t s) {
  if (N % BN != 0 || K % BK != 0 || M <= 0) return 1;
  const bool ok = (g_gemm_variant == 9 || g_gemm_variant >= 12 || g_gemm_variant < 0) && M >= 4096 && N % BN2 == 0 &&
                  n_partial % BN2 == 0 && n_partial > 0 && n_partial <= N && pp_domain(M, N, K, c_rows);
  if (!ok) return fr_gemm_nt_bf16(A, W, bias, nullptr, C, M, N, K, 0, c_rows, s);
  const int tiles_n = N / BN2, tiles_m = (M + BM2 - 1) / BM2, ntiles_max = tiles_m * tiles_n;
  const int G = ntiles_max < num_cus() ? ntiles_max : num_cus();
  const bf16* a = (const bf16*)A;
  const bf16* w = (const bf16*)W;
  bf16* c = (bf16*)C;
  if (g_gemm_variant != 9 && (g_gemm_variant >= 12 || M < (1 << 18))) {
    if (bias)
      hipLaunchKernelGGL((gemm_nt_pp3_kernel<0, true, false, true>), dim3(G), dim3(512), 0, s, a, w, bias, c, M, N, K,
                         tiles_n, ntiles_max, full_rows, n_partial / BN2);
    else
      hipLaunchKernelGGL((gemm_nt_pp3_kernel<0, false, false, true>), dim3(G), dim3(512), 0, s, a, w, bias, c, M, N,
                         K, tiles_n, ntiles_max, full_rows, n_partial / BN2);
    return 0;
  }
  if (bias)
    hipLaunchKernelGGL((gemm_nt_pp2_kernel<0, true, false>), dim3(G), dim3(512), 0, s, a, w, bias, nullptr, c, M, N, K,
                       tiles_n, ntiles_max, full_rows, n_partial / BN2);
  else
    hipLaunchKernelGGL((gemm_nt_pp2_kernel<0, false, false>), dim3(G), dim3(512), 0, s, a, w, bias, nullptr, c, M, N, K,
                       tiles_n, ntiles_max, full_rows, n_partial / BN2);
  return 0;
}

// Training FFN1: C = GELU(A W^T + bias) and Z = A W^T + bias from one pass (variant-9 kernel,
// its domain only: returns 3 otherwise and the caller runs GEMM + separate GELU).
// Training FFN2 dgrad with the GELU derivative and the FFN1 bias gradient: C = (A W^T) *
// GELU'(Z) and colpart[tiles_m * 2, N] = per-(row tile, wave row) column sums of C (summed on
// the host side in a fixed order).  Variant-9 kernel only: returns 3 outside its domain.
extern "C" int fr_gemm_gelu_bwd_colpart(const void* A, const void* W, const void* Z, void* C, float* colpart, int M,
                                        int N, int K, int c_rows, hipStream_t s) {
  const bool ok = (g_gemm_variant == 9 || g_gemm_variant >= 12 || g_gemm_variant < 0) && M >= 4096 && N % BN2 == 0 &&
                  K % BK == 0 && pp_domain(M, N, K, c_rows);
  if (!ok) return 3;
  const int tiles_n = N / BN2, tiles_m = (M + BM2 - 1) / BM2, ntiles = tiles_m * tiles_n;
  const int G = ntiles < num_cus() ? ntiles : num_cus();
  hipLaunchKernelGGL((gemm_nt_pp2_kernel<3, false, true>), dim3(G), dim3(512), 0, s, (const bf16*)A, (const bf16*)W,
                     nullptr, (const bf16*)Z, (bf16*)C, M, N, K, tiles_n, ntiles, nullptr, 0, nullptr, colpart);
  return 0;
}

extern "C" int fr_gemm_nt_bf16_dual(const void* A, const void* W, const float* bias, void* C, void* Z, int M, int N, int K,
                                    int c_rows, hipStream_t s) {
  const bool ok = (g_gemm_variant == 9 || g_gemm_variant >= 12 || g_gemm_variant < 0) && M >= 4096 && N % BN2 == 0 &&
                  K % BK == 0 && bias != nullptr && pp_domain(M, N, K, c_rows);
  if (!ok) return 3;
  const int tiles_n = N / BN2, tiles_m = (M + BM2 - 1) / BM2, ntiles = tiles_m * tiles_n;
  const int G = ntiles < num_cus() ? ntiles : num_cus();
  if (g_gemm_variant != 9 && (g_gemm_variant >= 12 || M < (1 << 18))) {
    hipLaunchKernelGGL((gemm_nt_pp3_kernel<1, true, true, true>), dim3(G), dim3(512), 0, s, (const bf16*)A, (const bf16*)W,
                       bias, (bf16*)C, M, N, K, tiles_n, ntiles, nullptr, 0, (bf16*)Z);
    return 0;
  }
  hipLaunchKernelGGL((gemm_nt_pp2_kernel<1, true, false, true>), dim3(G), dim3(512), 0, s, (const bf16*)A,
                     (const bf16*)W, bias, nullptr, (bf16*)C, M, N, K, tiles_n, ntiles, nullptr, 0, (bf16*)Z);
  return 0;
}
