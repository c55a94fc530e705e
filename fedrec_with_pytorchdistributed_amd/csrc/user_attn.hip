// User-encoder multi-head self-attention core (reference attention.py:32-82):
//
//   S = Q K^T / sqrt(d_k),  A = exp(S) / (rowsum exp(S) + 1e-8),  ctx = A V
//
// 20 heads x d_k 20 over the clicked news, fp32.  H <= 64 runs on the matrix cores in fp32
// (v_mfma_f32_16x16x4_f32, the "matrix-core forms" below); long histories (H > 64) on the
// VALU kernels at the end (online softmax over 64-row chunks).  (The round-2 VALU forms and a
// one-wave MFMA form measured slower at H <= 64 and were removed in round 4.)  The eps softmax is
// evaluated stably:
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

// K/V rows staged as [H][DK] fp32 (80-B rows, 16-B aligned): every key row is 5 broadcast
// ds_read_b128 instead of 20 ds_read_b32
__device__ __forceinline__ float dot20(const float (&q)[DK], const float* __restrict__ row) {
  float d = 0.f;
#pragma unroll
  for (int c4 = 0; c4 < DK / 4; ++c4) {
    const float4 k = *(const float4*)(row + 4 * c4);
    d += q[4 * c4] * k.x + q[4 * c4 + 1] * k.y + q[4 * c4 + 2] * k.z + q[4 * c4 + 3] * k.w;
  }
  return d;
}

__device__ __forceinline__ void axpy20(float (&acc)[DK], float a, const float* __restrict__ row) {
#pragma unroll
  for (int c4 = 0; c4 < DK / 4; ++c4) {
    const float4 v = *(const float4*)(row + 4 * c4);
    acc[4 * c4] += a * v.x;
    acc[4 * c4 + 1] += a * v.y;
    acc[4 * c4 + 2] += a * v.z;
    acc[4 * c4 + 3] += a * v.w;
  }
}

// ---------------------------------------------------------------------------------------
// Matrix-core forms (default for H <= 64): every product of the attention runs on
// v_mfma_f32_16x16x4_f32 -- fp32 in, fp32 accumulate, one rounding per product, so the numerics
// are the fp32 reference's (attention.py:38-44) up to summation order.  d_k = 20 is exactly 5
// k-steps of 4; the H <= 64 rows pad to 16-row tiles (rows >= H read as zeros, keys >= H get
// probability 0).  One wave per (impression, head); Q, K, V (and dctx) rows are staged in LDS
// as [64][20] fp32 (80-B rows: a 16 x 4 operand read hits 64 distinct banks), the probability /
// dS tile goes through a [64][68] LDS image to change its lane layout between products.
//
// v_mfma_f32_16x16x4_f32 lane maps (cdna_hip_programming.md §3): A[i][k] from lane
// (i = l & 15, k = l >> 4); B[k][j] from lane (k = l >> 4, j = l & 15); C[row][col] in lane
// (col = l & 15, row = 4 (l >> 4) + reg).
//
// forward:  S = Q K^T (80 MFMA), row softmax on the C layout (xor-shuffles over the 16 lanes
//           of a row), ctx = P V (P through LDS; <= 128 MFMA), saves (m, 1/l) per row.
// backward: S again -> P; dP = dctx V^T (80); D_t = sum_s P dP; dS = P (dP - D) / sqrt(d_k);
//           dV = P^T dctx, dQ = dS K, dK = dS^T Q (<= 128 each, P / dS through LDS).
// ---------------------------------------------------------------------------------------
constexpr int PLD = 68;  // LDS row stride of the [64 x 64] P / dS image (conflict-free both ways)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// rows [0, 16 NT) of NOP [H, DK] head slices (row stride ld each) into xs[o][64][DK], zero rows
// >= H.  Every load of every slice is issued before the first LDS store (5 NT / 4 float4 per
// lane and slice in flight), the row index is clamped and the padded rows zeroed by a select:
// a load guarded by a per-lane condition compiles to a branch around it with a vmcnt(0) wait
// per load (cdna_hip_programming.md §5 trap (c)), and staging the slices one after the other
// waited out one load latency per slice
template <int NT, int NOP>
__device__ __forceinline__ void stage_heads(float (*const (&xs)[NOP])[DK], const float* const (&src)[NOP],
                                            const size_t (&ld)[NOP], int H, int lane) {
  constexpr int N4 = NT * 16 * (DK / 4);  // float4 chunks of one padded slice
  constexpr int IT = (N4 + 63) / 64;
  float4 v[NOP][IT];
#pragma unroll
  for (int o = 0; o < NOP; ++o)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = lane + 64 * it;
      const int r = min(i / (DK / 4), H - 1), c = (i % (DK / 4)) * 4;
      v[o][it] = *(const float4*)(src[o] + (size_t)r * ld[o] + c);
    }
#pragma unroll
  for (int o = 0; o < NOP; ++o)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = lane + 64 * it;
      const int r = i / (DK / 4), c = (i - r * (DK / 4)) * 4;
      const bool z = r >= H;
      const float4 w = make_float4(z ? 0.f : v[o][it].x, z ? 0.f : v[o][it].y, z ? 0.f : v[o][it].z,
                                   z ? 0.f : v[o][it].w);
      if (i < N4) *(float4*)&xs[o][r][c] = w;
    }
}

// C[i][j] += X Y^T over d_k for 16-row tiles i, j < NT (X, Y: [64][DK] in LDS)
template <int NT>
__device__ __forceinline__ void mm_xyT(f32x4 (&c)[4][4], float (*X)[DK], float (*Y)[DK], int fr, int fq) {
#pragma unroll
  for (int kk = 0; kk < DK / 4; ++kk) {
    float a[NT], b[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) a[i] = X[i * 16 + fr][4 * kk + fq];
#pragma unroll
    for (int j = 0; j < NT; ++j) b[j] = Y[j * 16 + fr][4 * kk + fq];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) c[i][j] = mfma4(a[i], b[j], c[i][j]);
  }
}

// out[i][dj] = sum_k A(i*16 + fr, k) * Y[k][dj*16 + fr'] over k < KS*4, A read from the
// [64][PLD] image P either as P[row][k] (TRANS = false) or P[k][row] (TRANS = true)
template <int NT, bool TRANS>
__device__ __forceinline__ void mm_pY(f32x4 (&o)[4][2], const float* __restrict__ P, float (*Y)[DK], int KS, int fr,
                                      int fq) {
#pragma unroll
  for (int kk = 0; kk < NT * 4; ++kk) {  // unrolled to the tile bound: LDS reads hoist over MFMAs
    if (kk >= KS) break;
    const int k = 4 * kk + fq;
    // (column 16 + fr >= DK reads the next row -- the arrays carry a 16-float tail -- and is
    // zeroed by the select: no branch around the LDS read)
    const float y0 = Y[k][fr], y1r = Y[k][16 + fr], y1 = fr < DK - 16 ? y1r : 0.f;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const float a = TRANS ? P[k * PLD + i * 16 + fr] : P[(i * 16 + fr) * PLD + k];
      o[i][0] = mfma4(a, y0, o[i][0]);
      o[i][1] = mfma4(a, y1, o[i][1]);
    }
  }
}

// store rows (tile i: 4 fq + r) x columns (dj*16 + fr < DK) of o, scaled per row by rs[i][r]
template <int NT>
__device__ __forceinline__ void store_head(float* __restrict__ dst, size_t ld, const f32x4 (&o)[4][2],
                                           const float (*rs)[4], int H, int fr, int fq) {
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i * 16 + fq * 4 + r;
      if (row >= H) continue;
      const float sc = rs != nullptr ? rs[i][r] : 1.f;
      dst[(size_t)row * ld + fr] = o[i][0][r] * sc;
      if (fr < DK - 16) dst[(size_t)row * ld + 16 + fr] = o[i][1][r] * sc;
    }
}

// reductions over the 16 lanes of a DPP row (= one C-layout row of a 16x16 tile): four DPP
// butterflies (quad_perm xor 1, xor 2, row_half_mirror, row_mirror) -- VALU-speed lane moves,
// where __shfl_xor is a ds_bpermute round trip through the LDS crossbar per step
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
constexpr int DPP_XOR1 = 0xB1;       // quad_perm [1, 0, 3, 2]
constexpr int DPP_XOR2 = 0x4E;       // quad_perm [2, 3, 0, 1]
constexpr int DPP_HALF_MIRROR = 0x141;
constexpr int DPP_MIRROR = 0x140;
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp<DPP_XOR1>(v));
  v = fmaxf(v, dpp<DPP_XOR2>(v));
  v = fmaxf(v, dpp<DPP_HALF_MIRROR>(v));
  return fmaxf(v, dpp<DPP_MIRROR>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<DPP_XOR1>(v);
  v += dpp<DPP_XOR2>(v);
  v += dpp<DPP_HALF_MIRROR>(v);
  return v + dpp<DPP_MIRROR>(v);
}

// mask_padding option's key mask, attention.py:76-78: masked keys get weight exactly 0; a row
// with every key masked gives ctx = 0, as the torch oracle's eps-softmax)
__device__ __forceinline__ bool key_kept(const int* __restrict__ keep, int b, int H, int t) {
  return keep == nullptr || keep[(size_t)b * H + t] != 0;
}

// The attention forward of one (impression b, head h) once its Q, K, V slices sit in LDS (rows
// >= H zero): S = Q K^T, eps-softmax, ctx = P V, (m, 1/l) per row.  Wave w takes query rows
// [16 w, 16 w + 16).
__device__ __forceinline__ void attn_fwd_body(float (*qs)[DK], float (*ks)[DK], float (*vs)[DK], float* ps, int b,
                                              int h, int H, int NH, const int* __restrict__ keep,
                                              float* __restrict__ ctx, float* __restrict__ stats,
                                              bf16* __restrict__ ctx_b) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int D = NH * DK;
  const int i0 = wave * 16;
  if (i0 >= H) return;  // wave-uniform; no barrier follows
  const int NT = (H + 15) / 16;
  bool kept[4];  // this lane's key columns j * 16 + fr
#pragma unroll
  for (int j = 0; j < 4; ++j) kept[j] = j * 16 + fr < H && key_kept(keep, b, H, min(j * 16 + fr, H - 1));
  f32x4 s[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < DK / 4; ++kk) {
    const float a = qs[i0 + fr][4 * kk + fq];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < NT) s[j] = mfma4(a, ks[j * 16 + fr][4 * kk + fq], s[j]);
  }
  const float scale = rsqrtf((float)DK);
  float* pw = ps + wave * 16 * PLD;  // this wave's 16 rows of P
  float inv[4], mrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = (j < NT && kept[j]) ? s[j][r] * scale : -INFINITY;
      s[j][r] = v;
      m = fmaxf(m, v);
    }
    m = row16_max(m);
    if (m == -INFINITY) m = 0.f;  // every key masked: weights 0, ctx 0
    float l = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float p = __expf(s[j][r] - m);
      l += p;
      pw[(fq * 4 + r) * PLD + j * 16 + fr] = p;
    }
    l = row16_sum(l) + 1e-8f * __expf(-m);
    inv[r] = 1.0f / l;
    mrow[r] = m;
  }
  f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = o0;
  const int KS = (H + 3) / 4;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    if (kk >= KS) break;
    const int k = 4 * kk + fq;
    const float a = pw[fr * PLD + k];
    const float y0 = vs[k][fr], y1r = vs[k][16 + fr], y1 = fr < DK - 16 ? y1r : 0.f;
    o0 = mfma4(a, y0, o0);
    o1 = mfma4(a, y1, o1);
  }
  float* dst = ctx + (size_t)b * H * D + h * DK;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = i0 + fq * 4 + r;
    if (row >= H) continue;
    dst[(size_t)row * D + fr] = o0[r] * inv[r];
    if (fr < DK - 16) dst[(size_t)row * D + 16 + fr] = o1[r] * inv[r];
    if (ctx_b != nullptr) {  // lane pairs (fr, fr ^ 1) -> one 4-byte bf16x2 store by the even lane
      bf16* db = ctx_b + ((size_t)b * H + row) * D + h * DK;
      const float c0 = o0[r] * inv[r], c1 = o1[r] * inv[r];
      const float n0 = dpp<DPP_XOR1>(c0), n1 = dpp<DPP_XOR1>(c1);
      if ((fr & 1) == 0) {
        *(bf16x2*)(db + fr) = bf16x2{f2bf(c0), f2bf(n0)};
        if (fr < DK - 16) *(bf16x2*)(db + 16 + fr) = bf16x2{f2bf(c1), f2bf(n1)};
      }
    }
    if (fr == 0) {
      float* st = stats + (((size_t)b * NH + h) * H + row) * 2;
      st[0] = mrow[r];
      st[1] = inv[r];
    }
  }
}

// SR = 65: 33,008 B of LDS, four blocks per CU (64-row stages, five blocks per CU, measured
// neutral: profiles/r3_ab_segsum_ua.txt)
// ctx_b (optional): ctx rounded to bf16 as well (the att_fc1 GEMM's operand)
template <int SR>
__global__ __launch_bounds__(256) void user_attn_fwd_mfma4_kernel(const float* __restrict__ qkv,
                                                                  float* __restrict__ ctx, float* __restrict__ stats,
                                                                  int H, int NH, const int* __restrict__ keep,
                                                                  bf16* __restrict__ ctx_b) {
  __shared__ __attribute__((aligned(16))) float qs[SR][DK];
  __shared__ __attribute__((aligned(16))) float ks[SR][DK];
  __shared__ __attribute__((aligned(16))) float vs[SR][DK];
  __shared__ __attribute__((aligned(16))) float ps[64 * PLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x / NH, h = blockIdx.x - b * NH;
  const int ld = 3 * NH * DK, D = NH * DK;
  const float* base = qkv + (size_t)b * H * ld + h * DK;
  {  // 3 x 320 float4 chunks over 256 threads, every load in flight before the stores
    float4 v[3][2];
#pragma unroll
    for (int o = 0; o < 3; ++o)
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int i = tid + 256 * it;
        const int r = min(min(i, 319) / (DK / 4), H - 1), c = (i % (DK / 4)) * 4;
        v[o][it] = *(const float4*)(base + (size_t)o * D + (size_t)r * ld + c);
      }
    float (*const xs[3])[DK] = {qs, ks, vs};
#pragma unroll
    for (int o = 0; o < 3; ++o)
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int i = tid + 256 * it;
        const int r = i / (DK / 4), c = (i - r * (DK / 4)) * 4;
        const bool z = r >= H;
        const float4 w = make_float4(z ? 0.f : v[o][it].x, z ? 0.f : v[o][it].y, z ? 0.f : v[o][it].z,
                                     z ? 0.f : v[o][it].w);
        if (i < 320) *(float4*)&xs[o][r][c] = w;
      }
  }
  __syncthreads();
  attn_fwd_body(qs, ks, vs, ps, b, h, H, NH, keep, ctx, stats, ctx_b);
}

// Q|K|V projection fused into the attention forward (H <= 64, bf16 operands): the block of
// (b, h) computes its head's [H x 3 DK] slice of X' W^T + bias -- X' = the impression's H
// gathered, dropped-out history rows (bf16 [B H, Din]), W = the bf16 stack [Wq; Wk; Wv]
// (rows o D + h DK + c) -- on v_mfma_f32_16x16x32_bf16 with the fragments loaded straight into
// registers (small_gemm.hip's register-direct form: 4 waves in 2 x 2 over the 64 x 64 padded
// tile, 3 k-steps in flight, B as src0 so a lane holds 4 consecutive output columns), puts it
// in LDS (rows >= H zero) and in qkv [B H, 3 D] fp32 (the backward's input), and runs the
// attention on it.  The separate GEMM launch wrote the same qkv (same MFMA, same k order): one
// launch and the qkv read-back fewer per step.
constexpr uint32_t QA_OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t qa_rsrc(const void* p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), 0, 0x7FFFFFF0, 0x00020000);
}

template <int SR>
__global__ __launch_bounds__(256) void user_qkv_attn_fwd_kernel(const bf16* __restrict__ xd,
                                                                const bf16* __restrict__ W,
                                                                const float* __restrict__ bias, int Din,
                                                                float* __restrict__ qkv, float* __restrict__ ctx,
                                                                float* __restrict__ stats, int H, int NH,
                                                                const int* __restrict__ keep,
                                                                bf16* __restrict__ ctx_b) {
  __shared__ __attribute__((aligned(16))) float qs[SR][DK];
  __shared__ __attribute__((aligned(16))) float ks[SR][DK];
  __shared__ __attribute__((aligned(16))) float vs[SR][DK];
  __shared__ __attribute__((aligned(16))) float ps[64 * PLD];
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x / NH, h = blockIdx.x - b * NH;
  const int D = NH * DK;
  const int wm = wave >> 1, wn = wave & 1;
  const __amdgpu_buffer_rsrc_t rsa = qa_rsrc(xd), rsb = qa_rsrc(W);
  uint32_t oa[2], ob[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = wm * 32 + i * 16 + fr;  // history row of this impression
    oa[i] = m < H ? (uint32_t)(((size_t)b * H + m) * Din + 8 * fq) * 2u : QA_OOB;
    const int n = wn * 32 + i * 16 + fr;  // output column: o = n / DK (q, k, v), c = n % DK
    ob[i] = n < 3 * DK ? (uint32_t)(((n / DK) * D + h * DK + n % DK) * Din + 8 * fq) * 2u : QA_OOB;
  }
  constexpr int P = 3;
  const int nk = (Din + 31) >> 5;
  u32x4_t ra[P][2], rb[P][2];
  auto load = [&](int s, int kt) {
    const bool kok = kt * 32 + 8 * fq < Din;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ra[s][i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rsa, kok ? oa[i] + kt * 64 : QA_OOB, 0, 0));
      rb[s][i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rsb, kok ? ob[i] + kt * 64 : QA_OOB, 0, 0));
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int s) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, rb[s][j]),
                                                            __builtin_bit_cast(bf16x8, ra[s][i]), acc[i][j], 0, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < P; ++s) load(s, s);
  const int nfull = nk / P * P;
  for (int kt = 0; kt < nfull; kt += P) {
#pragma unroll
    for (int s = 0; s < P; ++s) {
      mma(s);
      load(s, kt + s + P);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int s = 0; s < P - 1; ++s)
    if (nfull + s < nk) mma(s);
  // lane holds C[m = wm 32 + 16 i + fr][n = wn 32 + 16 j + 4 fq + r]: 4 consecutive columns of one
  // of q / k / v (DK % 4 == 0)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 32 + j * 16 + 4 * fq;
    if (n >= 3 * DK) continue;
    const int o = n / DK, c = n - o * DK;
    float (*const xo)[DK] = o == 0 ? qs : (o == 1 ? ks : vs);
    const float4 bb = *(const float4*)(bias + o * D + h * DK + c);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = wm * 32 + i * 16 + fr;
      if (m >= SR) continue;
      const bool real = m < H;
      const float4 v = real ? make_float4(acc[i][j][0] + bb.x, acc[i][j][1] + bb.y, acc[i][j][2] + bb.z,
                                          acc[i][j][3] + bb.w)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      *(float4*)&xo[m][c] = v;
      if (real) *(float4*)(qkv + ((size_t)b * H + m) * (3 * D) + o * D + h * DK + c) = v;
    }
  }
  __syncthreads();
  attn_fwd_body(qs, ks, vs, ps, b, h, H, NH, keep, ctx, stats, ctx_b);
}

// Backward LDS: 38,208 B with PLDB = 68 and 65-row stages -- four blocks per CU.  P and dS share
// one [64][PLDB] image: P first (dV = P^T dctx reads it), then, after a barrier, dS (dQ and
// dK = dS^T Q); the dS values wait in registers (16 per lane) meanwhile.  (The first form kept
// both images, 55,616 B: two blocks per CU, 2.5 rounds of the 1,280 (impression, head) blocks.)
// OT: the dqkv element type (bf16: the input / weight gradient GEMMs' operand, rounded once here)
__device__ __forceinline__ float cvt_out(float v, float*) { return v; }
__device__ __forceinline__ bf16 cvt_out(float v, bf16*) { return f2bf(v); }

// FD: the additive pool's input-gradient GEMM fused in -- dctx = dctx_direct + dpre W1 (dctx_direct
// = alpha du from the pool's backward, in `dctx`; dpre bf16 [B H, Qd], W1^T bf16 [D, Qd]): the
// block of (b, h) computes its [H x DK] slice of dpre W1 on v_mfma_f32_16x16x32_bf16 with the
// fragments loaded straight into registers (wave w: rows 16 w.., both 16-column tiles of the
// head's DK = 20 columns), adds it to the staged dctx_direct -- (acc + 0) + dctx_direct, the
// small-GEMM epilogue's arithmetic, so the sum is bitwise the separate launch's -- and runs the
// attention backward on it.  One launch (and the dctx round trip) fewer per step.
template <int SR, int PLDB, typename OT = float, bool FD = false>
__global__ __launch_bounds__(256) void user_attn_bwd_mfma4_kernel(const float* __restrict__ qkv,
                                                                  const float* __restrict__ stats,
                                                                  const float* __restrict__ dctx,
                                                                  OT* __restrict__ dqkv, int H, int NH,
                                                                  const int* __restrict__ keep,
                                                                  const bf16* __restrict__ dpre = nullptr,
                                                                  const bf16* __restrict__ w1t = nullptr,
                                                                  int Qd = 0) {
  __shared__ __attribute__((aligned(16))) float qs[SR][DK];
  __shared__ __attribute__((aligned(16))) float ks[SR][DK];
  __shared__ __attribute__((aligned(16))) float vs[SR][DK];
  __shared__ __attribute__((aligned(16))) float gs[SR][DK];
  __shared__ __attribute__((aligned(16))) float pd[64 * PLDB];  // P, then dS
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x / NH, h = blockIdx.x - b * NH;
  const int ld = 3 * NH * DK, D = NH * DK;
  const float* base = qkv + (size_t)b * H * ld + h * DK;
  const float* gbase = dctx + (size_t)b * H * D + h * DK;
  {
    float4 v[4][2];
#pragma unroll
    for (int o = 0; o < 4; ++o)
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int i = tid + 256 * it;
        const int r = min(min(i, 319) / (DK / 4), H - 1), c = (i % (DK / 4)) * 4;
        v[o][it] = o < 3 ? *(const float4*)(base + (size_t)o * D + (size_t)r * ld + c)
                         : *(const float4*)(gbase + (size_t)r * D + c);
      }
    float (*const xs[4])[DK] = {qs, ks, vs, gs};
#pragma unroll
    for (int o = 0; o < 4; ++o)
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int i = tid + 256 * it;
        const int r = i / (DK / 4), c = (i - r * (DK / 4)) * 4;
        const bool z = r >= H;
        const float4 w = make_float4(z ? 0.f : v[o][it].x, z ? 0.f : v[o][it].y, z ? 0.f : v[o][it].z,
                                     z ? 0.f : v[o][it].w);
        if (i < 320) *(float4*)&xs[o][r][c] = w;
      }
  }
  if constexpr (FD) {
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rsa = qa_rsrc(dpre), rsb = qa_rsrc(w1t);
    const int m = wave * 16 + fr;
    const uint32_t oa = m < H ? (uint32_t)(((size_t)b * H + m) * Qd + 8 * fq) * 2u : QA_OOB;
    uint32_t ob[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = j * 16 + fr;
      ob[j] = c < DK ? (uint32_t)((h * DK + c) * Qd + 8 * fq) * 2u : QA_OOB;
    }
    constexpr int P = 3;
    const int nk = (Qd + 31) >> 5;
    u32x4_t ra[P], rb[P][2];
    auto load = [&](int sl, int kt) {
      const bool kok = kt * 32 + 8 * fq < Qd;
      ra[sl] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rsa, kok ? oa + kt * 64 : QA_OOB, 0, 0));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        rb[sl][j] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rsb, kok ? ob[j] + kt * 64 : QA_OOB, 0, 0));
    };
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    auto mma = [&](int sl) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, rb[sl][j]),
                                                         __builtin_bit_cast(bf16x8, ra[sl]), acc[j], 0, 0, 0);
    };
#pragma unroll
    for (int sl = 0; sl < P; ++sl) load(sl, sl);
    const int nfull = nk / P * P;
    for (int kt = 0; kt < nfull; kt += P) {
#pragma unroll
      for (int sl = 0; sl < P; ++sl) {
        mma(sl);
        load(sl, kt + sl + P);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int sl = 0; sl < P - 1; ++sl)
      if (nfull + sl < nk) mma(sl);
    __syncthreads();  // the staged dctx_direct rows are in LDS
    // lane holds (dpre W1)[m][c = 16 j + 4 fq + r]
    if (m < H) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = j * 16 + 4 * fq;
        if (c < DK) {
          float4 g = *(float4*)&gs[m][c];
          g.x = (acc[j][0] + 0.f) + g.x;
          g.y = (acc[j][1] + 0.f) + g.y;
          g.z = (acc[j][2] + 0.f) + g.z;
          g.w = (acc[j][3] + 0.f) + g.w;
          *(float4*)&gs[m][c] = g;
        }
      }
    }
  }
  const int i0 = wave * 16;
  const int NT = (H + 15) / 16;
  const float* st = stats + ((size_t)b * NH + h) * H * 2;
  float mrow[4], inv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = i0 + fq * 4 + r, rc = min(row, H - 1);
    const float mv = st[2 * rc], iv = st[2 * rc + 1];
    mrow[r] = row < H ? mv : 0.f;
    inv[r] = row < H ? iv : 0.f;
  }
  __syncthreads();
  const float scale = rsqrtf((float)DK);
  OT* dst = dqkv + (size_t)b * H * ld + h * DK;
  const int KS = (H + 3) / 4;
  const bool act = i0 < H;  // this wave's query / key tile holds real rows (wave-uniform)
  float dsv[4][4];          // this wave's dS rows (registers while P is read from LDS)
  if (act) {  // query tile: P, dP, D; P into LDS, dS kept
    bool kept[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) kept[j] = j * 16 + fr < H && key_kept(keep, b, H, min(j * 16 + fr, H - 1));
    f32x4 p[4], dp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = dp[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < DK / 4; ++kk) {
      const float a = qs[i0 + fr][4 * kk + fq], g = gs[i0 + fr][4 * kk + fq];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < NT) {
          p[j] = mfma4(a, ks[j * 16 + fr][4 * kk + fq], p[j]);
          dp[j] = mfma4(g, vs[j * 16 + fr][4 * kk + fq], dp[j]);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float Dt = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float pv = (j < NT && kept[j]) ? __expf(p[j][r] * scale - mrow[r]) * inv[r] : 0.f;
        p[j][r] = pv;
        Dt += pv * dp[j][r];
      }
      Dt = row16_sum(Dt);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pd[(i0 + fq * 4 + r) * PLDB + j * 16 + fr] = p[j][r];
        dsv[j][r] = p[j][r] * (dp[j][r] - Dt) * scale;
      }
    }
  }
  __syncthreads();  // every P row in LDS
  if (act) {  // key tile i0: dV = P^T dctx (sums over every query)
    f32x4 v0 = f32x4{0.f, 0.f, 0.f, 0.f}, v1 = v0;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      if (kk >= KS) break;
      const int t = 4 * kk + fq;
      const float pa = pd[t * PLDB + i0 + fr];
      const float g0 = gs[t][fr], g1r = gs[t][16 + fr], g1 = fr < DK - 16 ? g1r : 0.f;
      v0 = mfma4(pa, g0, v0);
      v1 = mfma4(pa, g1, v1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i0 + fq * 4 + r;
      if (row >= H) continue;
      dst[(size_t)row * ld + 2 * D + fr] = cvt_out(v0[r], dst);
      if (fr < DK - 16) dst[(size_t)row * ld + 2 * D + 16 + fr] = cvt_out(v1[r], dst);
    }
  }
  __syncthreads();  // every wave done reading P: the image takes dS
  if (act) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) pd[(i0 + fq * 4 + r) * PLDB + j * 16 + fr] = dsv[j][r];
    // dQ rows of this tile = dS K (this wave's own dS rows: written by this wave, in order)
    f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = o0;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      if (kk >= KS) break;
      const int k = 4 * kk + fq;
      const float a = pd[(i0 + fr) * PLDB + k];
      const float y0 = ks[k][fr], y1r = ks[k][16 + fr], y1 = fr < DK - 16 ? y1r : 0.f;
      o0 = mfma4(a, y0, o0);
      o1 = mfma4(a, y1, o1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i0 + fq * 4 + r;
      if (row >= H) continue;
      dst[(size_t)row * ld + fr] = cvt_out(o0[r], dst);
      if (fr < DK - 16) dst[(size_t)row * ld + 16 + fr] = cvt_out(o1[r], dst);
    }
  }
  __syncthreads();  // every dS row in LDS
  if (!act) return;
  // key tile i0: dK = dS^T Q
  f32x4 k0 = f32x4{0.f, 0.f, 0.f, 0.f}, k1 = k0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    if (kk >= KS) break;
    const int t = 4 * kk + fq;
    const float da = pd[t * PLDB + i0 + fr];
    const float q0 = qs[t][fr], q1r = qs[t][16 + fr], q1 = fr < DK - 16 ? q1r : 0.f;
    k0 = mfma4(da, q0, k0);
    k1 = mfma4(da, q1, k1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = i0 + fq * 4 + r;
    if (row >= H) continue;
    dst[(size_t)row * ld + D + fr] = cvt_out(k0[r], dst);
    if (fr < DK - 16) dst[(size_t)row * ld + D + 16 + fr] = cvt_out(k1[r], dst);
  }
}


// ---------------------------------------------------------------------------------------
// Long histories (H > 64): the reference pads but never truncates (dataset.py:84, quirk Q6;
// its shipped shard has H = 76), and SURVEY §5.7 asks for H limited only by memory.  Same
// math, one wave per (impression, head), query rows in chunks of 64 (lane = row), keys /
// values streamed through LDS in chunks of 64 rows.  Forward: online softmax (running max
// with rescale), so (m, 1/l) come out exactly as in the short kernel.  Backward: pass A
// (lane = query) keeps D_t in LDS for pass B (lane = key); per-row m, 1/l, D live in LDS,
// so H <= MAXL.
constexpr int CH = 64;
constexpr int MAXL = 2048;

__device__ __forceinline__ void stage_rows(float (*dst)[DK], const float* __restrict__ src, size_t ld, int r0,
                                           int n, int lane) {
  for (int i = lane; i < n * DK / 4; i += 64) {
    const int r = i / (DK / 4), c = (i - r * (DK / 4)) * 4;
    *(float4*)&dst[r][c] = *(const float4*)(src + (size_t)(r0 + r) * ld + c);
  }
}

__device__ __forceinline__ void load_row(float (&x)[DK], const float* __restrict__ p, float s) {
#pragma unroll
  for (int c4 = 0; c4 < DK / 4; ++c4) {
    const float4 v = *(const float4*)(p + 4 * c4);
    x[4 * c4] = v.x * s;
    x[4 * c4 + 1] = v.y * s;
    x[4 * c4 + 2] = v.z * s;
    x[4 * c4 + 3] = v.w * s;
  }
}

__global__ __launch_bounds__(64) void user_attn_fwd_long_kernel(const float* __restrict__ qkv, float* __restrict__ ctx,
                                                                float* __restrict__ stats, int B, int H, int NH,
                                                                const int* __restrict__ keep) {
  __shared__ __attribute__((aligned(16))) float ks[CH][DK];
  __shared__ __attribute__((aligned(16))) float vs[CH][DK];
  const int lane = threadIdx.x;
  const int b = blockIdx.x / NH, h = blockIdx.x - b * NH;
  const int ld = 3 * NH * DK, D = NH * DK;
  const float* base = qkv + (size_t)b * H * ld + h * DK;
  const float scale = rsqrtf((float)DK);
  for (int t0 = 0; t0 < H; t0 += CH) {
    const int t = t0 + lane;
    const bool valid = t < H;
    float q[DK], acc[DK];
    load_row(q, base + (size_t)(valid ? t : 0) * ld, scale);
#pragma unroll
    for (int c = 0; c < DK; ++c) acc[c] = 0.f;
    float m = -INFINITY, l = 0.f;
    for (int s0 = 0; s0 < H; s0 += CH) {
      const int n = min(CH, H - s0);
      __syncthreads();
      stage_rows(ks, base + D, ld, s0, n, lane);
      stage_rows(vs, base + 2 * D, ld, s0, n, lane);
      __syncthreads();
      float mc = m;
      for (int s = 0; s < n; ++s)
        if (key_kept(keep, b, H, s0 + s)) mc = fmaxf(mc, dot20(q, &ks[s][0]));
      // 0 on the first chunk with a kept key (m = -inf); a chunk before any kept key leaves
      // l = acc = 0, whatever the factor
      const float alpha = mc == -INFINITY ? 0.f : __expf(m - mc);
      l *= alpha;
#pragma unroll
      for (int c = 0; c < DK; ++c) acc[c] *= alpha;
      for (int s = 0; s < n; ++s) {
        if (!key_kept(keep, b, H, s0 + s)) continue;  // key index: the same for every lane
        const float p = __expf(dot20(q, &ks[s][0]) - mc);
        l += p;
        axpy20(acc, p, &vs[s][0]);
      }
      m = mc;
    }
    if (!valid) continue;
    if (m == -INFINITY) m = 0.f;  // every key masked: weights 0, ctx 0
    l += 1e-8f * __expf(-m);
    const float inv = 1.0f / l;
    float* o = ctx + ((size_t)b * H + t) * D + h * DK;
#pragma unroll
    for (int c4 = 0; c4 < DK / 4; ++c4)
      *(float4*)(o + 4 * c4) = make_float4(acc[4 * c4] * inv, acc[4 * c4 + 1] * inv, acc[4 * c4 + 2] * inv,
                                           acc[4 * c4 + 3] * inv);
    float* st = stats + (((size_t)b * NH + h) * H + t) * 2;
    st[0] = m;
    st[1] = inv;
  }
}

__global__ __launch_bounds__(64) void user_attn_bwd_long_kernel(const float* __restrict__ qkv,
                                                                const float* __restrict__ stats,
                                                                const float* __restrict__ dctx,
                                                                float* __restrict__ dqkv, int B, int H, int NH,
                                                                const int* __restrict__ keep) {
  __shared__ __attribute__((aligned(16))) float xs[CH][DK];  // keys (pass A) / queries (pass B)
  __shared__ __attribute__((aligned(16))) float ys[CH][DK];  // values (pass A) / dctx rows (pass B)
  __shared__ float ms[MAXL], is_[MAXL], Ds[MAXL];
  const int lane = threadIdx.x;
  const int b = blockIdx.x / NH, h = blockIdx.x - b * NH;
  const int ld = 3 * NH * DK, D = NH * DK;
  const float* base = qkv + (size_t)b * H * ld + h * DK;
  const float* gb = dctx + (size_t)b * H * D + h * DK;
  float* dbase = dqkv + (size_t)b * H * ld + h * DK;
  const float* st = stats + ((size_t)b * NH + h) * H * 2;
  for (int t = lane; t < H; t += 64) {
    ms[t] = st[2 * t];
    is_[t] = st[2 * t + 1];
  }
  const float scale = rsqrtf((float)DK);
  // pass A: lane = query t -> dq_t = scale (u - D_t w), D_t kept in LDS
  for (int t0 = 0; t0 < H; t0 += CH) {
    const int t = t0 + lane;
    const bool valid = t < H;
    const int tc = valid ? t : 0;
    float q[DK], g[DK], u[DK], w[DK];
    load_row(q, base + (size_t)tc * ld, scale);
    load_row(g, gb + (size_t)tc * D, 1.f);
#pragma unroll
    for (int c = 0; c < DK; ++c) u[c] = w[c] = 0.f;
    __syncthreads();  // ms / is_ written above (first chunk)
    const float m = ms[tc], inv = is_[tc];
    float Dt = 0.f;
    for (int s0 = 0; s0 < H; s0 += CH) {
      const int n = min(CH, H - s0);
      __syncthreads();
      stage_rows(xs, base + D, ld, s0, n, lane);
      stage_rows(ys, base + 2 * D, ld, s0, n, lane);
      __syncthreads();
      for (int s = 0; s < n; ++s) {
        if (!key_kept(keep, b, H, s0 + s)) continue;
        const float A = __expf(dot20(q, &xs[s][0]) - m) * inv;
        const float dA = dot20(g, &ys[s][0]);
        Dt += A * dA;
        axpy20(u, A * dA, &xs[s][0]);
        axpy20(w, A, &xs[s][0]);
      }
    }
    if (!valid) continue;
    Ds[t] = Dt;
    float* o = dbase + (size_t)t * ld;
#pragma unroll
    for (int c4 = 0; c4 < DK / 4; ++c4) {
      const int c = 4 * c4;
      *(float4*)(o + c) = make_float4(scale * (u[c] - Dt * w[c]), scale * (u[c + 1] - Dt * w[c + 1]),
                                      scale * (u[c + 2] - Dt * w[c + 2]), scale * (u[c + 3] - Dt * w[c + 3]));
    }
  }
  // pass B: lane = key s -> dk_s = sum_t dS_ts q_t, dv_s = sum_t A_ts dctx_t
  for (int s0 = 0; s0 < H; s0 += CH) {
    const int s = s0 + lane;
    const bool valid = s < H;
    const int sc = valid ? s : 0;
    float k[DK], v[DK], dk[DK], dv[DK];
    load_row(k, base + (size_t)sc * ld + D, scale);
    load_row(v, base + (size_t)sc * ld + 2 * D, 1.f);
    const float kf = key_kept(keep, b, H, sc) ? 1.f : 0.f;  // a masked key gets no gradient
#pragma unroll
    for (int c = 0; c < DK; ++c) dk[c] = dv[c] = 0.f;
    for (int t0 = 0; t0 < H; t0 += CH) {
      const int n = min(CH, H - t0);
      __syncthreads();  // also orders pass A's Ds writes before these reads
      stage_rows(xs, base, ld, t0, n, lane);
      stage_rows(ys, gb, D, t0, n, lane);
      __syncthreads();
      for (int j = 0; j < n; ++j) {
        const int t = t0 + j;
        const float A = kf * __expf(dot20(k, &xs[j][0]) - ms[t]) * is_[t];
        const float dA = dot20(v, &ys[j][0]);
        const float dS = A * (dA - Ds[t]) * scale;
        axpy20(dk, dS, &xs[j][0]);
        axpy20(dv, A, &ys[j][0]);
      }
    }
    if (!valid) continue;
    float* o = dbase + (size_t)s * ld;
#pragma unroll
    for (int c4 = 0; c4 < DK / 4; ++c4) {
      const int c = 4 * c4;
      *(float4*)(o + D + c) = make_float4(dk[c], dk[c + 1], dk[c + 2], dk[c + 3]);
      *(float4*)(o + 2 * D + c) = make_float4(dv[c], dv[c + 1], dv[c + 2], dv[c + 3]);
    }
  }
}

}  // namespace

// keep: optional [B, H] int32 key mask (mask_padding)
// ctx_b (optional, bf16 [B, H, NH dk]): ctx rounded to bf16 too -- short histories only (H <= 64;
// returns 2 otherwise, before launching anything)
extern "C" int fr_user_attn_fwd(const float* qkv, float* ctx, float* stats, int B, int H, int NH, int dk,
                                const int* keep, hipStream_t s, void* ctx_b) {
  if (dk != DK || H > MAXL || H < 1) return 1;
  if (ctx_b != nullptr && H > MAXH) return 2;
  const int pairs = B * NH;
  if (pairs == 0) return 0;
  if (H > MAXH)
    hipLaunchKernelGGL(user_attn_fwd_long_kernel, dim3(pairs), dim3(64), 0, s, qkv, ctx, stats, B, H, NH, keep);
  else
    hipLaunchKernelGGL(user_attn_fwd_mfma4_kernel<65>, dim3(pairs), dim3(256), 0, s, qkv, ctx, stats, H, NH, keep,
                       (bf16*)ctx_b);
  return 0;
}

// Q|K|V projection + attention forward in one launch (H <= 64; 1 = not this form's shape, nothing
// launched): xd bf16 [B H, Din], W bf16 [3 NH dk, Din] (the q / k / v row blocks), bias fp32
// [3 NH dk]; qkv [B H, 3 NH dk] fp32 is written for the backward
extern "C" int fr_user_qkv_attn_fwd(const void* xd, const void* W, const float* bias, int Din, float* qkv, float* ctx,
                                    float* stats, int B, int H, int NH, int dk, const int* keep, hipStream_t s,
                                    void* ctx_b) {
  if (dk != DK || H > MAXH || H < 1 || Din % 8 != 0 || Din < 8) return 1;
  if ((((uintptr_t)xd) & 15) || (((uintptr_t)W) & 15) || (((uintptr_t)bias) & 15) || (((uintptr_t)qkv) & 15)) return 1;
  if ((double)B * H * Din * 2 >= 2.0e9 || (double)3 * NH * DK * Din * 2 >= 2.0e9) return 1;  // 32-bit buffer offsets
  const int pairs = B * NH;
  if (pairs == 0) return 0;
  hipLaunchKernelGGL(user_qkv_attn_fwd_kernel<65>, dim3(pairs), dim3(256), 0, s, (const bf16*)xd, (const bf16*)W, bias,
                     Din, qkv, ctx, stats, H, NH, keep, (bf16*)ctx_b);
  return 0;
}

// The attention backward with the pool's dctx GEMM fused in (H <= 64, bf16 dqkv; 1 = not this
// form's shape, nothing launched): dctx holds dctx_direct (read only), dpre bf16 [B H, Qd], w1t
// bf16 [NH dk, Qd] (W1^T)
extern "C" int fr_user_attn_bwd_dctx(const float* qkv, const float* stats, const float* dctx, void* dqkv,
                                     const void* dpre, const void* w1t, int Qd, int B, int H, int NH, int dk,
                                     const int* keep, hipStream_t s) {
  if (dk != DK || H > MAXH || H < 1 || Qd % 8 != 0 || Qd < 8) return 1;
  if ((((uintptr_t)dpre) & 15) || (((uintptr_t)w1t) & 15)) return 1;
  if ((double)B * H * Qd * 2 >= 2.0e9) return 1;
  const int pairs = B * NH;
  if (pairs == 0) return 0;
  hipLaunchKernelGGL((user_attn_bwd_mfma4_kernel<65, 68, bf16, true>), dim3(pairs), dim3(256), 0, s, qkv, stats, dctx,
                     (bf16*)dqkv, H, NH, keep, (const bf16*)dpre, (const bf16*)w1t, Qd);
  return 0;
}

// out_bf16: dqkv is bf16 (short histories only; 2 otherwise, nothing launched)
extern "C" int fr_user_attn_bwd(const float* qkv, const float* stats, const float* dctx, void* dqkv, int B, int H,
                                int NH, int dk, const int* keep, hipStream_t s, int out_bf16) {
  if (dk != DK || H > MAXL || H < 1) return 1;
  if (out_bf16 && H > MAXH) return 2;
  const int pairs = B * NH;
  if (pairs == 0) return 0;
  if (H > MAXH)
    hipLaunchKernelGGL(user_attn_bwd_long_kernel, dim3(pairs), dim3(64), 0, s, qkv, stats, dctx, (float*)dqkv, B, H, NH,
                       keep);
  else if (out_bf16)
    hipLaunchKernelGGL((user_attn_bwd_mfma4_kernel<65, 68, bf16>), dim3(pairs), dim3(256), 0, s, qkv, stats, dctx,
                       (bf16*)dqkv, H, NH, keep);
  else
    hipLaunchKernelGGL((user_attn_bwd_mfma4_kernel<65, 68>), dim3(pairs), dim3(256), 0, s, qkv, stats, dctx,
                       (float*)dqkv, H, NH, keep);
  return 0;
}
