// Small fp32-in / fp32-out GEMMs on MFMA for the user encoder and the text head's FC
// (round-1 these were hipBLASLt fp32 calls plus torch glue).
//
//   C[m, n] = act(alpha * sum_k A(m, k) * B(n, k) + bias[n])  (+ C[m, n] when accumulating)
//
// Shapes are the user side's: M = B*H = 3200 history rows (or U titles), N / K in {200, 400,
// 768, 1200}, none of them multiples of the big GEMM's 128/64 tiling -- every edge is masked.
// Operands are converted fp32 -> bf16 on their way into LDS and multiplied with
// v_mfma_f32_16x16x32_bf16 (fp32 accumulate).  Layouts:
//   A: a_mode 0 = row-major [M, K] (optionally with a row gather m -> gidx[m] and a Philox
//      dropout on the gathered elements, index m * drop_ld + k: the user encoder's input
//      dropout fused into the QKV projection, K09), a_mode 1 = stored transposed [K, M]
//      (weight gradients dW = dY^T X);
//   B: b_mode 0 = [N, K] (nn.Linear weight: y = x W^T), b_mode 1 = [K, N] (dgrad dx = dy W;
//      or, with gidx / dropout, the forward's gathered dropped-out input X' for dW = dY^T X').
//   act: 0 none, 1 tanh.  drop_on: 0 none, 1 A elements (m, k), 2 B elements (k, n) of a K-major
//      B, 3 output elements (m, n) -- the input dropout's backward fused into the dgrad
//      epilogue.  gather_on: 0 none, 1 A rows (a_mode 0), 2 B rows (b_mode 1).
// Tile 64 x 64 x 32, 256 threads = 4 waves in 2 x 2, each wave 32 x 32 = 2 x 2 MFMA tiles.
// Several independent GEMMs run in ONE launch (GemmBatch: the Q/K/V projections, the three
// weight gradients of one backward, ...): blockIdx.x walks the concatenated tile lists.
// Deterministic: no split-K, no atomics.
#include "common.h"

namespace {

constexpr int TM = 64, TN = 64, TK = 32, LDT = TK + 8;  // LDS row stride 40 bf16 = 80 B
constexpr int MAXG = 6;

struct GemmDesc {
  const float* A;
  const int* gidx;  // row gather of A (gather_on 1, a_mode 0) or of B (gather_on 2, b_mode 1)
  const float* B;
  const float* bias;
  float* C;
  int M, N, K, lda, ldb, ldc;
  int a_mode, b_mode, act, accumulate;
  float alpha, pdrop;
  int drop_ld, drop_on, gather_on, tiles_n, tile_base;
  unsigned long long seed, offset;
};

struct GemmBatch {
  GemmDesc d[MAXG];
  int n;
};

__device__ __forceinline__ void load_tile(const GemmDesc& g, bool isA, int r0, int k0, bf16 (*S)[LDT], int tid) {
  const int mode = isA ? g.a_mode : g.b_mode;
  const float* P = isA ? g.A : g.B;
  const int ld = isA ? g.lda : g.ldb;
  const int R = isA ? g.M : g.N;
  if (mode == 0) {  // [R, K] row-major: thread -> (row, 8 consecutive k)
    const int r = tid >> 2, kk = (tid & 3) * 8;
    const int rr = r0 + r;
    float v[8];
    const bool rok = rr < R;
    const int src = rok ? ((isA && g.gather_on == 1) ? g.gidx[rr] : rr) : 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + kk + j;
      v[j] = (rok && k < g.K) ? P[(size_t)src * ld + k] : 0.f;
    }
    if (isA && g.drop_on == 1 && rok) {
      const unsigned long long e = (unsigned long long)rr * g.drop_ld + (k0 + kk);  // multiple of 4
      const float inv_keep = 1.0f / (1.0f - g.pdrop);
      const uint4 x0 = Philox::gen(g.seed, g.offset, e >> 2);
      const uint4 x1 = Philox::gen(g.seed, g.offset, (e >> 2) + 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= drop_scale(u4_get(j < 4 ? x0 : x1, j & 3), g.pdrop, inv_keep);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
    *(bf16x8*)&S[r][kk] = o;
  } else {  // stored [K, R]: thread -> (k, 8 consecutive rows), coalesced along the rows
    const int k = tid >> 3, rr8 = (tid & 7) * 8;
    const int kg = k0 + k;
    // B in mode 1 may be the gathered + dropped-out input of the forward (the weight
    // gradient dW = dY^T X' regenerates X' = drop(X[gidx]) instead of storing it)
    const bool gat = !isA && g.gather_on == 2;
    const bool drop = !isA && g.drop_on == 2;
    const size_t src = (kg < g.K) ? (size_t)(gat ? g.gidx[kg] : kg) : 0;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int rr = r0 + rr8 + j;
      v[j] = (kg < g.K && rr < R) ? P[src * ld + rr] : 0.f;
    }
    if (drop && kg < g.K) {
      const unsigned long long e = (unsigned long long)kg * g.drop_ld + (r0 + rr8);  // multiple of 8
      const float inv_keep = 1.0f / (1.0f - g.pdrop);
      const uint4 x0 = Philox::gen(g.seed, g.offset, e >> 2);
      const uint4 x1 = Philox::gen(g.seed, g.offset, (e >> 2) + 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= drop_scale(u4_get(j < 4 ? x0 : x1, j & 3), g.pdrop, inv_keep);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) S[rr8 + j][k] = f2bf(v[j]);
  }
}

__global__ __launch_bounds__(256) void small_gemm_kernel(const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) bf16 As[TM][LDT];
  __shared__ __attribute__((aligned(16))) bf16 Bs[TN][LDT];
  int gi = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < batch.n && (int)blockIdx.x >= batch.d[i].tile_base) gi = i;
  const GemmDesc& g = batch.d[gi];
  const int t = blockIdx.x - g.tile_base;
  const int m0 = (t / g.tiles_n) * TM, n0 = (t % g.tiles_n) * TN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < g.K; k0 += TK) {
    __syncthreads();
    load_tile(g, true, m0, k0, As, tid);
    load_tile(g, false, n0, k0, Bs, tid);
    __syncthreads();
    bf16x8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i] = *(const bf16x8*)&As[wm + i * 16 + fr][fq * 8];
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = *(const bf16x8*)&Bs[wn + j * 16 + fr][fq * 8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  // lane holds C[m = wm + 16 i + 4 fq + r][n = wn + 16 j + fr]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn + j * 16 + fr;
    if (n >= g.N) continue;
    const float bn = g.bias ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + fq * 4 + r;
        if (m >= g.M) continue;
        float v = g.alpha * acc[i][j][r] + bn;
        if (g.act == 1) v = tanhf(v);
        if (g.drop_on == 3) {  // dropout backward in the epilogue: element (m, n) of the dropped input
          const unsigned long long e = (unsigned long long)m * g.drop_ld + n;
          const uint4 x = Philox::gen(g.seed, g.offset, e >> 2);
          v *= drop_scale(u4_get(x, (int)(e & 3)), g.pdrop, 1.0f / (1.0f - g.pdrop));
        }
        float* c = g.C + (size_t)m * g.ldc + n;
        if (g.accumulate) v += *c;
        *c = v;
      }
  }
}

// Deterministic fp32 column sums (bias gradients): block = 64 columns, 4 waves take rows
// w, w + 4, ... and combine in a fixed order.  Several matrices per launch (ColsumBatch).
struct ColsumDesc {
  const float* X;
  float* out;
  int M, N, ld, col_blocks, block_base, accumulate;
};
struct ColsumBatch {
  ColsumDesc d[MAXG];
  int n;
};

__global__ __launch_bounds__(256) void colsum_f32_kernel(const ColsumBatch batch) {
  __shared__ float part[4][64];
  int gi = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < batch.n && (int)blockIdx.x >= batch.d[i].block_base) gi = i;
  const ColsumDesc& g = batch.d[gi];
  const int c = (blockIdx.x - g.block_base) * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  float s = 0.f;
  if (c < g.N)
    for (int m = w; m < g.M; m += 4) s += g.X[(size_t)m * g.ld + c];
  part[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && c < g.N) {
    const float v = (part[0][threadIdx.x] + part[1][threadIdx.x]) + (part[2][threadIdx.x] + part[3][threadIdx.x]);
    g.out[c] = g.accumulate ? g.out[c] + v : v;
  }
}

}  // namespace

// descs: 5 pointers + 13 ints + 2 floats + 2 u64 per GEMM, packed by binding.cpp small_gemm
extern "C" int fr_small_gemm(const void* const* ptrs, const int* ints, const float* floats,
                             const unsigned long long* seeds, int n, hipStream_t s) {
  if (n < 1 || n > MAXG) return 1;
  GemmBatch b{};
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    GemmDesc& d = b.d[i];
    d.A = (const float*)ptrs[5 * i + 0];
    d.gidx = (const int*)ptrs[5 * i + 1];
    d.B = (const float*)ptrs[5 * i + 2];
    d.bias = (const float*)ptrs[5 * i + 3];
    d.C = (float*)ptrs[5 * i + 4];
    const int* q = ints + 13 * i;
    d.M = q[0]; d.N = q[1]; d.K = q[2]; d.lda = q[3]; d.ldb = q[4]; d.ldc = q[5];
    d.a_mode = q[6]; d.b_mode = q[7]; d.act = q[8]; d.accumulate = q[9]; d.drop_ld = q[10];
    d.drop_on = q[11]; d.gather_on = q[12];
    d.alpha = floats[2 * i];
    d.pdrop = floats[2 * i + 1];
    d.seed = seeds[2 * i];
    d.offset = seeds[2 * i + 1];
    if (d.M < 0 || d.N < 0 || d.K < 0) return 2;
    if (d.drop_on < 0 || d.drop_on > 3 || d.gather_on < 0 || d.gather_on > 2 || d.act < 0 || d.act > 1) return 3;
    if (d.drop_on && (!(d.pdrop > 0.f && d.pdrop < 1.f) || d.drop_ld % 8 != 0 || (d.drop_on == 1 && d.a_mode != 0) ||
                      (d.drop_on == 2 && d.b_mode != 1)))
      return 3;
    if (d.gather_on && (!d.gidx || (d.gather_on == 1 && d.a_mode != 0) || (d.gather_on == 2 && d.b_mode != 1))) return 4;
    d.tiles_n = (d.N + TN - 1) / TN;
    d.tile_base = tiles;
    tiles += ((d.M + TM - 1) / TM) * d.tiles_n;
  }
  b.n = n;
  if (tiles == 0) return 0;
  hipLaunchKernelGGL(small_gemm_kernel, dim3(tiles), dim3(256), 0, s, b);
  return 0;
}

extern "C" int fr_colsum_f32(const float* const* xs, float* const* outs, const int* ints, int n, hipStream_t s) {
  if (n < 1 || n > MAXG) return 1;
  ColsumBatch b{};
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    ColsumDesc& d = b.d[i];
    d.X = xs[i];
    d.out = outs[i];
    d.M = ints[4 * i];
    d.N = ints[4 * i + 1];
    d.ld = ints[4 * i + 2];
    d.accumulate = ints[4 * i + 3];
    d.col_blocks = (d.N + 63) / 64;
    d.block_base = blocks;
    blocks += d.col_blocks;
  }
  b.n = n;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(colsum_f32_kernel, dim3(blocks), dim3(256), 0, s, b);
  return 0;
}
