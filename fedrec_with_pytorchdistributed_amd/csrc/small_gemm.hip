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
// Tile 64 x 64 x 64, 256 threads = 4 waves in 2 x 2, each wave 32 x 32 = 2 x 2 MFMA tiles;
// 16-byte global loads where aligned.  Several independent GEMMs run in ONE launch (GemmBatch:
// the Q/K/V projections, the weight gradients of one backward, ...): blockIdx.x walks the
// concatenated tile lists.  Long reductions with few output tiles (weight gradients over
// K = B*H = 3200 rows) split K over workgroups into fp32 partials that a second kernel sums in
// split order -- deterministic, no atomics.
#include "common.h"

namespace {

constexpr int TM = 64, TN = 64, TK = 64, LDT = TK + 8;  // LDS row stride 72 bf16 = 144 B
constexpr int MAXG = 6;

struct GemmDesc {
  const float* A;
  const int* gidx;  // row gather of A (gather_on 1, a_mode 0) or of B (gather_on 2, b_mode 1)
  const float* B;
  const float* B2;  // K-segmented B (b_mode 1): rows [kseg, 2 kseg) from B2, [2 kseg, 3 kseg) from B3
  const float* B3;
  const float* bias;
  float* C;
  float* P;  // split-K partials [splits, M, N] (splits > 1: the reduce kernel does the epilogue)
  int M, N, K, lda, ldb, ldc;
  int a_mode, b_mode, act, accumulate;
  float alpha, pdrop;
  int drop_ld, drop_on, gather_on, tiles_n, tile_base, splits, kchunk, kseg;
  unsigned long long seed, offset;  // offset += *dev_off when dev_off is set (graph replays)
};

struct GemmBatch {
  GemmDesc d[MAXG];
  const unsigned long long* dev_off;  // per-launch device counter added to the dropout offsets
  int n;
};

__device__ __forceinline__ void load16(const float* __restrict__ p, bool full, bool vec, int valid, float (&v)[16]) {
  if (full && vec) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 f = *(const float4*)(p + 4 * j);
      v[4 * j] = f.x; v[4 * j + 1] = f.y; v[4 * j + 2] = f.z; v[4 * j + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = j < valid ? p[j] : 0.f;
  }
}

__device__ __forceinline__ void apply_drop16(float (&v)[16], unsigned long long e, const GemmDesc& g,
                                             unsigned long long off) {  // e: element index of v[0], % 16 == 0
  const float inv_keep = 1.0f / (1.0f - g.pdrop);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 x = Philox::gen(g.seed, off, (e >> 2) + q);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * q + j] *= drop_scale(u4_get(x, j), g.pdrop, inv_keep);
  }
}

// one 64 x 64 operand tile (rows r0.., k0..): global -> 16 registers per thread (converted
// and dropout-scaled), then registers -> bf16 LDS [row][k] in a separate step, so the next
// tile's loads are in flight while the MFMAs consume the current one
__device__ __forceinline__ void load_regs(const GemmDesc& g, unsigned long long off, bool isA, int r0, int k0,
                                          int kend, int tid, float (&v)[16]) {
  const int mode = isA ? g.a_mode : g.b_mode;
  const float* P = isA ? g.A : g.B;
  const int ld = isA ? g.lda : g.ldb;
  const int R = isA ? g.M : g.N;
  if (mode == 0) {  // [R, K] row-major: thread -> (row, 16 consecutive k)
    const int r = tid >> 2, kk = (tid & 3) * 16;
    const int rr = r0 + r, k = k0 + kk;
    const bool rok = rr < R;
    const int src = rok ? ((isA && g.gather_on == 1) ? g.gidx[rr] : rr) : 0;
    const float* p = P + (size_t)src * ld + k;
    const int valid = rok ? min(16, kend - k) : 0;
    load16(p, valid == 16, ((uintptr_t)p & 15) == 0, valid, v);
    if (isA && g.drop_on == 1 && rok) apply_drop16(v, (unsigned long long)rr * g.drop_ld + k, g, off);
  } else {  // stored [K, R]: thread -> (k, 16 consecutive rows), coalesced along the rows
    const int k = tid >> 2, rr16 = (tid & 3) * 16;
    const int kg = k0 + k;
    const bool kok = kg < kend;
    // B in mode 1 may be the gathered + dropped-out input of the forward (the weight
    // gradient dW = dY^T X' regenerates X' = drop(X[gidx]) instead of storing it)
    size_t src = kok ? (size_t)((!isA && g.gather_on == 2) ? g.gidx[kg] : kg) : 0;
    if (!isA && g.kseg > 0 && kok) {  // one [K, N] operand stored as up to three row blocks
      const int seg = kg / g.kseg;
      P = seg == 0 ? g.B : (seg == 1 ? g.B2 : g.B3);
      src = kg - seg * g.kseg;
    }
    const float* p = P + src * ld + r0 + rr16;
    const int valid = kok ? min(16, R - (r0 + rr16)) : 0;
    load16(p, valid == 16, ((uintptr_t)p & 15) == 0, valid, v);
    if (!isA && g.drop_on == 2 && kok) apply_drop16(v, (unsigned long long)kg * g.drop_ld + r0 + rr16, g, off);
  }
}

__device__ __forceinline__ void store_regs(const GemmDesc& g, bool isA, int tid, const float (&v)[16],
                                           bf16 (*S)[LDT]) {
  if ((isA ? g.a_mode : g.b_mode) == 0) {
    const int r = tid >> 2, kk = (tid & 3) * 16;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[8 * h + j]);
      *(bf16x8*)&S[r][kk + 8 * h] = o;
    }
  } else {
    const int k = tid >> 2, rr16 = (tid & 3) * 16;
#pragma unroll
    for (int j = 0; j < 16; ++j) S[rr16 + j][k] = f2bf(v[j]);
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
  const unsigned long long off = g.offset + (batch.dev_off ? *batch.dev_off : 0ull);
  int t = blockIdx.x - g.tile_base;
  const int split = t % g.splits;
  t /= g.splits;
  const int m0 = (t / g.tiles_n) * TM, n0 = (t % g.tiles_n) * TN;
  const int kbeg = split * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // one K-tile in flight in registers (two in flight measured slower: 132 VGPRs cost the
  // bigger grids an occupancy step -- QKV 33 -> 38 us, weight gradients 33 -> 39 us)
  float va[16], vb[16];
  if (kbeg < kend) {
    load_regs(g, off, true, m0, kbeg, kend, tid, va);
    load_regs(g, off, false, n0, kbeg, kend, tid, vb);
  }
  for (int k0 = kbeg; k0 < kend; k0 += TK) {
    __syncthreads();  // the previous tile's fragments are consumed
    store_regs(g, true, tid, va, As);
    store_regs(g, false, tid, vb, Bs);
    __syncthreads();
    if (k0 + TK < kend) {  // next tile's global loads overlap this tile's MFMAs
      load_regs(g, off, true, m0, k0 + TK, kend, tid, va);
      load_regs(g, off, false, n0, k0 + TK, kend, tid, vb);
    }
#pragma unroll
    for (int ks = 0; ks < TK; ks += 32) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *(const bf16x8*)&As[wm + i * 16 + fr][ks + fq * 8];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *(const bf16x8*)&Bs[wn + j * 16 + fr][ks + fq * 8];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // lane holds C[m = wm + 16 i + 4 fq + r][n = wn + 16 j + fr]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn + j * 16 + fr;
    if (n >= g.N) continue;
    if (g.splits > 1) {  // raw partial; alpha / accumulate in splitk_reduce_kernel
      float* pp = g.P + (size_t)split * g.M * g.N;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm + i * 16 + fq * 4 + r;
          if (m < g.M) pp[(size_t)m * g.N + n] = acc[i][j][r];
        }
      continue;
    }
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
          const uint4 x = Philox::gen(g.seed, off, e >> 2);
          v *= drop_scale(u4_get(x, (int)(e & 3)), g.pdrop, 1.0f / (1.0f - g.pdrop));
        }
        float* c = g.C + (size_t)m * g.ldc + n;
        if (g.accumulate) v += *c;
        *c = v;
      }
  }
}

// split-K epilogue: C = act(alpha * sum_s P[s] + bias) (x the output dropout scale, drop_on 3)
// (+ C), partials summed in split order (deterministic) -- the single-pass epilogue's order
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmBatch batch, int total) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    int gi = 0, base = 0;
    for (int i = 0; i < batch.n; ++i) {
      const GemmDesc& d = batch.d[i];
      const int sz = d.splits > 1 ? d.M * d.N : 0;
      if (e < base + sz) { gi = i; break; }
      base += sz;
    }
    const GemmDesc& g = batch.d[gi];
    const int idx = e - base, m = idx / g.N, n = idx - m * g.N;
    float s = 0.f;
    for (int sp = 0; sp < g.splits; ++sp) s += g.P[(size_t)sp * g.M * g.N + idx];
    float* c = g.C + (size_t)m * g.ldc + n;
    float v = g.alpha * s + (g.bias ? g.bias[n] : 0.f);
    if (g.act == 1) v = tanhf(v);
    if (g.drop_on == 3) {  // as the single-pass epilogue: element (m, n) of the dropped input
      const unsigned long long off = g.offset + (batch.dev_off ? *batch.dev_off : 0ull);
      const unsigned long long el = (unsigned long long)m * g.drop_ld + n;
      const uint4 x = Philox::gen(g.seed, off, el >> 2);
      v *= drop_scale(u4_get(x, (int)(el & 3)), g.pdrop, 1.0f / (1.0f - g.pdrop));
    }
    *c = g.accumulate ? *c + v : v;
  }
}

// Deterministic fp32 column sums (bias gradients), two passes: (1) blocks of 64 columns x 128
// rows (4 waves x 32 rows) write per-chunk partials; (2) the partials are summed in chunk order.
// A desc of one row chunk (M <= 128: the loss sum, the pooled-user partial rows) is final after
// pass 1, and a launch of only such descs skips pass 2.  (A single-pass "last block sums"
// form with agent-scope fences measured 131 us/step vs 69: each release fence writes back L2.)
constexpr int CS_ROWS = 128;
struct ColsumDesc {
  const float* X;
  float* out;
  float* part;  // [chunks, N]
  int M, N, ld, col_blocks, chunks, block_base, block2_base, accumulate;
};
struct ColsumBatch {
  ColsumDesc d[MAXG];
  int n;
};

__global__ __launch_bounds__(256) void colsum_part_kernel(const ColsumBatch batch) {
  __shared__ float part[4][64];
  int gi = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < batch.n && (int)blockIdx.x >= batch.d[i].block_base) gi = i;
  const ColsumDesc& g = batch.d[gi];
  const int b = blockIdx.x - g.block_base;
  const int cb = b % g.col_blocks, ch = b / g.col_blocks;
  const int c = cb * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
  const int r0 = ch * CS_ROWS, r1 = min(g.M, r0 + CS_ROWS);
  float s = 0.f;
  if (c < g.N)
    for (int m = r0 + w; m < r1; m += 4) s += g.X[(size_t)m * g.ld + c];
  part[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && c < g.N) {
    const float tot = (part[0][threadIdx.x] + part[1][threadIdx.x]) + (part[2][threadIdx.x] + part[3][threadIdx.x]);
    if (g.chunks == 1)  // one row chunk: the final value (no second pass for this desc)
      g.out[c] = g.accumulate ? g.out[c] + tot : tot;
    else
      g.part[(size_t)ch * g.N + c] = tot;
  }
}

__global__ __launch_bounds__(64) void colsum_final_kernel(const ColsumBatch batch) {
  int gi = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < batch.n && (int)blockIdx.x >= batch.d[i].block2_base) gi = i;
  const ColsumDesc& g = batch.d[gi];
  const int c = (blockIdx.x - g.block2_base) * 64 + threadIdx.x;
  if (c >= g.N || g.chunks == 1) return;
  float s = 0.f;
  for (int ch = 0; ch < g.chunks; ++ch) s += g.part[(size_t)ch * g.N + c];
  g.out[c] = g.accumulate ? g.out[c] + s : s;
}

}  // namespace

// descs: 7 pointers + 14 ints + 2 floats + 2 u64 per GEMM, packed by binding.cpp small_gemm.
// scratch: split-K partial space (floats) the caller allocated; returns the floats it needs
// when scratch is null (query mode).
static int choose_splits(int M, int N, int K) {
  const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  if (K < 512) return 1;
  if (tiles >= 192) {
    // more than ~3/4 of a wave of tiles: split only when it fixes the wave quantisation by a
    // margin that pays for the reduce pass (the user dgrad: 350 tiles x K = 1200 = 1.37 waves
    // of 19-step tiles -> 2 splits = 700 half-length tiles, 3 rounds of 1/2 instead of 2 of 1)
    const int rounds1 = (tiles + 255) / 256;
    int best = 1;
    float bestc = (float)rounds1;
    for (int sp = 2; sp <= 4 && sp <= K / 256; ++sp) {
      const float c = (float)((tiles * sp + 255) / 256) / sp;
      if (c * 1.15f < bestc) {
        best = sp;
        bestc = c * 1.15f;
      }
    }
    return best;
  }
  int s = (256 + tiles - 1) / tiles;  // about one wave of workgroups over the 256 CUs
  s = min(s, K / 256);
  return max(1, min(s, 16));
}

extern "C" long fr_small_gemm(const void* const* ptrs, const int* ints, const float* floats,
                              const unsigned long long* seeds, const unsigned long long* dev_off, int n, float* scratch,
                              hipStream_t s) {
  if (n < 1 || n > MAXG) return -1;
  GemmBatch b{};
  b.dev_off = dev_off;
  int tiles = 0;
  long need = 0;
  int red_total = 0;
  for (int i = 0; i < n; ++i) {
    GemmDesc& d = b.d[i];
    d.A = (const float*)ptrs[7 * i + 0];
    d.gidx = (const int*)ptrs[7 * i + 1];
    d.B = (const float*)ptrs[7 * i + 2];
    d.bias = (const float*)ptrs[7 * i + 3];
    d.C = (float*)ptrs[7 * i + 4];
    d.B2 = (const float*)ptrs[7 * i + 5];
    d.B3 = (const float*)ptrs[7 * i + 6];
    const int* q = ints + 14 * i;
    d.M = q[0]; d.N = q[1]; d.K = q[2]; d.lda = q[3]; d.ldb = q[4]; d.ldc = q[5];
    d.a_mode = q[6]; d.b_mode = q[7]; d.act = q[8]; d.accumulate = q[9]; d.drop_ld = q[10];
    d.drop_on = q[11]; d.gather_on = q[12]; d.kseg = q[13];
    if (d.kseg > 0 && (d.b_mode != 1 || d.gather_on == 2 || !d.B2 || (d.K > 2 * d.kseg && !d.B3) || d.K > 3 * d.kseg))
      return -5;
    d.alpha = floats[2 * i];
    d.pdrop = floats[2 * i + 1];
    d.seed = seeds[2 * i];
    d.offset = seeds[2 * i + 1];
    if (d.M < 0 || d.N < 0 || d.K < 0) return -2;
    if (d.drop_on < 0 || d.drop_on > 3 || d.gather_on < 0 || d.gather_on > 2 || d.act < 0 || d.act > 1) return -3;
    if (d.drop_on && (!(d.pdrop > 0.f && d.pdrop < 1.f) || d.drop_ld % 16 != 0 || (d.drop_on == 1 && d.a_mode != 0) ||
                      (d.drop_on == 2 && d.b_mode != 1)))
      return -3;
    if (d.gather_on && (!d.gidx || (d.gather_on == 1 && d.a_mode != 0) || (d.gather_on == 2 && d.b_mode != 1))) return -4;
    // split-K: the reduce applies the whole epilogue (alpha, bias, tanh, output dropout, accumulate)
    d.splits = choose_splits(d.M, d.N, d.K);
    d.kchunk = d.splits > 1 ? ((d.K + d.splits - 1) / d.splits + TK - 1) / TK * TK : d.K;
    if (d.splits > 1) d.splits = (d.K + d.kchunk - 1) / d.kchunk;
    d.P = nullptr;
    if (d.splits > 1) {
      d.P = scratch ? scratch + need : nullptr;
      need += (long)d.splits * d.M * d.N;
      red_total += d.M * d.N;
    }
    d.tiles_n = (d.N + TN - 1) / TN;
    d.tile_base = tiles;
    tiles += ((d.M + TM - 1) / TM) * d.tiles_n * d.splits;
  }
  b.n = n;
  if (scratch == nullptr && need > 0) return need;  // query: the caller allocates and calls again
  if (tiles == 0) return 0;
  hipLaunchKernelGGL(small_gemm_kernel, dim3(tiles), dim3(256), 0, s, b);
  if (red_total > 0) {
    const int blocks = min(2048, (red_total + 255) / 256);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, b, red_total);
  }
  return 0;
}

// returns the scratch floats needed when part == nullptr (query mode), else launches
extern "C" long fr_colsum_f32(const float* const* xs, float* const* outs, const int* ints, int n, float* part,
                              hipStream_t s) {
  if (n < 1 || n > MAXG) return -1;
  ColsumBatch b{};
  int blocks = 0, blocks2 = 0;
  long need = 0;
  for (int i = 0; i < n; ++i) {
    ColsumDesc& d = b.d[i];
    d.X = xs[i];
    d.out = outs[i];
    d.M = ints[4 * i];
    d.N = ints[4 * i + 1];
    d.ld = ints[4 * i + 2];
    d.accumulate = ints[4 * i + 3];
    d.col_blocks = (d.N + 63) / 64;
    d.chunks = max(1, (d.M + CS_ROWS - 1) / CS_ROWS);
    d.part = part ? part + need : nullptr;
    need += (long)d.chunks * d.N;
    d.block_base = blocks;
    blocks += d.col_blocks * d.chunks;
    d.block2_base = blocks2;
    blocks2 += d.col_blocks;
  }
  b.n = n;
  if (part == nullptr) return need;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(colsum_part_kernel, dim3(blocks), dim3(256), 0, s, b);
  bool second = false;  // descs of one row chunk are final after the first pass
  for (int i = 0; i < n; ++i) second |= b.d[i].chunks > 1;
  if (second) hipLaunchKernelGGL(colsum_final_kernel, dim3(blocks2), dim3(64), 0, s, b);
  return 0;
}

// ---------------------------------------------------------------------------------------
// X'[m, k] = v[idx[m], k] * Z(m * K + k): the user encoder's gathered, dropped-out input
// (encoder.py:50), materialised once per step (fp32 [B*H, D], 5 MB) instead of regenerated in
// every GEMM tile that reads it -- the Q/K/V projection's A loads (21 column tiles each redid
// the Philox draws of their rows) and the weight-gradient GEMMs' B loads (one redo per output
// row tile).  Same mask, same fp32 product: bitwise the values those loads computed.
// One thread per 4 consecutive elements = one Philox draw (K % 4 == 0, host-checked).
namespace {
__global__ __launch_bounds__(256) void gather_dropout_kernel(const float* __restrict__ v, const int* __restrict__ idx,
                                                             float* __restrict__ out, int M, int K, float p,
                                                             unsigned long long seed, unsigned long long offset,
                                                             const unsigned long long* __restrict__ dev_off) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;  // float4 index
  const long n4 = (long)M * K / 4;
  if (q >= n4) return;
  const long e = q * 4;
  const int m = (int)(e / K), k = (int)(e - (long)m * K);
  float4 x = *(const float4*)(v + (size_t)idx[m] * K + k);
  if (p > 0.f) {
    const unsigned long long off = offset + (dev_off ? *dev_off : 0ull);
    const float inv_keep = 1.0f / (1.0f - p);
    const uint4 r = Philox::gen(seed, off, (unsigned long long)e >> 2);
    x.x *= drop_scale(r.x, p, inv_keep);
    x.y *= drop_scale(r.y, p, inv_keep);
    x.z *= drop_scale(r.z, p, inv_keep);
    x.w *= drop_scale(r.w, p, inv_keep);
  }
  *(float4*)(out + e) = x;
}
}  // namespace

extern "C" int fr_gather_dropout_f32(const float* v, const int* idx, float* out, int M, int K, float p,
                                     unsigned long long seed, unsigned long long offset,
                                     const unsigned long long* dev_off, hipStream_t s) {
  if (K % 4 != 0 || M < 0) return 1;
  const long n4 = (long)M * K / 4;
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(gather_dropout_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, v, idx, out, M, K, p,
                     seed, offset, dev_off);
  return 0;
}
