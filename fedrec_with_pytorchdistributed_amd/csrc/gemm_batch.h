// Small-GEMM launch descriptors and the split-K reduction body, shared by small_gemm.hip (its own
// reduce launch) and text_head.hip (whose tail reduce launch can run a deferred split-K
// reduction of the text FC's backward GEMM batch in extra blocks: one launch less per step).
#pragma once
#include "common.h"

namespace fr_sg {

constexpr int MAXG = 6;

struct GemmDesc {
  const void* A;
  const int* gidx;  // row gather of A (gather_on 1, a_mode 0) or of B (gather_on 2, b_mode 1)
  const void* B;
  const void* B2;  // K-segmented B (b_mode 1): rows [kseg, 2 kseg) from B2, [2 kseg, 3 kseg) from B3
  const void* B3;
  const float* bias;
  float* C;
  float* P;  // split-K partials [splits, M, N] (splits > 1: the reduce kernel does the epilogue)
  float* asum;  // optional (a_mode 1): asum[m] = sum_k A(m, k) in fp32 -- a weight gradient's bias
  float* AP;    // gradient dY^T 1 from the dY tiles the GEMM streams; partials [splits, M] if split
  int M, N, K, lda, ldb, ldc;
  int a_mode, b_mode, act, accumulate;
  float alpha, pdrop;
  int drop_ld, drop_on, gather_on, tiles_n, tile_base, splits, kchunk, kseg;
  int a_bf16, b_bf16;
  int red_base;   // first block of this desc's split-K reduction
  int ared_base;  // first block of its asum partial reduction (split asum descs)
  unsigned long long seed, offset;  // offset += *dev_off when dev_off is set (graph replays)
};

struct GemmBatch {
  GemmDesc d[MAXG];
  const unsigned long long* dev_off;  // per-launch device counter added to the dropout offsets
  int n;
};

// split-K epilogue of block bx: C = act(alpha * sum_s P[s] + bias) (x the output dropout scale,
// drop_on 3) (+ C), partials summed in split order (deterministic); blocks >= c_blocks sum the
// asum partials of split descs.  A lane takes 4 consecutive columns of one row.
__device__ __forceinline__ void splitk_reduce_block(const GemmBatch& batch, int c_blocks, int bx) {
  if (bx >= c_blocks) {  // the asum partials of split descs: asum[m] = sum_s AP[s][m]
    int ai = -1;
#pragma unroll
    for (int i = 0; i < MAXG; ++i)
      if (i < batch.n && batch.d[i].AP != nullptr && bx >= batch.d[i].ared_base) ai = i;
    if (ai < 0) return;
    const GemmDesc& a = batch.d[ai];
    const int m = (bx - a.ared_base) * 256 + threadIdx.x;
    if (m >= a.M) return;
    float v = a.AP[m];
    for (int sp = 1; sp < a.splits; ++sp) v += a.AP[(size_t)sp * a.M + m];
    a.asum[m] = v;
    return;
  }
  int gi = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < batch.n && batch.d[i].splits > 1 && bx >= batch.d[i].red_base) gi = i;
  const GemmDesc& g = batch.d[gi];
  if (g.splits <= 1) return;
  const long q = (long)(bx - g.red_base) * 256 + threadIdx.x;
  const long MN = (long)g.M * g.N;
  const long e = 4 * q;
  if (e >= MN) return;
  const int m = (int)(e / g.N), n = (int)(e - (long)m * g.N);
  float4 sum = *(const float4*)(g.P + e);
  for (int sp = 1; sp < g.splits; ++sp) {
    const float4 t = *(const float4*)(g.P + (size_t)sp * MN + e);
    sum.x += t.x; sum.y += t.y; sum.z += t.z; sum.w += t.w;
  }
  float v[4] = {sum.x, sum.y, sum.z, sum.w};
  float sc[4] = {1.f, 1.f, 1.f, 1.f};
  if (g.drop_on == 3) {  // as the single-pass epilogue: elements (m, n..n+3) of the dropped input
    const unsigned long long off = g.offset + (batch.dev_off ? *batch.dev_off : 0ull);
    const uint4 x = Philox::gen(g.seed, off, ((unsigned long long)m * g.drop_ld + n) >> 2);
    const float inv_keep = 1.0f / (1.0f - g.pdrop);
#pragma unroll
    for (int r = 0; r < 4; ++r) sc[r] = drop_scale(u4_get(x, r), g.pdrop, inv_keep);
  }
  float* c = g.C + (size_t)m * g.ldc + n;
  const bool vec = ((uintptr_t)c & 15) == 0;
  float cv[4] = {0.f, 0.f, 0.f, 0.f};
  if (g.accumulate) {
    if (vec) {
      const float4 t = *(const float4*)c;
      cv[0] = t.x; cv[1] = t.y; cv[2] = t.z; cv[3] = t.w;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) cv[r] = c[r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float x = g.alpha * v[r] + (g.bias ? g.bias[n + r] : 0.f);
    if (g.act == 1) x = tanhf(x);
    x *= sc[r];
    v[r] = g.accumulate ? cv[r] + x : x;
  }
  if (vec)
    *(float4*)c = make_float4(v[0], v[1], v[2], v[3]);
  else
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = v[r];
}

}  // namespace fr_sg
