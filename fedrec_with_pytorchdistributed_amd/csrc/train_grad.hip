// Gradient reductions of the unfrozen-backbone training path (BASELINE config 5):
//
//   colsum:     db[n] = sum_m dy[m, n]              bias gradient of every linear layer
//               (bf16 dy, fp32 out; two deterministic passes: per row-chunk partials, then
//               a fixed-order sum -- torch's generic reduction ran at ~3.4 TB/s here)
//   embed_grad: dword[tok] = sum over occurrences   word-embedding gradient from the
//               sorted token ids (one wave per distinct token, fixed order, no float
//               atomics; the pad token 0 -- most of the rows -- is skipped: nn.Embedding
//               padding_idx keeps its gradient zero, so the index_add hot spot disappears)
#include "common.h"

namespace {

constexpr int CS_CHUNKS = 128;

// grid (ceil(N / 512), CS_CHUNKS); lane owns 8 consecutive columns, the 4 waves of a block
// stride over the chunk's rows; partial[chunk][n]
__global__ __launch_bounds__(256) void colsum_partial_kernel(const bf16* __restrict__ x, int M, int N,
                                                             float* __restrict__ partial) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int rows_per = (M + CS_CHUNKS - 1) / CS_CHUNKS;
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < N) {
    int r = r0 + wave;
    for (; r + 4 < r1; r += 8) {  // two rows in flight per wave
      const bf16x8 a = *(const bf16x8*)(x + (size_t)r * N + c0);
      const bf16x8 b = *(const bf16x8*)(x + (size_t)(r + 4) * N + c0);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += (float)a[k] + (float)b[k];
    }
    for (; r < r1; r += 4) {
      const bf16x8 a = *(const bf16x8*)(x + (size_t)r * N + c0);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += (float)a[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[wave][lane * 8 + k] = acc[k];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int c = blockIdx.x * 512 + i;
    if (c < N) partial[(size_t)blockIdx.y * N + c] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ partial, int N,
                                                           float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= N) return;
  float s = 0.f;
  for (int k = 0; k < CS_CHUNKS; ++k) s += partial[(size_t)k * N + c];
  out[c] = s;
}

// one wave per sorted position b; only the first occurrence of each token (b == 0 or a new
// id) works: it sums rows perm[b .. end) of dx in sorted (= occurrence) order.  D % 256 == 0.
__global__ __launch_bounds__(256) void embed_grad_kernel(const bf16* __restrict__ dx, const int* __restrict__ sorted,
                                                         const int* __restrict__ perm, int R, int D,
                                                         float* __restrict__ dword) {
  const int b = blockIdx.x * 4 + (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= R) return;
  const int tok = sorted[b];
  if (tok == 0 || (b > 0 && sorted[b - 1] == tok)) return;
  int e = b + 1;
  while (e < R && sorted[e] == tok) ++e;
  for (int c0 = lane * 4; c0 < D; c0 += 256) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int r = b; r < e; ++r) {
      const bf16x4 v = *(const bf16x4*)(dx + (size_t)perm[r] * D + c0);
      a0 += (float)v[0];
      a1 += (float)v[1];
      a2 += (float)v[2];
      a3 += (float)v[3];
    }
    *(float4*)(dword + (size_t)tok * D + c0) = make_float4(a0, a1, a2, a3);
  }
}

}  // namespace

// partial: CS_CHUNKS * N floats of scratch
extern "C" int fr_colsum_bf16(const void* x, int M, int N, float* partial, float* out, hipStream_t s) {
  if (N % 8 != 0 || M <= 0) return 1;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((N + 511) / 512, CS_CHUNKS), dim3(256), 0, s, (const bf16*)x, M, N,
                     partial);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + 255) / 256), dim3(256), 0, s, partial, N, out);
  return 0;
}

extern "C" int fr_colsum_chunks() { return CS_CHUNKS; }

// dword must be zeroed by the caller (rows of tokens absent from the batch stay zero)
extern "C" int fr_embed_grad_bf16(const void* dx, const int* sorted, const int* perm, int R, int D, float* dword,
                                  hipStream_t s) {
  if (D % 256 != 0 || R <= 0) return R < 0 ? 1 : 0;
  hipLaunchKernelGGL(embed_grad_kernel, dim3((R + 3) / 4), dim3(256), 0, s, (const bf16*)dx, sorted, perm, R, D, dword);
  return 0;
}
