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

constexpr int CS_MAX_CHUNKS = 256;

// grid (ceil(N / 512), chunks); lane owns 8 consecutive columns, the 4 waves of a block
// stride over the chunk's rows (4 rows in flight per wave); partial[chunk][n].  chunks is
// chosen so the grid has ~1024 blocks whatever N is.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const bf16* __restrict__ x, int M, int N,
                                                             float* __restrict__ partial, int ld) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int rows_per = (M + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < N) {
    int r = r0 + wave;
    for (; r + 12 < r1; r += 16) {
      const bf16x8 a = *(const bf16x8*)(x + (size_t)r * ld + c0);
      const bf16x8 b = *(const bf16x8*)(x + (size_t)(r + 4) * ld + c0);
      const bf16x8 c = *(const bf16x8*)(x + (size_t)(r + 8) * ld + c0);
      const bf16x8 d = *(const bf16x8*)(x + (size_t)(r + 12) * ld + c0);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += ((float)a[k] + (float)b[k]) + ((float)c[k] + (float)d[k]);
    }
    for (; r < r1; r += 4) {
      const bf16x8 a = *(const bf16x8*)(x + (size_t)r * ld + c0);
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

// 64 columns per block, the 16 waves split the chunks (<= 16 loads per lane), fixed-order
// LDS combine
// GELU backward with the column sums of its output (training FFN1: dz = dF * GELU'(z) and
// the FFN1 bias gradient) in one streaming pass -- same grid / partials as colsum, so the
// sums are deterministic.  GELU' with erf from Abramowitz-Stegun 7.1.26 (|err| <= 1.5e-7).
__device__ __forceinline__ float gelu_grad_s(float x) {
  const float z = x * 0.70710678118654752f, az = fabsf(z);
  const float t = __frcp_rn(1.0f + 0.3275911f * az);
  const float y = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float erfv = copysignf(1.0f - y * __expf(-az * az), z);
  return 0.5f * (1.0f + erfv) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

__global__ __launch_bounds__(256) void gelu_bwd_colsum_partial_kernel(const bf16* __restrict__ df,
                                                                      const bf16* __restrict__ zz,
                                                                      bf16* __restrict__ dz, int M, int N,
                                                                      float* __restrict__ partial) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int rows_per = (M + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < N) {
    int r = r0 + wave;
    for (; r + 4 < r1; r += 8) {  // two rows in flight per wave
      const size_t o0 = (size_t)r * N + c0, o1 = (size_t)(r + 4) * N + c0;
      const bf16x8 g0 = *(const bf16x8*)(df + o0), z0 = *(const bf16x8*)(zz + o0);
      const bf16x8 g1 = *(const bf16x8*)(df + o1), z1 = *(const bf16x8*)(zz + o1);
      bf16x8 d0, d1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        d0[k] = f2bf((float)g0[k] * gelu_grad_s((float)z0[k]));
        d1[k] = f2bf((float)g1[k] * gelu_grad_s((float)z1[k]));
        acc[k] += (float)d0[k] + (float)d1[k];
      }
      *(bf16x8*)(dz + o0) = d0;
      *(bf16x8*)(dz + o1) = d1;
    }
    for (; r < r1; r += 4) {
      const size_t o0 = (size_t)r * N + c0;
      const bf16x8 g0 = *(const bf16x8*)(df + o0), z0 = *(const bf16x8*)(zz + o0);
      bf16x8 d0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        d0[k] = f2bf((float)g0[k] * gelu_grad_s((float)z0[k]));
        acc[k] += (float)d0[k];
      }
      *(bf16x8*)(dz + o0) = d0;
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

__global__ __launch_bounds__(1024) void colsum_final_kernel(const float* __restrict__ partial, int N, int chunks,
                                                            float* __restrict__ out) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < N)
    for (int k = wave; k < chunks; k += 16) s += partial[(size_t)k * N + c];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < N) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    out[c] = t;
  }
}

constexpr int EG_HEAVY = 64;  // segments longer than this go to the block-per-segment kernel

// one wave per sorted position b; only the first occurrence of each token (b == 0 or a new
// id) works: it sums rows perm[b .. end) of dx in sorted (= occurrence) order.  Segments
// longer than EG_HEAVY ([CLS], [SEP], frequent words) are appended to `heavy` instead.
__global__ __launch_bounds__(256) void embed_grad_kernel(const bf16* __restrict__ dx, const int* __restrict__ sorted,
                                                         const int* __restrict__ perm, int R, int D,
                                                         float* __restrict__ dword, int* __restrict__ heavy,
                                                         int* __restrict__ n_heavy) {
  const int b = blockIdx.x * 4 + (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= R) return;
  const int tok = sorted[b];
  if (tok == 0 || (b > 0 && sorted[b - 1] == tok)) return;
  int e = b + 1;
  while (e < R && e - b <= EG_HEAVY && sorted[e] == tok) ++e;
  if (e - b > EG_HEAVY) {
    if (lane == 0) heavy[atomicAdd(n_heavy, 1)] = b;
    return;
  }
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

// heavy segments: a persistent grid of 1024-thread blocks walks the heavy list; wave w of a
// block sums rows b+w, b+w+16, ... (lanes over columns, 12 per lane for D = 768), then a
// fixed-order combine of the 16 wave partials through LDS.  D <= 768.
__global__ __launch_bounds__(1024) void embed_grad_heavy_kernel(const bf16* __restrict__ dx,
                                                                const int* __restrict__ sorted,
                                                                const int* __restrict__ perm, int R, int D,
                                                                float* __restrict__ dword,
                                                                const int* __restrict__ heavy,
                                                                const int* __restrict__ n_heavy) {
  __shared__ float part[16][768];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nh = *n_heavy;
  const int nc = D / 256;  // column groups of 4 per lane
  for (int h = blockIdx.x; h < nh; h += gridDim.x) {
    const int b = heavy[h];
    const int tok = sorted[b];
    int e = b + 1;
    while (e < R && sorted[e] == tok) ++e;
    float acc[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    for (int r = b + wave; r < e; r += 16) {
      const bf16* row = dx + (size_t)perm[r] * D;
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (j < nc) {
          const bf16x4 v = *(const bf16x4*)(row + j * 256 + lane * 4);
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[j][k] += (float)v[k];
        }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j < nc) {
#pragma unroll
        for (int k = 0; k < 4; ++k) part[wave][j * 256 + lane * 4 + k] = acc[j][k];
      }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 1024) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < 16; ++w) sum += part[w][c];
      dword[(size_t)tok * D + c] = sum;
    }
    __syncthreads();
  }
}

}  // namespace

// partial: fr_colsum_chunks() * N floats of scratch
// ld: row stride in elements (>= N, a multiple of 8: e.g. the Q third of a [M, 3D] tensor)
extern "C" int fr_colsum_bf16(const void* x, int M, int N, float* partial, float* out, hipStream_t s, int ld) {
  if (ld <= 0) ld = N;
  if (N % 8 != 0 || ld % 8 != 0 || ld < N || M <= 0) return 1;
  const int cb = (N + 511) / 512;
  int chunks = 1024 / cb;
  chunks = chunks < 16 ? 16 : (chunks > CS_MAX_CHUNKS ? CS_MAX_CHUNKS : chunks);
  chunks = chunks < M ? chunks : M;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(cb, chunks), dim3(256), 0, s, (const bf16*)x, M, N, partial, ld);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + 63) / 64), dim3(1024), 0, s, partial, N, chunks, out);
  return 0;
}

extern "C" int fr_colsum_chunks() { return CS_MAX_CHUNKS; }

// dz = df * GELU'(z) (bf16 [M, N], contiguous) and out[N] = column sums of dz
extern "C" int fr_gelu_bwd_colsum_bf16(const void* df, const void* z, void* dz, int M, int N, float* partial,
                                       float* out, hipStream_t s) {
  if (N % 8 != 0 || M <= 0) return 1;
  const int cb = (N + 511) / 512;
  int chunks = 2048 / cb;
  chunks = chunks < 16 ? 16 : (chunks > CS_MAX_CHUNKS ? CS_MAX_CHUNKS : chunks);
  chunks = chunks < M ? chunks : M;
  hipLaunchKernelGGL(gelu_bwd_colsum_partial_kernel, dim3(cb, chunks), dim3(256), 0, s, (const bf16*)df,
                     (const bf16*)z, (bf16*)dz, M, N, partial);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + 63) / 64), dim3(1024), 0, s, partial, N, chunks, out);
  return 0;
}

// dword must be zeroed by the caller (rows of tokens absent from the batch stay zero);
// scratch: R + 1 ints (heavy list + its count, zeroed by the caller)
extern "C" int fr_embed_grad_bf16(const void* dx, const int* sorted, const int* perm, int R, int D, float* dword,
                                  int* scratch, hipStream_t s) {
  if (D % 256 != 0 || D > 768 || R < 0) return 1;
  if (R == 0) return 0;
  hipLaunchKernelGGL(embed_grad_kernel, dim3((R + 3) / 4), dim3(256), 0, s, (const bf16*)dx, sorted, perm, R, D, dword,
                     scratch + 1, scratch);
  hipLaunchKernelGGL(embed_grad_heavy_kernel, dim3(256), dim3(1024), 0, s, (const bf16*)dx, sorted, perm, R, D, dword,
                     scratch + 1, scratch);
  return 0;
}
