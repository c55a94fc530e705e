// LayerNorm kernels: one wave per row, row held in registers.
//
//   layer_norm : y = LN(x) * w + b                          (sa_layer_norm / output_layer_norm)
//   embed_ln   : y = LN(word[tok] + pos[t]) * w + b        (DistilBERT embeddings, eval mode)
//
// Rows are D bf16 elements (D = 768 for DistilBERT); lane l owns elements
// [256c + 4l, 256c + 4l + 4) for c < ceil(D/256), loaded as one 8-byte bf16x4 per chunk:
// each wave-instruction reads 512 contiguous bytes.  Statistics in fp32, two-pass
// (mean, then centred variance) from registers -- no extra memory pass.  HF uses the
// biased variance and eps inside the sqrt (eps = 1e-12).
#include "common.h"

namespace {

constexpr int MAXC = 4;  // D <= 1024

template <bool EMBED>
__global__ __launch_bounds__(256) void ln_kernel(const bf16* __restrict__ x, const int* __restrict__ tokens,
                                                 const bf16* __restrict__ word, const bf16* __restrict__ pos,
                                                 const float* __restrict__ w, const float* __restrict__ b,
                                                 bf16* __restrict__ y, int rows, int D, int T, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nc = (D + 255) >> 8;
  float v[MAXC][4];
  const bf16* src0;
  const bf16* src1 = nullptr;
  if constexpr (EMBED) {
    const int tok = tokens[row];
    src0 = word + (size_t)tok * D;
    src1 = pos + (size_t)(row % T) * D;
  } else {
    src0 = x + (size_t)row * D;
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int i = c * 256 + lane * 4;
    if (c < nc && i < D) {
      bf16x4 a = *(const bf16x4*)(src0 + i);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[c][k] = (float)a[k];
      if constexpr (EMBED) {
        bf16x4 p = *(const bf16x4*)(src1 + i);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[c][k] += (float)p[k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) s += v[c][k];
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[c][k] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int i = c * 256 + lane * 4;
    if (c < nc && i < D) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = v[c][k] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  bf16* out = y + (size_t)row * D;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int i = c * 256 + lane * 4;
    if (c < nc && i < D) {
      const float4 ww = *(const float4*)(w + i);
      const float4 bb = *(const float4*)(b + i);
      bf16x4 o = {f2bf((v[c][0] - mean) * rstd * ww.x + bb.x), f2bf((v[c][1] - mean) * rstd * ww.y + bb.y),
                  f2bf((v[c][2] - mean) * rstd * ww.z + bb.z), f2bf((v[c][3] - mean) * rstd * ww.w + bb.w)};
      *(bf16x4*)(out + i) = o;
    }
  }
}

}  // namespace

extern "C" int fr_layer_norm_bf16(const void* x, const float* w, const float* b, void* y, int rows, int D, float eps,
                                  hipStream_t s) {
  if (D % 4 != 0 || D > 256 * MAXC) return 1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL((ln_kernel<false>), dim3((rows + 3) / 4), dim3(256), 0, s, (const bf16*)x, nullptr, nullptr,
                     nullptr, w, b, (bf16*)y, rows, D, 1, eps);
  return 0;
}

extern "C" int fr_embed_ln_bf16(const int* tokens, const void* word, const void* pos, const float* w, const float* b,
                                void* y, int rows, int D, int T, float eps, hipStream_t s) {
  if (D % 4 != 0 || D > 256 * MAXC) return 1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL((ln_kernel<true>), dim3((rows + 3) / 4), dim3(256), 0, s, nullptr, tokens, (const bf16*)word,
                     (const bf16*)pos, w, b, (bf16*)y, rows, D, T, eps);
  return 0;
}
