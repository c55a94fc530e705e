// Elementwise dropout of the DistilBERT backbone in train mode (HF Embeddings.dropout after the
// embedding LayerNorm, FFN.dropout after lin2 -- SURVEY C26; the attention-probability dropout
// lives inside title_attn.hip / title_attn_bwd.hip).
//
//   out[e] = res[e] + h[e] * Z(e)       (res optional: res = nullptr -> out = h o Z)
//   Z(e)   = keep(seed, offset, e) / (1 - p)
//
// The same kernel is its own backward: dh = dout o Z (res = nullptr), the residual's gradient
// is dout itself.  The mask comes from common.h's Philox (counter e >> 2, component e & 3),
// so forward, backward and the torch oracle agree element for element.  One thread handles 8
// consecutive bf16 (16-byte loads/stores, two Philox calls); a scalar tail covers n % 8.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void dropout_add_kernel(const bf16* __restrict__ h, const bf16* __restrict__ res,
                                                          bf16* __restrict__ out, long n, float p, float inv_keep,
                                                          unsigned long long seed, unsigned long long offset) {
#pragma clang fp contract(off)  // res + h * Z rounded twice, exactly as the oracle (no FMA)
  const long n8 = n >> 3;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const bf16x8 hv = *(const bf16x8*)(h + i * 8);
    bf16x8 rv = {0, 0, 0, 0, 0, 0, 0, 0};
    if (res) rv = *(const bf16x8*)(res + i * 8);
    const uint4 r0 = Philox::gen(seed, offset, (unsigned long long)i * 2);
    const uint4 r1 = Philox::gen(seed, offset, (unsigned long long)i * 2 + 1);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t x = u4_get(j < 4 ? r0 : r1, j & 3);
      o[j] = f2bf(bf2f(rv[j]) + __fmul_rn(bf2f(hv[j]), drop_scale(x, p, inv_keep)));  // no FMA: = the oracle
    }
    *(bf16x8*)(out + i * 8) = o;
  }
  // tail (n % 8 elements) on the first block
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const long e = n8 * 8 + threadIdx.x;
    const uint4 r = Philox::gen(seed, offset, (unsigned long long)(e >> 2));
    const float rr = res ? bf2f(res[e]) : 0.f;
    out[e] = f2bf(rr + __fmul_rn(bf2f(h[e]), drop_scale(u4_get(r, (int)(e & 3)), p, inv_keep)));
  }
}

}  // namespace

extern "C" int fr_dropout_add_bf16(const void* h, const void* res, void* out, long n, float p, unsigned long long seed,
                                   unsigned long long offset, hipStream_t s) {
  if (!(p >= 0.f && p < 1.f)) return 2;
  if (n <= 0) return 0;
  long blocks = ((n >> 3) + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;  // grid-stride beyond 2M threads
  hipLaunchKernelGGL(dropout_add_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const bf16*)h, (const bf16*)res,
                     (bf16*)out, n, p, 1.0f / (1.0f - p), seed, offset);
  return 0;
}
