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

#include <stdlib.h>

namespace {

constexpr int MAXC = 4;  // D <= 1024

template <bool EMBED>
__global__ __launch_bounds__(256) void ln_kernel(const bf16* __restrict__ x, const int* __restrict__ tokens,
                                                 const bf16* __restrict__ word, const bf16* __restrict__ pos,
                                                 const float* __restrict__ w, const float* __restrict__ b,
                                                 bf16* __restrict__ y, int rows, int D, int T, float eps,
                                                 const bf16* __restrict__ res) {
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
    if (res != nullptr) src1 = res + (size_t)row * D;  // LN(x + residual)
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int i = c * 256 + lane * 4;
    if (c < nc && i < D) {
      bf16x4 a = *(const bf16x4*)(src0 + i);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[c][k] = (float)a[k];
      if (EMBED || src1 != nullptr) {
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

// Wide form for D % 256 == 0 (D = 768: 3 chunks): a half-wave (32 lanes) per row, each lane
// owning NC 16-byte chunks (8 bf16) at [256c + 8l', +8) -- every load/store is dwordx4 and a
// wave keeps RPW rows (RPW/2 per half) in flight before the first reduction.  Stats as
// above (two-pass from registers), reductions over the 32 lanes of the half.
template <bool EMBED, int NC, int RPH>
__global__ __launch_bounds__(256) void ln16_kernel(const bf16* __restrict__ x, const int* __restrict__ tokens,
                                                   const bf16* __restrict__ word, const bf16* __restrict__ pos,
                                                   const float* __restrict__ w, const float* __restrict__ b,
                                                   bf16* __restrict__ y, int rows, int T, float eps,
                                                   const bf16* __restrict__ res, const int* __restrict__ ridx) {
  // ridx (packed title rows): EMBED -> row r embeds flat token ridx[r] (token id and position
  // from it); otherwise -> row r is stored to output row ridx[r] (back to title order)
  constexpr int D = 256 * NC;
  const int lane = threadIdx.x & 63, half = lane >> 5, hl = lane & 31;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int row0 = (wave * 2 + half) * RPH;
  float v[RPH][NC][8];
#pragma unroll
  for (int q = 0; q < RPH; ++q) {
    int row = row0 + q;
    row = row < rows ? row : rows - 1;
    const bf16* s0;
    const bf16* s1 = nullptr;
    if constexpr (EMBED) {
      const int sr = ridx != nullptr ? ridx[row] : row;
      s0 = word + (size_t)tokens[sr] * D;
      s1 = pos + (size_t)(sr % T) * D;
    } else {
      s0 = x + (size_t)row * D;
      if (res != nullptr) s1 = res + (size_t)row * D;  // LN(x + residual)
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = c * 256 + hl * 8;
      const bf16x8 a = *(const bf16x8*)(s0 + i);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[q][c][k] = (float)a[k];
      if (EMBED || s1 != nullptr) {
        const bf16x8 p = *(const bf16x8*)(s1 + i);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[q][c][k] += (float)p[k];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < RPH; ++q) {
    const int row = row0 + q;
    float sm = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int k = 0; k < 8; ++k) sm += v[q][c][k];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
    const float mean = sm * (1.0f / D);
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[q][c][k] - mean;
        sq += d * d;
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    const float rstd = rsqrtf(sq * (1.0f / D) + eps);
    if (row < rows) {
      const int orow = (!EMBED && ridx != nullptr) ? ridx[row] : row;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = c * 256 + hl * 8;
        const float4 w0 = *(const float4*)(w + i), w1 = *(const float4*)(w + i + 4);
        const float4 b0 = *(const float4*)(b + i), b1 = *(const float4*)(b + i + 4);
        const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = f2bf((v[q][c][k] - mean) * rstd * ww[k] + bb[k]);
        *(bf16x8*)(y + (size_t)orow * D + i) = o;
      }
    }
  }
}

template <bool EMBED, int RPH>
bool launch_ln16_r(const bf16* x, const int* tok, const bf16* word, const bf16* pos, const float* w, const float* b,
                   bf16* y, int rows, int D, int T, float eps, hipStream_t s, const bf16* res, const int* ridx) {
  constexpr int RPB = 8 * RPH;  // 8 half-waves per 256-thread block
  const int blocks = (rows + RPB - 1) / RPB;
  if (D == 768)
    hipLaunchKernelGGL((ln16_kernel<EMBED, 3, RPH>), dim3(blocks), dim3(256), 0, s, x, tok, word, pos, w, b, y, rows, T, eps, res, ridx);
  else if (D == 512)
    hipLaunchKernelGGL((ln16_kernel<EMBED, 2, RPH>), dim3(blocks), dim3(256), 0, s, x, tok, word, pos, w, b, y, rows, T, eps, res, ridx);
  else if (D == 1024)
    hipLaunchKernelGGL((ln16_kernel<EMBED, 4, RPH>), dim3(blocks), dim3(256), 0, s, x, tok, word, pos, w, b, y, rows, T, eps, res, ridx);
  else if (D == 256)
    hipLaunchKernelGGL((ln16_kernel<EMBED, 1, RPH>), dim3(blocks), dim3(256), 0, s, x, tok, word, pos, w, b, y, rows, T, eps, res, ridx);
  else
    return false;
  return true;
}

// Persistent form of ln16 (plain LN / LN + residual / scattered store): a grid of 8 blocks
// per CU, each half-wave walks rows with a grid stride, loads w / b ONCE into registers
// (the one-shot kernel re-reads 192 B of w / b per lane per row: 12 extra vector loads per
// 9 data accesses) and keeps the next row's loads in flight while it normalises the current.
template <int NC>
__global__ __launch_bounds__(256) void ln16p_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                    const float* __restrict__ b, bf16* __restrict__ y, int rows,
                                                    float eps, const bf16* __restrict__ res,
                                                    const int* __restrict__ ridx) {
  constexpr int D = 256 * NC;
  const int lane = threadIdx.x & 63, half = lane >> 5, hl = lane & 31;
  const int hw = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + half;
  const int nhw = gridDim.x * 8;
  int row = hw;
  if (row >= rows) return;
  float ww[NC][8], bb[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = c * 256 + hl * 8;
    const float4 w0 = *(const float4*)(w + i), w1 = *(const float4*)(w + i + 4);
    const float4 b0 = *(const float4*)(b + i), b1 = *(const float4*)(b + i + 4);
    ww[c][0] = w0.x; ww[c][1] = w0.y; ww[c][2] = w0.z; ww[c][3] = w0.w;
    ww[c][4] = w1.x; ww[c][5] = w1.y; ww[c][6] = w1.z; ww[c][7] = w1.w;
    bb[c][0] = b0.x; bb[c][1] = b0.y; bb[c][2] = b0.z; bb[c][3] = b0.w;
    bb[c][4] = b1.x; bb[c][5] = b1.y; bb[c][6] = b1.z; bb[c][7] = b1.w;
  }
  const bf16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  bf16x8 ax[NC], ar[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    ax[c] = *(const bf16x8*)(x + (size_t)row * D + c * 256 + hl * 8);
    ar[c] = res != nullptr ? *(const bf16x8*)(res + (size_t)row * D + c * 256 + hl * 8) : zero;
  }
  while (true) {
    const int nrow = row + nhw;
    const int lrow = nrow < rows ? nrow : rows - 1;  // clamped: the prefetch is unconditional
    bf16x8 nx[NC], nr[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      nx[c] = *(const bf16x8*)(x + (size_t)lrow * D + c * 256 + hl * 8);
      nr[c] = res != nullptr ? *(const bf16x8*)(res + (size_t)lrow * D + c * 256 + hl * 8) : zero;
    }
    float v[NC][8];
    float sm = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[c][k] = (float)ax[c][k] + (float)ar[c][k];
        sm += v[c][k];
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
    const float mean = sm * (1.0f / D);
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[c][k] - mean;
        sq += d * d;
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    const float rstd = rsqrtf(sq * (1.0f / D) + eps);
    const int orow = ridx != nullptr ? ridx[row] : row;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = f2bf((v[c][k] - mean) * rstd * ww[c][k] + bb[c][k]);
      *(bf16x8*)(y + (size_t)orow * D + c * 256 + hl * 8) = o;
    }
    if (nrow >= rows) break;
    row = nrow;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      ax[c] = nx[c];
      ar[c] = nr[c];
    }
  }
}

int g_ln_cus = 0;

bool launch_ln16p(const bf16* x, const float* w, const float* b, bf16* y, int rows, int D, float eps, hipStream_t s,
                  const bf16* res, const int* ridx) {
  if (g_ln_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_ln_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_ln_cus <= 0) g_ln_cus = 256;
  }
  int blocks = g_ln_cus * 8;
  const int need = (rows + 7) / 8;
  blocks = blocks < need ? blocks : need;
  if (D == 768)
    hipLaunchKernelGGL((ln16p_kernel<3>), dim3(blocks), dim3(256), 0, s, x, w, b, y, rows, eps, res, ridx);
  else if (D == 512)
    hipLaunchKernelGGL((ln16p_kernel<2>), dim3(blocks), dim3(256), 0, s, x, w, b, y, rows, eps, res, ridx);
  else if (D == 1024)
    hipLaunchKernelGGL((ln16p_kernel<4>), dim3(blocks), dim3(256), 0, s, x, w, b, y, rows, eps, res, ridx);
  else if (D == 256)
    hipLaunchKernelGGL((ln16p_kernel<1>), dim3(blocks), dim3(256), 0, s, x, w, b, y, rows, eps, res, ridx);
  else
    return false;
  return true;
}

// 0: wave-per-row kernel; 1 (default) / 2 / 3: half-wave rows with 1 / 2 / 4 rows per half-wave;
// 4: the persistent half-wave kernel above (non-embedding forms only).
// Measured interleaved at 78850 x 768 (benchmarks/ln_ab.py): LN + residual 75 / 83 / 100 us,
// plain LN 43 / 46.5 / 52 us -- one row per half-wave keeps the most rows in flight per CU.
int g_ln_wide = 4;

template <bool EMBED>
bool launch_ln16(const bf16* x, const int* tok, const bf16* word, const bf16* pos, const float* w, const float* b,
                 bf16* y, int rows, int D, int T, float eps, hipStream_t s, const bf16* res = nullptr,
                 const int* ridx = nullptr) {
  if (!EMBED && g_ln_wide == 4) return launch_ln16p(x, w, b, y, rows, D, eps, s, res, ridx);
  if (g_ln_wide == 2) return launch_ln16_r<EMBED, 2>(x, tok, word, pos, w, b, y, rows, D, T, eps, s, res, ridx);
  if (g_ln_wide == 3) return launch_ln16_r<EMBED, 4>(x, tok, word, pos, w, b, y, rows, D, T, eps, s, res, ridx);
  return launch_ln16_r<EMBED, 1>(x, tok, word, pos, w, b, y, rows, D, T, eps, s, res, ridx);
}

// LayerNorm backward (unfrozen backbone): y = (x - mu) * rstd * w + b
//   dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w
//   dw = sum_rows dy * xhat, db = sum_rows dy   (per-lane partials over a grid-stride of
//   rows, reduced across the block's waves in LDS, one atomic per column per block)
template <bool PF>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                     const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                                     float* __restrict__ dw, float* __restrict__ db, int rows, int D,
                                                     float eps, float* __restrict__ dxs, bf16* __restrict__ dxz,
                                                     float pdrop, float inv_keep, unsigned long long seed,
                                                     unsigned long long offset) {
  // dxz (optional, with dxs): dx o Z, the dropout backward of the layer that fed the LN input
  // (HF FFN.dropout, dropout.hip's element-indexed mask), written beside dx; dxs then sums
  // dx o Z -- the lin2 bias gradient -- instead of dx
  // dxs (optional): column sums of the bf16 dx it writes -- the bias gradient of the linear
  // layer that produced the LN input (config 5 training blocks), without a separate pass
  __shared__ float red[3][4][256 * MAXC];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nc = (D + 255) >> 8;
  float pw[MAXC][4], pb[MAXC][4], px[MAXC][4];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) pw[c][k] = pb[c][k] = px[c][k] = 0.f;
  // the next row's x / dy are loaded while this row is reduced and written (one row in flight
  // ahead per wave: the row loop was a chain of load latencies, ~3 TB/s at 78850 x 768)
  const int stride = gridDim.x * 4;
  bf16x4 xa[MAXC], xd[MAXC];
  auto load_row = [&](int r) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int i = c * 256 + lane * 4;
      const bool ok = c < nc && i < D;
      const size_t src = ok ? (size_t)r * D + i : 0;  // masked lanes read row 0 (discarded below)
      xa[c] = *(const bf16x4*)(x + src);
      xd[c] = *(const bf16x4*)(dy + src);
    }
  };
  if (blockIdx.x * 4 + wv < rows) load_row(blockIdx.x * 4 + wv);
  for (int row = blockIdx.x * 4 + wv; row < rows; row += stride) {
    float v[MAXC][4], g[MAXC][4], dyv[MAXC][4];
    bf16x4 ca[MAXC], cd[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      ca[c] = xa[c];
      cd[c] = xd[c];
    }
    if (PF && row + stride < rows) load_row(row + stride);  // wave-uniform
    if (!PF && row + stride < rows) {  // A/B form: the next row only after this one is written
      __builtin_amdgcn_sched_barrier(0);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int i = c * 256 + lane * 4;
      const bool ok = c < nc && i < D;
      bf16x4 a = ok ? ca[c] : bf16x4{0, 0, 0, 0};
      bf16x4 d = ok ? cd[c] : bf16x4{0, 0, 0, 0};
      float4 ww = ok ? *(const float4*)(w + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float wa[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[c][k] = (float)a[k];
        dyv[c][k] = (float)d[k];
        g[c][k] = dyv[c][k] * wa[k];
        s += v[c][k];
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
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int i = c * 256 + lane * 4;
      if (c < nc && i < D) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float xh = (v[c][k] - mean) * rstd;
          v[c][k] = xh;
          sg += g[c][k];
          sgx += g[c][k] * xh;
          pw[c][k] += dyv[c][k] * xh;
          pb[c][k] += dyv[c][k];
        }
      }
    }
    const float mg = wave_sum(sg) / (float)D, mgx = wave_sum(sgx) / (float)D;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int i = c * 256 + lane * 4;
      if (c < nc && i < D) {
        bf16x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = f2bf(rstd * (g[c][k] - mg - v[c][k] * mgx));
        *(bf16x4*)(dx + (size_t)row * D + i) = o;
        if (dxz != nullptr) {
          // element e = row * D + i + k: Philox counter e >> 2, component k (i % 4 == 0);
          // rounded as dropout_add_kernel's own backward (bf16(dx) * Z, one rounding)
          const uint4 r = Philox::gen(seed, offset, ((unsigned long long)row * D + i) >> 2);
          bf16x4 oz;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            oz[k] = f2bf(__fmul_rn(bf2f(o[k]), drop_scale(u4_get(r, k), pdrop, inv_keep)));
            px[c][k] += (float)oz[k];
          }
          *(bf16x4*)(dxz + (size_t)row * D + i) = oz;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) px[c][k] += (float)o[k];
        }
      }
    }
    if (!PF && row + stride < rows) load_row(row + stride);
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[0][wv][(c * 64 + lane) * 4 + k] = pw[c][k];
      red[1][wv][(c * 64 + lane) * 4 + k] = pb[c][k];
      red[2][wv][(c * 64 + lane) * 4 + k] = px[c][k];
    }
  __syncthreads();
  for (int j = threadIdx.x; j < nc * 256; j += 256) {
    const int c = j >> 8, rem = j & 255, ln = rem >> 2, k = rem & 3;
    const int i = c * 256 + ln * 4 + k;
    if (i < D) {
      const int idx = (c * 64 + ln) * 4 + k;
      atomicAdd(dw + i, red[0][0][idx] + red[0][1][idx] + red[0][2][idx] + red[0][3][idx]);
      atomicAdd(db + i, red[1][0][idx] + red[1][1][idx] + red[1][2][idx] + red[1][3][idx]);
      if (dxs != nullptr) atomicAdd(dxs + i, red[2][0][idx] + red[2][1][idx] + red[2][2][idx] + red[2][3][idx]);
    }
  }
}

__device__ __forceinline__ float erf_fast2(float x) {
  const float ax = fabsf(x);
  const float t = __frcp_rn(1.0f + 0.3275911f * ax);
  const float y = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  return copysignf(1.0f - y * __expf(-ax * ax), x);
}

// GELU(erf) forward / backward as streaming kernels (training mode keeps the pre-activation)
__global__ __launch_bounds__(256) void gelu_kernel(const bf16* __restrict__ z, const bf16* __restrict__ dh,
                                                   bf16* __restrict__ out, long n4, int bwd) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const bf16x4 zz = *(const bf16x4*)(z + 4 * i);
    bf16x4 o;
    if (bwd) {
      const bf16x4 gg = *(const bf16x4*)(dh + 4 * i);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x = (float)zz[k];
        const float cdf = 0.5f * (1.0f + erf_fast2(x * 0.70710678118654752f));
        const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
        o[k] = f2bf((float)gg[k] * (cdf + x * pdf));
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x = (float)zz[k];
        o[k] = f2bf(0.5f * x * (1.0f + erf_fast2(x * 0.70710678118654752f)));
      }
    }
    *(bf16x4*)(out + 4 * i) = o;
  }
}

}  // namespace

extern "C" void fr_ln_set_wide(int v) { g_ln_wide = v; }

extern "C" int fr_layer_norm_bwd_bf16(const void* x, const float* w, const void* dy, void* dx, float* dw, float* db,
                                      int rows, int D, float eps, hipStream_t s, float* dxs, void* dxz, float pdrop,
                                      unsigned long long seed, unsigned long long offset) {
  if (D % 4 != 0 || D > 256 * MAXC) return 1;
  if (dxz != nullptr && (dxs == nullptr || !(pdrop > 0.f && pdrop < 1.f))) return 2;
  if (rows == 0) return 0;
  int blocks = (rows + 3) / 4;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(ln_bwd_kernel<true>, dim3(blocks), dim3(256), 0, s, (const bf16*)x, w, (const bf16*)dy,
                     (bf16*)dx, dw, db, rows, D, eps, dxs, (bf16*)dxz, pdrop, dxz ? 1.0f / (1.0f - pdrop) : 1.f,
                     seed, offset);
  return 0;
}

extern "C" int fr_gelu_bf16(const void* z, const void* dh, void* out, long n, int bwd, hipStream_t s) {
  if (n % 4 != 0) return 1;
  const long n4 = n / 4;
  if (n4 == 0) return 0;
  long b = (n4 + 255) / 256;
  if (b > 4096) b = 4096;
  hipLaunchKernelGGL(gelu_kernel, dim3((unsigned)b), dim3(256), 0, s, (const bf16*)z, (const bf16*)dh, (bf16*)out, n4,
                     bwd);
  return 0;
}

// y = LN(x [+ res]) * w + b; res may be null
extern "C" int fr_layer_norm_bf16(const void* x, const float* w, const float* b, void* y, int rows, int D, float eps,
                                  const void* res, hipStream_t s) {
  if (D % 4 != 0 || D > 256 * MAXC) return 1;
  if (rows == 0) return 0;
  if (g_ln_wide && launch_ln16<false>((const bf16*)x, nullptr, nullptr, nullptr, w, b, (bf16*)y, rows, D, 1, eps, s,
                                      (const bf16*)res))
    return 0;
  hipLaunchKernelGGL((ln_kernel<false>), dim3((rows + 3) / 4), dim3(256), 0, s, (const bf16*)x, nullptr, nullptr,
                     nullptr, w, b, (bf16*)y, rows, D, 1, eps, (const bf16*)res);
  return 0;
}

extern "C" int fr_embed_ln_bf16(const int* tokens, const void* word, const void* pos, const float* w, const float* b,
                                void* y, int rows, int D, int T, float eps, hipStream_t s) {
  if (D % 4 != 0 || D > 256 * MAXC) return 1;
  if (rows == 0) return 0;
  if (g_ln_wide && launch_ln16<true>(nullptr, tokens, (const bf16*)word, (const bf16*)pos, w, b, (bf16*)y, rows, D, T, eps, s))
    return 0;
  hipLaunchKernelGGL((ln_kernel<true>), dim3((rows + 3) / 4), dim3(256), 0, s, nullptr, tokens, (const bf16*)word,
                     (const bf16*)pos, w, b, (bf16*)y, rows, D, T, eps, nullptr);
  return 0;
}

// Packed-row variants (title_attn.hip, title_plan_kernel): embedding of row r = flat token
// src[r] of tokens [n*T]; LayerNorm storing row r to output row dst[r].  D % 256 == 0 only.
extern "C" int fr_embed_ln_rows_bf16(const int* tokens, const int* src, const void* word, const void* pos,
                                     const float* w, const float* b, void* y, int rows, int D, int T, float eps,
                                     hipStream_t s) {
  if (rows == 0) return 0;
  return launch_ln16<true>(nullptr, tokens, (const bf16*)word, (const bf16*)pos, w, b, (bf16*)y, rows, D, T, eps, s,
                           nullptr, src) ? 0 : 1;
}

extern "C" int fr_layer_norm_scatter_bf16(const void* x, const float* w, const float* b, void* y, int rows, int D,
                                          float eps, const void* res, const int* dst, hipStream_t s) {
  if (rows == 0) return 0;
  return launch_ln16<false>((const bf16*)x, nullptr, nullptr, nullptr, w, b, (bf16*)y, rows, D, 1, eps, s,
                            (const bf16*)res, dst) ? 0 : 1;
}
