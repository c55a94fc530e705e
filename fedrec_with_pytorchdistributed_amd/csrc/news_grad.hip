// Per-news gradient reduction with fused local differential privacy
// (reference client.py:26-48 process_news_grad, client.py:87-89 noise, model.py:105-109;
// SURVEY §2.3 K16/K17):
//
//   out[u] = sum_{r in segment u} ( clip_C(g_r) + N(0, std) )
//
// g_r is one occurrence's gradient w.r.t. a candidate/history news vector (400 floats).
// Rows are grouped by output id (perm/seg_ptr from the dedup kernel), so each output row
// is summed by ONE wave in a fixed order: deterministic, no float atomics.
//
// LDP: per-occurrence L2 clip to C (clip > 0), then Gaussian noise N(0, std) with
// std = sigma * C (default) or sigma (reference quirk Q10: no clip, std = sigma).  Noise
// comes from Philox-4x32-10 keyed by (seed, offset=step) with a counter derived from the
// occurrence row, so it does not depend on which wave processes it.  The default float4 chunk
// pass applies the clip + noise as it loads each occurrence row (one launch + the edge fix-up);
// the separate per-occurrence pass (ldp_rows_kernel) remains for the other forms.
#include "common.h"

#include <algorithm>

#include <stdlib.h>

namespace {

constexpr int MAXV = 8;   // D <= 512
constexpr int NW = 16;    // waves per segment block
constexpr int UNR = 4;    // rows in flight per wave

// Pass 1 (LDP only): one wave per occurrence row -- clip to C, add N(0, std).  Fully
// parallel over all R = B*(C+H) occurrences, so the per-element Philox work never sits
// behind one popular news id.  Each Philox call yields 4 uniforms -> 4 normals (2 x
// Box-Muller), counter = (row, element group of 4): independent of the launch geometry.
__global__ __launch_bounds__(256) void ldp_rows_kernel(const float* __restrict__ rows, float* __restrict__ out, int R,
                                                       int D, float clip, float noise_std, unsigned long long seed,
                                                       unsigned long long offset,
                                                       const unsigned long long* __restrict__ dev_off) {
  // dev_off (optional): a device step counter added to the offset, so a captured HIP graph
  // draws fresh noise at every replay (the host offset is frozen into the graph)
  if (dev_off != nullptr) offset += *dev_off;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* g = rows + (size_t)r * D;
  float v[MAXV];
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int d = lane + 64 * k;
    v[k] = d < D ? g[d] : 0.f;
    sq += v[k] * v[k];
  }
  float f = 1.0f;
  if (clip > 0.f) f = fminf(1.0f, clip / (sqrtf(wave_sum(sq)) + 1e-12f));
  // element d = lane + 64k; noise for elements (4j .. 4j+3) of the row from counter (r, j)
#pragma unroll
  for (int k = 0; k < MAXV; k += 4) {
    // lanes of this pass cover elements lane + 64k .. lane + 64(k+3): counter per (r, lane, k/4)
    float nz[4] = {0.f, 0.f, 0.f, 0.f};
    if (noise_std > 0.f) {
      const uint4 rnd = Philox::gen(seed, offset, ((unsigned long long)r << 16) | (unsigned)(lane * 2 + (k >> 2)));
      const float2 a = box_muller(rnd.x, rnd.y), b = box_muller(rnd.z, rnd.w);
      nz[0] = a.x; nz[1] = a.y; nz[2] = b.x; nz[3] = b.y;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int d = lane + 64 * (k + t);
      if (d < D) out[(size_t)r * D + d] = v[k + t] * f + noise_std * nz[t];
    }
  }
}

// Pass 2: deterministic segment sum.  One 1024-thread block (16 waves) per output row:
// wave w takes occurrences beg+w, beg+w+16, ... with UNR row loads in flight; the 16
// partials are combined in LDS in a fixed order.  The <unk>/pad row 0 -- every short
// history points at it, ~1000 occurrences per batch -- is spread over 16 waves.
__global__ __launch_bounds__(1024) void segsum_kernel(const float* __restrict__ rows, const int* __restrict__ perm,
                                                      const int* __restrict__ seg_ptr, float* __restrict__ out, int U,
                                                      int D) {
  __shared__ float part[NW][64 * MAXV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = blockIdx.x;
  float acc[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) acc[k] = 0.f;
  const int beg = seg_ptr[u], end = seg_ptr[u + 1];
  for (int i0 = beg + w; i0 < end; i0 += NW * UNR) {
    float v[UNR][MAXV];
#pragma unroll
    for (int j = 0; j < UNR; ++j) {
      const int i = i0 + j * NW;
      const int r = i < end ? perm[i] : -1;
      const float* g = rows + (size_t)(r < 0 ? 0 : r) * D;
#pragma unroll
      for (int k = 0; k < MAXV; ++k) {
        const int d = lane + 64 * k;
        v[j][k] = (r >= 0 && d < D) ? g[d] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < UNR; ++j)
#pragma unroll
      for (int k = 0; k < MAXV; ++k) acc[k] += v[j][k];
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) part[w][lane + 64 * k] = acc[k];
  __syncthreads();
  float* o = out + (size_t)u * D;
  for (int d = threadIdx.x; d < D; d += 1024) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) t += part[q][d];
    o[d] = t;
  }
}

// Chunked form (default): the one-block-per-output form above launches a 1024-thread block
// for every unique news (~1,600 per step, most with 1-3 occurrences) and serialises the
// ~1,000-occurrence pad row on one CU.  Here the grouped occurrence list (perm order) is cut
// into fixed chunks of SCH positions, one wave per chunk: the wave loads all its rows at once
// (SCH loads in flight), sums each segment run in order, and writes a segment that lies
// wholly inside the chunk straight to out[u]; a segment crossing a chunk edge leaves a
// partial in scratch[chunk][slot] (slot 0: started before the chunk, slot 1: ends after it).
// A second pass sums the partials of every crossing segment in chunk order.  The chunk grid
// is fixed by R alone, so the result is deterministic, and no float atomics are used.
// SCH: chunk length (16; 8 -- half the per-wave row registers, 89 vs 161 VGPRs, twice the
// waves -- measured neutral: 0.5694 / 0.5668 vs 0.5665 / 0.5702 ms per step,
// profiles/r3_ab_segsum_ua.txt)
template <int SCH>
__global__ __launch_bounds__(256) void segsum_chunk_kernel(const float* __restrict__ rows, const int* __restrict__ perm,
                                                           const int* __restrict__ seg_ptr, const int* __restrict__ inv,
                                                           float* __restrict__ out, float* __restrict__ scratch, int U,
                                                           int R, int D) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int p0 = c * SCH;
  if (p0 >= R) return;
  const int p1 = min(p0 + SCH, R);
  int u = inv[perm[p0]];  // segment of position p0
  float v[SCH][MAXV];
#pragma unroll
  for (int j = 0; j < SCH; ++j) {
    const int pp = p0 + j;
    const int r = perm[pp < p1 ? pp : p1 - 1];
    const float* g = rows + (size_t)r * D;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int d = lane + 64 * k;
      v[j][k] = d < D ? g[d] : 0.f;
    }
  }
  float acc[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) acc[k] = 0.f;
  int s_beg = seg_ptr[u], s_end = seg_ptr[u + 1];
#pragma unroll
  for (int j = 0; j < SCH; ++j) {
    const int pp = p0 + j;
    if (pp < p1) {
#pragma unroll
      for (int k = 0; k < MAXV; ++k) acc[k] += v[j][k];
      if (pp + 1 == s_end || pp + 1 == p1) {  // flush the run of segment u
        float* dst;
        if (s_beg >= p0 && s_end <= p1) dst = out + (size_t)u * D;
        else dst = scratch + ((size_t)c * 2 + (s_beg < p0 ? 0 : 1)) * D;
#pragma unroll
        for (int k = 0; k < MAXV; ++k) {
          const int d = lane + 64 * k;
          if (d < D) dst[d] = acc[k];
          acc[k] = 0.f;
        }
        if (pp + 1 == s_end && pp + 1 < p1) {
          ++u;
          s_beg = s_end;
          s_end = seg_ptr[u + 1];
        }
      }
    }
  }
}

template <int SCH>
__global__ __launch_bounds__(256) void segsum_fix_kernel(const int* __restrict__ seg_ptr, float* __restrict__ out,
                                                         const float* __restrict__ scratch, int U, int D) {
  // partials of a crossing segment: [scratch[c0][1], scratch[c0+1][0], ..., scratch[c1][0]];
  // wave w sums entries w, w+4, w+8, ... (8 loads in flight: the pad row's ~120 partials are a
  // chain of load rounds), then the 4 sums add in order -- a fixed partition, so the result
  // does not depend on timing
  __shared__ float part[4][64 * MAXV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = blockIdx.x;
  const int beg = seg_ptr[u], end = seg_ptr[u + 1];
  if (beg == end) {  // no occurrences (a padded unique slot of a step graph): a zero row
    for (int d = threadIdx.x; d < D; d += 256) out[(size_t)u * D + d] = 0.f;
    return;
  }
  const int c0 = beg / SCH, c1 = (end - 1) / SCH;
  if (c0 == c1) return;  // written whole by the chunk pass (block-uniform exit)
  const int n = c1 - c0 + 1;
  float acc[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) acc[k] = 0.f;
  for (int i0 = w; i0 < n; i0 += 32) {
    float v[8][MAXV];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = i0 + 4 * j;
      const size_t slot = i == 0 ? (size_t)c0 * 2 + 1 : (size_t)(c0 + i) * 2;
#pragma unroll
      for (int k = 0; k < MAXV; ++k) {
        const int d = lane + 64 * k;
        v[j][k] = (i < n && d < D) ? scratch[slot * D + d] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int k = 0; k < MAXV; ++k) acc[k] += v[j][k];
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) part[w][lane + 64 * k] = acc[k];
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += 256) out[(size_t)u * D + d] = ((part[0][d] + part[1][d]) + part[2][d]) + part[3][d];
}

// float4 form of the chunked pass (D % 4 == 0, 16-B aligned rows; variant 2): a lane holds
// columns 4 lane + 256 k (two float4 at D = 400) -- 2 loads per row instead of 7 scalar ones.
// Same chunk grid and scratch slots as segsum_chunk_kernel (segsum_fix_kernel finishes both).
//
// LDP = true (K16 fused into K17): every occurrence row is clipped to L2 norm C and
// gets N(0, std) noise as it is loaded -- no separate clip + noise pass over the rows and no
// second copy of them.  Noise of elements 4L .. 4L+3 of occurrence row r comes from Philox
// counter (r << 16) | L (4 uniforms -> 4 normals), keyed by (seed, offset + *dev_off): a pure
// function of the occurrence, whatever chunk / wave sums it.
constexpr int MAXV4 = 2;  // D <= 512
template <int SC, bool LDP = false>
__global__ __launch_bounds__(256) void segsum_chunk4_kernel(const float4* __restrict__ rows,
                                                            const int* __restrict__ perm,
                                                            const int* __restrict__ seg_ptr,
                                                            const int* __restrict__ inv, float4* __restrict__ out,
                                                            float4* __restrict__ scratch, int U, int R, int D4,
                                                            float clip = 0.f, float noise_std = 0.f,
                                                            unsigned long long seed = 0, unsigned long long offset = 0,
                                                            const unsigned long long* __restrict__ dev_off = nullptr) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int p0 = c * SC;
  if (p0 >= R) return;
  const int p1 = min(p0 + SC, R);
  int rr[SC];
#pragma unroll
  for (int j = 0; j < SC; ++j) rr[j] = perm[min(p0 + j, p1 - 1)];
  int u = inv[rr[0]];  // segment of position p0
  int s_beg = seg_ptr[u], s_end = seg_ptr[u + 1];
  float4 v[SC][MAXV4];
#pragma unroll
  for (int j = 0; j < SC; ++j)
#pragma unroll
    for (int k = 0; k < MAXV4; ++k) {
      const int d = lane + 64 * k;
      v[j][k] = d < D4 ? rows[(size_t)rr[j] * D4 + d] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  if constexpr (LDP) {
    const unsigned long long off = offset + (dev_off != nullptr ? *dev_off : 0ull);
#pragma unroll
    for (int j = 0; j < SC; ++j) {
      float f = 1.0f;
      if (clip > 0.f) {
        float sq = 0.f;
#pragma unroll
        for (int k = 0; k < MAXV4; ++k)
          sq += v[j][k].x * v[j][k].x + v[j][k].y * v[j][k].y + v[j][k].z * v[j][k].z + v[j][k].w * v[j][k].w;
        f = fminf(1.0f, clip / (sqrtf(wave_sum(sq)) + 1e-12f));
      }
#pragma unroll
      for (int k = 0; k < MAXV4; ++k) {
        const int d = lane + 64 * k;
        float4 nz = make_float4(0.f, 0.f, 0.f, 0.f);
        if (noise_std > 0.f && d < D4) {
          const uint4 rnd = Philox::gen(seed, off, ((unsigned long long)rr[j] << 16) | (unsigned)d);
          const float2 a = box_muller(rnd.x, rnd.y), b = box_muller(rnd.z, rnd.w);
          nz = make_float4(a.x, a.y, b.x, b.y);
        }
        v[j][k] = make_float4(v[j][k].x * f + noise_std * nz.x, v[j][k].y * f + noise_std * nz.y,
                              v[j][k].z * f + noise_std * nz.z, v[j][k].w * f + noise_std * nz.w);
      }
    }
  }
  float4 acc[MAXV4];
#pragma unroll
  for (int k = 0; k < MAXV4; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < SC; ++j) {
    const int pp = p0 + j;
    if (pp < p1) {
#pragma unroll
      for (int k = 0; k < MAXV4; ++k) {
        acc[k].x += v[j][k].x; acc[k].y += v[j][k].y; acc[k].z += v[j][k].z; acc[k].w += v[j][k].w;
      }
      if (pp + 1 == s_end || pp + 1 == p1) {  // flush the run of segment u
        float4* dst;
        if (s_beg >= p0 && s_end <= p1) dst = out + (size_t)u * D4;
        else dst = scratch + ((size_t)c * 2 + (s_beg < p0 ? 0 : 1)) * D4;
#pragma unroll
        for (int k = 0; k < MAXV4; ++k) {
          const int d = lane + 64 * k;
          if (d < D4) dst[d] = acc[k];
          acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (pp + 1 == s_end && pp + 1 < p1) {
          ++u;
          s_beg = s_end;
          s_end = seg_ptr[u + 1];
        }
      }
    }
  }
}

// LDP form of the float4 chunk pass with the clip + noise spread over a block: the transform of a
// chunk's 16 occurrence rows (a row norm, 2 Philox draws + 4 Box-Muller pairs per lane) is the
// bulk of the work, and one wave per chunk left it on ~220 waves for a config-2-sized batch
// (29 us vs 9 for the plain pass).  Here one 256-thread block per chunk: wave w transforms rows
// w, w + 4, ... into LDS, then wave 0 sums the runs exactly as segsum_chunk4_kernel<SC, true>
// (same transform arithmetic, same summation order: bitwise the same partials and rows).
template <int SC, bool LDP = true>
__global__ __launch_bounds__(256) void segsum_chunk4_ldp_kernel(const float4* __restrict__ rows,
                                                                const int* __restrict__ perm,
                                                                const int* __restrict__ seg_ptr,
                                                                const int* __restrict__ inv, float4* __restrict__ out,
                                                                float4* __restrict__ scratch, int U, int R, int D4,
                                                                float clip, float noise_std, unsigned long long seed,
                                                                unsigned long long offset,
                                                                const unsigned long long* __restrict__ dev_off) {
  __shared__ float4 ls[SC][64 * MAXV4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x;
  const int p0 = c * SC;
  if (p0 >= R) return;
  const int p1 = min(p0 + SC, R);
  const unsigned long long off = offset + (dev_off != nullptr ? *dev_off : 0ull);
#pragma unroll
  for (int jj = 0; jj < SC / 4; ++jj) {
    const int j = w + 4 * jj;
    const int r = perm[min(p0 + j, p1 - 1)];
    float4 v[MAXV4];
#pragma unroll
    for (int k = 0; k < MAXV4; ++k) {
      const int d = lane + 64 * k;
      v[k] = d < D4 ? rows[(size_t)r * D4 + d] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if constexpr (!LDP) {  // plain sum (A/B form of segsum_chunk4_kernel<SC, false>): rows as loaded
#pragma unroll
      for (int k = 0; k < MAXV4; ++k) ls[j][lane + 64 * k] = v[k];
      continue;
    }
    float f = 1.0f;
    if (clip > 0.f) {
      float sq = 0.f;
#pragma unroll
      for (int k = 0; k < MAXV4; ++k) sq += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
      f = fminf(1.0f, clip / (sqrtf(wave_sum(sq)) + 1e-12f));
    }
#pragma unroll
    for (int k = 0; k < MAXV4; ++k) {
      const int d = lane + 64 * k;
      float4 nz = make_float4(0.f, 0.f, 0.f, 0.f);
      if (noise_std > 0.f && d < D4) {
        const uint4 rnd = Philox::gen(seed, off, ((unsigned long long)r << 16) | (unsigned)d);
        const float2 a = box_muller(rnd.x, rnd.y), b = box_muller(rnd.z, rnd.w);
        nz = make_float4(a.x, a.y, b.x, b.y);
      }
      ls[j][d] = make_float4(v[k].x * f + noise_std * nz.x, v[k].y * f + noise_std * nz.y,
                             v[k].z * f + noise_std * nz.z, v[k].w * f + noise_std * nz.w);
    }
  }
  __syncthreads();
  if (w != 0) return;
  int u = inv[perm[p0]];  // segment of position p0
  int s_beg = seg_ptr[u], s_end = seg_ptr[u + 1];
  float4 acc[MAXV4];
#pragma unroll
  for (int k = 0; k < MAXV4; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < SC; ++j) {
    const int pp = p0 + j;
    if (pp < p1) {
#pragma unroll
      for (int k = 0; k < MAXV4; ++k) {
        const float4 t = ls[j][lane + 64 * k];
        acc[k].x += t.x; acc[k].y += t.y; acc[k].z += t.z; acc[k].w += t.w;
      }
      if (pp + 1 == s_end || pp + 1 == p1) {  // flush the run of segment u
        float4* dst;
        if (s_beg >= p0 && s_end <= p1) dst = out + (size_t)u * D4;
        else dst = scratch + ((size_t)c * 2 + (s_beg < p0 ? 0 : 1)) * D4;
#pragma unroll
        for (int k = 0; k < MAXV4; ++k) {
          const int d = lane + 64 * k;
          if (d < D4) dst[d] = acc[k];
          acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (pp + 1 == s_end && pp + 1 < p1) {
          ++u;
          s_beg = s_end;
          s_end = seg_ptr[u + 1];
        }
      }
    }
  }
}

int g_segsum_ldp_block = 1;  // 1: the block-per-chunk LDP pass (default); 0: one wave per chunk (A/B)
// the block-per-chunk form for the plain sum too (default): steady 0.4406 / 0.4431 vs 0.4430 /
// 0.4433 ms (A/B/A/B, config 2, profiles/r5_ab_segsum_plain_block.jsonl) -- neutral to slightly
// better, 29 instead of 161 VGPRs
int g_segsum_plain_block = 1;
int g_segsum_variant = 2;  // 2: chunked, float4 rows (default); 1: chunked, scalar; 0: one block per output row
constexpr int SCH = 16;    // chunk length (8-occurrence chunks measured neutral, r3_ab_segsum_ua.txt)

}  // namespace

extern "C" void fr_segsum_set_variant(int v) { g_segsum_variant = v; }
extern "C" void fr_segsum_set_ldp_block(int v) {  // bit 0: the LDP pass, bit 1: the plain pass (default 3)
  g_segsum_ldp_block = v & 1;
  g_segsum_plain_block = (v >> 1) & 1;
}
extern "C" int fr_segsum_chunks(int R) { return (R + SCH - 1) / SCH; }

extern "C" int fr_ldp_rows(const float* rows, float* out, int R, int D, float clip, float noise_std,
                           unsigned long long seed, unsigned long long offset, hipStream_t s,
                           const unsigned long long* dev_off) {
  if (D > 64 * MAXV) return 1;
  if (R == 0) return 0;
  hipLaunchKernelGGL(ldp_rows_kernel, dim3((R + 3) / 4), dim3(256), 0, s, rows, out, R, D, clip, noise_std, seed,
                     offset, dev_off);
  return 0;
}

// scratch: fr_segsum_chunks(R) * 2 * D floats (chunked form); R = total occurrences = seg_ptr[U]
// Rows of empty segments: the chunked form writes them as zeros (its fix pass); the
// block-per-row form needs zero_empty = 1 to clear the output first.
// clip + noise fused into the float4 chunk pass (one launch fewer, no clipped copy of the rows);
// returns 1 when the shape / alignment does not take the fused form (the caller runs the two passes)
extern "C" int fr_segment_sum_rows_ldp(const float* rows, const int* perm, const int* seg_ptr, const int* inv,
                                       float* out, int U, int D, int R, float* scratch, float clip, float noise_std,
                                       unsigned long long seed, unsigned long long offset,
                                       const unsigned long long* dev_off, hipStream_t s) {
  if (U == 0) return 0;
  if (g_segsum_variant != 2 || scratch == nullptr || inv == nullptr || R <= 0 || D % 4 != 0 || D > 256 * MAXV4 ||
      (((uintptr_t)rows | (uintptr_t)out | (uintptr_t)scratch) & 15) != 0 || (D / 4) > 65535)
    return 1;
  const int nch = (R + SCH - 1) / SCH;
  if (g_segsum_ldp_block)
    hipLaunchKernelGGL((segsum_chunk4_ldp_kernel<SCH>), dim3(nch), dim3(256), 0, s, (const float4*)rows, perm, seg_ptr,
                       inv, (float4*)out, (float4*)scratch, U, R, D / 4, clip, noise_std, seed, offset, dev_off);
  else
    hipLaunchKernelGGL((segsum_chunk4_kernel<SCH, true>), dim3((nch + 3) / 4), dim3(256), 0, s, (const float4*)rows,
                       perm, seg_ptr, inv, (float4*)out, (float4*)scratch, U, R, D / 4, clip, noise_std, seed, offset,
                       dev_off);
  hipLaunchKernelGGL(segsum_fix_kernel<SCH>, dim3(U), dim3(256), 0, s, seg_ptr, out, scratch, U, D);
  return 0;
}

extern "C" int fr_segment_sum_rows(const float* rows, const int* perm, const int* seg_ptr, const int* inv, float* out,
                                   int U, int D, int R, float* scratch, hipStream_t s, int zero_empty) {
  if (D > 64 * MAXV) return 1;
  if (U == 0) return 0;
  if (g_segsum_variant == 2 && scratch != nullptr && inv != nullptr && R > 0 && D % 4 == 0 && D <= 256 * MAXV4 &&
      (((uintptr_t)rows | (uintptr_t)out | (uintptr_t)scratch) & 15) == 0) {
    const int nch = (R + SCH - 1) / SCH;
    if (g_segsum_plain_block)
      hipLaunchKernelGGL((segsum_chunk4_ldp_kernel<SCH, false>), dim3(nch), dim3(256), 0, s, (const float4*)rows, perm,
                         seg_ptr, inv, (float4*)out, (float4*)scratch, U, R, D / 4, 0.f, 0.f, 0ull, 0ull,
                         (const unsigned long long*)nullptr);
    else
      hipLaunchKernelGGL((segsum_chunk4_kernel<SCH, false>), dim3((nch + 3) / 4), dim3(256), 0, s, (const float4*)rows,
                         perm, seg_ptr, inv, (float4*)out, (float4*)scratch, U, R, D / 4, 0.f, 0.f, 0ull, 0ull,
                         (const unsigned long long*)nullptr);
    hipLaunchKernelGGL(segsum_fix_kernel<SCH>, dim3(U), dim3(256), 0, s, seg_ptr, out, scratch, U, D);
    return 0;
  }
  if (g_segsum_variant >= 1 && scratch != nullptr && inv != nullptr && R > 0) {
    const int nch = (R + SCH - 1) / SCH;
    hipLaunchKernelGGL(segsum_chunk_kernel<SCH>, dim3((nch + 3) / 4), dim3(256), 0, s, rows, perm, seg_ptr, inv, out,
                       scratch, U, R, D);
    hipLaunchKernelGGL(segsum_fix_kernel<SCH>, dim3(U), dim3(256), 0, s, seg_ptr, out, scratch, U, D);
    return 0;
  }
  if (zero_empty) (void)hipMemsetAsync(out, 0, (size_t)U * D * sizeof(float), s);
  hipLaunchKernelGGL(segsum_kernel, dim3(U), dim3(1024), 0, s, rows, perm, seg_ptr, out, U, D);
  return 0;
}
