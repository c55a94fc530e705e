// On-device batch builder: news-id de-duplication for one training step.
//
// The reference encodes every candidate/history occurrence separately (model.py:41-61;
// E8: 39 unique titles out of 324 encoded).  This kernel turns the R = B*(C+H) occurrence
// ids of a batch into
//   uniq[U]      sorted unique news ids        -> the only titles the backbone encodes
//   inv[R]       occurrence -> row of uniq     -> gather of news vectors
//   perm[R]      occurrences grouped by row    -> deterministic per-news gradient sums
//   seg_ptr[U+1] segment offsets into perm     (replaces the host dict of client.py:26-48)
// in ONE workgroup: a bitonic sort of (id << 32 | occurrence) keys in LDS (stable by
// construction), then a block-wide scan of the "new id" flags.  R <= 8192 (64 KB of keys);
// larger batches take the sort-based torch path on the host side of the binding.
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int MAXR = 8192;
constexpr int NT = 1024;

// KeyT = uint32 (ids < 2^19, R <= 8192: key = id << 13 | occurrence) or uint64 (id << 32 | i).
// The 32-bit form halves the LDS image (32 KB): a step's dedup runs on the lookahead stream
// beside the step's kernels, and a 64 KB block kept the weight-gradient GEMM's 96 KB block
// off its CU (a one-wave grid then waits for that CU: 68 -> 120 us).
template <typename KeyT, int SHIFT>
__global__ __launch_bounds__(NT) void dedup_kernel(const int* __restrict__ ids, int R, int P, int* __restrict__ uniq,
                                                   int* __restrict__ inv, int* __restrict__ perm,
                                                   int* __restrict__ seg_ptr, int* __restrict__ u_count) {
  __shared__ KeyT key[MAXR];
  __shared__ int part[NT];
  __shared__ int wsum[NT / 64];
  const int tid = threadIdx.x;
  for (int i = tid; i < P; i += NT)
    key[i] = i < R ? (KeyT)((((KeyT)(unsigned)ids[i]) << SHIFT) | (KeyT)(unsigned)i) : (KeyT)~(KeyT)0;
  __syncthreads();
  // bitonic sort, ascending
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const KeyT a = key[i], b = key[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            key[i] = b;
            key[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // flags + block scan: thread handles a contiguous run of E elements
  const int E = (R + NT - 1) / NT;
  const int b0 = tid * E;
  int cnt = 0;
  for (int e = 0; e < E; ++e) {
    const int i = b0 + e;
    if (i < R) cnt += (i == 0 || (key[i] >> SHIFT) != (key[i - 1] >> SHIFT)) ? 1 : 0;
  }
  // inclusive scan of cnt over the block
  const int lane = tid & 63, w = tid >> 6;
  int x = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (w == 0) {
    int s = lane < NT / 64 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (lane < NT / 64) wsum[lane] = s;
  }
  __syncthreads();
  int run = x - cnt + (w > 0 ? wsum[w - 1] : 0);  // exclusive prefix of this thread's run
  for (int e = 0; e < E; ++e) {
    const int i = b0 + e;
    if (i >= R) break;
    const int id = (int)(key[i] >> SHIFT);
    const int r = (int)(key[i] & (KeyT)(((KeyT)1 << SHIFT) - 1));
    const bool f = (i == 0 || (key[i] >> SHIFT) != (key[i - 1] >> SHIFT));
    if (f) {
      uniq[run] = id;
      seg_ptr[run] = i;
      ++run;
    }
    perm[i] = r;
    inv[r] = run - 1;
  }
  if (tid == NT - 1) {
    const int U = wsum[NT / 64 - 1];
    *u_count = U;
    seg_ptr[U] = R;
  }
  (void)part;
}

// ---------------------------------------------------------------------------------------
// Register form (the default).  The kernel above runs all log2(P)(log2(P)+1)/2 compare-exchange
// stages through LDS with a barrier each: 78 barriered stages at P = 4096, 56 us per step on the
// lookahead stream.  Here thread t holds elements t + NT e (e < E) in registers, so the partner
// i ^ j of a stage is
//   j <  64:  lane t ^ j of the same wave, same slot  -> one shuffle, no barrier (57 of 78 stages)
//   j >= NT:  the same thread, slot e ^ (j / NT)       -> registers (3 stages)
//   else:     another wave                              -> LDS, double-buffered: one barrier
// P is padded to at least NT (every thread holds E >= 1 elements; pads sort last).
// ---------------------------------------------------------------------------------------
template <typename KeyT>
__device__ __forceinline__ KeyT shfl_xor_key(KeyT v, int j) {
  if constexpr (sizeof(KeyT) == 4) {
    return (KeyT)__shfl_xor((int)v, j, 64);
  } else {
    const int lo = __shfl_xor((int)(unsigned)(v & 0xffffffffull), j, 64);
    const int hi = __shfl_xor((int)(unsigned)(v >> 32), j, 64);
    return ((KeyT)(unsigned)hi << 32) | (KeyT)(unsigned)lo;
  }
}

template <typename KeyT, int SHIFT, int E>
__global__ __launch_bounds__(NT) void dedup2_kernel(const int* __restrict__ ids, int R, int* __restrict__ uniq,
                                                    int* __restrict__ inv, int* __restrict__ perm,
                                                    int* __restrict__ seg_ptr, int* __restrict__ u_count) {
  constexpr int P = NT * E;
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  KeyT* buf0 = (KeyT*)dsm;
  KeyT* buf1 = buf0 + P;
  __shared__ int wsum[NT / 64];
  const int tid = threadIdx.x;
  KeyT k_[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = tid + NT * e;
    k_[e] = i < R ? (KeyT)((((KeyT)(unsigned)ids[i]) << SHIFT) | (KeyT)(unsigned)i) : (KeyT)~(KeyT)0;
  }
  int pb = 0;  // LDS buffer parity
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= NT) {
        // slot partner e ^ js with js a compile-time constant per branch (no dynamic register index)
#pragma unroll
        for (int js = 1; js < E; js <<= 1) {
          if (j == NT * js) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
              const int ep = e ^ js;
              if (ep > e) {
                const int i = tid + NT * e;
                const bool up = (i & k) == 0;
                const KeyT a = k_[e], b = k_[ep];
                const bool sw = (a > b) == up;
                k_[e] = sw ? b : a;
                k_[ep] = sw ? a : b;
              }
            }
          }
        }
      } else if (j >= 64) {
        KeyT* bs = pb ? buf1 : buf0;
        pb ^= 1;
#pragma unroll
        for (int e = 0; e < E; ++e) bs[tid + NT * e] = k_[e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = tid + NT * e;
          const KeyT b = bs[i ^ j];
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          k_[e] = keep_min ? (b < k_[e] ? b : k_[e]) : (b > k_[e] ? b : k_[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = tid + NT * e;
          const KeyT b = shfl_xor_key(k_[e], j);
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          k_[e] = keep_min ? (b < k_[e] ? b : k_[e]) : (b > k_[e] ? b : k_[e]);
        }
      }
    }
  }
  KeyT* key = pb ? buf1 : buf0;  // a buffer no thread can still be reading (the last LDS stage used the other)
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; ++e) key[tid + NT * e] = k_[e];
  __syncthreads();
  // flags + block scan over contiguous runs, as dedup_kernel
  const int EC = (R + NT - 1) / NT;
  const int b0 = tid * EC;
  int cnt = 0;
  for (int e = 0; e < EC; ++e) {
    const int i = b0 + e;
    if (i < R) cnt += (i == 0 || (key[i] >> SHIFT) != (key[i - 1] >> SHIFT)) ? 1 : 0;
  }
  const int lane = tid & 63, w = tid >> 6;
  int x = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (w == 0) {
    int s = lane < NT / 64 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (lane < NT / 64) wsum[lane] = s;
  }
  __syncthreads();
  int run = x - cnt + (w > 0 ? wsum[w - 1] : 0);
  for (int e = 0; e < EC; ++e) {
    const int i = b0 + e;
    if (i >= R) break;
    const int id = (int)(key[i] >> SHIFT);
    const int r = (int)(key[i] & (KeyT)(((KeyT)1 << SHIFT) - 1));
    const bool f = (i == 0 || (key[i] >> SHIFT) != (key[i - 1] >> SHIFT));
    if (f) {
      uniq[run] = id;
      seg_ptr[run] = i;
      ++run;
    }
    perm[i] = r;
    inv[r] = run - 1;
  }
  if (tid == NT - 1) {
    const int U = wsum[NT / 64 - 1];
    *u_count = U;
    seg_ptr[U] = R;
  }
}

// the register-bitonic form (dedup2) where its key image fits 64 KB of LDS, else the LDS form

}  // namespace

// ---------------------------------------------------------------------------------------
// Batch sampler (reference TrainDataset.__getitem__, dataset.py:69-86, with newsample
// dataset.py:10-14): one wave per impression of the batch.
//   cand[b] = [pos, 4 negatives]   n >= 4: uniformly random ordered 4-subset (random.sample)
//                                  n <  4: the negatives in order, then <unk> (id 0)
//   his[b]  = the last min(len, H) history ids, zero padded (truncate) / first H (compat)
// Randomness: Philox(seed, offset = step) with counter (impression, draw): reproducible and
// independent of the launch geometry.
// valid = 1: the validation batch of client.py:158-165 -- cand[b] = [pos] + the LAST
// min(n, npr) negatives (negs[-4:]), zero padded; no randomness (data/sampler.valid_candidates).
__global__ __launch_bounds__(256) void sample_kernel(const int* __restrict__ rows, const int* __restrict__ pos,
                                                     const long long* __restrict__ neg_ptr, const int* __restrict__ negs,
                                                     const long long* __restrict__ his_ptr, const int* __restrict__ his,
                                                     int* __restrict__ cand, int* __restrict__ hout, int B, int npr,
                                                     int H, int truncate, unsigned long long seed,
                                                     unsigned long long offset, int valid) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int r = rows[b];
  const long long n0 = neg_ptr[r], n = neg_ptr[r + 1] - n0;
  int* cb = cand + (size_t)b * (npr + 1);
  if (valid) {
    if (lane == 0) cb[0] = pos[r];
    const long long take = n < npr ? n : npr;
    if (lane < npr) cb[1 + lane] = lane < take ? negs[n0 + n - take + lane] : 0;
  } else if (lane == 0) {
    cb[0] = pos[r];
    if (n < npr) {
      for (int j = 0; j < npr; ++j) cb[1 + j] = j < n ? negs[n0 + j] : 0;
    } else {
      int pick[16];
      int got = 0;
      unsigned long long ctr = (unsigned long long)r << 20;
      while (got < npr) {
        const uint4 x = Philox::gen(seed, offset, ctr++);
        const uint32_t u[4] = {x.x, x.y, x.z, x.w};
        for (int t = 0; t < 4 && got < npr; ++t) {
          const int idx = (int)(((unsigned long long)u[t] * (unsigned long long)n) >> 32);
          bool dup = false;
          for (int q = 0; q < got; ++q) dup |= pick[q] == idx;
          if (!dup) pick[got++] = idx;
        }
      }
      for (int j = 0; j < npr; ++j) cb[1 + j] = negs[n0 + pick[j]];
    }
  }
  const long long h0 = his_ptr[r], hl = his_ptr[r + 1] - h0;
  const long long take = hl < H ? hl : H;
  const long long start = truncate ? h0 + hl - take : h0;
  int* hb = hout + (size_t)b * H;
  for (int j = lane; j < H; j += 64) hb[j] = j < take ? his[start + j] : 0;
}

extern "C" int fr_sample_batch(const int* rows, const int* pos, const long long* neg_ptr, const int* negs,
                               const long long* his_ptr, const int* his, int* cand, int* hout, int B, int npr, int H,
                               int truncate, unsigned long long seed, unsigned long long offset, int valid,
                               hipStream_t s) {
  if (npr > 16 || B < 0) return 1;
  if (B == 0) return 0;
  hipLaunchKernelGGL(sample_kernel, dim3((B + 3) / 4), dim3(256), 0, s, rows, pos, neg_ptr, negs, his_ptr, his, cand,
                     hout, B, npr, H, truncate, seed, offset, valid);
  return 0;
}

extern "C" int fr_dedup(const int* ids, int R, int num_news, int* uniq, int* inv, int* perm, int* seg_ptr,
                        int* u_count, hipStream_t s) {
  if (R > MAXR || R < 1) return 1;
  int P = 1;
  while (P < R) P <<= 1;
  const bool narrow = num_news > 0 && num_news <= (1 << 19);
  const int E = P <= NT ? 1 : P / NT;
  const size_t lds = 2 * (size_t)NT * E * (narrow ? 4 : 8);  // two key buffers
  if (lds <= 65536) {
#define DEDUP2(KT, SH, EE)                                                                                    \
  hipLaunchKernelGGL((dedup2_kernel<KT, SH, EE>), dim3(1), dim3(NT), lds, s, ids, R, uniq, inv, perm, seg_ptr, \
                     u_count)
#define DEDUP2_E(KT, SH)        \
  do {                          \
    if (E == 1) DEDUP2(KT, SH, 1); \
    else if (E == 2) DEDUP2(KT, SH, 2); \
    else if (E == 4) DEDUP2(KT, SH, 4); \
    else DEDUP2(KT, SH, 8);     \
  } while (0)
    if (narrow) DEDUP2_E(unsigned, 13);
    else DEDUP2_E(unsigned long long, 32);
#undef DEDUP2_E
#undef DEDUP2
    return 0;
  }
  if (num_news > 0 && num_news <= (1 << 19))  // 13 bits of occurrence index (MAXR = 8192)
    hipLaunchKernelGGL((dedup_kernel<unsigned, 13>), dim3(1), dim3(NT), 0, s, ids, R, P, uniq, inv, perm, seg_ptr,
                       u_count);
  else
    hipLaunchKernelGGL((dedup_kernel<unsigned long long, 32>), dim3(1), dim3(NT), 0, s, ids, R, P, uniq, inv, perm,
                       seg_ptr, u_count);
  return 0;
}

// ---------------------------------------------------------------------------------------
// Several small copies in one launch (the step graph's static inputs: candidates, history,
// the padded unique list, occurrence maps, padded segment pointers): dst[i] = src[i] for
// i < n_src, = fill for n_src <= i < n_dst, in 4-byte words.  One launch instead of ~8
// copy / fill kernels, which cost ~5 us each as graph nodes.
namespace {
constexpr int MC_MAX = 8;
struct MultiCopy {
  const int* src[MC_MAX];
  int* dst[MC_MAX];
  long nsrc[MC_MAX], ndst[MC_MAX], base[MC_MAX + 1];
  int fill[MC_MAX];
  int n;
};

__global__ __launch_bounds__(256) void multi_copy_kernel(const MultiCopy mc) {
  const long total = mc.base[mc.n];
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    int s = 0;
#pragma unroll
    for (int i = 1; i < MC_MAX; ++i)
      if (i < mc.n && e >= mc.base[i]) s = i;
    const long j = e - mc.base[s];
    mc.dst[s][j] = j < mc.nsrc[s] ? mc.src[s][j] : mc.fill[s];
  }
}
}  // namespace

extern "C" int fr_multi_copy(const int* const* src, int* const* dst, const long* nsrc, const long* ndst,
                             const int* fill, int n, hipStream_t s) {
  if (n < 1 || n > MC_MAX) return 1;
  MultiCopy mc{};
  mc.n = n;
  mc.base[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (nsrc[i] > ndst[i] || nsrc[i] < 0) return 2;
    mc.src[i] = src[i];
    mc.dst[i] = dst[i];
    mc.nsrc[i] = nsrc[i];
    mc.ndst[i] = ndst[i];
    mc.fill[i] = fill[i];
    mc.base[i + 1] = mc.base[i] + ndst[i];
  }
  const long total = mc.base[n];
  if (total == 0) return 0;
  long blocks = (total + 255) / 256;
  blocks = blocks > 1024 ? 1024 : blocks;
  hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, mc);
  return 0;
}
