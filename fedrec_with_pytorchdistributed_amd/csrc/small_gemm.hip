// Small GEMMs on MFMA for the user encoder and the text head's FC (SURVEY §2.3 K07, K10, K14;
// round-1 these were hipBLASLt fp32 calls plus torch glue).
//
//   C[m, n] = act(alpha * sum_k A(m, k) * B(n, k) + bias[n])  (+ C[m, n] when accumulating)
//
// Shapes are the user side's: M = B*H = 3200 history rows (or U titles), N / K in {200, 400,
// 768, 1200}, none of them multiples of a power-of-two tiling -- every edge is masked.
// Operands are fp32 or bf16 per operand (a_bf16 / b_bf16); fp32 ones are converted to bf16 on
// their way into LDS, so an operand its producer already wrote in bf16 gives the bitwise same
// product at half the bytes.  v_mfma_f32_16x16x32_bf16, fp32 accumulate.  Layouts:
//   A: a_mode 0 = row-major [M, K] (optionally with a row gather m -> gidx[m] and a Philox
//      dropout on the gathered elements, index m * drop_ld + k), a_mode 1 = stored transposed
//      [K, M] (weight gradients dW = dY^T X);
//   B: b_mode 0 = [N, K] (nn.Linear weight: y = x W^T), b_mode 1 = [K, N] (dgrad dx = dy W;
//      or, with gidx / dropout, a gathered dropped-out input for dW = dY^T X').
//   act: 0 none, 1 tanh.  drop_on: 0 none, 1 A elements (m, k), 2 B elements (k, n) of a K-major
//      B (both fp32 operands only), 3 output elements (m, n) -- the input dropout's backward
//      fused into the dgrad epilogue.  gather_on: 0 none, 1 A rows (a_mode 0), 2 B rows (b_mode 1).
//
// Tiles: TM x TN x 64 with TM = 32 FM, TN = 32 FN (FM, FN in {2, 4}: 64 / 128), 256 threads =
// 4 waves in 2 x 2, each wave (TM/2) x (TN/2) = FM x FN MFMA tiles.  The K loop keeps the next
// k-tile's global loads in flight in registers (raw bits, converted when stored to LDS) while
// the MFMAs consume the current one.  These GEMMs are L2-bandwidth bound at 64 x 64 (each
// operand re-read once per tile of the other dimension: the Q|K|V projection moved ~235 MB
// through L2 for 3 GFLOP), so the host picks the biggest tile that still fills the chip.
// Several independent GEMMs run in ONE launch (GemmBatch: the weight gradients of one
// backward, ...): the XCD-remapped blockIdx walks the concatenated tile lists, consecutive
// tiles (the column tiles of one row panel, the splits of one tile) on one XCD's L2.  Long
// reductions with few output tiles split K over workgroups into fp32 partials that a second
// kernel sums in split order -- deterministic, no atomics.
// Stored-transposed operands (mode 1) of the 64 x 64 tiles stay k-major in LDS (TRI images,
// see tsw) and come back as MFMA fragments through ds_read_b64_tr_b16; the k-contiguous image
// needed 16 scalar 2-byte stores per chunk (LDS bank conflicts at 0.5-0.66 of the LDS busy
// cycles).  A register queue two k-tiles deep (SG_NQ = 2) measured slower on every launch of
// the config-2 step, even the ones with fewer tiles than CUs (profiles/r3_ab_sg_nq2.txt).
#include "common.h"
#include "gemm_batch.h"

#include <stdlib.h>
#include <string.h>

namespace {

constexpr int TK = 64, LDT = TK + 8;  // LDS row stride 72 bf16 = 144 B
using fr_sg::GemmBatch;
using fr_sg::GemmDesc;
using fr_sg::MAXG;
#ifndef SG_NQ
#define SG_NQ 1
#endif



// 16 consecutive elements -> raw register bits (fp32: 16 words; bf16: 8 words, 2 per word)
__device__ __forceinline__ void load16_f32(const float* __restrict__ p, int valid, uint32_t (&v)[16]) {
  if (valid == 16 && ((uintptr_t)p & 15) == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 f = *(const uint4*)(p + 4 * j);
      v[4 * j] = f.x; v[4 * j + 1] = f.y; v[4 * j + 2] = f.z; v[4 * j + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = j < valid ? __float_as_uint(p[j]) : 0u;
  }
}
__device__ __forceinline__ void load16_bf16(const unsigned short* __restrict__ p, int valid, uint32_t (&v)[16]) {
  if (valid == 16 && ((uintptr_t)p & 15) == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint4 f = *(const uint4*)(p + 8 * j);
      v[4 * j] = f.x; v[4 * j + 1] = f.y; v[4 * j + 2] = f.z; v[4 * j + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t lo = 2 * j < valid ? p[2 * j] : 0u, hi = 2 * j + 1 < valid ? p[2 * j + 1] : 0u;
      v[j] = lo | (hi << 16);
    }
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

// chunk c of a TR x 64 operand tile: mode 0 ([R, K] row-major) -> (row c / 4, 16 k from
// 16 (c % 4)); mode 1 (stored [K, R]) -> (k c / (TR/16), 16 rows from 16 (c % (TR/16)))
template <int TR>
__device__ __forceinline__ void load_raw(const GemmDesc& g, bool isA, int r0, int k0, int kend, int tid,
                                         uint32_t (&raw)[TR / 64][16]) {
  const int mode = isA ? g.a_mode : g.b_mode;
  const bool h = isA ? g.a_bf16 : g.b_bf16;
  const int ld = isA ? g.lda : g.ldb;
  const int R = isA ? g.M : g.N;
#pragma unroll
  for (int i = 0; i < TR / 64; ++i) {
    const int c = tid + 256 * i;
    const void* base = isA ? g.A : g.B;
    size_t src;
    int valid;
    if (mode == 0) {
      const int r = c >> 2, kk = (c & 3) * 16;
      const int rr = r0 + r, k = k0 + kk;
      const bool rok = rr < R;
      const int row = rok ? ((isA && g.gather_on == 1) ? g.gidx[rr] : rr) : 0;
      src = (size_t)row * ld + k;
      valid = rok ? min(16, kend - k) : 0;
    } else {
      constexpr int CPR = TR / 16;
      const int k = c / CPR, rr16 = (c % CPR) * 16;
      const int kg = k0 + k;
      const bool kok = kg < kend;
      size_t row = kok ? (size_t)((!isA && g.gather_on == 2) ? g.gidx[kg] : kg) : 0;
      if (!isA && g.kseg > 0 && kok) {  // one [K, N] operand stored as up to three row blocks
        const int seg = kg / g.kseg;
        base = seg == 0 ? g.B : (seg == 1 ? g.B2 : g.B3);
        row = kg - seg * g.kseg;
      }
      src = row * ld + r0 + rr16;
      valid = kok ? min(16, R - (r0 + rr16)) : 0;
    }
    if (h)
      load16_bf16((const unsigned short*)base + src, valid, raw[i]);
    else
      load16_f32((const float*)base + src, valid, raw[i]);
  }
}

// The same tile with no data-dependent branches around loads (FAST launches: every contiguous extent a
// multiple of 8 elements, 16-byte aligned rows): each 8-element half of a chunk is one
// unconditional load from its address or -- when it lies outside the operand -- from the
// operand's first row, and `vm` records which halves are real; the zeroing select waits until
// the chunk is stored to LDS, after the MFMAs.  (With per-lane branches around the loads the
// compiler joins the paths right after them and waits for the data there: every k-tile's
// loads became synchronous -- the 128-row tiles measured 2-4x SLOWER than 64-row ones.)
// (1) offsets: every chunk's two half byte offsets into its operand -- any row-gather index
// load happens here, before the first data load is issued, so its wait drains nothing else;
// a half outside the operand gets an offset past the descriptor's range, which the buffer
// unit answers with zeros; (2) the data loads, buffer_load_dwordx4 through a per-operand
// descriptor built from wave-uniform values.  (Plain pointer loads here compile to FLAT loads
// -- the operand pointers come out of the kernel-argument struct as generic pointers -- and a
// flat load also counts in lgkmcnt: the LDS-read wait before the MFMAs then waited for the
// next tile's prefetch as well, serialising the pipeline.)
constexpr uint32_t OOB = 0x80000000u;  // past num_records: the load returns zeros

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), 0, 0x7FFFFFF0, 0x00020000);
}

template <int TR, bool H>
__device__ __forceinline__ void chunk_offs(const GemmDesc& g, bool isA, int r0, int k0, int kend, int tid,
                                           uint32_t (&ol)[TR / 64], uint32_t (&oh)[TR / 64]) {
  const int mode = isA ? g.a_mode : g.b_mode;
  constexpr uint32_t ES = H ? 2 : 4;
  const int ld = isA ? g.lda : g.ldb;
  const int R = isA ? g.M : g.N;
#pragma unroll
  for (int i = 0; i < TR / 64; ++i) {
    const int c = tid + 256 * i;
    uint32_t src;
    int valid;
    if (mode == 0) {
      const int r = c >> 2, kk = (c & 3) * 16;
      const int rr = r0 + r, k = k0 + kk;
      const bool rok = rr < R;
      const int row = rok ? ((isA && g.gather_on == 1) ? g.gidx[rr] : rr) : 0;
      src = (uint32_t)row * ld + k;
      valid = rok ? kend - k : 0;
    } else {
      constexpr int CPR = TR / 16;
      const int k = c / CPR, rr16 = (c % CPR) * 16;
      const int kg = k0 + k;
      const bool kok = kg < kend;
      const uint32_t row = kok ? (uint32_t)((!isA && g.gather_on == 2) ? g.gidx[kg] : kg) : 0u;
      src = row * ld + r0 + rr16;
      valid = kok ? R - (r0 + rr16) : 0;
    }
    ol[i] = valid >= 8 ? src * ES : OOB;
    oh[i] = valid >= 16 ? src * ES + 8 * ES : OOB;
  }
}

template <int TR, bool H>
__device__ __forceinline__ void issue_loads(__amdgpu_buffer_rsrc_t rs, const uint32_t (&ol)[TR / 64],
                                            const uint32_t (&oh)[TR / 64], uint32_t (&raw)[TR / 64][16]) {
#pragma unroll
  for (int i = 0; i < TR / 64; ++i) {
    if (H) {  // 8 bf16 per half: one 16-byte load each
      const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, ol[i], 0, 0);
      const auto b = __builtin_amdgcn_raw_buffer_load_b128(rs, oh[i], 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        raw[i][q] = a[q];
        raw[i][4 + q] = b[q];
      }
    } else {  // 8 floats per half: two
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, ol[i] + 16 * j, 0, 0);
        const auto b = __builtin_amdgcn_raw_buffer_load_b128(rs, oh[i] + 16 * j, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          raw[i][4 * j + q] = a[q];
          raw[i][8 + 4 * j + q] = b[q];
        }
      }
    }
  }
}

// raw chunk -> 16 bf16 (fp32 operands: dropout-scaled first when it applies)
__device__ __forceinline__ void to_bf16x16(const uint32_t (&raw)[16], bool h, bool drop, unsigned long long e,
                                           const GemmDesc& g, unsigned long long off, bf16x8 (&o)[2]) {
  if (h) {
    o[0] = __builtin_bit_cast(bf16x8, uint4{raw[0], raw[1], raw[2], raw[3]});
    o[1] = __builtin_bit_cast(bf16x8, uint4{raw[4], raw[5], raw[6], raw[7]});
    return;
  }
  float v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = __uint_as_float(raw[j]);
  if (drop) apply_drop16(v, e, g, off);
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[hh][j] = f2bf(v[8 * hh + j]);
}

// TRI (transposed-image) form of a stored-transposed operand (mode 1, TR = 64): the tile stays
// as it sits in memory, [64 k rows][64 cols] bf16 (128-B rows), 16-B chunk c of row k at
// c ^ tsw(k), written with two ds_write_b128 per chunk of 16 columns instead of 16 scalar
// 2-byte stores into the k-contiguous image; the MFMA fragments (8 consecutive k of one
// column) come back with two ds_read_b64_tr_b16.  tsw spreads the 4 rows x 2 chunks a
// 16-lane group reads -- rows {8g + q}, g = lane / 16 -- over distinct 8-bank quarters
__device__ __forceinline__ int tsw(int k) { return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1; }

template <int TR, bool TRI = false>
__device__ __forceinline__ void store_lds(const GemmDesc& g, bool isA, int r0, int k0, int tid,
                                          const uint32_t (&raw)[TR / 64][16], unsigned long long off,
                                          bf16 (*S)[LDT], bool h) {
  const int mode = isA ? g.a_mode : g.b_mode;
  if (TRI && TR == 64 && mode == 1) {  // block-uniform
    bf16* img = &S[0][0];
    const int k = tid >> 2, c0 = (tid & 3) * 2;  // 16 columns = chunks c0, c0 + 1 of row k
    bf16x8 o[2];
    to_bf16x16(raw[0], h, !isA && g.drop_on == 2, (unsigned long long)(k0 + k) * g.drop_ld + r0 + c0 * 8, g, off, o);
    *(bf16x8*)(img + k * 64 + ((c0 ^ tsw(k)) << 3)) = o[0];
    *(bf16x8*)(img + k * 64 + (((c0 + 1) ^ tsw(k)) << 3)) = o[1];
    return;
  }
#pragma unroll
  for (int i = 0; i < TR / 64; ++i) {
    const int c = tid + 256 * i;
    bf16x8 o[2];
    if (mode == 0) {
      const int r = c >> 2, kk = (c & 3) * 16;
      to_bf16x16(raw[i], h, isA && g.drop_on == 1, (unsigned long long)(r0 + r) * g.drop_ld + k0 + kk, g, off, o);
      *(bf16x8*)&S[r][kk] = o[0];
      *(bf16x8*)&S[r][kk + 8] = o[1];
    } else {
      constexpr int CPR = TR / 16;
      const int k = c / CPR, rr16 = (c % CPR) * 16;
      to_bf16x16(raw[i], h, !isA && g.drop_on == 2, (unsigned long long)(k0 + k) * g.drop_ld + r0 + rr16, g, off, o);
#pragma unroll
      for (int j = 0; j < 16; ++j) S[rr16 + j][k] = o[j >> 3][j & 7];
    }
  }
}

// MFMA operand fragment (8 consecutive k of column col0 + lane % 16, k from 8 (lane / 16)) of a
// TRI image: two transposed 8-byte reads of 4 rows each
__device__ __forceinline__ bf16x8 tri_frag(const bf16* img, int ks, int col0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  bf16x4 v[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const int r = ks + 8 * g + 4 * hf + q;
    const int c = (col0 >> 3) + (p >> 1);
    const bf16* a = img + r * 64 + ((c ^ tsw(r)) << 3) + (p & 1) * 4;
    v[hf] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a)));
  }
  return bf16x8{v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
}

// dropout-backward scale of output element (m, n) (drop_on 3): element m * drop_ld + n of the
// dropped input
__device__ __forceinline__ float drop3(const GemmDesc& g, unsigned long long off, int m, int n) {
  const unsigned long long e = (unsigned long long)m * g.drop_ld + n;
  const uint4 x = Philox::gen(g.seed, off, e >> 2);
  return drop_scale(u4_get(x, (int)(e & 3)), g.pdrop, 1.0f / (1.0f - g.pdrop));
}

// FAST: branch-free operand loads with the operand dtypes fixed per launch (AH / BH: A / B
// bf16); generic: any alignment, per-desc dtypes, the dropout prologues
// tile index tg of the launch -> (desc, split, m0, n0); XCD-aware order: blocks bid = x, x + 8,
// ... (one XCD) take consecutive tiles (the column tiles of one row panel share its A rows)
__device__ __forceinline__ int tile_of_block(const GemmBatch& batch, int& gi) {
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, qq = nwg >> 3, rmd = nwg & 7;
  const int tg = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (bid >> 3);
  gi = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < batch.n && tg >= batch.d[i].tile_base) gi = i;
  return tg - batch.d[gi].tile_base;
}

// DB: two LDS buffers -- step s stores its tile into buffer s % 2, issues the next loads and
// meets ONE barrier before its MFMAs (the single-buffer step needs a second barrier in front,
// so no wave overwrites a tile another wave still reads); buffer s % 2 was last read by step
// s - 2, which every wave finished before passing step s - 1's barrier.
template <int FM, int FN, bool FAST, bool AH, bool BH, bool TRI = false, bool DB = false>
__device__ __forceinline__ void gemm_tile(const GemmDesc& g, unsigned long long off, int t,
                                          bf16 (*As)[LDT], bf16 (*Bs)[LDT], bf16 (*As2)[LDT] = nullptr,
                                          bf16 (*Bs2)[LDT] = nullptr) {
  constexpr int TM = 32 * FM, TN = 32 * FN;
  const int split = t % g.splits;
  t /= g.splits;
  const int m0 = (t / g.tiles_n) * TM, n0 = (t % g.tiles_n) * TN;
  const int kbeg = split * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * (TM / 2), wn = (wave & 1) * (TN / 2);
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // NQ k-tiles of operand loads in flight, in registers (a rotating queue, statically indexed by
  // unrolling the k loop NQ times): these GEMMs are short (K = 200..1200: 4-19 k-tiles) and
  // latency-bound -- with one k-tile in flight each k-step waited out a global-load latency
  // behind its 8 MFMAs per wave (15 us for the 0.5 GFLOP att_fc1 GEMM, 7 k-steps)
  constexpr int NQ = SG_NQ;
  uint32_t ra[NQ][TM / 64][16], rb[NQ][TN / 64][16];
  __amdgpu_buffer_rsrc_t rsa, rsb;
  if (FAST) {
    rsa = rsrc_of(g.A);
    rsb = rsrc_of(g.B);
  }
  auto load = [&](int k, uint32_t (&qa)[TM / 64][16], uint32_t (&qb)[TN / 64][16]) {
    if (FAST) {
      uint32_t oal[TM / 64], oah[TM / 64], obl[TN / 64], obh[TN / 64];
      chunk_offs<TM, AH>(g, true, m0, k, kend, tid, oal, oah);
      chunk_offs<TN, BH>(g, false, n0, k, kend, tid, obl, obh);
      issue_loads<TM, AH>(rsa, oal, oah, qa);
      issue_loads<TN, BH>(rsb, obl, obh, qb);
    } else {
      load_raw<TM>(g, true, m0, k, kend, tid, qa);
      load_raw<TN>(g, false, n0, k, kend, tid, qb);
    }
  };
  // asum: the column-0 tiles of an a_mode-1 desc also sum the raw A values they stage (chunk
  // = 16 consecutive m of one k), per lane, then across lanes / waves after the loop
  const bool do_as = g.asum != nullptr && n0 == 0;
  const bool ah = FAST ? AH : (bool)g.a_bf16;
  float as_[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) as_[j] = 0.f;
  // one k-step: the queued tile into LDS, then its MFMAs; the slot is refilled with the tile NQ
  // steps ahead right after its registers were stored
  auto step = [&](int k0, uint32_t (&qa)[TM / 64][16], uint32_t (&qb)[TN / 64][16]) {
    const bool alt = DB && ((((k0 - kbeg) / TK) & 1) != 0);  // block-uniform
    bf16 (*const Ab)[LDT] = alt ? As2 : As;
    bf16 (*const Bb)[LDT] = alt ? Bs2 : Bs;
    if (!DB) __syncthreads();  // the previous tile's fragments are consumed
    if (do_as) {
#pragma unroll
      for (int i = 0; i < TM / 64; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          as_[j] += ah ? __uint_as_float((j & 1 ? qa[i][j >> 1] & 0xFFFF0000u : qa[i][j >> 1] << 16))
                       : __uint_as_float(qa[i][j]);
    }
    store_lds<TM, TRI>(g, true, m0, k0, tid, qa, off, Ab, FAST ? AH : (bool)g.a_bf16);
    store_lds<TN, TRI>(g, false, n0, k0, tid, qb, off, Bb, FAST ? BH : (bool)g.b_bf16);
    if (DB) {
      if (k0 + NQ * TK < kend) load(k0 + NQ * TK, qa, qb);
      __syncthreads();
    } else {
      __syncthreads();
      if (k0 + NQ * TK < kend) load(k0 + NQ * TK, qa, qb);  // overlaps this and the next NQ-1 steps
    }
#pragma unroll
    for (int ks = 0; ks < TK; ks += 32) {
      bf16x8 a[FM], b[FN];
      const bool ta = TRI && TM == 64 && g.a_mode == 1, tb = TRI && TN == 64 && g.b_mode == 1;  // block-uniform
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[i] = ta ? tri_frag(&Ab[0][0], ks, wm + i * 16, lane) : *(const bf16x8*)&Ab[wm + i * 16 + fr][ks + fq * 8];
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[j] = tb ? tri_frag(&Bb[0][0], ks, wn + j * 16, lane) : *(const bf16x8*)&Bb[wn + j * 16 + fr][ks + fq * 8];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
#pragma unroll
  for (int q = 0; q < NQ; ++q)
    if (kbeg + q * TK < kend) load(kbeg + q * TK, ra[q], rb[q]);
  for (int k0 = kbeg; k0 < kend; k0 += NQ * TK) {
    step(k0, ra[0], rb[0]);
    if constexpr (NQ > 1) {
      if (k0 + TK >= kend) break;
      step(k0 + TK, ra[1], rb[1]);
    }
    if constexpr (NQ > 2) {
      if (k0 + 2 * TK >= kend) break;
      step(k0 + 2 * TK, ra[2], rb[2]);
    }
  }
  if (do_as) {  // lanes of one m group (tid % CPR) hold the same 16 m: xor-shuffle, then waves in order
    constexpr int CPR = TM / 16;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) as_[j] += __shfl_xor(as_[j], o, 64);
    }
    __syncthreads();  // the LDS tiles are free: reuse As as [4 waves][TM] floats
    float* red = (float*)&As[0][0];
    if (lane < CPR) {
#pragma unroll
      for (int j = 0; j < 16; ++j) red[wave * TM + lane * 16 + j] = as_[j];
    }
    __syncthreads();
    if (tid < TM && m0 + tid < g.M) {
      const float v = (red[tid] + red[TM + tid]) + (red[2 * TM + tid] + red[3 * TM + tid]);
      if (g.splits > 1)
        g.AP[(size_t)split * g.M + m0 + tid] = v;
      else
        g.asum[m0 + tid] = v;
    }
  }
  // lane holds C[m = wm + 16 i + 4 fq + r][n = wn + 16 j + fr]; every loop fully unrolled
  // (static accumulator indices: the earlier form, with the split-K store inside the loop
  // nest, stayed rolled at 128-row tiles and kept the accumulators in scratch)
  const bool part = g.splits > 1;
  float* const dst = part ? g.P + (size_t)split * g.M * g.N : g.C;
  const int ldd = part ? g.N : g.ldc;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn + j * 16 + fr;
    const bool nok = n < g.N;
    const float bn = (!part && nok && g.bias) ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + fq * 4 + r;
        if (!nok || m >= g.M) continue;
        float v = acc[i][j][r];
        float* c = dst + (size_t)m * ldd + n;
        if (!part) {  // raw partial otherwise: alpha / bias / act / accumulate in splitk_reduce_kernel
          v = g.alpha * v + bn;
          if (g.act == 1) v = tanhf(v);
          if (g.drop_on == 3) v *= drop3(g, off, m, n);
          if (g.accumulate) v += *c;
        }
        *c = v;
      }
  }
}

template <int FM, int FN, bool FAST, bool AH, bool BH, bool TRI = false, bool DB = false>
__global__ __launch_bounds__(256) void small_gemm_kernel(const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) bf16 As[DB ? 2 : 1][32 * FM][LDT];
  __shared__ __attribute__((aligned(16))) bf16 Bs[DB ? 2 : 1][32 * FN][LDT];
  int gi;
  const int t = tile_of_block(batch, gi);
  const GemmDesc& g = batch.d[gi];
  const unsigned long long off = g.offset + (batch.dev_off ? *batch.dev_off : 0ull);
  gemm_tile<FM, FN, FAST, AH, BH, TRI, DB>(g, off, t, As[0], Bs[0], As[DB ? 1 : 0], Bs[DB ? 1 : 0]);
}

// ---- bf16 x bf16 launches: an LDS-DMA ring ---------------------------------------------------
// The register-queue tile above keeps one k-tile in flight (a deeper queue costs VGPRs and
// measured slower), so a tile's k-steps are a chain of global-load latencies.  Here every
// k-tile goes global -> LDS by buffer_load ... lds (16 B per lane, no VGPR round trip,
// out-of-range rows / k answered with zeros by the buffer descriptor), NSTG stages deep.  64 x
// 64 tile, 4 waves in 2 x 2 (32 x 32 each = 2 x 2 MFMA fragments).  Each operand's stage is 64
// LDS rows of 128 B as it sits in memory: k-contiguous (mode 0) -> [64 rows][64 k], chunk c of
// row r at c ^ (r & 7), fragments by ds_read_b128; stored transposed (mode 1) -> [64 k][64
// rows], chunk c of row k at c ^ tsw(k) (the TRI image), fragments by two ds_read_b64_tr_b16.
// The swizzle goes on the source address (DMA images are lane-linear).  Column sums of a
// mode-1 A (asum, a weight gradient's bias gradient) come from one more MFMA per fragment
// against a ones operand, in the column-0 tiles.  Same operands, k order and epilogue as
// gemm_tile: C is bitwise that of the register-queue bf16 kernel.
constexpr int DMA_STAGE = 2 * 64 * 128;  // A and B, 64 rows x 128 B each
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 dma_read128(uint32_t addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ s16x4 dma_read_tr(uint32_t addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

// MFMA fragment of rows col0 + lane % 16, k = ks + 8 (lane / 16) .. + 7, from a 128-B-row image
// (opaque reads: a builtin LDS read after the DMA into the same array makes the compiler wait
// for every load in flight).  TR: the image is [k][rows] (tri_frag's addressing).
template <bool TR>
__device__ __forceinline__ u32x4 dma_frag(uint32_t img, int ks, int col0, int lane) {
  if constexpr (!TR) {
    const int r = col0 + (lane & 15);
    return dma_read128(img + r * 128 + ((((ks >> 3) + (lane >> 4)) ^ (r & 7)) << 4));
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int c = (col0 >> 3) + (p >> 1);
    s16x4 v[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int r = ks + 8 * g + 4 * hf + q;
      v[hf] = dma_read_tr(img + r * 128 + ((c ^ tsw(r)) << 4) + (p & 1) * 8);
    }
    return u32x4{__builtin_bit_cast(uint2, v[0]).x, __builtin_bit_cast(uint2, v[0]).y,
                 __builtin_bit_cast(uint2, v[1]).x, __builtin_bit_cast(uint2, v[1]).y};
  }
}

template <int DMA_NSTG>
__device__ __forceinline__ void gemm_tile_dma(const GemmDesc& g, unsigned long long off, int t, char* smem) {
  const int split = t % g.splits;
  t /= g.splits;
  const int m0 = (t / g.tiles_n) * 64, n0 = (t % g.tiles_n) * 64;
  const int kbeg = split * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int fr = lane & 15, fq = lane >> 4;
  const __amdgpu_buffer_rsrc_t rsa = rsrc_of(g.A), rsb = rsrc_of(g.B);
  const bool ta = g.a_mode == 1, tb = g.b_mode == 1;  // block-uniform
  // this lane's rows of the two 8-row pieces per operand (wave w: LDS rows 16 w .. 16 w + 15)
  const int prow = lane >> 3, pch = lane & 7;
  auto stage = [&](int st, int k0) {
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      const bool isA = op == 0;
      const bool tr = isA ? ta : tb;
      const int R = isA ? g.M : g.N, r0 = isA ? m0 : n0, ld = isA ? g.lda : g.ldb;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int row = wave * 16 + p * 8 + prow;
        uint32_t o;
        if (!tr) {  // row = an output row / column, chunk = 8 k
          const int k = k0 + ((pch ^ (row & 7)) << 3);
          o = (r0 + row < R && k < kend) ? (uint32_t)((r0 + row) * ld + k) * 2u : OOB;
        } else {  // row = a k, chunk = 8 output rows / columns
          const int c = r0 + ((pch ^ tsw(row)) << 3);
          o = (k0 + row < kend && c < R) ? (uint32_t)((k0 + row) * ld + c) * 2u : OOB;
        }
        char* dst = smem + st * DMA_STAGE + op * 64 * 128 + (wave * 16 + p * 8) * 128;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rsa : rsb, LDS_PTR(void, dst), 16, o, 0, 0, 0);
      }
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // asum: the column-0 tiles' n-wave 0 also multiplies its A fragments by ones
  const bool do_as = g.asum != nullptr && n0 == 0 && wn == 0;  // wave-uniform
  f32x4 as_[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const bf16x8 ones = bf16x8{(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f};
  const int nk = (kend - kbeg + 63) >> 6;
#pragma unroll
  for (int s = 0; s < DMA_NSTG - 1; ++s)
    if (s < nk) stage(s, kbeg + s * 64);
  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed for this wave (its younger stages -- at most NSTG - 2, 4 pieces each -- may
    // stay in flight), then every wave's: the barrier; the buffer refilled below was read at kt - 1
    const int younger = min(nk - 1 - kt, DMA_NSTG - 2);
    if (DMA_NSTG >= 4 && younger >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (DMA_NSTG >= 3 && younger >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // a bare barrier: __syncthreads' release fence would wait for every LDS-DMA load (vmcnt(0))
    asm volatile("s_barrier" ::: "memory");
    if (kt + DMA_NSTG - 1 < nk) stage((kt + DMA_NSTG - 1) % DMA_NSTG, kbeg + (kt + DMA_NSTG - 1) * 64);
    const uint32_t As = lds0 + (kt % DMA_NSTG) * DMA_STAGE, Bs = As + 64 * 128;
#pragma unroll
    for (int ks = 0; ks < 64; ks += 32) {
      u32x4 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = ta ? dma_frag<true>(As, ks, wm + i * 16, lane) : dma_frag<false>(As, ks, wm + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = tb ? dma_frag<true>(Bs, ks, wn + j * 16, lane) : dma_frag<false>(Bs, ks, wn + j * 16, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[i]),
                                                              __builtin_bit_cast(bf16x8, b[j]), acc[i][j], 0, 0, 0);
      if (do_as) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          as_[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[i]), ones, as_[i], 0, 0, 0);
      }
    }
  }
  const bool part = g.splits > 1;
  if (do_as && fr == 0) {  // lanes of column 0 hold the row sums of rows wm + 16 i + 4 fq + r
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + fq * 4 + r;
        if (m < g.M) {
          if (part) g.AP[(size_t)split * g.M + m] = as_[i][r];
          else g.asum[m] = as_[i][r];
        }
      }
  }
  // epilogue as gemm_tile: lane holds C[m = wm + 16 i + 4 fq + r][n = wn + 16 j + fr]
  float* const dst = part ? g.P + (size_t)split * g.M * g.N : g.C;
  const int ldd = part ? g.N : g.ldc;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn + j * 16 + fr;
    const bool nok = n < g.N;
    const float bn = (!part && nok && g.bias) ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + fq * 4 + r;
        if (!nok || m >= g.M) continue;
        float v = acc[i][j][r];
        float* c = dst + (size_t)m * ldd + n;
        if (!part) {
          v = g.alpha * v + bn;
          if (g.act == 1) v = tanhf(v);
          if (g.drop_on == 3) v *= drop3(g, off, m, n);
          if (g.accumulate) v += *c;
        }
        *c = v;
      }
  }
}

template <int NSTG>
__global__ __launch_bounds__(256) void small_gemm_dma_kernel(const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) char smem[NSTG * DMA_STAGE];
  int gi;
  const int t = tile_of_block(batch, gi);
  const GemmDesc& g = batch.d[gi];
  const unsigned long long off = g.offset + (batch.dev_off ? *batch.dev_off : 0ull);
  gemm_tile_dma<NSTG>(g, off, t, smem);
}

// FAST loads with the operand dtypes per desc: a block-uniform switch into the four typed
// bodies (one launch for, e.g., a backward's weight gradients over bf16 and fp32 inputs)
template <bool TRI = false, bool DB = false>
__global__ __launch_bounds__(256) void small_gemm_mixed_kernel(const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) bf16 As[DB ? 2 : 1][64][LDT];
  __shared__ __attribute__((aligned(16))) bf16 Bs[DB ? 2 : 1][64][LDT];
  int gi;
  const int t = tile_of_block(batch, gi);
  const GemmDesc& g = batch.d[gi];
  const unsigned long long off = g.offset + (batch.dev_off ? *batch.dev_off : 0ull);
  if (g.a_bf16) {
    if (g.b_bf16)
      gemm_tile<2, 2, true, true, true, TRI, DB>(g, off, t, As[0], Bs[0], As[DB ? 1 : 0], Bs[DB ? 1 : 0]);
    else
      gemm_tile<2, 2, true, true, false, TRI, DB>(g, off, t, As[0], Bs[0], As[DB ? 1 : 0], Bs[DB ? 1 : 0]);
  } else {
    if (g.b_bf16)
      gemm_tile<2, 2, true, false, true, TRI, DB>(g, off, t, As[0], Bs[0], As[DB ? 1 : 0], Bs[DB ? 1 : 0]);
    else
      gemm_tile<2, 2, true, false, false, TRI, DB>(g, off, t, As[0], Bs[0], As[DB ? 1 : 0], Bs[DB ? 1 : 0]);
  }
}


// ---- register-direct launches (bf16 x bf16, both operands k-contiguous) -------------------
// The LDS forms above spend each k-step on one global -> LDS latency behind a barrier: a launch
// of these shapes (K = 200..1200, ~1-4 tiles per CU) is a chain of such latencies, 13-26 us in
// the config-2 step for 0.5-3 GFLOP (profiles/r5m_launch_seq.txt).  Here an MFMA fragment is
// loaded straight into VGPRs: for v_mfma_f32_16x16x32_bf16 a lane needs 8 consecutive k (16 B)
// of row lane % 16 at k = 8 (lane / 16) of a 32-deep k-step, which is one buffer_load_dwordx4 of
// a k-contiguous operand.  Each wave owns a (16 FM) x (16 FN) tile and keeps P k-steps of
// fragments in flight (a ring in registers, statically indexed by unrolling the k loop by P):
// no LDS, no barrier, the wave waits only for its own oldest k-step.  A block is 4 waves in
// 2 x 2 over a (32 FM) x (32 FN) block tile (the two waves of a row / column share their A / B
// lines in L1).  The MFMA takes B as src0, so a lane ends with 4 consecutive columns of one
// row: float4 epilogue stores (the LDS forms' lanes hold 4 rows of one column: 4-byte stores).
// Rows past M / N and k past K load as zeros (buffer offsets past the descriptor's range).
// AF: A fp32 (two 16-B loads per fragment, rounded to bf16 in registers -- the rounding the LDS
// forms apply on their way into LDS).
template <int FM, int FN, int P, bool AF = false>
__global__ __launch_bounds__(256) void small_gemm_rd_kernel(const GemmBatch batch) {
  int gi;
  int t = tile_of_block(batch, gi);
  const GemmDesc& g = batch.d[gi];
  const unsigned long long off = g.offset + (batch.dev_off ? *batch.dev_off : 0ull);
  const int split = t % g.splits;
  t /= g.splits;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = (t / g.tiles_n) * (32 * FM) + (wave >> 1) * (16 * FM);
  const int n0 = (t % g.tiles_n) * (32 * FN) + (wave & 1) * (16 * FN);
  const int kbeg = split * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
  const int fr = lane & 15, fq = lane >> 4;
  const __amdgpu_buffer_rsrc_t rsa = rsrc_of(g.A), rsb = rsrc_of(g.B);
  // byte offsets of this lane's fragment rows at k = kbeg + 8 fq (OOB: a row past M / N)
  uint32_t oa[FM], ob[FN];
  constexpr uint32_t AES = AF ? 4u : 2u;  // A element bytes
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int r = m0 + i * 16 + fr;
    oa[i] = r < g.M ? (uint32_t)(r * g.lda + kbeg + 8 * fq) * AES : OOB;
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int r = n0 + j * 16 + fr;
    ob[j] = r < g.N ? (uint32_t)(r * g.ldb + kbeg + 8 * fq) * 2u : OOB;
  }
  const int nk = (kend - kbeg + 31) >> 5;
  u32x4 ra[P][FM][AF ? 2 : 1], rb[P][FN];
  auto load = [&](int s, int kt) {  // k-step kt into ring slot s (zeros past kend)
    const bool kok = kbeg + kt * 32 + 8 * fq < kend;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int h = 0; h < (AF ? 2 : 1); ++h)
        ra[s][i][h] = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsa, kok ? oa[i] + kt * 32 * AES + 16 * h : OOB, 0, 0));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      rb[s][j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsb, kok ? ob[j] + kt * 64 : OOB, 0, 0));
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto afrag = [&](int s, int i) -> bf16x8 {
    if constexpr (!AF) {
      return __builtin_bit_cast(bf16x8, ra[s][i][0]);
    } else {
      bf16x8 o;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q) o[4 * h + q] = f2bf(__uint_as_float(ra[s][i][AF ? h : 0][q]));
      return o;
    }
  };
  auto mma = [&](int s) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bf16x8 a = afrag(s, i);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, rb[s][j]), a, acc[i][j], 0, 0, 0);
    }
  };
#pragma unroll
  for (int s = 0; s < P; ++s) load(s, s);
  // whole groups of P k-steps with no branch inside (the compiler's wait pass then keeps the
  // younger slots in flight across the loop edge -- a branch per slot made it wait for every
  // load at the loop head); loads past the last k-step are zero-filled OOB loads, never used
  const int nfull = nk / P * P;
  for (int kt = 0; kt < nfull; kt += P) {
#pragma unroll
    for (int s = 0; s < P; ++s) {
      mma(s);
      load(s, kt + s + P);
      __builtin_amdgcn_sched_barrier(0);  // slot s refills here, not with the whole group at the end
    }
  }
#pragma unroll
  for (int s = 0; s < P - 1; ++s)
    if (nfull + s < nk) mma(s);
  // lane holds C[m0 + 16 i + fr][n0 + 16 j + 4 fq + r], r = 0..3
  const bool part = g.splits > 1;
  float* const dst = part ? g.P + (size_t)split * g.M * g.N : g.C;
  const int ldd = part ? g.N : g.ldc;
  const bool vec = (ldd & 3) == 0 && (((uintptr_t)dst) & 15) == 0;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + j * 16 + 4 * fq;
    if (n >= g.N) continue;
    const bool full = n + 3 < g.N;
    float bn[4] = {0.f, 0.f, 0.f, 0.f};
    if (!part && g.bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bn[r] = n + r < g.N ? g.bias[n + r] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + i * 16 + fr;
      if (m >= g.M) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      float* c = dst + (size_t)m * ldd + n;
      if (!part) {
        float dsc[4] = {1.f, 1.f, 1.f, 1.f};
        if (g.drop_on == 3) {  // n % 4 == 0 and drop_ld % 16 == 0: one Philox draw for the 4
          const unsigned long long e = (unsigned long long)m * g.drop_ld + n;
          const uint4 x = Philox::gen(g.seed, off, e >> 2);
          const float ik = 1.0f / (1.0f - g.pdrop);
#pragma unroll
          for (int r = 0; r < 4; ++r) dsc[r] = drop_scale(u4_get(x, r), g.pdrop, ik);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = g.alpha * v[r] + bn[r];
          if (g.act == 1) v[r] = tanhf(v[r]);
          v[r] *= dsc[r];
        }
      }
      if (full && vec) {
        float4 o = make_float4(v[0], v[1], v[2], v[3]);
        if (!part && g.accumulate) {
          const float4 p = *(const float4*)c;
          o.x += p.x; o.y += p.y; o.z += p.z; o.w += p.w;
        }
        *(float4*)c = o;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < g.N) c[r] = (!part && g.accumulate) ? v[r] + c[r] : v[r];
      }
    }
  }
}

// split-K epilogue: C = act(alpha * sum_s P[s] + bias) (x the output dropout scale, drop_on 3)
// (+ C), partials summed in split order (deterministic) -- the single-pass epilogue's order.
// Each desc owns a block range (red_base); a lane takes 4 consecutive columns of one row: 16-B
// partial loads, one Philox draw for the 4 dropout scales (drop_ld % 16 == 0, n % 4 == 0).
// N % 4 == 0 for every split desc (host-checked); C / bias / accumulate fall back to scalar
// accesses when a row of C is not 16-byte aligned.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmBatch batch, int c_blocks) {
  fr_sg::splitk_reduce_block(batch, c_blocks, (int)blockIdx.x);
}

// Deferred split-K reduction (fr_small_gemm_set_defer): a launch whose split descs are all
// weight gradients (a_mode 1: read only by the optimizer) leaves its reduction pending instead
// of launching it; the text head's tail reduce (fr_head_wgrad_g) takes it and runs it in extra
// blocks of its own launch, or fr_small_gemm_flush_pending launches it alone.  One pending
// reduction at a time (a second deferrable launch reduces at once), process-wide: it is taken
// only on the device it was deferred on, and the caller (ops/functional.py side_wgrads) defers
// within one backward on one stream and flushes whatever is left when that backward ends.
bool g_defer = false;
struct PendingReduce {
  GemmBatch b;
  int c_blocks, total;
  int device;
  bool set;
};
PendingReduce g_pend = {};

void finish_reduce(const GemmBatch& b, int c_blocks, int total, hipStream_t s) {
  if (total <= 0) return;
  bool deferrable = g_defer && !g_pend.set;
  for (int i = 0; i < b.n && deferrable; ++i)
    if (b.d[i].splits > 1 && b.d[i].a_mode != 1) deferrable = false;
  if (deferrable) {
    g_pend.b = b;
    g_pend.c_blocks = c_blocks;
    g_pend.total = total;
    g_pend.device = 0;
    (void)hipGetDevice(&g_pend.device);
    g_pend.set = true;
    return;
  }
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(total), dim3(256), 0, s, b, c_blocks);
}

// Deterministic fp32 column sums (bias gradients), two passes: (1) blocks of CS_ROWS rows x
// (256 columns as float4 per lane when the matrix allows 16-byte loads, else 64 columns)
// write per-chunk partials, 4 waves x CS_ROWS/4 rows each, 8 row loads in flight per lane;
// (2) the partials are summed in a fixed order, 4 waves per 64 columns.  A desc of one row chunk (the loss sum, the
// pooled-user partial rows) is final after pass 1, and a launch of only such descs skips
// pass 2.  (A single-pass "last block sums" form with agent-scope fences measured 131 us/step
// vs 69: each release fence writes back L2.  The scalar form -- one float per lane, 128 rows
// per block -- took 32 us for the user step's 18 MB of gradients.)
constexpr int CS_ROWS = 128;
struct ColsumDesc {
  const float* X;
  float* out;
  float* part;  // [chunks, N]
  int M, N, ld, col_blocks, chunks, block_base, block2_base, accumulate, vec;
};
struct ColsumBatch {
  ColsumDesc d[MAXG];
  int n;
};

__global__ __launch_bounds__(256) void colsum_part_kernel(const ColsumBatch batch) {
  __shared__ float4 part[4][64];
  int gi = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < batch.n && (int)blockIdx.x >= batch.d[i].block_base) gi = i;
  const ColsumDesc& g = batch.d[gi];
  const int b = blockIdx.x - g.block_base;
  const int cb = b % g.col_blocks, ch = b / g.col_blocks;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = ch * CS_ROWS, r1 = min(g.M, r0 + CS_ROWS);
  constexpr int RW = CS_ROWS / 4;  // rows per wave (contiguous)
  const int ra = r0 + w * RW, rb = min(r1, ra + RW);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (g.vec) {
    const int c = cb * 256 + 4 * l;
    if (c < g.N) {
      const float* x = g.X + c;
#pragma unroll 8
      for (int m = ra; m < rb; ++m) {
        const float4 v = *(const float4*)(x + (size_t)m * g.ld);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
    }
  } else {
    const int c = cb * 64 + l;
    if (c < g.N) {
#pragma unroll 8
      for (int m = ra; m < rb; ++m) s.x += g.X[(size_t)m * g.ld + c];
    }
  }
  part[w][l] = s;
  __syncthreads();
  if (w != 0) return;
  const float4 a = part[0][l], bq = part[1][l], cq = part[2][l], d = part[3][l];
  const float tot[4] = {(a.x + bq.x) + (cq.x + d.x), (a.y + bq.y) + (cq.y + d.y), (a.z + bq.z) + (cq.z + d.z),
                        (a.w + bq.w) + (cq.w + d.w)};
  const int nc = g.vec ? 4 : 1;
  const int c0 = g.vec ? cb * 256 + 4 * l : cb * 64 + l;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = c0 + q;
    if (q >= nc || c >= g.N) break;
    if (g.chunks == 1)  // one row chunk: the final value (no second pass for this desc)
      g.out[c] = g.accumulate ? g.out[c] + tot[q] : tot[q];
    else
      g.part[(size_t)ch * g.N + c] = tot[q];
  }
}

// pass 2: 64 columns per block, wave w sums chunks w, w + 4, ... (independent loads in flight),
// wave 0 adds the four wave sums in order (deterministic)
__global__ __launch_bounds__(256) void colsum_final_kernel(const ColsumBatch batch) {
  __shared__ float ws[4][64];
  int gi = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < batch.n && (int)blockIdx.x >= batch.d[i].block2_base) gi = i;
  const ColsumDesc& g = batch.d[gi];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.x - g.block2_base) * 64 + l;
  if (g.chunks == 1) return;  // block-uniform
  float s = 0.f;
  if (c < g.N)
#pragma unroll 4
    for (int ch = w; ch < g.chunks; ch += 4) s += g.part[(size_t)ch * g.N + c];
  ws[w][l] = s;
  __syncthreads();
  if (w == 0 && c < g.N) {
    const float t = (ws[0][l] + ws[1][l]) + (ws[2][l] + ws[3][l]);
    g.out[c] = g.accumulate ? g.out[c] + t : t;
  }
}

}  // namespace

// descs: 8 pointers + 16 ints + 2 floats + 2 u64 per GEMM, packed by binding.cpp small_gemm.
// scratch: split-K partial space (floats) the caller allocated; returns the floats it needs
// when scratch is null (query mode).
static int choose_splits(int tiles, int K, bool dma) {
  // a workgroup's k-steps are a chain of dependent global-load latencies (one k-tile in
  // flight): a long reduction over few output tiles is latency bound, not bandwidth bound.
  // Split K until the launch has ~2 workgroups per CU, keeping >= 6 k-tiles per split
  // (measured: the 1200 x 400 x 3200 weight gradient in 133 tiles -- 2 splits 69 us, four
  // 400-row descs in 6 splits 49 us; the 3200 x 400 x 1200 dgrad in 350 tiles -- 2 splits
  // 38.6 us, 3 splits 44.5: the partials' write + reduce outweigh the shorter chains).
  // fewest K per split: 384 (6 k-tiles) measured best of 192-768 (profiles/r3_ab_sg_mink.txt)
  // The LDS-DMA ring keeps a k-tile in flight behind the MFMAs, so its k-steps are cheap: it
  // splits only above 1,024 per split (the 3200 x 400 x 1200 dgrad 19.9 vs 22.4 us with 2
  // splits, the text fc 13.6 vs 15.0; the K = 3200 weight gradients still want theirs:
  // profiles/r4_sg_step_shapes_r.json)
  const int mink = dma ? 1024 : 384;
  if (K < 512) return 1;
  const int want = (512 + tiles - 1) / tiles;
  int s = min(want, K / mink);
  return max(1, min(s, 16));
}

// tile variants: 1 = 64 x 64, 2 = 128 x 64, 3 = 64 x 128, 4 = 128 x 128 (TM x TN)
static void tile_dims(int v, int& tm, int& tn) {
  tm = (v == 2 || v == 4) ? 128 : 64;
  tn = (v == 3 || v == 4) ? 128 : 64;
}

// auto: 64 x 64 unless the launch has >= 8 tiles of it per CU.  Per k-tile the bigger tiles
// cost the same (bandwidth-bound: fewer bytes, fewer waves), but a launch of ~1 tile per CU
// exposes each workgroup's serial prologue -> k-steps -> epilogue chain: at K = 64 the
// 128 x 128 form took 18.7 us vs 9.4 (3200 x 1200), and only caught up at >= 4 tiles per CU
// and K >= 512 (benchmarks/sg_latency_probe.py, profiles/r3_small_gemm_bench.json).
static int choose_tile(const GemmBatch& b) {
  long tiles = 0;
  for (int i = 0; i < b.n; ++i) tiles += (long)((b.d[i].M + 63) / 64) * ((b.d[i].N + 63) / 64);
  return tiles >= 2048 ? 4 : 1;
}

// can the launch take the FAST kernels (branch-free buffer loads, dtypes fixed per launch)?
static bool fast_ok(const GemmBatch& b) {
  bool fast = true;  // every operand's contiguous extent in whole 16-byte halves of a chunk
  for (int i = 0; i < b.n; ++i) {
    const GemmDesc& d = b.d[i];
    const int ea = d.a_bf16 ? 8 : 4, eb = d.b_bf16 ? 8 : 4;  // elements per 16 bytes
    const int ca = d.a_mode == 0 ? d.K : d.M, cb = d.b_mode == 0 ? d.K : d.N;  // contiguous extents
    // byte extents the 32-bit buffer offsets address
    const double ext_a = (double)(d.a_mode == 0 ? d.M : d.K) * d.lda * (d.a_bf16 ? 2 : 4);
    const double ext_b = (double)(d.b_mode == 0 ? d.N : d.K) * d.ldb * (d.b_bf16 ? 2 : 4);
    fast = fast && ca % 8 == 0 && cb % 8 == 0 && d.K % 8 == 0 && d.lda % ea == 0 && d.ldb % eb == 0 &&
           ((uintptr_t)d.A & 15) == 0 && ((uintptr_t)d.B & 15) == 0 && d.kseg == 0 && d.gather_on == 0 &&
           d.drop_on != 1 && d.drop_on != 2 && ext_a < 2.0e9 && ext_b < 2.0e9;
  }
  return fast;
}

// the LDS-DMA ring takes every bf16 x bf16 FAST launch (no gather / operand dropout / kseg,
// 16-B aligned extents); M and N multiples of 8 where the operand is stored transposed (its
// 16-B chunks run along them)
static bool dma_ok(const GemmBatch& b) {
  for (int i = 0; i < b.n; ++i)
    if ((b.d[i].a_mode == 1 && b.d[i].M % 8) || (b.d[i].b_mode == 1 && b.d[i].N % 8)) return false;
  return true;
}

static bool mixed_dtypes(const GemmBatch& b) {
  for (int i = 1; i < b.n; ++i)
    if (b.d[i].a_bf16 != b.d[0].a_bf16 || b.d[i].b_bf16 != b.d[0].b_bf16) return true;
  return false;
}

// the register-direct form takes bf16 x bf16 launches whose operands are both k-contiguous
// (a_mode 0, b_mode 0), no column sums, the output dropout at most
// (A fp32 or bf16, the same in every desc; B bf16)
static bool rd_ok(const GemmBatch& b) {
  for (int i = 0; i < b.n; ++i) {
    const GemmDesc& d = b.d[i];
    if (d.a_bf16 != b.d[0].a_bf16 || !d.b_bf16 || d.a_mode != 0 || d.b_mode != 0 || d.asum || d.drop_on == 1 ||
        d.drop_on == 2 || d.gather_on || d.kseg)
      return false;
  }
  return true;
}

int g_sg_rd = 0;  // auto picks the register-direct form: 0 off (benchmarks / A-B switch), 1 on
extern "C" void fr_small_gemm_set_rd(int v) { g_sg_rd = v; }

static int rd_auto(const GemmBatch& b) {
  if (!g_sg_rd) return 0;
  long t64 = 0;  // 64 x 64 block tiles of 32 x 32 wave tiles
  for (int i = 0; i < b.n; ++i) t64 += (long)((b.d[i].M + 63) / 64) * ((b.d[i].N + 63) / 64);
  return t64 >= 512 ? 1000 + 10 * 1 + 3 : 1000 + 4;  // 128 x 128 / P 3 at >= 2 small tiles per CU
}

static long launch_rd(GemmBatch& b, int code, float* scratch, hipStream_t s) {
  const bool allow_split = (code / 100) % 10 != 0;
  const int f = (code / 10) % 10, P = code % 10;
  // f: 0 = 32 x 32 waves, 1 = 64 x 64, 2 = 32 x 64, 3 = 64 x 32 (16 x 16 / 16 x 32 / 32 x 16 wave
  // tiles measured slower on every config-2 shape: profiles/r5_sg_rd_small_tiles.jsonl)
  static const int FMS[4] = {2, 4, 2, 4}, FNS[4] = {2, 4, 4, 2};
  if (P < 2 || P > 4 || f > 3) return -7;
  const int FM = FMS[f], FN = FNS[f];
  const int tm = 32 * FM, tn = 32 * FN;
  int tiles = 0, red_blocks = 0;
  long need = 0;
  for (int i = 0; i < b.n; ++i) {
    GemmDesc& d = b.d[i];
    d.tiles_n = (d.N + tn - 1) / tn;
    const int t = ((d.M + tm - 1) / tm) * d.tiles_n;
    d.splits = allow_split ? choose_splits(t, d.K, true) : 1;
    d.kchunk = d.splits > 1 ? ((d.K + d.splits - 1) / d.splits + 31) / 32 * 32 : d.K;
    if (d.splits > 1) d.splits = (d.K + d.kchunk - 1) / d.kchunk;
    if (d.splits > 1 && d.N % 4 != 0) {
      d.splits = 1;
      d.kchunk = d.K;
    }
    d.P = nullptr;
    d.AP = nullptr;
    d.red_base = red_blocks;
    d.ared_base = 0;
    if (d.splits > 1) {
      d.P = scratch ? scratch + need : nullptr;
      need += (long)d.splits * d.M * d.N;
      red_blocks += (int)(((long)d.M * d.N / 4 + 255) / 256);
    }
    d.tile_base = tiles;
    tiles += t * d.splits;
  }
  if (scratch == nullptr && need > 0) return need;
  if (tiles == 0) return 0;
#define RD_LAUNCH(FM_, FN_, P_)                                                                              \
  do {                                                                                                     \
    if (b.d[0].a_bf16) hipLaunchKernelGGL((small_gemm_rd_kernel<FM_, FN_, P_>), dim3(tiles), dim3(256), 0, s, b); \
    else hipLaunchKernelGGL((small_gemm_rd_kernel<FM_, FN_, P_, true>), dim3(tiles), dim3(256), 0, s, b);   \
  } while (0)
#define RD_P(FM_, FN_)          \
  do {                          \
    if (P == 2) RD_LAUNCH(FM_, FN_, 2); \
    else if (P == 3) RD_LAUNCH(FM_, FN_, 3); \
    else RD_LAUNCH(FM_, FN_, 4); \
  } while (0)
  if (FM == 2 && FN == 2) RD_P(2, 2);
  else if (FM == 4 && FN == 4) RD_P(4, 4);
  else if (FM == 2) RD_P(2, 4);
  else RD_P(4, 2);
#undef RD_P
#undef RD_LAUNCH
  finish_reduce(b, red_blocks, red_blocks, s);
  return 0;
}

extern "C" long fr_small_gemm(const void* const* ptrs, const int* ints, const float* floats,
                              const unsigned long long* seeds, const unsigned long long* dev_off, int n, float* scratch,
                              int tile, hipStream_t s) {
  if (n < 1 || n > MAXG) return -1;
  GemmBatch b{};
  b.dev_off = dev_off;
  for (int i = 0; i < n; ++i) {
    GemmDesc& d = b.d[i];
    d.A = ptrs[8 * i + 0];
    d.gidx = (const int*)ptrs[8 * i + 1];
    d.B = ptrs[8 * i + 2];
    d.bias = (const float*)ptrs[8 * i + 3];
    d.C = (float*)ptrs[8 * i + 4];
    d.B2 = ptrs[8 * i + 5];
    d.B3 = ptrs[8 * i + 6];
    d.asum = (float*)ptrs[8 * i + 7];
    const int* q = ints + 16 * i;
    d.M = q[0]; d.N = q[1]; d.K = q[2]; d.lda = q[3]; d.ldb = q[4]; d.ldc = q[5];
    d.a_mode = q[6]; d.b_mode = q[7]; d.act = q[8]; d.accumulate = q[9]; d.drop_ld = q[10];
    d.drop_on = q[11]; d.gather_on = q[12]; d.kseg = q[13]; d.a_bf16 = q[14] != 0; d.b_bf16 = q[15] != 0;
    if (d.kseg > 0 && (d.b_mode != 1 || d.gather_on == 2 || !d.B2 || (d.K > 2 * d.kseg && !d.B3) || d.K > 3 * d.kseg))
      return -5;
    d.alpha = floats[2 * i];
    d.pdrop = floats[2 * i + 1];
    d.seed = seeds[2 * i];
    d.offset = seeds[2 * i + 1];
    if (d.M < 0 || d.N < 0 || d.K < 0) return -2;
    if (d.drop_on < 0 || d.drop_on > 3 || d.gather_on < 0 || d.gather_on > 2 || d.act < 0 || d.act > 1) return -3;
    if (d.drop_on && (!(d.pdrop > 0.f && d.pdrop < 1.f) || d.drop_ld % 16 != 0 ||
                      (d.drop_on == 1 && (d.a_mode != 0 || d.a_bf16)) || (d.drop_on == 2 && (d.b_mode != 1 || d.b_bf16))))
      return -3;
    if (d.gather_on && (!d.gidx || (d.gather_on == 1 && d.a_mode != 0) || (d.gather_on == 2 && d.b_mode != 1))) return -4;
    if (d.asum && d.a_mode != 1) return -6;  // column sums of a stored-transposed A only
  }
  b.n = n;
  const bool fast = fast_ok(b), mixed = mixed_dtypes(b);
  // register-direct form: tile codes 1000 + 100 s + 10 f + P (s: split-K allowed, f: wave tile
  // 0 = 32 x 32, 1 = 64 x 64, 2 = 32 x 64, 3 = 64 x 32, P: k-steps in flight 2..4); 0 = auto
  // (a code the launch's operands do not allow falls back to the automatic choice)
  if (tile >= 1000 || tile == 0) {
    const int code = tile == 0 ? rd_auto(b) : tile;
    if (code >= 1000 && fast && rd_ok(b)) return launch_rd(b, code, scratch, s);
    tile = 0;
  }
  // benchmarks / tests: 5 = the 64 x 64 register-queue form (never the DMA ring), 6 / 7 / 8 =
  // the DMA ring with 2 / 3 / 4 stages where it applies, 9 = 2 stages and no split-K
  const bool regq = tile == 5;
  const int force_stg = (tile >= 6 && tile <= 8) ? tile - 4 : (tile == 9 ? 2 : 0);
  const bool nosplit = tile == 9;  // benchmarks: the 2-stage DMA ring without split-K
  int v = (tile >= 1 && tile <= 4) ? tile : (regq || force_stg) ? 1 : choose_tile(b);
  if (!fast || mixed) v = 1;  // the generic (any alignment) and mixed-dtype kernels: 64 x 64
  int tm, tn;
  tile_dims(v, tm, tn);
  const int dt = (b.d[0].a_bf16 ? 2 : 0) | (b.d[0].b_bf16 ? 1 : 0);
  // a DMA-ring launch (its split-K rule also applies to the register-queue form of the same
  // launch, tile 5, so the two stay bitwise comparable)
  const bool dma_shape = fast && !mixed && v == 1 && dt == 3 && dma_ok(b);
  const bool dma = dma_shape && !regq;
  int tiles = 0;
  long need = 0;
  int red_blocks = 0;
  for (int i = 0; i < n; ++i) {
    GemmDesc& d = b.d[i];
    d.tiles_n = (d.N + tn - 1) / tn;
    const int t = ((d.M + tm - 1) / tm) * d.tiles_n;
    // split-K: the reduce applies the whole epilogue (alpha, bias, tanh, output dropout, accumulate)
    d.splits = nosplit ? 1 : choose_splits(t, d.K, dma_shape);
    d.kchunk = d.splits > 1 ? ((d.K + d.splits - 1) / d.splits + TK - 1) / TK * TK : d.K;
    if (d.splits > 1) d.splits = (d.K + d.kchunk - 1) / d.kchunk;
    if (d.splits > 1 && d.N % 4 != 0) {  // the reduction takes 4 columns per lane
      d.splits = 1;
      d.kchunk = d.K;
    }
    d.P = nullptr;
    d.AP = nullptr;
    d.red_base = red_blocks;
    if (d.splits > 1) {
      d.P = scratch ? scratch + need : nullptr;
      need += (long)d.splits * d.M * d.N;
      red_blocks += (int)(((long)d.M * d.N / 4 + 255) / 256);
      if (d.asum) {
        d.AP = scratch ? scratch + need : nullptr;
        need += (long)d.splits * d.M;
      }
    }
    d.tile_base = tiles;
    tiles += t * d.splits;
  }
  if (scratch == nullptr && need > 0) return need;  // query: the caller allocates and calls again
  if (tiles == 0) return 0;
#define SG_LAUNCH(FM, FN)                                                                                  \
  do {                                                                                                     \
    if (dt == 0)                                                                                           \
      hipLaunchKernelGGL((small_gemm_kernel<FM, FN, true, false, false>), dim3(tiles), dim3(256), 0, s, b);  \
    else if (dt == 1)                                                                                      \
      hipLaunchKernelGGL((small_gemm_kernel<FM, FN, true, false, true>), dim3(tiles), dim3(256), 0, s, b);   \
    else if (dt == 2)                                                                                      \
      hipLaunchKernelGGL((small_gemm_kernel<FM, FN, true, true, false>), dim3(tiles), dim3(256), 0, s, b);   \
    else                                                                                                   \
      hipLaunchKernelGGL((small_gemm_kernel<FM, FN, true, true, true>), dim3(tiles), dim3(256), 0, s, b);    \
  } while (0)
  // stored-transposed operands of the 64x64 tiles staged as TRI images (0.5715 -> 0.5566 ms per
  // config-2 step, profiles/r3_ab_sg_tri.txt) with two LDS buffers and one barrier per k-step
  // (0.5484-0.5493 vs 0.5494-0.5520 ms, r3_ab_sg_db.txt); the 128-row / -column tiles keep the
  // k-contiguous image (their launches have >= 8 tiles per CU: bandwidth-, not latency-bound)
  if (!fast)
    hipLaunchKernelGGL((small_gemm_kernel<2, 2, false, false, false>), dim3(tiles), dim3(256), 0, s, b);
  else if (mixed)
    hipLaunchKernelGGL((small_gemm_mixed_kernel<true, true>), dim3(tiles), dim3(256), 0, s, b);
  else if (dma) {
    // two stages by default: a third / fourth measured slower on every config-2 shape (LDS per
    // block caps the blocks per CU; profiles/r4_sg_step_shapes.json)
    const int stg = force_stg ? force_stg : 2;
    if (stg == 2) hipLaunchKernelGGL(small_gemm_dma_kernel<2>, dim3(tiles), dim3(256), 0, s, b);
    else if (stg == 3) hipLaunchKernelGGL(small_gemm_dma_kernel<3>, dim3(tiles), dim3(256), 0, s, b);
    else hipLaunchKernelGGL(small_gemm_dma_kernel<4>, dim3(tiles), dim3(256), 0, s, b);
  }
  else if (v == 1) {
    if (dt == 0) hipLaunchKernelGGL((small_gemm_kernel<2, 2, true, false, false, true, true>), dim3(tiles), dim3(256), 0, s, b);
    else if (dt == 1) hipLaunchKernelGGL((small_gemm_kernel<2, 2, true, false, true, true, true>), dim3(tiles), dim3(256), 0, s, b);
    else if (dt == 2) hipLaunchKernelGGL((small_gemm_kernel<2, 2, true, true, false, true, true>), dim3(tiles), dim3(256), 0, s, b);
    else hipLaunchKernelGGL((small_gemm_kernel<2, 2, true, true, true, true, true>), dim3(tiles), dim3(256), 0, s, b);
  }
  else switch (v) {
    case 2: SG_LAUNCH(4, 2); break;
    case 3: SG_LAUNCH(2, 4); break;
    case 4: SG_LAUNCH(4, 4); break;
    default: SG_LAUNCH(2, 2); break;
  }
#undef SG_LAUNCH
  int ared_blocks = 0;
  for (int i = 0; i < n; ++i) {
    GemmDesc& d = b.d[i];
    d.ared_base = red_blocks + ared_blocks;
    if (d.splits > 1 && d.asum) ared_blocks += (d.M + 255) / 256;
  }
  if (red_blocks + ared_blocks > 0)
    finish_reduce(b, red_blocks, red_blocks + ared_blocks, s);
  return 0;
}

extern "C" void fr_small_gemm_set_defer(int on) { g_defer = on != 0; }
extern "C" int fr_small_gemm_has_pending() { return g_pend.set ? 1 : 0; }
extern "C" int fr_small_gemm_batch_bytes() { return (int)sizeof(GemmBatch); }
// copies the pending reduction (GemmBatch + its block counts) out and clears it; 0 if none
extern "C" int fr_small_gemm_take_pending(void* dst, int dst_bytes, int* c_blocks, int* total) {
  if (!g_pend.set || dst_bytes < (int)sizeof(GemmBatch)) return 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != g_pend.device) return 0;  // another device's pending reduction: left for its flush
  memcpy(dst, &g_pend.b, sizeof(GemmBatch));
  *c_blocks = g_pend.c_blocks;
  *total = g_pend.total;
  g_pend.set = false;
  return 1;
}
extern "C" int fr_small_gemm_flush_pending(hipStream_t s) {
  if (!g_pend.set) return 0;
  g_pend.set = false;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != g_pend.device) {  // (not a configuration the engine uses: one device per process)
    (void)hipSetDevice(g_pend.device);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(g_pend.total), dim3(256), 0, 0, g_pend.b, g_pend.c_blocks);
    (void)hipDeviceSynchronize();
    (void)hipSetDevice(dev);
    return 1;
  }
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(g_pend.total), dim3(256), 0, s, g_pend.b, g_pend.c_blocks);
  return 1;
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
    d.vec = (d.N % 4 == 0 && d.ld % 4 == 0 && ((uintptr_t)d.X & 15) == 0) ? 1 : 0;
    d.col_blocks = d.vec ? (d.N + 255) / 256 : (d.N + 63) / 64;
    d.chunks = max(1, (d.M + CS_ROWS - 1) / CS_ROWS);
    d.part = part ? part + need : nullptr;
    need += (long)d.chunks * d.N;
    d.block_base = blocks;
    blocks += d.col_blocks * d.chunks;
    d.block2_base = blocks2;
    blocks2 += (d.N + 63) / 64;
  }
  b.n = n;
  if (part == nullptr) return need;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(colsum_part_kernel, dim3(blocks), dim3(256), 0, s, b);
  bool second = false;  // descs of one row chunk are final after the first pass
  for (int i = 0; i < n; ++i) second |= b.d[i].chunks > 1;
  if (second) hipLaunchKernelGGL(colsum_final_kernel, dim3(blocks2), dim3(256), 0, s, b);
  return 0;
}

// ---------------------------------------------------------------------------------------
// X'[m, k] = v[idx[m], k] * Z(m * K + k): the user encoder's gathered, dropped-out input
// (encoder.py:50), materialised once per step ([B*H, D], fp32 or -- when every reader is a
// bf16-operand GEMM -- bf16, 2.5 MB) instead of regenerated in every GEMM tile that reads it.
// Same mask, same fp32 product; the bf16 form is exactly what the GEMMs' fp32 loads rounded
// the fp32 form to.  One thread per 4 consecutive elements = one Philox draw (K % 4 == 0).
namespace {
__device__ __forceinline__ void store4(float* out, long e, float4 x) { *(float4*)(out + e) = x; }
__device__ __forceinline__ void store4(bf16* out, long e, float4 x) {
  *(bf16x4*)(out + e) = bf16x4{f2bf(x.x), f2bf(x.y), f2bf(x.z), f2bf(x.w)};
}
template <typename OutT>
__global__ __launch_bounds__(256) void gather_dropout_kernel(const float* __restrict__ v, const int* __restrict__ idx,
                                                             OutT* __restrict__ out, int M, int K, float p,
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
  store4(out, e, x);
}
}  // namespace

extern "C" int fr_gather_dropout(const float* v, const int* idx, void* out, int out_bf16, int M, int K, float p,
                                 unsigned long long seed, unsigned long long offset, const unsigned long long* dev_off,
                                 hipStream_t s) {
  if (K % 4 != 0 || M < 0) return 1;
  const long n4 = (long)M * K / 4;
  if (n4 == 0) return 0;
  const dim3 grid((unsigned)((n4 + 255) / 256));
  if (out_bf16)
    hipLaunchKernelGGL(gather_dropout_kernel<bf16>, grid, dim3(256), 0, s, v, idx, (bf16*)out, M, K, p, seed, offset,
                       dev_off);
  else
    hipLaunchKernelGGL(gather_dropout_kernel<float>, grid, dim3(256), 0, s, v, idx, (float*)out, M, K, p, seed, offset,
                       dev_off);
  return 0;
}
