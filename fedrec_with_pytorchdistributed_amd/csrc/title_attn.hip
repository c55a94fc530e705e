// DistilBERT self-attention over news titles, eval mode, on MFMA.
//
// One wave owns one (title, head): T <= 64 title tokens (50 in MIND shards, padded to 64),
// head dim 64.  Everything for the pair stays in registers except V, which is staged
// through LDS so the P.V MFMA can read it transposed with ds_read_b64_tr_b16.
//
//   S^T = K . Q^T          16x16x32 bf16 MFMA, K as the A operand, Q as B (both read as
//                          16 contiguous bytes per lane straight from the fused qkv buffer);
//                          the accumulator gives each lane one query column t and 16 keys
//   softmax over keys      per lane + two xor-shuffles (lanes l, l^16, l^32, l^48 share t);
//                          HF semantics: padded keys (mask 0) score finfo.min, so an all-zero
//                          mask (news row 0) yields a uniform distribution over the T keys;
//                          keys >= T (tile padding) are excluded (-inf)
//   O^T = V^T . P^T        P re-used from the S^T accumulator layout as the B operand: the
//                          k order inside a 32-key step is permuted (keys 4g..4g+3 and
//                          16+4g..16+4g+3 for lane group g) and the V fragment is read with
//                          the SAME permutation through two transposed LDS reads
//                          (cdna_hip_programming.md §3 "accumulator as the next operand")
//
// qkv: [n*T, 3*D] bf16 (q | k | v, head h at columns h*64 of each part); mask: [n, T] int32;
// out: [n*T, D] bf16.
#include "common.h"

namespace {

constexpr int DH = 64;

// DROP: HF attention-probability dropout (train mode): P_ts *= keep(pair, t, s) / (1 - p) with the
// Philox mask of element ((pair * 64 + t) * 64 + s) -- title_attn_bwd.hip regenerates it
template <int NWAVE, bool DROP>
__global__ __launch_bounds__(64 * NWAVE) void title_attn_kernel(const bf16* __restrict__ qkv, const int* __restrict__ mask,
                                                                bf16* __restrict__ out, int n_titles, int T, int H, int D,
                                                                float pdrop, unsigned long long seed,
                                                                unsigned long long offset) {
  __shared__ __attribute__((aligned(16))) bf16 vs[NWAVE][64 * DH];  // 8 KB per wave
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pair = blockIdx.x * NWAVE + wave;
  const bool active = pair < n_titles * H;
  const int title = active ? pair / H : 0;
  const int h = active ? pair - title * H : 0;
  const size_t row0 = (size_t)title * T;
  const int ld = 3 * D;
  const bf16* qb = qkv + row0 * ld + h * DH;
  const bf16* kb = qb + D;
  const bf16* vb = qb + 2 * D;
  bf16* myv = vs[wave];

  // ---- V -> LDS (rows >= T zero: P is 0 there, but 0 * garbage could be NaN) ----
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int idx = c * 64 + lane;
    const int r = idx >> 3, ch = idx & 7;
    bf16x8 val;
    if (r < T) val = *(const bf16x8*)(vb + (size_t)r * ld + ch * 8);
    else val = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    *(bf16x8*)(myv + r * DH + ch * 8) = val;
  }

  const int fr = lane & 15, fq = lane >> 4;
  // ---- S^T = K Q^T ----
  f32x4 st[4][4];
#pragma unroll
  for (int is = 0; is < 4; ++is)
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) st[is][jq] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kd = 0; kd < 2; ++kd) {
    bf16x8 kf[4], qf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int r = i * 16 + fr;
      r = r < T ? r : T - 1;
      kf[i] = *(const bf16x8*)(kb + (size_t)r * ld + kd * 32 + fq * 8);
      qf[i] = *(const bf16x8*)(qb + (size_t)r * ld + kd * 32 + fq * 8);
    }
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int jq = 0; jq < 4; ++jq) st[is][jq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[is], qf[jq], st[is][jq], 0, 0, 0);
  }

  // ---- masked softmax over keys s = 16 is + 4 fq + r, for query t = 16 jq + fr ----
  const float scale = 0.125f;  // 1/sqrt(64)
  // the title's key mask as one 64-bit ballot (one coalesced load instead of 16 per lane)
  const unsigned long long mbits = __ballot(lane < T && mask[row0 + (lane < T ? lane : 0)] != 0);
  float kadd[4][4];            // 0 (valid), -FLT_MAX (masked, HF finfo.min), -inf (tile padding)
#pragma unroll
  for (int is = 0; is < 4; ++is)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = is * 16 + fq * 4 + r;
      kadd[is][r] = (s < T) ? (((mbits >> s) & 1ull) ? 0.f : -3.4028234663852886e38f) : -INFINITY;
    }
  bf16x8 pf[4][2];
#pragma unroll
  for (int jq = 0; jq < 4; ++jq) {
    float m = -INFINITY;
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = kadd[is][r];
        const float sc = (a == 0.f) ? st[is][jq][r] * scale : a;
        st[is][jq][r] = sc;
        m = fmaxf(m, sc);
      }
    m = group4_max(m);
    float l = 0.f;
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(st[is][jq][r] - m);
        st[is][jq][r] = p;
        l += p;
      }
    l = group4_sum(l);
    const float inv = 1.0f / l;
    if constexpr (DROP) {
      const float inv_keep = 1.0f / (1.0f - pdrop);
      const int t = jq * 16 + fr;
#pragma unroll
      for (int is = 0; is < 4; ++is) {
        const uint4 rnd = Philox::gen(seed, offset, ((unsigned long long)pair * 64 + t) * 16 + is * 4 + fq);
#pragma unroll
        for (int r = 0; r < 4; ++r) st[is][jq][r] *= drop_scale(u4_get(rnd, r), pdrop, inv_keep);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        f[r] = f2bf(st[2 * ks][jq][r] * inv);
        f[4 + r] = f2bf(st[2 * ks + 1][jq][r] * inv);
      }
      pf[jq][ks] = f;
    }
  }

  // make this wave's V image visible to all its lanes
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();

  // ---- O = P V ----
  f32x4 o[4][4];
#pragma unroll
  for (int jq = 0; jq < 4; ++jq)
#pragma unroll
    for (int jd = 0; jd < 4; ++jd) o[jq][jd] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qq = fr >> 2, pp = fr & 3;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int jd = 0; jd < 4; ++jd) {
      const bf16* a0 = myv + (ks * 32 + fq * 4 + qq) * DH + jd * 16 + pp * 4;
      const bf16* a1 = a0 + 16 * DH;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
      bf16x4 lob = __builtin_bit_cast(bf16x4, lo), hib = __builtin_bit_cast(bf16x4, hi);
      bf16x8 vf = {lob[0], lob[1], lob[2], lob[3], hib[0], hib[1], hib[2], hib[3]};
#pragma unroll
      for (int jq = 0; jq < 4; ++jq) o[jq][jd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[jq][ks], o[jq][jd], 0, 0, 0);
    }
  }
  if (!active) return;
  // ---- store: O^T accumulators (V as the A operand) -> lane holds O[t = 16 jq + fr][d = 16 jd
  // + 4 fq + r], 4 consecutive d -> one 8-byte store per (jq, jd) ----
  bf16* ob = out + row0 * D + h * DH;
#pragma unroll
  for (int jq = 0; jq < 4; ++jq) {
    const int t = jq * 16 + fr;
    if (t < T) {
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) {
        const bf16x4 v = {f2bf(o[jq][jd][0]), f2bf(o[jq][jd][1]), f2bf(o[jq][jd][2]), f2bf(o[jq][jd][3])};
        *(bf16x4*)(ob + (size_t)t * D + jd * 16 + fq * 4) = v;
      }
    }
  }
}

// Persistent form: a fixed grid of waves walks the (title, head) pairs with stride; the next
// pair's K/Q fragments, V rows and mask are loaded into registers while the current pair's
// softmax and P.V run, so every wave keeps one pair's ~19 KB in flight at all times (the
// one-shot kernel above spends ~2/3 of each wave's life waiting for its loads).
struct TAIn {
  bf16x8 kf[2][4], qf[2][4], vv[8];
  int mbit;
};

// K/Q fragments + mask of `pair` (issued right after the S MFMAs have read the previous ones)
__device__ __forceinline__ void ta_load_kq(TAIn& in, const bf16* __restrict__ qkv, const int* __restrict__ mask,
                                           int pair, int T, int H, int D, int lane) {
  const int title = pair / H, h = pair - title * H;
  const int ld = 3 * D;
  const bf16* qb = qkv + (size_t)title * T * ld + h * DH;
  const bf16* kb = qb + D;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int kd = 0; kd < 2; ++kd)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int r = i * 16 + fr;
      r = r < T ? r : T - 1;
      in.kf[kd][i] = *(const bf16x8*)(kb + r * ld + kd * 32 + fq * 8);
      in.qf[kd][i] = *(const bf16x8*)(qb + r * ld + kd * 32 + fq * 8);
    }
  in.mbit = mask[(size_t)title * T + (lane < T ? lane : 0)];
}

// V rows of `pair` (issued once the softmax no longer holds the score registers)
__device__ __forceinline__ void ta_load_v(TAIn& in, const bf16* __restrict__ qkv, int pair, int T, int H, int D,
                                          int lane) {
  const int title = pair / H, h = pair - title * H;
  const int ld = 3 * D;
  const bf16* vb = qkv + (size_t)title * T * ld + 2 * D + h * DH;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int idx = c * 64 + lane;
    int r = idx >> 3;
    r = r < T ? r : T - 1;  // rows >= T are zeroed when written to LDS
    in.vv[c] = *(const bf16x8*)(vb + r * ld + (idx & 7) * 8);
  }
}

// DROP: the train-mode forward (attention-probability dropout, the same Philox element index as
// title_attn_kernel<.., true>, so title_attn_bwd.hip regenerates the identical mask)
template <int OCC, int DEPTH, bool DROP = false>
__global__ __launch_bounds__(256, OCC) void title_attn_pkernel(const bf16* __restrict__ qkv, const int* __restrict__ mask,
                                                          bf16* __restrict__ out, int n_pairs, int T, int H, int D,
                                                          float pdrop = 0.f, unsigned long long seed = 0ull,
                                                          unsigned long long offset = 0ull) {
  __shared__ __attribute__((aligned(16))) bf16 vs[4][64 * DH];
  // wave index via readfirstlane: the compiler then knows pair / next are wave-uniform, so the
  // prefetch guards are scalar branches (a "divergent" guard around loads makes it drain
  // vmcnt(0) at the loop head and the 2-deep prefetch stops overlapping anything)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int stride = gridDim.x * 4;
  int pair = blockIdx.x * 4 + wave;
  if (pair >= n_pairs) return;
  bf16* myv = vs[wave];
  const int fr = lane & 15, fq = lane >> 4;
  const int qq = fr >> 2, pp = fr & 3;
  // one pair: consumes `in`, then refills it with the pair DEPTH strides ahead
  auto step = [&](TAIn& in, int pair) {
    const int title = pair / H, h = pair - title * H;
    const size_t row0 = (size_t)title * T;
    // V -> LDS (the previous pair's transposed reads were consumed by its MFMAs)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int idx = c * 64 + lane;
      const int r = idx >> 3;
      *(bf16x8*)(myv + r * DH + (idx & 7) * 8) = r < T ? in.vv[c] : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    const unsigned long long mbits = __ballot(lane < T && in.mbit != 0);
    f32x4 st[4][4];
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int jq = 0; jq < 4; ++jq) st[is][jq] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kd = 0; kd < 2; ++kd)
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int jq = 0; jq < 4; ++jq)
          st[is][jq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(in.kf[kd][is], in.qf[kd][jq], st[is][jq], 0, 0, 0);
    // prefetch the next pair (its registers are free once the S MFMAs have read them)
    const int next = pair + DEPTH * stride;
    if (next < n_pairs) ta_load_kq(in, qkv, mask, next, T, H, D, lane);

    const float scale = 0.125f;
    bf16x8 pf[4][2];
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) {
      float m = -INFINITY;
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int sidx = is * 16 + fq * 4 + r;
          const float a = (sidx < T) ? (((mbits >> sidx) & 1ull) ? 0.f : -3.4028234663852886e38f) : -INFINITY;
          const float sc = (a == 0.f) ? st[is][jq][r] * scale : a;
          st[is][jq][r] = sc;
          m = fmaxf(m, sc);
        }
      m = group4_max(m);
      float l = 0.f;
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __expf(st[is][jq][r] - m);
          st[is][jq][r] = e;
          l += e;
        }
      const float inv = 1.0f / group4_sum(l);
      if constexpr (DROP) {
        const float inv_keep = 1.0f / (1.0f - pdrop);
        const int t = jq * 16 + fr;
#pragma unroll
        for (int is = 0; is < 4; ++is) {
          const uint4 rnd = Philox::gen(seed, offset, ((unsigned long long)pair * 64 + t) * 16 + is * 4 + fq);
#pragma unroll
          for (int r = 0; r < 4; ++r) st[is][jq][r] *= drop_scale(u4_get(rnd, r), pdrop, inv_keep);
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f[r] = f2bf(st[2 * ks][jq][r] * inv);
          f[4 + r] = f2bf(st[2 * ks + 1][jq][r] * inv);
        }
        pf[jq][ks] = f;
      }
    }
    if (next < n_pairs) ta_load_v(in, qkv, next, T, H, D, lane);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's V image is in LDS
    __builtin_amdgcn_wave_barrier();
    f32x4 o[4][4];
#pragma unroll
    for (int jq = 0; jq < 4; ++jq)
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) o[jq][jd] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) {
        const bf16* a0 = myv + (ks * 32 + fq * 4 + qq) * DH + jd * 16 + pp * 4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0 + 16 * DH));
        bf16x4 lob = __builtin_bit_cast(bf16x4, lo), hib = __builtin_bit_cast(bf16x4, hi);
        bf16x8 vf = {lob[0], lob[1], lob[2], lob[3], hib[0], hib[1], hib[2], hib[3]};
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) o[jq][jd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[jq][ks], o[jq][jd], 0, 0, 0);
      }
    bf16* ob = out + row0 * D + h * DH;
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) {
      const int t = jq * 16 + fr;
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        const float v0[4] = {o[jq][2 * p2][0], o[jq][2 * p2][1], o[jq][2 * p2][2], o[jq][2 * p2][3]};
        const float v1[4] = {o[jq][2 * p2 + 1][0], o[jq][2 * p2 + 1][1], o[jq][2 * p2 + 1][2], o[jq][2 * p2 + 1][3]};
        store_pair16_if(ob + (size_t)(t < T ? t : 0) * D + p2 * 32, v0, v1, fq, t < T);
      }
    }
  };
  TAIn in0, in1;
  ta_load_kq(in0, qkv, mask, pair, T, H, D, lane);
  ta_load_v(in0, qkv, pair, T, H, D, lane);
  if (DEPTH == 2 && pair + stride < n_pairs) {
    ta_load_kq(in1, qkv, mask, pair + stride, T, H, D, lane);
    ta_load_v(in1, qkv, pair + stride, T, H, D, lane);
  }
  while (true) {
    step(in0, pair);
    pair += stride;
    if (pair >= n_pairs) break;
    // the next pair overwrites this wave's V image: its transposed reads must be done
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    if (DEPTH == 2) {
      step(in1, pair);
      pair += stride;
      if (pair >= n_pairs) break;
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// ---------------------------------------------------------------------------------------
// Packed-row layout (frozen backbone forward).  The n*T token rows of a batch are reordered
// so that every row the attention reads as a key/value ("kv rows": mask 1, or every row of an
// all-masked title) comes first, title-major and in position order, followed by the
// query-only rows (mask 0).  Only the kv rows need K and V, so the fused QKV GEMM computes
// all 3*D columns for them and only the Q columns for the rest (~2/3 of MIND title tokens
// are padding).  Attention has no positional term, so permuting its keys changes nothing;
// positions enter through the embedding, which reads each row's source index.
//
// title_count_kernel: one wave per title, kv_len[i] = popcount of its mask (-T if all
// masked).  title_rows_kernel: 16 titles per block; the block first reduces kv counts over
// all titles (its prefix and the total R; n ints from L2, no separate scan pass), then each
// wave assigns its title's rows from ballot ranks: rowmap[i*T + t] (packed row of token t
// of title i), its inverse src, and kv_start[i].  kv_len[i] < 0 marks an all-masked title
// (HF: uniform attention over all T keys); qstart[i] = the title's first query-only row.
__global__ __launch_bounds__(256) void title_count_kernel(const int* __restrict__ mask, int n, int T,
                                                          int* __restrict__ kv_len) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const unsigned long long b = __ballot(lane < T && mask[(size_t)i * T + (lane < T ? lane : 0)] != 0);
  const int c = __popcll(b);
  if (lane == 0) kv_len[i] = c == 0 ? -T : c;
}

__global__ __launch_bounds__(1024) void title_rows_kernel(const int* __restrict__ mask, int n, int T,
                                                          const int* __restrict__ kv_len, int* __restrict__ rowmap,
                                                          int* __restrict__ src, int* __restrict__ kv_start,
                                                          int* __restrict__ qstart, int* __restrict__ n_kv) {
  __shared__ int red[3][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i0 = blockIdx.x * 16;
  int pre = 0, tot = 0;
  for (int j = tid; j < n; j += 1024) {
    const int c = abs(kv_len[j]);
    tot += c;
    pre += j < i0 ? c : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    pre += __shfl_xor(pre, o, 64);
    tot += __shfl_xor(tot, o, 64);
  }
  const int i = i0 + wave;
  const int kl = i < n ? kv_len[i] : 0;
  if (lane == 0) {
    red[0][wave] = pre;
    red[1][wave] = tot;
    red[2][wave] = abs(kl);  // this block's titles, for the in-block prefix
  }
  __syncthreads();
  pre = 0;
  tot = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    pre += red[0][w] + (w < wave ? red[2][w] : 0);
    tot += red[1][w];
  }
  if (blockIdx.x == 0 && tid == 0) *n_kv = tot;
  if (i >= n) return;
  const bool in = lane < T;
  const bool kv = in && (kl < 0 || mask[(size_t)i * T + (in ? lane : 0)] != 0);
  const unsigned long long b = __ballot(kv);
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int rk = __popcll(b & below);
  const int row = kv ? pre + rk : tot + i * T - pre + (lane - rk);
  if (in) {
    rowmap[(size_t)i * T + lane] = row;
    src[row] = i * T + lane;
  }
  if (lane == 0) {
    kv_start[i] = pre;
    qstart[i] = tot + i * T - pre;
  }
}

struct TPIn {
  bf16x8 kf[2][4], qf[2][4], vv[8];
  int qrow[4];
  int kstart, klen;  // klen < 0: all-masked title, uniform over -klen keys
};

__device__ __forceinline__ void tp_load_kq(TPIn& in, const bf16* __restrict__ qkv, const int* __restrict__ rowmap,
                                           const int* __restrict__ kv_start, const int* __restrict__ kv_len,
                                           const int* __restrict__ qstart, int pair, int T, int H, int D, int lane) {
  const int title = pair / H, h = pair - title * H;
  const int ld = 3 * D;
  const int fr = lane & 15, fq = lane >> 4;
  in.kstart = kv_start[title];
  in.klen = kv_len[title];
  const int qs = qstart[title];
  const int nk = in.klen < 0 ? -in.klen : in.klen;
  // the title's T rows are its kv rows [kstart, +nk) and its query-only rows [qs, +T-nk); the
  // j-th query is the j-th of those rows (attention is order-free over queries too: each
  // output goes to its own packed row), so no rowmap load precedes the Q loads.  Every load
  // is unconditional (rows clamped): a load under a lane predicate makes the compiler drain
  // vmcnt(0) at the loop head and the prefetch pipeline stalls.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int t = i * 16 + fr;
    t = t < T ? t : T - 1;
    in.qrow[i] = t < nk ? in.kstart + t : qs + (t - nk);
  }
  const bf16* qb = qkv + h * DH;
  const bf16* kb = qkv + D + h * DH;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int sk = i * 16 + fr;
    const size_t krow = (size_t)in.kstart + (sk < nk ? sk : nk - 1);
#pragma unroll
    for (int kd = 0; kd < 2; ++kd) {
      in.kf[kd][i] = *(const bf16x8*)(kb + krow * ld + kd * 32 + fq * 8);
      in.qf[kd][i] = *(const bf16x8*)(qb + (size_t)in.qrow[i] * ld + kd * 32 + fq * 8);
    }
  }
}

__device__ __forceinline__ void tp_load_v(TPIn& in, const bf16* __restrict__ qkv, int pair, int H, int D, int lane) {
  const int h = pair % H;
  const int ld = 3 * D;
  const int nk = in.klen < 0 ? -in.klen : in.klen;
  const bf16* vb = qkv + 2 * D + h * DH;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int idx = c * 64 + lane;
    const int r = idx >> 3;
    in.vv[c] = *(const bf16x8*)(vb + ((size_t)in.kstart + (r < nk ? r : nk - 1)) * ld + (idx & 7) * 8);
  }
}

// Persistent 2-deep prefetching form (as title_attn_pkernel) over the packed rows; key tiles
// of 16 beyond the title's kv count are skipped (a MIND title has ~16 real tokens: 1 of the
// 4 key tiles, 1 of the 2 P.V k-steps).
__global__ __launch_bounds__(256, 1) void title_attn_packed_kernel(const bf16* __restrict__ qkv,
                                                                   const int* __restrict__ rowmap,
                                                                   const int* __restrict__ kv_start,
                                                                   const int* __restrict__ kv_len,
                                                                   const int* __restrict__ qstart,
                                                                   bf16* __restrict__ out, int n_pairs, int T, int H,
                                                                   int D) {
  __shared__ __attribute__((aligned(16))) bf16 vs[4][64 * DH];
  // wave index via readfirstlane: the compiler then knows pair / next are wave-uniform, so the
  // prefetch guards are scalar branches (a "divergent" guard around loads makes it drain
  // vmcnt(0) at the loop head and the 2-deep prefetch stops overlapping anything)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int stride = gridDim.x * 4;
  int pair = blockIdx.x * 4 + wave;
  if (pair >= n_pairs) return;
  bf16* myv = vs[wave];
  const int fr = lane & 15, fq = lane >> 4;
  const int qq = fr >> 2, pp = fr & 3;
  auto step = [&](TPIn& in, int pair) {
    const int h = pair % H;
    const int klen = in.klen, nk = klen < 0 ? -klen : klen;
    const bool allm = klen < 0;
    const int nks = (nk + 15) >> 4;  // 16-key tiles in use (wave-uniform)
    int qrow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) qrow[i] = in.qrow[i];
#pragma unroll
    for (int c = 0; c < 8; ++c) {  // V rows past the title's keys are zero (P is 0 there, 0 * x may be NaN)
      const int idx = c * 64 + lane;
      *(bf16x8*)(myv + (idx >> 3) * DH + (idx & 7) * 8) = (idx >> 3) < nk ? in.vv[c] : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    f32x4 st[4][4];
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int jq = 0; jq < 4; ++jq) st[is][jq] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kd = 0; kd < 2; ++kd)
#pragma unroll
      for (int is = 0; is < 4; ++is)
        if (is < nks) {
#pragma unroll
          for (int jq = 0; jq < 4; ++jq)
            st[is][jq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(in.kf[kd][is], in.qf[kd][jq], st[is][jq], 0, 0, 0);
        }
    // prefetch 2 strides ahead, unconditionally (clamped to the last pair: a conditional load
    // leaves the waitcnt pass a path with fewer loads in flight and it drains to vmcnt(0))
    const int next = min(pair + 2 * stride, n_pairs - 1);
    tp_load_kq(in, qkv, rowmap, kv_start, kv_len, qstart, next, T, H, D, lane);

    const float scale = 0.125f;
    bf16x8 pf[4][2];
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) {
      float m = -INFINITY;
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int sidx = is * 16 + fq * 4 + r;
          const float a = sidx < nk ? (allm ? -3.4028234663852886e38f : 0.f) : -INFINITY;
          const float sc = (a == 0.f) ? st[is][jq][r] * scale : a;
          st[is][jq][r] = sc;
          m = fmaxf(m, sc);
        }
      m = group4_max(m);
      float l = 0.f;
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __expf(st[is][jq][r] - m);
          st[is][jq][r] = e;
          l += e;
        }
      const float inv = 1.0f / group4_sum(l);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f[r] = f2bf(st[2 * ks][jq][r] * inv);
          f[4 + r] = f2bf(st[2 * ks + 1][jq][r] * inv);
        }
        pf[jq][ks] = f;
      }
    }
    tp_load_v(in, qkv, next, H, D, lane);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's V image is in LDS
    __builtin_amdgcn_wave_barrier();
    f32x4 o[4][4];
#pragma unroll
    for (int jq = 0; jq < 4; ++jq)
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) o[jq][jd] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      if (ks * 32 < nk) {
#pragma unroll
        for (int jd = 0; jd < 4; ++jd) {
          const bf16* a0 = myv + (ks * 32 + fq * 4 + qq) * DH + jd * 16 + pp * 4;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0 + 16 * DH));
          bf16x4 lob = __builtin_bit_cast(bf16x4, lo), hib = __builtin_bit_cast(bf16x4, hi);
          bf16x8 vf = {lob[0], lob[1], lob[2], lob[3], hib[0], hib[1], hib[2], hib[3]};
#pragma unroll
          for (int jq = 0; jq < 4; ++jq)
            o[jq][jd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[jq][ks], o[jq][jd], 0, 0, 0);
        }
      }
    bf16* ob = out + h * DH;
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) {
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        const float v0[4] = {o[jq][2 * p2][0], o[jq][2 * p2][1], o[jq][2 * p2][2], o[jq][2 * p2][3]};
        const float v1[4] = {o[jq][2 * p2 + 1][0], o[jq][2 * p2 + 1][1], o[jq][2 * p2 + 1][2], o[jq][2 * p2 + 1][3]};
        // t >= T lanes hold the clamped query T-1: they store the same values to the same row,
        // so the stores need no lane predicate (a predicated store is a divergent branch)
        store_pair16_if(ob + (size_t)qrow[jq] * D + p2 * 32, v0, v1, fq, true);
      }
    }
  };
  TPIn in0, in1;
  tp_load_kq(in0, qkv, rowmap, kv_start, kv_len, qstart, pair, T, H, D, lane);
  tp_load_v(in0, qkv, pair, H, D, lane);
  const int p1 = min(pair + stride, n_pairs - 1);
  tp_load_kq(in1, qkv, rowmap, kv_start, kv_len, qstart, p1, T, H, D, lane);
  tp_load_v(in1, qkv, p1, H, D, lane);
  while (true) {
    step(in0, pair);
    pair += stride;
    if (pair >= n_pairs) break;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    step(in1, pair);
    pair += stride;
    if (pair >= n_pairs) break;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
  }
}

int g_ta_waves = -2;  // default: persistent, 2-deep prefetch, 1 wave per SIMD (kernel_bench.py)
int g_ta_cus = 0;

}  // namespace

extern "C" void fr_title_attn_set_waves(int w) { g_ta_waves = w; }

extern "C" int fr_title_attention_long_bf16(const void* qkv, const int* mask, void* out, int n_titles, int T, int H,
                                            int D, hipStream_t s);  // title_attn_long.hip, 64 < T <= 512

extern "C" int fr_title_attention_bf16(const void* qkv, const int* mask, void* out, int n_titles, int T, int H, int D,
                                       hipStream_t s) {
  if (T > 64) return fr_title_attention_long_bf16(qkv, mask, out, n_titles, T, H, D, s);
  if (T < 1 || D != H * DH) return 1;
  const int pairs = n_titles * H;
  if (pairs == 0) return 0;
  const int w = g_ta_waves;
  if (w <= 0) {  // persistent, prefetching: w = 0 -> 2 waves/SIMD (spills a little), w = -1 -> 1 wave/SIMD
    if (g_ta_cus == 0) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&g_ta_cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (g_ta_cus <= 0) g_ta_cus = 256;
    }
    int blocks = g_ta_cus * (w == 0 ? 2 : 1);
    const int need = (pairs + 3) / 4;
    blocks = blocks < need ? blocks : need;
    if (w == -2)
      hipLaunchKernelGGL((title_attn_pkernel<1, 2>), dim3(blocks), dim3(256), 0, s, (const bf16*)qkv, mask, (bf16*)out, pairs,
                         T, H, D);
    else if (w == 0)
      hipLaunchKernelGGL((title_attn_pkernel<2, 1>), dim3(blocks), dim3(256), 0, s, (const bf16*)qkv, mask, (bf16*)out, pairs, T,
                         H, D);
    else
      hipLaunchKernelGGL((title_attn_pkernel<1, 1>), dim3(blocks), dim3(256), 0, s, (const bf16*)qkv, mask, (bf16*)out, pairs, T,
                         H, D);
  } else if (w == 1)
    hipLaunchKernelGGL((title_attn_kernel<1, false>), dim3(pairs), dim3(64), 0, s, (const bf16*)qkv, mask, (bf16*)out,
                       n_titles, T, H, D, 0.f, 0ull, 0ull);
  else if (w == 4)
    hipLaunchKernelGGL((title_attn_kernel<4, false>), dim3((pairs + 3) / 4), dim3(256), 0, s, (const bf16*)qkv, mask,
                       (bf16*)out, n_titles, T, H, D, 0.f, 0ull, 0ull);
  else
    hipLaunchKernelGGL((title_attn_kernel<2, false>), dim3((pairs + 1) / 2), dim3(128), 0, s, (const bf16*)qkv, mask,
                       (bf16*)out, n_titles, T, H, D, 0.f, 0ull, 0ull);
  return 0;
}

// train-mode forward with attention-probability dropout (T <= 64; 2 = unsupported shape)
extern "C" int fr_title_attention_drop_bf16(const void* qkv, const int* mask, void* out, int n_titles, int T, int H,
                                            int D, float pdrop, unsigned long long seed, unsigned long long offset,
                                            hipStream_t s) {
  if (T < 1 || T > 64 || D != H * DH || !(pdrop > 0.f && pdrop < 1.f)) return 2;
  const int pairs = n_titles * H;
  if (pairs == 0) return 0;
  if (g_ta_waves == -2) {  // persistent 2-deep prefetching form (default), as the eval forward
    if (g_ta_cus == 0) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&g_ta_cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (g_ta_cus <= 0) g_ta_cus = 256;
    }
    const int need = (pairs + 3) / 4;
    const int blocks = g_ta_cus < need ? g_ta_cus : need;
    hipLaunchKernelGGL((title_attn_pkernel<1, 2, true>), dim3(blocks), dim3(256), 0, s, (const bf16*)qkv, mask,
                       (bf16*)out, pairs, T, H, D, pdrop, seed, offset);
    return 0;
  }
  hipLaunchKernelGGL((title_attn_kernel<2, true>), dim3((pairs + 1) / 2), dim3(128), 0, s, (const bf16*)qkv, mask,
                     (bf16*)out, n_titles, T, H, D, pdrop, seed, offset);
  return 0;
}

extern "C" int fr_title_plan(const int* mask, int n, int T, int* rowmap, int* src, int* kv_start, int* kv_len,
                             int* qstart, int* n_kv, hipStream_t s) {
  if (T < 1 || T > 64 || n < 0) return 1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(title_count_kernel, dim3((n + 3) / 4), dim3(256), 0, s, mask, n, T, kv_len);
  hipLaunchKernelGGL(title_rows_kernel, dim3((n + 15) / 16), dim3(1024), 0, s, mask, n, T, kv_len, rowmap, src, kv_start,
                     qstart, n_kv);
  return 0;
}

// qkv: [n*T, 3*D] in packed row order (K/V columns valid on kv rows only); out: [n*T, D]
// in packed row order.
extern "C" int fr_title_attention_packed_bf16(const void* qkv, const int* rowmap, const int* kv_start, const int* kv_len,
                                              const int* qstart, void* out, int n_titles, int T, int H, int D,
                                              hipStream_t s) {
  if (T < 1 || T > 64 || D != H * DH) return 1;
  const int pairs = n_titles * H;
  if (pairs == 0) return 0;
  if (g_ta_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_ta_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_ta_cus <= 0) g_ta_cus = 256;
  }
  int blocks = g_ta_cus;
  const int need = (pairs + 3) / 4;
  blocks = blocks < need ? blocks : need;
  hipLaunchKernelGGL(title_attn_packed_kernel, dim3(blocks), dim3(256), 0, s, (const bf16*)qkv, rowmap, kv_start, kv_len,
                     qstart, (bf16*)out, pairs, T, H, D);
  return 0;
}
