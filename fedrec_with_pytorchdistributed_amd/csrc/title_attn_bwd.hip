// Backward of the DistilBERT title self-attention (unfrozen backbone, BASELINE config 5).
//
// One wave per (title, head), T <= 64, head dim 64, everything recomputed from qkv (no
// stored probabilities -- the forward never writes P):
//
//   S^T = K Q^T / 8  -> masked softmax -> P^T        (as the forward; lane = query column)
//   dP^T = V dO^T                                    (same MFMA layout as S^T)
//   D_t  = sum_s P_ts dP_ts ;  dS_ts = keep_s * P_ts (dP_ts - D_t) / 8
//   dQ = dS K          A operand straight from the dS^T registers (k permuted as in the
//                      forward's P.V), B = K by transposed LDS reads
//   dV = P^T dO, dK = dS^T Q
//                      A operand = P^T / dS^T rows: written once to LDS as bf16 [s][t] and
//                      read back with ds_read_b128; B = dO / Q by transposed LDS reads
//
// HF masked_fill semantics: a masked key's score is a constant, so its dS is exactly 0 (the
// all-masked <unk> row still passes gradient to V through its uniform P).
// qkv/dqkv: [n*T, 3*D] bf16; dout: [n*T, D] bf16; mask: [n, T] int32.
#include "common.h"

namespace {

constexpr int DH = 64;
constexpr int WPB = 2;  // waves per block (32 KB LDS per wave)

__device__ __forceinline__ bf16x8 tr_pair(const bf16* base_lo, const bf16* base_hi) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base_lo));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base_hi));
  bf16x4 a = __builtin_bit_cast(bf16x4, lo), b = __builtin_bit_cast(bf16x4, hi);
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// DROP: the forward applied P~ = P o Z (Z = keep / (1 - p), title_attn.hip's Philox mask), so
// dP = (dO V^T) o Z, D_t = sum_s P_ts dP_ts, dS as below, and dV = P~^T dO
template <bool DROP>
__global__ __launch_bounds__(64 * WPB) void title_attn_bwd_kernel(const bf16* __restrict__ qkv,
                                                                  const bf16* __restrict__ dout,
                                                                  const int* __restrict__ mask,
                                                                  bf16* __restrict__ dqkv, int n_titles, int T, int H,
                                                                  int D, float pdrop, unsigned long long seed,
                                                                  unsigned long long offset) {
  __shared__ __attribute__((aligned(16))) bf16 lds[WPB][4][64 * DH];  // Q, K, dO, P^T/dS^T scratch
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pair = blockIdx.x * WPB + wave;
  const bool active = pair < n_titles * H;
  const int title = active ? pair / H : 0;
  const int h = active ? pair - title * H : 0;
  const size_t row0 = (size_t)title * T;
  const int ld = 3 * D;
  const bf16* qb = qkv + row0 * ld + h * DH;
  const bf16* kb = qb + D;
  const bf16* vb = qb + 2 * D;
  const bf16* gb = dout + row0 * D + h * DH;
  bf16* Qs = lds[wave][0];
  bf16* Ks = lds[wave][1];
  bf16* Gs = lds[wave][2];
  bf16* Ps = lds[wave][3];
  // stage Q, K, dO row-major [64][64] (rows >= T zero)
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int idx = c * 64 + lane;
    const int r = idx >> 3, ch = idx & 7;
    const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool ok = r < T;
    *(bf16x8*)(Qs + r * DH + ch * 8) = ok ? *(const bf16x8*)(qb + (size_t)r * ld + ch * 8) : z;
    *(bf16x8*)(Ks + r * DH + ch * 8) = ok ? *(const bf16x8*)(kb + (size_t)r * ld + ch * 8) : z;
    *(bf16x8*)(Gs + r * DH + ch * 8) = ok ? *(const bf16x8*)(gb + (size_t)r * D + ch * 8) : z;
  }
  const int fr = lane & 15, fq = lane >> 4;
  // ---- S^T = K Q^T and dP^T = V dO^T ----
  f32x4 st[4][4], dp[4][4];
#pragma unroll
  for (int is = 0; is < 4; ++is)
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) st[is][jq] = dp[is][jq] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kd = 0; kd < 2; ++kd) {
    bf16x8 kf[4], qf[4], vf[4], gf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int r = i * 16 + fr;
      r = r < T ? r : T - 1;
      kf[i] = *(const bf16x8*)(kb + (size_t)r * ld + kd * 32 + fq * 8);
      qf[i] = *(const bf16x8*)(qb + (size_t)r * ld + kd * 32 + fq * 8);
      vf[i] = *(const bf16x8*)(vb + (size_t)r * ld + kd * 32 + fq * 8);
      gf[i] = *(const bf16x8*)(gb + (size_t)r * D + kd * 32 + fq * 8);
    }
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int jq = 0; jq < 4; ++jq) {
        st[is][jq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[is], qf[jq], st[is][jq], 0, 0, 0);
        dp[is][jq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[is], gf[jq], dp[is][jq], 0, 0, 0);
      }
  }
  // ---- softmax (forward recompute) and dS ----
  float keep[4][4], kadd[4][4];
#pragma unroll
  for (int is = 0; is < 4; ++is)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = is * 16 + fq * 4 + r;
      const bool valid = s < T;
      const bool on = valid && mask[row0 + s] != 0;
      keep[is][r] = on ? 1.f : 0.f;
      kadd[is][r] = valid ? (on ? 0.f : -3.4028234663852886e38f) : -INFINITY;
    }
  bf16x8 dsf[4][2];
#pragma unroll
  for (int jq = 0; jq < 4; ++jq) {
    float m = -INFINITY;
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sc = kadd[is][r] == 0.f ? st[is][jq][r] * 0.125f : kadd[is][r];
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
    float z[4][4];
#pragma unroll
    for (int is = 0; is < 4; ++is) {
      if constexpr (DROP) {
        const uint4 rnd = Philox::gen(seed, offset, ((unsigned long long)pair * 64 + jq * 16 + fr) * 16 + is * 4 + fq);
        const float inv_keep = 1.0f / (1.0f - pdrop);
#pragma unroll
        for (int r = 0; r < 4; ++r) z[is][r] = drop_scale(u4_get(rnd, r), pdrop, inv_keep);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) z[is][r] = 1.f;
      }
    }
    float dsum = 0.f;
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[is][jq][r] *= inv;
        if constexpr (DROP) dp[is][jq][r] *= z[is][r];
        dsum += st[is][jq][r] * dp[is][jq][r];
      }
    dsum = group4_sum(dsum);
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dp[is][jq][r] = keep[is][r] * st[is][jq][r] * (dp[is][jq][r] - dsum) * 0.125f;
        if constexpr (DROP) st[is][jq][r] *= z[is][r];  // P~ for dV
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        f[r] = f2bf(dp[2 * ks][jq][r]);
        f[4 + r] = f2bf(dp[2 * ks + 1][jq][r]);
      }
      dsf[jq][ks] = f;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
  const int qq = fr >> 2, pp = fr & 3;
  // ---- dQ = dS K (A from registers, B = K via transposed reads) ----
  f32x4 o[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) o[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int jd = 0; jd < 4; ++jd) {
      const bf16* a0 = Ks + (ks * 32 + fq * 4 + qq) * DH + jd * 16 + pp * 4;
      const bf16x8 kfr = tr_pair(a0, a0 + 16 * DH);
#pragma unroll
      // K^T as the A operand: the accumulator is dQ^T, so a lane holds 4 consecutive head
      // dims d = 16 jd + 4 fq + r of one query t = 16 jq + fr -> 16-byte stores below
      for (int jq = 0; jq < 4; ++jq) o[jq][jd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kfr, dsf[jq][ks], o[jq][jd], 0, 0, 0);
    }
  bf16* dq = dqkv + row0 * ld + h * DH;
  if (active) {
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) {
      const int t = jq * 16 + fr;  // lanes l and l^16 share t (the permlane16 pairs agree)
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        const float v0[4] = {o[jq][2 * p2][0], o[jq][2 * p2][1], o[jq][2 * p2][2], o[jq][2 * p2][3]};
        const float v1[4] = {o[jq][2 * p2 + 1][0], o[jq][2 * p2 + 1][1], o[jq][2 * p2 + 1][2], o[jq][2 * p2 + 1][3]};
        store_pair16_if(dq + (size_t)(t < T ? t : 0) * ld + p2 * 32, v0, v1, fq, t < T);
      }
    }
  }
  // ---- dV = P^T dO and dK = dS^T Q: A rows [s][t] via an LDS transpose of P^T / dS^T ----
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    // write X^T[s][t] (X = P for dV, dS for dK) as bf16 row-major [s][t]
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int jq = 0; jq < 4; ++jq)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = is * 16 + fq * 4 + r, t = jq * 16 + fr;
          Ps[s * 64 + t] = f2bf(pass == 0 ? st[is][jq][r] : dp[is][jq][r]);
        }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    const bf16* Bsrc = pass == 0 ? Gs : Qs;  // dO for dV, Q for dK
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) o[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(Ps + (i * 16 + fr) * 64 + kt * 32 + fq * 8);
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) {
        // B[k = t][d]: rows t = 32kt + 8fq + j  -> two transposed 4-row reads
        const bf16* b0 = Bsrc + (kt * 32 + fq * 8 + qq) * DH + jd * 16 + pp * 4;
        const bf16x8 bfr = tr_pair(b0, b0 + 4 * DH);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i][jd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr, af[i], o[i][jd], 0, 0, 0);
      }
    }
    bf16* dst = dqkv + row0 * ld + (pass == 0 ? 2 * D : D) + h * DH;
    if (active) {  // transposed accumulator: lane = key s = 16 i + fr, 4 consecutive d per (i, jd)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int sk = i * 16 + fr;
#pragma unroll
        for (int p2 = 0; p2 < 2; ++p2) {
          const float v0[4] = {o[i][2 * p2][0], o[i][2 * p2][1], o[i][2 * p2][2], o[i][2 * p2][3]};
          const float v1[4] = {o[i][2 * p2 + 1][0], o[i][2 * p2 + 1][1], o[i][2 * p2 + 1][2], o[i][2 * p2 + 1][3]};
          store_pair16_if(dst + (size_t)(sk < T ? sk : 0) * ld + p2 * 32, v0, v1, fq, sk < T);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------------------
// Persistent form (default).  The one-shot kernel above runs at 1 wave per SIMD (339
// VGPR+AGPR) with nothing in flight while a wave computes: every (title, head) pays the full
// global-load latency (~1.9 TB/s).  Here each wave walks (title, head) pairs with a grid
// stride and keeps the NEXT pair's Q / K / V / dO rows (and its mask) in flight in registers
// while it computes the current one from LDS.  All four operands are staged in LDS with a
// 16-byte XOR swizzle (chunk ^ row & 7), so the MFMA fragments come from ds_read_b128
// instead of a second round of global loads; V's buffer doubles as the P^T / dS^T scratch
// once dP^T is formed.  Same math, same outputs as title_attn_bwd_kernel.
struct TBIn {
  bf16x8 q[8], k[8], v[8], g[8];
  int mk;  // lane s: mask of key s (clamped row; s >= T is handled by the caller)
};

// element index of (row r, column c) in a swizzled [64][64] bf16 tile
__device__ __forceinline__ int swz(int r, int c) { return r * 64 + ((((c >> 3) ^ (r & 7)) << 3) | (c & 7)); }

template <int PART = 0>
__device__ __forceinline__ void tb_load(TBIn& in, const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                        const int* __restrict__ mask, int pair, int T, int H, int D, int lane) {
  const int title = pair / H, h = pair - title * H;
  const size_t row0 = (size_t)title * T;
  const int ld = 3 * D;
  const bf16* qb = qkv + row0 * ld + h * DH;
  const bf16* gb = dout + row0 * D + h * DH;
  const int part = PART;
#pragma unroll
  for (int c = 0; c < 8; ++c) {  // unconditional (rows clamped): see title_attn.hip on vmcnt drains
    const int idx = c * 64 + lane;
    int r = idx >> 3;
    r = r < T ? r : T - 1;
    const int ch = idx & 7;
    if (part != 2) {
      in.q[c] = *(const bf16x8*)(qb + (size_t)r * ld + ch * 8);
      in.k[c] = *(const bf16x8*)(qb + D + (size_t)r * ld + ch * 8);
    }
    if (part != 1) {
      in.v[c] = *(const bf16x8*)(qb + 2 * D + (size_t)r * ld + ch * 8);
      in.g[c] = *(const bf16x8*)(gb + (size_t)r * D + ch * 8);
    }
  }
  if (part != 2) in.mk = mask[row0 + (lane < T ? lane : T - 1)];
}

// DROP: as title_attn_bwd_kernel<true> (the forward's Philox mask regenerated per element,
// kept as 16-bit keep words per query: per-element scale arrays across the softmax spill).
// Reading keep bits stored by the forward instead (8 B per lane and pair) measured slower:
// 523 vs 437 us (profiles/r2_attn_drop_bits_bench.json) -- the bit unpacking spilled more.
// SPLIT: the next pair's Q / K are prefetched before dQ and its V / dO only after the dV pass,
// so half the staging registers are live through dQ / dV -- with DROP the Philox keep words
// otherwise push the kernel to 432 B/lane of spill (68 B with the split)
template <bool DROP, bool SPLIT = false>
__global__ __launch_bounds__(256, 1) void title_attn_bwd_pkernel(const bf16* __restrict__ qkv,
                                                                 const bf16* __restrict__ dout,
                                                                 const int* __restrict__ mask,
                                                                 bf16* __restrict__ dqkv, int n_pairs, int T, int H,
                                                                 int D, float pdrop, unsigned long long seed,
                                                                 unsigned long long offset) {
  __shared__ __attribute__((aligned(16))) bf16 lds[4][4][64 * DH];  // per wave: Q, K, V (then P^T/dS^T), dO
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int stride = gridDim.x * 4;
  int pair = blockIdx.x * 4 + wave;
  if (pair >= n_pairs) return;
  bf16* Qs = lds[wave][0];
  bf16* Ks = lds[wave][1];
  bf16* Vs = lds[wave][2];
  bf16* Gs = lds[wave][3];
  const int ld = 3 * D;
  const int fr = lane & 15, fq = lane >> 4;
  const int qq = fr >> 2, pp = fr & 3;
  const bf16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  TBIn in;
  tb_load(in, qkv, dout, mask, pair, T, H, D, lane);
  while (true) {
    // ---- stage the current pair (rows >= T zero) and its mask; then prefetch the next ----
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int idx = c * 64 + lane;
      const int r = idx >> 3, e = swz(r, (idx & 7) * 8);
      const bool ok = r < T;
      *(bf16x8*)(Qs + e) = ok ? in.q[c] : zero;
      *(bf16x8*)(Ks + e) = ok ? in.k[c] : zero;
      *(bf16x8*)(Vs + e) = ok ? in.v[c] : zero;
      *(bf16x8*)(Gs + e) = ok ? in.g[c] : zero;
    }
    // key-keep bits (lane = key s), wave-uniform: bit s set <=> s < T and mask[s] != 0
    const unsigned long long kbits = __ballot(lane < T && in.mk != 0);
    const int title = pair / H, h = pair - title * H;
    const size_t row0 = (size_t)title * T;
    const int next = min(pair + stride, n_pairs - 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the staged tiles are in LDS
    __builtin_amdgcn_wave_barrier();
    // dropout keep bits (DROP): query t = 16 jq + fr, key s = 16 is + 4 fq + r -> bit 4 is + r of
    // zbits[jq]; the same Philox elements as the forward.  Generated here, while the LDS writes
    // drain, and kept as 4 words (per-element scale arrays across the softmax spill)
    unsigned zbits[4] = {0u, 0u, 0u, 0u};
    const float inv_keep = DROP ? 1.0f / (1.0f - pdrop) : 1.f;
    if constexpr (DROP) {
#pragma unroll
      for (int jq = 0; jq < 4; ++jq)
#pragma unroll
        for (int is = 0; is < 4; ++is) {
          const uint4 rnd = Philox::gen(seed, offset, ((unsigned long long)pair * 64 + jq * 16 + fr) * 16 + is * 4 + fq);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            zbits[jq] |= (u32_to_unit(u4_get(rnd, r)) > pdrop ? 1u : 0u) << (is * 4 + r);
        }
    }
    // ---- S^T = K Q^T and dP^T = V dO^T from LDS fragments ----
    f32x4 st[4][4], dp[4][4];
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int jq = 0; jq < 4; ++jq) st[is][jq] = dp[is][jq] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kd = 0; kd < 2; ++kd) {
      bf16x8 kf[4], qf[4], vf[4], gf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = swz(i * 16 + fr, kd * 32 + fq * 8);
        kf[i] = *(const bf16x8*)(Ks + e);
        qf[i] = *(const bf16x8*)(Qs + e);
        vf[i] = *(const bf16x8*)(Vs + e);
        gf[i] = *(const bf16x8*)(Gs + e);
      }
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) {
          st[is][jq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[is], qf[jq], st[is][jq], 0, 0, 0);
          dp[is][jq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[is], gf[jq], dp[is][jq], 0, 0, 0);
        }
    }
    float keep[4][4], kadd[4][4];
#pragma unroll
    for (int is = 0; is < 4; ++is)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sk = is * 16 + fq * 4 + r;
        const bool on = (kbits >> sk) & 1ull;
        keep[is][r] = on ? 1.f : 0.f;
        kadd[is][r] = sk < T ? (on ? 0.f : -3.4028234663852886e38f) : -INFINITY;
      }
    // ---- softmax (forward recompute) and dS; P and dS leave as bf16 fragments ----
    bf16x8 dsf[4][2], psf[4][2];
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) {
      float m = -INFINITY;
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sc = kadd[is][r] == 0.f ? st[is][jq][r] * 0.125f : kadd[is][r];
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
      const unsigned zb = zbits[jq];
      float dsum = 0.f;
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          st[is][jq][r] *= inv;
          if constexpr (DROP) dp[is][jq][r] *= ((zb >> (is * 4 + r)) & 1u) ? inv_keep : 0.f;
          dsum += st[is][jq][r] * dp[is][jq][r];
        }
      dsum = group4_sum(dsum);
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dp[is][jq][r] = keep[is][r] * st[is][jq][r] * (dp[is][jq][r] - dsum) * 0.125f;
          if constexpr (DROP) st[is][jq][r] *= ((zb >> (is * 4 + r)) & 1u) ? inv_keep : 0.f;  // P~ for dV
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 f, g;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f[r] = f2bf(dp[2 * ks][jq][r]);
          f[4 + r] = f2bf(dp[2 * ks + 1][jq][r]);
          g[r] = f2bf(st[2 * ks][jq][r]);
          g[4 + r] = f2bf(st[2 * ks + 1][jq][r]);
        }
        dsf[jq][ks] = f;
        psf[jq][ks] = g;
      }
    }
    // the fp32 S / dP are dead: prefetch the next pair into the staging registers now (its
    // loads land during dQ, dV and dK of this pair)
    if constexpr (SPLIT) tb_load<1>(in, qkv, dout, mask, next, T, H, D, lane);
    else tb_load(in, qkv, dout, mask, next, T, H, D, lane);
    // ---- dQ = dS K (B = K via transposed reads of the swizzled tile) ----
    f32x4 o[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) o[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) {
        const int r = ks * 32 + fq * 4 + qq, c = jd * 16 + pp * 4;
        const bf16x8 kfr = tr_pair(Ks + swz(r, c), Ks + swz(r + 16, c));
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) o[jq][jd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kfr, dsf[jq][ks], o[jq][jd], 0, 0, 0);
      }
    bf16* dq = dqkv + row0 * ld + h * DH;
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) {
      const int t = jq * 16 + fr;
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        const float v0[4] = {o[jq][2 * p2][0], o[jq][2 * p2][1], o[jq][2 * p2][2], o[jq][2 * p2][3]};
        const float v1[4] = {o[jq][2 * p2 + 1][0], o[jq][2 * p2 + 1][1], o[jq][2 * p2 + 1][2], o[jq][2 * p2 + 1][3]};
        store_pair16_if(dq + (size_t)(t < T ? t : 0) * ld + p2 * 32, v0, v1, fq, t < T);
      }
    }
    // ---- dV = P^T dO and dK = dS^T Q: X^T [s][t] written into V's (now free) buffer ----
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int is = 0; is < 4; ++is)
#pragma unroll
        for (int jq = 0; jq < 4; ++jq)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int s = is * 16 + fq * 4 + r, t = jq * 16 + fr;
            Vs[swz(s, t)] = pass == 0 ? psf[jq][is >> 1][(is & 1) * 4 + r] : dsf[jq][is >> 1][(is & 1) * 4 + r];
          }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
      const bf16* Bsrc = pass == 0 ? Gs : Qs;  // dO for dV, Q for dK
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) o[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        bf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(Vs + swz(i * 16 + fr, kt * 32 + fq * 8));
#pragma unroll
        for (int jd = 0; jd < 4; ++jd) {
          const int r = kt * 32 + fq * 8 + qq, c = jd * 16 + pp * 4;
          const bf16x8 bfr = tr_pair(Bsrc + swz(r, c), Bsrc + swz(r + 4, c));
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i][jd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr, af[i], o[i][jd], 0, 0, 0);
        }
      }
      bf16* dst = dqkv + row0 * ld + (pass == 0 ? 2 * D : D) + h * DH;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int sk = i * 16 + fr;
#pragma unroll
        for (int p2 = 0; p2 < 2; ++p2) {
          const float v0[4] = {o[i][2 * p2][0], o[i][2 * p2][1], o[i][2 * p2][2], o[i][2 * p2][3]};
          const float v1[4] = {o[i][2 * p2 + 1][0], o[i][2 * p2 + 1][1], o[i][2 * p2 + 1][2], o[i][2 * p2 + 1][3]};
          store_pair16_if(dst + (size_t)(sk < T ? sk : 0) * ld + p2 * 32, v0, v1, fq, sk < T);
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // the scratch is rewritten by the next pass / pair
      if constexpr (SPLIT) {
        if (pass == 0) tb_load<2>(in, qkv, dout, mask, next, T, H, D, lane);  // V, dO of the next pair
      }
      __builtin_amdgcn_wave_barrier();
    }
    pair += stride;
    if (pair >= n_pairs) break;
  }
}

int g_tab_variant = 1;  // 1: persistent prefetching (default), 0: one-shot
int g_tab_cus = 0;
int g_tab_drop_split = 1;  // dropout backward: split prefetch (the variant setter's 10: one block)

int tab_cus() {
  if (g_tab_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_tab_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_tab_cus <= 0) g_tab_cus = 256;
  }
  return g_tab_cus;
}

}  // namespace

extern "C" void fr_title_attn_bwd_set_variant(int v) {
  if (v >= 10) g_tab_drop_split = v - 10;  // 10 / 11: the dropout backward's prefetch form
  else g_tab_variant = v;
}

extern "C" int fr_title_attention_bwd_long_bf16(const void* qkv, const void* dout, const int* mask, void* dqkv,
                                                int n_titles, int T, int H, int D, hipStream_t s);  // title_attn_long.hip

extern "C" int fr_title_attention_bwd_bf16(const void* qkv, const void* dout, const int* mask, void* dqkv,
                                           int n_titles, int T, int H, int D, hipStream_t s) {
  if (T > 64) return fr_title_attention_bwd_long_bf16(qkv, dout, mask, dqkv, n_titles, T, H, D, s);
  if (T < 1 || D != H * DH) return 1;
  const int pairs = n_titles * H;
  if (pairs == 0) return 0;
  if (g_tab_variant == 1) {
    int blocks = tab_cus();
    const int need = (pairs + 3) / 4;
    blocks = blocks < need ? blocks : need;
    hipLaunchKernelGGL(title_attn_bwd_pkernel<false>, dim3(blocks), dim3(256), 0, s, (const bf16*)qkv, (const bf16*)dout,
                       mask, (bf16*)dqkv, pairs, T, H, D, 0.f, 0ull, 0ull);
    return 0;
  }
  hipLaunchKernelGGL((title_attn_bwd_kernel<false>), dim3((pairs + WPB - 1) / WPB), dim3(64 * WPB), 0, s,
                     (const bf16*)qkv, (const bf16*)dout, mask, (bf16*)dqkv, n_titles, T, H, D, 0.f, 0ull, 0ull);
  return 0;
}

extern "C" int fr_title_attention_bwd_drop_bf16(const void* qkv, const void* dout, const int* mask, void* dqkv,
                                                int n_titles, int T, int H, int D, float pdrop, unsigned long long seed,
                                                unsigned long long offset, hipStream_t s) {
  if (T < 1 || T > 64 || D != H * DH || !(pdrop > 0.f && pdrop < 1.f)) return 2;
  const int pairs = n_titles * H;
  if (pairs == 0) return 0;
  if (g_tab_variant == 1) {
    const int need = (pairs + 3) / 4;
    const int blocks = tab_cus() < need ? tab_cus() : need;
    if (g_tab_drop_split)
      hipLaunchKernelGGL((title_attn_bwd_pkernel<true, true>), dim3(blocks), dim3(256), 0, s, (const bf16*)qkv,
                         (const bf16*)dout, mask, (bf16*)dqkv, pairs, T, H, D, pdrop, seed, offset);
    else
      hipLaunchKernelGGL((title_attn_bwd_pkernel<true, false>), dim3(blocks), dim3(256), 0, s, (const bf16*)qkv,
                         (const bf16*)dout, mask, (bf16*)dqkv, pairs, T, H, D, pdrop, seed, offset);
    return 0;
  }
  hipLaunchKernelGGL((title_attn_bwd_kernel<true>), dim3((pairs + WPB - 1) / WPB), dim3(64 * WPB), 0, s,
                     (const bf16*)qkv, (const bf16*)dout, mask, (bf16*)dqkv, n_titles, T, H, D, pdrop, seed, offset);
  return 0;
}

