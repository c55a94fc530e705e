// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of the engine.
//
// * wave64 everywhere: lane = threadIdx.x & 63, reductions use __shfl_xor over 64 lanes;
// * bf16 is clang's native __bf16 (f32->bf16 lowers to v_cvt_pk_bf16_f32 on gfx950,
//   which keeps NaNs -- MI355X_MICROARCH.md "Correctness boundaries");
// * MFMA fragment types for v_mfma_f32_16x16x32_bf16 / 32x32x16_bf16;
// * a Philox-4x32-10 counter RNG (LDP noise, dropout, secure-aggregation masks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))
#define GLOBAL_PTR(T, p) ((__attribute__((address_space(1))) T*)(p))

#define FR_CHECK_LAUNCH() (void)0

static __device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

static __device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// reduce across the lanes that share (lane & 15): xor 16 and 32
static __device__ __forceinline__ float group4_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
static __device__ __forceinline__ float group4_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}

static __device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
static __device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// ---------------------------------------------------------------------------------------
// Philox-4x32-10 (Salmon et al. 2011); counter = (offset, idx), key = seed.
struct Philox {
  static __device__ __forceinline__ void round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                               uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  static __device__ __forceinline__ uint4 gen(uint64_t seed, uint64_t offset, uint64_t idx) {
    uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32), c2 = (uint32_t)offset, c3 = (uint32_t)(offset >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      round(c0, c1, c2, c3, k0, k1);
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
  }
};

static __device__ __forceinline__ float u32_to_unit(uint32_t x) {  // (0, 1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// Dropout (HF train mode): element e of a dropout site keeps with probability 1-p
// and is scaled by 1/(1-p).  The mask is a pure function of (seed, offset, e): Philox counter
// e >> 2, component e & 3, keep iff unit(x) > p -- so a backward kernel regenerates exactly
// the forward's mask and the torch oracle (ops/reference.py philox4x32) reproduces it bit for bit.
static __device__ __forceinline__ float drop_scale(uint32_t x, float p, float inv_keep) {
  return u32_to_unit(x) > p ? inv_keep : 0.f;
}
static __device__ __forceinline__ uint32_t u4_get(const uint4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// Box-Muller: two standard normals from two uniforms
static __device__ __forceinline__ float2 box_muller(uint32_t a, uint32_t b) {
  float u1 = u32_to_unit(a), u2 = u32_to_unit(b);
  float r = sqrtf(-2.0f * logf(u1));
  float s, c;
  __sincosf(6.283185307179586f * u2, &s, &c);
  return make_float2(r * c, r * s);
}

// 16-byte stores of a 16x16x32 accumulator pair: lane (fr, fq) holds 4 consecutive columns
// [4fq, +4) of two 16-column groups v0 (cols 0..15) and v1 (cols 16..31) of one row; one
// permlane16 swap between lanes l and l^16 (same row) regroups them so every lane stores 8
// consecutive bf16 (half the store instructions of 8-byte stores; MI355X_MICROARCH.md
// "attention epilogue store tail").  Every lane must execute the swaps; `store` masks only
// the write.
static __device__ __forceinline__ void store_pair16_if(bf16* __restrict__ crow, const float (&v0)[4],
                                                       const float (&v1)[4], int fq, bool store) {
  const bf16x4 o0 = {f2bf(v0[0]), f2bf(v0[1]), f2bf(v0[2]), f2bf(v0[3])};
  const bf16x4 o1 = {f2bf(v1[0]), f2bf(v1[1]), f2bf(v1[2]), f2bf(v1[3])};
  uint2 a = __builtin_bit_cast(uint2, o0), b = __builtin_bit_cast(uint2, o1);
  auto r = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  a.x = r[0];
  b.x = r[1];
  r = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  a.y = r[0];
  b.y = r[1];
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  if (store) *GLOBAL_PTR(u32x4_t, crow + (fq & 1) * 16 + (fq >> 1) * 8) = u32x4_t{a.x, a.y, b.x, b.y};
}

// ---------------------------------------------------------------------------------------
// Last-arriver hand-off between the workgroups of one launch (split-K seams, partial-row
// sums): MI355X_MICROARCH.md "Valid forms" table row 1 -- the producers' data stored
// write-through (st_sc1: relaxed agent-scope stores = global_store sc1), every storing wave's
// vmcnt(0), a workgroup barrier, ONE agent-scope ticket add per workgroup; the workgroup whose
// add returns total - 1 reads the data with ld_sc1 (relaxed agent-scope loads) and re-arms the
// ticket for the next launch.  No release / acquire fences (a release writes back the XCD's
// whole L2: a fenced last-block column sum measured 131 vs 69 us per step).
static __device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
static __device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every thread of the workgroup; true in the workgroup that arrived last
static __device__ __forceinline__ bool last_arrival(unsigned* cnt, unsigned total) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned k = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = k == total - 1;
    if (s_last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last != 0;
}
