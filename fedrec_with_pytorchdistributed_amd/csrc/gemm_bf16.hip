// bf16 "NT" GEMM with fused epilogues on MFMA (gfx950):
//   C[M,N] = act(A[M,K] . W[N,K]^T + bias[N]) + R[M,N]      (bf16 in/out, fp32 accumulate)
//
// Every DistilBERT linear (fused Q|K|V N=2304, out-proj N=768, FFN1 N=3072 + GELU,
// FFN2 N=768 + residual) and the text head's att_fc1 (N=384 + tanh) run here
// (SURVEY §2.3 K02/K05/K06).  Both operands are K-contiguous, which is the natural
// layout for v_mfma_f32_16x16x32_bf16: each lane's A and B fragments are 16 contiguous
// bytes of one row.
//
// Structure (cdna_hip_programming.md §5, "minimum 2-phase"):
//   * 128x128x64 block tile, 256 threads = 4 waves in 2x2, 64x64 per wave
//     (4x4 MFMA tiles -> 64 accumulator VGPRs);
//   * global -> LDS by global_load_lds_dwordx4 (16 B per lane, no VGPR round trip),
//     two LDS stages (64 KB -> 2 blocks per CU), next tile issued before the MFMAs;
//   * LDS image is lane-linear (a glds constraint), so the bank-conflict XOR swizzle
//     (16-B chunk c of row r stored at chunk c ^ (r & 7)) is applied to the per-lane
//     SOURCE address and undone on the ds_read_b128 address (§5.4 rule 21);
//   * operands swapped (W as the MFMA A operand) so each lane ends with 4 consecutive
//     output columns -> one 8-byte bias load / residual load / store per 4 outputs;
//   * XCD-aware tile order: consecutive tiles (which share the A row panel) land on one
//     XCD's L2 (bijective remap, §5.5 T1).
// Requirements (checked on the host): N % 128 == 0, K % 64 == 0; any M (rows clamped on
// load, masked on store).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;  // 32 KB

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

template <int ACT>
__device__ __forceinline__ float act_fn(float x) {
  if constexpr (ACT == 1) return gelu_erf(x);
  else if constexpr (ACT == 2) return tanhf(x);
  else return x;
}

// issue the glds for one K-tile into stage `st`
__device__ __forceinline__ void stage_tile(char* smem, int st, const bf16* __restrict__ A, const bf16* __restrict__ W,
                                           int M, int K, int m0, int n0, int k0, int wave, int lane) {
  char* base = smem + st * STAGE_BYTES;
  const int rsub = lane >> 3;                    // row within the 8-row piece
  const int chunk = (lane & 7) ^ rsub;           // logical 16-B chunk this lane fetches
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 32 + i * 8 + rsub;    // 0..127
    int gm = m0 + row;
    gm = gm < M ? gm : M - 1;
    const bf16* src = A + (size_t)gm * K + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, src), LDS_PTR(void, base + (wave * 32 + i * 8) * 128),
                                     16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 32 + i * 8 + rsub;
    const bf16* src = W + (size_t)(n0 + row) * K + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, src),
                                     LDS_PTR(void, base + BM * 128 + (wave * 32 + i * 8) * 128), 16, 0, 0);
  }
}

template <int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                         const float* __restrict__ bias, const bf16* __restrict__ R,
                                                         bf16* __restrict__ C, int M, int N, int K, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  // bijective XCD remap: blocks b, b+8, ... share an XCD -> give each XCD a contiguous tile range
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, q = nwg >> 3, rmd = nwg & 7;
  const int tile = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + (bid >> 3);
  const int mt = tile / tiles_n, nt = tile - mt * tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage_tile(smem, 0, A, W, M, K, m0, n0, 0, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15;         // fragment row
  const int fq = lane >> 4;         // k quarter
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage_tile(smem, cur ^ 1, A, W, M, K, m0, n0, (kt + 1) * BK, wave, lane);
    const char* As = smem + cur * STAGE_BYTES;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int phys = ((kk * 4 + fq) ^ (fr & 7)) * 16;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *(const bf16x8*)(As + (wm * 64 + i * 16 + fr) * 128 + phys);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *(const bf16x8*)(Bs + (wn * 64 + j * 16 + fr) * 128 + phys);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane holds C[m][nb..nb+3]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wn * 64 + j * 16 + fq * 4;
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      if constexpr (HAS_BIAS) {
        const float4 bb = *(const float4*)(bias + nb);
        v0 += bb.x; v1 += bb.y; v2 += bb.z; v3 += bb.w;
      }
      v0 = act_fn<ACT>(v0); v1 = act_fn<ACT>(v1); v2 = act_fn<ACT>(v2); v3 = act_fn<ACT>(v3);
      if constexpr (HAS_RES) {
        const bf16x4 rr = *(const bf16x4*)(R + (size_t)m * N + nb);
        v0 += (float)rr[0]; v1 += (float)rr[1]; v2 += (float)rr[2]; v3 += (float)rr[3];
      }
      bf16x4 o = {f2bf(v0), f2bf(v1), f2bf(v2), f2bf(v3)};
      *(bf16x4*)(C + (size_t)m * N + nb) = o;
    }
  }
}

template <int ACT>
void launch_act(const bf16* A, const bf16* W, const float* bias, const bf16* R, bf16* C, int M, int N, int K,
                hipStream_t s) {
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  dim3 grid(tiles_m * tiles_n), block(256);
  if (bias && R) hipLaunchKernelGGL((gemm_nt_kernel<ACT, true, true>), grid, block, 0, s, A, W, bias, R, C, M, N, K, tiles_n);
  else if (bias) hipLaunchKernelGGL((gemm_nt_kernel<ACT, true, false>), grid, block, 0, s, A, W, bias, R, C, M, N, K, tiles_n);
  else if (R) hipLaunchKernelGGL((gemm_nt_kernel<ACT, false, true>), grid, block, 0, s, A, W, bias, R, C, M, N, K, tiles_n);
  else hipLaunchKernelGGL((gemm_nt_kernel<ACT, false, false>), grid, block, 0, s, A, W, bias, R, C, M, N, K, tiles_n);
}

}  // namespace

extern "C" int fr_gemm_nt_bf16(const void* A, const void* W, const float* bias, const void* R, void* C, int M, int N,
                               int K, int act, hipStream_t s) {
  if (N % BN != 0 || K % BK != 0 || M <= 0) return 1;
  const bf16* a = (const bf16*)A;
  const bf16* w = (const bf16*)W;
  const bf16* r = (const bf16*)R;
  bf16* c = (bf16*)C;
  switch (act) {
    case 0: launch_act<0>(a, w, bias, r, c, M, N, K, s); break;
    case 1: launch_act<1>(a, w, bias, r, c, M, N, K, s); break;
    case 2: launch_act<2>(a, w, bias, r, c, M, N, K, s); break;
    default: return 2;
  }
  return 0;
}
