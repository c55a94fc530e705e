// Weight-gradient ("TN") GEMM on MFMA (gfx950):
//   dW[N, K] (fp32) = dY[M, N]^T . X[M, K]          (bf16 in, fp32 accumulate and out)
//
// The backward of every linear of the training step (SURVEY §2.3 K02/K05/K06 backward, the
// text head's att_fc1, the unfrozen backbone of BASELINE config 5): the reduction runs over
// the long token dimension M (~80k rows), the output is a small [N, K] weight.
//
// Both operands are M-major (the reduction index is the row index), so an MFMA fragment --
// 8 consecutive reduction elements of one output row/column per lane -- is a COLUMN of the
// row-major tile.  The tiles are staged row-major exactly as they sit in HBM (glds, 16 B per
// lane, no VGPR round trip) and every fragment is read with ds_read_b64_tr_b16 (the gfx950
// LDS transpose read: 4 rows x 16 columns per 16-lane group, delivered column-major), two per
// fragment (cdna_hip_programming.md T10).
//
// Structure:
//   * output tile 256 (n) x 256 (k), 512 threads = 8 waves as 2 (n) x 4 (k), 128 x 64 per
//     wave (8 x 4 MFMA tiles -> 128 accumulator VGPRs);
//   * LDS stage = dY[32][256] + X[32][256] bf16 = 32 KB, three stages by default (96 KB, one
//     block per CU), two in flight; the fragment reads are opaque asm, so the compiler does
//     not drain vmcnt before them (with builtin reads it waited for every in-flight stage:
//     760-800 TF; pipelined: 974-1033 TF; 4 or 5 stages measured the same as 3);
//   * bank-conflict swizzle: 16-B chunk c of row r is stored at chunk c ^ swz(r), swz(r) =
//     2 * ((r & 3) | ((r >> 3) & 1) << 2); a 32-lane half of a transposed read touches rows
//     {q, 8 + q} x one 32-B column pair, which the XOR spreads over all 64 banks (applied to
//     the per-lane glds SOURCE address, since the glds image is lane-linear: §5.4 rule 21);
//   * split-K over M: S splits x (N/256 x K/256) tiles ~ one wave of workgroups on 256 CUs;
//     each split writes an fp32 partial [N, K], a second kernel sums the S partials in a
//     fixed order (deterministic, no float atomics); S = 1 writes dW directly;
//   * rows beyond M and columns beyond N / K load from a zero row instead (no clamping: the
//     reduction must not see duplicated rows);
//   * XCD-aware order: all tiles of one split (which read the same dY / X row panel) run on
//     one XCD's L2 (bijective blockIdx remap, §5.5 T1).
// Requirements (host-checked): N % 8 == 0, K % 8 == 0 (16-B row chunks), contiguous rows.
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int TN = 256, TKO = 256, TM = 32;        // output tile n x k, reduction rows per stage
constexpr int OP_BYTES = TM * 512;                 // one operand tile: 32 rows x 512 B
constexpr int WSTAGE = 2 * OP_BYTES;               // 32 KB

__device__ __attribute__((aligned(16))) bf16 g_zero_row[256];  // zero-initialised (bss)

__device__ __forceinline__ int swz(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }

// 32 rows x 256 columns of a row-major [rows, ld] operand into `dst` (swizzled): 16 glds of
// 1 KB (2 rows each), 2 per wave
__device__ __forceinline__ void stage_op(char* dst, const bf16* __restrict__ src, int ld, int cols, int c0, int m,
                                         int mend, int wave, int lane) {
  const int rsub = lane >> 5, pc = lane & 31;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = wave * 2 + i;
    const int row = 2 * blk + rsub;
    const int c = pc ^ swz(row);
    const int col = c0 + 8 * c;
    const int gm = m + row;
    const bf16* p = (gm < mend && col < cols) ? src + (size_t)gm * ld + col : g_zero_row + 8 * c;
    __builtin_amdgcn_global_load_lds(GLOBAL_PTR(const void, p), LDS_PTR(void, dst + blk * 1024), 16, 0, 0);
  }
}

// LDS byte offset of this lane's 8 bytes for a transposed read of rows r0 + q (q = 0..3),
// columns col0 + 4p .. +3 (lane 4q+p of its 16-lane group)
__device__ __forceinline__ uint32_t tr_off(int r0, int col0, int q, int p) {
  const int c = (col0 >> 3) + (p >> 1);
  const int r = r0 + q;
  return (uint32_t)(r * 512 + ((c ^ swz(r)) << 4) + (p & 1) * 8);
}

// ds_read_b64_tr_b16 as opaque asm: a plain (builtin) LDS read after a glds into the same LDS
// object makes the compiler drain vmcnt first -- every in-flight stage -- which serialises the
// pipeline.  The reads' completion is then ours to wait for (lgkm_tie*).
__device__ __forceinline__ s16x4 tr_read(uint32_t addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

#define LGKM_TIE8(r)                                                                                  \
  asm volatile("s_waitcnt lgkmcnt(0)"                                                                 \
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), \
                 "+v"(r[7]))

__device__ __forceinline__ bf16x8 join(s16x4 a, s16x4 b) {
  bf16x4 x = __builtin_bit_cast(bf16x4, a), y = __builtin_bit_cast(bf16x4, b);
  return bf16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

__device__ __forceinline__ void sync_stage(int inflight) {  // inflight younger stages may stay
  __builtin_amdgcn_sched_barrier(0);
  if (inflight >= 3) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
  else if (inflight == 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else if (inflight == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// NST LDS stages of 32 KB, NST - 1 in flight (3: 96 KB, the default; 4: 128 KB; 5: 160 KB)
template <int NST>
__global__ __launch_bounds__(512, 1) void wgrad_kernel(const bf16* __restrict__ dY, const bf16* __restrict__ X,
                                                       float* __restrict__ P, int M, int N, int K, int tiles_k,
                                                       int ntiles, int mchunk) {
  __shared__ __attribute__((aligned(16))) char smem[NST * WSTAGE];
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, qq = nwg >> 3, rmd = nwg & 7;
  const int t = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (bid >> 3);
  const int s = t / ntiles, tile = t - s * ntiles;
  const int nt = tile / tiles_k, kt = tile - nt * tiles_k;
  const int n0 = nt * TN, k0 = kt * TKO;
  const int mb = s * mchunk;
  const int me = min(M, mb + mchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 2, wk = wave & 3;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = me > mb ? (me - mb + TM - 1) / TM : 0;
#pragma unroll
  for (int i = 0; i < NST - 1; ++i) {
    if (i < nsteps) {
      char* b = smem + i * WSTAGE;
      stage_op(b, dY, N, N, n0, mb + i * TM, me, wave, lane);
      stage_op(b + OP_BYTES, X, K, K, k0, mb + i * TM, me, wave, lane);
    }
  }
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = g * 8;
  // per-lane offsets inside a stage: X fragments j (lo/hi rows), dY fragments i
  uint32_t xo[4][2], yo[8][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    xo[j][0] = OP_BYTES + tr_off(r0, wk * 64 + j * 16, q, p);
    xo[j][1] = OP_BYTES + tr_off(r0 + 4, wk * 64 + j * 16, q, p);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    yo[i][0] = tr_off(r0, wn * 128 + i * 16, q, p);
    yo[i][1] = tr_off(r0 + 4, wn * 128 + i * 16, q, p);
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
  for (int st = 0; st < nsteps; ++st) {
    // stage st landed (this wave's glds), then every wave's: barrier.  Every wave finished its
    // reads of step st-1 (lgkmcnt(0) before its MFMAs), so that buffer may be restaged.
    const int left = nsteps - 1 - st;
    sync_stage(left < NST - 2 ? left : NST - 2);
    if (st + NST - 1 < nsteps) {
      char* nx = smem + ((st + NST - 1) % NST) * WSTAGE;
      stage_op(nx, dY, N, N, n0, mb + (st + NST - 1) * TM, me, wave, lane);
      stage_op(nx + OP_BYTES, X, K, K, k0, mb + (st + NST - 1) * TM, me, wave, lane);
    }
    const uint32_t base = lds0 + (st % NST) * WSTAGE;
    s16x4 xr[8], y0[8], y1[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xr[2 * j] = tr_read(base + xo[j][0]);
      xr[2 * j + 1] = tr_read(base + xo[j][1]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y0[2 * i] = tr_read(base + yo[i][0]);
      y0[2 * i + 1] = tr_read(base + yo[i][1]);
    }
    LGKM_TIE8(xr);
    LGKM_TIE8(y0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y1[2 * i] = tr_read(base + yo[4 + i][0]);
      y1[2 * i + 1] = tr_read(base + yo[4 + i][1]);
    }
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 xb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xb[j] = join(xr[2 * j], xr[2 * j + 1]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16x8 ya = join(y0[2 * i], y0[2 * i + 1]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[j], ya, acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    LGKM_TIE8(y1);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16x8 ya = join(y1[2 * i], y1[2 * i + 1]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[j], ya, acc[4 + i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  // lane holds dW[n][k .. k+3]: n = tile row (lane % 16), k = 4 consecutive (lane / 16)
  float* out = P + (size_t)s * N * K;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = n0 + wn * 128 + i * 16 + (lane & 15);
    if (n >= N) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wk * 64 + j * 16 + 4 * g;
      if (k < K) *(f32x4*)(out + (size_t)n * K + k) = acc[i][j];
    }
  }
}

// C[i] = (accumulate ? C[i] : 0) + sum_s P[s][i], fixed order; n4 = N*K/4 float4s
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const f32x4* __restrict__ P, f32x4* __restrict__ C,
                                                           long n4, int S, int accumulate) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 v = accumulate ? C[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) v += P[(size_t)s * n4 + i];
    C[i] = v;
  }
}

int g_cus = 0;

void plan(int M, int N, int K, int& S, int& mchunk, int& ntiles, int& tiles_k) {
  if (g_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 256;
  }
  tiles_k = (K + TKO - 1) / TKO;
  ntiles = ((N + TN - 1) / TN) * tiles_k;
  // one wave of workgroups (one block per CU), each split >= 8 reduction steps
  int s = g_cus / ntiles;
  const int smax = (M + 16 * TM - 1) / (16 * TM);
  s = s < 1 ? 1 : (s > smax ? smax : s);
  const int rows = (M + s - 1) / s;
  mchunk = (rows + TM - 1) / TM * TM;
  S = (M + mchunk - 1) / mchunk;
  if (S < 1) S = 1;
}

}  // namespace

// Returns the fp32 scratch element count needed (0: none) when `scratch` is null, else
// launches; negative = unsupported shape.  accumulate: C += dY^T X.
extern "C" long fr_wgrad_bf16(const void* dY, const void* X, float* C, float* scratch, int M, int N, int K,
                              int accumulate, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || N % 8 != 0 || K % 8 != 0) return -1;
  int S, mchunk, ntiles, tiles_k;
  plan(M, N, K, S, mchunk, ntiles, tiles_k);
  const bool direct = S == 1 && !accumulate;
  const long need = direct ? 0 : (long)S * N * K;
  if (scratch == nullptr && need > 0) return need;
  float* P = direct ? C : scratch;
  // three LDS stages (96 KB): 4 and 5 measured the same in isolation, and the smaller block
  // leaves room on a CU for a lookahead-stream kernel (dedup: 32 KB) -- this grid is one wave of
  // blocks, so a CU that cannot host its block doubles the kernel
  hipLaunchKernelGGL(wgrad_kernel<3>, dim3(S * ntiles), dim3(512), 0, stream, (const bf16*)dY, (const bf16*)X, P, M, N,
                     K, tiles_k, ntiles, mchunk);
  if (!direct) {
    const long n4 = (long)N * K / 4;
    long blocks = (n4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const f32x4*)P, (f32x4*)C,
                       n4, S, accumulate);
  }
  return 0;
}
