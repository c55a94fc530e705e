// Fused Adam over the flat trainable buffer (reference model.py:22-23,89,93: two
// torch.optim.Adam(lr=5e-5) that always step together).
//
//   g' = g * grad_scale        (grad_scale = 1/W folds the all-reduce average in)
//   m = b1 m + (1-b1) g' ;  v = b2 v + (1-b2) g'^2
//   p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)          (torch.optim.Adam, no weight decay)
//
// One streaming pass, float4 vectorised; optionally writes a bf16 copy of p (unfrozen
// backbone: the compute weights are refreshed in the same pass).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void adam_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                   float4* __restrict__ m, float4* __restrict__ v,
                                                   bf16x4* __restrict__ plow, long n4, float lr, float b1, float b2,
                                                   float eps, float step_size, float inv_sqrt_bc2, float gs) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    float* pa = (float*)&pp;
    float* ga = (float*)&gg;
    float* ma = (float*)&mm;
    float* va = (float*)&vv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x = ga[k] * gs;
      ma[k] = b1 * ma[k] + (1.f - b1) * x;
      va[k] = b2 * va[k] + (1.f - b2) * x * x;
      const float denom = sqrtf(va[k]) * inv_sqrt_bc2 + eps;
      pa[k] -= step_size * ma[k] / denom;
    }
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
    if (plow) plow[i] = bf16x4{f2bf(pa[0]), f2bf(pa[1]), f2bf(pa[2]), f2bf(pa[3])};
  }
}

}  // namespace

extern "C" int fr_adam_flat(float* p, const float* g, float* m, float* v, void* plow, long n, float lr, float b1,
                            float b2, float eps, float bc1, float bc2, float grad_scale, hipStream_t s) {
  if (n % 4 != 0) return 1;
  const long n4 = n / 4;
  if (n4 == 0) return 0;
  long blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (float4*)p, (const float4*)g, (float4*)m,
                     (float4*)v, (bf16x4*)plow, n4, lr, b1, b2, eps, lr / bc1, 1.0f / sqrtf(bc2), grad_scale);
  return 0;
}

// ---------------------------------------------------------------------------------------
// The same step with the step count on the device, for a HIP graph that captures the whole
// training step (forward, backward, Adam) when no gradient all-reduce sits between the
// backward and the optimizer (one client): every block reads t (the step's cast launch -- the
// graph's first kernel -- advanced the counter) and forms the bias corrections itself (in
// double, then rounded as the host path rounds them); block 0 also copies this step's loss
// into slot (t - 1) % ring of a loss ring (no per-step clone launch).
namespace {
// Gradient segments (optional): the fresh per-parameter gradient tensors where autograd left
// them -- segment j covers flat elements [off[j], off[j] + n[j]) (off 4-aligned: the flat
// buffer aligns every parameter to 64 elements) and reads src[j]; the flat elements between
// segments (alignment gaps) are 0.  The kernel writes each gathered value into the flat
// gradient as it goes, so the flat buffer ends the step as the separate copy launch
// (FlatParams.end_backward's multi_cast) left it.
constexpr int ADAM_SEG = 48;
struct AdamSegs {
  const float* src[ADAM_SEG];
  long off[ADAM_SEG];
  long n[ADAM_SEG];
  int nseg;
};

// the table in LDS (a per-lane index into the kernel-argument struct is a chain of dependent
// global loads per lookup: 12.6 vs ~9 us for the whole launch)
struct SegLds {
  const float* src[ADAM_SEG];
  long off[ADAM_SEG];
  long n[ADAM_SEG];
};

__device__ __forceinline__ float4 seg_grad4(const SegLds& sg, int nseg, long e) {  // flat elements e .. e + 3
  int lo = 0, hi = nseg - 1;  // last segment with off <= e
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (sg.off[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  const long r = e - sg.off[lo];
  const float* src = sg.src[lo];
  const long n = sg.n[lo];
  if (src == nullptr || r < 0 || r >= n) return make_float4(0.f, 0.f, 0.f, 0.f);
  if (r + 4 <= n && (((uintptr_t)(src + r)) & 15) == 0) return *(const float4*)(src + r);
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
  float* oa = (float*)&o;
  for (int k = 0; k < 4 && r + k < n; ++k) oa[k] = src[r + k];
  return o;
}

__global__ __launch_bounds__(256) void adam_dev_kernel(float4* __restrict__ p, float4* __restrict__ g,
                                                       float4* __restrict__ m, float4* __restrict__ v,
                                                       bf16x4* __restrict__ plow, long n4, float lr, float b1, float b2,
                                                       float eps, float gs, const long long* __restrict__ step,
                                                       const float* __restrict__ loss, float* __restrict__ ring,
                                                       int ring_n, const AdamSegs segs,
                                                       const int* __restrict__ skip) {
  // skip (optional): the gradient all-reduce's status word (the IPC all-reduce sets it when a
  // peer timed out and poisons that call's output) -- then no update at all, and the step's loss
  // slot gets NaN, so the epoch's loss reads back non-finite and the engine's check raises
  if (skip != nullptr && __hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && ring != nullptr) ring[(step[0] - 1) % ring_n] = __builtin_nanf("");
    return;
  }
  // t = the device step count, already advanced for this step by the step's cast launch (an
  // earlier kernel of the same stream): no read-modify-write here (a same-address ticket per
  // block made this launch 20 us, against 7 for the eager kernel)
  __shared__ float bc_s[2];
  __shared__ SegLds sg_s;
  if ((int)threadIdx.x < segs.nseg) {
    sg_s.src[threadIdx.x] = segs.src[threadIdx.x];
    sg_s.off[threadIdx.x] = segs.off[threadIdx.x];
    sg_s.n[threadIdx.x] = segs.n[threadIdx.x];
  }
  const long long t = step[0];
  if (threadIdx.x == 0) {  // double pow once per block, as the host computes them for the eager kernel
    bc_s[0] = (float)(1.0 - pow((double)b1, (double)t));
    bc_s[1] = (float)(1.0 - pow((double)b2, (double)t));
  }
  __syncthreads();
  const float bc1 = bc_s[0], bc2 = bc_s[1];
  const float step_size = lr / bc1, inv_sqrt_bc2 = 1.0f / sqrtf(bc2);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 gg;
    if (segs.nseg > 0) {  // block-uniform
      gg = seg_grad4(sg_s, segs.nseg, 4 * i);
      g[i] = gg;
    } else {
      gg = g[i];
    }
    float4 pp = p[i], mm = m[i], vv = v[i];
    float* pa = (float*)&pp;
    float* ga = (float*)&gg;
    float* ma = (float*)&mm;
    float* va = (float*)&vv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x = ga[k] * gs;
      ma[k] = b1 * ma[k] + (1.f - b1) * x;
      va[k] = b2 * va[k] + (1.f - b2) * x * x;
      const float denom = sqrtf(va[k]) * inv_sqrt_bc2 + eps;
      pa[k] -= step_size * ma[k] / denom;
    }
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
    if (plow) plow[i] = bf16x4{f2bf(pa[0]), f2bf(pa[1]), f2bf(pa[2]), f2bf(pa[3])};
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && ring != nullptr) ring[(t - 1) % ring_n] = loss[0];
}

}  // namespace

// nseg > 0: the gradient is gathered from the segments (gsrc / goff / gn, sorted by offset;
// a null source = no gradient) and written into g
extern "C" int fr_adam_dev(float* p, float* g, float* m, float* v, void* plow, long n, float lr, float b1,
                           float b2, float eps, float grad_scale, const long long* step, const float* loss, float* ring,
                           int ring_n, hipStream_t s, int nseg, const float* const* gsrc, const long* goff,
                           const long* gn, const int* skip) {
  if (n % 4 != 0 || (ring != nullptr && (loss == nullptr || ring_n < 1))) return 1;
  if (nseg < 0 || nseg > ADAM_SEG) return 2;
  AdamSegs segs{};
  segs.nseg = nseg;
  for (int j = 0; j < nseg; ++j) {
    if (goff[j] % 4 != 0 || (j > 0 && goff[j] < goff[j - 1] + gn[j - 1]) || goff[j] + gn[j] > n) return 3;
    segs.src[j] = gsrc[j];
    segs.off[j] = goff[j];
    segs.n[j] = gn[j];
  }
  const long n4 = n / 4;
  long blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_dev_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (float4*)p, (float4*)g, (float4*)m,
                     (float4*)v, (bf16x4*)plow, n4, lr, b1, b2, eps, grad_scale, step, loss, ring, ring_n, segs, skip);
  return 0;
}
// ---------------------------------------------------------------------------------------
// Compute-weight refresh of the unfrozen backbone after an optimizer step: up to MCAST_SEG
// fp32 master tensors -> their bf16 (or fp32) compute copies in ONE launch, 8 elements per
// thread (two float4 loads, one 16-byte bf16 store).  Segment i may write into a slice of a
// bigger destination (q / k / v weights -> the fused [3D, D] QKV weight), so the per-step
// pack rebuild (a cat + a cast launch per weight, ~100 launches at BERT-base) becomes one
// streaming pass.  Blocks are assigned to segments in proportion to their size
// (MCAST_CHUNK elements per block); a block finds its segment by binary search.  Any size and
// alignment: 16-byte aligned segments take the vector path, the rest (and ragged tails) go
// element by element.
namespace {
constexpr int MCAST_SEG = 96;
constexpr int MCAST_CHUNK = 8192;  // 256 threads x 4 iterations x 8 elements
constexpr int MCAST_FILL = 8;
constexpr int MCAST_TSEG = 8;

struct MultiCast {
  const float* src[MCAST_SEG];
  void* dst[MCAST_SEG];
  long n[MCAST_SEG];
  int blk0[MCAST_SEG + 1];
  unsigned char bf[MCAST_SEG];   // 1: bf16 destination, 0: fp32
  unsigned char vec[MCAST_SEG];  // 1: 16-byte aligned (vector path), 0: element by element
  int nseg;
  long long* bump;   // optional: a device step counter advanced by one (block 0, lane 0)
  long long* bump2;  // optional: a second one (the in-graph Adam's step count)
  // up to MCAST_FILL copy segments (fp32 destination, 4-byte words of any type) may be longer
  // than their source: words past nsrc get the fill bits (a step graph's padded static inputs)
  signed char fslot[MCAST_SEG];  // -1: none, else index into nsrc / fill
  long nsrc[MCAST_FILL];
  int fill[MCAST_FILL];
  // transposed bf16 segments (after the others' blocks): fp32 [R, C] -> dst[c * ld + r], 64 x 64
  // tiles through LDS, any R / C (the register-direct GEMMs' k-contiguous weight copies)
  int ntseg;
  const float* tsrc[MCAST_TSEG];
  bf16* tdst[MCAST_TSEG];
  int tR[MCAST_TSEG], tC[MCAST_TSEG], tld[MCAST_TSEG];
  int tblk0[MCAST_TSEG + 1];
};

__device__ __forceinline__ void mcast_t_tile(const MultiCast& mc, int t) {
  __shared__ float tile[64][65];
  int sg = 0;
  while (sg + 1 < mc.ntseg && mc.tblk0[sg + 1] <= t) ++sg;
  t -= mc.tblk0[sg];
  const int R = mc.tR[sg], C = mc.tC[sg], ct = (C + 63) >> 6;
  const int r0 = (t / ct) * 64, c0 = (t % ct) * 64;
  const float* src = mc.tsrc[sg];
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; ++i) {  // 64 rows x 64 columns, one float per thread and pass
    const int r = (tid >> 6) + 4 * i, c = tid & 63;
    tile[r][c] = (r0 + r < R && c0 + c < C) ? src[(size_t)(r0 + r) * C + c0 + c] : 0.f;
  }
  __syncthreads();
  bf16* dst = mc.tdst[sg];
  const int ld = mc.tld[sg];
#pragma unroll
  for (int i = 0; i < 16; ++i) {  // destination row c0 + c, 64 consecutive r
    const int c = (tid >> 6) + 4 * i, r = tid & 63;
    if (c0 + c < C && r0 + r < R) dst[(size_t)(c0 + c) * ld + r0 + r] = f2bf(tile[r][c]);
  }
}

__global__ __launch_bounds__(256) void multi_cast_kernel(const MultiCast mc) {
  // the transposed tiles first (the lowest block ids start first): their load -> LDS -> store
  // chain then overlaps the streaming blocks instead of trailing them (+3 us per launch at the end)
  const int nt = mc.tblk0[mc.ntseg];
  if ((int)blockIdx.x < nt) {  // block-uniform
    mcast_t_tile(mc, (int)blockIdx.x);
    return;
  }
  const int bx = (int)blockIdx.x - nt;
  int lo = 0, hi = mc.nseg - 1;  // last segment with blk0 <= bx
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (mc.blk0[mid] <= bx) lo = mid;
    else hi = mid - 1;
  }
  const int sg = lo;
  if (bx == 0 && threadIdx.x == 0) {
    if (mc.bump != nullptr) *mc.bump += 1;
    if (mc.bump2 != nullptr) *mc.bump2 += 1;
  }
  const long base = (long)(bx - mc.blk0[sg]) * MCAST_CHUNK;
  const float4* s4 = (const float4*)mc.src[sg];
  const long n = mc.n[sg];
  const int fs = mc.fslot[sg];
  const long ns = fs >= 0 ? mc.nsrc[fs] : n;  // words read from the source (the rest: fill)
#pragma unroll
  for (int it = 0; it < MCAST_CHUNK / (256 * 8); ++it) {
    const long e = base + ((long)it * 256 + threadIdx.x) * 8;
    if (e < n && (!mc.vec[sg] || e + 8 > ns)) {  // unaligned segment, its ragged tail or fill
      const float* src = mc.src[sg];
      for (int j = 0; j < 8 && e + j < n; ++j) {
        if (mc.bf[sg]) ((bf16*)mc.dst[sg])[e + j] = f2bf(src[e + j]);
        else ((int*)mc.dst[sg])[e + j] = e + j < ns ? ((const int*)src)[e + j] : mc.fill[fs];  // bits
      }
    } else if (e < n) {
      const float4 a = s4[e >> 2], b = s4[(e >> 2) + 1];
      if (mc.bf[sg]) {
        *(bf16x8*)((bf16*)mc.dst[sg] + e) =
            bf16x8{f2bf(a.x), f2bf(a.y), f2bf(a.z), f2bf(a.w), f2bf(b.x), f2bf(b.y), f2bf(b.z), f2bf(b.w)};
      } else {
        float4* d4 = (float4*)((float*)mc.dst[sg] + e);
        d4[0] = a;
        d4[1] = b;
      }
    }
  }
}
}  // namespace

// 0 ok; 1 = too many segments / bad size or alignment (the caller rebuilds the pack instead).
// bump (optional): an int64 device counter the launch advances by one -- the training step's
// dropout / noise offset rides in the step's cast launch instead of a launch of its own
// nsrc (optional): per segment, the source words (< n[i]: fp32 / copy segments only; the
// rest of the destination gets fill[i]) -- at most MCAST_FILL such segments per launch
// ntseg transposed segments (tsrc fp32 [tR, tC] -> tdst bf16, element (r, c) at c * tld + r)
// follow the others in the same launch
extern "C" int fr_multi_cast(const float* const* src, void* const* dst, const long* n, const int* to_bf16, int nseg,
                             long long* bump, hipStream_t s, long long* bump2, const long* nsrc, const int* fill,
                             int ntseg, const float* const* tsrc, void* const* tdst, const int* tR, const int* tC,
                             const int* tld) {
  if (nseg < 1 || nseg > MCAST_SEG || ntseg < 0 || ntseg > MCAST_TSEG) return 1;
  MultiCast mc{};
  mc.ntseg = ntseg;
  long tb = 0;
  for (int i = 0; i < ntseg; ++i) {
    if (tR[i] <= 0 || tC[i] <= 0 || tld[i] < tR[i]) return 1;
    mc.tsrc[i] = tsrc[i];
    mc.tdst[i] = (bf16*)tdst[i];
    mc.tR[i] = tR[i];
    mc.tC[i] = tC[i];
    mc.tld[i] = tld[i];
    mc.tblk0[i] = (int)tb;
    tb += (long)((tR[i] + 63) / 64) * ((tC[i] + 63) / 64);
  }
  mc.tblk0[ntseg] = (int)tb;
  mc.nseg = nseg;
  mc.bump = bump;
  mc.bump2 = bump2;
  int nf = 0;
  for (int i = 0; i < nseg; ++i) {
    mc.fslot[i] = -1;
    if (nsrc != nullptr && nsrc[i] != n[i]) {
      if (nsrc[i] < 0 || nsrc[i] > n[i] || to_bf16[i] || nf == MCAST_FILL || fill == nullptr) return 1;
      mc.fslot[i] = (signed char)nf;
      mc.nsrc[nf] = nsrc[i];
      mc.fill[nf] = fill[i];
      ++nf;
    }
  }
  long blk = 0;
  for (int i = 0; i < nseg; ++i) {
    if (n[i] <= 0) return 1;
    mc.vec[i] = (((uintptr_t)src[i] & 15) == 0 && ((uintptr_t)dst[i] & 15) == 0) ? 1 : 0;
    mc.src[i] = src[i];
    mc.dst[i] = dst[i];
    mc.n[i] = n[i];
    mc.bf[i] = to_bf16[i] ? 1 : 0;
    mc.blk0[i] = (int)blk;
    blk += (n[i] + MCAST_CHUNK - 1) / MCAST_CHUNK;
  }
  mc.blk0[nseg] = (int)blk;
  if (blk + tb >= (1L << 31)) return 1;
  hipLaunchKernelGGL(multi_cast_kernel, dim3((unsigned)(blk + tb)), dim3(256), 0, s, mc);
  return 0;
}

// ---------------------------------------------------------------------------------------
// The same refresh into TRANSPOSED bf16 copies (unfrozen backbone: the input-gradient GEMMs
// run on W^T, which was a `wlow.t().contiguous()` copy launch per weight and step): segment i
// is an fp32 [R, C] master, written as bf16 dst[c * ld + r] (ld >= R: the q / k / v blocks
// land side by side in the fused [D, 3D] transposed QKV weight).  64 x 64 tiles through LDS
// (padded rows: conflict-free column reads), R % 64 == C % 64 == 0 (host-checked).
namespace {
constexpr int MCT_SEG = 96;

struct MultiCastT {
  const float* src[MCT_SEG];
  bf16* dst[MCT_SEG];
  int R[MCT_SEG], C[MCT_SEG], ld[MCT_SEG];
  int blk0[MCT_SEG + 1];
  int nseg;
};

__global__ __launch_bounds__(256) void multi_cast_t_kernel(const MultiCastT mc) {
  __shared__ float tile[64][65];
  int lo = 0, hi = mc.nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (mc.blk0[mid] <= (int)blockIdx.x) lo = mid;
    else hi = mid - 1;
  }
  const int sg = lo;
  const int t = blockIdx.x - mc.blk0[sg];
  const int ct = mc.C[sg] >> 6;
  const int r0 = (t / ct) * 64, c0 = (t % ct) * 64;
  const float* src = mc.src[sg];
  const int C = mc.C[sg];
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 64 rows x 16 float4
    const int r = (tid >> 4) + 16 * i, c = (tid & 15) * 4;
    const float4 v = *(const float4*)(src + (size_t)(r0 + r) * C + c0 + c);
    tile[r][c] = v.x;
    tile[r][c + 1] = v.y;
    tile[r][c + 2] = v.z;
    tile[r][c + 3] = v.w;
  }
  __syncthreads();
  bf16* dst = mc.dst[sg];
  const int ld = mc.ld[sg];
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 64 destination rows (source columns) x 8 chunks of 8
    const int c = (tid >> 3) + 32 * i, r = (tid & 7) * 8;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(tile[r + j][c]);
    *(bf16x8*)(dst + (size_t)(c0 + c) * ld + r0 + r) = o;
  }
}
}  // namespace

extern "C" int fr_multi_cast_t(const float* const* src, void* const* dst, const int* R, const int* C, const int* ld,
                               int nseg, hipStream_t s) {
  if (nseg < 1 || nseg > MCT_SEG) return 1;
  MultiCastT mc{};
  mc.nseg = nseg;
  long blk = 0;
  for (int i = 0; i < nseg; ++i) {
    if (R[i] <= 0 || C[i] <= 0 || R[i] % 64 || C[i] % 64 || ld[i] < R[i] || ld[i] % 8 || ((uintptr_t)src[i] & 15) ||
        ((uintptr_t)dst[i] & 15))
      return 1;
    mc.src[i] = src[i];
    mc.dst[i] = (bf16*)dst[i];
    mc.R[i] = R[i];
    mc.C[i] = C[i];
    mc.ld[i] = ld[i];
    mc.blk0[i] = (int)blk;
    blk += (long)(R[i] / 64) * (C[i] / 64);
  }
  mc.blk0[nseg] = (int)blk;
  hipLaunchKernelGGL(multi_cast_t_kernel, dim3((unsigned)blk), dim3(256), 0, s, mc);
  return 0;
}
