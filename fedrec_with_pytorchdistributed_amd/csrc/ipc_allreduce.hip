// Peer-to-peer all-reduce over IPC-mapped device buffers: the custom
// alternative to RCCL for the data plane's buckets on one node (one process per GPU, xGMI).
//
// Every rank owns one registered region, allocated uncached (hipDeviceMallocUncached: remote
// reads over xGMI and local writes never sit in a stale cache line) and exported with
// hipIpcGetMemHandle; the handles are exchanged over the gloo control group and every peer's
// region is opened with hipIpcOpenMemHandle.  Region layout:
//
//   [ flags: 2 phases x MAXW ranks x MAXB blocks x 8 B ][ slot 0 | slot 1 ]   slot = cap bytes,
//   used by call parity.  Flags are per (phase, writer rank, writer block): a reader block
//   proceeds only when EVERY block of every rank has published its part of the phase.
//
// A call with epoch e (monotonic, same on every rank):
//   one-shot  x -> my slot[e & 1]; release; flag[0][me] := e on every peer; wait until
//             every flag[0][p] of mine >= e (acquire); x[i] = sum_p slot_p[e & 1][i] in a fixed
//             peer order (0..W-1: every rank computes the bitwise-same sum).
//   two-shot  x -> my slot; barrier 0; rank r reduces slice r of every peer's slot into its
//             own slot's slice r; barrier 1 (phase-1 flags); x gathers every slice from its
//             owner.  2 (W-1)/W S read per rank instead of (W-1) S.
// Slot reuse: slot e & 1 is rewritten at epoch e + 2, after this rank passed the barrier of
// epoch e + 1, which every peer entered only after finishing its reads of epoch e.
// Types: fp32 SUM, int32 wrap-around SUM (secure aggregation's masked fixed point).
// Device epochs (a context created for capture, epoch argument 0): the epoch is NOT a launch
// argument but the context's device counter + 1, so a launch captured once in a HIP graph runs
// a fresh epoch on every replay.  Every block reads the counter first; a block that passed the
// phase-0 barrier knows every block of every rank has started (and read it), so it stores the
// new value back (the same value from every block; a vector store) -- the next launch on the
// stream reads it after this one completed.
//
// Liveness: the waits are bounded by a wall-clock deadline (the caller's collective timeout);
// then a status word records the timeout, the output is poisoned (NaN / INT_MIN) and the
// kernel exits, so a missing peer cannot hang the GPU and cannot yield a silently wrong sum;
// the host raises on the status word at its next check (IpcAllReduce.check: the GA step wrapper
// at every epoch end, the bench).  All flag traffic is vector stores / loads with system-scope
// ordering.
#include "common.h"

#include <stdint.h>

namespace {

constexpr int MAXW = 16, MAXB = 64;
constexpr int FLAG_BYTES = 2 * MAXW * MAXB * 8;
constexpr int AR_BLOCKS = 16, AR_THREADS = 256;

struct Peers {
  char* base[MAXW];  // every rank's region (own included), as mapped in this process
};

__device__ __forceinline__ long long* flag_ptr(char* region, int phase, int r, int blk) {
  return (long long*)(region + ((phase * MAXW + r) * MAXB + blk) * 8);
}

// grid-wide barrier among the W ranks for `phase` / `epoch`: this block publishes (its writes,
// then flag[phase][me][block] := epoch in every rank's region), then waits until every block of
// every rank has published.  Publication order: EVERY thread makes its own slot stores visible
// at system scope (release fence + drained vmcnt) before the workgroup barrier, and only then
// do lanes < W store the flags -- a workgroup-scope barrier alone orders other waves' stores
// for this CU, not for a remote agent.  The inline vmcnt(0) after the fences is deliberate: the
// compiler may drop the wait after the L2 write-back when it believes vmcnt is already empty.
// Waits are bounded by a wall-clock deadline (s_memrealtime, 100 MHz): on timeout the status
// word is set and the caller poisons its output; returns false then.
__device__ bool rank_barrier(const Peers& P, int me, int W, int phase, long long epoch, int* status, int blk,
                             int nb, unsigned long long deadline_ticks) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope, every thread: its own stores first
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave of this block has published its stores
  if (threadIdx.x < (unsigned)W) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag_ptr(P.base[threadIdx.x], phase, me, blk), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  bool ok = true;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int j = threadIdx.x; j < W * nb; j += blockDim.x) {
    long long* f = flag_ptr(P.base[me], phase, j / nb, j % nb);
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > deadline_ticks) {  // a peer never arrived
        ok = false;
        __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return __syncthreads_and(ok);
}

// a timed-out call leaves this block's part of x poisoned (fp32: NaN, int32: INT_MIN, a value
// no masked sum depends on being), so a caller that misses the status word still fails loudly
template <typename T>
__device__ void poison(T* __restrict__ x, long n4, long t0, long stride) {
  const T v = __is_same(T, int) ? (T)(-2147483647 - 1) : (T)__builtin_nanf("");
  for (long i = t0; i < n4; i += stride) {
    T* p = x + 4 * i;
    p[0] = v;
    p[1] = v;
    p[2] = v;
    p[3] = v;
  }
}

template <typename T>
__device__ __forceinline__ void add4(T (&a)[4], const T* __restrict__ p) {
  if constexpr (sizeof(T) == 4 && __is_same(T, int)) {
    const int4 v = *(const int4*)p;
    a[0] = (int)((unsigned)a[0] + (unsigned)v.x);
    a[1] = (int)((unsigned)a[1] + (unsigned)v.y);
    a[2] = (int)((unsigned)a[2] + (unsigned)v.z);
    a[3] = (int)((unsigned)a[3] + (unsigned)v.w);
  } else {
    const float4 v = *(const float4*)p;
    a[0] += v.x;
    a[1] += v.y;
    a[2] += v.z;
    a[3] += v.w;
  }
}

// One launch per rank (me = me_arg, grid = nb blocks) -- or, for the single-process rehearsal,
// ONE launch playing every rank (xs.x[r] per rank, grid = W x nb blocks, rank = block / nb):
// then all ranks are co-resident by construction, whatever the stream-to-queue mapping.
template <typename T>
struct Xs {
  T* x[MAXW];
  int* status[MAXW];
};

// x: n elements (n % 4 == 0), in place.  mode 0 one-shot, 1 two-shot.
template <typename T>
__global__ __launch_bounds__(AR_THREADS) void ipc_allreduce_kernel(Xs<T> xs, long n, Peers P, int me_arg, int W,
                                                                  long long epoch, long cap, int mode, int nb,
                                                                  int multi, unsigned long long deadline,
                                                                  long long* __restrict__ dev_epoch) {
  const int me = multi ? (int)blockIdx.x / nb : me_arg;
  const int blk = multi ? (int)blockIdx.x % nb : (int)blockIdx.x;
  T* __restrict__ x = xs.x[multi ? me : 0];
  int* status = xs.status[multi ? me : 0];
  if (dev_epoch != nullptr) epoch = __hip_atomic_load(dev_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const long slot_off = FLAG_BYTES + (long)(epoch & 1) * cap;
  T* mine = (T*)(P.base[me] + slot_off);
  const long n4 = n / 4;
  const long stride = (long)nb * blockDim.x;
  const long t0 = (long)blk * blockDim.x + threadIdx.x;
  // a previous call timed out: the peers' epochs no longer line up -- fail fast (poisoned)
  if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
    poison(x, n4, t0, stride);
    return;
  }
  for (long i = t0; i < n4; i += stride) *(float4*)(mine + 4 * i) = *(const float4*)(x + 4 * i);
  if (!rank_barrier(P, me, W, 0, epoch, status, blk, nb, deadline)) {
    poison(x, n4, t0, stride);
    return;
  }
  if (dev_epoch != nullptr && threadIdx.x == 0)
    __hip_atomic_store(dev_epoch, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (mode == 0) {
    for (long i = t0; i < n4; i += stride) {
      T acc[4] = {0, 0, 0, 0};
      for (int p = 0; p < W; ++p) add4(acc, (const T*)(P.base[p] + slot_off) + 4 * i);
      *(float4*)(x + 4 * i) = __builtin_bit_cast(float4, acc);
    }
    return;
  }
  // two-shot: slice r = [lo_r, hi_r) in units of 4 elements
  const long per = (n4 + W - 1) / W;
  const long lo = (long)me * per, hi = lo + per < n4 ? lo + per : n4;
  for (long i = lo + t0; i < hi; i += stride) {
    T acc[4] = {0, 0, 0, 0};
    for (int p = 0; p < W; ++p) add4(acc, (const T*)(P.base[p] + slot_off) + 4 * i);
    *(float4*)(mine + 4 * i) = __builtin_bit_cast(float4, acc);  // own slice of own slot: reduced
  }
  if (!rank_barrier(P, me, W, 1, epoch, status, blk, nb, deadline)) {
    poison(x, n4, t0, stride);
    return;
  }
  // gather: four independent remote loads in flight per thread (xGMI latency)
  long i = t0;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long j = i + u * stride;
      v[u] = *(const float4*)((const T*)(P.base[(int)(j / per)] + slot_off) + 4 * j);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) *(float4*)(x + 4 * (i + u * stride)) = v[u];
  }
  for (; i < n4; i += stride) {
    const int owner = (int)(i / per);
    *(float4*)(x + 4 * i) = *(const float4*)((const T*)(P.base[owner] + slot_off) + 4 * i);
  }
}

struct Ctx {
  char* region = nullptr;
  long cap = 0;
  int me = 0, W = 0;
  Peers P{};
  bool opened[MAXW] = {};
  int* status = nullptr;
  long long* dev_epoch = nullptr;  // device epochs (epoch argument 0)
};

Ctx* g_ctx[64] = {};

}  // namespace

// allocate this rank's region (flags + 2 slots of cap bytes); returns a context id >= 0 and the
// 64-byte IPC handle in `handle_out`
extern "C" int fr_ipc_create(long cap, void* handle_out) {
  int id = -1;
  for (int i = 0; i < 64; ++i)
    if (g_ctx[i] == nullptr) {
      id = i;
      break;
    }
  if (id < 0 || cap <= 0 || cap % 16 != 0) return -1;
  Ctx* c = new Ctx();
  c->cap = cap;
  const size_t bytes = FLAG_BYTES + 2 * (size_t)cap;
  if (hipExtMallocWithFlags((void**)&c->region, bytes, hipDeviceMallocUncached) != hipSuccess) {
    delete c;
    return -2;
  }
  if (hipMemset(c->region, 0, FLAG_BYTES) != hipSuccess || hipMalloc((void**)&c->status, sizeof(int)) != hipSuccess ||
      hipMemset(c->status, 0, sizeof(int)) != hipSuccess ||
      hipMalloc((void**)&c->dev_epoch, sizeof(long long)) != hipSuccess ||
      hipMemset(c->dev_epoch, 0, sizeof(long long)) != hipSuccess) {
    (void)hipFree(c->region);
    if (c->status) (void)hipFree(c->status);
    if (c->dev_epoch) (void)hipFree(c->dev_epoch);
    delete c;
    return -3;
  }
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, c->region) != hipSuccess) {
    (void)hipFree(c->region);
    (void)hipFree(c->status);
    (void)hipFree(c->dev_epoch);
    delete c;
    return -4;
  }
  for (int i = 0; i < 64; ++i) ((char*)handle_out)[i] = h.reserved[i];
  (void)hipDeviceSynchronize();
  g_ctx[id] = c;
  return id;
}

// handles: W x 64 bytes (rank order).  local_ptrs (optional, nullable): regions of ranks that
// live in THIS process (the single-process rehearsal), used instead of opening their handle.
extern "C" int fr_ipc_open(int id, const void* handles, int me, int W, const long long* local_ptrs) {
  if (id < 0 || id >= 64 || g_ctx[id] == nullptr || W < 1 || W > MAXW || me < 0 || me >= W) return -1;
  Ctx* c = g_ctx[id];
  c->me = me;
  c->W = W;
  for (int p = 0; p < W; ++p) {
    if (p == me) {
      c->P.base[p] = c->region;
      continue;
    }
    if (local_ptrs != nullptr && local_ptrs[p] != 0) {
      c->P.base[p] = (char*)local_ptrs[p];
      continue;
    }
    hipIpcMemHandle_t h;
    for (int i = 0; i < 64; ++i) h.reserved[i] = ((const char*)handles)[p * 64 + i];
    void* ptr = nullptr;
    if (hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -10 - p;
    c->P.base[p] = (char*)ptr;
    c->opened[p] = true;
  }
  return 0;
}

extern "C" long long fr_ipc_region(int id) {
  return (id >= 0 && id < 64 && g_ctx[id]) ? (long long)(uintptr_t)g_ctx[id]->region : 0;
}

extern "C" int* fr_ipc_status(int id) { return (id >= 0 && id < 64 && g_ctx[id]) ? g_ctx[id]->status : nullptr; }

// x: device pointer of n elements (is_int: int32 wrap-around sum, else fp32); n % 4 == 0 and
// n * 4 <= cap (host-checked by the caller)
// timeout_s: bound of every barrier wait (wall clock; the status word records a timeout)
// epoch 0: the context's device epoch (capturable); a context must use one kind only
extern "C" int fr_ipc_allreduce(int id, void* x, long n, int is_int, long long epoch, int mode, int blocks,
                                double timeout_s, hipStream_t s) {
  if (id < 0 || id >= 64 || g_ctx[id] == nullptr) return -1;
  Ctx* c = g_ctx[id];
  if (n % 4 != 0 || n * 4 > c->cap || c->W < 1 || epoch < 0) return -2;
  if (n == 0) return 0;
  const int nb = blocks > 0 ? (blocks < MAXB ? blocks : MAXB) : AR_BLOCKS;
  const unsigned long long dl = (unsigned long long)((timeout_s > 0 ? timeout_s : 60.0) * 1e8);
  long long* de = epoch == 0 ? c->dev_epoch : nullptr;
  if (is_int) {
    Xs<int> xs{};
    xs.x[0] = (int*)x;
    xs.status[0] = c->status;
    hipLaunchKernelGGL(ipc_allreduce_kernel<int>, dim3(nb), dim3(AR_THREADS), 0, s, xs, n, c->P, c->me, c->W, epoch,
                       c->cap, mode, nb, 0, dl, de);
  } else {
    Xs<float> xs{};
    xs.x[0] = (float*)x;
    xs.status[0] = c->status;
    hipLaunchKernelGGL(ipc_allreduce_kernel<float>, dim3(nb), dim3(AR_THREADS), 0, s, xs, n, c->P, c->me, c->W,
                       epoch, c->cap, mode, nb, 0, dl, de);
  }
  return 0;
}

// single-process rehearsal: ids[W] contexts of this process (opened with local_ptrs), xs[W] their
// inputs; one launch plays every rank
extern "C" int fr_ipc_allreduce_local(const int* ids, void* const* xs_in, int W, long n, int is_int, long long epoch,
                                      int mode, int blocks, double timeout_s, hipStream_t s) {
  if (W < 1 || W > MAXW) return -1;
  for (int r = 0; r < W; ++r)
    if (ids[r] < 0 || ids[r] >= 64 || g_ctx[ids[r]] == nullptr || g_ctx[ids[r]]->me != r) return -1;
  Ctx* c = g_ctx[ids[0]];
  if (n % 4 != 0 || n * 4 > c->cap) return -2;
  if (n == 0) return 0;
  const int nb = blocks > 0 ? (blocks < MAXB ? blocks : MAXB) : AR_BLOCKS;
  const unsigned long long dl = (unsigned long long)((timeout_s > 0 ? timeout_s : 60.0) * 1e8);
  if (is_int) {
    Xs<int> xs{};
    for (int r = 0; r < W; ++r) {
      xs.x[r] = (int*)xs_in[r];
      xs.status[r] = g_ctx[ids[r]]->status;
    }
    hipLaunchKernelGGL(ipc_allreduce_kernel<int>, dim3(nb * W), dim3(AR_THREADS), 0, s, xs, n, c->P, 0, W, epoch,
                       c->cap, mode, nb, 1, dl, (long long*)nullptr);
  } else {
    Xs<float> xs{};
    for (int r = 0; r < W; ++r) {
      xs.x[r] = (float*)xs_in[r];
      xs.status[r] = g_ctx[ids[r]]->status;
    }
    hipLaunchKernelGGL(ipc_allreduce_kernel<float>, dim3(nb * W), dim3(AR_THREADS), 0, s, xs, n, c->P, 0, W, epoch,
                       c->cap, mode, nb, 1, dl, (long long*)nullptr);
  }
  return 0;
}

extern "C" int fr_ipc_destroy(int id) {
  if (id < 0 || id >= 64 || g_ctx[id] == nullptr) return -1;
  Ctx* c = g_ctx[id];
  (void)hipDeviceSynchronize();
  for (int p = 0; p < MAXW; ++p)
    if (c->opened[p]) (void)hipIpcCloseMemHandle(c->P.base[p]);
  (void)hipFree(c->region);
  (void)hipFree(c->status);
  (void)hipFree(c->dev_epoch);
  delete c;
  g_ctx[id] = nullptr;
  return 0;
}
