// One-shot all-reduce (sum, bf16) over IPC-mapped peer buffers, for the small tensor-parallel
// decode messages (8-16 KB x batch, latency-bound; a ring is
// per-link bound on xGMI while a one-shot read of all peers uses every link at once).
//
// Every rank owns one fine-grained *uncached* allocation (hipDeviceMallocUncached, so peer reads and
// flag polls see memory, not a stale L2 line) mapped into every other rank with hipIpc handles:
//   [ data half 0 : cap elems ][ data half 1 : cap elems ][ flags : AR_MAX_BLOCKS x AR_MAX_RANKS u32 ]
//   [ ctr : u32 ][ done : u32 ][ err : i32 ]
// Block b of every rank owns the same element chunk b.  One call (epoch e = ctr + 1, half = e & 1):
//   1. copy chunk b of the input into my half;  2. system-scope release, then store e into
//   flags[b][me] of every peer;  3. wait until my flags[b][p] >= e for every p (acquire, bounded
//   wait -> err instead of a hang, spin_wait);  4. sum chunk b over all ranks' halves in fp32, write the output;
//   5. the last block to finish stores ctr = e.
// The epoch lives in device memory, so the launch can be captured once in a hipGraph and replayed.
// Halves alternate by epoch parity: a rank rewrites half h in call e + 2 only after every peer has
// signalled call e + 1, i.e. after every peer's call e (which read h) has completed on its stream.
#include <cstring>

#include "common.h"

#define AR_MAX_RANKS 8
#define AR_MAX_BLOCKS 64

// Bounded wait for a peer's flag: wall-clock bound (s_memrealtime, 100 MHz) of AR_SPIN_SECONDS — long
// enough for the first steps' host-side skew between ranks (lazy kernel loading, eager prefill
// setup), short of the engine's step watchdog — after which `err` is set instead of hanging the GPU;
// once `err` is set every later wait gives up at once, so a dead peer costs one bound per process,
// not one per collective.  The host reads `err` with every step (engine/runner.py) and never uses a
// step that set it.
#ifndef AR_SPIN_SECONDS
#define AR_SPIN_SECONDS 20
#endif
KA_DEV void spin_wait(unsigned* f, unsigned epoch, int* err) {
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > (unsigned long long)AR_SPIN_SECONDS * 100000000ull) {
      atomicExch(err, 1);   // a peer never arrived: report, never hang the GPU
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

struct ArArgs {
  bf16_t* data[AR_MAX_RANKS];
  unsigned* flags[AR_MAX_RANKS];
};

__global__ __launch_bounds__(512) void allreduce_oneshot_kernel(ArArgs a, const bf16_t* __restrict__ in,
                                                                bf16_t* out, unsigned* ctr, unsigned* done,
                                                                int* err, int rank, int world, int n, int cap) {
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const unsigned epoch = s_epoch;
  const size_t half = (size_t)(epoch & 1u) * cap;
  const int chunk = ((n + (int)gridDim.x - 1) / (int)gridDim.x + 7) / 8 * 8;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);

  bf16_t* mine = a.data[rank] + half;
  for (int i = beg + threadIdx.x * 8; i < end; i += blockDim.x * 8)
    *reinterpret_cast<u32x4*>(mine + i) = *reinterpret_cast<const u32x4*>(in + i);
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < world) {
    const int p = threadIdx.x;
    __hip_atomic_store(a.flags[p] + blockIdx.x * AR_MAX_RANKS + rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* f = a.flags[rank] + blockIdx.x * AR_MAX_RANKS + p;
    spin_wait(f, epoch, err);
  }
  __syncthreads();

  for (int i = beg + threadIdx.x * 8; i < end; i += blockDim.x * 8) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // every peer's piece is loaded before the first add (one remote round trip, not `world`);
    // summed in rank order
    u32x4 v[AR_MAX_RANKS];
#pragma unroll
    for (int p = 0; p < AR_MAX_RANKS; ++p)
      if (p < world) v[p] = *reinterpret_cast<const u32x4*>(a.data[p] + half + i);
#pragma unroll
    for (int p = 0; p < AR_MAX_RANKS; ++p) {
      if (p < world) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s[2 * j] += lo_f(v[p][j]);
          s[2 * j + 1] += hi_f(v[p][j]);
        }
      }
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack2(s[2 * j], s[2 * j + 1]);
    *reinterpret_cast<u32x4*>(out + i) = o;
  }

  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {   // every block has read ctr and finished: publish the epoch
      *done = 0u;
      __hip_atomic_store(ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One-shot all-gather on the same buffers, flags and epoch sequence (A3: the vocab-parallel
// argmax winners; graph-capturable like the all-reduce, so a TP decode graph holds every
// collective).  n16 = payload size in 16-bit units (multiple of 8); out receives world * n16
// units in rank order.  Calls of both kernels share `ctr`: every rank issues the same sequence.
__global__ __launch_bounds__(512) void allgather_oneshot_kernel(ArArgs a, const bf16_t* __restrict__ in,
                                                                bf16_t* out, unsigned* ctr, unsigned* done,
                                                                int* err, int rank, int world, int n, int cap) {
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const unsigned epoch = s_epoch;
  const size_t half = (size_t)(epoch & 1u) * cap;
  const int chunk = ((n + (int)gridDim.x - 1) / (int)gridDim.x + 7) / 8 * 8;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);

  bf16_t* mine = a.data[rank] + half;
  for (int i = beg + threadIdx.x * 8; i < end; i += blockDim.x * 8)
    *reinterpret_cast<u32x4*>(mine + i) = *reinterpret_cast<const u32x4*>(in + i);
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < world) {
    const int p = threadIdx.x;
    __hip_atomic_store(a.flags[p] + blockIdx.x * AR_MAX_RANKS + rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* f = a.flags[rank] + blockIdx.x * AR_MAX_RANKS + p;
    spin_wait(f, epoch, err);
  }
  __syncthreads();
  for (int p = 0; p < world; ++p)
    for (int i = beg + threadIdx.x * 8; i < end; i += blockDim.x * 8)
      *reinterpret_cast<u32x4*>(out + (size_t)p * n + i) = *reinterpret_cast<const u32x4*>(a.data[p] + half + i);

  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {
      *done = 0u;
      __hip_atomic_store(ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One-shot all-reduce fused with the residual add + RMSNorm that follows every row-parallel
// projection (A1 after O-proj, A2 after down-proj): block b owns whole rows, so after the flag
// handshake it sums its rows over the ranks, adds the residual (updated in place) and normalises —
// the reduced activation never makes a round trip through memory and one launch replaces two.
// Arithmetic is that of all-reduce -> rmsnorm_kernel (elementwise.hip) exactly: the rank sum is
// rounded to bf16, the residual sum is rounded to bf16, fp32 sum of squares.  hidden <= 8192.
// split > 1: `in` holds the producing GEMM's split-K partial slabs [split, rows, hidden] (fp32, or bf16
// when in_bf16) and this rank's contribution is their fp32 sum rounded to bf16 — what splitk_reduce
// would have written — computed while staging it into the exchange buffer: the row-parallel O / down
// projections of a TP rank hand their partials straight to the collective (one launch and one HBM
// round trip fewer per projection, as the TP = 1 path's fused split-K reduce + RMSNorm).
__global__ __launch_bounds__(512) void allreduce_rmsnorm_kernel(ArArgs a, const void* __restrict__ in,
                                                                bf16_t* __restrict__ out, bf16_t* residual,
                                                                const bf16_t* __restrict__ w, float eps,
                                                                unsigned* ctr, unsigned* done, int* err, int rank,
                                                                int world, int rows, int hidden, int cap, int split,
                                                                int in_bf16) {
  __shared__ unsigned s_epoch;
  __shared__ float red[8];
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const unsigned epoch = s_epoch;
  const size_t half = (size_t)(epoch & 1u) * cap;
  const int rpb = (rows + (int)gridDim.x - 1) / (int)gridDim.x;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  const int beg = r0 * hidden, end = r1 * hidden;

  bf16_t* mine = a.data[rank] + half;
  if (split <= 1 && in_bf16) {
    const bf16_t* src = static_cast<const bf16_t*>(in);
    for (int i = beg + threadIdx.x * 8; i < end; i += blockDim.x * 8)
      *reinterpret_cast<u32x4*>(mine + i) = *reinterpret_cast<const u32x4*>(src + i);
  } else {
    const size_t ps = (size_t)rows * hidden;   // elements per slab
    // the slabs are loaded AR_SK_BATCH at a time, each batch issued before its first add (a rolled
    // loop waited for every slab); summed in slab order
    constexpr int AR_SK_BATCH = 4;
    for (int i = beg + threadIdx.x * 8; i < end; i += blockDim.x * 8) {
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int z0 = 0; z0 < split; z0 += AR_SK_BATCH) {
        if (in_bf16) {
          u32x4 v[AR_SK_BATCH];
#pragma unroll
          for (int z = 0; z < AR_SK_BATCH; ++z)
            if (z0 + z < split) v[z] = *reinterpret_cast<const u32x4*>(static_cast<const bf16_t*>(in) + (z0 + z) * ps + i);
#pragma unroll
          for (int z = 0; z < AR_SK_BATCH; ++z) {
            if (z0 + z < split) {
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                s[2 * k] += lo_f(v[z][k]);
                s[2 * k + 1] += hi_f(v[z][k]);
              }
            }
          }
        } else {
          f32x4 v0[AR_SK_BATCH], v1[AR_SK_BATCH];
#pragma unroll
          for (int z = 0; z < AR_SK_BATCH; ++z) {
            if (z0 + z < split) {
              const float* f = static_cast<const float*>(in) + (z0 + z) * ps + i;
              v0[z] = *reinterpret_cast<const f32x4*>(f);
              v1[z] = *reinterpret_cast<const f32x4*>(f + 4);
            }
          }
#pragma unroll
          for (int z = 0; z < AR_SK_BATCH; ++z) {
            if (z0 + z < split) {
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                s[k] += v0[z][k];
                s[4 + k] += v1[z][k];
              }
            }
          }
        }
      }
      u32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = pack2(s[2 * k], s[2 * k + 1]);
      *reinterpret_cast<u32x4*>(mine + i) = o;
    }
  }
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < world) {
    const int p = threadIdx.x;
    __hip_atomic_store(a.flags[p] + blockIdx.x * AR_MAX_RANKS + rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* f = a.flags[rank] + blockIdx.x * AR_MAX_RANKS + p;
    spin_wait(f, epoch, err);
  }
  __syncthreads();

  const int nvec = hidden >> 3;
  for (int row = r0; row < r1; ++row) {
    float v[2][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = threadIdx.x + i * 512;
      if (idx >= nvec) continue;
      const size_t e = (size_t)row * hidden + idx * 8;
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      // every peer's contribution (and the residual) is loaded before the first add, so the peer
      // reads over xGMI overlap instead of costing one remote round trip each; summed in rank order
      u32x4 pv[AR_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < AR_MAX_RANKS; ++p)
        if (p < world) pv[p] = *reinterpret_cast<const u32x4*>(a.data[p] + half + e);
      u32x4 b = u32x4{0u, 0u, 0u, 0u};
      if (residual != nullptr) b = *reinterpret_cast<const u32x4*>(residual + e);
#pragma unroll
      for (int p = 0; p < AR_MAX_RANKS; ++p) {
        if (p < world) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            s[2 * k] += lo_f(pv[p][k]);
            s[2 * k + 1] += hi_f(pv[p][k]);
          }
        }
      }
      uint32_t o[4];
      if (residual != nullptr) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t aw = pack2(s[2 * k], s[2 * k + 1]);   // the all-reduce output, bf16
          v[i][2 * k] = bf2f(f2bf(lo_f(aw) + lo_f(b[k])));
          v[i][2 * k + 1] = bf2f(f2bf(hi_f(aw) + hi_f(b[k])));
          o[k] = pack2(v[i][2 * k], v[i][2 * k + 1]);
        }
        *reinterpret_cast<u32x4*>(residual + e) = u32x4{o[0], o[1], o[2], o[3]};
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t aw = pack2(s[2 * k], s[2 * k + 1]);
          v[i][2 * k] = lo_f(aw);
          v[i][2 * k + 1] = hi_f(aw);
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) ss += v[i][k] * v[i][k];
    }
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) tot += red[i];
    const float scale = rsqrtf(tot / (float)hidden + eps);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = threadIdx.x + i * 512;
      if (idx >= nvec) continue;
      const size_t e = (size_t)row * hidden + idx * 8;
      const u32x4 g = *reinterpret_cast<const u32x4*>(w + idx * 8);
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = pack2(v[i][2 * k] * scale * lo_f(g[k]), v[i][2 * k + 1] * scale * hi_f(g[k]));
      *reinterpret_cast<u32x4*>(out + e) = u32x4{o[0], o[1], o[2], o[3]};
    }
    __syncthreads();   // red[] is rewritten by the next row
  }

  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {
      *done = 0u;
      __hip_atomic_store(ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- host helpers (ops/_hip.py ctypes; parallel/custom_allreduce.py) ----
extern "C" int ka_ar_alloc(void** ptr, size_t bytes) {
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*ptr, 0, bytes);
}

extern "C" int ka_ar_free(void* ptr) { return (int)hipFree(ptr); }

extern "C" int ka_ar_get_handle(void* ptr, void* out64) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e == hipSuccess) memcpy(out64, &h, sizeof(h));
  return (int)e;
}

extern "C" int ka_ar_open_handle(const void* in64, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, in64, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int ka_ar_close_handle(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// data / flags: host arrays of `world` device pointers (rank order); ctr/done/err: this rank's
// counters.  n must be a multiple of 8 and <= cap.
extern "C" int ka_allreduce_oneshot(void* out, const void* in, void* const* data, void* const* flags, void* ctr,
                                    void* done, void* err, int rank, int world, int n, int cap, int nblocks,
                                    hipStream_t stream) {
  if (n <= 0) return 0;
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || n % 8 || n > cap || nblocks < 1 ||
      nblocks > AR_MAX_BLOCKS)
    return (int)hipErrorInvalidValue;
  ArArgs a;
  for (int p = 0; p < AR_MAX_RANKS; ++p) {
    a.data[p] = p < world ? static_cast<bf16_t*>(data[p]) : nullptr;
    a.flags[p] = p < world ? static_cast<unsigned*>(flags[p]) : nullptr;
  }
  // nblocks must be identical on every rank (block b of each rank owns chunk b)
  hipLaunchKernelGGL(allreduce_oneshot_kernel, dim3(nblocks), dim3(512), 0, stream, a,
                     static_cast<const bf16_t*>(in), static_cast<bf16_t*>(out), static_cast<unsigned*>(ctr),
                     static_cast<unsigned*>(done), static_cast<int*>(err), rank, world, n, cap);
  KA_CHECK_LAUNCH();
}

// out: world * n16 16-bit units; in: n16 units (n16 % 8 == 0, n16 <= cap)
extern "C" int ka_allgather_oneshot(void* out, const void* in, void* const* data, void* const* flags, void* ctr,
                                    void* done, void* err, int rank, int world, int n16, int cap, int nblocks,
                                    hipStream_t stream) {
  if (n16 <= 0) return 0;
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || n16 % 8 || n16 > cap || nblocks < 1 ||
      nblocks > AR_MAX_BLOCKS)
    return (int)hipErrorInvalidValue;
  ArArgs a;
  for (int p = 0; p < AR_MAX_RANKS; ++p) {
    a.data[p] = p < world ? static_cast<bf16_t*>(data[p]) : nullptr;
    a.flags[p] = p < world ? static_cast<unsigned*>(flags[p]) : nullptr;
  }
  hipLaunchKernelGGL(allgather_oneshot_kernel, dim3(nblocks), dim3(512), 0, stream, a,
                     static_cast<const bf16_t*>(in), static_cast<bf16_t*>(out), static_cast<unsigned*>(ctr),
                     static_cast<unsigned*>(done), static_cast<int*>(err), rank, world, n16, cap);
  KA_CHECK_LAUNCH();
}

// in: this rank's partial [rows, hidden] bf16 (split <= 1, in_bf16 = 1), or split-K partial slabs
// [split, rows, hidden] of fp32 (in_bf16 = 0) / bf16 (in_bf16 = 1); out: rmsnorm(sum + residual) * w;
// residual (may be null) is updated in place to sum + residual.  rows * hidden <= cap, hidden % 8 == 0,
// <= 8192; nblocks (identical on every rank) <= min(rows, AR_MAX_BLOCKS).
extern "C" int ka_allreduce_rmsnorm(void* out, const void* in, void* residual, const void* w, float eps,
                                    void* const* data, void* const* flags, void* ctr, void* done, void* err, int rank,
                                    int world, int rows, int hidden, int cap, int nblocks, int split, int in_bf16,
                                    hipStream_t stream) {
  if (rows <= 0) return 0;
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || hidden % 8 || hidden > 8192 ||
      (long)rows * hidden > cap || nblocks < 1 || nblocks > AR_MAX_BLOCKS || nblocks > rows || split < 1 ||
      (split == 1 && !in_bf16))
    return (int)hipErrorInvalidValue;
  ArArgs a;
  for (int p = 0; p < AR_MAX_RANKS; ++p) {
    a.data[p] = p < world ? static_cast<bf16_t*>(data[p]) : nullptr;
    a.flags[p] = p < world ? static_cast<unsigned*>(flags[p]) : nullptr;
  }
  hipLaunchKernelGGL(allreduce_rmsnorm_kernel, dim3(nblocks), dim3(512), 0, stream, a, in,
                     static_cast<bf16_t*>(out), static_cast<bf16_t*>(residual),
                     static_cast<const bf16_t*>(w), eps, static_cast<unsigned*>(ctr), static_cast<unsigned*>(done),
                     static_cast<int*>(err), rank, world, rows, hidden, cap, split, in_bf16);
  KA_CHECK_LAUNCH();
}
