// Deep-prefetch LDS-DMA MFMA GEMM for decode-sized M (<= 256 rows per tile):
//   Y[M, N] = X[M, K] * W[N, K]^T, bf16 in/out, fp32 accumulate, optional split-K partials.
//
// Why another decode GEMM: at M = 256 the Llama-3-8B projections are HBM-bound (256 FLOP per
// weight byte against the chip's ~400), yet the register-staged tile kernel (gemm_tile.hip) and
// hipBLASLt keep only ONE k-step of weights in flight per workgroup, so each k-step pays a full
// loaded-HBM latency: O-proj 26 us for 33.5 MB (1.3 TB/s), QKV ~25 us for 50 MB.  What a CU needs
// to stream at its share of 6 TB/s is tens of KB of weights in flight (MI355X_MICROARCH.md:
// "72 KiB in flight per CU hide most of an HBM miss").  Design (guide §5 "Pipelining across
// barriers", "Projection GEMM at M = 256"):
//   * BK = 32 stages (64-B rows), so the 160 KB LDS holds S = 4..8 stages: S - 1 stages of W AND X
//     are in flight while one is consumed;
//   * both operands arrive by LDS-DMA (`global_load_lds_dwordx4`, 1 KB = 16 rows per
//     wave-instruction, lane-linear image) — no VGPR staging, no ds_write pass, and no ordinary
//     VGPR-destination global load anywhere in the k-loop (hipcc would drain the DMA queue with
//     vmcnt(0) at its use: guide §5 trap (b));
//   * the image is XOR-swizzled on the SOURCE address: LDS row r holds its 16-B chunk c at slot
//     c ^ ((r >> 1) & 3), which makes every ds_read_b128 lane group of a 16x16x32 fragment read
//     (rows r16 = lane & 15, chunk lane >> 4) hit 16 distinct 16-B bank slots (brute-forced
//     against MI355X_MICROARCH.md's ds_read_b128 lane groups);
//   * one barrier per k-step: counted `s_waitcnt vmcnt((S-2) * loads_per_stage)` retires this
//     thread's DMAs for stage t, the raw `s_barrier` then makes every wave's stage t visible AND
//     proves every wave finished reading stage t-1, whose slot is refilled with stage t+S-1 right
//     after the barrier.  Stages past the end re-load the last stage (L2 hit) into a slot nobody
//     reads again, so the wait counts stay compile-time constants; the DMA queue is drained
//     (vmcnt(0)) before the epilogue so no LDS write lands after the workgroup retires;
//   * W is loaded non-temporal (streamed once per call) so the X panel, re-read by every column
//     tile, stays in the XCD's L2.
// Output: bf16 Y, or fp32 partials P[z][M][N] for split-K (consumed by a fused reduction:
// rmsnorm_splitk / rope_kv_splitk / silu_mul_splitk, or splitk_reduce_kernel).
#include "common.h"

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
KA_DEV void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

KA_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

KA_DEV int sw4(int row, int c) { return c ^ ((row >> 1) & 3); }

template <int WN, int WM, int TN, int TM, int S>
struct StreamCfg {
  static constexpr int BN = WN * TN * 16;
  static constexpr int BM = WM * TM * 16;
  static constexpr int NW = WN * WM;
  static constexpr int NT = 64 * NW;
  static constexpr int ROWS = BN + BM;             // LDS rows per stage: W rows, then X rows
  static constexpr int STAGE_BYTES = ROWS * 64;
  static constexpr int IW = BN / 16 / NW;          // W DMA wave-instructions per wave per stage
  static constexpr int IX = BM / 16 / NW;          // X DMA wave-instructions per wave per stage
  static constexpr int LDS_BYTES = S * STAGE_BYTES;
  static_assert(BN % (16 * NW) == 0 && BM % (16 * NW) == 0, "row groups must split evenly over waves");
  static_assert(S >= 3, "need at least two stages in flight");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS is 160 KB per CU");
};

template <int WN, int WM, int TN, int TM, int S, int WAUX>
__global__ __launch_bounds__(64 * WN * WM) void gemm_stream_kernel(const bf16_t* __restrict__ X,
                                                                   const bf16_t* __restrict__ W,
                                                                   bf16_t* __restrict__ Y, float* __restrict__ P,
                                                                   int M, int N, int K, int kps) {
  using C = StreamCfg<WN, WM, TN, TM, S>;
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  char* lbase = reinterpret_cast<char*>(lds);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int n0 = blockIdx.x * C::BN, m0 = blockIdx.y * C::BM;
  const int kb = blockIdx.z * kps;
  const int nk = min(kps, K - kb) / 32;

  // DMA sources: instruction i of this wave covers LDS rows g*16 .. g*16+15 (g = i*NW + wave);
  // lane -> (row g*16 + lane/4, slot lane%4) holds global chunk sw4(row, slot)
  const bf16_t* wsrc[C::IW];
  const bf16_t* xsrc[C::IX];
  int wdst[C::IW], xdst[C::IX];
#pragma unroll
  for (int i = 0; i < C::IW; ++i) {
    const int g = i * C::NW + wave, row = g * 16 + (lane >> 2);
    wsrc[i] = W + (size_t)min(n0 + row, N - 1) * K + kb + sw4(row, lane & 3) * 8;
    wdst[i] = g * 1024;
  }
#pragma unroll
  for (int i = 0; i < C::IX; ++i) {
    const int g = i * C::NW + wave, row = g * 16 + (lane >> 2);     // X row index within the tile
    xsrc[i] = X + (size_t)min(m0 + row, M - 1) * K + kb + sw4(C::BN + row, lane & 3) * 8;
    xdst[i] = (C::BN / 16 + g) * 1024;
  }

  // (the source goes in as a non-const void*: handed a const pointer, hipcc's host pass (ROCm 7.2)
  // silently drops the kernel's launch stub and the library fails to load)
#define KA_STREAM_ISSUE(t, slot)                                                                   \
  {                                                                                                \
    const int ko_ = min((t), nk - 1) * 32;                                                         \
    char* sb_ = lbase + (slot) * C::STAGE_BYTES;                                                   \
    _Pragma("unroll") for (int i = 0; i < C::IW; ++i)                                              \
      __builtin_amdgcn_global_load_lds((void*)(wsrc[i] + ko_), (lds_ptr_t)(sb_ + wdst[i]), 16, 0, WAUX);    \
    _Pragma("unroll") for (int i = 0; i < C::IX; ++i)                                              \
      __builtin_amdgcn_global_load_lds((void*)(xsrc[i] + ko_), (lds_ptr_t)(sb_ + xdst[i]), 16, 0, 0);       \
  }

  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, grp = lane >> 4;
  // per-lane LDS byte offsets of the fragments (slot-independent)
  int aoff[TN], boff[TM];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int row = wn * TN * 16 + i * 16 + r16;
    aoff[i] = row * 64 + sw4(row, grp) * 16;
  }
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int row = C::BN + wm * TM * 16 + j * 16 + r16;
    boff[j] = row * 64 + sw4(row, grp) * 16;
  }

  if (nk > 0) {
#pragma unroll
    for (int s = 0; s < S - 1; ++s) KA_STREAM_ISSUE(s, s);
    int cslot = 0, islot = S - 1;
    for (int t = 0; t < nk; ++t) {
      vm_wait<(S - 2) * (C::IW + C::IX)>();
      lds_barrier();
      KA_STREAM_ISSUE(t + S - 1, islot);
      const char* sb = lbase + cslot * C::STAGE_BYTES;
      bf16x8 a[TN], b[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) a[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(sb + aoff[i]));
#pragma unroll
      for (int j = 0; j < TM; ++j) b[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(sb + boff[j]));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      cslot = cslot == S - 1 ? 0 : cslot + 1;
      islot = islot == S - 1 ? 0 : islot + 1;
    }
    vm_wait<0>();   // no LDS-DMA may land after the workgroup retires
  }

#undef KA_STREAM_ISSUE

  // epilogue: acc[i][j][r] = C[n = .. + 4*grp + r][m = .. + r16]  ->  Y[m][n .. n+3]
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + wn * TN * 16 + i * 16 + 4 * grp;
    if (n >= N) continue;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * TM * 16 + j * 16 + r16;
      if (m >= M) continue;
      const f32x4 v = acc[i][j];
      if (P == nullptr) {
        *reinterpret_cast<uint2*>(Y + (size_t)m * N + n) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      } else {
        *reinterpret_cast<f32x4*>(P + ((size_t)blockIdx.z * M + m) * N + n) = v;
      }
    }
  }
}

template <int WN, int WM, int TN, int TM, int S, int WAUX>
static void launch_stream(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int split,
                          int kps, hipStream_t stream) {
  using C = StreamCfg<WN, WM, TN, TM, S>;
  static bool lds_attr = false;   // > 64 KB of dynamic LDS must be opted into
  if (!lds_attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_stream_kernel<WN, WM, TN, TM, S, WAUX>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS_BYTES);
    lds_attr = true;
  }
  dim3 grid((N + C::BN - 1) / C::BN, (M + C::BM - 1) / C::BM, split);
  hipLaunchKernelGGL((gemm_stream_kernel<WN, WM, TN, TM, S, WAUX>), grid, dim3(C::NT), C::LDS_BYTES, stream, X, W,
                     Y, P, M, N, K, kps);
}

// Stream configurations (index = cfg - 10 of ka_gemm_tile):
//   10: 128 x 256 (BN x BM), 8 waves (2 N x 4 M, 64x64 per wave), 6 stages, W non-temporal
//   11:  64 x 256, 4 waves (1 x 4), 7 stages
//   12: 128 x 128, 4 waves (2 x 2), 8 stages
//   13: 256 x 256, 8 waves (4 x 2, 64x128 per wave), 4 stages
//   14: cfg 10 with W loaded through the default cache policy
#define KA_STREAM_CFGS(X)              \
  X(10, 2, 4, 4, 4, 6, 2)              \
  X(11, 1, 4, 4, 4, 7, 2)              \
  X(12, 2, 2, 4, 4, 8, 2)              \
  X(13, 4, 2, 4, 8, 4, 2)              \
  X(14, 2, 4, 4, 4, 6, 0)

extern "C" int ka_gemm_stream_bm(int cfg) {
#define X_(id, wn, wm, tn, tm, s, aux) \
  if (cfg == id) return StreamCfg<wn, wm, tn, tm, s>::BM;
  KA_STREAM_CFGS(X_)
#undef X_
  return -1;
}

extern "C" int ka_gemm_stream_bn(int cfg) {
#define X_(id, wn, wm, tn, tm, s, aux) \
  if (cfg == id) return StreamCfg<wn, wm, tn, tm, s>::BN;
  KA_STREAM_CFGS(X_)
#undef X_
  return -1;
}

// Launch (called by ka_gemm_tile for cfg >= 10): kps = K per split, a multiple of 32.
extern "C" int ka_gemm_stream_launch(bf16_t* Y, const bf16_t* X, const bf16_t* W, float* P, int M, int N, int K,
                                     int split, int kps, int cfg, hipStream_t stream) {
#define X_(id, wn, wm, tn, tm, s, aux)                                                 \
  if (cfg == id) {                                                                     \
    launch_stream<wn, wm, tn, tm, s, aux>(X, W, Y, P, M, N, K, split, kps, stream);    \
    return 0;                                                                          \
  }
  KA_STREAM_CFGS(X_)
#undef X_
  return (int)hipErrorInvalidValue;
}
