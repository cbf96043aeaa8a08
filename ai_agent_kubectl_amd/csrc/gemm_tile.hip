// LDS-tiled MFMA GEMM for the moderate-M projections (decode batches 64..512, mixed steps):
//   Y[M, N] = X[M, K] * W[N, K]^T, bf16 in/out, fp32 accumulate.
//
// Why not hipBLASLt: with every layer's weights streaming cold from HBM, its best M = 256 solutions
// run the Llama-3-8B projections at ~0.3-0.8 PFLOP/s (QKV 30 us, O 24, gate_up 71, down 66 per layer,
// TunableOp with a 1 GB rotating buffer) while the shape is balanced between the 8 TB/s and MFMA
// roofs (~90-100 us per layer).  Design (guide §5, T2, T14):
//   * workgroup tile BN (weight rows) x BM (activation rows), waves laid out WN x WM, each wave
//     TN x TM MFMA 16x16x32 tiles; W is the MFMA A operand and X the B operand, so a lane's four
//     accumulator values are four consecutive output columns (8-B bf16 / 16-B fp32 stores);
//   * both operands are K-contiguous: one 64-k step of each tile is staged global -> VGPR -> LDS
//     with 16-B loads/stores, XOR-swizzled (slot = chunk ^ ((row >> 1) & 7)) so the 16 rows a
//     ds_read_b128 group touches land on 16 distinct 16-B segments of the 256-B bank row;
//   * issue-early / write-late register staging with two LDS buffers and one barrier per k-step:
//     the next step's global loads are in flight during this step's MFMAs and are written to the
//     other buffer afterwards (plain loads survive __syncthreads; no LDS-DMA in flight);
//   * split-K over gridDim.z writes fp32 partials P[z][M][N], summed by splitk_reduce_kernel
//     (gemm_skinny.hip); split == 1 stores bf16 directly.
#include "common.h"

__device__ __forceinline__ int sw_slot(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int WN, int WM, int TN, int TM>
struct TileCfg {
  static constexpr int BN = WN * TN * 16;
  static constexpr int BM = WM * TM * 16;
  static constexpr int NT = 64 * WN * WM;
  static constexpr int WP = BN * 8 / NT;  // 16-B pieces of the W tile per thread per k-step
  static constexpr int XP = BM * 8 / NT;
  static constexpr int LDS_BYTES = 2 * (BN + BM) * 128;
  static_assert(BN * 8 % NT == 0 && BM * 8 % NT == 0, "tile pieces must divide the thread count");
};

// SWIGLU: X is the fused gate_up output GU [M, 2K] and the activation is computed while staging
// (swiglu8, common.h) — the down projection consumes the gate_up output directly.

// PF2: two register stages in flight (k-step t+2 is issued before computing t, t+1 is written to
// LDS after it): hides about two loaded-HBM latencies instead of one; K per split must then be a
// multiple of 128 (the loop is unrolled by two so hipcc counts vmcnt statically; loads past the
// end are clamped to the last step and land in a buffer nobody reads again).
// pbf16: the split-K slices P are stored as bf16 (half the slab traffic; the consumer — RMSNorm or
// the fused decode attention — sums them in fp32, like a bf16 tensor-parallel all-reduce would).
template <int WN, int WM, int TN, int TM, bool SWIGLU = false, bool PF2 = false>
__global__ __launch_bounds__(64 * WN * WM) void gemm_tile_kernel(const bf16_t* __restrict__ X,
                                                                 const bf16_t* __restrict__ W,
                                                                 bf16_t* __restrict__ Y, float* __restrict__ P, int M,
                                                                 int N, int K, int kps, int pbf16) {
  using C = TileCfg<WN, WM, TN, TM>;
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];   // [2][BN*8] W then [2][BM*8] X
  u32x4* ws = lds;
  u32x4* xs = lds + 2 * C::BN * 8;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WN, wm = wave / WN;
  const int n0 = blockIdx.x * C::BN, m0 = blockIdx.y * C::BM;
  const int kb = blockIdx.z * kps;
  const int nk = min(kps, K - kb) / 64;

  // per-thread global source rows (clamped: out-of-range rows load a valid row, stores are skipped)
  const bf16_t* wsrc[C::WP];
  const bf16_t* xsrc[C::XP];
  int wdst[C::WP], xdst[C::XP];
#pragma unroll
  for (int i = 0; i < C::WP; ++i) {
    const int p = tid + i * C::NT, row = p >> 3, ch = p & 7;
    wsrc[i] = W + (size_t)min(n0 + row, N - 1) * K + kb + ch * 8;
    wdst[i] = row * 8 + sw_slot(row, ch);
  }
  const size_t ldx = SWIGLU ? 2 * (size_t)K : (size_t)K;
#pragma unroll
  for (int i = 0; i < C::XP; ++i) {
    const int p = tid + i * C::NT, row = p >> 3, ch = p & 7;
    xsrc[i] = X + (size_t)min(m0 + row, M - 1) * ldx + kb + ch * 8;
    xdst[i] = row * 8 + sw_slot(row, ch);
  }

  u32x4 wr[C::WP], xr[C::XP];
  auto load = [&](int t) {
#pragma unroll
    for (int i = 0; i < C::WP; ++i) wr[i] = *reinterpret_cast<const u32x4*>(wsrc[i] + t * 64);
#pragma unroll
    for (int i = 0; i < C::XP; ++i) {
      if constexpr (SWIGLU) {
        xr[i] = swiglu8(*reinterpret_cast<const u32x4*>(xsrc[i] + t * 64),
                        *reinterpret_cast<const u32x4*>(xsrc[i] + K + t * 64));
      } else {
        xr[i] = *reinterpret_cast<const u32x4*>(xsrc[i] + t * 64);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < C::WP; ++i) ws[buf * C::BN * 8 + wdst[i]] = wr[i];
#pragma unroll
    for (int i = 0; i < C::XP; ++i) xs[buf * C::BM * 8 + xdst[i]] = xr[i];
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, grp = lane >> 4;
  auto compute = [&](int buf) {
    const u32x4* wb = ws + buf * C::BN * 8;
    const u32x4* xb = xs + buf * C::BM * 8;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + grp;
      bf16x8 a[TN], b[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int row = wn * TN * 16 + i * 16 + r16;
        a[i] = __builtin_bit_cast(bf16x8, wb[row * 8 + sw_slot(row, ch)]);
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int row = wm * TM * 16 + j * 16 + r16;
        b[j] = __builtin_bit_cast(bf16x8, xb[row * 8 + sw_slot(row, ch)]);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (PF2) {
    static_assert(!SWIGLU, "PF2 variant is plain X staging only");
    u32x4 wr2[C::WP], xr2[C::XP];
    auto load2 = [&](u32x4 (&w)[C::WP], u32x4 (&x)[C::XP], int t) {
      t = min(t, nk - 1);
#pragma unroll
      for (int i = 0; i < C::WP; ++i) w[i] = *reinterpret_cast<const u32x4*>(wsrc[i] + t * 64);
#pragma unroll
      for (int i = 0; i < C::XP; ++i) x[i] = *reinterpret_cast<const u32x4*>(xsrc[i] + t * 64);
    };
    auto store2 = [&](const u32x4 (&w)[C::WP], const u32x4 (&x)[C::XP], int buf) {
#pragma unroll
      for (int i = 0; i < C::WP; ++i) ws[buf * C::BN * 8 + wdst[i]] = w[i];
#pragma unroll
      for (int i = 0; i < C::XP; ++i) xs[buf * C::BM * 8 + xdst[i]] = x[i];
    };
    if (nk > 0) {
      load2(wr, xr, 0);
      load2(wr2, xr2, 1);
      store2(wr, xr, 0);
    }
    __syncthreads();
    for (int t = 0; t < nk; t += 2) {   // nk is even
      load2(wr, xr, t + 2);
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch above the MFMAs (hipcc sinks it otherwise)
      compute(0);
      store2(wr2, xr2, 1);
      __syncthreads();
      load2(wr2, xr2, t + 3);
      __builtin_amdgcn_sched_barrier(0);
      compute(1);
      store2(wr, xr, 0);
      __syncthreads();
    }
  } else {
    if (nk > 0) {
      load(0);
      store(0);
    }
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      const int buf = t & 1;
      if (t + 1 < nk) load(t + 1);
      compute(buf);
      if (t + 1 < nk) store(buf ^ 1);
      __syncthreads();
    }
  }

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
      } else if (pbf16) {
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(P) + ((size_t)blockIdx.z * M + m) * N + n) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      } else {
        *reinterpret_cast<f32x4*>(P + ((size_t)blockIdx.z * M + m) * N + n) = v;
      }
    }
  }
}


// ------------------------------------------------------------------------------------------------
// "Wide" variant for decode M (<= 256 per tile row): W never touches LDS.  Each wave owns TN*16
// weight rows and streams its MFMA A fragments global -> VGPR (16-B loads, a two-step register
// ring: step t+2 is issued right after step t's MFMAs), while the BM = TM*16 activation rows are
// staged once per k-step in LDS and shared by all waves.  LDS bytes read per MFMA = 1024 / TN
// (256 B at TN = 4, half of a 64x64-per-wave tile), so the loop is bound by the W stream, which is
// what a decode GEMM should be bound by.  blockIdx.x walks the M tiles so the tiles that share a
// weight panel are dispatched back to back (the second read hits the MALL).  K per split must be a
// multiple of 128 (the k loop is unrolled by two steps with unconditional, clamped loads so hipcc
// can count vmcnt statically — guide §5 item 4c).
template <int NWV, int TN, int TM>
struct WideCfg {
  static constexpr int BN = NWV * TN * 16;
  static constexpr int BM = TM * 16;
  static constexpr int NT = 64 * NWV;
  static constexpr int XP = BM * 8 / NT;
  static constexpr int LDS_BYTES = 2 * BM * 128;
  static_assert(BM * 8 % NT == 0, "X tile pieces must divide the thread count");
};

template <int NWV, int TN, int TM>
__global__ __launch_bounds__(64 * NWV) void gemm_wide_kernel(const bf16_t* __restrict__ X,
                                                             const bf16_t* __restrict__ W,
                                                             bf16_t* __restrict__ Y, float* __restrict__ P, int M,
                                                             int N, int K, int kps) {
  using C = WideCfg<NWV, TN, TM>;
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];   // [2][BM*8] X
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, grp = lane >> 4;
  const int m0 = blockIdx.x * C::BM, n0 = blockIdx.y * C::BN;
  const int kb = blockIdx.z * kps;
  const int nk = min(kps, K - kb) / 64;   // even (host guarantees kps % 128 == 0, K % 128 == 0)

  const bf16_t* wp[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i)
    wp[i] = W + (size_t)min(n0 + wave * TN * 16 + i * 16 + r16, N - 1) * K + kb + grp * 8;
  const bf16_t* xsrc[C::XP];
  int xdst[C::XP];
#pragma unroll
  for (int i = 0; i < C::XP; ++i) {
    const int p = tid + i * C::NT, row = p >> 3, ch = p & 7;
    xsrc[i] = X + (size_t)min(m0 + row, M - 1) * K + kb + ch * 8;
    xdst[i] = row * 8 + sw_slot(row, ch);
  }

  u32x4 wa[TN][2], wb[TN][2], xr[C::XP];
  auto load_w = [&](u32x4 (&w)[TN][2], int t) {
    t = min(t, nk - 1);
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      w[i][0] = *reinterpret_cast<const u32x4*>(wp[i] + t * 64);
      w[i][1] = *reinterpret_cast<const u32x4*>(wp[i] + t * 64 + 32);
    }
  };
  auto load_x = [&](int t) {
    t = min(t, nk - 1);
#pragma unroll
    for (int i = 0; i < C::XP; ++i) xr[i] = *reinterpret_cast<const u32x4*>(xsrc[i] + t * 64);
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < C::XP; ++i) lds[buf * C::BM * 8 + xdst[i]] = xr[i];
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const u32x4 (&w)[TN][2], int buf) {
    const u32x4* xb = lds + buf * C::BM * 8;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + grp;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int row = j * 16 + r16;
        const bf16x8 b = __builtin_bit_cast(bf16x8, xb[row * 8 + sw_slot(row, ch)]);
#pragma unroll
        for (int i = 0; i < TN; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w[i][kk]), b, acc[i][j],
                                                              0, 0, 0);
      }
    }
  };

  if (nk > 0) {
    load_w(wa, 0);
    load_w(wb, 1);
    load_x(0);
    store_x(0);
  }
  __syncthreads();
  for (int t = 0; t < nk; t += 2) {
    load_x(t + 1);
    __builtin_amdgcn_sched_barrier(0);   // keep the prefetch above the MFMAs (hipcc sinks it otherwise)
    compute(wa, 0);
    load_w(wa, t + 2);
    store_x(1);
    __syncthreads();
    load_x(t + 2);
    __builtin_amdgcn_sched_barrier(0);
    compute(wb, 1);
    load_w(wb, t + 3);
    store_x(0);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + wave * TN * 16 + i * 16 + 4 * grp;
    if (n >= N) continue;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + j * 16 + r16;
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

template <int NWV, int TN, int TM>
static void launch_wide(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int split,
                        int kps, hipStream_t stream) {
  using C = WideCfg<NWV, TN, TM>;
  dim3 grid((M + C::BM - 1) / C::BM, (N + C::BN - 1) / C::BN, split);
  hipLaunchKernelGGL((gemm_wide_kernel<NWV, TN, TM>), grid, dim3(C::NT), C::LDS_BYTES, stream, X, W, Y, P, M, N, K,
                     kps);
}

extern "C" void ka_splitk_reduce_launch(bf16_t* Y, const float* P, int split, long mn, hipStream_t stream);

template <int WN, int WM, int TN, int TM, bool SW = false, bool PF2 = false>
static void launch_tile(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int split,
                        int kps, hipStream_t stream, int pbf16 = 0) {
  using C = TileCfg<WN, WM, TN, TM>;
  static bool lds_attr = false;   // > 64 KB of dynamic LDS must be opted into (160 KB per CU on gfx950)
  if (!lds_attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tile_kernel<WN, WM, TN, TM, SW, PF2>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS_BYTES);
    lds_attr = true;
  }
  dim3 grid((N + C::BN - 1) / C::BN, (M + C::BM - 1) / C::BM, split);
  hipLaunchKernelGGL((gemm_tile_kernel<WN, WM, TN, TM, SW, PF2>), grid, dim3(C::NT), C::LDS_BYTES, stream, X, W, Y, P, M,
                     N, K, kps, pbf16);
}

// Configurations (BN x BM, waves): 0 = 128x256 (2x4 waves, 64x64 per wave), 1 = 64x256 (1x4),
// 2 = 128x128 (2x2), 3 = 128x256 (2x2 waves, 64x128 per wave), 4 = 256x128 (4x2);
// wide (W in VGPRs): 5 = 256x128 (4 waves x 64 rows), 6 = 128x128 (2 waves), 7 = 128x64 (2 waves),
// 8 = 64x128 (1 wave x 64 rows), 9 = 128x128 (4 waves x 32 rows).
extern "C" int ka_gemm_stream_bm(int cfg);
extern "C" int ka_gemm_stream_bn(int cfg);
extern "C" int ka_gemm_stream_launch(bf16_t* Y, const bf16_t* X, const bf16_t* W, float* P, int M, int N, int K,
                                     int split, int kps, int cfg, hipStream_t stream);

// PF2 (two register stages in flight): 17 = 128x128 (2x2 waves), 18 = 128x256 (2x2, 64x128 per
// wave), 19 = 128x256 (2x4 waves), 20 = 256x128 (4x2 waves).
#define KA_PF2_CFGS(X) X(17, 2, 2, 4, 4) X(18, 2, 2, 4, 8) X(19, 2, 4, 4, 4) X(20, 4, 2, 4, 4)

extern "C" int ka_gemm_tile_bm(int cfg) {
#define X_(id, a, b, c, d) if (cfg == id) return TileCfg<a, b, c, d>::BM;
  KA_PF2_CFGS(X_)
#undef X_
  if (cfg == 15) return TileCfg<4, 2, 4, 8>::BM;
  if (cfg == 16) return TileCfg<2, 4, 8, 4>::BM;
  if (cfg >= 10) return ka_gemm_stream_bm(cfg);
  switch (cfg) {
    case 0: return TileCfg<2, 4, 4, 4>::BM;
    case 1: return TileCfg<1, 4, 4, 4>::BM;
    case 2: return TileCfg<2, 2, 4, 4>::BM;
    case 3: return TileCfg<2, 2, 4, 8>::BM;
    case 4: return TileCfg<4, 2, 4, 4>::BM;
    case 5: return WideCfg<4, 4, 8>::BM;
    case 6: return WideCfg<2, 4, 8>::BM;
    case 7: return WideCfg<2, 4, 4>::BM;
    case 8: return WideCfg<1, 4, 8>::BM;
    case 9: return WideCfg<4, 2, 8>::BM;
    default: return -1;
  }
}

extern "C" int ka_gemm_tile_bn(int cfg) {
#define X_(id, a, b, c, d) if (cfg == id) return TileCfg<a, b, c, d>::BN;
  KA_PF2_CFGS(X_)
#undef X_
  if (cfg == 15) return TileCfg<4, 2, 4, 8>::BN;
  if (cfg == 16) return TileCfg<2, 4, 8, 4>::BN;
  if (cfg >= 10) return ka_gemm_stream_bn(cfg);
  switch (cfg) {
    case 0: return TileCfg<2, 4, 4, 4>::BN;
    case 1: return TileCfg<1, 4, 4, 4>::BN;
    case 2: return TileCfg<2, 2, 4, 4>::BN;
    case 3: return TileCfg<2, 2, 4, 8>::BN;
    case 4: return TileCfg<4, 2, 4, 4>::BN;
    case 5: return WideCfg<4, 4, 8>::BN;
    case 6: return WideCfg<2, 4, 8>::BN;
    case 7: return WideCfg<2, 4, 4>::BN;
    case 8: return WideCfg<1, 4, 8>::BN;
    case 9: return WideCfg<4, 2, 8>::BN;
    default: return -1;
  }
}

// split > 1 requires a workspace of split * M * N floats (the reduce kernel then writes Y).
// p_bf16 (Y == nullptr, LDS-tiled configurations 0-4 and 15-20 only): the slices are bf16.
extern "C" int ka_gemm_tile(void* Y, const void* X, const void* W, void* workspace, int M, int N, int K, int split,
                            int cfg, int p_bf16, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 32 != 0 || N % 16 != 0 || split < 1 || cfg < 0 || ka_gemm_tile_bm(cfg) < 0) return (int)hipErrorInvalidValue;
  if (p_bf16 && (Y != nullptr || (cfg >= 5 && cfg < 15))) return (int)hipErrorInvalidValue;
  // k quantum: stream kernels (cfg >= 10) 32-deep stages, wide kernels pairs of 64-steps, tile 64
  const int kq = cfg >= 17 ? 128 : cfg >= 15 ? 64 : cfg >= 10 ? 32 : cfg >= 5 ? 128 : 64;
  if (K % kq != 0) return (int)hipErrorInvalidValue;
  int kps = (K / split + kq - 1) / kq * kq;
  split = (K + kps - 1) / kps;
  auto* x = static_cast<const bf16_t*>(X);
  auto* w = static_cast<const bf16_t*>(W);
  auto* y = static_cast<bf16_t*>(Y);
  float* p = split > 1 ? static_cast<float*>(workspace) : nullptr;
  const int pb = split > 1 ? p_bf16 : 0;
#define X_(id, a, b, c, d) \
  if (cfg == id) launch_tile<a, b, c, d, false, true>(x, w, y, p, M, N, K, split, kps, stream, pb);
  KA_PF2_CFGS(X_)
#undef X_
  if (cfg == 15) launch_tile<4, 2, 4, 8>(x, w, y, p, M, N, K, split, kps, stream, pb);
  if (cfg == 16) launch_tile<2, 4, 8, 4>(x, w, y, p, M, N, K, split, kps, stream, pb);
  if (cfg >= 10 && cfg < 15) {
    const int rc = ka_gemm_stream_launch(y, x, w, p, M, N, K, split, kps, cfg, stream);
    if (rc) return rc;
  }
  switch (cfg) {
    case 0: launch_tile<2, 4, 4, 4>(x, w, y, p, M, N, K, split, kps, stream, pb); break;
    case 1: launch_tile<1, 4, 4, 4>(x, w, y, p, M, N, K, split, kps, stream, pb); break;
    case 2: launch_tile<2, 2, 4, 4>(x, w, y, p, M, N, K, split, kps, stream, pb); break;
    case 3: launch_tile<2, 2, 4, 8>(x, w, y, p, M, N, K, split, kps, stream, pb); break;
    case 4: launch_tile<4, 2, 4, 4>(x, w, y, p, M, N, K, split, kps, stream, pb); break;
    case 5: launch_wide<4, 4, 8>(x, w, y, p, M, N, K, split, kps, stream); break;
    case 6: launch_wide<2, 4, 8>(x, w, y, p, M, N, K, split, kps, stream); break;
    case 7: launch_wide<2, 4, 4>(x, w, y, p, M, N, K, split, kps, stream); break;
    case 8: launch_wide<1, 4, 8>(x, w, y, p, M, N, K, split, kps, stream); break;
    case 9: launch_wide<4, 2, 8>(x, w, y, p, M, N, K, split, kps, stream); break;
  }
  // Y == nullptr: leave the fp32 partials for a fused consumer (ka_rmsnorm_splitk)
  if (split > 1 && y != nullptr) ka_splitk_reduce_launch(y, p, split, (long)M * N, stream);
  KA_CHECK_LAUNCH();
}

// Y = swiglu(GU) * W^T with GU = [M, 2K] (gate | up); cfg 0-4 (the LDS-tiled variants).
extern "C" int ka_gemm_tile_swiglu(void* Y, const void* GU, const void* W, void* workspace, int M, int N, int K,
                                   int split, int cfg, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 64 != 0 || N % 16 != 0 || split < 1 || cfg < 0 || cfg > 4) return (int)hipErrorInvalidValue;
  int kps = (K / split + 63) / 64 * 64;
  split = (K + kps - 1) / kps;
  auto* x = static_cast<const bf16_t*>(GU);
  auto* w = static_cast<const bf16_t*>(W);
  auto* y = static_cast<bf16_t*>(Y);
  float* p = split > 1 ? static_cast<float*>(workspace) : nullptr;
  switch (cfg) {
    case 0: launch_tile<2, 4, 4, 4, true>(x, w, y, p, M, N, K, split, kps, stream); break;
    case 1: launch_tile<1, 4, 4, 4, true>(x, w, y, p, M, N, K, split, kps, stream); break;
    case 2: launch_tile<2, 2, 4, 4, true>(x, w, y, p, M, N, K, split, kps, stream); break;
    case 3: launch_tile<2, 2, 4, 8, true>(x, w, y, p, M, N, K, split, kps, stream); break;
    case 4: launch_tile<4, 2, 4, 4, true>(x, w, y, p, M, N, K, split, kps, stream); break;
  }
  if (split > 1 && y != nullptr) ka_splitk_reduce_launch(y, p, split, (long)M * N, stream);
  KA_CHECK_LAUNCH();
}
