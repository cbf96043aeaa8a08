// Weight-streaming MFMA GEMM for decode (K13):  Y[M, N] = X[M, K] * W[N, K]^T,  M <= 256, bf16.
//
// In a decode step every weight byte is read exactly once, so the projections are HBM-bound on W
// (Llama-3-8B: 16 GB per step); hipBLASLt's tiles for M <= 256 leave most CUs idle on N = 4096
// (128 workgroups, K = 14336 streamed by each: 1.4-2 TB/s measured).  This kernel:
//   * workgroup = 4 waves = 64 output columns (one 16-column MFMA tile per wave) x all M rows,
//     over one K slice (split-K so that the grid covers the 256 CUs several times);
//   * W is the MFMA A operand: lane l's fragment (row n = l&15, k = 8*(l>>4)..+7) is one contiguous
//     16-B global load straight into VGPRs (no reuse across waves -> no LDS round trip), with a
//     two-chunk-deep register ring (two named sets, ping-pong) so 4 KiB per wave stay in flight;
//   * X (re-read by every column tile, L2/MALL-resident) is the B operand, staged per 64-k chunk
//     in LDS by all 256 threads with an XOR swizzle (slot = chunk ^ (row & 7)) against the
//     16-rows-same-column ds_read_b128 conflict (guide §5.5 T2), register-staged one chunk ahead;
//   * C = 16 n x 16 m per MFMA: each lane owns 4 consecutive n of one m -> 8-B bf16 / 16-B fp32
//     stores.  split == 1 writes bf16 Y; split > 1 writes fp32 partials P[split][M][N] that
//     `ka_splitk_reduce` (or a fused consumer) sums.
#include "common.h"

#define NW 64  // output columns per workgroup

// X staging: piece p -> row p >> 3, 16-B chunk p & 7 of a 64-k chunk; LDS slot = chunk ^ (row & 7)
template <int MT>
__device__ __forceinline__ void sk_load_x(u32x4 (&xr)[(MT * 128 + 255) / 256], const bf16_t* __restrict__ X, int M,
                                          int K, int k_begin, int c, int tid) {
  constexpr int PIECES = MT * 128;
#pragma unroll
  for (int i = 0; i < (PIECES + 255) / 256; ++i) {
    const int p = tid + 256 * i;
    if (PIECES % 256 == 0 || p < PIECES) {
      const int row = min(p >> 3, M - 1);
      xr[i] = *reinterpret_cast<const u32x4*>(X + (size_t)row * K + k_begin + c * 64 + (p & 7) * 8);
    }
  }
}

template <int MT>
__device__ __forceinline__ void sk_store_x(const u32x4 (&xr)[(MT * 128 + 255) / 256], uint4* xs, int tid) {
  constexpr int PIECES = MT * 128;
#pragma unroll
  for (int i = 0; i < (PIECES + 255) / 256; ++i) {
    const int p = tid + 256 * i;
    if (PIECES % 256 == 0 || p < PIECES)
      reinterpret_cast<u32x4*>(xs)[(p >> 3) * 8 + ((p & 7) ^ ((p >> 3) & 7))] = xr[i];
  }
}

__device__ __forceinline__ void sk_load_w(uint4& w0, uint4& w1, const bf16_t* __restrict__ wp, int c, int nchunks) {
  c = min(c, nchunks - 1);
  w0 = *reinterpret_cast<const uint4*>(wp + c * 64);
  w1 = *reinterpret_cast<const uint4*>(wp + c * 64 + 32);
}

template <int MT>
__device__ __forceinline__ void sk_compute(f32x4 (&acc)[MT], const uint4& w0, const uint4& w1, const uint4* xs,
                                           int col, int grp) {
  const bf16x8 a0 = as_bf16x8(w0), a1 = as_bf16x8(w1);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = mt * 16 + col;
    acc[mt] = mfma16x16x32(a0, as_bf16x8(xs[row * 8 + (grp ^ (row & 7))]), acc[mt]);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = mt * 16 + col;
    acc[mt] = mfma16x16x32(a1, as_bf16x8(xs[row * 8 + ((4 + grp) ^ (row & 7))]), acc[mt]);
  }
}

template <int MT>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                          bf16_t* __restrict__ Y, float* __restrict__ P, int M,
                                                          int N, int K, int kps) {
  constexpr int ROWS = MT * 16;
  constexpr int XR = (MT * 128 + 255) / 256;        // 16-B X pieces per thread per 64-k chunk
  __shared__ __attribute__((aligned(16))) uint4 xs[ROWS * 8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int n0 = blockIdx.x * NW;
  const int split = blockIdx.y;
  const int k_begin = split * kps;
  const int k_end = min(K, k_begin + kps);
  const int nchunks = (k_end - k_begin) >> 6;

  // W row this lane streams (clamped; out-of-range columns are computed but never stored)
  const int wn = min(n0 + wave * 16 + col, N - 1);
  const bf16_t* wp = W + (size_t)wn * K + k_begin + 8 * grp;

  u32x4 xr[XR];
  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 wa0 = make_uint4(0, 0, 0, 0), wa1 = wa0, wb0 = wa0, wb1 = wa0;  // two register sets
  if (nchunks > 0) {
    sk_load_w(wa0, wa1, wp, 0, nchunks);
    sk_load_w(wb0, wb1, wp, 1, nchunks);
    sk_load_x<MT>(xr, X, M, K, k_begin, 0, tid);
    sk_store_x<MT>(xr, xs, tid);
    __syncthreads();
    int c = 0;
    for (; c + 1 < nchunks; c += 2) {
      sk_load_x<MT>(xr, X, M, K, k_begin, c + 1, tid);   // chunk c with set A
      sk_compute<MT>(acc, wa0, wa1, xs, col, grp);
      sk_load_w(wa0, wa1, wp, c + 2, nchunks);
      __syncthreads();
      sk_store_x<MT>(xr, xs, tid);
      __syncthreads();
      // chunk c + 1 with set B; loads past the end are clamped to the last chunk (harmless
      // re-reads) so that no staging register is written under a branch (keeps xr in VGPRs)
      sk_load_x<MT>(xr, X, M, K, k_begin, min(c + 2, nchunks - 1), tid);
      sk_compute<MT>(acc, wb0, wb1, xs, col, grp);
      sk_load_w(wb0, wb1, wp, c + 3, nchunks);
      __syncthreads();
      sk_store_x<MT>(xr, xs, tid);
      __syncthreads();
    }
    if (c < nchunks) sk_compute<MT>(acc, wa0, wa1, xs, col, grp);  // odd tail (its X is in LDS)
  }

  // epilogue: lane holds n = n0 + wave*16 + 4*grp + r (r = 0..3) for m = mt*16 + col
  const int nb = n0 + wave * 16 + 4 * grp;
  if (nb >= N) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + col;
    if (m >= M) continue;
    if (P) {
      float* dst = P + ((size_t)split * M + m) * N + nb;
      if (nb + 3 < N) {
        *reinterpret_cast<float4*>(dst) = make_float4(acc[mt][0], acc[mt][1], acc[mt][2], acc[mt][3]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (nb + r < N) dst[r] = acc[mt][r];
      }
    } else {
      bf16_t* dst = Y + (size_t)m * N + nb;
      if (nb + 3 < N) {
        *reinterpret_cast<uint2*>(dst) = make_uint2(pack2(acc[mt][0], acc[mt][1]), pack2(acc[mt][2], acc[mt][3]));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (nb + r < N) dst[r] = f2bf(acc[mt][r]);
      }
    }
  }
}

// M <= GEMV_MAX_M ("GEMV") variant.  With one MFMA row tile the X operand is tiny, so instead of
// re-staging it through LDS every 64-k chunk (two barriers per chunk, an L2 round trip exposed per
// chunk) the workgroup stages its whole K slice of X once (M rows x kps, 16-B pieces XOR-swizzled by
// row) and the k loop only streams W: RING chunks per wave in flight in a register ring, no
// barriers (guide §5 table, 'GEMV / M <= 16' row: straight to VGPRs, deep unroll, late vmcnt).  The
// ring's first loads are issued before the X staging so their HBM latency overlaps it.  Loads past
// the slice end are clamped to its last chunk (L2 re-reads) so every wait count stays static.
// SWIGLU: X is the gate_up output GU [M, 2K] and the staged operand is swiglu8(gate, up) — the
// down projection of a batch-1..4 decode step without the SiLU kernel (bit-identical result).
template <int RING, bool SWIGLU = false>
__global__ __launch_bounds__(256) void gemv_ring_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                        bf16_t* __restrict__ Y, float* __restrict__ P, int M, int N,
                                                        int K, int kps) {
  extern __shared__ __attribute__((aligned(16))) uint4 xsd[];   // [M][klen / 8] pieces
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int n0 = blockIdx.x * NW;
  const int split = blockIdx.y;
  const int k_begin = split * kps;
  const int klen = min(K, k_begin + kps) - k_begin;
  const int nchunks = klen >> 6;
  const int pr = klen >> 3;

  const int wn = min(n0 + wave * 16 + col, N - 1);
  const bf16_t* wp = W + (size_t)wn * K + k_begin + 8 * grp;
  uint4 w[RING][2];
#pragma unroll
  for (int r = 0; r < RING; ++r) {
    const int c = min(r, nchunks - 1);
    w[r][0] = *reinterpret_cast<const uint4*>(wp + c * 64);
    w[r][1] = *reinterpret_cast<const uint4*>(wp + c * 64 + 32);
  }
  // X staged XB pieces per thread per batch, every batch's loads issued before its LDS stores (one
  // piece per iteration waited for each piece's L2 round trip: M * pr / 256 of them in sequence)
  constexpr int XB = 4;
  for (int p0 = tid; p0 < M * pr; p0 += 256 * XB) {
    u32x4 xa[XB], xb[XB];
#pragma unroll
    for (int j = 0; j < XB; ++j) {
      const int p = p0 + j * 256;
      if (p < M * pr) {
        const int row = p / pr, pc = p - row * pr;
        if constexpr (SWIGLU) {
          const bf16_t* g = X + (size_t)row * 2 * K + k_begin + pc * 8;
          xa[j] = *reinterpret_cast<const u32x4*>(g);
          xb[j] = *reinterpret_cast<const u32x4*>(g + K);
        } else {
          xa[j] = *reinterpret_cast<const u32x4*>(X + (size_t)row * K + k_begin + pc * 8);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < XB; ++j) {
      const int p = p0 + j * 256;
      if (p < M * pr) {
        const int row = p / pr, pc = p - row * pr;
        const u32x4 v = SWIGLU ? swiglu8(xa[j], xb[j]) : xa[j];
        xsd[row * pr + (pc ^ (row & 7))] = __builtin_bit_cast(uint4, v);
      }
    }
  }
  __syncthreads();

  const int xrow = min(col, M - 1);
  const uint4* xr = xsd + xrow * pr;
  const int sw = xrow & 7;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < nchunks; c0 += RING) {
#pragma unroll
    for (int r = 0; r < RING; ++r) {
      const int c = c0 + r;
      if (c < nchunks) {
        acc = mfma16x16x32(as_bf16x8(w[r][0]), as_bf16x8(xr[(c * 8 + grp) ^ sw]), acc);
        acc = mfma16x16x32(as_bf16x8(w[r][1]), as_bf16x8(xr[(c * 8 + 4 + grp) ^ sw]), acc);
      }
      const int cn = min(c + RING, nchunks - 1);
      w[r][0] = *reinterpret_cast<const uint4*>(wp + cn * 64);
      w[r][1] = *reinterpret_cast<const uint4*>(wp + cn * 64 + 32);
    }
  }

  const int nb = n0 + wave * 16 + 4 * grp;
  const int m = col;
  if (nb >= N || m >= M) return;
  if (P) {
    float* dst = P + ((size_t)split * M + m) * N + nb;
    if (nb + 3 < N) {
      *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (nb + r < N) dst[r] = acc[r];
    }
  } else {
    bf16_t* dst = Y + (size_t)m * N + nb;
    if (nb + 3 < N) {
      *reinterpret_cast<uint2*>(dst) = make_uint2(pack2(acc[0], acc[1]), pack2(acc[2], acc[3]));
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (nb + r < N) dst[r] = f2bf(acc[r]);
    }
  }
}

// KA_GEMV_RING: ring depth 4 (default) or 8, 0 disables the variant (A/B runs).  Measured on
// MI355X against the staged kernel (profiles/gemv_ring_ab.txt): ring 4 wins O / gate_up at
// M = 1..4 by 3-10 %, ring 8 is no better, and at M = 16 the staged kernel was faster (QKV 14.5
// vs 17.9 us) while the X staging loaded one piece per wait.  With the staging batched (round 6,
// profiles/r6/latency_chains/gemv_*): up to 8 rows the 70B TP = 8 rank's B = 8 step is 2.2 % faster on
// the ring variant and Llama-3-8B's B = 8 within 0.4 %; 16 rows is 1.5 % slower on the 8B.
#define GEMV_MAX_M 8
#define GEMV_SWIGLU_MAX_M 4   // ka_gemv_swiglu (ops.GEMV_SWIGLU_MAX_M)
// KA_GEMV_MAX_M: rows up to which ka_gemm_skinny takes the ring variant (default GEMV_MAX_M; <= 16, one
// MFMA row tile) — an A/B switch for the batched X staging
static int gemv_max_m() {
  static int mm = -1;
  if (mm < 0) {
    const char* e = getenv("KA_GEMV_MAX_M");
    mm = e ? atoi(e) : GEMV_MAX_M;
    if (mm < 0 || mm > 16) mm = GEMV_MAX_M;
  }
  return mm;
}
static int gemv_ring_depth() {
  static int ring = -1;
  if (ring < 0) {
    const char* e = getenv("KA_GEMV_RING");
    ring = e ? atoi(e) : 4;
    if (ring != 0 && ring != 8) ring = 4;
  }
  return ring;
}

// Y[m, n] = bf16(sum_s P[s, m, n])
__global__ __launch_bounds__(256) void splitk_reduce_kernel(bf16_t* __restrict__ Y, const float* __restrict__ P,
                                                            int split, long mn) {
  for (long i = (blockIdx.x * (long)blockDim.x + threadIdx.x) * 4; i < mn; i += (long)gridDim.x * blockDim.x * 4) {
    // slices 4 at a time, each batch issued before its first add (summed in slice order)
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k0 = 0; k0 < split; k0 += 4) {
      float4 t[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k0 + k < split) t[k] = *reinterpret_cast<const float4*>(P + (size_t)(k0 + k) * mn + i);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k0 + k < split) {
          s.x += t[k].x;
          s.y += t[k].y;
          s.z += t[k].z;
          s.w += t[k].w;
        }
      }
    }
    *reinterpret_cast<uint2*>(Y + i) = make_uint2(pack2(s.x, s.y), pack2(s.z, s.w));
  }
}

// Y[mn] = sum_k P[k][mn] in bf16 (also gemm_mfma.hip's EPI_P32 path with an output)
extern "C" void ka_splitk_reduce_launch(bf16_t* Y, const float* P, int split, long mn, hipStream_t stream) {
  long blocks = (mn / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((int)blocks), dim3(256), 0, stream, Y, P, split, mn);
}

// Row-streaming GEMV for M <= 16: each wave owns RW consecutive weight rows, i.e. one contiguous
// RW x klen block of W, and streams it 1 KB per load instruction (64 lanes x 16 B along K) through
// a RING-deep register ring; the dot products run on v_dot2c_f32_bf16 against the workgroup's
// LDS-staged X slice, and each finished row is summed across the wave (xor shuffles).  Against
// gemv_ring_kernel (16 rows x 128 B per load, MFMA with one live row) this issues HBM-friendly
// sequential streams and lets the grid be sized by rows per wave instead of 64-row tiles.
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
KA_DEV float dot8(uint4 w, uint4 x, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, w.x), __builtin_bit_cast(bf16x2v, x.x), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, w.y), __builtin_bit_cast(bf16x2v, x.y), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, w.z), __builtin_bit_cast(bf16x2v, x.z), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, w.w), __builtin_bit_cast(bf16x2v, x.w), acc, false);
  return acc;
}

template <bool NT>
KA_DEV uint4 ld_w16(const bf16_t* p) {
  if constexpr (NT) return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
  else return *reinterpret_cast<const uint4*>(p);
}

template <int MR, int RING, bool SWIGLU, bool NT = false>
__global__ __launch_bounds__(256) void gemv_rows_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                        bf16_t* __restrict__ Y, float* __restrict__ P, int M, int N,
                                                        int K, int kps, int RW) {
  extern __shared__ __attribute__((aligned(16))) uint4 xsr[];   // [MR][klen / 8]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.y;
  const int k_begin = split * kps;
  const int klen = min(K, k_begin + kps) - k_begin;
  const int KC = klen >> 9;          // 512-element chunks per row
  const int pr = klen >> 3;          // 16-B pieces per X row
  const int r0 = (blockIdx.x * 4 + wave) * RW;
  const int nrows = max(0, min(RW, N - r0));
  const int total = nrows * KC;      // loads of this wave (wave-uniform)

  // weight stream: load i covers row i / KC, chunk i % KC; past the end the pointer stays on the
  // last chunk (L2 re-reads) so the ring's wait counts stay static
  const bf16_t* lp = W + (size_t)min(r0, N - 1) * K + k_begin + lane * 8;
  int lc = 0, issued = 0;
  const int row_skip = K - klen;
  uint4 w[RING];
#pragma unroll
  for (int r = 0; r < RING; ++r) {
    w[r] = ld_w16<NT>(lp);
    if (issued + 1 < total) {
      lp += 512;
      if (++lc == KC) { lc = 0; lp += row_skip; }
    }
    ++issued;
  }
  for (int p = tid; p < MR * pr; p += 256) {
    const int m = p / pr, pc = p - m * pr;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (m < M) {
      if constexpr (SWIGLU) {
        const bf16_t* g = X + (size_t)m * 2 * K + k_begin + pc * 8;
        v = __builtin_bit_cast(uint4, swiglu8(*reinterpret_cast<const u32x4*>(g), *reinterpret_cast<const u32x4*>(g + K)));
      } else {
        v = *reinterpret_cast<const uint4*>(X + (size_t)m * K + k_begin + pc * 8);
      }
    }
    xsr[p] = v;
  }
  __syncthreads();

  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.f;
  int cc = 0, crow = r0;
  for (int base = 0; base < total; base += RING) {
#pragma unroll
    for (int r = 0; r < RING; ++r) {
      if (base + r < total) {
#pragma unroll
        for (int m = 0; m < MR; ++m) acc[m] = dot8(w[r], xsr[m * pr + cc * 64 + lane], acc[m]);
        if (++cc == KC) {
          cc = 0;
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            float v = acc[m];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            acc[m] = 0.f;
            if (lane == m && m < M) {
              if (P) P[((size_t)split * M + m) * N + crow] = v;
              else Y[(size_t)m * N + crow] = f2bf(v);
            }
          }
          ++crow;
        }
      }
      w[r] = ld_w16<NT>(lp);
      if (issued + 1 < total) {
        lp += 512;
        if (++lc == KC) { lc = 0; lp += row_skip; }
      }
      ++issued;
    }
  }
}

// M <= 16 GEMV / SwiGLU-down through gemv_rows_kernel: `rw` weight rows per wave, K split `split` ways
// (`swiglu` = flags, below)
// (K % (512 * split) == 0); P (split > 1) receives fp32 partials (Y == nullptr: left for a fused
// consumer, else reduced into Y).  Returns hipErrorInvalidValue for shapes it does not take.
extern "C" int ka_gemv_rows(void* Y, const void* X, const void* W, void* workspace, int M, int N, int K, int split,
                            int rw, int swiglu, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 16 || split < 1 || rw < 1 || K % (512 * split) != 0) return (int)hipErrorInvalidValue;
  const int kps = K / split;
  // X rows staged per workgroup: the next power of two >= M (8 / 16: the decode buckets above batch 4,
  // where the weight stream still sets the time and hipBLASLt's tiles do not reach the HBM rate)
  const int mr = M == 1 ? 1 : M == 2 ? 2 : M <= 4 ? 4 : M <= 8 ? 8 : 16;
  const size_t lds = (size_t)mr * kps * 2;
  if (lds > 65536) return (int)hipErrorInvalidValue;
  auto* x = static_cast<const bf16_t*>(X);
  auto* w = static_cast<const bf16_t*>(W);
  auto* y = static_cast<bf16_t*>(Y);
  float* p = split > 1 ? static_cast<float*>(workspace) : nullptr;
  dim3 grid((N + 4 * rw - 1) / (4 * rw), split);
  // flags bit 0: SwiGLU X staging; bit 1: 16-deep ring (measurement only); bit 2: non-temporal
  // weight loads (the engine's setting: profiles/r3/gemv_rows)
  const int var = swiglu >> 1;
  const bool sw = swiglu & 1;
#define KA_ROWS_LAUNCH(MRV, SW, RG, NTV) \
  hipLaunchKernelGGL((gemv_rows_kernel<MRV, RG, SW, NTV>), grid, dim3(256), lds, stream, x, w, y, p, M, N, K, kps, rw)
#define KA_ROWS_MR(SW, RG, NTV) \
  do { if (mr == 1) KA_ROWS_LAUNCH(1, SW, RG, NTV); else if (mr == 2) KA_ROWS_LAUNCH(2, SW, RG, NTV); \
       else if (mr == 4) KA_ROWS_LAUNCH(4, SW, RG, NTV); else if (mr == 8) KA_ROWS_LAUNCH(8, SW, RG, NTV); \
       else KA_ROWS_LAUNCH(16, SW, RG, NTV); } while (0)
#define KA_ROWS_VAR(SW) \
  do { if (var == 0) KA_ROWS_MR(SW, 8, false); else if (var == 1) KA_ROWS_MR(SW, 16, false); \
       else if (var == 2) KA_ROWS_MR(SW, 8, true); else KA_ROWS_MR(SW, 16, true); } while (0)
  if (sw) KA_ROWS_VAR(true);
  else KA_ROWS_VAR(false);
#undef KA_ROWS_VAR
#undef KA_ROWS_MR
#undef KA_ROWS_LAUNCH
  if (split > 1 && y != nullptr) ka_splitk_reduce_launch(y, p, split, (long)M * N, stream);
  KA_CHECK_LAUNCH();
}

template <int MT>
static void launch_mt(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int split, int kps,
                      hipStream_t stream) {
  dim3 grid((N + NW - 1) / NW, split);
  hipLaunchKernelGGL(gemm_skinny_kernel<MT>, grid, dim3(256), 0, stream, X, W, Y, P, M, N, K, kps);
}

// split > 1 requires a workspace P of split * M * N floats; Y is then produced by the reduce kernel.
extern "C" int ka_gemm_skinny(void* Y, const void* X, const void* W, void* workspace, int M, int N, int K, int split,
                              hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 256 || K % 64 != 0 || N % 4 != 0 || split < 1) return (int)hipErrorInvalidValue;
  int kps = (K / split + 63) / 64 * 64;
  split = (K + kps - 1) / kps;
  auto* x = static_cast<const bf16_t*>(X);
  auto* w = static_cast<const bf16_t*>(W);
  auto* y = static_cast<bf16_t*>(Y);
  float* p = split > 1 ? static_cast<float*>(workspace) : nullptr;
  const int mt = (M + 15) / 16;
  const size_t gemv_lds = (size_t)M * kps * 2;
  const int ring = gemv_ring_depth();
  if (M <= gemv_max_m() && ring > 0 && gemv_lds <= 65536) {
    dim3 grid((N + NW - 1) / NW, split);
    if (ring == 4)
      hipLaunchKernelGGL(gemv_ring_kernel<4>, grid, dim3(256), gemv_lds, stream, x, w, y, p, M, N, K, kps);
    else
      hipLaunchKernelGGL(gemv_ring_kernel<8>, grid, dim3(256), gemv_lds, stream, x, w, y, p, M, N, K, kps);
  } else if (mt <= 1) launch_mt<1>(x, w, y, p, M, N, K, split, kps, stream);
  else if (mt <= 2) launch_mt<2>(x, w, y, p, M, N, K, split, kps, stream);
  else if (mt <= 4) launch_mt<4>(x, w, y, p, M, N, K, split, kps, stream);
  else if (mt <= 6) launch_mt<6>(x, w, y, p, M, N, K, split, kps, stream);
  else if (mt <= 8) launch_mt<8>(x, w, y, p, M, N, K, split, kps, stream);
  else if (mt <= 12) launch_mt<12>(x, w, y, p, M, N, K, split, kps, stream);
  else launch_mt<16>(x, w, y, p, M, N, K, split, kps, stream);
  // Y == nullptr: leave the fp32 partials for a fused consumer (ka_rmsnorm_splitk)
  if (split > 1 && y != nullptr) ka_splitk_reduce_launch(y, p, split, (long)M * N, stream);
  KA_CHECK_LAUNCH();
}

// Y = swiglu(GU) * W^T for M <= GEMV_SWIGLU_MAX_M (GU = [M, 2K] gate | up): the batch-1..4 down projection
// with the SiLU*mul computed while staging X.  split > 1 needs the split * M * N float workspace;
// Y == nullptr leaves the partials for a fused consumer.  Returns hipErrorInvalidValue for shapes
// this path does not take (the caller then runs silu_mul + linear).
extern "C" int ka_gemv_swiglu(void* Y, const void* GU, const void* W, void* workspace, int M, int N, int K,
                              int split, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > GEMV_SWIGLU_MAX_M || K % 64 != 0 || N % 4 != 0 || split < 1) return (int)hipErrorInvalidValue;
  int kps = (K / split + 63) / 64 * 64;
  split = (K + kps - 1) / kps;
  const size_t lds = (size_t)M * kps * 2;
  if (lds > 65536) return (int)hipErrorInvalidValue;
  auto* y = static_cast<bf16_t*>(Y);
  float* p = split > 1 ? static_cast<float*>(workspace) : nullptr;
  dim3 grid((N + NW - 1) / NW, split);
  hipLaunchKernelGGL((gemv_ring_kernel<4, true>), grid, dim3(256), lds, stream, static_cast<const bf16_t*>(GU),
                     static_cast<const bf16_t*>(W), y, p, M, N, K, kps);
  if (split > 1 && y != nullptr) ka_splitk_reduce_launch(y, p, split, (long)M * N, stream);
  KA_CHECK_LAUNCH();
}
