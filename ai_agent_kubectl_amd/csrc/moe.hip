// Mixtral MoE on MFMA (K12): route alignment -> grouped expert GEMMs -> weighted combine.
// Shape-static for a given token count, so the whole block is captured in the decode hipGraphs.
//
//   moe_align:    topk_ids [T, k] -> per-local-expert row lists (rows r = t*k + j routed to local
//                 expert e, e in [e0, e0 + El)); counts[El], lists[El][T*k] (order within a list is
//                 irrelevant: every row is computed independently and the combine sums in j order).
//   moe_gemm:     Y[r, :] = A[src(r), :] @ W[e]^T for every listed row r of expert e.  A row source
//                 is r / k (the token, first GEMM) or r (the slot, second GEMM).  Structure of
//                 gemm_skinny.hip: workgroup = 64 output columns x up to MT*16 rows of one expert,
//                 W fragments streamed HBM -> VGPR with a two-chunk register ring, gathered A rows
//                 staged through an XOR-swizzled LDS tile; expert weights are streamed once per
//                 (column tile, row chunk).
//   moe_combine:  out[t, :] = sum_j w[t, j] * Y[t*k + j, :] over local experts (EP partial; the
//                 caller's TP/EP all-reduce completes the sum).
#include "common.h"

__global__ __launch_bounds__(256) void moe_align_kernel(int* __restrict__ counts, int* __restrict__ lists,
                                                        const int* __restrict__ topk_ids, int rows, int e0, int el,
                                                        int list_stride) {
  __shared__ int cnt[64];
  for (int e = threadIdx.x; e < el; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    const int e = topk_ids[r] - e0;
    if (e >= 0 && e < el) {
      const int pos = atomicAdd(&cnt[e], 1);
      lists[e * list_stride + pos] = r;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < el; e += blockDim.x) counts[e] = cnt[e];
}

template <int MT>
__global__ __launch_bounds__(256) void moe_gemm_kernel(bf16_t* __restrict__ Y, float* __restrict__ P,
                                                       const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                       const int* __restrict__ counts, const int* __restrict__ lists,
                                                       int list_stride, int N, int K, int src_div, int n_rchunks,
                                                       int kps, int R) {
  constexpr int ROWS = MT * 16;
  constexpr int PIECES = ROWS * 8;
  constexpr int XR = (PIECES + 255) / 256;
  __shared__ __attribute__((aligned(16))) u32x4 xs[ROWS * 8];
  const int e = blockIdx.y;
  const int count = counts[e];
  const int ks = blockIdx.z / n_rchunks;             // split-K slice (P != nullptr when > 1 slices)
  const int r0 = (blockIdx.z % n_rchunks) * ROWS;
  const int kb = ks * kps;
  if (r0 >= count) return;
  const int nrows = min(ROWS, count - r0);
  const int* list = lists + (size_t)e * list_stride + r0;
  const bf16_t* We = W + (size_t)e * N * K;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int n0 = blockIdx.x * 64;
  const int wn = min(n0 + wave * 16 + col, N - 1);
  const bf16_t* wp = We + (size_t)wn * K + kb + 8 * grp;
  const int nchunks = min(kps, K - kb) >> 6;

  // per-thread source rows of the X staging pieces (fixed over the K loop)
  int srow[XR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int p = tid + 256 * i;
    const int rr = min(p >> 3, nrows - 1);
    srow[i] = list[rr] / src_div;
  }
  u32x4 xr[XR];
  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_x = [&](int c) {
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int p = tid + 256 * i;
      xr[i] = *reinterpret_cast<const u32x4*>(A + (size_t)srow[i] * K + kb + c * 64 + (p & 7) * 8);
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int p = tid + 256 * i;
      if (PIECES % 256 == 0 || p < PIECES) xs[(p >> 3) * 8 + ((p & 7) ^ ((p >> 3) & 7))] = xr[i];
    }
  };
  auto compute = [&](const uint4& w0, const uint4& w1) {
    const bf16x8 a0 = as_bf16x8(w0), a1 = as_bf16x8(w1);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = mt * 16 + col;
      acc[mt] = mfma16x16x32(a0, __builtin_bit_cast(bf16x8, xs[row * 8 + (grp ^ (row & 7))]), acc[mt]);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = mt * 16 + col;
      acc[mt] = mfma16x16x32(a1, __builtin_bit_cast(bf16x8, xs[row * 8 + ((4 + grp) ^ (row & 7))]), acc[mt]);
    }
  };
  auto load_w = [&](uint4& w0, uint4& w1, int c) {
    c = min(c, nchunks - 1);
    w0 = *reinterpret_cast<const uint4*>(wp + c * 64);
    w1 = *reinterpret_cast<const uint4*>(wp + c * 64 + 32);
  };

  uint4 wa0, wa1, wb0, wb1;
  load_w(wa0, wa1, 0);
  load_w(wb0, wb1, 1);
  load_x(0);
  store_x();
  __syncthreads();
  int c = 0;
  for (; c + 1 < nchunks; c += 2) {
    load_x(c + 1);
    compute(wa0, wa1);
    load_w(wa0, wa1, c + 2);
    __syncthreads();
    store_x();
    __syncthreads();
    load_x(min(c + 2, nchunks - 1));
    compute(wb0, wb1);
    load_w(wb0, wb1, c + 3);
    __syncthreads();
    store_x();
    __syncthreads();
  }
  if (c < nchunks) compute(wa0, wa1);

  const int nb = n0 + wave * 16 + 4 * grp;
  if (nb >= N) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + col;
    if (m < nrows) {
      if (P != nullptr) {
        *reinterpret_cast<f32x4*>(P + ((size_t)ks * R + list[m]) * N + nb) = acc[mt];
      } else {
        bf16_t* dst = Y + (size_t)list[m] * N + nb;
        *reinterpret_cast<uint2*>(dst) = make_uint2(pack2(acc[mt][0], acc[mt][1]), pack2(acc[mt][2], acc[mt][3]));
      }
    }
  }
}

__global__ __launch_bounds__(256) void moe_combine_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ Y,
                                                          const float* __restrict__ P, int split,
                                                          const float* __restrict__ topk_w,
                                                          const int* __restrict__ topk_ids, int k, int H, int e0,
                                                          int el) {
  const size_t pstride = (size_t)gridDim.x * k * H;   // one split-K slice of P: [T * k, H]
  const int t = blockIdx.x;
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int e = topk_ids[t * k + j] - e0;
      if (e < 0 || e >= el) continue;
      const float w = topk_w[t * k + j];
      if (P != nullptr) {   // the expert GEMM's split-K slices: reduce them here (fp32, no bf16 round)
        const float* pr = P + ((size_t)t * k + j) * H + c;
        // slices 4 at a time, each batch issued before its first add (summed in slice order)
        f32x4 y0 = f32x4{0.f, 0.f, 0.f, 0.f}, y1 = y0;
        for (int s0 = 0; s0 < split; s0 += 4) {
          f32x4 a[4], b[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (s0 + q < split) {
              a[q] = *reinterpret_cast<const f32x4*>(pr + (s0 + q) * pstride);
              b[q] = *reinterpret_cast<const f32x4*>(pr + (s0 + q) * pstride + 4);
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (s0 + q < split) {
              y0 += a[q];
              y1 += b[q];
            }
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q] += w * y0[q];
          acc[4 + q] += w * y1[q];
        }
        continue;
      }
      const uint4 y = *reinterpret_cast<const uint4*>(Y + ((size_t)t * k + j) * H + c);
      const uint32_t yw[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += w * lo_f(yw[q]);
        acc[2 * q + 1] += w * hi_f(yw[q]);
      }
    }
    *reinterpret_cast<uint4*>(out + (size_t)t * H + c) =
        make_uint4(pack2(acc[0], acc[1]), pack2(acc[2], acc[3]), pack2(acc[4], acc[5]), pack2(acc[6], acc[7]));
  }
}

// Routed rows sorted by local expert for the grouped prefill GEMM (csrc/gemm_big.hip, grouped mode).
// Block (e, y): expert e's rows [64 y, 64 y + 64) of its list go to sorted rows start_e + i (start_e =
// the row counts of the experts before e): xs[start_e + i] = x[lists[e][i] / src_div], slot[start_e + i]
// = lists[e][i].  Block (e, 0) also writes e's chunk-table entries (e, first sorted row, rows, 0), one
// per 256 rows, after the chunks of the experts before it; the last expert's block zeroes the entries
// past the last chunk up to max_chunks.
__global__ __launch_bounds__(256) void moe_sort_kernel(bf16_t* __restrict__ xs, int* __restrict__ slot,
                                                       int* __restrict__ tab, const bf16_t* __restrict__ x,
                                                       const int* __restrict__ counts, const int* __restrict__ lists,
                                                       int lstride, int src_div, int H, int el, int max_chunks) {
  const int e = blockIdx.x, y = blockIdx.y;
  int start = 0, cbase = 0;
  for (int i = 0; i < e; ++i) {   // el <= 64: every block sums the counts before its expert itself
    const int c = counts[i];
    start += c;
    cbase += (c + 255) >> 8;
  }
  const int cnt = counts[e];
  if (y == 0) {
    const int nch = (cnt + 255) >> 8;
    for (int c = threadIdx.x; c < nch; c += blockDim.x) {
      int* t = tab + 4 * (cbase + c);
      t[0] = e;
      t[1] = start + 256 * c;
      t[2] = min(256, cnt - 256 * c);
      t[3] = 0;
    }
    if (e == el - 1)
      for (int c = cbase + nch + threadIdx.x; c < max_chunks; c += blockDim.x) {
        int* t = tab + 4 * c;
        t[0] = t[1] = t[2] = t[3] = 0;
      }
  }
  const int r0 = 64 * y;
  if (r0 >= cnt) return;
  const int nr = min(64, cnt - r0);
  const int* li = lists + (size_t)e * lstride + r0;
  const int vec = H >> 3;   // 16-B pieces per row
  for (int p = threadIdx.x; p < nr * vec; p += blockDim.x) {
    const int i = p / vec, c = p - i * vec;
    reinterpret_cast<uint4*>(xs + (size_t)(start + r0 + i) * H)[c] =
        reinterpret_cast<const uint4*>(x + (size_t)(li[i] / src_div) * H)[c];
  }
  for (int i = threadIdx.x; i < nr; i += blockDim.x) slot[start + r0 + i] = li[i];
}

template <int MT>
static void launch_gemm(bf16_t* Y, float* P, const bf16_t* A, const bf16_t* W, const int* counts, const int* lists,
                        int stride, int el, int N, int K, int src_div, int max_rows, int split, int kps,
                        hipStream_t s) {
  const int n_rchunks = (max_rows + MT * 16 - 1) / (MT * 16);
  dim3 grid((N + 63) / 64, el, n_rchunks * split);
  hipLaunchKernelGGL(moe_gemm_kernel<MT>, grid, dim3(256), 0, s, Y, P, A, W, counts, lists, stride, N, K, src_div,
                     n_rchunks, kps, max_rows);
}

extern "C" int ka_moe_align(int* counts, int* lists, const int* topk_ids, int rows, int e0, int el, hipStream_t s) {
  if (rows <= 0) return 0;
  if (el > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_align_kernel, dim3(1), dim3(256), 0, s, counts, lists, topk_ids, rows, e0, el, rows);
  KA_CHECK_LAUNCH();
}

// Y [rows_total, N] (rows_total = T*k), A [T or T*k, K], W [el, N, K]; max_rows = T*k (worst case per expert).
// split > 1: K is cut into `split` slices of a multiple of 64 and every slice writes fp32 partials
// P [split, max_rows, N] (Y unused) for a consumer that reduces them (silu_mul_splitk after the
// w13 GEMM, moe_combine after w2).  At decode row counts only a couple of experts are active, so
// without a K split the w2 GEMM (N = 4096) would put ~128 workgroups on 256 CUs, each streaming
// 1.8 MB of weights through a latency-bound register ring.
extern "C" int ka_moe_gemm(void* Y, const void* A, const void* W, const int* counts, const int* lists, int list_stride,
                           int el, int N, int K, int src_div, int max_rows, int split, void* P, hipStream_t s) {
  if (max_rows <= 0) return 0;
  if (K % 64 != 0 || N % 4 != 0 || split < 1 || (split > 1 && P == nullptr)) return (int)hipErrorInvalidValue;
  const int kps = (K / 64 + split - 1) / split * 64;
  if ((K + kps - 1) / kps != split) return (int)hipErrorInvalidValue;   // every slice non-empty
  auto* y = static_cast<bf16_t*>(Y);
  auto* p = split > 1 ? static_cast<float*>(P) : nullptr;
  auto* a = static_cast<const bf16_t*>(A);
  auto* w = static_cast<const bf16_t*>(W);
  const int mt = (max_rows + 15) / 16;  // rows per expert never exceed max_rows
  if (mt <= 1) launch_gemm<1>(y, p, a, w, counts, lists, list_stride, el, N, K, src_div, max_rows, split, kps, s);
  else if (mt <= 2) launch_gemm<2>(y, p, a, w, counts, lists, list_stride, el, N, K, src_div, max_rows, split, kps, s);
  else if (mt <= 4) launch_gemm<4>(y, p, a, w, counts, lists, list_stride, el, N, K, src_div, max_rows, split, kps, s);
  else launch_gemm<8>(y, p, a, w, counts, lists, list_stride, el, N, K, src_div, max_rows, split, kps, s);
  KA_CHECK_LAUNCH();
}

// P != nullptr: read the w2 GEMM's split-K partials P [split, T*k, H] (fp32) instead of Y.
extern "C" int ka_moe_combine(void* out, const void* Y, const float* P, int split, const float* topk_w,
                              const int* topk_ids, int T, int k, int H, int e0, int el, hipStream_t s) {
  if (T <= 0) return 0;
  if (H % 8 != 0 || split < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, s, static_cast<bf16_t*>(out),
                     static_cast<const bf16_t*>(Y), P, split, topk_w, topk_ids, k, H, e0, el);
  KA_CHECK_LAUNCH();
}

// Expert-sorted rows and the chunk table of the grouped gemm_big prefill path (moe_sort_kernel):
// xs [rows, H], slot [rows], tab [max_chunks][4]; rows = T * k (the lists' stride and capacity),
// max_chunks >= ceil(rows / 256) + el.
extern "C" int ka_moe_sort(void* xs, int* slot, int* tab, const void* x, const int* counts, const int* lists, int rows,
                           int src_div, int H, int el, int max_chunks, hipStream_t s) {
  if (rows <= 0) return 0;
  if (el > 64 || H % 8 != 0 || max_chunks < (rows + 255) / 256 + el) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_sort_kernel, dim3(el, (rows + 63) / 64), dim3(256), 0, s, static_cast<bf16_t*>(xs), slot, tab,
                     static_cast<const bf16_t*>(x), counts, lists, rows, src_div, H, el, max_chunks);
  KA_CHECK_LAUNCH();
}
