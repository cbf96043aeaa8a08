// Greedy sampling with the SAFE_DECODE token mask (K10 epilogue) and the Mixtral router top-k (K11).
//
// masked_argmax: one workgroup per row; each lane scans 8 logits per 16-B load, skips tokens whose
// bit is clear in the row's mask (mask_idx[row] < 0 = unmasked), keeps (max, lowest index), then a
// wave shuffle + LDS reduction.  The same kernel serves the vocab-parallel LM head under TP: each
// rank reports (value, global index = local + vocab_offset) and the ranks' winners are combined
// after an all-gather (ops/__init__.py: tp_argmax).  temperature=0 in the reference (app.py:109).
#include "common.h"

// Small batches: the row is cut into gridDim.y slices (one workgroup each, partial (max, idx) to
// part_val / part_idx [rows][slices]) and argmax_finish_kernel picks the winner per row — one
// workgroup per 128k-entry row would leave the chip idle for ~30 us at batch 1.
template <int NT>
__global__ __launch_bounds__(NT) void masked_argmax_kernel(int* __restrict__ out_idx, float* __restrict__ out_val,
                                                           const bf16_t* __restrict__ logits,
                                                           const uint32_t* __restrict__ mask_bits,
                                                           const int* __restrict__ mask_idx, int vocab,
                                                           int mask_words, int vocab_offset,
                                                           float* __restrict__ part_val,
                                                           int* __restrict__ part_idx) {
  const int row = blockIdx.x;
  const bf16_t* lr = logits + (size_t)row * vocab;
  const int mi = mask_idx ? mask_idx[row] : -1;
  const uint32_t* mrow = mi >= 0 ? mask_bits + (size_t)mi * mask_words : nullptr;
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  const int nvec_all = vocab >> 3;
  const int per = (nvec_all + gridDim.y - 1) / gridDim.y;
  const int v0 = blockIdx.y * per;
  const int nvec = min(nvec_all, v0 + per);
  // Batches of UN vectors per lane: the UN mask words are loaded together, then the logits of the
  // vectors with any bit set, then all are scanned.  One vector per iteration waited for its mask
  // word and then for its logits: two serial memory latencies per 8 tokens per lane.  Within a lane
  // the vectors are still scanned in increasing index order.
  constexpr int UN = 8;
  for (int v = v0 + threadIdx.x; v < nvec; v += NT * UN) {
    uint32_t bits[UN], raw[UN];
    uint4 q[UN];
#pragma unroll
    for (int j = 0; j < UN; ++j) {
      const int gb = ((v + j * NT) << 3) + vocab_offset;   // the mask is indexed by the global token id
      raw[j] = 0xffffffffu;
      if (mrow && v + j * NT < nvec) raw[j] = mrow[gb >> 5];
    }
#pragma unroll
    for (int j = 0; j < UN; ++j) {
      const int gb = ((v + j * NT) << 3) + vocab_offset;
      bits[j] = v + j * NT < nvec ? (mrow ? (raw[j] >> (gb & 31)) & 0xffu : 0xffu) : 0u;
      if (bits[j]) q[j] = *reinterpret_cast<const uint4*>(lr + ((v + j * NT) << 3));
    }
#pragma unroll
    for (int j = 0; j < UN; ++j) {
      if (!bits[j]) continue;
      const int base = (v + j * NT) << 3;
      uint32_t w[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float x = (k & 1) ? hi_f(w[k >> 1]) : lo_f(w[k >> 1]);
        if (((bits[j] >> k) & 1u) && x > best) {  // strict '>' keeps the lowest index within a lane
          best = x;
          bidx = base + k;
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ob > best || (ob == best && oi < bidx)) {
      best = ob;
      bidx = oi;
    }
  }
  __shared__ float sb[NT / 64];
  __shared__ int si[NT / 64];
  if ((threadIdx.x & 63) == 0) {
    sb[threadIdx.x >> 6] = best;
    si[threadIdx.x >> 6] = bidx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = sb[0];
    int bi = si[0];
    for (int i = 1; i < NT / 64; ++i)
      if (sb[i] > b || (sb[i] == b && si[i] < bi)) {
        b = sb[i];
        bi = si[i];
      }
    if (part_val != nullptr) {   // sliced row: the finish kernel decides
      part_val[row * gridDim.y + blockIdx.y] = b;
      part_idx[row * gridDim.y + blockIdx.y] = bi;
      return;
    }
    if (bi == 0x7fffffff) bi = 0;  // fully masked row (cannot happen with a valid mask): token 0
    out_idx[row] = bi + vocab_offset;
    if (out_val) out_val[row] = b;
  }
}

__global__ __launch_bounds__(64) void argmax_finish_kernel(int* __restrict__ out_idx, float* __restrict__ out_val,
                                                           const float* __restrict__ part_val,
                                                           const int* __restrict__ part_idx, int slices,
                                                           int vocab_offset) {
  const int row = blockIdx.x;
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int i = threadIdx.x; i < slices; i += 64) {   // slices in index order: '>' keeps the lowest index
    const float v = part_val[row * slices + i];
    const int ix = part_idx[row * slices + i];
    if (v > best || (v == best && ix < bidx)) {
      best = v;
      bidx = ix;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ob > best || (ob == best && oi < bidx)) {
      best = ob;
      bidx = oi;
    }
  }
  if (threadIdx.x == 0) {
    if (bidx == 0x7fffffff) bidx = 0;
    out_idx[row] = bidx + vocab_offset;
    if (out_val) out_val[row] = best;
  }
}

// Per-slice (max, index) partials of another producer (the fused LM-head GEMM, gemm_big.hip) -> winner.
extern "C" int ka_argmax_finish(int* out_idx, float* out_val, const float* part_val, const int* part_idx, int rows,
                                int slices, int vocab_offset, hipStream_t stream) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(argmax_finish_kernel, dim3(rows), dim3(64), 0, stream, out_idx, out_val, part_val, part_idx,
                     slices, vocab_offset);
  KA_CHECK_LAUNCH();
}

// Vocab-parallel greedy combine under TP (A3): vals / idxs [ranks][rows] all-gathered from every
// rank's (max, global token id); out_idx[row] = the id of the largest value, the lowest id on ties
// (= the lowest rank: each rank owns a contiguous vocab slice).  One lane per row.
__global__ __launch_bounds__(256) void argmax_combine_kernel(int* __restrict__ out_idx, const float* __restrict__ vals,
                                                             const int* __restrict__ idxs, int rows, int ranks) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float best = vals[row];
  int bidx = idxs[row];
  for (int r = 1; r < ranks; ++r) {
    const float v = vals[(size_t)r * rows + row];
    const int ix = idxs[(size_t)r * rows + row];
    if (v > best || (v == best && ix < bidx)) {
      best = v;
      bidx = ix;
    }
  }
  out_idx[row] = bidx;
}

extern "C" int ka_argmax_combine(int* out_idx, const float* vals, const int* idxs, int rows, int ranks,
                                 hipStream_t stream) {
  if (rows <= 0) return 0;
  if (ranks < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(argmax_combine_kernel, dim3((rows + 255) / 256), dim3(256), 0, stream, out_idx, vals, idxs, rows,
                     ranks);
  KA_CHECK_LAUNCH();
}

// slices > 1 needs a workspace of rows * slices floats + rows * slices ints (ka_argmax_slices).
extern "C" int ka_argmax_slices(int rows, int vocab) {
  if (rows >= 128) return 1;
  int s = 1;
  while (s < 64 && rows * s * 2 <= 512 && vocab / (s * 2) >= 4096) s *= 2;
  return s;
}

extern "C" int ka_masked_argmax(int* out_idx, float* out_val, const void* logits, const uint32_t* mask_bits,
                                const int* mask_idx, int rows, int vocab, int mask_words, int vocab_offset,
                                void* workspace, int slices, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (vocab % 8 != 0 || vocab_offset % 8 != 0 || slices < 1 || (slices > 1 && workspace == nullptr))
    return (int)hipErrorInvalidValue;
  float* pv = slices > 1 ? static_cast<float*>(workspace) : nullptr;
  int* pi = slices > 1 ? reinterpret_cast<int*>(pv + (size_t)rows * slices) : nullptr;
  hipLaunchKernelGGL((masked_argmax_kernel<512>), dim3(rows, slices), dim3(512), 0, stream, out_idx, out_val,
                     static_cast<const bf16_t*>(logits), mask_bits, mask_idx, vocab, mask_words, vocab_offset, pv,
                     pi);
  if (slices > 1)
    hipLaunchKernelGGL(argmax_finish_kernel, dim3(rows), dim3(64), 0, stream, out_idx, out_val, pv, pi, slices,
                       vocab_offset);
  KA_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// Mixtral router: softmax over E experts (fp32), top-k (ties -> lower expert id), renormalised.
__global__ __launch_bounds__(256) void moe_topk_kernel(float* __restrict__ topk_w, int* __restrict__ topk_ids,
                                                       const bf16_t* __restrict__ logits, int tokens, int experts,
                                                       int k) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tokens) return;
  const bf16_t* l = logits + (size_t)t * experts;
  float mx = -INFINITY;
  for (int e = 0; e < experts; ++e) mx = fmaxf(mx, bf2f(l[e]));
  float p[64];
  float den = 0.f;
  for (int e = 0; e < experts; ++e) {
    p[e] = __expf(bf2f(l[e]) - mx);
    den += p[e];
  }
  unsigned long long used = 0ull;
  float wsum = 0.f;
  for (int j = 0; j < k; ++j) {
    int bi = -1;
    float bv = -1.f;
    for (int e = 0; e < experts; ++e)
      if (!((used >> e) & 1ull) && p[e] > bv) {
        bv = p[e];
        bi = e;
      }
    used |= 1ull << bi;
    topk_ids[t * k + j] = bi;
    topk_w[t * k + j] = bv / den;
    wsum += bv / den;
  }
  for (int j = 0; j < k; ++j) topk_w[t * k + j] /= wsum;
}

extern "C" int ka_moe_topk(float* topk_w, int* topk_ids, const void* logits, int tokens, int experts, int k,
                           hipStream_t stream) {
  if (tokens <= 0) return 0;
  if (experts > 64 || k > experts) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_topk_kernel, dim3((tokens + 255) / 256), dim3(256), 0, stream, topk_w, topk_ids,
                     static_cast<const bf16_t*>(logits), tokens, experts, k);
  KA_CHECK_LAUNCH();
}
