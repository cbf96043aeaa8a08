// Paged attention on MFMA (K5 prefill, K6 decode) for head_dim 128, KV block size 16, GQA group G.
//
// Cache layouts (written by rope_kv_kernel in elementwise.hip):
//   k_cache [NB, Hkv, 16, 128]  token-major: the K^T B-operand fragment of lane l (token l&15, dims
//                               8*(l>>4)..+7 of a 32-wide k-step) is one contiguous 16-B load;
//   v_cache [NB, Hkv, 128, 16]  dim-major:   the V B-operand fragment of lane l (tokens 8*(l>>4)..+7,
//                               dim l&15 of an n-tile) is one contiguous 16-B load.
// MFMA: v_mfma_f32_16x16x32_bf16.  A[row l&15][k 8*(l>>4)+j], B[k 8*(l>>4)+j][col l&15],
//       C[row 4*(l>>4)+r][col l&15] (cdna_hip_programming.md §3).
// Softmax is online (running max m, running sum l per query row) in the exp2 domain.
//
// Decode (one query token per sequence): one workgroup per (kv head, sequence); the G query heads
// sharing the kv head are the 16 (zero-padded) MFMA rows; the 4 waves stride over 32-token chunks
// of the context, K/V fragments go straight from HBM to VGPRs (guide §5 table, 'GEMV / M <= 16'
// row: no reuse across waves, so an LDS round trip would be pure overhead), and the waves' partial
// (m, l, O) are merged through LDS.  P is re-laid from the C layout to the A layout through a
// per-wave LDS scratch.
//
// Prefill (varlen, with cached context for prefix caching / chunked prefill): one workgroup per
// (64 query rows = 64/G tokens x G heads, kv head, sequence); 4 waves x 16 rows.  K and V^T tiles
// of 32 tokens are shared by all 4 waves, so they are staged in LDS (XOR-swizzled against bank
// conflicts, guide §5.5 T2) with the next tile's global loads issued into registers before the
// current tile's MFMAs (T14 issue-early / write-late).
#include "common.h"

#define HD 128
#define KBS 16

// P re-layout scratch (per wave): the softmax probabilities leave the MFMA C layout (lane (col, grp)
// holds rows 4 grp + r, keys col and 16 + col) and are re-read in the A layout (lane holds row col,
// keys 8 grp .. 8 grp + 7).  16 rows x PSTR = 40 bf16 (64 B of P + 16 B of padding); 16-B chunk c of
// row x sits at slot c ^ p_slot_xor(x >> 2).  Neighbouring lanes swap one probability so that every
// lane stores one dword (even lanes keys col, col + 1; odd lanes keys 15 + col, 16 + col).  With the
// 80-B stride and this XOR both the stores (2 x 32 lanes on 32 banks) and the ds_read_b128 reads
// (4 x 16 lanes on 64 banks, MI355X_MICROARCH.md §LDS) are conflict-free — found by exhaustive search
// over strides and XOR maps; the previous 64-B rows cost 15-20 % extra LDS cycles.
constexpr int PSTR = 40;
KA_DEV int p_slot_xor(int q) { return (q ^ (q >> 1)) & 1; }
KA_DEV void p_store(bf16_t* pw, int prow, int col, float p0, float p1) {
  const float q0 = dpp_f<0xB1>(p0), q1 = dpp_f<0xB1>(p1);   // lane ^ 1
  const bool even = (col & 1) == 0;
  const int key = even ? col : 15 + col;
  const uint32_t v = even ? pack2(p0, q0) : pack2(q1, p1);
  const int slot = (key >> 3) ^ p_slot_xor(prow >> 2);
  *reinterpret_cast<uint32_t*>(pw + prow * PSTR + (slot << 3) + (key & 7)) = v;
}
KA_DEV bf16x8 p_load(const bf16_t* pw, int col, int grp) {
  return as_bf16x8(*reinterpret_cast<const uint4*>(pw + col * PSTR + ((grp ^ p_slot_xor((col >> 2) & 3)) << 3)));
}

// ------------------------------------------------------------------------------------------------
// Fused decode step (FUSED = true): the workgroup of (kv head h, sequence b) first does what
// rope_kv_kernel would do for its slice of the QKV projection (reducing the split-K partials on the
// fly when the projection left them): RoPE on its G query heads and its key head at position
// positions[b], the new K/V appended at slot_mapping[b].  The rotated queries go to LDS (never to
// HBM), the chunk loop runs over the ctx - 1 cached tokens, and the new token's score and value are
// folded into the cross-wave merge straight from LDS — no read-back of the slot being written, one
// kernel and one launch boundary less per layer.
struct DecodeFuse {
  const bf16_t* qkv;        // [B, (hq + 2 hkv) * 128] bf16, or nullptr when P is given
  const float* P;           // [split, B, (hq + 2 hkv) * 128] fp32 (or, pbf16, bf16) split-K partials
  int split;
  int pbf16;
  size_t pstride;
  const int* positions;
  const float* cos_sin;     // [max_pos, 128]: cos | sin halves
  const int* slot_mapping;
  bf16_t* k_cache;
  bf16_t* v_cache;
  // cascade (shared-prefix) mode, nshared != nullptr and *nshared > 0: the first *nshared blocks of
  // every sequence's table are the same physical blocks (prefix cache).  The chunk loop then skips
  // them, the rotated q rows go to q_out, and the merged (unnormalised o, max, denominator) go to
  // part_o / part_ml instead of `out`; cascade_prefix_kernel attends the shared blocks once per
  // (kv head, 16 query rows) and merges.
  const int* nshared;
  bf16_t* q_out;      // [B, hq, 128]
  float* part_o;      // [B, hq, 128]
  float* part_ml;     // [B, hq, 2]
};

// The slices are loaded DQ_UNROLL at a time, each batch issued before its first add (a rolled loop
// waited for each slice's load before issuing the next: `split` serial memory latencies in the
// kernel's prologue; the TP = 8 rank's QKV runs split 12).  Summed in order k = 0, 1, ...
constexpr int DQ_UNROLL = 4;
__device__ __forceinline__ uint2 dq_ld4(const DecodeFuse& f, size_t off) {
  if (f.P == nullptr) return *reinterpret_cast<const uint2*>(f.qkv + off);
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  if (f.pbf16) {   // bf16 slices (gemm_mfma EPI_P16): summed in fp32
    const bf16_t* pb = reinterpret_cast<const bf16_t*>(f.P);
    for (int k0 = 0; k0 < f.split; k0 += DQ_UNROLL) {
      uint2 q[DQ_UNROLL];
#pragma unroll
      for (int k = 0; k < DQ_UNROLL; ++k)
        if (k0 + k < f.split) q[k] = *reinterpret_cast<const uint2*>(pb + (k0 + k) * f.pstride + off);
#pragma unroll
      for (int k = 0; k < DQ_UNROLL; ++k)
        if (k0 + k < f.split) s += f32x4{lo_f(q[k].x), hi_f(q[k].x), lo_f(q[k].y), hi_f(q[k].y)};
    }
    return make_uint2(pack2(s[0], s[1]), pack2(s[2], s[3]));
  }
  for (int k0 = 0; k0 < f.split; k0 += DQ_UNROLL) {
    f32x4 p[DQ_UNROLL];
#pragma unroll
    for (int k = 0; k < DQ_UNROLL; ++k)
      if (k0 + k < f.split) p[k] = *reinterpret_cast<const f32x4*>(f.P + (k0 + k) * f.pstride + off);
#pragma unroll
    for (int k = 0; k < DQ_UNROLL; ++k)
      if (k0 + k < f.split) s += p[k];
  }
  return make_uint2(pack2(s[0], s[1]), pack2(s[2], s[3]));
}

// N reads of dq_ld4 at once (a thread's q / k rotary halves and its new-value dims): every batch
// issues the N reads' slices together, so the N reductions cost one round trip per batch, not N.
template <int N>
__device__ __forceinline__ void dq_ld4n(const DecodeFuse& f, const size_t (&off)[N], const bool (&en)[N],
                                        uint2 (&out)[N]) {
  if (f.P == nullptr) {
#pragma unroll
    for (int n = 0; n < N; ++n)
      if (en[n]) out[n] = *reinterpret_cast<const uint2*>(f.qkv + off[n]);
    return;
  }
  f32x4 s[N];
#pragma unroll
  for (int n = 0; n < N; ++n) s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (f.pbf16) {
    const bf16_t* pb = reinterpret_cast<const bf16_t*>(f.P);
    for (int k0 = 0; k0 < f.split; k0 += DQ_UNROLL) {
      uint2 q[DQ_UNROLL][N];
#pragma unroll
      for (int k = 0; k < DQ_UNROLL; ++k)
#pragma unroll
        for (int n = 0; n < N; ++n)
          if (en[n] && k0 + k < f.split) q[k][n] = *reinterpret_cast<const uint2*>(pb + (k0 + k) * f.pstride + off[n]);
#pragma unroll
      for (int k = 0; k < DQ_UNROLL; ++k)
#pragma unroll
        for (int n = 0; n < N; ++n)
          if (en[n] && k0 + k < f.split) s[n] += f32x4{lo_f(q[k][n].x), hi_f(q[k][n].x), lo_f(q[k][n].y), hi_f(q[k][n].y)};
    }
  } else {   // fp32 slices: half the batch (twice the registers per slice)
    constexpr int U = DQ_UNROLL / 2;
    for (int k0 = 0; k0 < f.split; k0 += U) {
      f32x4 p[U][N];
#pragma unroll
      for (int k = 0; k < U; ++k)
#pragma unroll
        for (int n = 0; n < N; ++n)
          if (en[n] && k0 + k < f.split) p[k][n] = *reinterpret_cast<const f32x4*>(f.P + (k0 + k) * f.pstride + off[n]);
#pragma unroll
      for (int k = 0; k < U; ++k)
#pragma unroll
        for (int n = 0; n < N; ++n)
          if (en[n] && k0 + k < f.split) s[n] += p[k][n];
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) out[n] = make_uint2(pack2(s[n][0], s[n][1]), pack2(s[n][2], s[n][3]));
}

// NW = waves per workgroup.  4: wave w takes the 32-token chunks w, w + 4, ... (one chunk each at
// the serving context); 2: chunks w, w + 2, ... with half the LDS (8 workgroups per CU instead of
// 4), so a B = 256 step's 2048 (kv head, sequence) workgroups run in ONE round of the chip instead
// of two — chosen on the host when B * hkv exceeds what one round of 4-wave workgroups holds.
template <bool FUSED, int NW = 4>
__global__ __launch_bounds__(64 * NW, 4) void paged_decode_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ q,
                                                           const bf16_t* __restrict__ k_cache,
                                                           const bf16_t* __restrict__ v_cache,
                                                           const int* __restrict__ block_tables, int max_blocks,
                                                           const int* __restrict__ ctx_lens, int hq, int hkv,
                                                           float scale_log2, DecodeFuse fz) {
  const int h = blockIdx.x, b = blockIdx.y;
  const int G = hq / hkv;
  // fused: wave-uniform (readfirstlane), so the block-table reads below become scalar loads issued
  // together, not vector loads each waited for before the K / V loads they address (the non-fused
  // kernel keeps the vector form: with scalar indices it spills 3 VGPRs in the chunk loop)
  const int lane = threadIdx.x & 63, wave = FUSED ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  int ns = 0;   // cascade: shared leading blocks, attended by cascade_prefix_kernel
  // fused: the row's position and cache slot are read before the K loads are issued, so that waiting
  // for them (in-order vmcnt) does not also wait for K
  int pos_b = 0, slot_b = -1;
  if constexpr (FUSED) {
    if (fz.nshared != nullptr) ns = *fz.nshared;
    pos_b = __builtin_amdgcn_readfirstlane(fz.positions[b]);
    slot_b = __builtin_amdgcn_readfirstlane(fz.slot_mapping[b]);
  }
  // fused: the chunk loop covers the cached tokens only; the new one is merged from LDS
  const int ctx = ctx_lens[b] - (FUSED ? 1 : 0) - ns * KBS;

  __shared__ __attribute__((aligned(16))) float smem[NW * 16 * 2 + NW * 16 * (HD + 4)];
  // per-wave P scratch; fused: first the staging of the G rotated q rows + k ((G + 1) x 128 bf16,
  // which the host guarantees fits: G + 1 <= NW * 16 * PSTR / 128)
  __shared__ __attribute__((aligned(16))) bf16_t p_lds[NW][16 * PSTR];
  // fused: new token's value and per-row score (the rotated q rows and k are staged in p_lds)
  __shared__ __attribute__((aligned(16))) float new_lds[FUSED ? HD / 2 + 16 : 4];
  float* sm = smem;                 // [NW][16]
  float* sl = smem + NW * 16;       // [NW][16]
  float* so = smem + NW * 32;       // [NW][16][HD+4]

  // The wave's first 32-token chunk of K and V is fetched before anything else: those loads
  // depend only on the block table, so their HBM latency overlaps the fused prologue's (split-K
  // partial loads, RoPE, cache append) instead of following it.  At the serving shape (context
  // <= 128 tokens, one chunk per wave) that is the whole chunk loop's memory traffic.
  const int* bt = block_tables + (size_t)b * max_blocks + ns;
  const int nchunks = (ctx + 31) >> 5;
  const size_t head_stride = (size_t)KBS * HD;  // elements per (block, head)
  uint4 kr[2][4], vr[8];
  // Chunk c's two 16-token blocks (the second used only when the chunk reaches past its first).  The
  // fused kernel reads them with scalar loads (uniform wave index); the second entry shares the first
  // one's scalar-cache line.  The second index is clamped to the row.
  const int last_entry = max_blocks - ns - 1;
  auto blocks = [&](int c, int& blk0, int& blk1) {
    blk0 = bt[2 * c];
    const int e1 = bt[min(2 * c + 1, last_entry)];
    blk1 = (c * 32 + 16 < ctx) ? e1 : blk0;
  };
  auto load_k = [&](int c) {
    int blk0, blk1;
    blocks(c, blk0, blk1);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16_t* kp = k_cache + ((size_t)(j ? blk1 : blk0) * hkv + h) * head_stride + col * HD + 8 * grp;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) kr[j][ks] = *reinterpret_cast<const uint4*>(kp + 32 * ks);
    }
  };
  auto load_v = [&](int c) {
    int blk0, blk1;
    blocks(c, blk0, blk1);
    const int blk = (grp >> 1) ? blk1 : blk0;
    const bf16_t* vp = v_cache + ((size_t)blk * hkv + h) * head_stride + col * KBS + 8 * (grp & 1);
#pragma unroll
    for (int n = 0; n < 8; ++n) vr[n] = *reinterpret_cast<const uint4*>(vp + (size_t)n * 16 * KBS);
  };
  if (wave < nchunks) {
    load_k(wave);
    // fused: V after the prologue (issuing it here too measured 24.3 vs 23.4 us at B = 256,
    // 9.9 vs 10.4 at B = 1: profiles/r3/decode_attn_early_v/)
    if constexpr (!FUSED) load_v(wave);
  }

  if constexpr (FUSED) {
    const int half = HD / 2;
    const size_t stride = (size_t)(hq + 2 * hkv) * HD;
    const size_t rowoff = (size_t)b * stride;
    const float* cs = fz.cos_sin + (size_t)pos_b * HD;
    const int slot = slot_b;   // -1: padding row (no cache write, empty output)
    const int blk = slot >= 0 ? slot / KBS : 0, off = slot >= 0 ? slot % KBS : 0;
    // (G query heads + 1 key head) x 16 items of 4 rotary pairs; in its first item a thread < 32 also
    // reads the new value's 4 dims, in the same batches as the item's two halves ((G + 1) * 16 >= 32)
    uint2 vnew = make_uint2(0u, 0u);
    for (int it = threadIdx.x; it < (G + 1) * 16; it += 64 * NW) {
      const int hh = it >> 4, i = (it & 15) * 4;
      const size_t col0 = hh < G ? (size_t)(h * G + hh) * HD : (size_t)(hq + h) * HD;
      const size_t offs[3] = {rowoff + col0 + i, rowoff + col0 + i + half,
                              rowoff + (size_t)(hq + hkv + h) * HD + threadIdx.x * 4};
      const bool en[3] = {true, true, it == (int)threadIdx.x && threadIdx.x < HD / 4};
      uint2 rd[3];
      dq_ld4n<3>(fz, offs, en, rd);
      if (en[2]) vnew = rd[2];
      const uint2 a = rd[0], c2 = rd[1];
      const float4 c = *reinterpret_cast<const float4*>(cs + i);
      const float4 sn = *reinterpret_cast<const float4*>(cs + half + i);
      const float x1[4] = {lo_f(a.x), hi_f(a.x), lo_f(a.y), hi_f(a.y)};
      const float x2[4] = {lo_f(c2.x), hi_f(c2.x), lo_f(c2.y), hi_f(c2.y)};
      const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
      float o1[4], o2[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o1[k] = x1[k] * cc[k] - x2[k] * ss[k];
        o2[k] = x2[k] * cc[k] + x1[k] * ss[k];
      }
      const uint2 r1 = make_uint2(pack2(o1[0], o1[1]), pack2(o1[2], o1[3]));
      const uint2 r2 = make_uint2(pack2(o2[0], o2[1]), pack2(o2[2], o2[3]));
      bf16_t* dl = &p_lds[0][0] + hh * HD;   // rows 0..G-1: q heads, row G: k
      *reinterpret_cast<uint2*>(dl + i) = r1;
      *reinterpret_cast<uint2*>(dl + i + half) = r2;
      if (hh == G && slot >= 0) {
        bf16_t* kd = fz.k_cache + (((size_t)blk * hkv + h) * KBS + off) * HD;
        *reinterpret_cast<uint2*>(kd + i) = r1;
        *reinterpret_cast<uint2*>(kd + i + half) = r2;
      }
    }
    // value: 32 items of 4 dims -> LDS and the dim-major cache slot
    if (threadIdx.x < HD / 4) {
      const int i = threadIdx.x * 4;
      const uint2 v = vnew;
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(new_lds) + i) = v;
      if (slot >= 0) {
      bf16_t* vd = fz.v_cache + (((size_t)blk * hkv + h) * HD + i) * KBS + off;
      vd[0] = (bf16_t)v.x;
      vd[KBS] = (bf16_t)(v.x >> 16);
      vd[2 * KBS] = (bf16_t)v.y;
      vd[3 * KBS] = (bf16_t)(v.y >> 16);
      }
    }
    __syncthreads();
    if (ns > 0) {   // cascade: the rotated q rows for cascade_prefix_kernel
      for (int i = threadIdx.x; i < G * 16; i += 64 * NW) {
        const int row = i >> 4, c8 = (i & 15) * 8;
        *reinterpret_cast<uint4*>(fz.q_out + ((size_t)b * hq + h * G + row) * HD + c8) =
            *reinterpret_cast<const uint4*>(&p_lds[0][0] + row * HD + c8);
      }
    }
  }

  if constexpr (FUSED) {
    if (wave < nchunks) load_v(wave);
  }
  bf16x8 qf[4];
  {
    const int row = col;
    if (row < G) {
      const bf16_t* qp = FUSED ? &p_lds[0][0] + row * HD + 8 * grp : q + ((size_t)b * hq + h * G + row) * HD + 8 * grp;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) qf[ks] = as_bf16x8(*reinterpret_cast<const uint4*>(qp + 32 * ks));
    } else {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) qf[ks] = as_bf16x8(make_uint4(0, 0, 0, 0));
    }
  }
  if constexpr (FUSED) {
    // new token's score per query row (wave 0): lane (col = row, grp) holds dims 8*grp + 32*ks
    if (wave == 0 && col < G) {
      const bf16_t* kp = &p_lds[0][0] + G * HD + 8 * grp;
      float dot = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const uint4 ka = *reinterpret_cast<const uint4*>(kp + 32 * ks);
        const uint4 qa = __builtin_bit_cast(uint4, qf[ks]);
        const uint32_t qw[4] = {qa.x, qa.y, qa.z, qa.w}, kw[4] = {ka.x, ka.y, ka.z, ka.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) dot += lo_f(qw[k]) * lo_f(kw[k]) + hi_f(qw[k]) * hi_f(kw[k]);
      }
      dot += __shfl_xor(dot, 16, 64);
      dot += __shfl_xor(dot, 32, 64);
      if (grp == 0) new_lds[HD / 2 + col] = slot_b >= 0 ? dot * scale_log2 : -INFINITY;
    }
    __syncthreads();   // p_lds is the chunk loop's P scratch from here on
  }
  float m[4], l[4];
  f32x4 o[8];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
  }
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16_t* pw = p_lds[wave];
  // Later chunks (contexts > 32 NW tokens): K(c) and V(c) are issued together at the loop's top (both
  // register sets are free once PV(c - NW) has read vr), so a chunk waits one memory latency instead
  // of two (K, then V after the QK).  Issue order = use order: the compiler's counted vmcnt wait lets
  // K through while V is still in flight (plain loads retire in order).  Prefetching K(c + NW) during
  // chunk c instead needs kr live across the softmax: 29 VGPRs of spills at 128.
  for (int c = wave; c < nchunks; c += NW) {
    const int t0 = c * 32;
    if (c != wave) {
      load_k(c);
      load_v(c);
    }
    // ---- S = Q K^T for the two 16-token halves ----
    f32x4 s[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = mfma16x16x32(qf[ks], as_bf16x8(kr[j][ks]), acc);
      s[j] = acc;
    }
    // ---- online softmax over this chunk ----
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x0 = (t0 + col < ctx) ? s[0][r] * scale_log2 : -INFINITY;
      float x1 = (t0 + 16 + col < ctx) ? s[1][r] * scale_log2 : -INFINITY;
      const float mx = row16_max(fmaxf(x0, x1));
      const float mn = fmaxf(m[r], mx);
      alpha[r] = exp2f(m[r] - mn);
      const float p0 = exp2f(x0 - mn), p1 = exp2f(x1 - mn);
      l[r] = l[r] * alpha[r] + row16_sum(p0 + p1);
      m[r] = mn;
      p_store(pw, 4 * grp + r, col, p0, p1);
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[n][r] *= alpha[r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bf16x8 pf = p_load(pw, col, grp);
#pragma unroll
    for (int n = 0; n < 8; ++n) o[n] = mfma16x16x32(pf, as_bf16x8(vr[n]), o[n]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // P scratch reads done before next chunk's writes
  }

  // ---- merge the NW waves ----
  if (col == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sm[wave * 16 + 4 * grp + r] = m[r];
      sl[wave * 16 + 4 * grp + r] = l[r];
    }
  }
#pragma unroll
  for (int n = 0; n < 8; ++n) {
#pragma unroll
    for (int r = 0; r < 4; ++r) so[(wave * 16 + 4 * grp + r) * (HD + 4) + n * 16 + col] = o[n][r];
  }
  __syncthreads();
  const int d0 = (threadIdx.x & 15) * 8;     // 8 dims per thread, 4 NW rows per pass
  for (int row = threadIdx.x >> 4; row < G; row += 4 * NW) {
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, sm[w * 16 + row]);
    float s_new = -INFINITY;
    if constexpr (FUSED) {
      s_new = new_lds[HD / 2 + row];
      M = fmaxf(M, s_new);
    }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float den = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float e = exp2f(sm[w * 16 + row] - M);
        den += e * sl[w * 16 + row];
        const float* src = so + (w * 16 + row) * (HD + 4) + d0;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += e * src[k];
      }
      if constexpr (FUSED) {
        const float e = exp2f(s_new - M);
        den += e;
        const uint4 va = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(new_lds) + d0);
        const uint32_t vw[4] = {va.x, va.y, va.z, va.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[2 * k] += e * lo_f(vw[k]);
          acc[2 * k + 1] += e * hi_f(vw[k]);
        }
      }
    }
    if (FUSED && ns > 0) {   // cascade: the unnormalised partial, merged by cascade_prefix_kernel
      const size_t idx = (size_t)b * hq + h * G + row;
      float* po = fz.part_o + idx * HD + d0;
      *reinterpret_cast<float4*>(po) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(po + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
      if (d0 == 0) *reinterpret_cast<float2*>(fz.part_ml + idx * 2) = make_float2(M, den);
      continue;
    }
    const float inv = den > 0.f ? 1.f / den : 0.f;
    uint4 res = make_uint4(pack2(acc[0] * inv, acc[1] * inv), pack2(acc[2] * inv, acc[3] * inv),
                           pack2(acc[4] * inv, acc[5] * inv), pack2(acc[6] * inv, acc[7] * inv));
    *reinterpret_cast<uint4*>(out + ((size_t)b * hq + h * G + row) * HD + d0) = res;
  }
}


// 2-wave workgroups once the grid exceeds one round of 4-wave ones (4 per CU by LDS and VGPRs):
// KA_DECODE_NW2_MIN_WGS (default 4 x CUs = 1024; 0 = never).  The fused prologue stages G + 1 rows
// of 128 in the 2-wave P scratch: G <= 9.
static bool decode_two_waves(int batch, int hq, int hkv) {
  static int min_wgs = -1;
  if (min_wgs < 0) {
    const char* e = getenv("KA_DECODE_NW2_MIN_WGS");
    int cus = 256, dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    min_wgs = e ? atoi(e) : 4 * cus;
  }
  const int G = hq / hkv;
  return min_wgs > 0 && (long)batch * hkv > min_wgs && (G + 1) * HD <= 2 * 16 * PSTR;
}

extern "C" int ka_paged_decode(void* out, const void* q, const void* k_cache, const void* v_cache,
                               const int* block_tables, int max_blocks, const int* ctx_lens, int batch, int hq,
                               int hkv, int head_dim, int block_size, float scale, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (head_dim != HD || block_size != KBS || hq % hkv != 0 || hq / hkv > 16) return (int)hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  auto args = [&](auto kern, int nw) {
    hipLaunchKernelGGL(kern, dim3(hkv, batch), dim3(64 * nw), 0, stream, static_cast<bf16_t*>(out),
                       static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k_cache),
                       static_cast<const bf16_t*>(v_cache), block_tables, max_blocks, ctx_lens, hq, hkv, scale_log2,
                       DecodeFuse{});
  };
  if (decode_two_waves(batch, hq, hkv)) args(paged_decode_kernel<false, 2>, 2);
  else args(paged_decode_kernel<false, 4>, 4);
  KA_CHECK_LAUNCH();
}

// Fused RoPE + KV append + paged decode attention (one query token per sequence; every
// slot_mapping entry must be a valid slot).  qkv: bf16 [B, (hq + 2 hkv) * 128], or P: fp32 split-K
// partials [split, B, (hq + 2 hkv) * 128], bf16 when p_bf16 (qkv ignored when P is non-null).
// ctx_lens include the new token.
extern "C" int ka_paged_decode_rope(void* out, const void* qkv, const float* P, int split, int p_bf16, void* k_cache,
                                    void* v_cache, const int* positions, const float* cos_sin,
                                    const int* slot_mapping, const int* block_tables, int max_blocks,
                                    const int* ctx_lens, int batch, int hq, int hkv, int head_dim, int block_size,
                                    float scale, hipStream_t stream) {
  if (batch <= 0) return 0;
  // the rotated q rows + k are staged in the 4 KB P scratch: G + 1 <= 16 rows of 128
  if (head_dim != HD || block_size != KBS || hq % hkv != 0 || hq / hkv > 15) return (int)hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  DecodeFuse fz{static_cast<const bf16_t*>(qkv), P, split, p_bf16, (size_t)batch * (hq + 2 * hkv) * HD, positions,
                cos_sin, slot_mapping, static_cast<bf16_t*>(k_cache), static_cast<bf16_t*>(v_cache),
                nullptr, nullptr, nullptr, nullptr};
  auto args = [&](auto kern, int nw) {
    hipLaunchKernelGGL(kern, dim3(hkv, batch), dim3(64 * nw), 0, stream, static_cast<bf16_t*>(out), nullptr,
                       static_cast<const bf16_t*>(k_cache), static_cast<const bf16_t*>(v_cache), block_tables,
                       max_blocks, ctx_lens, hq, hkv, scale_log2, fz);
  };
  if (decode_two_waves(batch, hq, hkv)) args(paged_decode_kernel<true, 2>, 2);
  else args(paged_decode_kernel<true, 4>, 4);
  KA_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// Cascade decode attention, part 2 (after paged_decode_kernel<true> in cascade mode): the nshared
// leading blocks that every sequence of the batch shares (the prefix cache hands all of them the
// same physical blocks) are attended ONCE per (kv head, 16 query rows) instead of once per
// sequence: at B = 256 with an 80-token shared prefix the chain kernel read those blocks 256 times
// (≈ 80 MB of L2 traffic per layer).  Wave w of workgroup (h, y) takes sequences
// (4 y + w) 16 / G ..: 16 query rows (16 / G sequences x G heads) on MFMA 16x16x32 over 32-token
// chunks (the layouts of paged_decode_kernel), then merges with the per-sequence partial.
template <int G>
__global__ __launch_bounds__(256) void cascade_prefix_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ qrot,
                                                             const float* __restrict__ part_o,
                                                             const float* __restrict__ part_ml,
                                                             const bf16_t* __restrict__ k_cache,
                                                             const bf16_t* __restrict__ v_cache,
                                                             const int* __restrict__ block_tables,
                                                             const int* __restrict__ nshared, int batch, int hq, int hkv,
                                                             float scale_log2) {
  const int ns = *nshared;
  if (ns <= 0) return;   // no shared prefix this step: paged_decode_kernel wrote the outputs
  constexpr int SPW = 16 / G;   // sequences per wave
  const int h = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int s0 = (blockIdx.y * 4 + wave) * SPW;
  __shared__ __attribute__((aligned(16))) bf16_t p_lds[4][16 * PSTR];
  if (s0 >= batch) return;   // (no workgroup barrier below)
  const int ntok = ns * KBS, nchunks = (ntok + 31) >> 5;
  const size_t head_stride = (size_t)KBS * HD;
  const int qs = s0 + col / G;   // query row col: sequence qs, head h G + col % G
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    qf[ks] = as_bf16x8(qs < batch ? *reinterpret_cast<const uint4*>(qrot + ((size_t)qs * hq + h * G + col % G) * HD +
                                                                  8 * grp + 32 * ks)
                                  : make_uint4(0, 0, 0, 0));
  float m[4], l[4];
  f32x4 o[8];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
  }
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16_t* pw = p_lds[wave];
  for (int c = 0; c < nchunks; ++c) {
    const int t0 = c * 32;
    const int blk0 = block_tables[2 * c], blk1 = 2 * c + 1 < ns ? block_tables[2 * c + 1] : blk0;
    uint4 kr[2][4], vr[8];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16_t* kp = k_cache + ((size_t)(j ? blk1 : blk0) * hkv + h) * head_stride + col * HD + 8 * grp;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) kr[j][ks] = *reinterpret_cast<const uint4*>(kp + 32 * ks);
    }
    const bf16_t* vp = v_cache + ((size_t)((grp >> 1) ? blk1 : blk0) * hkv + h) * head_stride + col * KBS + 8 * (grp & 1);
#pragma unroll
    for (int n = 0; n < 8; ++n) vr[n] = *reinterpret_cast<const uint4*>(vp + (size_t)n * 16 * KBS);
    f32x4 sc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = mfma16x16x32(qf[ks], as_bf16x8(kr[j][ks]), acc);
      sc[j] = acc;
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x0 = t0 + col < ntok ? sc[0][r] * scale_log2 : -INFINITY;
      const float x1 = t0 + 16 + col < ntok ? sc[1][r] * scale_log2 : -INFINITY;
      const float mn = fmaxf(m[r], row16_max(fmaxf(x0, x1)));
      alpha[r] = exp2f(m[r] - mn);
      const float p0 = exp2f(x0 - mn), p1 = exp2f(x1 - mn);
      l[r] = l[r] * alpha[r] + row16_sum(p0 + p1);
      m[r] = mn;
      p_store(pw, 4 * grp + r, col, p0, p1);
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[n][r] *= alpha[r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bf16x8 pf = p_load(pw, col, grp);
#pragma unroll
    for (int n = 0; n < 8; ++n) o[n] = mfma16x16x32(pf, as_bf16x8(vr[n]), o[n]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // merge: lane (col, grp) holds rows 4 grp + r, dims 16 n + col
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * grp + r, seq = s0 + row / G;
    if (seq >= batch) continue;
    const size_t idx = (size_t)seq * hq + h * G + row % G;
    const float2 ml = *reinterpret_cast<const float2*>(part_ml + idx * 2);
    const float M = fmaxf(m[r], ml.x);
    const float ea = exp2f(m[r] - M), eb = ml.x == -INFINITY ? 0.f : exp2f(ml.x - M);
    const float inv = 1.f / (ea * l[r] + eb * ml.y);
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int d = n * 16 + col;
      out[idx * HD + d] = f2bf((ea * o[n][r] + eb * part_o[idx * HD + d]) * inv);
    }
  }
}

// Workspace bytes of the cascade mode: partial o (fp32) + (max, denominator) + rotated q (bf16).
extern "C" size_t ka_decode_cascade_ws(int batch, int hq) {
  return (size_t)batch * hq * (HD * 4 + 8 + HD * 2);
}

// ka_paged_decode_rope with the shared-prefix cascade: nshared (device int [1]) leading blocks of
// every block table are shared by the whole batch (0: the plain kernel's result, the second kernel
// returns at once).  Needs hq / hkv in {1, 2, 4, 8, 16}.
extern "C" int ka_paged_decode_rope_cascade(void* out, const void* qkv, const float* P, int split, int p_bf16,
                                            void* k_cache, void* v_cache, const int* positions, const float* cos_sin,
                                            const int* slot_mapping, const int* block_tables, int max_blocks,
                                            const int* ctx_lens, int batch, int hq, int hkv, int head_dim,
                                            int block_size, float scale, const int* nshared, void* ws,
                                            hipStream_t stream) {
  if (batch <= 0) return 0;
  const int G = hq / hkv;
  if (head_dim != HD || block_size != KBS || hq % hkv != 0 || G > 15 || 16 % G != 0 || ws == nullptr ||
      nshared == nullptr)
    return (int)hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  float* part_o = static_cast<float*>(ws);
  float* part_ml = part_o + (size_t)batch * hq * HD;
  bf16_t* q_out = reinterpret_cast<bf16_t*>(part_ml + (size_t)batch * hq * 2);
  DecodeFuse fz{static_cast<const bf16_t*>(qkv), P, split, p_bf16, (size_t)batch * (hq + 2 * hkv) * HD, positions,
                cos_sin, slot_mapping, static_cast<bf16_t*>(k_cache), static_cast<bf16_t*>(v_cache),
                nshared, q_out, part_o, part_ml};
  auto args = [&](auto kern, int nw) {
    hipLaunchKernelGGL(kern, dim3(hkv, batch), dim3(64 * nw), 0, stream, static_cast<bf16_t*>(out), nullptr,
                       static_cast<const bf16_t*>(k_cache), static_cast<const bf16_t*>(v_cache), block_tables,
                       max_blocks, ctx_lens, hq, hkv, scale_log2, fz);
  };
  if (decode_two_waves(batch, hq, hkv)) args(paged_decode_kernel<true, 2>, 2);
  else args(paged_decode_kernel<true, 4>, 4);
  const int spw = 16 / G;
  const dim3 grid(hkv, (batch + 4 * spw - 1) / (4 * spw));
#define KA_CASCADE(GV)                                                                                                    \
  hipLaunchKernelGGL(cascade_prefix_kernel<GV>, grid, dim3(256), 0, stream, static_cast<bf16_t*>(out), q_out, part_o, \
                     part_ml, static_cast<const bf16_t*>(k_cache), static_cast<const bf16_t*>(v_cache), block_tables,   \
                     nshared, batch, hq, hkv, scale_log2)
  switch (G) {
    case 1: KA_CASCADE(1); break;
    case 2: KA_CASCADE(2); break;
    case 4: KA_CASCADE(4); break;
    default: KA_CASCADE(8); break;
  }
#undef KA_CASCADE
  KA_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// Varlen paged prefill.  q/out [T, Hq, 128]; seq s owns query rows q_starts[s] .. q_starts[s+1]-1,
// which are the LAST q_len positions of its ctx_lens[s]-token context (earlier positions are
// already in the cache: shared prefix blocks or previous chunks).  Causal within the context.
struct PrefillSmem {
  uint4 k[32][16];        // [token][16-B chunk ^ (token & 15)]            8 KiB
  uint4 v[HD][4];         // [dim][16-B chunk ^ (((dim >> 2) & 1) << 1)] tokens 8 KiB
  bf16_t p[4][16 * PSTR]; // per-wave P scratch (p_store / p_load)         5 KiB
};

__device__ __forceinline__ void prefill_load_tile(u32x4 (&kreg)[2], u32x4 (&vreg)[2], const bf16_t* __restrict__ k_cache,
                                                  const bf16_t* __restrict__ v_cache, const int* __restrict__ bt,
                                                  int nblocks, int tile, int h, int hkv) {
  const int tid = threadIdx.x;
  const size_t head_stride = (size_t)KBS * HD;
  // the tile's two blocks, read once per workgroup as scalar loads (tile is uniform): a per-lane
  // bt[bi] was a vector load that every K / V load of the tile waited for
  const int i0 = 2 * tile < nblocks ? 2 * tile : 0, i1 = 2 * tile + 1 < nblocks ? 2 * tile + 1 : 0;
  const int blk0 = bt[__builtin_amdgcn_readfirstlane(i0)], blk1 = bt[__builtin_amdgcn_readfirstlane(i1)];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tid + 256 * i;           // 512 pieces of 16 B per operand
    // K: token = p >> 4, chunk = p & 15
    {
      const int tok = p >> 4, ch = p & 15;
      const int blk = (tok >> 4) ? blk1 : blk0;
      kreg[i] = *reinterpret_cast<const u32x4*>(k_cache + ((size_t)blk * hkv + h) * head_stride + (tok & 15) * HD + ch * 8);
    }
    // V^T: dim = p >> 2, chunk = p & 3 (chunks 0,1 from the first block, 2,3 from the second)
    {
      const int dim = p >> 2, ch = p & 3;
      const int blk = (ch >> 1) ? blk1 : blk0;
      vreg[i] = *reinterpret_cast<const u32x4*>(v_cache + ((size_t)blk * hkv + h) * head_stride + dim * KBS + (ch & 1) * 8);
    }
  }
}

__device__ __forceinline__ void prefill_store_tile(PrefillSmem& s, const u32x4 (&kreg)[2], const u32x4 (&vreg)[2]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tid + 256 * i;
    const int tok = p >> 4, ch = p & 15;
    reinterpret_cast<u32x4*>(s.k[tok])[ch ^ (tok & 15)] = kreg[i];
    const int dim = p >> 2, vc = p & 3;
    reinterpret_cast<u32x4*>(s.v[dim])[vc ^ (((dim >> 2) & 1) << 1)] = vreg[i];
  }
}

__global__ __launch_bounds__(256, 3) void paged_prefill_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ q,
                                                            const bf16_t* __restrict__ k_cache,
                                                            const bf16_t* __restrict__ v_cache,
                                                            const int* __restrict__ block_tables, int max_blocks,
                                                            const int* __restrict__ q_starts,
                                                            const int* __restrict__ ctx_lens, int hq, int hkv,
                                                            float scale_log2) {
  const int qt = blockIdx.x, h = blockIdx.y, sq = blockIdx.z;
  const int G = hq / hkv;
  const int tpt = 64 / G;  // tokens per tile
  const int q0 = q_starts[sq];
  const int qlen = q_starts[sq + 1] - q0;
  const int tile_tok0 = qt * tpt;
  if (tile_tok0 >= qlen) return;
  const int ctx = ctx_lens[sq];
  const int base_pos = ctx - qlen;
  const int last_tok = min(tile_tok0 + tpt, qlen) - 1;
  const int kv_end = base_pos + last_tok + 1;
  const int ntiles = (kv_end + 31) >> 5;
  const int nblocks = (ctx + KBS - 1) / KBS;
  const int* bt = block_tables + (size_t)sq * max_blocks;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  __shared__ PrefillSmem s;

  // Q fragments for A rows (row = wave*16 + col)
  bf16x8 qf[4];
  {
    const int row = wave * 16 + col;
    const int tok = tile_tok0 + row / G;
    const int g = row % G;
    if (tok < qlen) {
      const bf16_t* qp = q + ((size_t)(q0 + tok) * hq + h * G + g) * HD + 8 * grp;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) qf[ks] = as_bf16x8(*reinterpret_cast<const uint4*>(qp + 32 * ks));
    } else {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) qf[ks] = as_bf16x8(make_uint4(0, 0, 0, 0));
    }
  }
  // query positions of this lane's 4 C rows
  int qpos[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = wave * 16 + 4 * grp + r;
    const int tok = tile_tok0 + row / G;
    qpos[r] = tok < qlen ? base_pos + tok : kv_end - 1;
  }
  float m[4], l[4];
  f32x4 o[8];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
  }
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 kreg[2], vreg[2];
  prefill_load_tile(kreg, vreg, k_cache, v_cache, bt, nblocks, 0, h, hkv);
  bf16_t* pw = s.p[wave];
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();  // previous tile's LDS reads are done
    prefill_store_tile(s, kreg, vreg);
    __syncthreads();
    if (t + 1 < ntiles) prefill_load_tile(kreg, vreg, k_cache, v_cache, bt, nblocks, t + 1, h, hkv);
    const int t0 = t * 32;
    f32x4 sc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tok = 16 * j + col;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const uint4 kf = s.k[tok][(4 * ks + grp) ^ (tok & 15)];
        acc = mfma16x16x32(qf[ks], as_bf16x8(kf), acc);
      }
      sc[j] = acc;
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x0 = (t0 + col <= qpos[r]) ? sc[0][r] * scale_log2 : -INFINITY;
      const float x1 = (t0 + 16 + col <= qpos[r]) ? sc[1][r] * scale_log2 : -INFINITY;
      const float mx = row16_max(fmaxf(x0, x1));
      const float mn = fmaxf(m[r], mx);
      // mn == -inf only if every key so far is masked for this row (not possible for t == 0)
      alpha[r] = (mn == -INFINITY) ? 1.f : exp2f(m[r] - mn);
      const float p0 = (mn == -INFINITY) ? 0.f : exp2f(x0 - mn);
      const float p1 = (mn == -INFINITY) ? 0.f : exp2f(x1 - mn);
      l[r] = l[r] * alpha[r] + row16_sum(p0 + p1);
      m[r] = mn;
      p_store(pw, 4 * grp + r, col, p0, p1);
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[n][r] *= alpha[r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bf16x8 pf = p_load(pw, col, grp);
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int dim = n * 16 + col;
      const uint4 vf = s.v[dim][grp ^ (((dim >> 2) & 1) << 1)];   // 64-B rows: conflict-free ds_read_b128
      o[n] = mfma16x16x32(pf, as_bf16x8(vf), o[n]);
    }
  }
  // epilogue: rows 4*grp + r of this wave
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = wave * 16 + 4 * grp + r;
    const int tok = tile_tok0 + row / G;
    const int g = row % G;
    if (tok >= qlen) continue;
    const float inv = l[r] > 0.f ? 1.f / l[r] : 0.f;
    bf16_t* op = out + ((size_t)(q0 + tok) * hq + h * G + g) * HD + col;
#pragma unroll
    for (int n = 0; n < 8; ++n) op[n * 16] = f2bf(o[n][r] * inv);
  }
}

extern "C" int ka_paged_prefill(void* out, const void* q, const void* k_cache, const void* v_cache,
                                const int* block_tables, int max_blocks, const int* q_starts, const int* ctx_lens,
                                int num_seqs, int max_q_len, int hq, int hkv, int head_dim, int block_size,
                                float scale, hipStream_t stream) {
  if (num_seqs <= 0 || max_q_len <= 0) return 0;
  const int G = hkv > 0 ? hq / hkv : 0;
  if (head_dim != HD || block_size != KBS || hq % hkv != 0 || G > 64 || 64 % G != 0) return (int)hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  const int tpt = 64 / G;
  const int qtiles = (max_q_len + tpt - 1) / tpt;
  hipLaunchKernelGGL(paged_prefill_kernel, dim3(qtiles, hkv, num_seqs), dim3(256), 0, stream,
                     static_cast<bf16_t*>(out), static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k_cache),
                     static_cast<const bf16_t*>(v_cache), block_tables, max_blocks, q_starts, ctx_lens, hq, hkv,
                     scale_log2);
  KA_CHECK_LAUNCH();
}
