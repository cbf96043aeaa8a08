// Persistent small-batch decode: every decoder layer of a Llama model (TP = 1, head_dim 128, KV block 16)
// for the next token of B = 1 or 2 sequences in ONE launch (the serving path's B = 1 / 2 hipGraphs
// replay it once per step).  Each weight byte is streamed once per step whatever B is: a wave's 1-KB
// piece is dotted against the B activation rows staged in LDS.
// 2.85 ms/step for Llama-3-8B against 3.45 for the ~7-kernels-per-layer chain
// (profiles/r4/persistent_decode/README.md).
//
// One 512-thread workgroup per CU (the dynamic LDS request admits no second one).  Per layer l
// (group h = the G / hkv workgroups of KV head h; its first workgroup is the group's leader):
//   P1  every workgroup: RMSNorm of the fp32 residual -> x (LDS); its waves' QKV rows of head h ->
//       qkv (sc1 stores, row pairs packed); group arrival.  The leader then DMAs each wave's first
//       32-token chunk of this layer's cached K / V into its (idle) weight ring.
//   P2  the leader, after its group's arrivals: RoPE on q / k, attention on MFMA 16x16x32 over
//       32-token chunks (K / V from the ring; from global memory past 8 chunks), merged across
//       waves and with the new token through LDS -> attn; then the KV append
//   P3  O GEMV rows (the non-leaders' waves) -> residual +=
//   P4  RMSNorm -> x; gate + up rows -> act = silu(g) * u
//   P5  down GEMV rows (K = I) -> residual +=
// Grid barriers between the phases (B after P2, C after P3, D after P4, E after P5): arrival
// counters sharded per XCD slot (wg mod 8), each on its own 128-B line; one lane per shard polls
// with relaxed sc1 loads.  Everything that crosses workgroups is written and read with sc1 accesses
// (MI355X_MICROARCH.md hand-off table, row 1: no fences).  Spins are bounded: a workgroup that is
// never scheduled sets the error word instead of hanging the chip (the runner reads it back with
// the step's tokens and falls back to the kernel chain).
//
// Weight streaming (Stream): each wave streams its rows 1 KB per LDS-DMA instruction (nt) through a
// 16-slot LDS ring (no VGPRs held by bytes in flight), consumes two pieces per iteration against x in
// LDS with v_dot2, and refills the slots; the next phase's first 16 pieces are issued between the
// barrier arrival and the wait, so they stream while the grid synchronises.
#include "common.h"

#include <algorithm>

namespace pd {

#define KA_HD __host__ __device__ __forceinline__

#ifndef KA_PD_RING
#define KA_PD_RING 16
#endif
#ifndef KA_PD_ROT
#define KA_PD_ROT 0   // measured: no effect (profiles/r4/persistent_decode)
#endif
#ifndef KA_PD_PREISSUE    // pieces of the next phase issued before a grid barrier's wait (the rest after it);
#define KA_PD_PREISSUE 16 // (deferring all of the polling wave's pieces measured +2.5 us per barrier)
#endif
#ifndef KA_PD_NT
#define KA_PD_NT 1
#endif
// LDS-DMA wait schedule of the weight streams.  LDS-DMA pieces of one wave do not always complete in
// issue order (profiles/r5/gemm_big_clamp/), so only vmcnt(0) proves that a given piece has landed.
//   1 (default, drained halves): the ring is two halves of RING / 2 slots; a wave waits vmcnt(0) for the
//     half it is about to read, which at that moment is the only batch it has in flight (the next half
//     is issued right after the wait, then dotted against while the first is consumed).
//   0 (counted, rounds 4-5): RING - 2 pieces stay in flight across each counted wait; correct only
//     under in-order completion, kept for A/B measurements.
#ifndef KA_PD_SAFE
#define KA_PD_SAFE 1
#endif
constexpr int NT = 512, NW = NT / 64, HD = 128, KBS = 16, NT_ = NT;
// LDS-DMA ring slots (1 KB) per wave: KA_PD_RING (16) in every phase, except the down rows at B = 2,
// whose two act rows (2 x I bf16) take LDS the ring gives up there (12 slots, 96 KB per CU in flight;
// 8 slots measured 16.4 us per layer for the down rows against 13.2 at B = 1)
template <int B, int RG = KA_PD_RING>
constexpr int ring_down() { return B == 1 ? RG : (RG < 12 ? RG : 12); }
static_assert((KA_PD_RING & (KA_PD_RING - 1)) == 0 && KA_PD_RING >= 2 && KA_PD_RING <= 16, "ring: a power of two <= 16");
constexpr int MAXB = 2;     // sequences per launch
constexpr int XR_MAX_RANKS = 8, XR_MAX_WG = 256, XR_MAX_H = 16384;   // the in-kernel all-reduce's limits
// The attention leader's scratch (aliases the x rows) for GR = 4 or 8 rows per KV group (GQA <= 4 /
// <= 8): P re-layout 10 KB | rotated q GR x 128 bf16 | new k, v | per-wave m, l | new-token scores |
// GR 4: per-wave o [NW][4][128] fp32.  GR 8 writes each wave's o [8][128] (4 KB) into the wave's own
// weight ring instead, idle by then (its prefetched K / V consumed, no O rows on a leader): the 32 KB
// of a scratch o would leave the GQA-8 geometry only 12-slot rings (and one prefetched K/V block).
KA_HD int scratch_bytes(int gr) { return 10240 + gr * 256 + 1024 + 2 * 8 * gr * 4 + 64 + (gr > 4 ? 0 : 8 * gr * 128 * 4); }
constexpr int XS_MIN = 29 * 1024;   // GR = 4: 28.3 KB

struct Layer {
  const bf16_t* wqkv;   // [(hq + 2 hkv) 128, H]
  const bf16_t* wo;     // [H, hq 128]
  const bf16_t* w13;    // [2 I, H]: gate rows then up rows
  const bf16_t* w2;     // [H, I]
  const bf16_t* ln1;    // [H]
  const bf16_t* ln2;    // [H]
};

struct Args {
  const Layer* layers;
  int L, H, hq, hkv, I;
  float eps, scale_log2;
  const bf16_t* h0;     // [B][H] the tokens' embeddings
  bf16_t* h_out;        // [B][H] the residual streams after the last layer (bf16)
  bf16_t* k_cache;      // [L][NB][hkv][16][128]
  bf16_t* v_cache;      // [L][NB][hkv][128][16]
  size_t cache_layer;   // elements per layer of each cache
  const int* pos;       // [B] positions of the tokens
  const int* slot;      // [B] their cache slots
  const int* bt;        // [B][bt_stride] the sequences' block tables
  const int* ctx;       // [B] context lengths including the token
  const float* cos_sin; // [max_pos][128]
  float* res;           // workspace: [B][H] fp32 residual
  bf16_t* qkv;          // [B][(hq + 2 hkv) 128]
  bf16_t* attn;         // [B][hq 128]
  bf16_t* act;          // [B][I]
  int bt_stride;        // ints per block-table row
  int xh_bytes;         // LDS bytes per staged x / attn row of one sequence (H, hq 128 bf16)
  int xs_bytes;         // LDS bytes per staged act row (I bf16; B = 1: the larger of the two)
  int lds_ring;         // LDS byte offset of the QKV / O / gate_up weight rings (after the x rows)
  int lds_ring_d;       // ... of the down rows' rings (after the act rows)
  int lds_red;          // ... of the norm reduction (64 B), then the phases' row results (1 KB per sequence)
  int* sync;            // SYNC_BYTES: grid arrival shards, group arrivals, the error word (zeroed per launch)
  unsigned long long* stamps;   // diagnostics (nullptr: off): [G workgroups][L][16] s_memrealtime (100 MHz)
  // tensor parallelism (world > 1): the row-parallel O / down outputs are all-reduced inside the kernel
  // (see xreduce); world 0 / 1: added to the residual as they are (TP = 1, or a virtual rank whose
  // collectives are no-ops)
  int world, rank;
  float* xdata[XR_MAX_RANKS];      // every rank's exchange halves [2][MAXB][H] fp32 (IPC-mapped, uncached)
  unsigned* xflag[XR_MAX_RANKS];   // every rank's flags [XR_MAX_WG][XR_MAX_RANKS] (IPC-mapped, uncached)
  unsigned* xctr;                  // this rank's epoch counter (local; 2 L per launch)
};

KA_DEV float ld_sc1(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
KA_DEV void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
KA_DEV uint32_t ld_sc1u(const bf16_t* p) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
KA_DEV void st_sc1u(bf16_t* p, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
KA_DEV const bf16_t* uniform_ptr(const bf16_t* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const bf16_t*>((uintptr_t)(((uint64_t)hi << 32) | lo));
}

// An SGPR holding 0 (a literal 0 is not accepted as the soffset of the LDS-DMA form)
KA_DEV uint32_t sgpr_zero() {
  uint32_t z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}
// One 1-KB LDS-DMA piece: 16 B per lane from base + voff (base wave-uniform) to LDS lds_dst + 16 lane
KA_DEV void dma_1k(const bf16_t* base, uint32_t voff, uint32_t lds_dst) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(uniform_ptr(base)), (short)0,
                                                                      1 << 30, 0x00020000);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(__builtin_amdgcn_readfirstlane(lds_dst)), "v"(voff), "s"(rs), "s"(sgpr_zero())
               : "memory");
}

// Four 16-B sc1 loads in flight, one wait (hand-off table row 1 admits 16-B sc1 loads of bytes stored
// sc1 in 4-B words); the addresses must all be valid (callers clamp).  The wait also covers the
// caller's weight pieces in flight — staging runs right after a barrier, when they have landed.
KA_DEV void ld4_sc1(const uint4* p0, const uint4* p1, const uint4* p2, const uint4* p3, uint4 (&o)[4]) {
  asm volatile(
      "global_load_dwordx4 %0, %4, off sc1\n\tglobal_load_dwordx4 %1, %5, off sc1\n\t"
      "global_load_dwordx4 %2, %6, off sc1\n\tglobal_load_dwordx4 %3, %7, off sc1\n\ts_waitcnt vmcnt(0)"
      : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3])
      : "v"(p0), "v"(p1), "v"(p2), "v"(p3)
      : "memory");
}
// n16 16-B words of a handed-off activation (sc1) -> LDS, 4 loads per lane in flight
KA_DEV void stage_sc1(uint4* dst, const void* src, int n16) {
  const uint4* sp = static_cast<const uint4*>(src);
  for (int b0 = 0; b0 < n16; b0 += 4 * NT_) {
    const int i0 = b0 + (int)threadIdx.x;
    uint4 o[4];
    ld4_sc1(sp + min(i0, n16 - 1), sp + min(i0 + NT_, n16 - 1), sp + min(i0 + 2 * NT_, n16 - 1),
            sp + min(i0 + 3 * NT_, n16 - 1), o);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i0 + k * NT_ < n16) dst[i0 + k * NT_] = o[k];
  }
}

// Arrival: every wave's stores drained, a workgroup barrier, then one lane adds (MI355X_MICROARCH.md
// hand-off table, row 1: the add comes after the wait of every wave it signals for).
// vmcnt(0) expcnt(7) lgkmcnt(15) as a builtin: hipcc sees the scoreboard empty after it.  Placed where
// the wave's vector memory has drained anyway (arrivals, after handed-off loads), so that no stale
// "pending" state reaches a streaming loop, where hipcc would put an s_waitcnt vmcnt(0) — a ring
// drain — into every iteration.
KA_DEV void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }
KA_DEV void arrive(int* cnt) {
  vm_drain();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait until `*cnt >= target` (one lane polls; the others join at the workgroup barrier).  Bounded:
// ~0.5 s, or at once when another workgroup already gave up (the error word).
KA_DEV void wait_for(const int* cnt, int target, int* err) {
  if (threadIdx.x == 0) {
    int spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if ((++spins & 255) == 0 &&
          (spins > (1 << 20) || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}
// Sync words, each counter on a 128-B line of its own: the grid arrival counter in SH shards (workgroup
// wg adds to shard wg % SH: the workgroups of one XCD under round-robin placement; one unsharded
// counter serialises 256 adds at ~12 ns each, MI355X_MICROARCH.md price list, fanin / barrier-xcd),
// the KV groups' arrival counters, the error word.
constexpr int SH = 8, SYNC_BYTES = 4096, SYNC_GROUP = 256, SYNC_ERR = 1008;
KA_DEV int* grid_shard(int* sync, int wg) { return sync + 32 * (wg % SH); }
// Grid wait: lanes 0 .. SH-1 of wave 0 poll one shard each (sc1 loads: hand-off table row 1, every
// shard of a sharded counter), until every shard holds nbar x its workgroup count.
KA_DEV void wait_grid(const int* sync, int nbar, int G, int* err) {
  if (threadIdx.x < 64) {
    const int s = threadIdx.x;
    const bool mine = s < SH && s < G;
    const int target = mine ? nbar * ((G - s + SH - 1) / SH) : 0;
    int spins = 0;
    while (true) {
      const bool ok = !mine || __hip_atomic_load(sync + 32 * s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(2);
      if ((++spins & 255) == 0 &&
          (spins > (1 << 20) || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        if (s == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

KA_DEV uint4 ld_w(const bf16_t* p) {
  return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
}

typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
KA_DEV float dot8(uint4 w, uint4 x, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, w.x), __builtin_bit_cast(bf16x2v, x.x), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, w.y), __builtin_bit_cast(bf16x2v, x.y), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, w.z), __builtin_bit_cast(bf16x2v, x.z), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, w.w), __builtin_bit_cast(bf16x2v, x.w), acc, false);
  return acc;
}

// P re-layout scratch of the leader's MFMA attention (the scheme of csrc/attention.hip): the
// probabilities leave the MFMA C layout (lane (col, g) holds rows 4 g + r, keys col and 16 + col) and
// are re-read in the A layout (lane holds row col, keys 8 g .. 8 g + 7); 16 rows x PSTR bf16 per wave,
// 16-B chunk c of row x at slot c ^ p_slot_xor(x >> 2): conflict-free stores and reads.
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
KA_DEV bf16x8 p_load(const bf16_t* pw, int col, int g) {
  return as_bf16x8(*reinterpret_cast<const uint4*>(pw + col * PSTR + ((g ^ p_slot_xor((col >> 2) & 3)) << 3)));
}

// Sum over the 64 lanes as a wave-uniform value: the 16-lane rows by DPP, the four row sums by
// v_readlane (no LDS round trip, unlike __shfl_xor's ds_bpermute)
KA_DEV float wave_total(float v) {
  v = row16_sum(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0)) +
         __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16)) +
         __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32)) +
         __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
}

// One wave's weight stream over `n` rows of length K (row(i) -> global row index): 1 KB per load
// instruction (64 lanes x 16 B along K) by LDS-DMA (`buffer_load_dwordx4 ... lds`) into the wave's own
// RING-slot LDS ring, so the bytes in flight cost no VGPRs (a register ring of the same depth spilled).
// start() issues the first RING pieces (before the wait for the activations); run() takes the pieces
// two at a time: waits for them (a static vmcnt: exactly RING pieces are always outstanding, the tail
// re-reads the last chunk), reads both and their x chunks back from LDS under one lgkmcnt wait,
// refills the two slots and dots.  Row results stay in registers (lane i holds row i: no store may sit
// between the counted loads) and are returned by run(); the caller writes them after drain().
// Every instruction between the counted loads is asm or VALU / SALU: a compiler-visible vector-memory
// access there would get an s_waitcnt vmcnt(0) from hipcc — a drain of the whole ring.
// Row results of a stream: v[b] = the row's dot product with activation row b (lane i holds row i)
template <int B>
struct RowVals {
  float v[B];
};

template <int B, int RG, class RowFn>
struct Stream {
  static_assert(RG >= 2 && RG <= 16 && RG % 2 == 0, "ring slots: even, <= 16 (RG - 2 pieces in flight per wait)");
  const bf16_t* W;
  int K, KC, total, lane;
  RowFn row;
  uint32_t nbytes;
  uint32_t ring;   // LDS byte address of this wave's ring (wave-uniform)
  int issued, ni, nc;   // pieces issued; row / chunk of the next piece to issue
  int rot;              // every row is read from chunk `rot` on, wrapping (see make_stream)
  KA_DEV void issue() {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(ring + ((uint32_t)issued % (uint32_t)RG) * 1024u);
    // wave-uniform part of the byte offset (row start + chunk) -> soffset; the lane's 16 B -> voffset
    const int c = nc + rot >= KC ? nc + rot - KC : nc + rot;
    const uint32_t so = __builtin_amdgcn_readfirstlane(((uint32_t)row(ni) * (uint32_t)K + (uint32_t)(c * 512)) * 2u);
    const uint32_t off = (uint32_t)lane * 16u;
    // W is wave-uniform (uniform_ptr at the layer's top): the descriptor lives in SGPRs
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(W), (short)0,
                                                                        (int)nbytes, 0x00020000);
    uint32_t keep;
    // nt: weights are read once per token (MI355X_MICROARCH.md nt-weights: issued -> landed -18 %)
#if KA_PD_NT
#define KA_PD_LDS_LOAD "buffer_load_dwordx4 %2, %3, %4 offen nt lds"
#else
#define KA_PD_LDS_LOAD "buffer_load_dwordx4 %2, %3, %4 offen lds"
#endif
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t" KA_PD_LDS_LOAD "\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(dst), "v"(off), "s"(rs), "s"(so)
                 : "memory");
    if (++issued < total && ++nc == KC) {   // past the end: the last piece again (keeps the count static)
      nc = 0;
      ++ni;
    }
  }
  static constexpr int HB = RG / 2;   // drained schedule: slots per half (one batch)
  // the first N pieces (N < RG: the rest by top_up<N>() after the barrier wait, so the wait's polls
  // queue behind fewer of the CU's own pieces).  Drained schedule: the first batch (half the ring)
  template <int N = RG>
  KA_DEV void start() {
    issued = ni = nc = 0;
    if (total <= 0) return;
#if KA_PD_SAFE
    for (int r = 0; r < min(HB, total); ++r) issue();
#else
#pragma unroll
    for (int r = 0; r < (N < RG ? N : RG); ++r) issue();
#endif
  }
  template <int N>
  KA_DEV void top_up() {
#if !KA_PD_SAFE
    if (total <= 0) return;
#pragma unroll
    for (int r = (N < RG ? N : RG); r < RG; ++r) issue();
#endif
  }
  // xaddr: LDS byte address of activation row 0 (K bf16), row b at xaddr + b xstride
  KA_DEV RowVals<B> run(uint32_t xaddr, uint32_t xstride) {
    RowVals<B> mine;
#pragma unroll
    for (int b = 0; b < B; ++b) mine.v[b] = 0.f;
    if (total <= 0) return mine;
    float acc[B];
#pragma unroll
    for (int b = 0; b < B; ++b) acc[b] = 0.f;
    int cc = 0, ri = 0;
    const uint32_t lo16 = (uint32_t)lane * 16u;
    auto finish = [&]() {
      if (++cc == KC) {
        cc = 0;
#pragma unroll
        for (int b = 0; b < B; ++b) {
          const float v = wave_total(acc[b]);
          if (lane == ri) mine.v[b] = v;
          acc[b] = 0.f;
        }
        ++ri;
      }
    };
    int j = 0;
#if KA_PD_SAFE
    // batches of HB pieces in alternating halves: wait for batch [j, j + n) (the only pieces in flight),
    // issue the next batch into the other half (read by the batch before, whose reads have completed),
    // then read and dot this one, two pieces at a time
    while (j < total) {
      const int n = min(HB, total - j);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int r = min(HB, total - j - n); r > 0; --r) issue();
      const int je = j + n;
      for (; j + 1 < je; j += 2) {
#else
    for (; j + 1 < total; j += 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RG - 2) : "memory");   // pieces j, j + 1 have landed
#endif
      const int xc = cc + rot >= KC ? cc + rot - KC : cc + rot;   // x chunks of pieces j, j + 1
      const int xc1 = xc + 1 == KC ? 0 : xc + 1;
      const uint32_t r0 = ring + ((uint32_t)j % (uint32_t)RG) * 1024u + lo16, r1 = ring + ((uint32_t)(j + 1) % (uint32_t)RG) * 1024u + lo16;
      const uint32_t a0 = xaddr + (uint32_t)xc * 1024u + lo16, a1 = xaddr + (uint32_t)xc1 * 1024u + lo16;
      uint4 w0, w1, x0[B], x1[B];
      if constexpr (B == 1) {
        asm volatile(
            "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(w0), "=&v"(w1), "=&v"(x0[0]), "=&v"(x1[0])
            : "v"(r0), "v"(r1), "v"(a0), "v"(a1)
            : "memory");
      } else {
        static_assert(B == 2, "rows per launch");
        asm volatile(
            "ds_read_b128 %0, %6\n\tds_read_b128 %1, %7\n\tds_read_b128 %2, %8\n\tds_read_b128 %3, %9\n\t"
            "ds_read_b128 %4, %10\n\tds_read_b128 %5, %11\n\ts_waitcnt lgkmcnt(0)"
            : "=&v"(w0), "=&v"(w1), "=&v"(x0[0]), "=&v"(x1[0]), "=&v"(x0[1]), "=&v"(x1[1])
            : "v"(r0), "v"(r1), "v"(a0), "v"(a1), "v"(a0 + xstride), "v"(a1 + xstride)
            : "memory");
      }
#if !KA_PD_SAFE
      issue();   // both slots are free again: refill them RG pieces ahead
      issue();
#endif
#pragma unroll
      for (int b = 0; b < B; ++b) acc[b] = dot8(w0, x0[b], acc[b]);
      finish();
#pragma unroll
      for (int b = 0; b < B; ++b) acc[b] = dot8(w1, x1[b], acc[b]);
      finish();
    }
#if KA_PD_SAFE
    if (j < je) {   // an odd batch: its last piece
#else
    if (j < total) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RG - 1) : "memory");
#endif
      const uint32_t r0 = ring + ((uint32_t)j % (uint32_t)RG) * 1024u + lo16;
      const uint32_t a0 = xaddr + (uint32_t)(cc + rot >= KC ? cc + rot - KC : cc + rot) * 1024u + lo16;
      uint4 w0, x0[B];
      if constexpr (B == 1) {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(w0), "=&v"(x0[0])
                     : "v"(r0), "v"(a0)
                     : "memory");
      } else {
        asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b128 %2, %5\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(w0), "=&v"(x0[0]), "=&v"(x0[1])
                     : "v"(r0), "v"(a0), "v"(a0 + xstride)
                     : "memory");
      }
#if !KA_PD_SAFE
      issue();
#endif
#pragma unroll
      for (int b = 0; b < B; ++b) acc[b] = dot8(w0, x0[b], acc[b]);
      finish();
#if KA_PD_SAFE
      ++j;
#endif
    }
#if KA_PD_SAFE
    }
#endif
    return mine;
  }
  KA_DEV void drain() const { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
};
// gw: the wave's grid-wide index.  Each wave starts its rows at chunk gw mod K/512: waves that leave
// a grid barrier together would otherwise all read the same 1-KB column of their rows at once —
// addresses equal modulo the row pitch, the same few HBM channels.
template <int B, int RG, class RowFn>
KA_DEV Stream<B, RG, RowFn> make_stream(const bf16_t* W, int N, int K, int n, int lane, uint32_t ring, RowFn row, int gw) {
  Stream<B, RG, RowFn> s{W, K, K / 512, n * (K / 512), lane, row, (uint32_t)N * (uint32_t)K * 2u, ring, 0, 0, 0,
                         KA_PD_ROT ? gw % (K / 512) : 0};
  return s;
}

// x[i] = bf16(res[i] * rstd * g[i]) into LDS (every workgroup): the fp32 residual read once by 16-B
// sc1 loads (H / 4 words, <= 8 per lane at H <= 16384) and held in registers for the scaling pass
KA_DEV void rmsnorm_to_lds(const Args& a, const float* res, const bf16_t* g, bf16_t* xs, float* red) {
  const int H = a.H, n16 = H / 4;
  const uint4* rp = reinterpret_cast<const uint4*>(res);
  uint4 rv[8];
  ld4_sc1(rp + min((int)threadIdx.x, n16 - 1), rp + min((int)threadIdx.x + NT, n16 - 1),
          rp + min((int)threadIdx.x + 2 * NT, n16 - 1), rp + min((int)threadIdx.x + 3 * NT, n16 - 1),
          *reinterpret_cast<uint4(*)[4]>(&rv[0]));
  if (n16 > 4 * NT)
    ld4_sc1(rp + min((int)threadIdx.x + 4 * NT, n16 - 1), rp + min((int)threadIdx.x + 5 * NT, n16 - 1),
            rp + min((int)threadIdx.x + 6 * NT, n16 - 1), rp + min((int)threadIdx.x + 7 * NT, n16 - 1),
            *reinterpret_cast<uint4(*)[4]>(&rv[4]));
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if ((int)threadIdx.x + k * NT < n16) {
      const float4 f = __builtin_bit_cast(float4, rv[k]);
      ss += f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
    }
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) tot += red[w];
  const float rstd = rsqrtf(tot / (float)H + a.eps);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int i = (int)threadIdx.x + k * NT;
    if (i < n16) {
      const float4 f = __builtin_bit_cast(float4, rv[k]);
      const uint2 gw = *reinterpret_cast<const uint2*>(g + 4 * i);
      uint2 o;
      o.x = pack2(f.x * rstd * lo_f(gw.x), f.y * rstd * hi_f(gw.x));
      o.y = pack2(f.z * rstd * lo_f(gw.y), f.w * rstd * hi_f(gw.y));
      *reinterpret_cast<uint2*>(xs + 4 * i) = o;
    }
  }
  __syncthreads();
}

// x_b = bf16(res_b * rstd_b * g) for the B rows at once (B = 2, H <= 8192): every row's residual loaded
// before one reduction of the B sums of squares (one workgroup barrier instead of B)
template <int B>
KA_DEV void rmsnorm_rows_to_lds(const Args& a, const float* res, const bf16_t* g, bf16_t* xs, int xstride, float* red) {
  if constexpr (B == 1) {
    rmsnorm_to_lds(a, res, g, xs, red);
  } else {
    const int H = a.H, n16 = H / 4;   // <= 4 NT (ka_decode_persistent_max_b)
    uint4 rv[B][4];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const uint4* rp = reinterpret_cast<const uint4*>(res + (size_t)b * H);
      ld4_sc1(rp + min((int)threadIdx.x, n16 - 1), rp + min((int)threadIdx.x + NT, n16 - 1),
              rp + min((int)threadIdx.x + 2 * NT, n16 - 1), rp + min((int)threadIdx.x + 3 * NT, n16 - 1), rv[b]);
    }
    float ss[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      ss[b] = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if ((int)threadIdx.x + k * NT < n16) {
          const float4 f = __builtin_bit_cast(float4, rv[b][k]);
          ss[b] += f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
        }
      }
      ss[b] = wave_sum(ss[b]);
      if ((threadIdx.x & 63) == 0) red[b * NW + (threadIdx.x >> 6)] = ss[b];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < B; ++b) {
      float tot = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) tot += red[b * NW + w];
      const float rstd = rsqrtf(tot / (float)H + a.eps);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = (int)threadIdx.x + k * NT;
        if (i < n16) {
          const float4 f = __builtin_bit_cast(float4, rv[b][k]);
          const uint2 gw = *reinterpret_cast<const uint2*>(g + 4 * i);
          uint2 o;
          o.x = pack2(f.x * rstd * lo_f(gw.x), f.y * rstd * hi_f(gw.x));
          o.y = pack2(f.z * rstd * lo_f(gw.y), f.w * rstd * hi_f(gw.y));
          *reinterpret_cast<uint2*>(xs + (size_t)b * xstride + 4 * i) = o;
        }
      }
    }
    __syncthreads();
  }
}

// In-kernel all-reduce of a row-parallel projection (tensor parallelism; MI355X_MICROARCH.md hand-off
// table, system scope).  Every rank splits the output rows over its workgroups the same way, so
// workgroup wg of every rank owns the same rows: it publishes its partial rows into half e & 1 of its
// own exchange buffer (uncached, IPC-mapped), releases at system scope, stores epoch e into flag
// [wg][rank] of every peer, waits until its own flags [wg][p] reach e (bounded: the error word instead
// of a hang), then sums the peers' rows in rank order.  Alternating halves: a rank rewrites half h at
// epoch e + 2 only after every peer's workgroup wg signalled e + 1, i.e. finished reading e.
// v[b] = this lane's partial of row `row` (valid when `mine`); returns the sum over ranks.
template <int B, int RG>
KA_DEV void xreduce(const Args& a, unsigned epoch, int wg, int row, bool mine, float (&v)[B], int* err) {
  const size_t hb = (size_t)MAXB * a.H, half = (size_t)(epoch & 1u) * hb;
  if (mine) {
#pragma unroll
    for (int b = 0; b < B; ++b)
      __hip_atomic_store(a.xdata[a.rank] + half + (size_t)b * a.H + row, v[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < a.world) {
    const int p = threadIdx.x;
    __hip_atomic_store(a.xflag[p] + wg * XR_MAX_RANKS + a.rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* f = a.xflag[a.rank] + wg * XR_MAX_RANKS + p;
    int spins = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if ((++spins & 255) == 0 &&
          (spins > (1 << 22) || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // 2: a peer rank never came
        break;
      }
    }
  }
  __syncthreads();
  if (mine) {
    // the peers' rows are loaded XB at a time, each batch before its first add (2 remote round
    // trips at TP = 8 instead of 8; a batch of 8 spills at this kernel's 256-VGPR budget, and so does
    // a batch of 4 in the B = 2 / 16-slot instantiation, which keeps one peer per round trip);
    // summed in rank order
    constexpr int XB = (B == 2 && RG == 16) ? 1 : 4;
#pragma unroll
    for (int b = 0; b < B; ++b) {
      float sum = 0.f;
      for (int p0 = 0; p0 < a.world; p0 += XB) {
        float pv[XB];
#pragma unroll
        for (int p = 0; p < XB; ++p)
          if (p0 + p < a.world)
            pv[p] = __hip_atomic_load(a.xdata[p0 + p] + half + (size_t)b * a.H + row, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
        for (int p = 0; p < XB; ++p)
          if (p0 + p < a.world) sum += pv[p];
      }
      v[b] = sum;
    }
  }
}

// LDS layout (bytes), phase by phase (each region is dead when the next phase's DMA reaches it):
//   QKV / O / gate_up: the B x / attn rows (a.xh_bytes each) at 0 (the attention leader's scratch,
//     28.3 KB, reuses it: x is dead between the QKV rows and the O rows); the waves' 16-slot weight
//     rings at a.lds_ring;
//   down: the B act rows (a.xs_bytes each) at 0; the waves' ring_down<B>-slot rings at a.lds_ring_d;
// then the norm reduction and the phases' bf16 row results (1 KB per sequence) at a.lds_red, past both.
// > 80 KB: one workgroup per CU.
constexpr int LDS_X = 0, LDS_ATT = 0;

// RG: weight-ring slots per wave (16; 14 for B = 2 of the 70B tensor-parallel rank, hq / hkv = 8, whose
// 16-KB x rows take the LDS; pd_ring)
template <int B, int RG>
__global__ __launch_bounds__(NT, 1) void decode_layers_kernel(Args a) {
  constexpr int RGD = ring_down<B, RG>();
  extern __shared__ __attribute__((aligned(16))) uint4 lds_u4[];
  char* const lds = reinterpret_cast<char*>(lds_u4);
  bf16_t* const xs = reinterpret_cast<bf16_t*>(lds + LDS_X);
  const int lds_ring = a.lds_ring, xsb = a.xs_bytes, xhb = a.xh_bytes;
  float* const red = reinterpret_cast<float*>(lds + a.lds_red);
  bf16_t* const ob = reinterpret_cast<bf16_t*>(lds + a.lds_red + 64);   // [B][512]
  // this wave's LDS-DMA weight rings (LDS byte addresses; dynamic LDS is the kernel's only LDS object)
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)lds_u4;
  const uint32_t xaddr = __builtin_amdgcn_readfirstlane(lds_base + LDS_X);
  const uint32_t ring = __builtin_amdgcn_readfirstlane(lds_base + lds_ring + (threadIdx.x >> 6) * RG * 1024);
  const uint32_t ring_d = __builtin_amdgcn_readfirstlane(lds_base + a.lds_ring_d + (threadIdx.x >> 6) * RGD * 1024);
  const int G = gridDim.x, wg = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gw = wg * NW + wave, nwaves = G * NW;
  const int H = a.H, hq = a.hq, hkv = a.hkv, I = a.I, Gq = hq / hkv;
  const int per_group = G / hkv, grp = wg / per_group, in_grp = wg - grp * per_group;
  const int QKVN = (hq + 2 * hkv) * HD;
  // the group's first B workgroups are its attention leaders, workgroup b for sequence b
  const bool leader = in_grp < B;
  const int lb = leader ? in_grp : 0;
  const int qkv_rows = (Gq + 2) * HD;                       // rows of one KV head's group
  const int qkv_per_wave = (qkv_rows + per_group * NW - 1) / (per_group * NW);
  const int h_per_wave = (H + nwaves - 1) / nwaves;         // O / down rows = owned residual elements
  const int i_per_wave = (I + nwaves - 1) / nwaves;         // gate (and up) rows
  int* const gcnt = grid_shard(a.sync, wg);
  int* const err = a.sync + SYNC_ERR;
  int nbar = 0;   // grid barriers passed
  const bool tp = a.world > 1;
  // the all-reduce epochs of this launch: base + 1 .. base + 2 L (the counter moves on at the end)
  const unsigned ebase = tp ? __builtin_amdgcn_readfirstlane(__hip_atomic_load(a.xctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : 0u;

  // residual := the embedding (each wave initialises the elements it owns)
  const int own0 = gw * h_per_wave, own1 = min(H, own0 + h_per_wave);
  // a leader's sequence: position / slot / context (fixed for the launch) and the attention loop's trip count
  const int p = a.pos[lb], slot = a.slot[lb], ctx = a.ctx[lb];
  const int* const bt = a.bt + (size_t)lb * a.bt_stride;
  const int ncached = ctx - 1, nblk = (ncached + KBS - 1) / KBS;
  // a leader wave's first 32-token chunk: context blocks 2 w, 2 w + 1 (fixed for the launch; the first
  // PJ of them prefetched into the idle ring every layer; a missing second block repeats the first:
  // finite values, weight 0)
  constexpr int PJ = RG >= 16 ? 2 : RG >= 8 ? 1 : 0;   // 8 KB (K + V of 16 tokens) per block
  const int blk_w0 = __builtin_amdgcn_readfirstlane(2 * wave < nblk ? bt[2 * wave] : 0);
  const int blk_w1 = __builtin_amdgcn_readfirstlane(2 * wave + 1 < nblk ? bt[2 * wave + 1] : blk_w0);
#pragma unroll
  for (int b = 0; b < B; ++b)
    for (int r = own0 + lane; r < own1; r += 64) st_sc1(a.res + (size_t)b * H + r, bf2f(a.h0[(size_t)b * H + r]));
  arrive(gcnt);

  const int qv0 = (in_grp * NW + wave) * qkv_per_wave;
  const int nq = max(0, min(qkv_rows, qv0 + qkv_per_wave) - qv0);
  auto qkv_grow = [=](int r) {   // group-local row -> row of wqkv (q heads of the group, its k, its v)
    return r < Gq * HD ? grp * Gq * HD + r : r < (Gq + 1) * HD ? hq * HD + grp * HD + (r - Gq * HD)
                                                            : (hq + hkv) * HD + grp * HD + (r - (Gq + 1) * HD);
  };
  auto qkv_row = [=](int i) { return qkv_grow(qv0 + i); };
  // the workgroup's group-local QKV rows and act elements: even starts and counts, so their bf16 results
  // leave in 4-B sc1 stores of row pairs (every segment boundary of qkv_grow is even too)
  const int wq0 = in_grp * NW * qkv_per_wave, wqn = max(0, min(qkv_rows, wq0 + NW * qkv_per_wave) - wq0);
  const int wa0 = wg * NW * i_per_wave, wan = max(0, min(I, wa0 + NW * i_per_wave) - wa0);
  const int no = max(0, own1 - own0);
  auto own_row = [=](int i) { return own0 + i; };
  // O rows go to the workgroups that run no attention only: a leader's context loads would otherwise
  // queue behind its own O weight pieces (issued before the attention).  O's residual element != its
  // down owner is fine: each phase has one writer per element and a barrier after it.
  const int o_per_wave = (H + (G - B * hkv) * NW - 1) / ((G - B * hkv) * NW);
  const int ow0 = leader ? 0 : ((grp * (per_group - B) + in_grp - B) * NW + wave) * o_per_wave;
  const int n_o = leader ? 0 : max(0, min(H, ow0 + o_per_wave) - ow0);
  auto o_row = [=](int i) { return ow0 + i; };
  const int g0 = gw * i_per_wave, ng = max(0, min(I, g0 + i_per_wave) - g0);
  auto gu_row = [=](int i) { return (i & 1) ? I + g0 + (i >> 1) : g0 + (i >> 1); };   // gate, up, gate, ...

  // phase stamps of every workgroup (diagnostics)
  unsigned long long* const st = (a.stamps != nullptr && tid == 0) ? a.stamps + (size_t)wg * a.L * 16 : nullptr;
#define PD_STAMP(k) \
  do {              \
    if (st) st[l * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  for (int l = 0; l < a.L; ++l) {
    // the layer's pointers made wave-uniform (SGPRs) here, once: left in the VGPRs of their vector
    // load, hipcc's wait insertion put an s_waitcnt vmcnt(0) — a drain of the whole weight ring — into
    // every streaming-loop iteration that used them
    Layer Lw = a.layers[l];
    Lw.wqkv = uniform_ptr(Lw.wqkv);
    Lw.wo = uniform_ptr(Lw.wo);
    Lw.w13 = uniform_ptr(Lw.w13);
    Lw.w2 = uniform_ptr(Lw.w2);
    Lw.ln1 = uniform_ptr(Lw.ln1);
    Lw.ln2 = uniform_ptr(Lw.ln2);
    // ---- P1: norm + QKV rows of the group ----
    // The weight pieces of each phase are issued between the arrival and the wait of the barrier before
    // it: after the arrival (its vmcnt(0) would otherwise hold the arrival back until they landed),
    // in flight while the workgroup waits for the others.
    auto sq = make_stream<B, RG>(Lw.wqkv, QKVN, H, nq, lane, ring, qkv_row, gw);
    sq.template start<KA_PD_PREISSUE>();
    wait_grid(a.sync, ++nbar, G, err);
    sq.template top_up<KA_PD_PREISSUE>();
    PD_STAMP(0);
    if (st && l > 0) st[(l - 1) * 16 + 12] = st[l * 16];   // the previous layer's barrier E ends here
    rmsnorm_rows_to_lds<B>(a, a.res, Lw.ln1, xs, xhb / 2, red);
    PD_STAMP(1);
    {
      const RowVals<B> v = sq.run(xaddr, (uint32_t)xhb);
      sq.drain();
#pragma unroll
      for (int b = 0; b < B; ++b)
        if (lane < nq) ob[b * 512 + wave * qkv_per_wave + lane] = f2bf(v.v[b]);
      __syncthreads();
#pragma unroll
      for (int b = 0; b < B; ++b)
        if (2 * tid < wqn)
          st_sc1u(a.qkv + (size_t)b * QKVN + qkv_grow(wq0 + 2 * tid), reinterpret_cast<const uint32_t*>(ob)[b * 256 + tid]);
    }
    // the O rows' weights are issued now: they stream while the group waits and attention runs
    PD_STAMP(2);
    auto so = make_stream<B, RG>(Lw.wo, H, hq * HD, n_o, lane, ring, o_row, gw);
    arrive(a.sync + SYNC_GROUP + 32 * grp);   // this workgroup's QKV rows are published
    so.start();
    if (leader) {
      // the leader (no O rows: its ring is idle now): each wave's first 32-token chunk of this layer's
      // cached K / V (blocks 2 w, 2 w + 1) into its ring by LDS-DMA, in flight while the group's QKV
      // rows finish.  K rows land XOR-swizzled (16-B chunk c16 of token t at slot c16 ^ t: the MFMA
      // operand reads of 16 tokens hit distinct banks); V [128][16 tokens] as is.
      const size_t hs = (size_t)KBS * HD;
      if (2 * wave < nblk) {
        const int tk = lane >> 4, sl = lane & 15;   // token within a 1-KB piece, slot of the lane
#pragma unroll
        for (int j = 0; j < PJ; ++j) {
          const size_t boff = ((size_t)(j ? blk_w1 : blk_w0) * hkv + grp) * hs + (size_t)l * a.cache_layer;
#pragma unroll
          for (int pc = 0; pc < 4; ++pc) {
            const int t = 4 * pc + tk;
            dma_1k(a.k_cache + boff, (uint32_t)(t * 256 + ((sl ^ t) << 4)), ring + (uint32_t)(j * 8 + pc) * 1024u);
            dma_1k(a.v_cache + boff, (uint32_t)pc * 1024u + (uint32_t)lane * 16u, ring + (uint32_t)(j * 8 + 4 + pc) * 1024u);
          }
        }
      }
    }
    if (leader) {
      // ---- P2: the group's attention for sequence lb (its leader workgroup lb) ----
      wait_for(a.sync + SYNC_GROUP + 32 * grp, (l + 1) * per_group, err);
      PD_STAMP(3);
      // scratch (LDS_ATT): per-wave P re-layout | rotated q (bf16) | new k, v (fp32) | per-wave m, l |
      // new-token scores | per-wave o of the group's q rows
      // (GR = 4 or 8 rows per KV group: scratch_bytes)
      const int GR = Gq > 4 ? 8 : 4;
      bf16_t* const pscr = reinterpret_cast<bf16_t*>(lds + LDS_ATT);             // [NW][16 PSTR]
      bf16_t* const qb = reinterpret_cast<bf16_t*>(lds + LDS_ATT + 10240);       // [GR][128]
      float* const kn = reinterpret_cast<float*>(lds + LDS_ATT + 10240 + GR * 256);   // [128]
      float* const vn = kn + HD;                                                  // [128]
      float* const mo = vn + HD;                                                  // [NW][GR]
      float* const lo = mo + NW * GR;                                             // [NW][GR]
      float* const snr = lo + NW * GR;                                            // [GR] (+ pad)
      float* const oo = snr + 16;                                                 // [NW][4][128] (GR 4)
      // wave w's o rows [GR][128]: the scratch (GR 4) or the wave's idle ring (GR 8, see scratch_bytes)
      auto oo_of = [&](int w) -> float* {
        return GR > 4 ? reinterpret_cast<float*>(lds + lds_ring + w * RG * 1024) : oo + w * GR * HD;
      };
      const float* cs = a.cos_sin + (size_t)p * HD;
      // RoPE (neox halves) on the group's q heads and k; v as is
      for (int it = tid; it < (Gq + 2) * (HD / 2); it += NT) {
        const int hh = it / (HD / 2), i = it - hh * (HD / 2);
        const int base = hh < Gq ? (grp * Gq + hh) * HD : hh == Gq ? (hq + grp) * HD : (hq + hkv + grp) * HD;
        const bf16_t* const qs = a.qkv + (size_t)lb * QKVN;
        const uint32_t w0 = ld_sc1u(qs + base + (i & ~1)), w1 = ld_sc1u(qs + base + HD / 2 + (i & ~1));
        const float x1 = (i & 1) ? hi_f(w0) : lo_f(w0), x2 = (i & 1) ? hi_f(w1) : lo_f(w1);
        if (hh <= Gq) {
          const float c = cs[i], s = cs[HD / 2 + i];
          // bf16 rounding of the rotated values, as the cache / the unfused kernels hold them
          const bf16_t r1 = f2bf(x1 * c - x2 * s), r2 = f2bf(x2 * c + x1 * s);
          if (hh < Gq) {
            qb[hh * HD + i] = r1;
            qb[hh * HD + HD / 2 + i] = r2;
          } else {
            kn[i] = bf2f(r1);
            kn[HD / 2 + i] = bf2f(r2);
          }
        } else {
          vn[i] = x1;
          vn[HD / 2 + i] = x2;
        }
      }
      __syncthreads();
      bf16_t* const kc = a.k_cache + (size_t)l * a.cache_layer;
      bf16_t* const vc = a.v_cache + (size_t)l * a.cache_layer;
      const size_t hs = (size_t)KBS * HD;   // elements per (block, head)
      // the ring's K / V have landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      PD_STAMP(13);
      // cached tokens [0, ctx - 1) in 32-token chunks, chunk c on wave c mod NW, on MFMA 16x16x32
      // (the layouts of csrc/attention.hip's paged_decode_kernel): S = Q K^T with the group's q heads
      // as rows (zero rows past Gq), online softmax, O += P V.  Lane (col, gq) = (lane & 15, lane >> 4).
      const int col = lane & 15, gq = lane >> 4;
      bf16x8 qfr[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        qfr[ks] = as_bf16x8(col < Gq ? *reinterpret_cast<const uint4*>(qb + col * HD + 32 * ks + 8 * gq)
                                     : make_uint4(0, 0, 0, 0));
      float m[4], lsum[4];
      f32x4 o[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        m[r] = -INFINITY;
        lsum[r] = 0.f;
      }
#pragma unroll
      for (int n = 0; n < 8; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      bf16_t* const pw = pscr + wave * 16 * PSTR;
      const char* const rb = lds + lds_ring + wave * RG * 1024;   // the wave's first chunk (ring)
      const int nch = (ncached + 31) / 32;
      for (int c = wave; c < nch; c += NW) {
        const int t0 = c * 32;
        const bool first = c == wave;   // its first PJ blocks are in the ring
        int blk0 = 0, blk1 = 0;
        if (!first || PJ < 2) {
          blk0 = first ? blk_w0 : bt[2 * c];
          blk1 = first ? blk_w1 : t0 + 16 < ncached ? bt[2 * c + 1] : blk0;
        }
        f32x4 sc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bool in_ring = first && j < PJ;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            uint4 kf;
            if (in_ring)   // swizzled rows: 16-B chunk c16 of token t at (c16 ^ t)
              kf = *reinterpret_cast<const uint4*>(rb + j * 8192 + col * 256 + (((4 * ks + gq) ^ col) << 4));
            else
              kf = *reinterpret_cast<const uint4*>(kc + ((size_t)(j ? blk1 : blk0) * hkv + grp) * hs + col * HD +
                                                   8 * gq + 32 * ks);
            acc = mfma16x16x32(qfr[ks], as_bf16x8(kf), acc);
          }
          sc[j] = acc;
        }
        if (c == wave) PD_STAMP(15);   // the first chunk's scores
        uint4 vf[8];
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          if (first && (gq >> 1) < PJ)   // lanes gq >> 1 read block gq >> 1 of the chunk
            vf[n] = *reinterpret_cast<const uint4*>(rb + (gq >> 1) * 8192 + 4096 + (n * 16 + col) * 32 + (gq & 1) * 16);
          else
            vf[n] = *reinterpret_cast<const uint4*>(vc + ((size_t)((gq >> 1) ? blk1 : blk0) * hkv + grp) * hs +
                                                    (n * 16 + col) * KBS + 8 * (gq & 1));
        }
        float alpha[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x0 = t0 + col < ncached ? sc[0][r] * a.scale_log2 : -INFINITY;
          const float x1 = t0 + 16 + col < ncached ? sc[1][r] * a.scale_log2 : -INFINITY;
          const float mn = fmaxf(m[r], row16_max(fmaxf(x0, x1)));
          alpha[r] = exp2f(m[r] - mn);
          const float p0 = exp2f(x0 - mn), p1 = exp2f(x1 - mn);
          lsum[r] = lsum[r] * alpha[r] + row16_sum(p0 + p1);
          m[r] = mn;
          p_store(pw, 4 * gq + r, col, p0, p1);
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[n][r] *= alpha[r];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const bf16x8 pf = p_load(pw, col, gq);
#pragma unroll
        for (int n = 0; n < 8; ++n) o[n] = mfma16x16x32(pf, as_bf16x8(vf[n]), o[n]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // P scratch read before the next chunk's writes
      }
      // per-wave (m, l, o) of rows 0 .. Gq - 1 (lanes gq hold rows 4 gq + r) -> LDS
      if (4 * gq < Gq) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 4 * gq + r;
          if (row < Gq) {
            if (col == 0) {
              mo[wave * GR + row] = m[r];
              lo[wave * GR + row] = lsum[r];
            }
#pragma unroll
            for (int n = 0; n < 8; ++n) oo_of(wave)[row * HD + n * 16 + col] = o[n][r];
          }
        }
      }
      if (wave < Gq) {   // the new token's score of q head `wave`
        const float v = wave_total(bf2f(qb[wave * HD + 2 * lane]) * kn[2 * lane] +
                                   bf2f(qb[wave * HD + 2 * lane + 1]) * kn[2 * lane + 1]);
        if (lane == 0) snr[wave] = v * a.scale_log2;
      }
      __syncthreads();
      PD_STAMP(14);
      // merge the waves and the new token: thread -> (row, dim)
      for (int it = tid; it < Gq * HD; it += NT) {
        const int r = it / HD, d = it - r * HD;
        const float sn = snr[r];
        float M = sn;
        for (int w = 0; w < NW; ++w) M = fmaxf(M, mo[w * GR + r]);
        float den = exp2f(sn - M), num = den * vn[d];
        for (int w = 0; w < NW; ++w) {
          const float mw = mo[w * GR + r];
          if (mw == -INFINITY) continue;
          const float e = exp2f(mw - M);
          den += e * lo[w * GR + r];
          num += e * oo_of(w)[r * HD + d];
        }
        const float o1 = num / den;
        const float o2 = __shfl_xor(o1, 1, 64);   // d and d ^ 1 are neighbouring lanes
        if ((d & 1) == 0)
          st_sc1u(a.attn + (size_t)lb * hq * HD + (grp * Gq + r) * HD + d, pack2(o1, o2));
      }
      if (slot >= 0 && tid < HD) {          // append the new token (read by the NEXT launches only; after the
                                            // attention: hipcc waits for these stores before reusing their VGPRs)
        const int blk = slot / KBS, off = slot % KBS;
        kc[((size_t)blk * hkv + grp) * hs + off * HD + tid] = f2bf(kn[tid]);
        vc[((size_t)blk * hkv + grp) * hs + tid * KBS + off] = f2bf(vn[tid]);
      }
    }
    PD_STAMP(4);
    // ---- P3: O rows -> residual ----
    arrive(gcnt);
    wait_grid(a.sync, ++nbar, G, err);
    PD_STAMP(5);
#pragma unroll
    for (int b = 0; b < B; ++b)   // attn (sc1) -> LDS
      stage_sc1(reinterpret_cast<uint4*>(lds + LDS_X + b * xhb), a.attn + (size_t)b * hq * HD, hq * HD / 8);
    vm_drain();
    __syncthreads();
    {
      RowVals<B> v = so.run(xaddr, (uint32_t)xhb);
      so.drain();
      // (leader workgroups own no O rows on any rank: they take no part in its all-reduce)
      if (tp && !leader) xreduce<B, RG>(a, ebase + 2u * (unsigned)l + 1u, wg, ow0 + lane, lane < n_o, v.v, err);
#pragma unroll
      for (int b = 0; b < B; ++b) {
        float* const rr = a.res + (size_t)b * H + ow0 + lane;
        if (lane < n_o) st_sc1(rr, ld_sc1(rr) + bf2f(f2bf(v.v[b])));
      }
    }
    PD_STAMP(6);
    auto sg = make_stream<B, RG>(Lw.w13, 2 * I, H, 2 * ng, lane, ring, gu_row, gw);
    arrive(gcnt);
    sg.template start<KA_PD_PREISSUE>();
    wait_grid(a.sync, ++nbar, G, err);
    sg.template top_up<KA_PD_PREISSUE>();
    PD_STAMP(7);
    // ---- P4: norm + gate / up -> act ----
    rmsnorm_rows_to_lds<B>(a, a.res, Lw.ln2, xs, xhb / 2, red);
    PD_STAMP(8);
    {
      const RowVals<B> v = sg.run(xaddr, (uint32_t)xhb);   // lane 2 k: gate row k, lane 2 k + 1: its up row
      sg.drain();
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const float u = bf2f(f2bf(__shfl_down(v.v[b], 1, 64)));
        const float gt = bf2f(f2bf(v.v[b]));
        if (!(lane & 1) && (lane >> 1) < ng)
          ob[b * 512 + wave * i_per_wave + (lane >> 1)] = f2bf(gt / (1.f + __expf(-gt)) * u);
      }
      __syncthreads();
#pragma unroll
      for (int b = 0; b < B; ++b)
        if (2 * tid < wan)
          st_sc1u(a.act + (size_t)b * I + wa0 + 2 * tid, reinterpret_cast<const uint32_t*>(ob)[b * 256 + tid]);
    }
    PD_STAMP(9);
    auto sd = make_stream<B, RGD>(Lw.w2, H, I, no, lane, ring_d, own_row, gw);
    arrive(gcnt);
    sd.template start<KA_PD_PREISSUE>();
    wait_grid(a.sync, ++nbar, G, err);
    sd.template top_up<KA_PD_PREISSUE>();
    PD_STAMP(10);
    // ---- P5: down rows -> residual ----
#pragma unroll
    for (int b = 0; b < B; ++b)   // act (sc1) -> LDS
      stage_sc1(reinterpret_cast<uint4*>(lds + LDS_X + b * xsb), a.act + (size_t)b * I, I / 8);
    vm_drain();
    __syncthreads();
    {
      RowVals<B> v = sd.run(xaddr, (uint32_t)xsb);
      sd.drain();
      if (tp) xreduce<B, RG>(a, ebase + 2u * (unsigned)l + 2u, wg, own0 + lane, lane < no, v.v, err);
#pragma unroll
      for (int b = 0; b < B; ++b) {
        float* const rr = a.res + (size_t)b * H + own0 + lane;
        if (lane < no) st_sc1(rr, ld_sc1(rr) + bf2f(f2bf(v.v[b])));
      }
    }
    PD_STAMP(11);
    arrive(gcnt);   // the next layer's QKV pieces are issued before the wait (top of the loop)
  }
#undef PD_STAMP
  wait_grid(a.sync, ++nbar, G, err);
#pragma unroll
  for (int b = 0; b < B; ++b)
    for (int r = own0 + lane; r < own1; r += 64) a.h_out[(size_t)b * H + r] = f2bf(ld_sc1(a.res + (size_t)b * H + r));
  // every workgroup has read the epoch base (it did so before its first barrier): move it on
  if (tp && wg == 0 && tid == 0) __hip_atomic_store(a.xctr, ebase + 2u * (unsigned)a.L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void zero_sync_kernel(int* __restrict__ sync) {
  for (int i = threadIdx.x; i < SYNC_BYTES / 4; i += 256) sync[i] = 0;
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

}  // namespace pd

// Workspace bytes for up to MAXB sequences: residual (fp32 B H) + qkv + attn + act (bf16) + the sync words.
extern "C" size_t ka_decode_persistent_ws(int H, int hq, int hkv, int I) {
  return pd::SYNC_BYTES +
         (size_t)pd::MAXB * ((size_t)H * 4 + (size_t)(hq + 2 * hkv) * 128 * 2 + (size_t)hq * 128 * 2 + (size_t)I * 2) + 1024;
}

// Weight-ring slots per wave for a geometry (gq = hq / hkv): 16, or 14 for two sequences of the GQA-8
// geometry (their two 16-KB x rows leave room for no more)
static int pd_ring(int gq, int B) { return gq > 4 ? (B == 1 ? 16 : 14) : KA_PD_RING; }

// LDS layout of a B-sequence launch (see decode_layers_kernel); returns its bytes
static int pd_layout(int B, int H, int hq, int I, pd::Args* a, int gq = 4) {
  auto kb = [](int bytes) { return (bytes + 1023) / 1024 * 1024; };
  const int xh = kb(std::max(H, hq * 128) * 2), xs = kb(std::max(std::max(H, I), hq * 128) * 2);
  const int scr = gq > 4 ? kb(pd::scratch_bytes(8)) : pd::XS_MIN;
  const int rg = pd_ring(gq, B);
  const int ring = std::max(B * (B == 1 ? xs : xh), scr);
  const int ring_d = B == 1 ? ring : B * xs;
  const int rd = B == 1 ? rg : std::min(rg, 12);
  const int red = std::max(ring + pd::NW * rg * 1024, ring_d + pd::NW * rd * 1024);
  if (a) {
    a->xh_bytes = B == 1 ? xs : xh;
    a->xs_bytes = xs;
    a->lds_ring = ring;
    a->lds_ring_d = ring_d;
    a->lds_red = red;
  }
  return red + 64 + B * 1024;
}

// Largest batch (1 or 2) the persistent kernel takes for this model within the LDS of one CU; 0: none.
// gq = hq / hkv (the attention scratch of GQA 8 takes 46 KB of LDS instead of 29)
extern "C" int ka_decode_persistent_max_b2(int H, int hq, int I, int gq) {
  if (H <= 4 * pd::NT * 4 && pd_layout(2, H, hq, I, nullptr, gq) <= 160 * 1024) return 2;   // rmsnorm_rows_to_lds
  if (pd_layout(1, H, hq, I, nullptr, gq) <= 160 * 1024) return 1;
  return 0;
}
extern "C" int ka_decode_persistent_max_b(int H, int hq, int I) { return ka_decode_persistent_max_b2(H, hq, I, 4); }

template <int B, int RG>
static int pd_launch(const pd::Args& a, int G, hipStream_t stream) {
  const int lds = pd_layout(B, a.H, a.hq, a.I, nullptr, a.hq / a.hkv);
  static int attr = 0;
  if (attr < lds) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pd::decode_layers_kernel<B, RG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = lds;
  }
  hipLaunchKernelGGL((pd::decode_layers_kernel<B, RG>), dim3(G), dim3(pd::NT), lds, stream, a);
  return (int)hipGetLastError();
}

// Every layer of a decode step of B = 1 or 2 sequences (see the header).  layers: device array of L x 6
// pointers (wqkv, wo, w13, w2, ln1, ln2); h0 / h_out [B][H]; pos / slot / ctx: device int [B]; bt: the
// sequences' block tables [B][bt_stride]; stamps: nullptr, or [G][L][16] uint64 phase timestamps
// (diagnostics; G <= the CU count).
// Requirements: head_dim 128, block 16, hq % hkv == 0, hq / hkv <= 8, H % 512 == 0, I % 512 == 0,
// hq * 128 % 512 == 0, the B activation rows and the rings within LDS (ka_decode_persistent_max_b),
// the grid (the CU count, rounded down to a multiple of hkv) all resident.
// Tensor parallelism (ka_decode_persistent_tp): world ranks (2 .. 8) of a TP group, this one `rank`;
// xdata / xflag: host arrays of every rank's exchange buffer / flag words (IPC-mapped, uncached:
// parallel/custom_allreduce.py pd_buffers), xctr: this rank's epoch counter (device u32, zero at
// start, advanced by 2 L per launch on every rank alike).  The O and down projections' partial rows
// are all-reduced inside the kernel.  KA_PD_GRID caps the grid (tests: two ranks sharing one GPU).
extern "C" int ka_decode_persistent_tp(void* h_out, const void* h0, const void* layers, int L, int H, int hq, int hkv,
                                       int I, float eps, float scale, void* k_cache, void* v_cache, long cache_layer,
                                       const int* pos, const int* slot, const int* bt, const int* ctx,
                                       const float* cos_sin, void* ws, void* stamps, int B, int bt_stride, int world,
                                       int rank, void* const* xdata, void* const* xflag, void* xctr,
                                       hipStream_t stream) {
  if (L <= 0) return 0;
  if (world > 1 && (world > pd::XR_MAX_RANKS || rank < 0 || rank >= world || xdata == nullptr || xflag == nullptr ||
                    xctr == nullptr || H > pd::XR_MAX_H))
    return (int)hipErrorInvalidValue;
  if (B < 1 || B > pd::MAXB || hq % hkv || hq / hkv > 8 || hkv > 16 || H % 512 || I % 512 || (hq * 128) % 512 ||
      H > 16384 ||   // rmsnorm_to_lds holds a row in 8 16-B words per thread
      ws == nullptr || B > ka_decode_persistent_max_b2(H, hq, I, hq / hkv) || (B > 1 && bt_stride <= 0))
    return (int)hipErrorInvalidValue;
  int cus = pd::num_cus();
  if (const char* e = getenv("KA_PD_GRID")) cus = std::min(cus, std::max(1, atoi(e)));
  const int G = (std::min(cus, pd::XR_MAX_WG) / hkv) * hkv;
  if (G < hkv) return (int)hipErrorInvalidValue;
  {   // every wave's rows fit its 64 lanes (lane i = row i) and the LDS result buffer
    const int per_group = G / hkv, nw = G * pd::NW;
    if (per_group < B + 1) return (int)hipErrorInvalidValue;
    const int q = ((hq / hkv + 2) * 128 + per_group * pd::NW - 1) / (per_group * pd::NW);
    const int hpw = (H + nw - 1) / nw, ipw = (I + nw - 1) / nw;
    const int opw = (H + (G - B * hkv) * pd::NW - 1) / ((G - B * hkv) * pd::NW);
    if (q > 64 || hpw > 64 || 2 * ipw > 64 || opw > 64) return (int)hipErrorInvalidValue;
  }
  char* w = static_cast<char*>(ws);
  pd::Args a;
  a.layers = static_cast<const pd::Layer*>(layers);
  a.L = L;
  a.H = H;
  a.hq = hq;
  a.hkv = hkv;
  a.I = I;
  a.eps = eps;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.h0 = static_cast<const bf16_t*>(h0);
  a.h_out = static_cast<bf16_t*>(h_out);
  a.k_cache = static_cast<bf16_t*>(k_cache);
  a.v_cache = static_cast<bf16_t*>(v_cache);
  a.cache_layer = (size_t)cache_layer;
  a.pos = pos;
  a.slot = slot;
  a.bt = bt;
  a.ctx = ctx;
  a.cos_sin = cos_sin;
  a.sync = reinterpret_cast<int*>(w);
  a.stamps = static_cast<unsigned long long*>(stamps);
  a.res = reinterpret_cast<float*>(w + pd::SYNC_BYTES);
  a.qkv = reinterpret_cast<bf16_t*>(w + pd::SYNC_BYTES + (size_t)pd::MAXB * H * 4);
  a.attn = a.qkv + (size_t)pd::MAXB * (hq + 2 * hkv) * 128;
  a.act = a.attn + (size_t)pd::MAXB * hq * 128;
  a.bt_stride = bt_stride;
  a.world = world > 1 ? world : 0;
  a.rank = rank;
  for (int p = 0; p < pd::XR_MAX_RANKS; ++p) {
    a.xdata[p] = (world > 1 && p < world) ? static_cast<float*>(xdata[p]) : nullptr;
    a.xflag[p] = (world > 1 && p < world) ? static_cast<unsigned*>(xflag[p]) : nullptr;
  }
  a.xctr = static_cast<unsigned*>(xctr);
  pd_layout(B, H, hq, I, &a, hq / hkv);
  // the arrival counters and the error word start at zero in every launch.  A kernel, not
  // hipMemsetAsync: captured into a hipGraph, the memset node left the words at 0xF3C00000 on
  // ROCm 7.2 (every grid wait then ran out; scripts/debug_pd_graph.py)
  hipLaunchKernelGGL(pd::zero_sync_kernel, dim3(1), dim3(256), 0, stream, reinterpret_cast<int*>(w));
  const int rc = (int)hipGetLastError();
  if (rc != 0) return rc;
  if (B == 2 && pd_ring(hq / hkv, 2) == 14) return pd_launch<2, 14>(a, G, stream);
  return B == 1 ? pd_launch<1, KA_PD_RING>(a, G, stream) : pd_launch<2, KA_PD_RING>(a, G, stream);
}

extern "C" int ka_decode_persistent(void* h_out, const void* h0, const void* layers, int L, int H, int hq, int hkv,
                                    int I, float eps, float scale, void* k_cache, void* v_cache, long cache_layer,
                                    const int* pos, const int* slot, const int* bt, const int* ctx,
                                    const float* cos_sin, void* ws, void* stamps, int B, int bt_stride,
                                    hipStream_t stream) {
  return ka_decode_persistent_tp(h_out, h0, layers, L, H, hq, hkv, I, eps, scale, k_cache, v_cache, cache_layer, pos,
                                 slot, bt, ctx, cos_sin, ws, stamps, B, bt_stride, 0, 0, nullptr, nullptr, nullptr,
                                 stream);
}

// Exchange bytes per rank of the in-kernel all-reduce: two halves of [MAXB][XR_MAX_H] fp32, then the
// flags [XR_MAX_WG][XR_MAX_RANKS] u32 (parallel/custom_allreduce.py appends them to its IPC buffer).
extern "C" size_t ka_decode_persistent_xbytes() {
  return (size_t)2 * pd::MAXB * pd::XR_MAX_H * 4 + (size_t)pd::XR_MAX_WG * pd::XR_MAX_RANKS * 4;
}
extern "C" size_t ka_decode_persistent_xflag_offset() { return (size_t)2 * pd::MAXB * pd::XR_MAX_H * 4; }

// Byte offset of the error word in the workspace (the runner reads it back with every B = 1 step).
extern "C" int ka_decode_persistent_err_offset() { return pd::SYNC_ERR * 4; }

// The error word of the last launch (a barrier wait that ran out: some workgroup never ran), cleared.
extern "C" int ka_decode_persistent_err(void* ws, hipStream_t stream) {
  int v = 0;
  if (ws == nullptr) return 0;
  (void)hipMemcpyAsync(&v, static_cast<char*>(ws) + pd::SYNC_ERR * 4, 4, hipMemcpyDeviceToHost, stream);
  (void)hipStreamSynchronize(stream);
  return v;
}
