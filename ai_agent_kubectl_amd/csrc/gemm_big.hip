// gemm_big: the prefill / mixed-step projection GEMM (M > 512 token rows):
//   Y[M, N] = X[M, K] * W[N, K]^T, bf16 in, fp32 accumulate, fused epilogues.
//
// Structure (one wave per SIMD, the register budget spent on the MFMA work — the shape rocBLAS' own
// MT256x256x64 prefill kernel has in profiles/r2/pmc_gemm_r2.md: ~85 % MFMA busy, no barrier waits):
//   * 256 x 256 output tile per 256-thread workgroup, BK = 64; wave w owns a 128 x 128 quadrant
//     (W rows 128 * (w & 1), X rows 128 * (w >> 1)): 8 x 8 MFMA 16x16x32 tiles, 256 fp32
//     accumulators per lane (the AGPR half of the 512-register file), so each k-step reads 16
//     fragments (ds_read_b128) for 64 MFMAs — a quarter of the LDS traffic per MFMA of the 8-wave
//     64 x 128-per-wave layout of gemm_mfma.hip's ping-pong kernel;
//   * W is the MFMA A operand and X the B operand: a lane's four accumulators are four consecutive
//     output columns (8-B bf16 stores), and the SwiGLU epilogue finds gate and up of one output in
//     the same lane;
//   * both operands staged HBM/L2 -> LDS by LDS-DMA (buffer_load dwordx4 ... lds), 2 buffers x 64 KB;
//     the XOR swizzle slot = chunk ^ ((row >> 1) & 7) is applied to the per-lane global source and
//     to the ds_read address (rule 21), conflict-free fragment reads.  A wave's 1-KB pieces of a
//     k-tile are 4-KB contiguous groups written under one M0 value (the immediate offset selects the
//     piece): 4 M0 writes per 16 pieces instead of 16, +6-7 % on every shape
//     (profiles/r3/gemm_big/gb_m0_ab.log);
//   * persistent: one workgroup per CU walks its tiles; the next tile's first two k-tiles are staged
//     during the current tile's last two k-steps and the epilogue transposes through a separate
//     32 KB of LDS, so it overlaps their landing (+0.5-1 %, gb_p_ab.log);
//   * two register fragment sets (F0 = k 0..31, F1 = k 32..63 of a k-tile), the fragment reads and
//     the LDS-DMA pieces in separate windows of the 128-MFMA stream (profiles/r3/gemm_big/gbs_ab.log):
//       MFMA F0(t) 0-15 | read F1(t) <- buffer t&1
//       vmcnt(0), lgkmcnt(0), barrier (every wave's reads of buffer t&1 done, and k-tile t+1 --
//                                      the only pieces in flight -- landed in buffer (t+1)&1)
//       MFMA F0(t) 16-63, F1(t) 0-31 | 16 DMA pieces of k-tile t+2 -> buffer t&1, one per 5 MFMAs
//       MFMA F1(t) 32-63 | read F0(t+1) <- buffer (t+1)&1 from MFMA 48 on, waited for per fragment
//                          row by the next k-tile's first MFMAs;
//     one fragment read per MFMA in the read windows (gb_rp_ab.log).  Rounds 3-4 waited for k-tile
//     t+1 with a counted vmcnt(16) at a second barrier, keeping t+2's pieces in flight across it:
//     4-10 % faster, but LDS-DMA pieces do not complete in order and that wait let stale rows through
//     in some launches (round 5, profiles/r5/gemm_big_clamp/);
//   * XCD-aware tile order (T1): the bijective round-robin remap, then GM m-tiles x all n-tiles
//     super-rows so the panels of the tiles running together on one XCD are L2 hits.
// Measured (round 5, after the drain fix, profiles/r5/gemm_big_clamp/, interleaved with rocBLAS in one
// process): gate_up + SwiGLU 0.99-1.05x rocBLAS's plain GEMM (+ its separate SiLU pass); QKV on 192-wide
// tiles 1.01-1.10x at 2048-6144 rows; O / down 0.80-0.92x.  Engine dispatch: EPI_SWIGLU (prefill /
// mixed-step gate_up, ops.linear_swiglu), EPI_BF16 for QKV where the persisted prefill plan measured it
// faster (ops.linear_big), the grouped mode for MoE prefill, and EPI_ARGMAX (the fused LM head,
// ops.lm_head_argmax, per decode bucket where ModelRunner.tune_lm_head times it faster).  The harness
// (tools/gemm_big_bench.hip) and profiles/r3/scripts/gb_diag.py compare EPI_BF16 against rocBLAS /
// fp32; EPI_ADD and the split-K slabs were measured for the O / down
// projections and decode shapes and lost there (profiles/r3/gemm_big/), so nothing dispatches them.
// Epilogues: bf16 store; SwiGLU over the un-interleaved [gate; up] weight (the tile's W rows are
// gathered as alternating 16-row gate / up chunks by the DMA source addresses, so the [M, 2I]
// gate_up output never exists); residual add (Y = X W^T + R, R may alias Y).
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <utility>


namespace gb {

// Tile geometry per TN = 16-row W (MFMA A) fragments per wave: TN 8 is the 256 x 256 tile, TN 6 a
// 192 (W rows) x 256 (X rows) tile for shapes whose 256-wide tiles leave a fractional last round
// (QKV, N = 6144: 384 tiles = 1.5 rounds of 256 CUs at M = 4096; 512 x 192-row tiles = 2 full rounds).
constexpr int BM = 256, BK = 64, NT = 256;
template <int TN>
struct Geo {
  static constexpr int BN = 32 * TN;                        // W rows of a tile (two waves of 16 TN)
  static constexpr int TILE_A = BN * BK * 2;                // 32 / 24 KB
  static constexpr int TILE_B = BM * BK * 2;                // 32 KB
  static constexpr int STAGE = TILE_A + TILE_B;
  static constexpr int LDS = 2 * STAGE;   // two 64-deep buffers (a 5-slot ring of 32-deep stages measured slower)
  static constexpr int LDS_TOTAL = LDS + 4 * 8192;         // + the epilogue scratch (8 KB per wave)
  static constexpr int PIECES = TN + 8;                     // 1-KB LDS-DMA pieces per wave per k-tile
};
constexpr int BN = Geo<8>::BN;   // the 256-wide tile (SwiGLU / argmax / split-K epilogues)

enum Epi : int { EPI_BF16 = 0, EPI_P32 = 1, EPI_P16 = 2, EPI_SWIGLU = 3, EPI_ADD = 4, EPI_ARGMAX = 5 };

struct Args {
  const bf16_t* X;   // [M, ldx]
  const bf16_t* W;   // [N, K]  (SwiGLU: [2I, K], gate rows then up rows)
  bf16_t* Y;         // [M, ldy]
  const bf16_t* R;   // EPI_ADD: residual [M, ldy] (may be Y)
  int M, N, K, ldx, ldy, tiles_m, tiles_n, gm;
  int I;             // SwiGLU: the up rows start at W row I (N == 2I)
  // EPI_ARGMAX (the LM head + greedy SAFE_DECODE sampling): logits never leave the registers; each
  // tile writes its per-row (max, lowest index) of the bf16-rounded, mask-allowed logits to
  // part_val / part_idx [M][tiles_n] (argmax_finish_kernel picks the winner per row)
  const uint32_t* mask_bits;   // [masks][mask_words], bit = global token id (nullptr: no mask)
  const int* mask_idx;         // [M] mask row per output row, < 0 = unmasked
  int mask_words, vocab_offset;
  float* part_val;
  int* part_idx;
  // split-K (EPI_P32 / EPI_P16): workgroup (tile, ks) sums k in [ks kp, (ks + 1) kp) into the partial
  // slab P[ks] of [split][M][N] (fp32 / bf16), reduced by the consumer (ops.SplitK)
  int split, kp;
  void* P;
  // split tail (EPI_BF16 / SWIGLU / ADD): units [0, full) are whole tiles (full = a multiple of the
  // persistent grid); the tail_tiles tiles after them would leave most CUs idle in a last partial
  // round, so each is cut into tail_s K-slices run by different workgroups of ONE XCD.  Every wave
  // of a slice publishes its fp32 quadrant (stores, the wave's own vmcnt(0), an agent-scope release),
  // then adds to its quadrant's arrival counter; the wave whose add returns
  // tail_s - 1 acquires at agent scope, sums the slices and runs the epilogue — no wait on other
  // workgroups — and resets the counter for the next launch.
  int full, tail_s, tail_tiles, span;
  float* slab;   // [tail tile][tail_s slices][4 waves][64 accumulators][64 lanes] f32x4
  int* cnt;      // [tail tile][4 waves][arrivals, spare]
  int* err;      // reserved error word (0)
  // grouped (MoE experts, gemm256_kernel<.., GR>): X holds the routed rows sorted by expert
  // (ka_moe_sort), chunk_tab[tiles_m][4] = (expert, first sorted row, rows, 0) of the 256-row chunks
  // (rows 0: an unused entry); W is [groups][N][K]; EPI_BF16 stores sorted row r at output row
  // out_rows[r] (the slot order moe_combine reads), EPI_SWIGLU at sorted row r (the next GEMM's X)
  const int* chunk_tab;
  const int* out_rows;
  int groups;
};

// Every instruction of the k-loop is an asm statement, so the program order written below IS the
// issue order (hipcc may not hoist, sink or regroup volatile asm), and hipcc inserts no waits of its
// own for these loads: the s_waitcnt / s_barrier statements below are the whole synchronisation.
//  * ds_read_b128: fragment read (16-bit immediate offset);
//  * LDS-DMA: buffer_load_dwordx4 ... offen lds through a buffer descriptor (wave-uniform base in
//    SGPRs, k offset in soffset, one 32-bit VGPR offset per lane); M0 = the LDS destination group,
//    saved by a group's first piece and restored by its fourth (M0 is compiler-reserved; nothing
//    hipcc emits between them uses it);
//  * MFMA with the accumulator pinned in place in the AGPR file ("+a"): the builtin form lets the
//    register allocator rotate the 64 accumulators through VGPRs (~100 v_accvgpr moves per k-tile
//    at this register pressure).  An MFMA's D read by anything but the next MFMA's C needs the wait
//    states of mfma_drain() (hipcc pads nothing inside asm).
// compile-time unrolled loop: f(std::integral_constant<int, 0>{}) ... f(..N-1): asm immediates
// ("i" operands) need constants, which a #pragma-unrolled loop variable is not
template <class F, int... S>
KA_DEV void static_for_impl(F&& f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}
template <int N, class F>
KA_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int OFF>
KA_DEV void ds_read16(bf16x8& dst, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(OFF));
}
// the same piece under a shared M0: piece P (< 4) of a 4-KB LDS group writes M0 + 1024 P (the immediate
// offset applies to both the LDS destination and the global address, so the lane's global offset is
// pre-biased by -1024 P); P == 0 saves M0 and points it at the group, P == 3 restores it
// LAST: the group's final piece (P == 3 of a 4-piece group; P == 1 of the 2-piece W group of TN 6)
#ifndef KA_GB_CLAMP
#define KA_GB_CLAMP 0     // diagnostic: rows past the end clamped to the last row (duplicate addresses)
#endif
template <int P, bool LAST>
KA_DEV void dma16g(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, uint32_t lds_addr, uint32_t& keep) {
  static_assert(P > 0 || !LAST, "a group has at least two pieces");
  if constexpr (P == 0)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds"
                 : "=&s"(keep)
                 : "v"(voff), "s"(r), "s"(lds_addr), "s"(soff)
                 : "memory");
  else if constexpr (LAST)
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen offset:%3 lds\n\ts_mov_b32 m0, %4"
                 :
                 : "v"(voff), "s"(r), "s"(soff), "i"(P * 1024), "s"(keep)
                 : "memory");
  else
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen offset:%3 lds"
                 :
                 : "v"(voff), "s"(r), "s"(soff), "i"(P * 1024)
                 : "memory");
}
KA_DEV void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
KA_DEV void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }
// LDS-DMA completion is NOT ordered: a counted `s_waitcnt vmcnt(N)` (N younger pieces still allowed in
// flight) passed while an older piece had not landed, in some launches (X piece 7 of a k-tile read
// stale: 5/40 launches at M = 4096, N = 1152 with clamped duplicate rows, 1/80 at M = 2944, N = 6144 with
// distinct rows), and a vmcnt(0) drain in the same places never failed (0/160, clamped rows included):
// profiles/r5/gemm_big_clamp/.  So every LDS-DMA wait of this kernel is vmcnt(0), placed where the
// only pieces in flight are the ones about to be read (KA_GB_DRAIN_B1 below).
#ifndef KA_GB_DRAIN_B1
#define KA_GB_DRAIN_B1 1  // 0: the old counted vmcnt(PIECES) at barrier #2 (unsafe, for A/B timing only)
#endif
template <int N>
KA_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
KA_DEV void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <int N>
KA_DEV void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }
KA_DEV void block_sync() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// dispatch index -> logical index, XCD-contiguous (bijective over the grid: consecutive logical
// indices run on one XCD and share its L2)
KA_DEV int xcd_logical(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}
// logical tile -> (m tile, n tile): GM m-tiles x all n-tiles super-rows
KA_DEV void tile_of(int L, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per = gm * tiles_n;
  const int g = L / per, first = g * gm;
  const int rows = min(gm, tiles_m - first);
  const int in = L - g * per;
  tm = first + in % rows;
  tn = in / rows;
}

// 16-B store / load of the tail hand-off.  KA_GB_TAIL_MODE 0: plain accesses ordered by agent-scope
// release / acquire fences; 1: sc1 (write-through) asm stores + the same fences; 2: sc1 asm stores and
// loads, no fence (MI355X_MICROARCH.md hand-off table, row 1: one signalling lane per storing wave,
// per-wave counter, the consumer told by the value its own add returned, all stores and loads sc1
// 16 B, hipMalloc memory); 3: the sc1 loads of 2 after the fences of 1.  hipcc does not pad the
// VMEM-store-data / VALU-write hazard around asm it cannot see, so the asm stores carry their own
// wait states (without them a few lanes' data were corrupted: profiles/r4/gemm_big_tail/).
// Round 5 full-matrix repeats (profiles/r5/gemm_big_tail_modes/): before the LDS-DMA drain fix, modes
// 0 and 1 read stale data in some first launches; after it, all four modes were exact in every launch
// (48 full checks each, after_drain/), so those failures were the DMA hazard.  Mode 2 stays the
// default because it is the fastest: 2944 x 28672 SwiGLU 639-647 us against 650-667 for the fenced
// modes, 78-83 against 90-113 us on an all-split shape.
#ifndef KA_GB_TAIL_MODE
#define KA_GB_TAIL_MODE 2
#endif
template <int N>
KA_DEV void st_slab(float* p, const f32x4 (&v)[N], const int (&q)[N]) {
#if KA_GB_TAIL_MODE == 0
#pragma unroll
  for (int e = 0; e < N; ++e) *reinterpret_cast<f32x4*>(p + q[e] * 256) = v[e];
#else
  // all stores in ONE asm statement followed by the wait states of the VMEM-store-data / VALU-write
  // hazard (hipcc cannot see the stores: with per-store statements and 2 wait states each, the
  // register allocator's next VALU write corrupted store data in a few lanes)
  static_assert(N == 6 || N == 8, "slab width");
  if constexpr (N == 8)
    asm volatile(
        "global_store_dwordx4 %0, %8, off sc1\n\tglobal_store_dwordx4 %1, %9, off sc1\n\t"
        "global_store_dwordx4 %2, %10, off sc1\n\tglobal_store_dwordx4 %3, %11, off sc1\n\t"
        "global_store_dwordx4 %4, %12, off sc1\n\tglobal_store_dwordx4 %5, %13, off sc1\n\t"
        "global_store_dwordx4 %6, %14, off sc1\n\tglobal_store_dwordx4 %7, %15, off sc1\n\ts_nop 4" ::"v"(p + q[0] * 256),
        "v"(p + q[1] * 256), "v"(p + q[2] * 256), "v"(p + q[3] * 256), "v"(p + q[4] * 256), "v"(p + q[5] * 256),
        "v"(p + q[6] * 256), "v"(p + q[7] * 256), "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]),
        "v"(v[6]), "v"(v[7])
        : "memory");
  else
    asm volatile(
        "global_store_dwordx4 %0, %6, off sc1\n\tglobal_store_dwordx4 %1, %7, off sc1\n\t"
        "global_store_dwordx4 %2, %8, off sc1\n\tglobal_store_dwordx4 %3, %9, off sc1\n\t"
        "global_store_dwordx4 %4, %10, off sc1\n\tglobal_store_dwordx4 %5, %11, off sc1\n\ts_nop 4" ::"v"(p + q[0] * 256),
        "v"(p + q[1] * 256), "v"(p + q[2] * 256), "v"(p + q[3] * 256), "v"(p + q[4] * 256), "v"(p + q[5] * 256),
        "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5])
        : "memory");
#endif
}
template <int N>
KA_DEV void ld_slab(f32x4 (&t)[N], const float* p, const int (&q)[N]) {
#if KA_GB_TAIL_MODE >= 2   // 2: sc1 loads without fences; 3: sc1 loads after the fences of mode 1
#pragma unroll
  for (int e = 0; e < N; ++e)
    asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(t[e]) : "v"(p + q[e] * 256) : "memory");
  // the loads' registers are operands of the wait, so no use (or copy) is scheduled above it
  static_assert(N == 6 || N == 8, "slab width");
  if constexpr (N == 8)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]),
                 "+v"(t[6]), "+v"(t[7])::"memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5])::"memory");
#else
#pragma unroll
  for (int e = 0; e < N; ++e) t[e] = *reinterpret_cast<const f32x4*>(p + q[e] * 256);
#endif
}

// Tail slice hand-off of one wave's 128 x 128 quadrant (Args.full .. comment): every slice publishes
// its fp32 quadrant to slot k of the tile's slab (the epilogue's mode 1, tail_store), waits for its
// own stores, then takes an arrival ticket; the slice whose ticket is the last one (all others have
// published before arriving) runs the epilogue on the sum of the slots (mode 2, tail_fetch) and
// resets the counter for the next launch.  The accumulators are read at ONE place of the epilogue
// (a second read, or summing into them, made hipcc move the whole tile into VGPRs and spill).
KA_DEV bool tail_ticket(const Args& a, int tt, int w, int lane) {
  // release at agent scope: this wave's slab stores are done and written back past its XCD's L2
  // before its ticket (the slices of a tile are meant to share an XCD for speed, but placement is
  // only observed, never promised).  The asm wait after the fence: MI355X_MICROARCH.md 'Compiler hazard'.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if KA_GB_TAIL_MODE != 2
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  int* const c = a.cnt + (tt * 4 + w) * 2;
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old != a.tail_s - 1) return false;
  if (lane == 0) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // tile complete
#if KA_GB_TAIL_MODE != 2
  // acquire at agent scope before this wave reads the other slices' slabs
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  return true;
}

// slab slot of (tail tile tt, slice k, wave w): [TN 8 accumulator rows of 64 lanes] f32x4 per wave
template <int TN>
KA_DEV float* tail_slot(const Args& a, int tt, int k, int w, int lane) {
  return a.slab + ((((size_t)tt * a.tail_s + k) * 4 + w) * (TN * 8)) * 256 + lane * 4;
}

// this slice's accumulators q[e] -> its slot
template <int TN, int N>
KA_DEV void tail_store(const Args& a, int tt, int k, int w, int lane, const int (&q)[N], const f32x4 (&v)[N]) {
  st_slab<N>(tail_slot<TN>(a, tt, k, w, lane), v, q);
}

// v[e] = sum over the tile's ts slots of accumulator q[e] of this lane (after tail_ticket's acquire)
template <int TN, int N>
KA_DEV void tail_fetch(const Args& a, int tt, int w, int lane, const int (&q)[N], f32x4 (&v)[N]) {
  const int ts = a.tail_s;
#pragma unroll
  for (int e = 0; e < N; ++e) v[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < ts; ++k) {
    const float* const p = tail_slot<TN>(a, tt, k, w, lane);
    f32x4 t[N];
    ld_slab<N>(t, p, q);
#pragma unroll
    for (int e = 0; e < N; ++e) v[e] += t[e];
  }
}

template <int EPI, int TN, bool GR = false>
__global__ __launch_bounds__(NT, 1) void gemm256_kernel(Args a) {
  using GE = Geo<TN>;
  constexpr int BNT = GE::BN, TILE_A = GE::TILE_A, STAGE = GE::STAGE, PIECES = GE::PIECES;
  static_assert(TN == 8 || ((EPI == EPI_BF16 || EPI == EPI_ADD) && TN == 6), "TN 6: plain / residual epilogues");
  static_assert(!GR || (TN == 8 && (EPI == EPI_BF16 || EPI == EPI_SWIGLU)), "grouped: bf16 / SwiGLU, 256 x 256");
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  char* const L = reinterpret_cast<char*>(lds);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = w & 1, wm = w >> 1;
  constexpr bool SPLIT = EPI == EPI_P32 || EPI == EPI_P16;
  // Persistent: workgroup b computes the output tiles of virtual dispatch ids b, b + G, b + 2G, ...
  // (G = gridDim.x, a multiple of 8 whenever G < total), each mapped like a one-tile-per-workgroup
  // grid of `total` workgroups would be: an id keeps its XCD (b mod 8), so the tiles running together
  // on one XCD are still neighbours.  The next tile's first two k-tiles are staged during the last
  // two k-steps of the current one, so the epilogue overlaps their landing.
  constexpr bool TAILOK = (EPI == EPI_BF16 || EPI == EPI_SWIGLU || EPI == EPI_ADD) && !GR;
  const int total = SPLIT ? a.tiles_m * a.tiles_n * a.split : (TAILOK ? a.full + a.span : a.tiles_m * a.tiles_n);
  const int nkt = a.K / BK;
  // unit v -> tile (tm, tn), k-tiles [kt0, kt0 + nk), tail tile index tt (-1: a whole tile / split-K slice);
  // false for the holes of the last tail group (tail_tiles not a multiple of 8)
  // GR: (ge, gr0, gnr) = the chunk's expert, first sorted row and row count (scalar loads of the
  // chunk table, here at a tile boundary, outside every counted wait window); false for an unused entry
  auto decode = [&](int v, int& tm, int& tn, int& kt0, int& nk, int& tt, int& tk, int& ge, int& gr0,
                    int& gnr) -> bool {
    tt = -1;
    tk = 0;
    ge = 0;
    gr0 = 0;
    gnr = 0;
    if constexpr (SPLIT) {   // the split slices of a tile on one XCD
      int lg = xcd_logical(v, total);
      const int ks = lg % a.split;
      lg /= a.split;
      tile_of(lg, a.tiles_m, a.tiles_n, a.gm, tm, tn);
      kt0 = ks * (a.kp / BK);
      nk = a.kp / BK;
      return true;
    }
    if (!TAILOK || v < a.full) {
      tile_of(xcd_logical(v, TAILOK ? a.full : total), a.tiles_m, a.tiles_n, a.gm, tm, tn);
      kt0 = 0;
      nk = nkt;
      if constexpr (GR) {
        const int* c = a.chunk_tab + 4 * tm;
        ge = c[0];
        gr0 = c[1];
        gnr = c[2];
        return gnr > 0;
      }
      return true;
    }
    // tail: groups of 8 tiles x tail_s slices; slice k of tile 8 g + l is unit 8 (g tail_s + k) + l, so
    // a tile's slices share v mod 8, i.e. one XCD (their slab hand-off stays in its L2)
    const int u = v - a.full, ts = a.tail_s;
    const int g = u / (8 * ts), r = u - g * 8 * ts, k = r >> 3;
    tt = g * 8 + (r & 7);
    tk = k;
    if (tt >= a.tail_tiles) return false;
    tile_of(a.full + tt, a.tiles_m, a.tiles_n, a.gm, tm, tn);
    const int trips = nkt >> 1;   // the k-loop runs two k-tiles per trip
    const int t0 = k * trips / ts, t1 = (k + 1) * trips / ts;
    kt0 = 2 * t0;
    nk = 2 * (t1 - t0);
    return true;
  };
  const int G = (int)gridDim.x;
  int vb = blockIdx.x, tm = 0, tn = 0, kt0 = 0, nku = nkt, tt = -1, tslice = 0, ge = 0, gr0 = 0, gnr = 0;
  while (vb < total && !decode(vb, tm, tn, kt0, nku, tt, tslice, ge, gr0, gnr)) vb += G;
  if (vb >= total) return;   // only holes for this workgroup: nothing staged, nothing to wait for

  // the descriptors start BIAS bytes before the operands, so the per-lane offsets (pre-biased by
  // -1024 (j & 3) for the immediate offset of dma16g) never wrap; nothing below an operand is read
  constexpr uint32_t BIAS = 3072;
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(a.W)) - BIAS, (short)0,
      (int)((uint32_t)(GR ? a.groups : 1) * (uint32_t)a.N * (uint32_t)a.K * 2u + BIAS), 0x00020000);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(a.X)) - BIAS, (short)0,
      (int)((uint32_t)a.M * (uint32_t)a.ldx * 2u + BIAS), 0x00020000);
  // LDS byte address of the staging array (dynamic LDS: the only LDS object of this kernel)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) u32x4*)lds;
  const int r16 = lane & 15, grp = lane >> 4;
  // DMA sources: wave-instruction j of this wave fills staged W rows 8 TN w + 8 j .. + 8 (j < TN) and
  // X rows 64 w + 8 j .. + 8 (j < 8), 1 KB each, so a wave's pieces are contiguous 1-KB blocks (up to
  // 4 per M0 value)
  const int r8 = lane >> 3, slot = lane & 7;
  uint32_t offA[TN], offB[8];
  auto set_offsets = [&](int tm_, int tn_, int kt0_, int ge_, int gr0_, int gnr_) {
    const int m0_ = tm_ * BM;
    const uint32_t kb = (uint32_t)kt0_ * (uint32_t)(BK * 2);   // byte offset of the unit's k range
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = 8 * TN * w + 8 * j + r8;
      const uint32_t ch = (uint32_t)(slot ^ ((row >> 1) & 7)) * 8;
      int wrow;
      if constexpr (EPI == EPI_SWIGLU) {
        // tile tn covers output columns [128 tn, 128 tn + 128): 16-row chunk c of the staged W tile
        // is gate (c even) or up (c odd) of output columns 128 tn + 16 (c >> 1) + 0..15
        wrow = 128 * tn_ + 16 * (row >> 5) + (row & 15) + ((row >> 4) & 1) * a.I;
      } else {
        // rows past the last one read distinct valid rows (their results are not stored): clamping
        // them all to row N - 1 made 64-lane LDS-DMA pieces of duplicate addresses, and with them
        // other pieces' rows came out wrong in some launches (profiles/r5/gemm_big_clamp/)
        wrow = tn_ * BNT + row;
#if KA_GB_CLAMP
        wrow = min(wrow, a.N - 1);   // diagnostic: the old clamp
#else
        if (wrow >= a.N) wrow %= a.N;
#endif
      }
      if constexpr (GR) wrow += ge_ * a.N;   // expert ge_'s weights
      offA[j] = ((uint32_t)wrow * (uint32_t)a.K + ch) * 2u + kb + BIAS - (uint32_t)(j & 3) * 1024u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 64 * w + 8 * j + r8;
      const uint32_t ch = (uint32_t)(slot ^ ((row >> 1) & 7)) * 8;
      // GR: the chunk's rows; rows past its count read other rows of the chunk (not stored)
      // (rows past the end: distinct valid rows, as for W above)
      int xr;
      if constexpr (GR) xr = gr0_ + (row < gnr_ ? row : row % gnr_);
#if KA_GB_CLAMP
      else xr = min(m0_ + row, a.M - 1);   // diagnostic: the old clamp
#else
      else xr = m0_ + row < a.M ? m0_ + row : (m0_ + row) % a.M;
#endif
      offB[j] = ((uint32_t)xr * (uint32_t)a.ldx + ch) * 2u + kb + BIAS - (uint32_t)(j & 3) * 1024u;
    }
  };
  set_offsets(tm, tn, kt0, ge, gr0, gnr);
  // DMA piece s (< PIECES) of a k-tile: W (s < TN) or X (s >= TN); M0 is set once per group of up to 4
  // pieces and restored after the group's last
  const uint32_t ldsw = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)w * (uint32_t)(TN * 1024));
  const uint32_t ldsx = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)TILE_A + (uint32_t)w * 8192u);
  uint32_t m0keep = 0;
  auto dma = [&](auto sc, auto bufc, int T) {
    constexpr int S = decltype(sc)::value, BUF = decltype(bufc)::value;
    const uint32_t soff = (uint32_t)T * (BK * 2);
    if constexpr (S < TN) {
      constexpr int P = S & 3;
      constexpr bool LAST = P == 3 || S == TN - 1;
      dma16g<P, LAST>(rW, offA[S], soff, ldsw + BUF * STAGE + (S >> 2) * 4096, m0keep);
    } else {
      constexpr int J = S - TN, P = J & 3;
      dma16g<P, P == 3>(rX, offB[J], soff, ldsx + BUF * STAGE + (J >> 2) * 4096, m0keep);
    }
  };

  // fragment read bases (bytes, LDS address): [buffer][k half] of the A (W) and B (X) quadrants
  const int sw = (r16 >> 1) & 7;
  const uint32_t c0 = ((0 + grp) ^ sw) * 16, c1 = ((4 + grp) ^ sw) * 16;
  const uint32_t rA = lds0 + (wn * TN * 16 + r16) * 128, rB = lds0 + TILE_A + (wm * 128 + r16) * 128;
  const uint32_t bA00 = rA + c0, bA01 = rA + c1, bA10 = rA + STAGE + c0, bA11 = rA + STAGE + c1;
  const uint32_t bB00 = rB + c0, bB01 = rB + c1, bB10 = rB + STAGE + c0, bB11 = rB + STAGE + c1;

  f32x4 acc[TN][8];
  bf16x8 fa0[TN], fb0[8], fa1[TN], fb1[8];

  // the k-loop schedule per k-tile (two fragment sets F0 = k 0..31 and F1 = k 32..63, NQ MFMAs each,
  // issued as groups of 4)
  constexpr int NRD = TN + 8;        // fragment reads per set
  constexpr int NQ = TN * 8;         // MFMAs per set
  constexpr int GPS = NQ / 4;        // groups per set
  constexpr int NG = 2 * GPS;        // groups per k-tile (32 at TN 8)
  constexpr int RW = NG - 4;         // F0(t + 1) read window: the k-tile's last 4 groups
#ifndef KA_GB_B1
#define KA_GB_B1 4
#endif
  constexpr int B1 = KA_GB_B1;       // barrier #1's group: 4 = right after the F1 read window; 5 / 6
                                     // give the window's last reads 4 / 8 more MFMAs before lgkmcnt(0)
  static_assert(B1 >= 4 && B1 <= 6, "barrier #1 group");
#ifndef KA_GB_DMA_END
#define KA_GB_DMA_END (KA_GB_DRAIN_B1 ? 24 : 0)
#endif
  // the DMA window: groups B1 .. DE - 1.  The drain at the next call's barrier #1 waits for the window's
  // last piece, so a shorter window leaves it more time to land; but the 64 KB a k-tile stages per CU
  // need about half the k-tile's MFMA time at the L1 fill rate, and windows of 12 groups stalled the
  // MFMA stream (measured, profiles/r5/gemm_big_clamp/README.md: 12 / 16 lose 3-10 %, 20-28 are within
  // 2 % of each other, 24 the best on the gate_up + SwiGLU shape).
  constexpr int DE = KA_GB_DMA_END > 0 && KA_GB_DMA_END < RW ? KA_GB_DMA_END : RW;
  static_assert(DE > B1 && DE <= RW, "DMA window");
  static_assert(NRD <= 16, "a read window holds 16 reads");
  // read S of a fragment set in window order 1 (A0 B0 A1 B1 ..., the B's past A(TN-1) last):
  auto rd1 = [&](auto sc, bf16x8* FA, bf16x8* FB, uint32_t ba, uint32_t bb) {
    constexpr int S = decltype(sc)::value;
    if constexpr (S < 2 * TN) {
      if constexpr (S & 1) ds_read16<(S >> 1) * 2048>(FB[S >> 1], bb);
      else ds_read16<(S >> 1) * 2048>(FA[S >> 1], ba);
    } else {
      ds_read16<(S - TN) * 2048>(FB[S - TN], bb);
    }
  };
  // ... and in window order 2 (B0 .. B7, then A0 .. A(TN-1)): row 0 of the next call needs A0 and every B
  auto rd2 = [&](auto sc, bf16x8* FA, bf16x8* FB, uint32_t ba, uint32_t bb) {
    constexpr int S = decltype(sc)::value;
    if constexpr (S < 8) ds_read16<S * 2048>(FB[S], bb);
    else ds_read16<(S - 8) * 2048>(FA[S - 8], ba);
  };
  // MFMAs 4S .. 4S+3 of the TN x 8 set
  auto mma4 = [&](auto sc, const bf16x8* FA, const bf16x8* FB) {
    constexpr int S = decltype(sc)::value;
    static_for<4>([&](auto qc) {
      constexpr int q = 4 * S + decltype(qc)::value;
      mfma_acc(acc[q >> 3][q & 7], FA[q >> 3], FB[q & 7]);
    });
  };
  // one 64-deep k-tile per call as NG groups of 4 MFMAs (groups 0 .. GPS-1 on F0, the rest on F1),
  // the fragment reads and the LDS-DMA pieces in separate windows of the MFMA stream (the order
  // hipBLASLt's MT256x256x64 DirectToLds kernel uses; it measured faster than a window carrying both):
  //   groups 0-3:   F1(t) <- buffer BUF, one read before each MFMA
  //   vmcnt(0) + lgkmcnt(0) + barrier #1: every wave's reads of buffer BUF are done (F0(t) was read
  //                 at the end of the previous call), and the k-tile staged one call earlier -- the
  //                 only DMA in flight -- has landed in buffer BUF ^ 1
  //   groups 4 .. DE-1: the PIECES pieces of k-tile T into buffer BUF, spread evenly
  //   groups RW .. NG-1: F0(t + 1) <- buffer BUF ^ 1, one read before each MFMA (F0(t) retired at
  //                 group GPS - 1)
  // (KA_GB_DRAIN_B1 0 restores the rounds 3-4 order for timing: lgkmcnt(0) alone at barrier #1 and a
  // counted vmcnt(PIECES) + barrier #2 at group RW, unsafe: see wait_vm.)
  // (Every DMA is issued unconditionally: skipping the last unit's re-stage behind a runtime flag put
  // VALU work (the flag's mask) into the MFMA stream, where hipcc's register reuse wrote an A-fragment
  // VGPR still being read by an in-flight asm MFMA it cannot see (sparse wrong outputs in the SwiGLU
  // and argmax epilogues), and it bought nothing measurable on the single-round shapes.)
  auto iter = [&](auto bufc, int T) {
    constexpr int BUF = decltype(bufc)::value;
    static_for<NG>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      if constexpr (g < 4 || g >= RW) {   // read windows: one fragment read before each MFMA
        static_for<4>([&](auto qc) {
          constexpr int qq = decltype(qc)::value;
          constexpr int S = 4 * (g < 4 ? g : g - RW) + qq;
          if constexpr (S < NRD) {
            if constexpr (g < 4)
              rd1(std::integral_constant<int, S>{}, fa1, fb1, BUF ? bA11 : bA01, BUF ? bB11 : bB01);
            else
              rd2(std::integral_constant<int, S>{}, fa0, fb0, BUF ? bA00 : bA10, BUF ? bB00 : bB10);
          }
          constexpr int q = 4 * (g % GPS) + qq;
          // the previous call's F0 reads (order 2) are waited for here, per A fragment: row 0 (A0,
          // all B) before MFMA 0 (A1.. and this call's first read may still be in flight), row 1 (A1)
          // before MFMA 8; rows 2.. are covered by barrier #1's lgkmcnt(0).  No copy of a fragment
          // register sits between (checked in the disassembly: the loop has no v_mov)
          if constexpr (g < 4 && q == 0) wait_lgkm<TN>();
          if constexpr (g < 4 && q == 8) wait_lgkm<TN + 7>();
          if constexpr (g < GPS) mfma_acc(acc[q >> 3][q & 7], fa0[q >> 3], fb0[q & 7]);
          else mfma_acc(acc[q >> 3][q & 7], fa1[q >> 3], fb1[q & 7]);
        });
      }
      if constexpr (g == 4 && B1 > 4) wait_lgkm<15>();   // row 2 (A2) of F0: all but 15 reads done
      if constexpr (g == B1) {
        if constexpr (KA_GB_DRAIN_B1) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else wait_lgkm0();
        block_sync();
      }
      if constexpr (g >= B1 && g < DE) {   // the DMA pieces whose slot falls in this group
        static_for<PIECES>([&](auto pc) {
          constexpr int pp = decltype(pc)::value;
          if constexpr (B1 + (pp * (DE - B1)) / PIECES == g) dma(pc, bufc, T);
        });
      }
      if constexpr (g == RW && !KA_GB_DRAIN_B1) {
        wait_vm<PIECES>();
        block_sync();
      }
      if constexpr (g >= 4 && g < RW) {
        if constexpr (g < GPS) mma4(std::integral_constant<int, g>{}, fa0, fb0);
        else mma4(std::integral_constant<int, g - GPS>{}, fa1, fb1);
      }
    });
    // (no lgkmcnt wait here: the next call waits per fragment; the tile's last call waits below)
  };
  // (A five-segment schedule with per-operand counted vmcnt waits, after hipBLASLt's gfx950
  // MT256x256x64 DirectToLds kernel, measured no faster in round 3 and relied on ordered LDS-DMA
  // completion: removed in round 5.)
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // prologue of the first tile: k-tiles 0 and 1 in flight
  static_for<PIECES>([&](auto sc) { dma(sc, I0{}, 0); });
  static_for<PIECES>([&](auto sc) { dma(sc, I1{}, 1); });
  // epilogue scratch: 8 KB per wave past the two staging buffers (never a DMA target)
  char* const Q = L + 2 * STAGE + w * 8192;

  for (;;) {
    int nvb = vb + G, ntm = tm, ntn = tn, nkt0 = kt0, nnk = nku, ntt = tt, ntk = tslice, nge = ge, ngr0 = gr0,
        ngnr = gnr;
    while (nvb < total && !decode(nvb, ntm, ntn, nkt0, nnk, ntt, ntk, nge, ngr0, ngnr)) nvb += G;
    const bool more = nvb < total;
    if (!more) {   // without a next unit: re-stage this one (never consumed)
      ntm = tm;
      ntn = tn;
      nkt0 = kt0;
      nge = ge;
      ngr0 = gr0;
      ngnr = gnr;
    }
    const int nk = nku;
    const int m0 = GR ? gr0 : tm * BM;
    const int mend = GR ? gr0 + gnr : a.M;   // rows past it are not stored
    // k-tile 0 landed: the PIECES youngest vector-memory operations are k-tile 1's DMA or the previous
    // tile's epilogue stores, everything older (k-tile 0) is done.  (The previous tile's last call
    // already read these fragments; reading them again here keeps F0 dead across the epilogue,
    // which would otherwise spill.)
    wait_vm<KA_GB_DRAIN_B1 ? 0 : PIECES>();
    block_sync();
    static_for<NRD>([&](auto sc) { rd2(sc, fa0, fb0, bA00, bB00); });
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    wait_lgkm0();

    // two k-tiles per trip so every buffer index is a compile-time constant (K % 128 == 0: no odd
    // tail).  The last trip stages the next tile's k-tiles 0 and 1 (its offsets replace this
    // tile's, whose last DMA was the previous trip's).
    for (int t = 0; t < nk; t += 2) {
      const bool last = t + 2 >= nk;
      if (last) set_offsets(ntm, ntn, nkt0, nge, ngr0, ngnr);
      iter(I0{}, last ? 0 : t + 2);
      iter(I1{}, last ? 1 : t + 3);
      // the MFMA wait states inside the loop, before its exit: hipcc does not know the asm MFMAs'
      // latency and may copy accumulators (v_accvgpr_mov) on the exit edge, which would read
      // results still in flight (seen: the argmax epilogue's accumulators shuffled before a drain
      // placed after the loop)
      if (last) {
        mfma_drain();
        wait_lgkm0();   // the last call's F0 reads land before the epilogue may reuse those registers
      }
    }
    // epilogue.  acc[i][j][r] = C[n = 16 TN wn + 16 i + 4 grp + r][m = 128 wm + 16 j + r16] of the
    // tile.  bf16 / SwiGLU: the wave's quadrant is transposed through its 8 KB of LDS in row passes
    // into [m][n] rows and stored as whole 16-B lanes instead of 8-B pieces scattered over 16 rows.
#pragma unroll
    for (int i = 0; i < TN; ++i)   // the asm MFMAs' results are read only after mfma_drain's wait states
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
    // the epilogue of a whole tile / split-K slice / the last-arriving tail slice (a lambda called from
    // two branches: merging the tail combine's accumulators back into one path made hipcc keep the
    // whole tile in VGPRs and spill)
    // mode 0: the output of a whole tile / split-K slice; 1: publish this tail slice; 2: the output of
    // the last tail slice from the sum of the published slices
    auto epilogue = [&](int mode) {
      if constexpr (SPLIT) {
        // partial slab rows m, columns n .. n + 3 of the lane's accumulators: 16 B (fp32) / 8 B (bf16)
        // per lane, the 4 lanes of a row contiguous
  #pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int m = m0 + 128 * wm + 16 * j + r16;
          if (m >= a.M) continue;
  #pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int n = tn * BN + 128 * wn + 16 * i + 4 * grp;
            if (n >= a.N) continue;
            const size_t o = ((size_t)(kt0 / (a.kp / BK)) * a.M + m) * a.N + n;
            const f32x4 v = acc[i][j];
            if constexpr (EPI == EPI_P32) *reinterpret_cast<f32x4*>(static_cast<float*>(a.P) + o) = v;
            else *reinterpret_cast<uint2*>(static_cast<bf16_t*>(a.P) + o) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
          }
        }
      } else if constexpr (EPI == EPI_ARGMAX) {
        // lane (r16, grp) holds, for output row m = 128 wm + 16 j + r16, the 32 logits of columns
        // n = 128 wn + 16 i + 4 grp + r (i < 8, r < 4).  Values are compared after bf16 rounding (what
        // the unfused path's bf16 logits hold); i and r ascend, so strict '>' keeps the lowest index.
        float* const Sv = reinterpret_cast<float*>(L + 2 * STAGE);            // [4 waves][128 rows]
        int* const Si = reinterpret_cast<int*>(L + 2 * STAGE + 4 * 128 * 4);
  #pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int m = m0 + 128 * wm + 16 * j + r16;
          const int mi = (a.mask_bits != nullptr && m < a.M) ? a.mask_idx[m] : -1;
          const uint32_t* mrow = mi >= 0 ? a.mask_bits + (size_t)mi * a.mask_words : nullptr;
          float best = -INFINITY;
          int bidx = 0x7fffffff;
  #pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int n0 = tn * BN + 128 * wn + 16 * i + 4 * grp;
            uint32_t bits = 0xfu;
            if (mrow) {   // n0 + vocab_offset is a multiple of 4: the 4 bits share one mask word
              const int gb = n0 + a.vocab_offset;
              bits = (mrow[gb >> 5] >> (gb & 31)) & 0xfu;
            }
            if (n0 >= a.N) bits = 0;
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float x = lo_f(pack2(acc[i][j][r], 0.f));
              if (((bits >> r) & 1u) && x > best) {
                best = x;
                bidx = n0 + r;
              }
            }
          }
  #pragma unroll
          for (int o = 16; o < 64; o <<= 1) {   // the 4 lanes of row r16 (grp 0..3)
            const float ob = __shfl_xor(best, o, 64);
            const int oi = __shfl_xor(bidx, o, 64);
            if (ob > best || (ob == best && oi < bidx)) {
              best = ob;
              bidx = oi;
            }
          }
          if (grp == 0) {
            Sv[w * 128 + 16 * j + r16] = best;
            Si[w * 128 + 16 * j + r16] = bidx;
          }
        }
        wait_lgkm0();   // block_sync is a bare s_barrier: the other waves read these stores after it
        block_sync();
        {   // thread t: tile row t = 128 wm' + rr, from waves 2 wm' (columns 0..127) and 2 wm' + 1
          const int wm2 = tid >> 7, rr = tid & 127, m = m0 + tid;
          float b0 = Sv[(2 * wm2) * 128 + rr], b1 = Sv[(2 * wm2 + 1) * 128 + rr];
          int i0 = Si[(2 * wm2) * 128 + rr], i1 = Si[(2 * wm2 + 1) * 128 + rr];
          if (b1 > b0 || (b1 == b0 && i1 < i0)) {
            b0 = b1;
            i0 = i1;
          }
          if (m < a.M) {
            a.part_val[(size_t)m * a.tiles_n + tn] = b0;
            a.part_idx[(size_t)m * a.tiles_n + tn] = i0;
          }
        }
        // the next tile's epilogue rewrites Sv / Si only after its k-loop's barriers
      } else if constexpr (EPI == EPI_SWIGLU) {
        // quadrant: 128 rows (m) x 64 output columns = 128 B per row, in 2 passes of 64 rows;
        // 16-B chunk index ^ (row & 7).  Groups of 8: v[2 jj] = gate, v[2 jj + 1] = up of column group pp
        const int rl = lane >> 3, cl = lane & 7;
        const int ocol = 128 * tn + 64 * wn + 8 * cl;
        static_for<2>([&](auto pc) {
          constexpr int p = decltype(pc)::value;
          static_for<4>([&](auto ppc) {
            constexpr int pp = decltype(ppc)::value;
            f32x4 v[8];
            const int q[8] = {16 * pp + 4 * p, 16 * pp + 8 + 4 * p, 16 * pp + 4 * p + 1, 16 * pp + 8 + 4 * p + 1,
                              16 * pp + 4 * p + 2, 16 * pp + 8 + 4 * p + 2, 16 * pp + 4 * p + 3, 16 * pp + 8 + 4 * p + 3};
            if (mode == 2) {
              tail_fetch<TN>(a, tt, w, lane, q, v);
            } else {
              static_for<4>([&](auto jc) {
                constexpr int jj = decltype(jc)::value;
                v[2 * jj] = acc[2 * pp][4 * p + jj];
                v[2 * jj + 1] = acc[2 * pp + 1][4 * p + jj];
              });
              if (mode == 1) {
                tail_store<TN>(a, tt, tslice, w, lane, q, v);
                return;
              }
            }
  #pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const f32x4 g = v[2 * jj], u = v[2 * jj + 1];
              float o[4];
  #pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = g[r] / (1.f + __expf(-g[r])) * u[r];
              const int row = 16 * jj + r16, col = 16 * pp + 4 * grp;   // col: bf16 index in the row
              const int ch = (col >> 3) ^ (row & 7);
              *reinterpret_cast<uint2*>(Q + row * 128 + ch * 16 + (col & 4) * 2) =
                  make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
            }
          });
          if (mode == 1) return;
  #pragma unroll
          for (int it = 0; it < 8; ++it) {
            const int row = 8 * it + rl, m = m0 + 128 * wm + 64 * p + row;
            const u32x4 v = *reinterpret_cast<const u32x4*>(Q + row * 128 + ((cl ^ (row & 7)) * 16));
            if (m < mend) *reinterpret_cast<u32x4*>(a.Y + (size_t)m * a.ldy + ocol) = v;
          }
        });
      } else {
        // quadrant: 128 rows (m) x 16 TN columns (n), 256-B LDS rows (2 TN of their 16 chunks used), in
        // 4 passes of 32 rows; 16-B chunk index ^ (row & 15)
        const int rl = lane >> 4, cl = lane & 15;
        const int n = tn * BNT + wn * 16 * TN + 8 * cl;
        static_for<4>([&](auto pc) {
          constexpr int p = decltype(pc)::value;
          static_for<2>([&](auto jc) {   // groups of TN: accumulator column 2 p + jj, all i
            constexpr int jj = decltype(jc)::value;
            f32x4 v8[TN];
            int q[TN];
  #pragma unroll
            for (int i = 0; i < TN; ++i) q[i] = 8 * i + 2 * p + jj;
            if (mode == 2) {
              tail_fetch<TN>(a, tt, w, lane, q, v8);
            } else {
              static_for<TN>([&](auto ic) { v8[decltype(ic)::value] = acc[decltype(ic)::value][2 * p + jj]; });
              if (mode == 1) {
                tail_store<TN>(a, tt, tslice, w, lane, q, v8);
                return;
              }
            }
  #pragma unroll
            for (int i = 0; i < TN; ++i) {
              const f32x4 v = v8[i];
              const int row = 16 * jj + r16, col = 16 * i + 4 * grp;
              const int ch = (col >> 3) ^ (row & 15);
              *reinterpret_cast<uint2*>(Q + row * 256 + ch * 16 + (col & 4) * 2) =
                  make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
            }
          });
          if (mode != 1 && cl < 2 * TN && n < a.N) {
  #pragma unroll
            for (int it = 0; it < 8; ++it) {
              const int row = 4 * it + rl, m = m0 + 128 * wm + 32 * p + row;
              u32x4 v = *reinterpret_cast<const u32x4*>(Q + row * 256 + ((cl ^ (row & 15)) * 16));
              if (m >= mend) continue;
              bf16_t* y = a.Y + (size_t)(GR ? a.out_rows[m] : m) * a.ldy + n;
              if constexpr (EPI == EPI_ADD) {
                const u32x4 rr = *reinterpret_cast<const u32x4*>(a.R + (size_t)m * a.ldy + n);
  #pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = pack2(lo_f(v[q]) + lo_f(rr[q]), hi_f(v[q]) + hi_f(rr[q]));
              }
              *reinterpret_cast<u32x4*>(y) = v;
            }
          }
        });
      }
    };
    // the accumulators are read at one call site (see tail_ticket): a tail slice publishes them (mode
    // 1); the last one to arrive then stores the output from the published slices (mode 2, which
    // reads no accumulator)
    const int mode = (TAILOK && tt >= 0) ? 1 : 0;
    epilogue(mode);
    if (TAILOK && mode == 1 && tail_ticket(a, tt, w, lane)) epilogue(2);
    if (!more) break;
    vb = nvb;
    tm = ntm;
    tn = ntn;
    kt0 = nkt0;
    nku = nnk;
    tt = ntt;
    tslice = ntk;
    ge = nge;
    gr0 = ngr0;
    gnr = ngnr;
  }
  wait_vm<0>();   // the trailing re-stage DMA: nothing may land in LDS after the workgroup ends
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

// Workspace of the split tail: [err + pad 256 B][counters: TAIL_MAX_TILES x 4 waves x 2][slabs]
constexpr int TAIL_MAX_TILES = 1024;
constexpr size_t TAIL_HDR = 256 + (size_t)TAIL_MAX_TILES * 8 * 4;
constexpr size_t tail_slab(int tn) { return (size_t)BM * 32 * tn * 4; }   // one tile's fp32 accumulators
constexpr size_t TAIL_SLAB = tail_slab(8);

// The tail split for T tiles on G persistent workgroups, in k-tile times: the tail's last round
// takes ceil(span / G) slices of ~nkt / s k-tiles; each slice publishes its fp32 tile and the last
// arriving one reads all s back (XCD-local L2) before its epilogue.
// Returns s (1: no split) and sets full / tail tiles.
static int choose_tail(int T, int G, int nkt, size_t ws_bytes, int& full, int& tail, size_t slab = TAIL_SLAB) {
  full = T;
  tail = 0;
  const int rem = T % G;
  if (rem == 0 || ws_bytes < TAIL_HDR) return 1;
  const int trips = nkt / 2;
  double best = (double)nkt;   // s = 1: one more round of whole tiles
  int bs = 1;
  for (int s = 2; s <= 8 && s <= trips; ++s) {
    if (TAIL_HDR + (size_t)rem * s * slab > ws_bytes || rem > TAIL_MAX_TILES) break;
    const int span = (rem + 7) / 8 * 8 * s;
    // + publishing the quadrant (~1.5 k-tile times) + the last slice reading s slabs (~1.8 each)
    const double t = (double)((span + G - 1) / G) * (double)((trips + s - 1) / s) * 2.0 + 1.5 + 1.8 * s;
    if (t < best * 0.95) {   // a clear win only: the hand-off's cost model is coarse
      best = t;
      bs = s;
    }
  }
  if (bs > 1) {
    full = T - rem;
    tail = rem;
  }
  return bs;
}

// Tile width for the plain / residual epilogues: the 192-row W tile (TN 6) when the 256-wide tiles
// leave a fractional last round that the 192-wide ones fill (QKV, N = 6144, at M = 4096: 384 tiles =
// 1.5 rounds vs 512 = 2 rounds of 3/4 the work).  Cost in rounds of a 256 x 256 tile: whole rounds,
// plus a last partial round at ~0.5 + 0.65 x its fill (the split tail: measured 0.62 of a round at a
// 1/8 fill, 0.82 at 1/2), the 192 tile's round at 0.78 (3/4 of the MFMAs, a little less staging
// reuse): QKV at M = 4096 runs 167 us on 192-wide tiles vs 204 on 256-wide, at M = 2944 152 vs 169
// (profiles/r5/gemm_big_tn/).  KA_GB_TN=6|8 forces a width where it applies.
static int choose_tn(int M, int N, int epi, int G) {
  if ((epi != EPI_BF16 && epi != EPI_ADD) || N % 192 != 0) return 8;
  static int force = -1;
  if (force < 0) {
    const char* e = getenv("KA_GB_TN");
    force = e ? atoi(e) : 0;
  }
  if (force == 6 || force == 8) return force;
  const int tm = (M + BM - 1) / BM;
  auto cost = [&](int tiles, double unit, bool tail) {
    const int whole = tiles / G, rem = tiles % G;
    const double part = rem ? (tail ? std::min(1.0, 0.5 + 0.65 * rem / (double)G) : 1.0) : 0.0;
    return (whole + part) * unit;
  };
  // TN 6 runs without the split tail (launch): its last partial round costs a whole one
  return cost(tm * (N / 192), 0.78, false) < cost(tm * ((N + 255) / 256), 1.0, true) ? 6 : 8;
}

template <int EPI, int TN>
static int launch(const Args& a0, hipStream_t st, void* ws = nullptr, size_t ws_bytes = 0) {
  using GE = Geo<TN>;
  static bool attr = false;
  auto kern = &gemm256_kernel<EPI, TN>;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              GE::LDS_TOTAL);
    attr = true;
  }
  Args a = a0;
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = EPI == EPI_SWIGLU ? a.I / 128 : (a.N + GE::BN - 1) / GE::BN;
  const int split = (EPI == EPI_P32 || EPI == EPI_P16) ? a.split : 1;
  const int tiles = a.tiles_m * a.tiles_n;
  // one workgroup per CU (the LDS allows no more); a persistent grid is a multiple of 8 (XCDs)
  const int cus = num_cus() & ~7;
  int total = tiles * split;
  a.full = tiles;
  a.tail_s = 1;
  a.tail_tiles = 0;
  a.span = 0;
  // the split tail runs on the 256-wide tile only.  (The wrong rows first blamed on TN 6 tails came
  // from the clamped duplicate-address DMA rows fixed in set_offsets: profiles/r5/gemm_big_clamp/.)
  // choose_tn prices TN 6 without a tail, and at M = 2944, N = 6144 it costs the same (two rounds of
  // 0.78), so the 192-wide path stays the simpler one.
  if ((EPI == EPI_BF16 || EPI == EPI_SWIGLU || EPI == EPI_ADD) && TN == 8) {
    a.tail_s = choose_tail(tiles, cus, a.K / BK, ws ? ws_bytes : 0, a.full, a.tail_tiles, tail_slab(TN));
    if (a.tail_s > 1) {
      char* base = static_cast<char*>(ws);
      a.err = reinterpret_cast<int*>(base);
      a.cnt = reinterpret_cast<int*>(base + 256);
      a.slab = reinterpret_cast<float*>(base + TAIL_HDR);
      a.span = (a.tail_tiles + 7) / 8 * 8 * a.tail_s;
      total = a.full + a.span;
    }
  }
  const int grid = total <= cus ? total : cus;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), GE::LDS_TOTAL, st, a);
  return (int)hipGetLastError();
}

// grouped: tiles_m = the chunk table's entries (an upper bound of the chunks the routing produces:
// unused entries are skipped), no split tail
template <int EPI>
static int launch_grouped(const Args& a0, hipStream_t st) {
  static bool attr = false;
  auto kern = &gemm256_kernel<EPI, 8, true>;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              Geo<8>::LDS_TOTAL);
    attr = true;
  }
  Args a = a0;
  a.tiles_n = EPI == EPI_SWIGLU ? a.I / 128 : a.N / BN;
  a.full = a.tiles_m * a.tiles_n;
  a.tail_s = 1;
  a.tail_tiles = 0;
  a.span = 0;
  const int cus = num_cus() & ~7;
  const int total = a.full;
  hipLaunchKernelGGL(kern, dim3(total <= cus ? total : cus), dim3(NT), Geo<8>::LDS_TOTAL, st, a);
  return (int)hipGetLastError();
}

template <int EPI>
static int launch_tn(const Args& a, hipStream_t st, void* ws, size_t ws_bytes) {
  if constexpr (EPI == EPI_BF16 || EPI == EPI_ADD) {
    if (choose_tn(a.M, a.N, EPI, num_cus() & ~7) == 6) return launch<EPI, 6>(a, st, ws, ws_bytes);
  }
  return launch<EPI, 8>(a, st, ws, ws_bytes);
}

}  // namespace gb

// Y = X W^T (+ R).  epi: 0 bf16 Y [M, ldy]; 3 SwiGLU: W = [gate; up] rows (N = 2I), Y [M, ldy] gets
// silu(x gate^T) * (x up^T), I columns; 4: Y = X W^T + R (R [M, ldy], may alias Y).
// Requirements: K % 128 == 0, N % 128 == 0 (SwiGLU: I % 128 == 0), 16-B aligned rows (ldx % 8 == 0).
// ws (optional, zero-filled once, ka_gemm_big_ws_bytes): the split tail's counters and slabs; the
// kernel leaves the counters zeroed again.  nullptr: no split tail.
extern "C" int ka_gemm_big(void* Y, const void* R, const void* X, const void* W, int M, int N, int K, int ldx, int ldy,
                           int epi, int gm, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 128 != 0 || N % 128 != 0 || ldx % 8 != 0 || ldy % 8 != 0) return (int)hipErrorInvalidValue;
  // 32-bit buffer-descriptor record counts (past them loads return zeros, silently)
  if ((double)M * ldx * 2.0 >= 2147483648.0 - 4096.0 || (double)N * K * 2.0 >= 2147483648.0 - 4096.0)
    return (int)hipErrorInvalidValue;
  gb::Args a{static_cast<const bf16_t*>(X), static_cast<const bf16_t*>(W), static_cast<bf16_t*>(Y),
             static_cast<const bf16_t*>(R), M, N, K, ldx, ldy, 0, 0, gm > 0 ? gm : 8, N / 2};
  switch (epi) {
    case gb::EPI_BF16: return gb::launch_tn<gb::EPI_BF16>(a, stream, ws, ws_bytes);
    case gb::EPI_SWIGLU:
      if (N % 256 != 0) return (int)hipErrorInvalidValue;
      return gb::launch<gb::EPI_SWIGLU, 8>(a, stream, ws, ws_bytes);
    case gb::EPI_ADD:
      if (R == nullptr) return (int)hipErrorInvalidValue;
      return gb::launch_tn<gb::EPI_ADD>(a, stream, ws, ws_bytes);
  }
  return (int)hipErrorInvalidValue;
}

// Grouped (MoE) GEMM over expert-sorted rows (ka_moe_sort): for every chunk c < chunks of the table
// (expert e, first row r0, n rows), Y rows of X[r0 .. r0 + n) W[e]^T.  W [groups][N][K] (SwiGLU:
// [groups][2I][K], gate rows then up rows per expert).  epi 0: Y [*, ldy] row out_rows[r] for sorted
// row r; epi 3: Y [M, ldy] sorted row r = silu(x gate^T) * (x up^T).  X [M, ldx] (M = the sorted rows'
// capacity).  Requirements: K % 128 == 0, N % 256 == 0, groups * N * K * 2 and M * ldx * 2 < 2^31 - 4 KB.
extern "C" int ka_gemm_big_grouped(void* Y, const void* X, const void* W, const int* chunk_tab, int chunks,
                                   const int* out_rows, int M, int N, int K, int ldx, int ldy, int groups, int epi,
                                   hipStream_t stream) {
  if (M <= 0 || N <= 0 || chunks <= 0) return 0;
  if (K % 128 != 0 || N % 256 != 0 || ldx % 8 != 0 || ldy % 8 != 0 || groups < 1 || chunk_tab == nullptr ||
      (double)groups * N * K * 2.0 >= 2147483648.0 - 4096.0 || (epi == gb::EPI_BF16 && out_rows == nullptr))
    return (int)hipErrorInvalidValue;
  // the X descriptor's record count is 32-bit too: past it the buffer loads read zeros, silently
  if ((double)M * ldx * 2.0 >= 2147483648.0 - 4096.0) return (int)hipErrorInvalidValue;
  gb::Args a{static_cast<const bf16_t*>(X), static_cast<const bf16_t*>(W), static_cast<bf16_t*>(Y), nullptr, M, N, K,
             ldx, ldy, chunks, 0, 8, N / 2};
  a.chunk_tab = chunk_tab;
  a.out_rows = out_rows;
  a.groups = groups;
  switch (epi) {
    case gb::EPI_BF16: return gb::launch_grouped<gb::EPI_BF16>(a, stream);
    case gb::EPI_SWIGLU: return gb::launch_grouped<gb::EPI_SWIGLU>(a, stream);
  }
  return (int)hipErrorInvalidValue;
}

// Workspace bytes of ka_gemm_big's split tail: 512 tile slabs (128 MB; choose_tail keeps tail tiles x
// slices within the workspace it is given).
extern "C" size_t ka_gemm_big_ws_bytes() { return gb::TAIL_HDR + (size_t)512 * gb::TAIL_SLAB; }

// The split that ka_gemm_big would use (tests / diagnostics): tail_s, and the whole / tail tile counts.
extern "C" int ka_gemm_big_plan(int M, int N, int epi, int K, size_t ws_bytes, int* full, int* tail) {
  const int G = gb::num_cus() & ~7;
  const int TN = gb::choose_tn(M, N, epi, G);
  const int tm = (M + gb::BM - 1) / gb::BM, tn = epi == gb::EPI_SWIGLU ? N / 256 : (N + 32 * TN - 1) / (32 * TN);
  if (TN != 8) {   // no split tail on 192-wide tiles (launch)
    *full = tm * tn;
    *tail = 0;
    return 1;
  }
  return gb::choose_tail(tm * tn, G, K / gb::BK, ws_bytes, *full, *tail, gb::tail_slab(TN));
}

// The tile width ka_gemm_big runs (M, N, epi) with: 8 (256 W rows) or 6 (192 W rows).
extern "C" int ka_gemm_big_tn(int M, int N, int epi) { return gb::choose_tn(M, N, epi, gb::num_cus() & ~7); }

// Error word of the split tail (a slice that waited ~0.1 s for the others); cleared by the read.
extern "C" int ka_gemm_big_err(void* ws, hipStream_t stream) {
  int v = 0;
  if (ws == nullptr) return 0;
  (void)hipMemcpyAsync(&v, ws, 4, hipMemcpyDeviceToHost, stream);
  (void)hipStreamSynchronize(stream);
  if (v) (void)hipMemsetAsync(ws, 0, 4, stream);
  return v;
}

// Split-K partials: P[ks][M][N] = X[:, ks kp : (ks + 1) kp] W[:, same]^T with kp = K / split, fp32
// (bf16_out = 0) or bf16 (1), for a consumer that fuses the reduction (ops.SplitK).
// Requirements: K % (128 split) == 0, N % 128 == 0, ldx % 8 == 0.
extern "C" int ka_gemm_big_splitk(void* P, const void* X, const void* W, int M, int N, int K, int ldx, int split,
                                  int bf16_out, int gm, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (split < 1 || K % (128 * split) != 0 || N % 128 != 0 || ldx % 8 != 0 || P == nullptr)
    return (int)hipErrorInvalidValue;
  gb::Args a{static_cast<const bf16_t*>(X), static_cast<const bf16_t*>(W), nullptr, nullptr, M, N, K, ldx, 8, 0, 0,
             gm > 0 ? gm : 8, N / 2};
  a.split = split;
  a.kp = K / split;
  a.P = P;
  return bf16_out ? gb::launch<gb::EPI_P16, 8>(a, stream) : gb::launch<gb::EPI_P32, 8>(a, stream);
}

extern "C" int ka_argmax_finish(int* out_idx, float* out_val, const float* part_val, const int* part_idx, int rows,
                                int slices, int vocab_offset, hipStream_t stream);

// Workspace bytes of ka_gemm_big_argmax: per-row, per-tile (max, index).
extern "C" size_t ka_gemm_big_argmax_ws(int M, int N) { return (size_t)M * ((N + gb::BN - 1) / gb::BN) * 8; }

// Fused LM head + greedy sampling: out_idx[m] = vocab_offset + argmax over allowed n of bf16(X W^T)[m, n]
// (lowest index on ties; mask row mask_idx[m], < 0 or mask_bits == nullptr = all tokens allowed),
// out_val[m] its value (for the vocab-parallel combine under TP).  The [M, N] logits are never written.
extern "C" int ka_gemm_big_argmax(int* out_idx, float* out_val, const void* X, const void* W, int M, int N, int K,
                                  int ldx, const uint32_t* mask_bits, const int* mask_idx, int mask_words,
                                  int vocab_offset, void* workspace, hipStream_t stream) {
  if (M <= 0) return 0;
  if (K % 128 != 0 || N % 128 != 0 || ldx % 8 != 0 || vocab_offset % 4 != 0 || workspace == nullptr ||
      (mask_bits != nullptr && mask_idx == nullptr))
    return (int)hipErrorInvalidValue;
  const int tiles_n = (N + gb::BN - 1) / gb::BN;
  float* pv = static_cast<float*>(workspace);
  int* pi = reinterpret_cast<int*>(pv + (size_t)M * tiles_n);
  gb::Args a{static_cast<const bf16_t*>(X), static_cast<const bf16_t*>(W), nullptr, nullptr, M, N, K, ldx, 8, 0, 0,
             8, N / 2, mask_bits, mask_idx, mask_words, vocab_offset, pv, pi};
  int rc = gb::launch<gb::EPI_ARGMAX, 8>(a, stream);
  if (rc != 0) return rc;
  return ka_argmax_finish(out_idx, out_val, pv, pi, M, tiles_n, vocab_offset, stream);
}
