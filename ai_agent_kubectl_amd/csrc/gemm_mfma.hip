// gemm_mfma: LDS-DMA ring MFMA GEMM family for decode batches and small mixed steps,
// Y[M, N] = X[M, K] * W[N, K]^T, bf16 in, fp32 accumulate, fused epilogues.  It runs only where
// the engine-start autotuner (ops/autotune.py) measured it fastest for an (M <= 512, N, K) shape;
// larger M (prefill, big mixed steps) dispatches to hipBLASLt (ops.linear), and the grouped
// variant serves MoE prefill (ops.grouped_linear).
//
// Design (cdna_hip_programming.md §5 "Canonical CDNA GEMM", T1, T2, "glds vs register staging"):
//   * workgroup tile BN weight rows x BM activation rows, BK = 64; waves laid out WN x WM, each
//     wave TN x TM MFMA 16x16x32 tiles.  W is the MFMA A operand and X the B operand, so a lane's
//     four accumulator values are four consecutive output columns (8-B bf16 stores) and, for the
//     interleaved gate_up weight, a lane holds gate and up of the same output element;
//   * both operands are K-contiguous and staged HBM/L2 -> LDS by LDS-DMA (global_load_lds
//     dwordx4): no VGPR round trip, one 16-B DMA per lane.  The LDS image is lane-linear per
//     wave-instruction (8 rows x 128 B); the XOR swizzle (slot = chunk ^ ((row >> 1) & 7)) is
//     applied to the per-lane GLOBAL source address and to the ds_read_b128 address (rule 21), and
//     makes the 16 rows a ds_read_b128 lane group touches land on 16 distinct 16-B bank slots;
//   * an LDS ring with stage t + 2 in flight while stage t is computed, waited for with vmcnt(0)
//     only (KA_GM_SCHED below: LDS-DMA completion is unordered, so a wave never waits while a
//     younger stage of its own is in flight); the barrier after the wait publishes every wave's DMA
//     of the stage and retires the reads of the slot about to be refilled; then ds_read + MFMA;
//   * XCD-aware tile order (T1): consecutive logical tiles share an XCD (bijective remap of the
//     round-robin dispatch) and are grouped GM M-tiles x N so the W and X panels of the blocks
//     running together on one XCD are L2 hits;
//   * split-K over gridDim.z (fp32 or bf16 partial slabs for a fused consumer: RMSNorm, decode
//     attention, SiLU) and epilogues: bf16 store, partial slab, SwiGLU (interleaved gate_up rows,
//     silu(g) * u computed from the accumulators: the [M, 2I] gate_up output never exists).
// KA_HIPCC_FLAGS: -mllvm -amdgpu-mfma-vgpr-form
// (accumulators in VGPRs with in-place MFMAs; the tables in profiles/r2/ were measured with it.  One
// wave per SIMD issues 16x16x32 bf16 MFMAs every 17 clocks in this form, against 27 with the default
// codegen: profiles/r5/mfma_rate/)
#include "common.h"

#include <utility>

namespace gm {

constexpr int BK = 64;

// diagnostic builds only (tools/gemm_bench, wrong results on purpose): leave out the weight DMA (1),
// the activation DMA (2), the MFMAs (4) or the fragment reads (8), to find what bounds a shape
#ifndef KA_GM_ABL
#define KA_GM_ABL 0
#endif


enum Epi : int { EPI_BF16 = 0, EPI_P32 = 1, EPI_P16 = 2, EPI_SWIGLU = 3 };

// LDS-DMA wait schedule of the ring kernel (KA_GM_SCHED).  LDS-DMA pieces of one wave do NOT always
// complete in issue order (profiles/r5/gemm_big_clamp/: a younger piece that hits in L2 can retire
// before an older one), so a counted `s_waitcnt vmcnt(N)` with N > 0 does not prove that the oldest
// pieces have landed.  The only wait that does is vmcnt(0), so the default schedules are built so that
// whenever a wave waits for a stage, that stage is the ONLY one it has in flight:
//   1 (set):  the waves form two sets (w < NW/2, w >= NW/2: one wave of each set per SIMD when
//             NW = 8); stage t is issued whole by set t & 1, three slots.  At step t set t & 1 holds
//             only stage t (its next stage, t + 2, is issued after the barrier) and waits vmcnt(0);
//             the other set holds only stage t + 1 and does not wait.  Same lookahead (stage t + 2
//             issued at step t) and the same DMA pieces per SIMD per step as the counted ring.
//   2 (pair): four slots, stages issued in pairs: at even steps every wave drains (vmcnt(0): stages
//             t, t + 1), one barrier, then issues t + 2, t + 3; odd steps have no wait and no barrier
//             (the even barrier already published stage t + 1 and every wave finished reading the
//             slots refilled there).  Configurations whose four slots do not fit LDS use `set`.
//   0 (counted, rounds 2-5): STAGES slots, vmcnt(PER (STAGES - 2)) + a barrier every step — correct
//             only under in-order completion; kept for A/B measurements (tools/gemm_bench).
#ifndef KA_GM_SCHED
#define KA_GM_SCHED 1
#endif

template <int BN_, int BM_, int WN_, int WM_, int STAGES_, int BK_ = 64>
struct Cfg {
  static constexpr int BN = BN_, BM = BM_, WN = WN_, WM = WM_, KT = BK_;
  static constexpr int NW = WN * WM, NT = 64 * NW;
  static constexpr int TN = BN / WN / 16, TM = BM / WM / 16;
  static constexpr int RB = KT * 2;                                  // bytes per staged row
  static constexpr int A_BYTES = BN * RB, B_BYTES = BM * RB;         // one k-step of W / of X
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int SCHED = KA_GM_SCHED == 2 ? (4 * STAGE_BYTES <= 160 * 1024 ? 2 : 1) : KA_GM_SCHED;
  static constexpr int STAGES = SCHED == 1 ? 3 : SCHED == 2 ? 4 : STAGES_;
  static constexpr int LDS = STAGES * STAGE_BYTES;
  // waves that issue one stage's pieces (set: half of them) and each one's DMAs per k-step
  static constexpr int NI = SCHED == 1 ? NW / 2 : NW;
  static constexpr int GA = A_BYTES / (NI * 64 * 16), GB = B_BYTES / (NI * 64 * 16);
  static_assert(KT == 64 || KT == 32, "k-step is 64 (128-B rows) or 32 (64-B rows)");
  static_assert(TN * WN * 16 == BN && TM * WM * 16 == BM, "tile / wave layout mismatch");
  static_assert(GA * NI * 64 * 16 == A_BYTES && GB * NI * 64 * 16 == B_BYTES, "tile rows must fill whole DMA waves");
  static_assert(SCHED != 1 || NW % 2 == 0, "set schedule: an even wave count");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// 16-B slot of chunk `ch` of staged row `row` (bank-conflict-free ds_read_b128 fragment reads):
// 128-B rows: ch ^ ((row >> 1) & 7); 64-B rows: ch ^ ((row >> 2) & 2)
template <int KT>
KA_DEV int swz(int row, int ch) {
  if constexpr (KT == 64) return ch ^ ((row >> 1) & 7);
  else return ch ^ ((row >> 2) & 2);
}

// DMA source row for staged row r of an n-row operand: r itself, or r % n past the end
KA_DEV int wrap_row(int r, int n) { return r < n ? r : r % n; }

template <int AUX = 0>
KA_DEV void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, AUX);
}

template <int N>
KA_DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `ahead` stages of PER DMAs each are in flight (ahead <= N, static counts)
template <int N, int PER>
KA_DEV void wait_ahead(int ahead) {
  static_assert(N * PER <= 63, "vmcnt immediate");
  if constexpr (N == 0) {
    wait_vm<0>();
  } else {
    if (ahead >= N) wait_vm<N * PER>();
    else wait_ahead<N - 1, PER>(ahead);
  }
}

KA_DEV void block_sync() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// fragment read in asm with an immediate offset: the compiler neither sees it nor counts it, so the
// k-loop's counted lgkmcnt waits (wait_frags) are the whole synchronisation of the fragment registers
template <int OFF>
KA_DEV void lds_rd(bf16x8& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
}
// fragments f[I..N) of one k-half: lds_rd at BASE + I * STRIDE (compile-time immediates)
template <int I, int N, int STRIDE, int BASE>
struct RdFrags {
  static KA_DEV void run(bf16x8* f, uint32_t a) {
    if constexpr (I < N) {
      lds_rd<BASE + I * STRIDE>(f[I], a);
      RdFrags<I + 1, N, STRIDE, BASE>::run(f, a);
    }
  }
};

struct Args {
  const bf16_t* X;   // [M, ldx]
  const bf16_t* W;   // [N, K]
  void* Y;           // EPI_BF16: bf16 [M, ldy]; EPI_SWIGLU: bf16 [M, ldy] (= N / 2 columns)
  void* P;           // EPI_P32 / EPI_P16: [split, M, N]
  int M, N, K, ldx, ldy, kps, tiles_m, tiles_n, gm;
  // grouped (MoE expert) GEMMs: W is [groups, N, K]; group e owns the output rows
  // lists[e * lstride + i], i < counts[e], whose X row is lists[..] / src_div
  const int* counts;
  const int* lists;
  int lstride, src_div, groups;
  int wnt;   // 1: weight DMAs non-temporal (aux = 2) so the streamed weights do not evict X from L2
  // EPI_SWIGLU over a [gate; up] weight (up rows from row swi = I, N = 2I) instead of one whose rows
  // are interleaved in 16-row chunks: the DMA sources gather the interleaved order (0: interleaved)
  int swi;
};

// logical tile -> (m tile, n tile): XCD-contiguous, then GM m-tiles x all n-tiles super-rows
KA_DEV void tile_of(int bid, int nwg, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per = gm * tiles_n;
  const int g = L / per, first = g * gm;
  const int rows = min(gm, tiles_m - first);
  const int in = L - g * per;
  tm = first + in % rows;
  tn = in / rows;
}

// grouped GEMMs: global row chunk `c` (of BM rows, over all groups in order) -> its group's weights,
// output-row list and row count; false past the last group's rows
template <int BM>
KA_DEV bool group_chunk(const Args& a, int c, const bf16_t*& Wg, const int*& rows_of, int& nrows, int& chunk) {
  int e = 0;
  for (; e < a.groups; ++e) {
    const int n = (a.counts[e] + BM - 1) / BM;
    if (c < n) break;
    c -= n;
  }
  if (e == a.groups) return false;
  chunk = c;
  nrows = a.counts[e] - c * BM;
  rows_of = a.lists + (size_t)e * a.lstride + c * BM;
  Wg = a.W + (size_t)e * a.N * a.K;
  return true;
}

#ifdef GM_BSTAMPS
// diagnostic build only (tools/gemm_bench.hip -DGM_BSTAMPS): per-block wall-clock stamps
// (s_memrealtime, 100 MHz) of wave 0 — 0 start, 1 first stage landed, 2 k-loop done, 3 epilogue
// issued — stored by all 64 lanes (vector stores) to [block][stamp][lane]
__device__ unsigned long long* g_bstamps;
#define BSTAMP(i)                                                                                        \
  do {                                                                                                   \
    if (tid < 64) {                                                                                      \
      const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                    \
      g_bstamps[(((size_t)blockIdx.z * gridDim.x + blockIdx.x) * 4 + (i)) * 64 + tid] = t_;              \
    }                                                                                                    \
  } while (0)
#else
#define BSTAMP(i) do {} while (0)
#endif
#ifdef GM_KSTAMP
// diagnostic build only (tools/gemm_bench.hip -DGM_KSTAMP): per-wave shader-clock cycles of the k-loop
// phases summed over the k-steps, [block][wave][4]: wait + barrier, fragment reads + DMA issue + first
// half's MFMA issue + reads wait, second half's MFMA issue, loop overhead
__device__ unsigned long long* g_kstamps;
#endif

// GROUPED: blockIdx.x = n tile, blockIdx.y = chunk of BM rows over all groups in order (the grid
// holds ceil(R / BM) + groups chunks, an upper bound computed on the host without reading counts;
// chunks past the last group's rows exit at once).  X rows are gathered through the row lists by
// the LDS-DMA source addresses, output rows scattered through them in the epilogue.
template <class C, int EPI, bool GROUPED = false>
__global__ __launch_bounds__(C::NT) void gemm_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  char* const lds_c = reinterpret_cast<char*>(lds);
  const int tid = threadIdx.x, lane = tid & 63;
  BSTAMP(0);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % C::WN, wm = wave / C::WN;
  int tmi, tni;
  const bf16_t* Wg = a.W;
  const int* rows_of = nullptr;   // GROUPED: this chunk's output rows
  int nrows = 0;                  // GROUPED: valid rows in this chunk (may exceed BM: clamped on use)
  if constexpr (GROUPED) {
    tni = blockIdx.x;
    // uniform: a block past the last group's rows leaves before any LDS / barrier use
    if (!group_chunk<C::BM>(a, blockIdx.y, Wg, rows_of, nrows, tmi)) return;
  } else {
    tile_of(blockIdx.x, gridDim.x, a.tiles_m, a.tiles_n, a.gm, tmi, tni);
  }
  const int n0 = tni * C::BN, m0 = tmi * C::BM;
  const int kb = blockIdx.z * a.kps;
  const int nk = min(a.kps, a.K - kb) / C::KT;

  // per-lane DMA source offsets (bytes, 32-bit): wave-instruction j covers 1 KB = RPI staged rows.
  // Piece p = j * NI + wi of a stage is issued by issuer wi (set schedule: the wave's index in its set)
  constexpr int CPR = C::RB / 16, RPI = 64 / CPR;   // 16-B chunks per row, rows per instruction
  const int rl = lane / CPR, slot = lane % CPR;
  const int wi = C::SCHED == 1 ? wave % C::NI : wave;
  const int wset = C::SCHED == 1 ? wave / C::NI : 0;   // set schedule: this wave issues the stages t, t & 1 == wset
  uint32_t offA[C::GA], offB[C::GB];
#pragma unroll
  for (int j = 0; j < C::GA; ++j) {
    const int row = (j * C::NI + wi) * RPI + rl;
    const int ch = swz<C::KT>(row, slot);
    // rows past N / M / the list re-read DISTINCT real rows (r % N), never one clamped row: a
    // piece whose lanes share one address intermittently corrupted other LDS-DMA pieces in
    // gemm_big (profiles/r5/gemm_big_clamp/)
    int wr = wrap_row(n0 + row, a.N);
    if (EPI == EPI_SWIGLU && a.swi > 0) {   // interleaved row ri: 16-row chunk ri >> 4 of gate (even) / up (odd)
      const int ri = wr;
      wr = ((ri >> 5) << 4) + (ri & 15) + ((ri >> 4) & 1) * a.swi;
    }
    offA[j] = (uint32_t)(wr * (uint32_t)a.K + kb + ch * 8) * 2u;
  }
#pragma unroll
  for (int j = 0; j < C::GB; ++j) {
    const int row = (j * C::NI + wi) * RPI + rl;
    const int ch = swz<C::KT>(row, slot);
    int src;
    if constexpr (GROUPED) src = rows_of[wrap_row(row, nrows)] / a.src_div;   // padding rows: re-read a real row
    else src = wrap_row(m0 + row, a.M);
    offB[j] = (uint32_t)(src * (uint32_t)a.ldx + kb + ch * 8) * 2u;
  }
  const char* Wb = reinterpret_cast<const char*>(Wg);
  const char* Xb = reinterpret_cast<const char*>(a.X);

  // every kernel argument the k-loop needs is read into registers here, before the loop: under
  // KA_GM_PIPE 2 the asm fragment reads are waited for with a counted lgkmcnt, which a scalar
  // (s_load) kernarg read issued between the reads and that wait would break.  The asm makes wnt an
  // opaque SGPR value, so hipcc cannot rematerialise it from the kernarg segment inside the loop
  // (build.py check_lgkm_windows verifies the k-loop's read windows in the generated assembly).
  int wnt = a.wnt;
  asm volatile("" : "+s"(wnt));
  // the wave's pieces of a stage, W pieces then X pieces; part 0 / 1: the first / second half of that
  // list, -1: all (a call site's part is a constant: the loops fold)
  constexpr int NPC = C::GA + C::GB, HALF_P = NPC / 2;
  auto issue = [&](int stage, int t, int part) {
    char* sa = lds_c + stage * C::STAGE_BYTES;
    char* sb = sa + C::A_BYTES;
    const uint32_t kofs = (uint32_t)t * C::RB;
    const int lo = part == 1 ? HALF_P : 0, hi = part == 0 ? HALF_P : NPC;
    if (!(KA_GM_ABL & 1)) {
      if (wnt) {
#pragma unroll
        for (int j = 0; j < C::GA; ++j)
          if (j >= lo && j < hi) glds16<2>(Wb + offA[j] + kofs, sa + (j * C::NI + wi) * 1024);
      } else {
#pragma unroll
        for (int j = 0; j < C::GA; ++j)
          if (j >= lo && j < hi) glds16(Wb + offA[j] + kofs, sa + (j * C::NI + wi) * 1024);
      }
    }
    if (!(KA_GM_ABL & 2)) {
#pragma unroll
      for (int j = 0; j < C::GB; ++j)
        if (C::GA + j >= lo && C::GA + j < hi) glds16(Xb + offB[j] + kofs, sb + (j * C::NI + wi) * 1024);
    }
  };
  // stage t's pieces, issued by the waves that own it (every wave, or set t & 1)
  auto issue_own = [&](int t, int part = -1) {
    if (t >= nk) return;
    if (C::SCHED == 1 && (t & 1) != wset) return;
    issue(t % C::STAGES, t, part);
  };

  f32x4 acc[C::TN][C::TM];
#pragma unroll
  for (int i = 0; i < C::TN; ++i)
#pragma unroll
    for (int j = 0; j < C::TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read addresses: row (base + i*16 + r16), chunk swz(r16, kk*4 + grp) (the swizzle of
  // a row depends only on row % 16)
  const int r16 = lane & 15, grp = lane >> 4;
  const int rdA = (wn * C::TN * 16 + r16) * C::RB, rdB = (wm * C::TM * 16 + r16) * C::RB;
  const int ch0 = swz<C::KT>(r16, grp) * 16, ch1 = swz<C::KT>(r16, 4 + grp) * 16;

  // k-loop, one barrier per k-step.  After the barrier a wave issues all 2 (TN + TM) fragment reads
  // of its stage at once, then the DMA of stage t + STAGES - 1 (which refills the slot every wave
  // finished reading before the barrier), then the MFMAs: one LDS round trip per k-step is exposed,
  // overlapped with the DMA issue, instead of one per k-half with the DMA issue in front (with one
  // wave per SIMD nothing else hides it): 2-7 % on the decode plan's shapes (profiles/r4/gm_pipe/).
  // KA_GM_PIPE 2 (default): the reads are asm and each k-half's MFMAs wait with a counted lgkmcnt
  // for their own fragments only (hipcc's own bookkeeping emits lgkmcnt(0) before the first MFMA):
  // 0-10 % more.  1: the same order with compiler-issued reads and waits.  A branch-free variant (tail
  // DMAs clamped, one constant vmcnt) measured no better and lost 7 % on 8-step k-loops.
#ifndef KA_GM_PIPE
#define KA_GM_PIPE 2
#endif
  bf16x8 fa[C::KT / 32][C::TN], fb[C::KT / 32][C::TM];
#if KA_GM_PIPE == 2
  // asm fragment reads, in the order fa[0][..], fb[0][..], fa[1][..], ...: k-half kk's MFMAs wait with
  // lgkmcnt((KT / 32 - 1 - kk) (TN + TM)) for their own fragments only (LDS-DMA counts on vmcnt alone)
  static_assert(C::TN + C::TM <= 15, "lgkmcnt immediate");
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) u32x4*)lds;
  auto read_frags_asm = [&](int stage) {
    if (KA_GM_ABL & 8) return;
    const uint32_t base = lds0 + (uint32_t)(stage * C::STAGE_BYTES);
#pragma unroll
    for (int kk = 0; kk < C::KT / 32; ++kk) {
      const uint32_t aA = base + (uint32_t)(rdA + (kk ? ch1 : ch0));
      const uint32_t aB = base + (uint32_t)(rdB + (kk ? ch1 : ch0));
      RdFrags<0, C::TN, 16 * C::RB, 0>::run(fa[kk], aA);
      RdFrags<0, C::TM, 16 * C::RB, C::A_BYTES>::run(fb[kk], aB);
    }
  };
  // the fragment registers of k-half kk are operands of the wait, so no MFMA reading them is
  // scheduled above it
  auto wait_frags = [&](int kk) {   // kk is a constant at both call sites (the branch folds)
    if (kk == 0 && C::KT == 64)
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(C::TN + C::TM) : "memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < C::TN; ++i) asm volatile("" : "+v"(fa[kk][i]));
#pragma unroll
    for (int j = 0; j < C::TM; ++j) asm volatile("" : "+v"(fb[kk][j]));
  };
#endif
  auto read_frags = [&](int stage) {
    const char* sa = lds_c + stage * C::STAGE_BYTES;
    const char* sb = sa + C::A_BYTES;
#pragma unroll
    for (int kk = 0; kk < C::KT / 32; ++kk) {
      const int ch = kk ? ch1 : ch0;
#pragma unroll
      for (int i = 0; i < C::TN; ++i)
        fa[kk][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(sa + rdA + i * 16 * C::RB + ch));
#pragma unroll
      for (int j = 0; j < C::TM; ++j)
        fb[kk][j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(sb + rdB + j * 16 * C::RB + ch));
    }
  };
  auto mma_half = [&](int kk) {
    if (KA_GM_ABL & 4) return;
#pragma unroll
    for (int i = 0; i < C::TN; ++i)
#pragma unroll
      for (int j = 0; j < C::TM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
  };
  auto mma = [&]() {
#pragma unroll
    for (int kk = 0; kk < C::KT / 32; ++kk) mma_half(kk);
  };

  // prologue: STAGES - 1 stages in flight (set / pair schedules: stages 0 and 1)
#pragma unroll
  for (int s = 0; s < (C::SCHED == 0 ? C::STAGES - 1 : 2); ++s) issue_own(s);
  constexpr int PER = C::GA + C::GB;
#if KA_GM_PIPE == 2
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // no scalar load left in flight: lgkm counts in order
#endif
#ifdef GM_KSTAMP
  unsigned long long ks[4] = {0, 0, 0, 0}, kt_e = __builtin_amdgcn_s_memtime();
#endif
  for (int t = 0; t < nk; ++t) {
#ifdef GM_KSTAMP
    const unsigned long long kt_a = __builtin_amdgcn_s_memtime();
    ks[3] += kt_a - kt_e;
#endif
    // stage t landed (this wave's part), then the barrier publishes every wave's part
    if constexpr (C::SCHED == 1) {
      if ((t & 1) == wset) wait_vm<0>();   // stage t is this set's only stage in flight
      block_sync();
    } else if constexpr (C::SCHED == 2) {
      if (!(t & 1)) {                      // stages t, t + 1: this wave's only pieces in flight
        wait_vm<0>();
        block_sync();
      }
    } else if constexpr (C::STAGES >= 3) {
      // counted: stages t+1 .. min(nk-1, t+STAGES-2) of this wave stay in flight
      wait_ahead<C::STAGES - 2, PER>(min(nk - 1 - t, C::STAGES - 2));
      block_sync();
    } else {
      wait_vm<0>();
      block_sync();
    }
#ifdef GM_KSTAMP
    const unsigned long long kt_b = __builtin_amdgcn_s_memtime();
    ks[0] += kt_b - kt_a;
#endif
    if (t == 0) BSTAMP(1);
    // refill: the slot(s) every wave finished reading before the last barrier.  KA_GM_SPLIT_ISSUE: the
    // set / pair schedules issue twice a wave's usual pieces at once, so half of them go after the
    // first k-half's MFMAs (issued while the matrix pipe works) instead of all ahead of them
    auto refill = [&](int part) {
      if constexpr (C::SCHED == 2) {
        if (!(t & 1)) {
          if (part != 1) issue_own(t + 2);
          if (part != 0) issue_own(t + 3);
        }
      } else {
        issue_own(t + C::STAGES - 1, part);
      }
    };
#ifndef KA_GM_SPLIT_ISSUE
#define KA_GM_SPLIT_ISSUE 1
#endif
    constexpr bool split_issue = KA_GM_SPLIT_ISSUE && C::SCHED != 0 && C::KT == 64;
#if KA_GM_PIPE == 2
    read_frags_asm(t % C::STAGES);
    refill(split_issue ? 0 : -1);
    wait_frags(0);
    mma_half(0);
    if constexpr (C::KT == 64) {
      if constexpr (split_issue) {
        __builtin_amdgcn_sched_barrier(0);
        refill(1);
      }
      __builtin_amdgcn_sched_barrier(0);   // the first k-half's MFMAs stay above the second wait
      wait_frags(1);
#ifdef GM_KSTAMP
      const unsigned long long kt_d = __builtin_amdgcn_s_memtime();
      ks[1] += kt_d - kt_b;
#endif
      mma_half(1);
#ifdef GM_KSTAMP
      kt_e = __builtin_amdgcn_s_memtime();
      ks[2] += kt_e - kt_d;
#endif
    }
#else
    read_frags(t % C::STAGES);
    __builtin_amdgcn_sched_barrier(0);
    refill(-1);
    __builtin_amdgcn_sched_barrier(0);
    mma();
#endif
  }
  BSTAMP(2);
#ifdef GM_KSTAMP
  if (lane == 0) {
    unsigned long long* d = g_kstamps + (((size_t)blockIdx.z * gridDim.x + blockIdx.x) * C::NW + wave) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = ks[i] / (unsigned long long)max(nk, 1);
  }
#endif

  // epilogue: acc[i][j][r] = C[n = .. + i*16 + 4*grp + r][m = .. + j*16 + r16]
  const int nb = n0 + wn * C::TN * 16 + 4 * grp;
  const int mb = m0 + wm * C::TM * 16 + r16;
  if constexpr (EPI == EPI_SWIGLU) {
    // W rows interleaved in 16-row chunks (gate c, up c): tiles 2p / 2p+1 are the gate / up rows of
    // output columns (n0 + wn*TN*16)/2 + 16p + 4*grp + r
    static_assert(C::TN % 2 == 0, "SwiGLU epilogue needs gate/up tile pairs");
    static_assert(!GROUPED, "grouped GEMMs store bf16 rows or partial slabs");
    const int cb = (n0 + wn * C::TN * 16) / 2 + 4 * grp;
#pragma unroll
    for (int p = 0; p < C::TN / 2; ++p) {
      const int c = cb + 16 * p;
      if (2 * c >= a.N) continue;
#pragma unroll
      for (int j = 0; j < C::TM; ++j) {
        const int m = mb + j * 16;
        if (m >= a.M) continue;
        const f32x4 g = acc[2 * p][j], u = acc[2 * p + 1][j];
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = g[r] / (1.f + __expf(-g[r])) * u[r];
        *reinterpret_cast<uint2*>(static_cast<bf16_t*>(a.Y) + (size_t)m * a.ldy + c) =
            make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  } else {
    int mrow[C::TM];   // output row of accumulator column j (-1: none)
#pragma unroll
    for (int j = 0; j < C::TM; ++j) {
      if constexpr (GROUPED) {
        const int lr = mb - m0 + j * 16;
        mrow[j] = lr < nrows && lr < C::BM ? rows_of[lr] : -1;
      } else {
        mrow[j] = mb + j * 16 < a.M ? mb + j * 16 : -1;
      }
    }
#pragma unroll
    for (int i = 0; i < C::TN; ++i) {
      const int n = nb + i * 16;
      if (n >= a.N) continue;
#pragma unroll
      for (int j = 0; j < C::TM; ++j) {
        const int m = mrow[j];
        if (m < 0) continue;
        const f32x4 v = acc[i][j];
        if constexpr (EPI == EPI_BF16) {
          *reinterpret_cast<uint2*>(static_cast<bf16_t*>(a.Y) + (size_t)m * a.ldy + n) =
              make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        } else if constexpr (EPI == EPI_P16) {
          *reinterpret_cast<uint2*>(static_cast<bf16_t*>(a.P) + ((size_t)blockIdx.z * a.M + m) * a.N + n) =
              make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        } else {
          *reinterpret_cast<f32x4*>(static_cast<float*>(a.P) + ((size_t)blockIdx.z * a.M + m) * a.N + n) = v;
        }
      }
    }
  }
  BSTAMP(3);
}

// ---- 256 x 256 ping-pong kernel ----------------------------------------------------------------
// Eight waves in two groups of four, one wave of each group per SIMD.  Group g computes W rows
// [128g, 128g + 128) of the tile (its A half-tile is private to it) against X rows [64c, 64c + 64)
// (c = wave & 3).  Group 1 runs one barrier behind group 0, so on every SIMD one wave issues MFMAs
// while its partner reads LDS / issues DMAs (T3/T4 structure, counted vmcnt, raw s_barrier, setprio
// T5).  LDS: 2 buffers x {A0, A1, B0, B1} half-tiles of 128 rows x 128 B (16 KB), XOR-swizzled.
// WAR: a half-tile is refilled only after the last reader group passed the barrier following the
// C phase that consumed its reads (the analysis is in docs/ARCHITECTURE.md).  A 4-phase variant
// (16 MFMAs per phase) measured slower than this 2-phase one (profiles/r2/gemm_pp_phase_stamps.txt:
// ~120 cycles of barrier bubble per interval) and was removed.
struct PP {
  static constexpr int BN = 256, BM = 256, NT = 512;
  static constexpr int HALF = 16384, BUF = 4 * HALF, LDS = 2 * BUF;
};

// Two phases per k-tile (32 MFMAs per C phase: the barrier bubble measured by the s_memtime
// stamps, ~120 cycles per barrier interval, is paid half as often).  Phase a: n-half 0 against
// all of the wave's B columns (R_a: A-sub0 + B = 16 reads), phase b: n-half 1 (R_b: A-sub1).
// DMA schedule (group 0 | group 1), tile t+2 into buffer t & 1:
//   B0 B1 (t+2):  G0 in R_a(t+1) | G1 in R_b(t)       (B of tile t last read by G1's R_a(t))
//   A0 A1 (t+2):  G0 in R_b(t+1) | G1 in R_a(t+1)     (A_g of tile t last read by group g's R_b(t))
// Waits before the barrier that ends interval 4t+7: G0 (end of C_b(t+1)) vmcnt(0), G1 (end of its
// R_b(t+1), which issued B(t+3)) vmcnt(4).
// KA_PP_SAFE 1: the counted vmcnt(4) of G1 is only correct under in-order LDS-DMA completion
// (see KA_GM_SCHED), so group 0 issues every piece instead: B(t+1) in its R_a(t), A(t+1) in its R_b(t)
// (4 pieces per wave and half-tile), and drains vmcnt(0) at the end of C_b(t) — its only pieces in
// flight are tile t+1's — before the barrier ahead of the first read of tile t+1; group 1 never waits.
// WAR: B(t+1) overwrites B(t-1), last read by G1's R_a(t-1) three intervals earlier; A(t+1) overwrites
// A(t-1), last read by G1's R_b(t-1), retired before G1's C_b(t-1), one interval before G0's R_b(t).
// KA_PP_SAFE 2 (default): both groups issue, each drains with nothing younger in flight: G0 as above
// with its half of the pieces (B(t+1) in R_a(t), A(t+1) in R_b(t), vmcnt(0) at the end of C_b(t)); G1
// issues its halves of A(t+1) AND B(t+1) in its R_a(t) and drains vmcnt(0) at the end of its R_b(t),
// the barrier before G0's R_a(t+1).  WAR for G1's B(t+1): B(t-1) was last read by G1's R_a(t-1).
#ifndef KA_PP_SAFE
#define KA_PP_SAFE 2
#endif
template <int EPI, bool GROUPED = false>
__global__ __launch_bounds__(512) void gemm_pp2_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  char* const L = reinterpret_cast<char*>(lds);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, wc = w & 3;
  int tmi, tni;
  const bf16_t* Wg = a.W;
  const int* rows_of = nullptr;
  int nrows = 0;
  if constexpr (GROUPED) {   // as gemm_kernel's grouped mode
    tni = blockIdx.x;
    if (!group_chunk<PP::BM>(a, blockIdx.y, Wg, rows_of, nrows, tmi)) return;
  } else {
    tile_of(blockIdx.x, gridDim.x, a.tiles_m, a.tiles_n, a.gm, tmi, tni);
  }
  const int n0 = tni * PP::BN, m0 = tmi * PP::BM;
  const int kb = blockIdx.z * a.kps;
  const int nk = min(a.kps, a.K - kb) / BK;

  const int r8 = lane >> 3, slot = lane & 7;
  // pieces of a half-tile issued per wave (KA_PP_SAFE: group 0 issues all 16), and the wave's index
  constexpr int PJ = KA_PP_SAFE == 1 ? 4 : 2, PW = KA_PP_SAFE == 1 ? 4 : 8;
  const int wq = KA_PP_SAFE == 1 ? wc : w;
  uint32_t off[4][PJ];
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    const int row = (j * PW + wq) * 8 + r8;
    const uint32_t ch = (uint32_t)(slot ^ ((row >> 1) & 7)) * 8;
    off[0][j] = ((uint32_t)wrap_row(n0 + row, a.N) * (uint32_t)a.K + kb + ch) * 2u;
    off[1][j] = ((uint32_t)wrap_row(n0 + 128 + row, a.N) * (uint32_t)a.K + kb + ch) * 2u;
    uint32_t x0, x1;
    if constexpr (GROUPED) {
      x0 = rows_of[wrap_row(row, nrows)] / a.src_div;
      x1 = rows_of[wrap_row(128 + row, nrows)] / a.src_div;
    } else {
      x0 = wrap_row(m0 + row, a.M);
      x1 = wrap_row(m0 + 128 + row, a.M);
    }
    off[2][j] = (x0 * (uint32_t)a.ldx + kb + ch) * 2u;
    off[3][j] = (x1 * (uint32_t)a.ldx + kb + ch) * 2u;
  }
  const char* Wb = reinterpret_cast<const char*>(Wg);
  const char* Xb = reinterpret_cast<const char*>(a.X);
  auto issue = [&](int h, int t) {
    if (t >= nk) return;
    const char* src = h < 2 ? Wb : Xb;
    char* dst = L + (t & 1) * PP::BUF + h * PP::HALF;
    const uint32_t kofs = (uint32_t)t * (BK * 2);
    if (h < 2 && a.wnt) {
#pragma unroll
      for (int j = 0; j < PJ; ++j) glds16<2>(src + off[h][j] + kofs, dst + (j * PW + wq) * 1024);
    } else {
#pragma unroll
      for (int j = 0; j < PJ; ++j) glds16(src + off[h][j] + kofs, dst + (j * PW + wq) * 1024);
    }
  };

  const int r16 = lane & 15, grp = lane >> 4, sw = (r16 >> 1) & 7;
  const int ch0 = ((0 + grp) ^ sw) * 16, ch1 = ((4 + grp) ^ sw) * 16;
  const int rdA = g * PP::HALF + r16 * 128;
  const int rdB = 2 * PP::HALF + (wc >> 1) * PP::HALF + (64 * (wc & 1) + r16) * 128;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[4][2], fb[4][2];

  auto rd = [&](const char* p) { return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p)); };
  auto read_a = [&](const char* buf, int half) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i][0] = rd(buf + rdA + (4 * half + i) * 2048 + ch0);
      fa[i][1] = rd(buf + rdA + (4 * half + i) * 2048 + ch1);
    }
  };
  auto read_b = [&](const char* buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fb[j][0] = rd(buf + rdB + j * 2048 + ch0);
      fb[j][1] = rd(buf + rdB + j * 2048 + ch1);
    }
  };
  auto mma = [&](int ah) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 * ah + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kk], fb[j][kk], acc[4 * ah + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

#if KA_PP_SAFE == 2
  // prologue: tile 0 (every wave its pieces), drained; then tile 1, drained by each group at its point
  for (int h = 0; h < 4; ++h) issue(h, 0);
  wait_vm<0>();
  for (int h = 0; h < 4; ++h) issue(h, 1);
  block_sync();
  if (g == 1) block_sync();

  for (int t = 0; t < nk; ++t) {
    const char* buf = L + (t & 1) * PP::BUF;
    const int t1 = t == 0 ? nk : t + 1;   // tile 1 was issued whole by the prologue
    // phase a
    read_a(buf, 0); read_b(buf);
    if (g == 0) { issue(2, t1); issue(3, t1); }                                   // B(t+1), G0 half
    else { issue(0, t1); issue(1, t1); issue(2, t1); issue(3, t1); }             // A(t+1), B(t+1), G1 halves
    block_sync();
    mma(0);
    block_sync();
    // phase b
    read_a(buf, 1);
    if (g == 0) { issue(0, t1); issue(1, t1); }                                   // A(t+1), G0 half
    else wait_vm<0>();                     // tile t+1: G1's only pieces in flight
    block_sync();
    mma(1);
    if (g == 0) wait_vm<0>();              // tile t+1: G0's only pieces in flight
    block_sync();
  }
  if (g == 0) block_sync();
#elif KA_PP_SAFE == 1
  // prologue: group 0 issues tile 0, drains it, issues tile 1 (drained at the end of C_b(0))
  if (g == 0) {
    for (int h = 0; h < 4; ++h) issue(h, 0);
    wait_vm<0>();
    for (int h = 0; h < 4; ++h) issue(h, 1);
  }
  block_sync();
  if (g == 1) block_sync();

  for (int t = 0; t < nk; ++t) {
    const char* buf = L + (t & 1) * PP::BUF;
    const int t1 = t == 0 ? nk : t + 1;   // tile 1 was issued whole by the prologue
    // phase a
    read_a(buf, 0); read_b(buf);
    if (g == 0) { issue(2, t1); issue(3, t1); }   // B(t+1): G0 in R_a(t)
    block_sync();
    mma(0);
    block_sync();
    // phase b
    read_a(buf, 1);
    if (g == 0) { issue(0, t1); issue(1, t1); }   // A(t+1): G0 in R_b(t)
    block_sync();
    mma(1);
    if (g == 0) wait_vm<0>();                     // tile t+1: G0's only pieces in flight
    block_sync();
  }
  if (g == 0) block_sync();
#else
  // prologue: tiles 0 and 1 (all four half-tiles each); wait for tile 0; group 1 one barrier behind
  for (int h = 0; h < 4; ++h) issue(h, 0);
  for (int h = 0; h < 4; ++h) issue(h, 1);
  if (nk > 1) wait_vm<8>(); else wait_vm<0>();
  block_sync();
  if (g == 1) block_sync();

  for (int t = 0; t < nk; ++t) {
    const char* buf = L + (t & 1) * PP::BUF;
    const int t1 = t == 0 ? nk : t + 1;   // tile 1 was issued whole by the prologue
    // phase a
    read_a(buf, 0); read_b(buf);
    if (g == 0) { issue(2, t1); issue(3, t1); }   // B(t+1): G0 in R_a(t)
    else { issue(0, t1); issue(1, t1); }          // A(t+1): G1 in R_a(t)
    block_sync();
    mma(0);
    block_sync();
    // phase b
    read_a(buf, 1);
    if (g == 0) { issue(0, t1); issue(1, t1); }   // A(t+1): G0 in R_b(t)
    else { issue(2, t + 2); issue(3, t + 2); }    // B(t+2): G1 in R_b(t)
    if (g == 1) { if (t + 2 < nk) wait_vm<4>(); else wait_vm<0>(); }
    block_sync();
    mma(1);
    if (g == 0) wait_vm<0>();
    block_sync();
  }
  if (g == 0) block_sync();
#endif

  const int nb = n0 + 128 * g + 4 * grp;
  const int mb = m0 + 64 * wc + r16;
  if constexpr (EPI == EPI_SWIGLU) {
    static_assert(!GROUPED, "grouped GEMMs store bf16 rows or partial slabs");
    const int cb = (n0 + 128 * g) / 2 + 4 * grp;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int c = cb + 16 * p;
      if (2 * c >= a.N) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mb + j * 16;
        if (m >= a.M) continue;
        const f32x4 gv = acc[2 * p][j], u = acc[2 * p + 1][j];
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = gv[r] / (1.f + __expf(-gv[r])) * u[r];
        *reinterpret_cast<uint2*>(static_cast<bf16_t*>(a.Y) + (size_t)m * a.ldy + c) =
            make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  } else {
    int mrow[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (GROUPED) {
        const int lr = mb - m0 + j * 16;
        mrow[j] = lr < nrows ? rows_of[lr] : -1;
      } else {
        mrow[j] = mb + j * 16 < a.M ? mb + j * 16 : -1;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n = nb + i * 16;
      if (n >= a.N) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mrow[j];
        if (m < 0) continue;
        const f32x4 v = acc[i][j];
        if constexpr (EPI == EPI_BF16) {
          *reinterpret_cast<uint2*>(static_cast<bf16_t*>(a.Y) + (size_t)m * a.ldy + n) =
              make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        } else if constexpr (EPI == EPI_P16) {
          *reinterpret_cast<uint2*>(static_cast<bf16_t*>(a.P) + ((size_t)blockIdx.z * a.M + m) * a.N + n) =
              make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        } else {
          *reinterpret_cast<f32x4*>(static_cast<float*>(a.P) + ((size_t)blockIdx.z * a.M + m) * a.N + n) = v;
        }
      }
    }
  }
}

template <int EPI>
static int launch_pp_grouped(const Args& a0, int split, hipStream_t st) {
  static bool attr = false;
  auto kern = &gemm_pp2_kernel<EPI, true>;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, PP::LDS);
    attr = true;
  }
  Args a = a0;
  a.tiles_n = (a.N + PP::BN - 1) / PP::BN;
  const int chunks = (a.M + PP::BM - 1) / PP::BM + a.groups;
  hipLaunchKernelGGL(kern, dim3(a.tiles_n, chunks, split), dim3(PP::NT), PP::LDS, st, a);
  return (int)hipGetLastError();
}

template <int EPI>
static int launch_pp(const Args& a0, int split, hipStream_t st) {
  static bool attr = false;
  auto kern = &gemm_pp2_kernel<EPI>;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, PP::LDS);
    attr = true;
  }
  Args a = a0;
  a.tiles_m = (a.M + PP::BM - 1) / PP::BM;
  a.tiles_n = (a.N + PP::BN - 1) / PP::BN;
  hipLaunchKernelGGL(kern, dim3(a.tiles_m * a.tiles_n, 1, split), dim3(PP::NT), PP::LDS, st, a);
  return (int)hipGetLastError();
}

template <class C, int EPI>
static int launch_grouped(const Args& a0, int split, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<C, EPI, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  Args a = a0;
  a.tiles_n = (a.N + C::BN - 1) / C::BN;
  const int chunks = (a.M + C::BM - 1) / C::BM + a.groups;
  hipLaunchKernelGGL((gemm_kernel<C, EPI, true>), dim3(a.tiles_n, chunks, split), dim3(C::NT), C::LDS, st, a);
  return (int)hipGetLastError();
}

// ---- configurations ------------------------------------------------------------------------------
// id: BN x BM tile, WN x WM waves (per-wave tile), ring stages of BK = 64:
//   2: 128 x 256, 2 x 4 waves (64 x 64), 3 stages                (8 waves, 144 KB: 1 block/CU)
//   3: 256 x 128, 4 x 2 waves ( 64 x 64), 3 stages
//   4: 128 x 128, 2 x 2 waves ( 64 x 64), 3 stages                (4 waves, 96 KB: 1 block/CU)
//   5: 128 x  64, 2 x 1 waves ( 64 x 64), 3 stages                (decode M <= 64)
//  12: 128 x 128 with 4 stages
//  19: 256 x 256 2-phase ping-pong (gemm_pp2_kernel), 8 waves in two staggered groups
// (ids are stable across rounds: the removed configurations' numbers are not reused)
#define GM_CFGS(X)               \
  X(2, 128, 256, 2, 4, 3, 64)    \
  X(3, 256, 128, 4, 2, 3, 64)    \
  X(4, 128, 128, 2, 2, 3, 64)    \
  X(5, 128, 64, 2, 1, 3, 64)     \
  X(12, 128, 128, 2, 2, 4, 64)    \
  X(6, 96, 256, 2, 2, 3, 64)      \
  X(8, 192, 128, 2, 2, 3, 64)     \
  GM_EXTRA_CFGS(X)
// measurement-only configurations (tools/gemm_bench -DKA_GM_EXTRA): 32-deep k-steps, deeper rings
#ifdef KA_GM_EXTRA
#define GM_EXTRA_CFGS(X)          \
  X(20, 128, 256, 2, 4, 6, 32)    \
  X(21, 128, 128, 2, 2, 8, 32)    \
  X(22, 256, 128, 4, 2, 6, 32)    \
  X(23, 128, 256, 2, 4, 5, 32)
#else
#define GM_EXTRA_CFGS(X)
#endif

template <class C, int EPI>
static int launch(const Args& a0, int split, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<C, EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  Args a = a0;
  a.tiles_m = (a.M + C::BM - 1) / C::BM;
  a.tiles_n = (a.N + C::BN - 1) / C::BN;
  hipLaunchKernelGGL((gemm_kernel<C, EPI>), dim3(a.tiles_m * a.tiles_n, 1, split), dim3(C::NT), C::LDS, st, a);
  return (int)hipGetLastError();
}

template <int EPI>
static int dispatch(int cfg, const Args& a, int split, hipStream_t st) {
  if (cfg == 19) return launch_pp<EPI>(a, split, st);
  // the SwiGLU epilogue pairs gate / up tiles within a wave: configurations with an odd TN lack it
#define X_(id, bn, bm, wn, wm, s, kt)                                                    \
  if (cfg == id) {                                                                       \
    if constexpr (EPI == EPI_SWIGLU && Cfg<bn, bm, wn, wm, s, kt>::TN % 2 != 0)          \
      return (int)hipErrorInvalidValue;                                                  \
    else                                                                                 \
      return launch<Cfg<bn, bm, wn, wm, s, kt>, EPI>(a, split, st);                      \
  }
  GM_CFGS(X_)
#undef X_
  return (int)hipErrorInvalidValue;
}

template <int EPI>
static int dispatch_grouped(int cfg, const Args& a, int split, hipStream_t st) {
  if (cfg == 19) return launch_pp_grouped<EPI>(a, split, st);
#define X_(id, bn, bm, wn, wm, s, kt) \
  if (cfg == id) return launch_grouped<Cfg<bn, bm, wn, wm, s, kt>, EPI>(a, split, st);
  GM_CFGS(X_)
#undef X_
  return (int)hipErrorInvalidValue;
}

}  // namespace gm

extern "C" int ka_gm_bn(int cfg) {
  if (cfg == 19) return gm::PP::BN;
#define X_(id, bn, bm, wn, wm, s, kt) if (cfg == id) return bn;
  GM_CFGS(X_)
#undef X_
  return -1;
}
extern "C" int ka_gm_bm(int cfg) {
  if (cfg == 19) return gm::PP::BM;
#define X_(id, bn, bm, wn, wm, s, kt) if (cfg == id) return bm;
  GM_CFGS(X_)
#undef X_
  return -1;
}

// Y = X W^T.  epi: 0 bf16 Y [M, ldy]; 1 / 2: fp32 / bf16 split-K slabs P [split, M, N] (Y unused);
// 3: SwiGLU of interleaved gate/up rows -> Y [M, ldy] with N / 2 columns.
// Requirements: K % (64 * split) == 0 (kps = K / split), N % 16 == 0, 16-B aligned rows
// (ldx % 8 == 0); epi 3 needs N % 32 == 0 and split == 1.
extern "C" void ka_splitk_reduce_launch(bf16_t* Y, const float* P, int split, long mn, hipStream_t stream);

// epi 1 with Y != nullptr: the fp32 slabs are then reduced into Y [M, N] (ldy == N) by splitk_reduce.
extern "C" int ka_gemm_mfma(void* Y, void* P, const void* X, const void* W, int M, int N, int K, int ldx, int ldy,
                            int split, int cfg, int epi, int gm, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (split < 1 || K % (64 * split) != 0 || N % 16 != 0 || ldx % 8 != 0 || ka_gm_bn(cfg) < 0)
    return (int)hipErrorInvalidValue;
  if (epi == gm::EPI_SWIGLU && (split != 1 || N % 32 != 0)) return (int)hipErrorInvalidValue;
  if ((epi == gm::EPI_BF16 || epi == gm::EPI_SWIGLU) && split != 1) return (int)hipErrorInvalidValue;
  gm::Args a{static_cast<const bf16_t*>(X), static_cast<const bf16_t*>(W), Y, P, M, N, K, ldx, ldy, K / split,
             0, 0, gm > 0 ? gm : 8};
  a.wnt = M <= 512;   // decode-sized: each weight byte is read once per step (2-4 % faster with nt,
                      // prefill re-reads weight panels from L2 and loses 1-2 %: profiles/r2/gemm_wnt_ab.txt)
  switch (epi) {
    case gm::EPI_BF16: return gm::dispatch<gm::EPI_BF16>(cfg, a, split, stream);
    case gm::EPI_P32: {
      const int rc = gm::dispatch<gm::EPI_P32>(cfg, a, split, stream);
      if (rc || Y == nullptr) return rc;
      if (ldy != N) return (int)hipErrorInvalidValue;
      ka_splitk_reduce_launch(static_cast<bf16_t*>(Y), static_cast<const float*>(P), split, (long)M * N, stream);
      return (int)hipGetLastError();
    }
    case gm::EPI_P16: return gm::dispatch<gm::EPI_P16>(cfg, a, split, stream);
    case gm::EPI_SWIGLU: return gm::dispatch<gm::EPI_SWIGLU>(cfg, a, split, stream);
  }
  return (int)hipErrorInvalidValue;
}

// Y [M, ldy] = silu(X gate^T) * (X up^T) for W = [gate; up] ([2I, K], the model's gate_up layout):
// the decode-size gate_up with its SiLU·mul epilogue (no [M, 2I] output, no separate SiLU kernel).
// Requirements: K % 64 == 0, I % 16 == 0, ldx % 8 == 0; cfg one of GM_CFGS (not 19).
extern "C" int ka_gemm_mfma_swiglu(void* Y, const void* X, const void* W, int M, int I, int K, int ldx, int ldy,
                                   int cfg, hipStream_t stream) {
  if (M <= 0 || I <= 0) return 0;
  if (K % 64 != 0 || I % 16 != 0 || ldx % 8 != 0 || cfg == 19 || ka_gm_bn(cfg) < 0)
    return (int)hipErrorInvalidValue;
  gm::Args a{static_cast<const bf16_t*>(X), static_cast<const bf16_t*>(W), Y, nullptr, M, 2 * I, K, ldx, ldy, K,
             0, 0, 8};
  a.wnt = M <= 512;
  a.swi = I;
  return gm::dispatch<gm::EPI_SWIGLU>(cfg, a, 1, stream);
}

// Grouped (MoE expert) GEMM with device-side routing, no host read of the counts:
//   for e < groups, i < counts[e]: r = lists[e * lstride + i];
//     Y[r, :] = X[r / src_div, :] @ W[e]^T          (epi 0: bf16 Y [R, ldy])
//     P[z, r, :] = split-K slice z of it            (epi 1 / 2: fp32 / bf16 slabs [split, R, N])
// R bounds the row indices (and sizes the launch: ceil(R / BM) + groups row chunks per n tile).
extern "C" int ka_gemm_mfma_grouped(void* Y, void* P, const void* X, const void* W, const int* counts, const int* lists,
                                    int lstride, int src_div, int groups, int R, int N, int K, int ldx, int ldy,
                                    int split, int cfg, int epi, hipStream_t stream) {
  if (R <= 0 || N <= 0 || groups <= 0) return 0;
  if (split < 1 || K % (64 * split) != 0 || N % 16 != 0 || ldx % 8 != 0 || src_div < 1 || ka_gm_bn(cfg) < 0)
    return (int)hipErrorInvalidValue;
  if (epi == gm::EPI_SWIGLU || (epi == gm::EPI_BF16 && split != 1)) return (int)hipErrorInvalidValue;
  gm::Args a{static_cast<const bf16_t*>(X), static_cast<const bf16_t*>(W), Y, P, R, N, K, ldx, ldy, K / split,
             0, 0, 8, counts, lists, lstride, src_div, groups};
  a.wnt = 0;          // grouped expert GEMMs re-read each expert's weights for every row chunk
  switch (epi) {
    case gm::EPI_BF16: return gm::dispatch_grouped<gm::EPI_BF16>(cfg, a, split, stream);
    case gm::EPI_P32: return gm::dispatch_grouped<gm::EPI_P32>(cfg, a, split, stream);
    case gm::EPI_P16: return gm::dispatch_grouped<gm::EPI_P16>(cfg, a, split, stream);
  }
  return (int)hipErrorInvalidValue;
}
