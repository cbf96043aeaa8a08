// Persistent batch-1 decode: every decoder layer of a Llama model (TP = 1, head_dim 128, KV block 16)
// for ONE token in ONE launch (the serving path's B = 1 hipGraph replays it once per token).
//
// Why: at batch 1 the chain of ~7 kernels per layer (norm, QKV GEMV, fused RoPE + attention, O GEMV,
// norm, gate_up GEMV, down GEMV + SiLU) pays a launch boundary, a ramp and a tail per kernel — the
// layer took ~110 us against ~71 us of weight streaming at the HBM rate (docs/PERFORMANCE.md).  Here
// one workgroup per CU (the dynamic LDS request admits no second one) walks the layers; the weight
// stream of each phase is ISSUED before the grid-wide wait that precedes it (the register ring of
// the row-streaming GEMV is filled, then the workgroup waits for the activations), so a phase's
// first weight bytes are in flight while the previous phase drains — the "stream ahead of the data
// dependencies" structure (MI355X_MICROARCH.md, Persistent kernels).
//
// Phases of layer l (G workgroups x 8 waves; group h = the G / hkv workgroups of KV head h):
//   P1  every workgroup: RMSNorm of the fp32 residual -> x (LDS); the group's waves compute the QKV
//       rows of head h (its 4 q heads, k, v) -> qkv (sc1 stores); group arrival counter
//   P2  the group's first workgroup, after its group's arrivals: RoPE on q / k, KV append, attention
//       over the context + the new token (exp2 online softmax, 8 waves over 16-token blocks, merged
//       through LDS) -> attn; the others go straight to the grid barrier with their O rows issued
//   P3  O GEMV rows of each wave -> residual += (each residual element owned by one wave)
//   P4  RMSNorm of the residual -> x; gate + up rows -> act = silu(g) * u
//   P5  down GEMV rows (K = I) -> residual +=
// Grid barriers between the phases (B: after P2, C: after P3, D: after P4, E: after P5): one
// monotonic counter, lane 0 of each workgroup adds behind a workgroup barrier after every wave's
// `s_waitcnt vmcnt(0)`, one lane polls with relaxed agent-scope loads; all activations that cross
// workgroups are written and read with agent-scope (sc1) accesses — the MI355X_MICROARCH.md hand-off
// table, row 1 (no fence).  Spins are bounded: a workgroup that is never scheduled (the GPU shared
// with another kernel) sets the error word instead of hanging the chip, and every later wait skips.
// Weights stream with non-temporal 16-B loads (read once per token).
#include "common.h"

namespace pd {

constexpr int NT = 512, NW = NT / 64, RING = 16, HD = 128, KBS = 16;

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
  const bf16_t* h0;     // [H] the token's embedding
  bf16_t* h_out;        // [H] the residual stream after the last layer (bf16)
  bf16_t* k_cache;      // [L][NB][hkv][16][128]
  bf16_t* v_cache;      // [L][NB][hkv][128][16]
  size_t cache_layer;   // elements per layer of each cache
  const int* pos;       // [1] position of the token
  const int* slot;      // [1] its cache slot
  const int* bt;        // [max_blocks] the sequence's block table
  const int* ctx;       // [1] context length including the token
  const float* cos_sin; // [max_pos][128]
  float* res;           // workspace: [H] fp32 residual
  bf16_t* qkv;          // [(hq + 2 hkv) 128]
  bf16_t* attn;         // [hq 128]
  bf16_t* act;          // [I]
  int* sync;            // [0] grid arrivals, [1 .. hkv] group arrivals, [63] error word (zeroed per launch)
  unsigned long long* stamps;   // diagnostics (nullptr: off): [G workgroups][L][16] s_memrealtime (100 MHz)
};

KA_DEV float ld_sc1(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
KA_DEV void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
KA_DEV uint32_t ld_sc1u(const bf16_t* p) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
KA_DEV void st_sc1u(bf16_t* p, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Arrival: every wave's stores drained, a workgroup barrier, then one lane adds (MI355X_MICROARCH.md
// hand-off table, row 1: the add comes after the wait of every wave it signals for).
KA_DEV void arrive(int* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
KA_DEV void arrive_wait(int* cnt, int target, int* err) {
  arrive(cnt);
  wait_for(cnt, target, err);
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

// One wave's weight stream over `n` rows of length K (row(i) -> global row index): 1 KB per load
// instruction (64 lanes x 16 B along K) by LDS-DMA (`buffer_load_dwordx4 ... lds`) into the wave's own
// RING-slot LDS ring, so the bytes in flight cost no VGPRs (a register ring of the same depth spilled).
// start() issues the first RING pieces (before the wait for the activations); run() waits for the
// oldest piece (a static vmcnt: exactly RING pieces are always outstanding, the tail re-reads the last
// chunk), reads it back (each lane its own 16 B), dots it with x in LDS and refills the slot.  Row
// results stay in registers (lane i holds row i: no store may sit between the counted loads) and
// are returned by run(); the caller writes them after drain().
template <class RowFn>
struct Stream {
  const bf16_t* W;
  int K, KC, total, lane;
  RowFn row;
  uint32_t nbytes;
  uint32_t ring;   // LDS byte address of this wave's ring (wave-uniform)
  int issued;
  // wave-uniform part of piece j's byte offset (row start + chunk) -> soffset; the lane's 16 B -> voffset
  KA_DEV uint32_t soff(int j) const {
    const int jj = min(j, total - 1);
    const int i = jj / KC, c = jj - i * KC;
    return __builtin_amdgcn_readfirstlane(((uint32_t)row(i) * (uint32_t)K + (uint32_t)(c * 512)) * 2u);
  }
  KA_DEV void issue(int j) {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(ring + (uint32_t)(j % RING) * 1024u), so = soff(j);
    const uint32_t off = (uint32_t)lane * 16u;
    // rebuild the descriptor from wave-uniform (readfirstlane) halves so it lives in SGPRs
    const uint64_t wp = (uint64_t)(uintptr_t)W;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)wp),
                   hi = __builtin_amdgcn_readfirstlane((uint32_t)(wp >> 32)),
                   nb = __builtin_amdgcn_readfirstlane(nbytes);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>((uintptr_t)(((uint64_t)hi << 32) | lo)), (short)0, (int)nb, 0x00020000);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(dst), "v"(off), "s"(rs), "s"(so)
                 : "memory");
  }
  KA_DEV void start() {
    issued = 0;
    if (total <= 0) return;
#pragma unroll
    for (int r = 0; r < RING; ++r) issue(issued++);
  }
  KA_DEV float run(const uint4* xs) {
    float mine = 0.f;
    if (total <= 0) return mine;
    float acc = 0.f;
    int cc = 0, ri = 0;
    for (int j = 0; j < total; ++j) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RING - 1) : "memory");   // piece j has landed
      uint4 w;
      const uint32_t src = ring + (uint32_t)(j % RING) * 1024u + (uint32_t)lane * 16u;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(src) : "memory");
      issue(issued++);   // the slot is free again: refill it RING pieces ahead
      acc = dot8(w, xs[cc * 64 + lane], acc);
      if (++cc == KC) {
        cc = 0;
        float v = acc;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == ri) mine = v;
        ++ri;
        acc = 0.f;
      }
    }
    return mine;
  }
  KA_DEV void drain() const { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
};
template <class RowFn>
KA_DEV Stream<RowFn> make_stream(const bf16_t* W, int N, int K, int n, int lane, uint32_t ring, RowFn row) {
  Stream<RowFn> s{W, K, K / 512, n * (K / 512), lane, row, (uint32_t)N * (uint32_t)K * 2u, ring, 0};
  return s;
}

// x[i] = bf16(res[i] * rstd * g[i]) into LDS (every workgroup; res read with sc1 loads)
KA_DEV void rmsnorm_to_lds(const Args& a, const bf16_t* g, bf16_t* xs, float* red) {
  const int H = a.H;
  float ss = 0.f;
  for (int i = threadIdx.x; i < H; i += NT) {
    const float v = ld_sc1(a.res + i);
    ss += v * v;
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) tot += red[w];
  const float rstd = rsqrtf(tot / (float)H + a.eps);
  for (int i = threadIdx.x; i < H; i += NT) xs[i] = f2bf(ld_sc1(a.res + i) * rstd * bf2f(g[i]));
  __syncthreads();
}

// LDS layout (bytes): x / act staging [0, 28 KB) (the attention leader's scratch reuses it: x is dead
// between the QKV rows and the O rows); the waves' weight rings [28 KB, 28 KB + 8 x RING KB); the norm
// reduction at the end.  > 80 KB: one workgroup per CU.
constexpr int LDS_X = 0, LDS_ATT = 0, LDS_RING = 28 * 1024, LDS_RED = LDS_RING + NW * RING * 1024;
constexpr int LDS_BYTES = LDS_RED + 64;

__global__ __launch_bounds__(NT, 1) void decode_layers_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds_u4[];
  char* const lds = reinterpret_cast<char*>(lds_u4);
  bf16_t* const xs = reinterpret_cast<bf16_t*>(lds + LDS_X);
  const uint4* const xs4 = reinterpret_cast<const uint4*>(lds + LDS_X);
  float* const red = reinterpret_cast<float*>(lds + LDS_RED);
  // this wave's LDS-DMA weight ring (LDS byte address; dynamic LDS is the kernel's only LDS object)
  const uint32_t ring = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)lds_u4 + LDS_RING + (threadIdx.x >> 6) * RING * 1024);
  const int G = gridDim.x, wg = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gw = wg * NW + wave, nwaves = G * NW;
  const int H = a.H, hq = a.hq, hkv = a.hkv, I = a.I, Gq = hq / hkv;
  const int per_group = G / hkv, grp = wg / per_group, in_grp = wg - grp * per_group;
  const int qkv_rows = (Gq + 2) * HD;                       // rows of one KV head's group
  const int qkv_per_wave = (qkv_rows + per_group * NW - 1) / (per_group * NW);
  const int h_per_wave = (H + nwaves - 1) / nwaves;         // O / down rows = owned residual elements
  const int i_per_wave = (I + nwaves - 1) / nwaves;         // gate (and up) rows
  int* const gcnt = a.sync;
  int* const err = a.sync + 63;
  int nbar = 0;   // grid barriers passed

  // residual := the embedding (each wave initialises the elements it owns)
  const int own0 = gw * h_per_wave, own1 = min(H, own0 + h_per_wave);
  for (int r = own0 + lane; r < own1; r += 64) st_sc1(a.res + r, bf2f(a.h0[r]));
  arrive(gcnt);

  const int qv0 = (in_grp * NW + wave) * qkv_per_wave;
  const int nq = max(0, min(qkv_rows, qv0 + qkv_per_wave) - qv0);
  auto qkv_row = [=](int i) {   // group-local row -> row of wqkv (q heads of the group, its k, its v)
    const int r = qv0 + i;
    return r < Gq * HD ? grp * Gq * HD + r : r < (Gq + 1) * HD ? hq * HD + grp * HD + (r - Gq * HD)
                                                            : (hq + hkv) * HD + grp * HD + (r - (Gq + 1) * HD);
  };
  const int no = max(0, own1 - own0);
  auto own_row = [=](int i) { return own0 + i; };
  const int g0 = gw * i_per_wave, ng = max(0, min(I, g0 + i_per_wave) - g0);
  auto gu_row = [=](int i) { return (i & 1) ? I + g0 + (i >> 1) : g0 + (i >> 1); };   // gate, up, gate, ...

  // phase stamps of every workgroup (diagnostics)
  unsigned long long* const st = (a.stamps != nullptr && tid == 0) ? a.stamps + (size_t)wg * a.L * 16 : nullptr;
#define PD_STAMP(k) \
  do {              \
    if (st) st[l * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  for (int l = 0; l < a.L; ++l) {
    const Layer Lw = a.layers[l];
    // ---- P1: norm + QKV rows of the group ----
    // The weight pieces of each phase are issued between the arrival and the wait of the barrier before
    // it: after the arrival (its vmcnt(0) would otherwise hold the arrival back until they landed),
    // in flight while the workgroup waits for the others.
    auto sq = make_stream(Lw.wqkv, (hq + 2 * hkv) * HD, H, nq, lane, ring, qkv_row);
    sq.start();
    wait_for(gcnt, ++nbar * G, err);
    PD_STAMP(0);
    if (st && l > 0) st[(l - 1) * 16 + 12] = st[l * 16];   // the previous layer's barrier E ends here
    rmsnorm_to_lds(a, Lw.ln1, xs, red);
    PD_STAMP(1);
    {
      const float v = sq.run(xs4);
      sq.drain();
      if (lane < nq)   // pairs of rows share a 4-B word: bf16 halves by 2-B sc1 stores
        __hip_atomic_store(reinterpret_cast<unsigned short*>(a.qkv + qkv_row(lane)),
                           __builtin_bit_cast(unsigned short, f2bf(v)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the O rows' weights are issued now: they stream while the group waits and attention runs
    PD_STAMP(2);
    auto so = make_stream(Lw.wo, H, hq * HD, no, lane, ring, own_row);
    arrive(a.sync + 1 + grp);   // this workgroup's QKV rows are published
    so.start();
    if (in_grp == 0) {
      // ---- P2: the group's attention (its first workgroup) ----
      wait_for(a.sync + 1 + grp, (l + 1) * per_group, err);
      PD_STAMP(3);
      float* const qf = reinterpret_cast<float*>(lds + LDS_ATT);            // [Gq][128] rotated q
      float* const kn = qf + Gq * HD;                                        // [128] rotated new k
      float* const vn = kn + HD;                                             // [128] new v
      float* const pw = vn + HD;                                             // [NW][Gq][16] probabilities
      float* const mo = pw + NW * Gq * 16;                                   // [NW][Gq] (m, l) + [NW][Gq][128] o
      float* const lo = mo + NW * Gq;
      float* const oo = lo + NW * Gq;
      const int p = a.pos[0], slot = a.slot[0], ctx = a.ctx[0];
      const float* cs = a.cos_sin + (size_t)p * HD;
      // RoPE (neox halves) on the group's q heads and k; v as is
      for (int it = tid; it < (Gq + 2) * (HD / 2); it += NT) {
        const int hh = it / (HD / 2), i = it - hh * (HD / 2);
        const int base = hh < Gq ? (grp * Gq + hh) * HD : hh == Gq ? (hq + grp) * HD : (hq + hkv + grp) * HD;
        const uint32_t w0 = ld_sc1u(a.qkv + base + (i & ~1)), w1 = ld_sc1u(a.qkv + base + HD / 2 + (i & ~1));
        const float x1 = (i & 1) ? hi_f(w0) : lo_f(w0), x2 = (i & 1) ? hi_f(w1) : lo_f(w1);
        if (hh <= Gq) {
          const float c = cs[i], s = cs[HD / 2 + i];
          float* dst = hh < Gq ? qf + hh * HD : kn;
          // bf16 rounding of the rotated values, as the cache / the unfused kernels hold them
          dst[i] = bf2f(f2bf(x1 * c - x2 * s));
          dst[HD / 2 + i] = bf2f(f2bf(x2 * c + x1 * s));
        } else {
          vn[i] = x1;
          vn[HD / 2 + i] = x2;
        }
      }
      __syncthreads();
      bf16_t* const kc = a.k_cache + (size_t)l * a.cache_layer;
      bf16_t* const vc = a.v_cache + (size_t)l * a.cache_layer;
      const size_t hs = (size_t)KBS * HD;   // elements per (block, head)
      if (slot >= 0 && tid < HD) {          // append the new token (read by the NEXT launches only)
        const int blk = slot / KBS, off = slot % KBS;
        kc[((size_t)blk * hkv + grp) * hs + off * HD + tid] = f2bf(kn[tid]);
        vc[((size_t)blk * hkv + grp) * hs + tid * KBS + off] = f2bf(vn[tid]);
      }
      // cached tokens [0, ctx - 1): wave w takes blocks w, w + NW, ...; lane (hh = lane >> 4, t = lane & 15)
      const int ncached = ctx - 1, nblk = (ncached + KBS - 1) / KBS;
      float m_w = -INFINITY, l_w = 0.f;   // this lane's row hh (lanes of one 16-lane row agree)
      float acc[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};   // o[hh][2 lane + e], hh < 4
      const int hh = lane >> 4, t = lane & 15;
      for (int bi = wave; bi < nblk; bi += NW) {
        const int blk = a.bt[bi];
        const int tok = bi * KBS + t;
        float s = -INFINITY;
        if (hh < Gq && tok < ncached) {
          const bf16_t* kp = kc + ((size_t)blk * hkv + grp) * hs + t * HD;
          const float* qp = qf + hh * HD;
          float d = 0.f;
#pragma unroll
          for (int c = 0; c < HD / 8; ++c) {
            const uint4 k8 = *reinterpret_cast<const uint4*>(kp + c * 8);
            const uint32_t kw[4] = {k8.x, k8.y, k8.z, k8.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) d += qp[c * 8 + 2 * e] * lo_f(kw[e]) + qp[c * 8 + 2 * e + 1] * hi_f(kw[e]);
          }
          s = d * a.scale_log2;
        }
        const float mx = row16_max(s);
        const float mn = fmaxf(m_w, mx);
        const float alpha = mn == -INFINITY ? 1.f : exp2f(m_w - mn);
        const float pr = s == -INFINITY ? 0.f : exp2f(s - mn);
        l_w = l_w * alpha + row16_sum(pr);
        m_w = mn;
        if (hh < Gq) pw[(wave * Gq + hh) * 16 + t] = pr;
        // every lane rescales the o of all Gq rows: fetch each row's alpha from its 16-lane row
        float al[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) al[r] = __shfl(alpha, r * 16, 64);
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // P V: lane owns dims 2 lane, 2 lane + 1 of every row; V block is [dim][16 tokens]
        const int nvalid = min(KBS, ncached - bi * KBS);
        const bf16_t* vp = vc + ((size_t)blk * hkv + grp) * hs + (2 * lane) * KBS;
        const uint4 va0 = *reinterpret_cast<const uint4*>(vp), va1 = *reinterpret_cast<const uint4*>(vp + 8);
        const uint4 vb0 = *reinterpret_cast<const uint4*>(vp + KBS), vb1 = *reinterpret_cast<const uint4*>(vp + KBS + 8);
        const uint32_t v0[8] = {va0.x, va0.y, va0.z, va0.w, va1.x, va1.y, va1.z, va1.w};
        const uint32_t v1[8] = {vb0.x, vb0.y, vb0.z, vb0.w, vb1.x, vb1.y, vb1.z, vb1.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (r >= Gq) break;
          float s0 = acc[0][r] * al[r], s1 = acc[1][r] * al[r];
          const float* pp = pw + (wave * Gq + r) * 16;
#pragma unroll
          for (int tt = 0; tt < 16; ++tt) {
            if (tt < nvalid) {   // slots past the context may hold anything (never multiply them by 0)
              const float pv = pp[tt];
              s0 += pv * ((tt & 1) ? hi_f(v0[tt >> 1]) : lo_f(v0[tt >> 1]));
              s1 += pv * ((tt & 1) ? hi_f(v1[tt >> 1]) : lo_f(v1[tt >> 1]));
            }
          }
          acc[0][r] = s0;
          acc[1][r] = s1;
        }
        __builtin_amdgcn_wave_barrier();
      }
      // per-wave (m, l, o) -> LDS; rows hh < Gq (lane t == 0 of each 16-lane row writes m, l)
      if (t == 0 && hh < Gq) {
        mo[wave * Gq + hh] = m_w;
        lo[wave * Gq + hh] = l_w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (r >= Gq) break;
        oo[(wave * Gq + r) * HD + 2 * lane] = acc[0][r];
        oo[(wave * Gq + r) * HD + 2 * lane + 1] = acc[1][r];
      }
      __syncthreads();
      // merge the waves and the new token: thread -> (row, dim)
      for (int it = tid; it < Gq * HD; it += NT) {
        const int r = it / HD, d = it - r * HD;
        float sn = 0.f;
        for (int k = 0; k < HD; ++k) sn += qf[r * HD + k] * kn[k];
        sn *= a.scale_log2;
        float M = sn;
        for (int w = 0; w < NW; ++w) M = fmaxf(M, mo[w * Gq + r]);
        float den = exp2f(sn - M), num = den * vn[d];
        for (int w = 0; w < NW; ++w) {
          const float mw = mo[w * Gq + r];
          if (mw == -INFINITY) continue;
          const float e = exp2f(mw - M);
          den += e * lo[w * Gq + r];
          num += e * oo[(w * Gq + r) * HD + d];
        }
        const float o = num / den;
        const float o2 = __shfl_xor(o, 1, 64);   // d and d ^ 1 are neighbouring lanes
        if ((d & 1) == 0)
          st_sc1u(a.attn + (grp * Gq + r) * HD + d, pack2(o, o2));
      }
    }
    PD_STAMP(4);
    // ---- P3: O rows -> residual ----
    arrive_wait(gcnt, ++nbar * G, err);
    PD_STAMP(5);
    for (int i = tid; i < hq * HD / 8; i += NT) {   // attn (sc1) -> LDS
      const bf16_t* src = a.attn + i * 8;
      uint4 v;
      v.x = ld_sc1u(src);
      v.y = ld_sc1u(src + 2);
      v.z = ld_sc1u(src + 4);
      v.w = ld_sc1u(src + 6);
      reinterpret_cast<uint4*>(lds + LDS_X)[i] = v;
    }
    __syncthreads();
    {
      const float v = so.run(xs4);
      so.drain();
      if (lane < no) st_sc1(a.res + own0 + lane, ld_sc1(a.res + own0 + lane) + bf2f(f2bf(v)));
    }
    PD_STAMP(6);
    auto sg = make_stream(Lw.w13, 2 * I, H, 2 * ng, lane, ring, gu_row);
    arrive(gcnt);
    sg.start();
    wait_for(gcnt, ++nbar * G, err);
    PD_STAMP(7);
    // ---- P4: norm + gate / up -> act ----
    rmsnorm_to_lds(a, Lw.ln2, xs, red);
    PD_STAMP(8);
    {
      const float v = sg.run(xs4);   // lane 2 k: gate row k, lane 2 k + 1: its up row
      sg.drain();
      const float u = bf2f(f2bf(__shfl_down(v, 1, 64)));
      const float gt = bf2f(f2bf(v));
      if (!(lane & 1) && (lane >> 1) < ng)
        __hip_atomic_store(reinterpret_cast<unsigned short*>(a.act + g0 + (lane >> 1)),
                           __builtin_bit_cast(unsigned short, f2bf(gt / (1.f + __expf(-gt)) * u)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    PD_STAMP(9);
    auto sd = make_stream(Lw.w2, H, I, no, lane, ring, own_row);
    arrive(gcnt);
    sd.start();
    wait_for(gcnt, ++nbar * G, err);
    PD_STAMP(10);
    // ---- P5: down rows -> residual ----
    for (int i = tid; i < I / 8; i += NT) {
      const bf16_t* src = a.act + i * 8;
      uint4 v;
      v.x = ld_sc1u(src);
      v.y = ld_sc1u(src + 2);
      v.z = ld_sc1u(src + 4);
      v.w = ld_sc1u(src + 6);
      reinterpret_cast<uint4*>(lds + LDS_X)[i] = v;
    }
    __syncthreads();
    {
      const float v = sd.run(xs4);
      sd.drain();
      if (lane < no) st_sc1(a.res + own0 + lane, ld_sc1(a.res + own0 + lane) + bf2f(f2bf(v)));
    }
    PD_STAMP(11);
    arrive(gcnt);   // the next layer's QKV pieces are issued before the wait (top of the loop)
  }
#undef PD_STAMP
  wait_for(gcnt, ++nbar * G, err);
  for (int r = own0 + lane; r < own1; r += 64) a.h_out[r] = f2bf(ld_sc1(a.res + r));
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

// Workspace bytes: residual (fp32 H) + qkv + attn + act (bf16) + the sync words.
extern "C" size_t ka_decode_persistent_ws(int H, int hq, int hkv, int I) {
  return 256 + (size_t)H * 4 + (size_t)(hq + 2 * hkv) * 128 * 2 + (size_t)hq * 128 * 2 + (size_t)I * 2 + 1024;
}

// Every layer of a batch-1 decode step (see the header).  layers: device array of L x 6 pointers
// (wqkv, wo, w13, w2, ln1, ln2); pos / slot / ctx: device int [1]; bt: the sequence's block table;
// stamps: nullptr, or [G][L][16] uint64 phase timestamps (diagnostics; G <= the CU count).
// Requirements: head_dim 128, block 16, hq % hkv == 0, hq / hkv <= 4, H % 512 == 0, I % 512 == 0,
// hq * 128 % 512 == 0, the grid (the CU count, rounded down to a multiple of hkv) all resident.
extern "C" int ka_decode_persistent(void* h_out, const void* h0, const void* layers, int L, int H, int hq, int hkv,
                                    int I, float eps, float scale, void* k_cache, void* v_cache, long cache_layer,
                                    const int* pos, const int* slot, const int* bt, const int* ctx,
                                    const float* cos_sin, void* ws, void* stamps, hipStream_t stream) {
  if (L <= 0) return 0;
  if (hq % hkv || hq / hkv > 4 || H % 512 || I % 512 || (hq * 128) % 512 || H > 16384 || I > 16384 ||
      ws == nullptr)
    return (int)hipErrorInvalidValue;
  const int G = (pd::num_cus() / hkv) * hkv;
  if (G < hkv) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pd::decode_layers_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, pd::LDS_BYTES);
    attr = true;
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
  a.res = reinterpret_cast<float*>(w + 256);
  a.qkv = reinterpret_cast<bf16_t*>(w + 256 + (size_t)H * 4);
  a.attn = a.qkv + (size_t)(hq + 2 * hkv) * 128;
  a.act = a.attn + (size_t)hq * 128;
  // the arrival counters and the error word start at zero in every launch (a memset node in the graph)
  hipError_t e = hipMemsetAsync(w, 0, 256, stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(pd::decode_layers_kernel, dim3(G), dim3(pd::NT), pd::LDS_BYTES, stream, a);
  KA_CHECK_LAUNCH();
}

// The error word of the last launch (a barrier wait that ran out: some workgroup never ran), cleared.
extern "C" int ka_decode_persistent_err(void* ws, hipStream_t stream) {
  int v = 0;
  if (ws == nullptr) return 0;
  (void)hipMemcpyAsync(&v, static_cast<char*>(ws) + 63 * 4, 4, hipMemcpyDeviceToHost, stream);
  (void)hipStreamSynchronize(stream);
  return v;
}
