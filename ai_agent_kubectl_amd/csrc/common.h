// Shared helpers for the CDNA4 (gfx950, MI355X) kernels of the kubectl-agent inference engine.
//
// Conventions (see /opt/skills/guides/cdna_hip_programming.md):
//   * wave = 64 lanes; every block size is a multiple of 64;
//   * bf16 is moved as raw 16-bit words and converted with bit ops (round-to-nearest-even, the
//     same rounding torch uses), loads/stores are 16 B per lane wherever the layout allows
//     (Guideline 13: hipcc never vectorises scalar bf16 accesses);
//   * every launcher is `extern "C"`, takes the HIP stream explicitly and returns the hipError_t
//     of the launch, so the Python side (ops/_hip.py, ctypes) can be captured in hipGraphs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define KA_DEV __device__ __forceinline__

KA_DEV float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }

// fp32 -> bf16 round-to-nearest-even (torch's rounding) in one instruction: gfx950's
// v_cvt_pk_bf16_f32 (the bit-twiddling form costs ~6 VALU ops per value, which showed up in the
// VALU-bound softmax / epilogue loops)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
KA_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// two packed bf16 <-> two floats
KA_DEV float lo_f(uint32_t w) { return __uint_as_float(w << 16); }
KA_DEV float hi_f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
KA_DEV uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}

// Cross-lane exchange within a row of 16 lanes by DPP (a VALU operand modifier: no LDS traffic, unlike
// __shfl_xor, which compiles to ds_bpermute_b32).  Controls (gfx9 DPP): quad_perm [1,0,3,2] = 0xB1,
// quad_perm [2,3,0,1] = 0x4E, row_half_mirror = 0x141, row_mirror = 0x140.
template <int CTRL>
KA_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// reduce over the 16 lanes that share (lane >> 4): the column index of an MFMA 16x16 C tile.  Each
// step pairs lanes whose partial results are equal sets of the row, so all 16 lanes end with the
// same (bitwise) value: neighbours, quads, half-rows (mirror within 8), rows (mirror within 16).
KA_DEV float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return v;
}
KA_DEV float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}

// whole-wave reductions: the 16-lane row by DPP, then the four rows by two lane swaps
KA_DEV float wave_sum(float v) {
  v = row16_sum(v);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
KA_DEV float wave_max(float v) {
  v = row16_max(v);
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}

KA_DEV f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

KA_DEV bf16x8 as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }

#define KA_CHECK_LAUNCH() return (int)hipGetLastError()

// X[m][k] = bf16(silu(GU[m][k]) * GU[m][K + k]) for 8 bf16 lanes — bit-identical to silu_mul_kernel
// (elementwise.hip), so GEMMs that compute the activation while staging their X operand (gemv_ring
// SWIGLU) match the unfused SiLU kernel + GEMM exactly.
KA_DEV u32x4 swiglu8(u32x4 g, u32x4 u) {
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float g0 = lo_f(g[k]), g1 = hi_f(g[k]);
    const float s0 = g0 / (1.f + __expf(-g0)), s1 = g1 / (1.f + __expf(-g1));
    o[k] = pack2(s0 * lo_f(u[k]), s1 * hi_f(u[k]));
  }
  return o;
}
