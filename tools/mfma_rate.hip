// MFMA issue-rate microbenchmark: v_mfma_f32_16x16x32_bf16 back to back from registers, 16 independent
// accumulators per wave (no dependent-latency stalls), 1 or 2 waves per SIMD on every CU.  Prints the
// chip's bf16 MFMA FLOP/s and the cycles per MFMA per SIMD it implies at the measured shader clock.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mfma_rate.hip -o tools/mfma_rate && tools/mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

template <int WAVES_PER_SIMD>
__global__ __launch_bounds__(256 * WAVES_PER_SIMD) void mfma_loop(float* out, int iters, unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (lane + i));
    b[i] = (__bf16)(0.002f * (lane - i));
  }
  f32x4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

// builtin MFMAs with 4 distinct A / B operand pairs
template <int WAVES_PER_SIMD>
__global__ __launch_bounds__(256 * WAVES_PER_SIMD) void mfma_loop_b4(float* out, int iters, unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[4];
  for (int k = 0; k < 4; ++k)
    for (int i = 0; i < 8; ++i) {
      a[k][i] = (__bf16)(0.001f * (lane + i + k));
      b[k][i] = (__bf16)(0.002f * (lane - i + k));
    }
  f32x4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 3], b[(i >> 2) & 3], acc[i], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

// the same with the accumulators pinned in AGPRs by asm MFMAs (gemm_big's form) and 4 distinct A / B
// operand pairs
template <int WAVES_PER_SIMD>
__global__ __launch_bounds__(256 * WAVES_PER_SIMD) void mfma_loop_agpr(float* out, int iters, unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[4];
  for (int k = 0; k < 4; ++k)
    for (int i = 0; i < 8; ++i) {
      a[k][i] = (__bf16)(0.001f * (lane + i + k));
      b[k][i] = (__bf16)(0.002f * (lane - i + k));
    }
  f32x4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i]) : "v"(a[i & 3]), "v"(b[(i >> 2) & 3]));
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) {
    asm volatile("" : "+a"(acc[i]));
    s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int W, int KIND = 0>
static void run(int cus, int iters) {
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, (size_t)cus * 256 * W * sizeof(float)));
  CK(hipMalloc(&clk, (size_t)cus * sizeof(unsigned long long)));
  auto kern = KIND == 2 ? mfma_loop_agpr<W> : KIND == 1 ? mfma_loop_b4<W> : mfma_loop<W>;
  hipLaunchKernelGGL(kern, dim3(cus), dim3(256 * W), 0, 0, out, 10, clk);   // warm-up
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(cus), dim3(256 * W), 0, 0, out, iters, clk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long c0;
  CK(hipMemcpy(&c0, clk, sizeof(c0), hipMemcpyDeviceToHost));
  const double mfmas_per_simd = (double)iters * 16 * W;   // W waves per SIMD, 16 MFMAs per iteration
  const double flop = (double)cus * 4 * mfmas_per_simd * 16 * 16 * 32 * 2;
  const double ghz = (double)c0 / (ms * 1e-3) / 1e9;   // block 0's loop cycles over the launch time (lower bound)
  printf("%s waves/SIMD %d: %.3f ms  %.1f TFLOP/s bf16  | block-0 loop %llu clk -> %.2f clk per MFMA per SIMD"
         " (shader clock ~%.2f GHz by launch time)\n",
         KIND == 2 ? "asm+AGPR, 4 operand pairs:  " : KIND == 1 ? "builtin, 4 operand pairs:   " : "builtin, one operand pair:  ", W, ms, flop / (ms * 1e-3) / 1e12, c0, (double)c0 / mfmas_per_simd, ghz);
  CK(hipFree(out));
  CK(hipFree(clk));
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  printf("CUs: %d\n", cus);
  run<1, 0>(cus, 20000);
  run<1, 1>(cus, 20000);
  run<1, 2>(cus, 20000);
  run<2, 0>(cus, 10000);
  run<2, 1>(cus, 10000);
  run<2, 2>(cus, 10000);
  return 0;
}
