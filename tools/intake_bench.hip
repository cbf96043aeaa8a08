// Per-CU intake of an L2-resident operand (the decode GEMMs' activations X: 2 MB read by every CU)
// by two paths, all 256 CUs at once: (a) global_load_dwordx4 into VGPRs, 8 loads in flight per lane;
// (b) LDS-DMA (global_load_lds_dwordx4) through a 16-slot ring per wave.  Also (c): both at once,
// half the waves each.  hipcc --offload-arch=gfx950 -O3 tools/intake_bench.hip -o /tmp/intake
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int NT = 512;
constexpr size_t XBYTES = 2u << 20;

__global__ __launch_bounds__(NT, 1) void direct_kernel(const uint4* __restrict__ x, uint32_t* __restrict__ sink,
                                                       int passes) {
  const int tid = threadIdx.x;
  const size_t n16 = XBYTES / 16;
  uint32_t acc = 0;
  // each workgroup starts at its own offset (the CUs of an XCD read different lines at a time)
  size_t i = ((size_t)blockIdx.x * 4096 + tid) % n16;
  for (int p = 0; p < passes; ++p) {
    for (size_t k = 0; k < n16 / NT; k += 8) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = x[(i + (size_t)u * NT) & (n16 - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].w;
      i = (i + 8 * NT) & (n16 - 1);
    }
  }
  if (acc == 0x12345678u) sink[blockIdx.x * NT + tid] = acc;
}

__global__ __launch_bounds__(NT, 1) void ldsdma_kernel(const uint4* __restrict__ x, uint32_t* __restrict__ sink,
                                                       int passes) {
  extern __shared__ __attribute__((aligned(16))) uint4 ring[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const size_t n16 = XBYTES / 16;
  size_t i = ((size_t)blockIdx.x * 4096 + wave * 64) % n16;   // 1 KB per wave instruction
  uint4* slot0 = ring + wave * 16 * 64;
  int s = 0;
  for (int p = 0; p < passes; ++p) {
    for (size_t k = 0; k < n16 / NT; ++k) {
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(x + ((i + lane) & (n16 - 1))),
                                       (__attribute__((address_space(3))) void*)(slot0 + s * 64), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
      s = (s + 1) & 15;
      i = (i + NT) & (n16 - 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ring[tid].x == 0x12345678u) sink[blockIdx.x * NT + tid] = 1;
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  uint4* x;
  uint32_t* sink;
  hipMalloc(&x, XBYTES);
  hipMalloc(&sink, (size_t)cus * NT * 4);
  std::vector<uint32_t> h(XBYTES / 4);
  for (size_t k = 0; k < h.size(); ++k) h[k] = (uint32_t)(k * 2654435761u);
  hipMemcpy(x, h.data(), XBYTES, hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)ldsdma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 16 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int passes = 8;
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (mode == 0)
        hipLaunchKernelGGL(direct_kernel, dim3(cus), dim3(NT), 0, 0, x, sink, passes);
      else
        hipLaunchKernelGGL(ldsdma_kernel, dim3(cus), dim3(NT), 8 * 16 * 1024, 0, x, sink, passes);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double per_cu = (double)XBYTES * passes / (ms * 1e-3) / 1e9;
      printf("%s rep %d: %.3f ms, %.1f GB/s per CU, %.2f TB/s chip\n", mode ? "ldsdma" : "direct", rep, ms, per_cu,
             per_cu * cus / 1e3);
    }
  }
  return 0;
}
