// Harness for csrc/gemm_big.hip (the prefill projection GEMM): correctness against an fp32 reference
// on sampled rows, and timing against rocBLAS (bf16 in/out, fp32 compute, torch F.linear's TN layout)
// in the same process, interleaved per round (cdna_hip_programming.md §5.4 rule 24).  No torch.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_big_bench.hip -lrocblas -o tools/gemm_big_bench
//   tools/gemm_big_bench M,N,K,epi[,gm[,tn]] ... epi: 0 bf16, 3 SwiGLU (N = 2I), 4 residual add,
//                                               5 fused LM head + masked argmax (rocBLAS: GEMM only),
//                                               1 / 2 split-K fp32 / bf16 partials (the 5th field is the
//                                               split; the consumer's reduction is not timed);
//                                               tn 6 / 8 (epi 0 / 4): also time that tile width
//                                               (`alt`) beside the automatic choice
//
// Weights rotate over copies that exceed the 256 MB Infinity Cache unless GB_WARM=1.
#include "../ai_agent_kubectl_amd/csrc/gemm_big.hip"
#include "../ai_agent_kubectl_amd/csrc/sampling.hip"

#include <rocblas/rocblas.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void fill_kernel(bf16_t* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = f2bf(((h & 0xffffff) / 8388608.f - 1.f) * scale);
  }
}

// out[s][n] = sum_k X[rows[s]][k] * W[n][k] in fp32
__global__ void ref_kernel(float* out, const bf16_t* X, const bf16_t* W, const int* rows, int S, int N, int K, int ldx) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, s = blockIdx.y;
  if (n >= N || s >= S) return;
  const bf16_t* x = X + (size_t)rows[s] * ldx;
  const bf16_t* w = W + (size_t)n * K;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc += bf2f(x[k]) * bf2f(w[k]);
  out[(size_t)s * N + n] = acc;
}

static float bf(uint16_t v) {
  uint32_t u = (uint32_t)v << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

int main(int argc, char** argv) {
  rocblas_handle rb;
  rocblas_create_handle(&rb);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  rocblas_set_stream(rb, st);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int warm = getenv("GB_WARM") ? atoi(getenv("GB_WARM")) : 0;
  // GB_TAIL=0: no split tail (the whole-tile schedule of rounds 1-3)
  const int tail = getenv("GB_TAIL") ? atoi(getenv("GB_TAIL")) : 1;
  const size_t ws_tail_bytes = ka_gemm_big_ws_bytes();
  void* ws_tail = nullptr;
  CK(hipMalloc(&ws_tail, ws_tail_bytes));
  CK(hipMemset(ws_tail, 0, ws_tail_bytes));
  const int rounds = getenv("GB_ROUNDS") ? atoi(getenv("GB_ROUNDS")) : 3;
  int bad = 0;

  for (int ci = 1; ci < argc; ++ci) {
    int M, N, K, epi, gm = 8, tn_alt = 0;
    if (sscanf(argv[ci], "%d,%d,%d,%d,%d,%d", &M, &N, &K, &epi, &gm, &tn_alt) < 4) {
      fprintf(stderr, "bad case %s\n", argv[ci]);
      return 2;
    }
    const bool sw = epi == 3;
    const int ldy = sw ? N / 2 : N;
    const size_t wbytes = (size_t)N * K * 2;
    const int nrot = warm ? 1 : (int)std::max<size_t>(1, (size_t)(768ull << 20) / wbytes + 1);
    bf16_t *X, *W, *Y, *Yb, *R = nullptr;
    CK(hipMalloc(&X, (size_t)M * K * 2));
    CK(hipMalloc(&W, wbytes * nrot));
    const bool part = epi == 1 || epi == 2;
    const int split = part ? gm : 1;
    void* P = nullptr;
    if (part) CK(hipMalloc(&P, (size_t)split * M * N * 4));
    CK(hipMalloc(&Y, (size_t)M * ldy * 2));
    CK(hipMalloc(&Yb, (size_t)M * N * 2));
    hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, st, X, (size_t)M * K, 1234u, 1.0f);
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, st, W, (size_t)N * K * nrot, 777u, 1.0f / sqrtf((float)K));
    if (epi == 4) {
      CK(hipMalloc(&R, (size_t)M * N * 2));
      hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, st, R, (size_t)M * N, 99u, 1.0f);
    }
    // EPI 5: two mask rows (0: tokens n % 3 != 0, 1: all), row m uses m % 3 - 1 (-1 = unmasked)
    const int words = (N + 31) / 32;
    uint32_t* dmask = nullptr;
    int *dmidx = nullptr, *didx = nullptr;
    float* dval = nullptr;
    void* ws = nullptr;
    std::vector<uint32_t> hmask(2 * (size_t)words, 0xffffffffu);
    std::vector<int> hmidx(M);
    if (epi == 5) {
      for (int n = 0; n < N; n += 3) hmask[n >> 5] &= ~(1u << (n & 31));
      for (int m = 0; m < M; ++m) hmidx[m] = m % 3 - 1;
      CK(hipMalloc(&dmask, hmask.size() * 4));
      CK(hipMalloc(&dmidx, M * 4));
      CK(hipMalloc(&didx, M * 4));
      CK(hipMalloc(&dval, M * 4));
      CK(hipMalloc(&ws, ka_gemm_big_argmax_ws(M, N)));
      CK(hipMemcpy(dmask, hmask.data(), hmask.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(dmidx, hmidx.data(), M * 4, hipMemcpyHostToDevice));
    }
    CK(hipStreamSynchronize(st));

    auto mine = [&](int r) {
      const bf16_t* w = W + (size_t)(r % nrot) * N * K;
      if (epi == 5) return ka_gemm_big_argmax(didx, dval, X, w, M, N, K, K, dmask, dmidx, words, 0, ws, st);
      if (part) return ka_gemm_big_splitk(P, X, w, M, N, K, K, split, epi == 2, 8, st);
      return ka_gemm_big(Y, R, X, w, M, N, K, K, ldy, epi, gm, tail ? ws_tail : nullptr, tail ? ws_tail_bytes : 0, st);
    };
    // the other tile width, launched directly (same split-tail workspace)
    auto alt = [&](int r) {
      const bf16_t* w = W + (size_t)(r % nrot) * N * K;
      gb::Args a{X, w, Y, R, M, N, K, K, ldy, 0, 0, gm, N / 2};
      void* wsp = tail ? ws_tail : nullptr;
      const size_t wsb = tail ? ws_tail_bytes : 0;
      if (epi == 4) return tn_alt == 6 ? gb::launch<gb::EPI_ADD, 6>(a, st, wsp, wsb) : gb::launch<gb::EPI_ADD, 8>(a, st, wsp, wsb);
      return tn_alt == 6 ? gb::launch<gb::EPI_BF16, 6>(a, st, wsp, wsb) : gb::launch<gb::EPI_BF16, 8>(a, st, wsp, wsb);
    };
    const bool has_alt = (epi == 0 || epi == 4) && (tn_alt == 6 || tn_alt == 8) && N % (32 * tn_alt) == 0;
    auto blas = [&](int r) {
      const bf16_t* w = W + (size_t)(r % nrot) * N * K;
      const float alpha = 1.f, beta = 0.f;
      return (int)rocblas_gemm_ex(rb, rocblas_operation_transpose, rocblas_operation_none, N, M, K, &alpha, w,
                                  rocblas_datatype_bf16_r, K, X, rocblas_datatype_bf16_r, K, &beta, Yb,
                                  rocblas_datatype_bf16_r, N, Yb, rocblas_datatype_bf16_r, N, rocblas_datatype_f32_r,
                                  rocblas_gemm_algo_standard, 0, 0);
    };
    // correctness (EPI_ADD: Y = X W^T + R with R kept separate so the check is exact about it)
    int rc = mine(0);
    if (rc) {
      printf("%s: launch error %d\n", argv[ci], rc);
      bad = 1;
      continue;
    }
    CK(hipStreamSynchronize(st));
    // GB_FULL=1: every row checked (and the correctness run repeated GB_FULL_REPS times): the split
    // tail's hand-off is validated on the whole matrix, not on 32 sampled rows
    const int full_check = getenv("GB_FULL") ? atoi(getenv("GB_FULL")) : 0;
    const int S = full_check ? M : std::min(M, 32);
    std::vector<int> rows(S);
    for (int s = 0; s < S; ++s) rows[s] = (int)((long)s * (M - 1) / std::max(1, S - 1));
    int* drows;
    float* dref;
    CK(hipMalloc(&drows, S * 4));
    CK(hipMalloc(&dref, (size_t)S * N * 4));
    CK(hipMemcpy(drows, rows.data(), S * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, S), dim3(256), 0, st, dref, X, W, drows, S, N, K, K);
    CK(hipStreamSynchronize(st));
    std::vector<float> ref((size_t)S * N);
    CK(hipMemcpy(ref.data(), dref, ref.size() * 4, hipMemcpyDeviceToHost));
    std::vector<uint16_t> got((size_t)ldy), rr((size_t)N);
    double err = 0, mr = 0;
    if (epi == 5) {   // the chosen token is allowed and its reference logit is within tolerance of the max
      std::vector<int> hidx(M);
      CK(hipMemcpy(hidx.data(), didx, M * 4, hipMemcpyDeviceToHost));
      for (int s = 0; s < S; ++s) {
        const int m = rows[s], mi = hmidx[m];
        auto ok = [&](int n) { return mi < 0 || ((hmask[(size_t)mi * words + (n >> 5)] >> (n & 31)) & 1u); };
        double best = -1e30;
        for (int n = 0; n < N; ++n)
          if (ok(n)) best = std::max(best, (double)ref[(size_t)s * N + n]);
        const int g = hidx[m];
        const double d = (g >= 0 && g < N && ok(g)) ? best - ref[(size_t)s * N + g] : 1e30;
        err = std::max(err, d);
        mr = std::max(mr, std::fabs(best));
      }
    }
    if (part) {   // sum of the slices' partials
      std::vector<float> pf((size_t)N);
      std::vector<uint16_t> ph((size_t)N);
      for (int s = 0; s < S; ++s) {
        std::vector<double> sum((size_t)N, 0.0);
        for (int k = 0; k < split; ++k) {
          const size_t o = ((size_t)k * M + rows[s]) * N;
          if (epi == 1) {
            CK(hipMemcpy(pf.data(), static_cast<float*>(P) + o, N * 4, hipMemcpyDeviceToHost));
            for (int c = 0; c < N; ++c) sum[c] += pf[c];
          } else {
            CK(hipMemcpy(ph.data(), static_cast<uint16_t*>(P) + o, N * 2, hipMemcpyDeviceToHost));
            for (int c = 0; c < N; ++c) sum[c] += bf(ph[c]);
          }
        }
        for (int c = 0; c < N; ++c) {
          err = std::max(err, std::fabs(sum[c] - ref[(size_t)s * N + c]));
          mr = std::max(mr, (double)std::fabs(ref[(size_t)s * N + c]));
        }
      }
    }
    const int creps = full_check ? (getenv("GB_FULL_REPS") ? atoi(getenv("GB_FULL_REPS")) : 4) : 1;
    for (int cr = 0; cr < creps; ++cr) {
    if (cr > 0) {
      if (mine(0)) bad = 1;
      CK(hipStreamSynchronize(st));
    }
    double rep_err = 0;
    for (int s = 0; s < S && epi != 5 && !part; ++s) {
      CK(hipMemcpy(got.data(), Y + (size_t)rows[s] * ldy, ldy * 2, hipMemcpyDeviceToHost));
      if (R) CK(hipMemcpy(rr.data(), R + (size_t)rows[s] * N, N * 2, hipMemcpyDeviceToHost));
      for (int c = 0; c < ldy; ++c) {
        double r;
        if (sw) {
          const double g = ref[(size_t)s * N + c], u = ref[(size_t)s * N + N / 2 + c];
          r = g / (1.0 + std::exp(-g)) * u;
        } else {
          r = ref[(size_t)s * N + c] + (R ? bf(rr[c]) : 0.0);
        }
        err = std::max(err, std::fabs(bf(got[c]) - r));
        rep_err = std::max(rep_err, std::fabs(bf(got[c]) - r));
        mr = std::max(mr, std::fabs(r));
      }
    }
    if (full_check) printf("  full check rep %d: max err %.4g\n", cr, rep_err);
    }
    CK(hipFree(drows));
    CK(hipFree(dref));
    const bool mismatch = !(err <= 0.02 * std::max(1.0, mr));
    bad |= mismatch;

    // timing: rounds of (mine, rocBLAS) back to back
    const int iters = 20;
    auto time = [&](auto&& fn) {
      for (int r = 0; r < 2; ++r) fn(r + 1);
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < iters; ++r) fn(r + 3);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms * 1e3 / iters;
    };
    // the alternative width's correctness on the same sampled rows (Y is overwritten by it)
    double alt_err = 0;
    if (has_alt) {
      if (alt(0)) {
        printf("%s: alt launch error\n", argv[ci]);
        bad = 1;
      }
      CK(hipStreamSynchronize(st));
      std::vector<uint16_t> g2((size_t)ldy), r2((size_t)N);
      for (int s = 0; s < S; ++s) {
        CK(hipMemcpy(g2.data(), Y + (size_t)rows[s] * ldy, ldy * 2, hipMemcpyDeviceToHost));
        if (R) CK(hipMemcpy(r2.data(), R + (size_t)rows[s] * N, N * 2, hipMemcpyDeviceToHost));
        for (int c = 0; c < ldy; ++c)
          alt_err = std::max(alt_err, std::fabs(bf(g2[c]) - (ref[(size_t)s * N + c] + (R ? bf(r2[c]) : 0.0))));
      }
      if (!(alt_err <= 0.02 * std::max(1.0, mr))) {
        printf("%s: alt tn=%d MISMATCH %g\n", argv[ci], tn_alt, alt_err);
        bad = 1;
      }
    }
    std::vector<double> tm, tb, ta;
    for (int r = 0; r < rounds; ++r) {
      tm.push_back(time(mine));
      if (has_alt) ta.push_back(time(alt));
      tb.push_back(time(blas));
    }
    std::sort(tm.begin(), tm.end());
    std::sort(tb.begin(), tb.end());
    std::sort(ta.begin(), ta.end());
    const double fl = 2.0 * M * N * K;
    int pf = 0, pt = 0;
    const int ps = (epi == 0 || epi == 3 || epi == 4) && tail ? ka_gemm_big_plan(M, N, epi, K, ws_tail_bytes, &pf, &pt) : 1;
    int terr = 0;
    CK(hipMemcpy(&terr, ws_tail, 4, hipMemcpyDeviceToHost));
    if (terr) {
      printf("%s: split-tail error word set\n", argv[ci]);
      bad = 1;
    }
    printf("tn=%d tail s=%d (%d whole + %d split tiles) ", ka_gemm_big_tn(M, N, epi), ps, pf, pt);
    if (has_alt) printf("[alt tn=%d %8.2f us %7.1f TF/s ratio %.3f] ", tn_alt, ta[0], 2.0 * M * N * K / (ta[0] * 1e-6) / 1e12, tb[0] / ta[0]);
    printf("M=%5d N=%6d K=%5d epi=%d gm=%d : gemm_big %8.2f us %7.1f TF/s | rocBLAS %8.2f us %7.1f TF/s | "
           "ratio %.3f | maxerr %.3g (ref max %.3g)%s\n",
           M, N, K, epi, gm, tm[0], fl / (tm[0] * 1e-6) / 1e12, tb[0], fl / (tb[0] * 1e-6) / 1e12, tb[0] / tm[0], err,
           mr, mismatch ? "  <-- MISMATCH" : "");
    fflush(stdout);
    CK(hipFree(X));
    CK(hipFree(W));
    CK(hipFree(Y));
    CK(hipFree(Yb));
    if (R) CK(hipFree(R));
    if (P) CK(hipFree(P));
    if (epi == 5) {
      CK(hipFree(dmask));
      CK(hipFree(dmidx));
      CK(hipFree(didx));
      CK(hipFree(dval));
      CK(hipFree(ws));
    }
  }
  rocblas_destroy_handle(rb);
  return bad;
}
