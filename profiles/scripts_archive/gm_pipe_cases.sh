#!/bin/bash
# A/B of the ring GEMM k-loop order (KA_GM_PIPE): tools/gemm_bench (1) vs tools/gemm_bench_pipe0 (0)
# on the decode plan's shapes, interleaved twice.  One GPU call; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gmpipe
C="256,28672,4096,2,1,3 256,6144,4096,12,2,2 256,6144,4096,2,4,2 256,4096,4096,12,4,2 256,4096,4096,4,4,2 256,4096,14336,2,8,2 256,4096,14336,3,8,2 128,28672,4096,4,1,3 128,6144,4096,4,4,2 128,4096,4096,5,4,2 128,4096,14336,4,8,2 64,28672,4096,5,1,3 64,4096,4096,5,8,2 32,28672,4096,5,1,3 512,6144,4096,3,2,2 512,4096,4096,3,4,2 256,28672,4096,-1,1,0"
for rep in 1 2; do
  timeout -k 10 120 tools/gemm_bench $C > gpurun_out/gmpipe/pipe1_r$rep.log 2>&1 &&
  timeout -k 10 120 tools/gemm_bench_pipe0 $C > gpurun_out/gmpipe/pipe0_r$rep.log 2>&1 || exit 1
done
