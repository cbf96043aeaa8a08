#!/bin/bash
# A/B of gemm_big harness builds (tools/gemm_big_bench_<variant>), interleaved reps, one GPU call
set -o pipefail
mkdir -p gpurun_out
C=${GB_CASES:-"4096,28672,4096,0 4096,28672,4096,3 4096,4096,14336,0 4096,4096,4096,0 4096,6144,4096,0 3072,28672,4096,3 2944,28672,4096,3 2944,6144,4096,0"}
for r in 1 2; do for v in ${GB_VARIANTS:-m0g1 m0g2}; do
  echo "$v rep$r"; timeout -k 10 120 tools/gemm_big_bench_$v $C || exit 1
done; done
