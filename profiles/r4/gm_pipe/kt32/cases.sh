#!/bin/bash
# BK = 32 deep-ring configurations (20: 128 x 256, 5 stages; 21: 128 x 128, 6 stages) against the
# plan's BK = 64 ones on the decode shapes, twice.  One GPU call; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kt32
C="256,28672,4096,2,1,3 256,28672,4096,20,1,3 256,6144,4096,2,4,2 256,6144,4096,20,4,2 256,6144,4096,21,4,2 256,4096,14336,2,8,2 256,4096,14336,20,8,2 256,4096,4096,4,4,2 256,4096,4096,21,4,2 256,4096,4096,20,4,2 128,28672,4096,4,1,3 128,28672,4096,21,1,3 128,4096,14336,4,8,2 128,4096,14336,21,8,2"
for rep in 1 2; do
  timeout -k 10 120 tools/gemm_bench $C > gpurun_out/kt32/r$rep.log 2>&1 || exit 1
done
