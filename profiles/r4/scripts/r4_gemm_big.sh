#!/bin/bash
# gemm_big split-tail check: GPU numerics tests, then the harness against rocBLAS with and without
# the split tail (interleaved rounds in one process per setting).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4c}
mkdir -p $OUT
SHAPES="${SHAPES:-4096,6144,4096,0 2944,6144,4096,0 3328,6144,4096,0 8192,6144,4096,0 4096,4096,4096,0 2944,4096,4096,0 4096,4096,14336,0 2944,4096,14336,0 4096,28672,4096,3 2944,28672,4096,3 3328,28672,4096,3 8192,28672,4096,3 1100,28672,4096,3}"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_big" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gb.log 2>&1 &&
GB_TAIL=1 timeout -k 10 300 tools/gemm_big_bench $SHAPES > $OUT/gb_tail.log 2>&1 &&
GB_TAIL=0 timeout -k 10 300 tools/gemm_big_bench $SHAPES > $OUT/gb_notail.log 2>&1
rc=$?
echo "exit=$rc"
tail -4 $OUT/pytest_gb.log; cat $OUT/gb_tail.log $OUT/gb_notail.log 2>/dev/null
exit $rc
