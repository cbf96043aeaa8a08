#!/bin/bash
# Round 5, GPU call b: gemm_big tile width (TN 6 / 8) + no-restage fix: correctness, timing vs rocBLAS;
# the full-depth decode tests.
set -o pipefail
O=gpurun_out/r5b
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big or lm_head or swiglu" > $O/pytest_kernels.log 2>&1
rc=$?; [ $rc -le 1 ] || stop kernels $rc
timeout -k 10 300 tools/gemm_big_bench 4096,6144,4096,0,8,8 4080,6144,4096,0,8,8 2944,6144,4096,0,8,6 4096,4096,4096,0 4096,4096,8192,0 4096,4096,16384,0 8192,4096,4096,0 4096,4096,14336,0 4096,28672,4096,3 4080,4096,4096,4 4080,4096,14336,4 > $O/gemm_big_bench.log 2>&1
rc=$?; [ $rc -le 1 ] || stop gemm_big_bench $rc
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_model_full_depth_gpu.py -s > $O/pytest_full_depth.log 2>&1
rc=$?; [ $rc -le 1 ] || stop full_depth $rc
echo ALL DONE
