#!/bin/bash
# Round 5, GPU call r: split tail off for 192-wide tiles — full-matrix repeats, the previously failing
# GPU tests, the prefill plan re-tuned for the new tile / tail choices.
set -o pipefail
O=gpurun_out/r5r
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
CASES="4096,6144,4096,0 2944,6144,4096,0 4096,1152,4096,0 2944,6144,4096,0 1000,1152,2048,0 2944,28672,4096,3 3072,6144,4096,0 2944,6144,4096,0"
GB_FULL=1 GB_FULL_REPS=10 GB_ROUNDS=1 timeout -k 10 300 tools/gemm_big_bench_m2 $CASES > $O/stress.log 2>&1
rc=$?; [ $rc -le 1 ] || stop stress $rc
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big" tests/test_model_full_depth_gpu.py tests/test_model_gpu.py::test_last_layer_pruning_hidden_matches_full_gpu > $O/tests.log 2>&1
rc=$?; [ $rc -le 1 ] || stop tests $rc
export KA_GEMM_PLAN=write PLAN_COPY_TO=$O/tuned KA_AUTOTUNE_ROUNDS=3
PLAN_ONLY=prefill PLAN_BUCKETS=1 timeout -k 10 600 python -u scripts/write_gemm_plan.py llama3-8b mixtral-8x7b > $O/prefill_plan.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop prefill_plan $rc
echo ALL DONE
