#!/bin/bash
# Round 5, GPU call c: gemm_big fix verification, full-depth parity, plan re-tune with the ladder rule,
# decode graph ladder 1..512, bench.
set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big or lm_head or swiglu" > $O/pytest_kernels.log 2>&1
rc=$?; [ $rc -le 1 ] || stop kernels $rc
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_model_full_depth_gpu.py -s > $O/pytest_full_depth.log 2>&1
rc=$?; [ $rc -le 1 ] || stop full_depth $rc
timeout -k 10 300 tools/gemm_big_bench 4096,6144,4096,0,8,8 2944,6144,4096,0,8,8 4096,4096,4096,0 4096,28672,4096,3 2944,28672,4096,3 > $O/gemm_big_bench.log 2>&1
rc=$?; [ $rc -le 1 ] || stop gemm_big_bench $rc
PLAN_COPY_TO=$O/tuned timeout -k 10 900 python -u scripts/write_gemm_plan.py llama3-8b > $O/plan_write.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop plan_write $rc
timeout -k 10 600 python -u scripts/bench_decode_graph.py --buckets 1,2,4,8,16,32,48,64,96,128,160,192,256,320,384,448,512 --persistent 1 > $O/decode_ladder.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop ladder $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop bench $rc
echo ALL DONE
