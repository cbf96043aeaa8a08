#!/bin/bash
# round-3 probe (one GPU call): gemm_big decode shapes, fused LM head tests, model tests, a short
# ASGI bench and the TCP scheduler sweep.  Every step has its own time limit; a failing GPU step ends it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 tools/gemm_big_bench 256,128256,4096,5 200,64128,4096,5 128,128256,4096,5 4096,28672,4096,3 \
  4096,4096,14336,0 256,4096,14336,2,8 > gpurun_out/gb_decode.log 2>&1 || exit 1
cat gpurun_out/gb_decode.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "lm_head or argmax" tests/test_model_gpu.py > gpurun_out/lmh_tests.log 2>&1 || { tail -30 gpurun_out/lmh_tests.log; exit 1; }
tail -2 gpurun_out/lmh_tests.log
timeout -k 10 300 python bench.py --transport asgi --steps 10 --warmup 3 --no-prefix-off-pass > gpurun_out/bench_lmh.log 2>&1 || exit 1
tail -1 gpurun_out/bench_lmh.log | cut -c1-1200
profiles/scripts_archive/tcp_sched_sweep.sh "base:X=1" "hold16:KA_PREFILL_HOLD_STEPS=16 KA_PREFILL_HOLD_MAX_MS=150 KA_GATHER_MAX_MS=60" \
  "w8c8:BENCH_API_WORKERS=8 BENCH_CLIENT_PROCS=8" 2>&1 | tee gpurun_out/tcp_sweep4.txt
