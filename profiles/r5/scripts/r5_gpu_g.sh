#!/bin/bash
# Round 5, GPU call g: persisted kernel plans for BASELINE configs #3 / #4 (Llama-3-70B TP = 1 and the
# TP = 8 per-rank shard, Mixtral-8x7B EP = 1 and the EP = 8 shard) and the virtual-rank step times.
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big" > $O/gb_tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop gb_tests $rc
export KA_GEMM_PLAN=write PLAN_COPY_TO=$O/tuned KA_AUTOTUNE_ROUNDS=3
# the prefill section of Llama-3-8B again: tuned in call d with the fenced tail hand-off (mode 1)
PLAN_ONLY=prefill PLAN_BUCKETS=1 timeout -k 10 400 python -u scripts/write_gemm_plan.py llama3-8b > $O/prefill_8b.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop prefill_8b $rc
timeout -k 10 900 python -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,2,4,8,16,32,64,128,256 > $O/vrank_70b_tp8.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop vrank70 $rc
timeout -k 10 900 python -u scripts/bench_virtual_rank.py --model mixtral-8x7b --tp 8 --buckets 1,2,4,8,16,32,64,128,256 > $O/vrank_mixtral_ep8.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop vrank_mixtral $rc
PLAN_BUCKETS=1,2,4,8,16,32,64,128,256 timeout -k 10 900 python -u scripts/write_gemm_plan.py mixtral-8x7b > $O/plan_mixtral.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop plan_mixtral $rc
echo ALL DONE
