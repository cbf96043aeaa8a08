#!/bin/bash
# Round 5, GPU call aa: after the gemm_big drain fix — prefill plan re-tuned (8B, Mixtral), the MoE
# prefill comparison, then the headline bench with the re-tuned plan.
set -o pipefail
O=gpurun_out/r5aa
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
export KA_AUTOTUNE_ROUNDS=3
PLAN_ONLY=prefill PLAN_BUCKETS=1 PLAN_COPY_TO=$O/tuned timeout -k 10 500 python -u scripts/write_gemm_plan.py llama3-8b mixtral-8x7b > $O/prefill_plan.log 2>&1 || stop prefill_plan $?
unset KA_AUTOTUNE_ROUNDS
timeout -k 10 200 python -u scripts/bench_moe_prefill.py > $O/moe_prefill.log 2>&1 || stop moe $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || stop bench $?
echo ALL DONE
