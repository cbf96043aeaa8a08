#!/bin/bash
# Round 5, GPU call ab: Llama-3-70B (TP 1) prefill plan re-tuned after the gemm_big drain fix.
set -o pipefail
O=gpurun_out/r5ab
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
KA_AUTOTUNE_ROUNDS=3 PLAN_ONLY=prefill PLAN_BUCKETS=1 PLAN_COPY_TO=$O/tuned timeout -k 10 1000 python -u scripts/write_gemm_plan.py llama3-70b > $O/prefill_plan_70b.log 2>&1 || stop prefill_plan $?
echo ALL DONE
