#!/bin/bash
# Round 6, call i: every prefill-plan entry re-timed on one box in one run (two interleaved passes; no
# write: a check of the persisted decisions), then the Llama-3-70B (TP = 1) plans re-tuned and written on
# the drained-schedule kernels, copied back to gpurun_out/r6i/tuned.
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O/tuned
timeout -k 10 500 python -u scripts/retime_prefill_plan.py > $O/retime_prefill.log 2>&1; echo "retime rc=$?"; tail -2 $O/retime_prefill.log
PLAN_COPY_TO=$O/tuned timeout -k 10 650 python -u scripts/write_gemm_plan.py llama3-70b > $O/plan_70b.log 2>&1; echo "plan 70b rc=$?"; tail -2 $O/plan_70b.log
cp ai_agent_kubectl_amd/ops/tuned/gemm_plan_mi355x.json $O/tuned/gemm_plan_mi355x.json
