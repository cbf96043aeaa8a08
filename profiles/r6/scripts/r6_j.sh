#!/bin/bash
# Round 6, call j: the Mixtral-8x7B plans re-tuned and written on the drained-schedule kernels.
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O/tuned
PLAN_COPY_TO=$O/tuned timeout -k 10 1000 python -u scripts/write_gemm_plan.py mixtral-8x7b > $O/plan_mixtral.log 2>&1; echo "plan mixtral rc=$?"; tail -2 $O/plan_mixtral.log
cp ai_agent_kubectl_amd/ops/tuned/gemm_plan_mi355x.json $O/tuned/gemm_plan_mi355x.json
