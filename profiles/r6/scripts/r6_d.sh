#!/bin/bash
# Round 6, call d: full-depth parity against the fp32 truth; then the Llama-3-8B decode plan re-tuned
# on the drained-schedule ring kernels (one box, one run), copied back to gpurun_out/r6d/tuned.
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O/tuned
timeout -k 10 900 python -u -m pytest tests/test_model_full_depth_gpu.py -v -s --timeout 600 --timeout-method thread > $O/full_depth.log 2>&1
echo "full depth rc=$?"
grep -E "agreement|repeats|passed|failed" $O/full_depth.log | tail -20
PLAN_COPY_TO=$O/tuned timeout -k 10 900 python -u scripts/write_gemm_plan.py llama3-8b > $O/plan.log 2>&1
echo "plan rc=$?"
tail -5 $O/plan.log
cp ai_agent_kubectl_amd/ops/tuned/gemm_plan_mi355x.json $O/tuned/gemm_plan_mi355x.json
