#!/bin/bash
# Round 6 session 3: re-tune the Llama-3-8B decode GEMM plan for the small buckets now that the
# consumers it is timed with (split-K norm, fused attention prologue) read their slices in batches;
# then A/B the decode graph step on the old and the new plan file.
set -o pipefail
O=gpurun_out/r6s3_plan2
mkdir -p $O
cp ai_agent_kubectl_amd/ops/tuned/gemm_plan_mi355x.json $O/plan_old.json
PLAN_ONLY=decode PLAN_BUCKETS=2,4,8,16,32,64,128 PLAN_COPY_TO=$O/new timeout -k 10 900 python -u scripts/write_gemm_plan.py llama3-8b > $O/retune.log 2>&1
rc=$?; echo "retune rc $rc"; tail -3 $O/retune.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  timeout -k 10 400 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 4,8,64,128 --reps 50 > $O/graph_new_$pass.log 2>&1 || exit 1
  KA_GEMM_PLAN_FILE=$O/plan_old.json timeout -k 10 400 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 4,8,64,128 --reps 50 > $O/graph_old_$pass.log 2>&1 || exit 1
  echo "pass $pass new: $(grep 'B=' $O/graph_new_$pass.log) | old: $(grep 'B=' $O/graph_old_$pass.log)"
done
