#!/bin/bash
# A/B of the per-step token budget on the headline bench (TCP only, no prefix-off pass), specs
# interleaved so box drift hits every budget alike.  One GPU call; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/budget_ab
S=${BENCH_STEPS:-20}; W=${BENCH_WARMUP:-5}
for rep in ${REPS:-1 2}; do
  for B in ${BUDGETS:-4096 4608 5120}; do
    name=b${B}_r${rep}
    timeout -k 10 300 python bench.py --steps $S --warmup $W --transport tcp --no-prefix-off-pass \
      --max-batched-tokens $B > gpurun_out/budget_ab/$name.log 2>&1 || { echo "FAILED: $name"; tail -5 gpurun_out/budget_ab/$name.log; exit 1; }
    echo "$name: $(tail -1 gpurun_out/budget_ab/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x.get("decode_ms_per_step"), x.get("prefill_ms_per_step"))')"
  done
done
