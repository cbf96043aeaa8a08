#!/bin/bash
# Token-budget sweep of the headline bench: small per-step budgets turn each wave's one 8k-token
# prefill into chunks that ride in mixed steps beside the running decodes (decode rows then cost
# prefill-GEMM efficiency instead of a decode step of their own).  One GPU call; the first failure
# ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/budget
S=${BENCH_STEPS:-20}; W=${BENCH_WARMUP:-5}
run() {  # name, env..., -- args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps $S --warmup $W > gpurun_out/budget/$name.log 2>&1 || { echo "FAILED: $name"; tail -5 gpurun_out/budget/$name.log; exit 1; }
  echo "$name: $(tail -1 gpurun_out/budget/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x.get("decode_ms_per_step"), x.get("prefill_ms_per_step"))')"
}
for spec in ${BUDGET_SPECS:-"16384:0.25:15" "4096:0:0" "2048:0:0" "1024:0:0"}; do
  IFS=: read B F Wt <<< "$spec"
  run b${B}_f${F}_w${Wt} BENCH_MAX_BATCHED_TOKENS=$B KA_PREFILL_MIN_FRAC=$F KA_PREFILL_MAX_WAIT_MS=$Wt
done
