#!/bin/bash
# Open-loop (Poisson 900 req/s) p50 / p99 under the 4096 and 16384 token budgets, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/open
summ() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x.get("prefill_ms_per_step"))'; }
for r in 1 2; do for b in 4096 16384; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --load open --rate 900 --max-batched-tokens $b > gpurun_out/open/b${b}_r$r.log 2>&1 || { echo FAIL; tail -3 gpurun_out/open/b${b}_r$r.log; exit 1; }
  echo "open900 b=$b r=$r: $(tail -1 gpurun_out/open/b${b}_r$r.log | summ)"
done; done
