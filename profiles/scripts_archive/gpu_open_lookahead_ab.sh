#!/bin/bash
# Open loop (Poisson 900 req/s) with and without lookahead, two interleaved reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/open_la
summ() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x.get("decode_ms_per_step"), x.get("prefill_ms_per_step"), x.get("prefill_tokens"))'; }
for r in 1 2; do for la in ${LA:-0 1}; do
  KA_LOOKAHEAD=$la timeout -k 10 300 python bench.py --steps 10 --warmup 3 --load open --rate 900 > gpurun_out/open_la/la${la}_r$r.log 2>&1 || { echo FAIL; tail -3 gpurun_out/open_la/la${la}_r$r.log; exit 1; }
  echo "open900 la=$la r=$r: $(tail -1 gpurun_out/open_la/la${la}_r$r.log | summ)"
done; done
