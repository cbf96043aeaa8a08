#!/bin/bash
# Lookahead A/B at the driver config: off vs margins (KA_LOOKAHEAD_MARGIN_MS), interleaved reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lookahead
summ() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x.get("decode_ms_per_step"), x.get("prefill_ms_per_step"))'; }
for r in 1 2 3; do
  for spec in ${LA_SPECS:-"0:3" "1:3" "1:6" "1:10"}; do
    IFS=: read on mg <<< "$spec"
    KA_LOOKAHEAD=$on KA_LOOKAHEAD_MARGIN_MS=$mg timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/lookahead/la${on}_m${mg}_r$r.log 2>&1 || { echo FAIL; tail -3 gpurun_out/lookahead/la${on}_m${mg}_r$r.log; exit 1; }
    echo "la=$on margin=$mg r=$r: $(tail -1 gpurun_out/lookahead/la${on}_m${mg}_r$r.log | summ)"
  done
done
