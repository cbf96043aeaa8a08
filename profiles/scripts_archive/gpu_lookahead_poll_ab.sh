#!/bin/bash
# Lookahead wait after an eager step: polling the progress event (KA_LOOKAHEAD_POLL_US) vs a blocking
# event synchronize (0), interleaved reps at the driver config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/poll
summ() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x.get("decode_ms_per_step"), x.get("prefill_ms_per_step"))'; }
for r in 1 2 3; do for pu in 300 0 2000; do
  KA_LOOKAHEAD_POLL_US=$pu timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/poll/p${pu}_r$r.log 2>&1 || { echo FAIL; tail -3 gpurun_out/poll/p${pu}_r$r.log; exit 1; }
  echo "poll_us=$pu r=$r: $(tail -1 gpurun_out/poll/p${pu}_r$r.log | summ)"
done; done
