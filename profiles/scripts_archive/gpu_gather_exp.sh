#!/bin/bash
# Gather-window sweep at C=256 (wave merging): quiet gap / max window.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "3 15" "5 20" "8 30"; do
  set -- $cfg
  KA_GATHER_QUIET_MS=$1 KA_GATHER_MAX_MS=$2 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/gather_q$1_m$2.log 2>&1 || exit 1
done
for f in gpurun_out/gather_*.log; do echo "$f $(grep -o '"value": [0-9.]*\|"p50_ms": [0-9.]*\|"prefill_steps": [0-9]*\|"prefill_ms_per_step": [0-9.]*\|"engine_idle_ms_per_step": [0-9.]*' $f | tr '\n' ' ')"; done
