#!/bin/bash
# Bigger models on one GPU through the headline bench (TP = 1, full-size random-init weights).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/modes
timeout -k 10 500 python bench.py --model mixtral-8x7b --concurrency 128 --steps 10 --warmup 3 > gpurun_out/modes/mixtral_c128.log 2>&1 || { echo FAIL mixtral; tail -5 gpurun_out/modes/mixtral_c128.log; exit 1; }
echo "mixtral: $(tail -1 gpurun_out/modes/mixtral_c128.log | cut -c1-200)"
timeout -k 10 500 python bench.py --model llama3-70b --concurrency 64 --steps 8 --warmup 2 > gpurun_out/modes/llama70b_c64.log 2>&1 || { echo FAIL 70b; tail -5 gpurun_out/modes/llama70b_c64.log; exit 1; }
echo "70b: $(tail -1 gpurun_out/modes/llama70b_c64.log | cut -c1-200)"
